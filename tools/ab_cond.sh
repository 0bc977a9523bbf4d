set -e
mkdir -p gpurun_out
L="default tools/ubench/libvar_head.so tools/ubench/libvar_early.so movement"
for a in "--kind extreme --quality 10" "--kind uniform --quality 100" "--kind uniform --quality 50" "--kind smooth --quality 90 --adaptive 1"; do
  timeout -k 10 150 python tools/lib_ab.py --rounds 14 $a $L >> gpurun_out/ab_early.log 2>&1
done
