set -e
export TMPDIR=/tmp
L="default tools/ubench/libvar_t2.so tools/ubench/libvar_t3.so tools/ubench/libvar_t4.so tools/ubench/libvar_t6.so movement"
for cfg in "--kind extreme --quality 10" "--kind uniform --quality 100" "--kind uniform --quality 50" "--kind uniform --quality 90" "--kind smooth --quality 90 --adaptive 1"; do
  timeout -k 10 200 python tools/lib_ab.py --rounds 6 --b2b 3 $cfg $L 2>&1 | grep -v amdgpu
done
