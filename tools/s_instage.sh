set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
L="default tools/ubench/libvar_old.so tools/ubench/libvar_t4.so tools/ubench/libvar_t16.so tools/ubench/libvar_t65.so movement"
for cfg in "--kind extreme --quality 10" "--kind uniform --quality 100" "--kind uniform --quality 50" "--kind smooth --quality 90 --adaptive 1"; do
  timeout -k 10 200 python tools/lib_ab.py --rounds 6 --b2b 3 $cfg $L 2>&1 | grep -v amdgpu
done
