set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu
L="default tools/ubench/libvar_old.so movement"
for cfg in "--kind extreme --quality 10" "--kind uniform --quality 100" "--kind uniform --quality 50"; do
  timeout -k 10 200 python tools/lib_ab.py --rounds 6 --b2b 3 $cfg $L 2>&1 | grep -v amdgpu
done
timeout -k 10 200 python tools/rt_bench.py 64 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/small_ab.py 2>&1 | grep -v amdgpu
