export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
cat /sys/fs/cgroup/cpu.max > gpurun_out/cpuinfo.log 2>&1; env | grep -i -E "omp|threads|jobs" >> gpurun_out/cpuinfo.log; timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; echo "bench rc=$?"
