#!/bin/bash
# Round 6 final evidence for profiles/r06/final/ (one gpurun call, from the repo root).
# Each GPU step has its own time limit and the steps are chained: the first failure ends the run.
#   1. the whole -m gpu suite, then smoke()
#   2. separate --pmc FETCH_SIZE / WRITE_SIZE passes over the bench step -> traffic.json (library hash recorded)
#   3. rocprofv3 --kernel-trace --stats over the bench command
#   4. bench.py as the driver runs it (picks traffic.json up)
#   5. kernel stats of the round trip and the secondary kernels (rt_bench.py, aux_bench.py)
set -u -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06_final}
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
echo "smoke ok" &&
B="python bench.py --steps 3 --warmup 1 --no-cpu --round-trip-steps 0 --encode-steps 0 --ceiling-rounds 0 --prewarm-ms 0" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1 &&
python tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv \
  --frames 64 --kind uniform --quality 50 --adaptive 0 --launches 1 -o $O/traffic.json &&
cp $O/traffic.json profiles/traffic.json &&
echo "traffic ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu --round-trip-steps 0 --encode-steps 0 --ceiling-rounds 0 > $O/prof_bench.log 2>&1 &&
echo "prof ok" &&
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err &&
echo "bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rt -o run --output-format csv -- \
  python tools/rt_bench.py 64 > $O/rt_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_aux -o run --output-format csv -- \
  python tools/aux_bench.py > $O/aux_bench.log 2>&1 &&
echo "collected"
