#!/bin/bash
# tools/collect_profiles.sh -- on the GPU box (via gpurun), from the repo root:
# the round's evidence for profiles/rNN/ in gpurun_out/prof_final/ (copy it over
# afterwards).  Each GPU step has its own time limit; any failure ends the run.
#   1. separate --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py -> traffic.json
#      (configuration + library hash recorded: bench.py uses it only for a matching run)
#   2. rocprofv3 --kernel-trace --stats over the bench command (with its clock pre-warm)
#   3. bench.py (the driver's command), which picks traffic.json up
#   4. kernel stats of the round trip, RLE and Huffman kernels (tools/rt_bench.py, aux_bench.py)
#   5. the forward kernel over every input kind x plan beside its movement (tools/perf_matrix.py)
#      and the Huffman sizes per input kind (tools/huf_ab.py)
set -eu
export TMPDIR=/tmp
O=gpurun_out/prof_final
mkdir -p $O
B="python bench.py --steps 3 --warmup 1 --no-cpu --round-trip-steps 0 --encode-steps 0 --ceiling-rounds 0 --prewarm-ms 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1
python tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv \
  --frames 64 --kind uniform --quality 50 --adaptive 0 --launches 1 -o $O/traffic.json
cp $O/traffic.json profiles/traffic.json
echo "traffic done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu --round-trip-steps 0 --encode-steps 0 --ceiling-rounds 0 > $O/prof_bench.log 2>&1
echo "prof done"
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
echo "bench done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rt -o run --output-format csv -- \
  python tools/rt_bench.py 64 > $O/rt_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_aux -o run --output-format csv -- \
  python tools/aux_bench.py > $O/aux_bench.log 2>&1
echo "aux done"
timeout -k 10 300 python tools/perf_matrix.py > $O/perf_matrix.log 2>&1
timeout -k 10 200 python tools/huf_ab.py > $O/huf.log 2>&1
echo collected
