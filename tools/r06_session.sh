#!/bin/bash
# round-6 GPU session: the new/changed GPU tests, then the PMC passes of the shipped
# round trip (roundtrip8) and huffman_bits.  Each step has its own time limit.
set -u -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r06b}
K=${2:-"many_streams or handle_reuse or legacy_threads or encode_planes_fused or encode_capacity or c_host_programs or bench_gpus2_gloo or dist_legs or bench_json"}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 420 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
if [ "${PMC:-1}" = 1 ]; then
  bash tools/pmc_rt.sh $O/pmc_rt && bash tools/pmc_huf.sh $O/pmc_huf uniform
fi
