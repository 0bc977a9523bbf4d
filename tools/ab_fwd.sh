#!/bin/bash
# tools/ab_fwd.sh LIB... -- on the GPU box: tools/lib_ab.py (steady state, 3 launches
# back to back per sample) over the bench step for the listed builds, on the
# uniform q50 input and the tie-heavy plans (q100, extremes q10, adaptive).
set -u
mkdir -p gpurun_out
for args in "" "--quality 100" "--kind extreme --quality 10" "--adaptive 1" "--kind smooth"; do
  timeout -k 10 240 python tools/lib_ab.py --b2b 3 --rounds 10 $args "$@" || exit $?
done
