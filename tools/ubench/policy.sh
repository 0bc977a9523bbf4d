#!/bin/bash
# Diagnostic copies of libdct_amd.so whose bulk coefficient stores use other
# gfx950 cache-policy bits: tools/ubench/libpolicy_<aux>.so (outputs are correct).
# DIAG=1 also links diag.hip, so the movement kernel of the same policy can be
# timed (tools/lib_ab.py movement:PATH).
set -e
cd "$(dirname "$0")/../.."
srcs=$(python -c "import dct_amd.build as b; print(' '.join('dct_amd/csrc/' + s for s in b.SOURCES + (b.DIAG_SOURCES if '${DIAG:-0}' == '1' else [])))")
for a in ${@:-1 2 16 17 3}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
    -Wno-unused-command-line-argument ${EXTRA:-} -DDCTQ_STORE_AUX=$a -Iinclude -Idct_amd/csrc \
    $srcs \
    -o tools/ubench/libpolicy_${TAG:-}$a.so &
done
wait
