#!/bin/bash
# Diagnostic copies of libdct_amd.so whose bulk coefficient stores use other
# gfx950 cache-policy bits: tools/ubench/libpolicy_<aux>.so (outputs are correct).
set -e
cd "$(dirname "$0")/../.."
for a in ${@:-1 2 16 17 3}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
    -Wno-unused-command-line-argument ${EXTRA:-} -DDCTQ_STORE_AUX=$a -Iinclude -Idct_amd/csrc \
    dct_amd/csrc/api.hip dct_amd/csrc/legacy.hip dct_amd/csrc/fdct8.hip dct_amd/csrc/fdct8_aux.hip dct_amd/csrc/f64_pair.hip dct_amd/csrc/rle.hip \
    -o tools/ubench/libpolicy_${TAG:-}$a.so &
done
wait
