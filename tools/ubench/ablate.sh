#!/bin/bash
# Build diagnostic copies of libdct_amd.so with parts of the v2 forward kernel
# removed (outputs are WRONG in these builds): tools/ubench/libablate_<mask>.so
set -e
cd "$(dirname "$0")/../.."
srcs=$(python -c "import dct_amd.build as b; print(' '.join('dct_amd/csrc/' + s for s in b.SOURCES))")
for m in ${@:-8 16 32}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
    -Wno-unused-command-line-argument -DDCTQ_ABLATE=$m -Iinclude -Idct_amd/csrc \
    $srcs \
    -o tools/ubench/libablate_$m.so &
done
wait
