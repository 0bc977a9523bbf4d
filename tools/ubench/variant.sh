#!/bin/bash
# Diagnostic copy of libdct_amd.so built with extra -D flags:
#   tools/ubench/variant.sh TAG -DFOO=1 ...   ->  tools/ubench/libvar_TAG.so
set -e
cd "$(dirname "$0")/../.."
tag=$1; shift
srcs=$(python -c "import dct_amd.build as b; print(' '.join('dct_amd/csrc/' + s for s in b.SOURCES))")
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -Wno-unused-command-line-argument "$@" -Iinclude -Idct_amd/csrc $srcs -o tools/ubench/libvar_$tag.so
