#!/bin/bash
# Diagnostic copy of libdct_amd.so with ONE source file replaced (A/B of a
# rewritten kernel against another version of it):
#   tools/ubench/variant_src.sh TAG huffman.hip /path/to/other/huffman.hip [-DFOO=1 ...]
#     ->  tools/ubench/libvar_TAG.so
set -e
cd "$(dirname "$0")/../.."
tag=$1; name=$2; alt=$3; shift 3
srcs=$(python -c "import dct_amd.build as b; print(' '.join(('$alt' if s == '$name' else 'dct_amd/csrc/' + s) for s in b.SOURCES))")
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -Wno-unused-command-line-argument "$@" -Iinclude -Idct_amd/csrc $srcs -o tools/ubench/libvar_$tag.so
