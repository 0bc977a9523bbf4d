#!/bin/bash
# Diagnostic copy of libdct_amd.so built with extra -D flags:
#   tools/ubench/variant.sh TAG -DFOO=1 ...   ->  tools/ubench/libvar_TAG.so
# DIAG=1 also links diag.hip (the diagnostic entry points: movement kernels for
# tools/lib_ab.py movement:PATH).
set -e
tag=$1; shift
cd "$(dirname "$0")/../.."
srcs=$(python -c "import dct_amd.build as b; print(' '.join('dct_amd/csrc/' + s for s in b.SOURCES + (b.DIAG_SOURCES if '${DIAG:-0}' == '1' else [])))")
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -Wno-unused-command-line-argument "$@" -Iinclude -Idct_amd/csrc $srcs -o tools/ubench/libvar_$tag.so
