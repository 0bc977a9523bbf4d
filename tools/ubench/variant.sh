#!/bin/bash
# Diagnostic copy of libdct_amd.so built with extra -D flags:
#   tools/ubench/variant.sh TAG -DFOO=1 ...   ->  tools/ubench/libvar_TAG.so
# DIAG=1 also links diag.hip (the diagnostic entry points: movement kernels for
# tools/lib_ab.py movement:PATH).
# PERFILE=1 compiles one object per source with dct_amd/build.py's flags and
# -cuid, then links -- the product's build structure (one code object per
# source); the default is one hipcc line over all sources (one code object).
set -e
tag=$1; shift
cd "$(dirname "$0")/../.."
srcs=$(python -c "import dct_amd.build as b; print(' '.join('dct_amd/csrc/' + s for s in b.SOURCES + (b.DIAG_SOURCES if '${DIAG:-0}' == '1' else [])))")
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wno-unused-command-line-argument -Iinclude -Idct_amd/csrc"
if [ "${PERFILE:-0}" = "1" ]; then
  od=$(mktemp -d /tmp/var_$tag.XXXX)
  objs=""
  for s in $srcs; do
    b=$(basename $s .hip)
    hipcc $flags "$@" -cuid=dctamd_$b -c $s -o $od/$b.o &
    objs="$objs $od/$b.o"
  done
  wait
  hipcc $flags -shared $objs -o tools/ubench/libvar_$tag.so
  rm -rf $od
else
  hipcc $flags -shared "$@" $srcs -o tools/ubench/libvar_$tag.so
fi
