#!/bin/bash
# tools/ubench/baseline.sh REV TAG -- build libdct_amd.so as of git revision REV
# (a temporary worktree, the same flags as dct_amd/build.py) into
# tools/ubench/libvar_TAG.so, the A/B baseline for tools/lib_ab.py / huf_ab.py.
set -e
cd "$(dirname "$0")/../.."
rev=$1; tag=$2
wt=$(mktemp -d /tmp/dctq_wt.XXXXXX)
git worktree add -f -q --detach "$wt" "$rev"
srcs=$(cd "$wt" && python -c "import dct_amd.build as b; print(' '.join('dct_amd/csrc/' + s for s in b.SOURCES))")
(cd "$wt" && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize \
  -Wno-unused-command-line-argument -Iinclude -Idct_amd/csrc $srcs -o "$OLDPWD/tools/ubench/libvar_$tag.so")
git worktree remove --force "$wt"
echo tools/ubench/libvar_$tag.so
