#!/bin/bash
# SQ counters of huffman_bits_kernel per input kind (one rocprofv3 --pmc pass per counter set)
set -u
export TMPDIR=/tmp
O=gpurun_out/pmc_huf2
mkdir -p $O
for kind in uniform smooth; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $O/$kind -o run --output-format csv -- python tools/huf_one.py $kind > $O/$kind.log 2>&1 || exit 1
done
echo done
