#!/bin/bash
# SQ counters of huffman_bits_kernel per input kind (one rocprofv3 --pmc pass per counter set)
#   bash tools/pmc_huf.sh [out_dir] [kinds...]
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_huf3}
shift || true
KINDS=${*:-uniform smooth}
mkdir -p $O
for kind in $KINDS; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $O/${kind}_a -o run --output-format csv -- python tools/huf_one.py $kind > $O/${kind}_a.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE -d $O/${kind}_b -o run --output-format csv -- python tools/huf_one.py $kind > $O/${kind}_b.log 2>&1 || exit 1
done
echo done
