#!/bin/bash
# SQ / traffic counters of the fused round trip (roundtrip8) and of its
# no-arithmetic twin (roundtrip_movement), bench step, one rocprofv3 --pmc pass
# per counter set (each under its own kill timeout):
#   bash tools/pmc_rt.sh [out_dir] [extra rt_one.py args...]
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_rt}
shift || true
mkdir -p $O
P="python tools/rt_one.py uniform 64 $*"
pass() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$n -o run --output-format csv -- $P > $O/$n.log 2>&1 || { echo "FAIL $n"; exit 1; }
}
pass a SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SALU
pass b SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pass f FETCH_SIZE
pass w WRITE_SIZE
# per-type VALU counts, when this box's counter list has them (optional pass)
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
if grep -q SQ_INSTS_VALU_FMA_F64 $O/counters.txt; then
  pass c SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32
fi
echo done
