#!/bin/bash
# Box-to-box spread of the forward kernel's movement pattern against the flat 1:2 stream:
# the box's partition modes, clocks and firmware, then bench.py's ceiling leg alone.
set -u
export TMPDIR=/tmp
O=gpurun_out/probe
mkdir -p $O
{ rocm-smi --showmemorypartition --showcomputepartition 2>&1; rocm-smi --showclocks 2>&1; rocm-smi --showfwinfo 2>&1 | grep -i -E "SMC|PSP|MC |VBIOS|RLC" ; rocm-smi --showserial --showuniqueid 2>&1; rocm-smi --showmemvendor 2>&1; rocm-smi -t 2>&1; } > $O/info.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu --round-trip-steps 0 --encode-steps 0 --ceiling-rounds 6 > $O/bench.log 2>&1
python - <<'PY'
import json
l = [x for x in open("gpurun_out/probe/bench.log") if x.startswith("{")][-1]
d = json.loads(l); h = d["roofline"]["movement_ceiling"]["hw_ceilings"]
print("forward %.1f movement %.1f flat %.1f flat_plain %.1f read %.1f write %.1f" % tuple(
    h[k]["median_us"] for k in ("forward", "movement_v2", "flat_1to2_nt_nt", "flat_1to2_nt_plain", "read_only", "write_only")))
PY
