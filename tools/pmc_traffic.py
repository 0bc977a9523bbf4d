#!/usr/bin/env python3
"""HBM traffic per fdct8 launch from two separate rocprofv3 --pmc passes.

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV --frames F --kind K [--quality Q --adaptive A]
                                [-o profiles/traffic.json]

The record carries the configuration and the sha256 of dct_amd/libdct_amd.so:
bench.py uses it only for a run with the same frames, kind, quality, adaptive
mode, launches per step and library build.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half of the
bytes of a coalesced streaming read (MI355X_MICROARCH.md "HBM"), so the read
side is doubled; WRITE_SIZE is exact for streaming stores.  bench.py launches
the luma planes and the chroma planes alternately (same kernel), and its
roofline `achieved` is the average over both launches, so the traffic is
averaged over every forward-quant dispatch the same way.
"""
import argparse
import csv
import hashlib
import json
import os
import statistics

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dct_amd", "libdct_amd.so")


def per_dispatch(path, counter, match):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and match in r["Kernel_Name"]:
            vals[int(r["Dispatch_Id"])] = vals.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--frames", type=int, required=True)
    ap.add_argument("--kind", required=True)
    ap.add_argument("--quality", type=int, default=50)
    ap.add_argument("--adaptive", type=int, default=0)
    ap.add_argument("--kernel", default="fdct8_quant_v")  # v2 or v3, whichever the dispatch ran
    ap.add_argument("--launches", type=int, default=1, help="forward-quant dispatches per bench step")
    ap.add_argument("-o", "--out", default="profiles/traffic.json")
    a = ap.parse_args()
    f = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not f or not w or len(f) % a.launches or len(w) % a.launches:
        raise SystemExit(f"expected groups of {a.launches} dispatches, got {len(f)} fetch / {len(w)} write")
    rd = 2 * statistics.mean(f) * 1024
    wr = statistics.mean(w) * 1024
    blocks = a.frames * (480 * 270 + 2 * 240 * 135) / a.launches  # average blocks per launch
    out = {"kernel": a.kernel, "frames": a.frames, "kind": a.kind, "quality": a.quality, "adaptive": a.adaptive,
           "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(), "dispatches": len(f),
           "launches_per_step": a.launches,
           "read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "bytes_per_launch": rd + wr,
           "algorithmic_bytes_per_launch": 192 * blocks, "traffic_over_algorithmic": (rd + wr) / (192 * blocks),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "bench.py --steps 3 --warmup 1 --no-cpu; read = 2*FETCH_SIZE KiB (gfx950 half-count), "
                     "write = WRITE_SIZE KiB; mean over all forward-quant dispatches"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
