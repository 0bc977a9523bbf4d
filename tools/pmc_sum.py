"""Summarise rocprofv3 --pmc counter CSVs for one kernel: mean per dispatch,
and per 64-block tile when --tiles is given.
    python tools/pmc_sum.py KERNEL_SUBSTR [--tiles N] CSV..."""
import csv
import sys
from collections import defaultdict

args = sys.argv[1:]
kern = args.pop(0)
tiles = None
if args and args[0] == "--tiles":
    tiles = float(args[1])
    args = args[2:]
vals = defaultdict(list)
for path in args:
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    m = sum(v) / len(v)
    print(f"{k:24s} n={len(v):2d} mean {m:16.1f}" + (f"  per tile {m / tiles:10.2f}" if tiles else ""))
