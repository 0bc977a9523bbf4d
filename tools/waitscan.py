#!/usr/bin/env python3
"""List the control flow, VMEM ops and vmcnt waits of one kernel in a .s file.

    python tools/waitscan.py FILE.s SUBSTRING_OF_MANGLED_NAME
"""
import sys

s = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
start = next(i for i, l in enumerate(s) if l.startswith("_Z") and key in l and l.rstrip().endswith(":") or
             (l.startswith("_Z") and key in l.split(":")[0]))
end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
for i in range(start, end):
    l = s[i].strip()
    if (("s_waitcnt" in l and "vmcnt" in l) or l.startswith(".LBB") or "s_cbranch" in l or l.startswith("s_branch")
            or "global_load" in l or "buffer_store" in l or "global_store" in l or "buffer_load" in l):
        print(i - start, l[:90])
