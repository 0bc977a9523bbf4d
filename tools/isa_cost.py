"""Static VALU cost of a kernel's main loop from its .s (gfx950 cost model,
profiles/r01/valu_issue_rates.md): full-rate ops 2.4 cycles, half-rate 4.35."""
import re
import sys
from collections import Counter

FULL = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|fmamk|fmaak|mac)_f32(_e32|_e64)?$|^v_(add|sub|subrev)_u32(_e32|_e64)?$|^v_(xor|and|or|lshlrev|lshrrev|ashrrev)_b32(_e32|_e64)?$|^v_mov_b32(_e32)?$|^v_(max|min)_f32(_e32)?$")


def cost(line):
    op = line.split()[0]
    if not op.startswith("v_") or op.startswith("v_readfirstlane") or op.startswith("v_readlane") or op.startswith("v_writelane"):
        return None
    sgpr = re.search(r"(?<![\w\[])s\[?\d", line.split(None, 1)[1] if " " in line else "")
    if FULL.match(op) and not sgpr and "_sdwa" not in op:
        return 2.4
    return 4.35


def main(path, kernel, start_pat=None, end_pat=None):
    s = open(path).read()
    st = s.index(kernel + ":")
    en = s.index(".Lfunc_end", st)
    body = [l.strip() for l in s[st:en].split("\n")]
    lo, hi = 0, len(body)
    if start_pat:
        lo = next(i for i, l in enumerate(body) if re.search(start_pat, l))
    if end_pat:
        hi = next(i for i in range(lo + 1, len(body)) if re.search(end_pat, body[i]))
    total, n, ops = 0.0, 0, Counter()
    for l in body[lo:hi]:
        if not l or l.startswith((".", ";")):
            continue
        c = cost(l)
        if c is None:
            continue
        total += c
        n += 1
        ops[(l.split()[0], c)] += 1
    print(f"{n} VALU instructions, est. {total:.0f} SIMD cycles per wave-iteration ({total/64:.1f} per block)")
    for (op, c), k in ops.most_common(25):
        print(f"  {op:28s} {c:4.2f} x{k}")


if __name__ == "__main__":
    main(*sys.argv[1:])
