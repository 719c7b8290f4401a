"""Instruction histogram of one kernel (or its hottest loop) in a hipcc -S listing.

    python tools/isa_hist.py FILE.s SYMBOL_SUBSTRING [--loop]

--loop: restrict to the largest basic-block range between a backward branch
target label and the branch (the main loop)."""
import re
import sys
from collections import Counter


def body(lines, sym):
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith(sym + ":"):
            start = i
        elif start is not None and l.strip().startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("symbol not found")


def main():
    f, sym = sys.argv[1], sys.argv[2]
    lines = open(f).read().split("\n")
    cands = [l.split(":")[0] for l in lines if re.match(r"^[A-Za-z_]\S*:", l) and sym in l.split(":")[0]]
    if not cands:
        raise SystemExit("no symbol matches")
    b = body(lines, cands[0])
    if "--loop" in sys.argv:
        labels = {l.split(":")[0]: i for i, l in enumerate(b) if l.startswith(".LBB")}
        best = None
        for i, l in enumerate(b):
            m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
            if m and m.group(2) in labels and labels[m.group(2)] < i:
                span = (labels[m.group(2)], i)
                if best is None or span[1] - span[0] > best[1] - best[0]:
                    best = span
        b = b[best[0]:best[1] + 1]
        print("loop lines", best)
    c = Counter()
    for l in b:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        c[t.split()[0]] += 1
    tot = sum(c.values())
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(cands[0][:80], "instructions", tot, "VALU", valu)
    for k, v in c.most_common(45):
        print(f"{v:7d} {k}")


if __name__ == "__main__":
    main()
