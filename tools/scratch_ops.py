"""Every scratch (spill) access of one kernel in `hipcc -gline-tables-only -S`
output, with the source line it belongs to and the loop (compiler header
comment) it sits in: where a kernel's spills live and which loops reload them.

    python tools/scratch_ops.py kernels.s SYMBOL"""
import re
import sys


def main(path, sym):
    lines = open(path).read().split("\n")
    s = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    e = next(i for i in range(s, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    files = {}
    for l in lines[:s]:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[m.group(1)] = m.group(2).split("/")[-1]
    loc, cur = None, ""
    for i in range(s, e):
        l = lines[i]
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (files.get(m.group(1)), int(m.group(2)))
            continue
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):?", l):
            m = re.search(r"(?:Header=|Loop Header: Depth=)(\S+)", l)
            cur = re.search(r"(Loop Header: Depth=\d+|in Loop: Header=\S+ Depth=\d+)", l)
            cur = cur.group(1) if cur else ""
            continue
        if "scratch_" in l:
            print(f"{loc[0]}:{loc[1]:<5d} {l.strip():60s} {cur}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
