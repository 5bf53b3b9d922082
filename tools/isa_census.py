"""Instruction census of one kernel from the compiler's assembly (VERDICT r04
item 6): every instruction of the kernel's hot path classified by opcode
class and, when the assembly carries a line table (-gline-tables-only), by
the source function it was inlined from; each loop's body weighted by its
trip count per signature, so the totals are dynamic VALU wave-instructions
per 64 signatures (one wave) and can be checked against the PMC count
(SQ_INSTS_VALU / (n / 64)).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -gline-tables-only -x hip \
        --cuda-device-only -S haskoin-node_amd/csrc/hkv_kernels.hip -o /tmp/k.s
    python tools/isa_census.py /tmp/k.s [--kernel SYMBOL] [--trips loops.json]

Hot path: the compiler places blocks a rare branch leads to (the carry-fold
continuations, the degenerate-addition fixes) out of line, after an
unconditional branch, reached only by a conditional branch; those blocks
(and loop headers' nothing else) are counted as cold (zero weight). Loop
trip counts per signature are given per loop header in source order (the
order the loops appear in the kernel), defaulting to the ecmult kernel's:
grid-stride 1, table forward 6, table backward 7, windows 33, doublings
4 (x 32 windows: 128 / 33 per window), slots 2."""
from __future__ import annotations

import argparse
import collections
import json
import re
import sys

DEFAULT_KERNEL = "_ZN3hkv17hkv_ecmult_kernelILb0ELb0EEEvPjjjS1_PyNS_7StdArgsE"


def classify(op: str) -> str:
    if op.startswith("s_nop"):
        return "s_nop (hazard pad)"
    if op.startswith("s_"):
        return "scalar"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        if "load" in op:
            return "vmem load"
        return "vmem store"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "v_mad_u64_u32"
    if re.match(r"v_(add|sub|subrev)_co_u32|v_addc_co_u32|v_subb_co_u32|v_subbrev_co_u32", op):
        return "carry add/sub"
    if op.startswith("v_cndmask"):
        return "select (v_cndmask)"
    if op.startswith(("v_mov_b32", "v_mov_b64", "v_accvgpr", "v_readlane", "v_readfirstlane", "v_writelane")):
        return "move"
    if op.startswith(("v_alignbit", "v_lshlrev", "v_lshrrev", "v_ashrrev", "v_lshl_", "v_bfe", "v_bfi",
                      "v_alignbyte", "v_perm")):
        return "shift/bitfield"
    if op.startswith(("v_xor", "v_and", "v_or", "v_not", "v_bitop3")):
        return "logic"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "compare"
    if op.startswith(("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_add3_u32", "v_mul_lo", "v_mul_hi",
                      "v_mul_u32", "v_lshl_add", "v_add_lshl", "v_mad_u32", "v_max", "v_min")):
        return "int add/mul (no carry)"
    if op.startswith("v_"):
        return "other valu"
    return "other"


def parse(path: str, kernel: str):
    """Blocks of the kernel: [(label, loop header or None, depth, header?, lines)]"""
    lines = open(path).read().splitlines()
    file_of = {}
    for l in lines:
        m = re.match(r"\s*\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", l)
        if m:
            file_of[m.group(1)] = m.group(2).split("/")[-1]
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks = []
    cur = {"label": "entry", "loop": None, "depth": 0, "header": False, "ins": []}
    loc = None
    for raw in lines[start + 1:end]:
        l = raw.rstrip()
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (m.group(1), int(m.group(2)))
            continue
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?(.*)$", l)
        if m:
            blocks.append(cur)
            rest = m.group(2)
            hm = re.search(r"Loop Header: Depth=(\d+)", rest)
            im = re.search(r"in Loop: Header=(\w+) Depth=(\d+)", rest)
            pm = re.search(r"Parent Loop (\w+) Depth=(\d+)", rest)
            label = m.group(1).lstrip("; %").replace("bb.", "bb")
            cur = {"label": label, "loop": None, "depth": 0, "header": bool(hm), "ins": []}
            if hm:
                cur["loop"] = label.lstrip(".L").replace("LBB", "BB") if label.startswith(".L") else label
                cur["depth"] = int(hm.group(1))
            elif im:
                cur["loop"], cur["depth"] = im.group(1), int(im.group(2))
            continue
        if re.match(r"^\s*;\s*=>\s*This (Inner )?Loop Header: Depth=(\d+)", l):
            cur["header"] = True
            cur["loop"] = cur["label"].lstrip(".L").replace("LBB", "BB")
            cur["depth"] = int(re.search(r"Depth=(\d+)", l).group(1))
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        cur["ins"].append((op, s, loc))
    blocks.append(cur)
    # parent of each loop (from the nesting in layout order)
    return [b for b in blocks if b["ins"] or b["header"]], file_of


def cold_blocks(blocks):
    """Blocks a rare branch leads to, counted with zero weight:
    1. rare diamonds: R ends in `s_branch T` and some block P ends in a
       conditional branch with {fall-through, target} = {R, T} — the carry /
       borrow continuations of the field chains (`__any(k != 0)`), whether
       the compiler placed them out of line or inline.
    Regions the rule cannot see (the degenerate T == acc doubling under
    __any(degen), a multi-block hammock) are given with --cold-range."""
    cold = set()
    label_at = {b["label"]: k for k, b in enumerate(blocks)}
    for k, p in enumerate(blocks):
        if not p["ins"] or not p["ins"][-1][0].startswith("s_cbranch") or k + 1 >= len(blocks):
            continue
        tgt = p["ins"][-1][1].split()[-1]
        fall = blocks[k + 1]["label"]
        for r, t in ((tgt, fall), (fall, tgt)):
            rb = blocks[label_at[r]] if r in label_at else None
            if rb and rb["ins"] and rb["ins"][-1][0] == "s_branch" and rb["ins"][-1][1].split()[-1] == t \
                    and not rb["header"]:
                cold.add(r)
    return cold


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default=DEFAULT_KERNEL)
    ap.add_argument("--trips", default=None, help="JSON list of trip counts per loop header, in layout order")
    ap.add_argument("--cold-range", action="append", default=[],
                    help="FIRST:LAST block labels (inclusive, layout order) to count as cold, e.g. the degenerate "
                         "T == acc doubling inside the accumulate loop, which the structural rule cannot see")
    ap.add_argument("--json", action="store_true")
    args = ap.parse_args()
    blocks, file_of = parse(args.asm, args.kernel)
    # gej_double's lines inside a gej_accumulate loop: the degenerate T == acc fix
    cold = cold_blocks(blocks)
    labels = [b["label"] for b in blocks]
    for rng in args.cold_range:
        a, _, z = rng.partition(":")
        i, j = labels.index(a), labels.index(z)
        cold.update(labels[i:j + 1])
    headers = [b["loop"] for b in blocks if b["header"]]
    trips = json.loads(args.trips) if args.trips else [1, 6, 7, 33, 128 / 33, 2]
    tripmap = {h: trips[i] if i < len(trips) else 1 for i, h in enumerate(headers)}
    # loop nesting: a header's parent is the loop of the block before it
    parent = {}
    for k, b in enumerate(blocks):
        if b["header"]:
            j = k - 1
            while j >= 0 and blocks[j]["loop"] is None:
                j -= 1
            # the enclosing loop is the innermost loop of lower depth seen before
            par = None
            for jj in range(k - 1, -1, -1):
                bb = blocks[jj]
                if bb["loop"] is not None and bb["depth"] == b["depth"] - 1:
                    par = bb["loop"]
                    break
            parent[b["loop"]] = par

    def weight(loop):
        w = 1.0
        while loop is not None:
            w *= tripmap.get(loop, 1)
            loop = parent.get(loop)
        return w

    by_class = collections.Counter()
    by_loop = collections.defaultdict(collections.Counter)
    by_func = collections.Counter()
    static_hot = collections.Counter()
    for b in blocks:
        if b["label"] in cold:
            continue
        w = weight(b["loop"])
        for op, s, loc in b["ins"]:
            c = classify(op)
            by_class[c] += w
            by_loop[b["loop"]][c] += w
            static_hot[c] += 1
            if loc is not None:
                by_func[(file_of.get(loc[0], loc[0]), loc[1], c)] += w
    valu = sum(v for c, v in by_class.items() if c not in ("scalar", "s_nop (hazard pad)", "vmem load", "vmem store",
                                                            "lds", "other"))
    out = {"kernel": args.kernel, "loops": {h: {"trips": tripmap[h], "parent": parent.get(h),
                                                 "weight": weight(h)} for h in headers},
           "per_wave_signature": {c: round(v, 1) for c, v in by_class.most_common()},
           "valu_total": round(valu, 1),
           "per_loop": {str(l): {c: round(v, 1) for c, v in cnt.most_common()} for l, cnt in by_loop.items()},
           "cold_blocks": len(cold), "blocks": len(blocks)}
    if by_func:
        agg = collections.defaultdict(collections.Counter)
        for (f, line, c), v in by_func.items():
            agg[(f, line)][c] += v
        out["top_lines"] = [{"file": f, "line": line, "total": round(sum(cnt.values()), 1),
                             "classes": {c: round(v, 1) for c, v in cnt.most_common()}}
                            for (f, line), cnt in sorted(agg.items(), key=lambda kv: -sum(kv[1].values()))[:60]]
    if args.json:
        print(json.dumps(out, indent=1))
        return
    print(f"kernel {args.kernel}: {len(blocks)} blocks, {len(cold)} cold")
    for h in headers:
        print(f"  loop {h}: trips {tripmap[h]:.3g} parent {parent.get(h)} weight {weight(h):.4g}")
    print(f"dynamic instructions per wave (64 signatures), hot path: VALU {valu:,.0f}")
    for c, v in by_class.most_common():
        print(f"  {c:28s} {v:12,.0f}   (static hot {static_hot[c]})")
    for l, cnt in by_loop.items():
        print(f"  loop {l}: " + ", ".join(f"{c} {v:,.0f}" for c, v in cnt.most_common(8)))
    if by_func:
        print("top source lines:")
        for row in out["top_lines"][:40]:
            print(f"  {row['file']}:{row['line']:<5d} {row['total']:10,.0f}  {row['classes']}")


if __name__ == "__main__":
    sys.exit(main())
