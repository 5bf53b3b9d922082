import sys, collections
sys.path.insert(0, "/root/repo/tools")
import isa_census as ic
blocks, file_of = ic.parse(sys.argv[1], sys.argv[2])
cold = ic.cold_blocks(blocks)
loops = collections.OrderedDict()
for b in blocks:
    if b["loop"] is None: continue
    d = loops.setdefault(b["loop"], {"depth": b["depth"], "ins": 0, "lane": 0, "scratch": 0, "locs": collections.Counter(), "spl": collections.Counter()})
    if b["label"] in cold: continue
    for op, s, loc in b["ins"]:
        d["ins"] += 1
        if loc: d["locs"][(file_of.get(loc[0], loc[0]), loc[1])] += 1
        if op.startswith(("v_writelane", "v_readlane")):
            d["lane"] += 1; d["spl"][(op, file_of.get(loc[0], loc[0]) if loc else None, loc[1] if loc else None)] += 1
        if op.startswith("scratch_") or (op.startswith("buffer_") and "off" in s):
            d["scratch"] += 1
for h, d in loops.items():
    if d["ins"] < 100: continue
    top = ", ".join(f"{f}:{l}" for (f, l), _ in d["locs"].most_common(3))
    print(f"{h} depth {d['depth']}: {d['ins']} hot insts, lane spills {d['lane']}, scratch {d['scratch']}  [{top}]")
    for k, v in d["spl"].most_common(6):
        print("     ", v, k)
