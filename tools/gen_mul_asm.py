"""Generate haskoin-node_amd/csrc/hkv_mul_asm.h: 256x256 -> 512-bit product
by product scanning (column-wise) in gfx950 inline asm.

Per product: one v_mad_u64_u32 into the column's 64-bit accumulator (its
carry-out goes to an SGPR pair) and one v_addc_co_u32 that adds that carry
into the column's top word. The carry is consumed >= 2 instructions after it
is written (gfx950 VALU-writes-SGPR -> VALU-reads-SGPR spacing); three SGPR
pairs rotate. Between columns the accumulator shifts by 32 bits (C level).

    python tools/gen_mul_asm.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "haskoin-node_amd", "csrc", "hkv_mul_asm.h")


def column_block(k, pairs, name):
    """asm for one column: products `pairs` = [(i, j)], acc "+v", top "=&v"."""
    m = len(pairs)
    lines = []
    ops_in = []
    # operands: %0 acc, %1 top, %2..%4 carry pairs, then a/b regs
    regs = {}
    for (i, j) in pairs:
        for nm in (f"a{i}", f"b{j}"):
            if nm not in regs:
                regs[nm] = len(regs)
    base = 5
    ref = lambda nm: f"%{base + regs[nm]}"
    seq = []  # (kind, p)
    # schedule: mad_p at position, addc_p after mad_{p+2} (or at the end)
    for p in range(m):
        seq.append(("mad", p))
        if p - 2 >= 0:
            seq.append(("add", p - 2))
    for p in range(max(0, m - 2), m):
        seq.append(("add", p))
    emitted_mad = {}
    first_add = True
    for idx, (kind, p) in enumerate(seq):
        c = f"%{2 + p % 3}"
        if kind == "mad":
            i, j = pairs[p]
            lines.append(f"v_mad_u64_u32 %0, {c}, {ref('a%d' % i)}, {ref('b%d' % j)}, %0")
            emitted_mad[p] = len(lines) - 1
        else:
            # spacing since the mad that wrote carry p
            dist = len(lines) - 1 - emitted_mad[p]
            if dist < 2:
                lines.append(f"s_nop {1 - dist}")
            if first_add:
                lines.append(f"v_addc_co_u32_e64 %1, {c}, 0, 0, {c}")
                first_add = False
            else:
                lines.append(f"v_addc_co_u32_e64 %1, {c}, %1, 0, {c}")
    asm = "\\n\\t".join(lines)
    ins = ", ".join(f'"v"({nm[0]}[{nm[1:]}])' for nm in regs)
    return (f'  asm("{asm}"\n      : "+v"(acc), "=&v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2)\n'
            f'      : {ins});')


def column_block2(k, pairs1, pairs2):
    """asm for column k of two independent products interleaved mad by mad:
    %0 acc1, %1 top1, %2 acc2, %3 top2 (64-bit accs "+v", tops "=&v"),
    %4 %5 carry pairs of product 1, %6 %7 of product 2, then the a/b regs
    (names a*, b* for product 1 and c*, d* for product 2). A product's carry
    is read >= 2 instructions after its mad (the other product's instructions
    fill the gap that s_nop fills in the single form), so two rotating SGPR
    pairs per product suffice."""
    regs = {}
    for (i, j) in pairs1:
        for nm in (f"a{i}", f"b{j}"):
            regs.setdefault(nm, len(regs))
    for (i, j) in pairs2:
        for nm in (f"c{i}", f"d{j}"):
            regs.setdefault(nm, len(regs))
    base = 8
    ref = lambda nm: f"%{base + regs[nm]}"
    streams = []
    for q, (pairs, an, bn) in enumerate(((pairs1, "a", "b"), (pairs2, "c", "d"))):
        seq = []
        m = len(pairs)
        for p in range(m):
            seq.append(("mad", q, p, pairs[p], an, bn))
            if p - 1 >= 0:
                seq.append(("add", q, p - 1, None, an, bn))
        if m:
            seq.append(("add", q, m - 1, None, an, bn))
        streams.append(seq)
    # interleave the two streams item by item
    merged = []
    for x in range(max(len(streams[0]), len(streams[1]))):
        for q in (0, 1):
            if x < len(streams[q]):
                merged.append(streams[q][x])
    lines = []
    emitted = {}
    first_add = [True, True]
    acc = ["%0", "%2"]
    top = ["%1", "%3"]
    for kind, q, p, pr, an, bn in merged:
        c = f"%{4 + 2 * q + p % 2}"
        if kind == "mad":
            i, j = pr
            lines.append(f"v_mad_u64_u32 {acc[q]}, {c}, {ref(an + str(i))}, {ref(bn + str(j))}, {acc[q]}")
            emitted[(q, p)] = len(lines) - 1
        else:
            dist = len(lines) - 1 - emitted[(q, p)]
            if dist < 2:
                lines.append(f"s_nop {1 - dist}")
            if first_add[q]:
                lines.append(f"v_addc_co_u32_e64 {top[q]}, {c}, 0, 0, {c}")
                first_add[q] = False
            else:
                lines.append(f"v_addc_co_u32_e64 {top[q]}, {c}, {top[q]}, 0, {c}")
    asm = "\\n\\t".join(lines)
    ins = ", ".join(f'"v"({nm[0]}[{nm[1:]}])' for nm in regs)
    return (f'  asm("{asm}"\n      : "+v"(acc1), "=&v"(top1), "+v"(acc2), "=&v"(top2), "=&s"(c0), "=&s"(c1), "=&s"(e0), "=&s"(e1)\n'
            f'      : {ins});')


def pair_functions():
    out = ["",
           "// Two independent 256x256 products with their columns interleaved mad by",
           "// mad: at one wave per SIMD (the small-batch split kernel) each mad's",
           "// dependency latency is filled by the other product's instructions.",
           "__device__ __forceinline__ void mul256_ps2(uint32_t t1[16], const uint32_t* a, const uint32_t* b,",
           "                                           uint32_t t2[16], const uint32_t* c, const uint32_t* d) {",
           "  uint64_t acc1 = 0, acc2 = 0;",
           "  uint32_t top1, top2;",
           "  uint64_t c0, c1, e0, e1;"]
    for k in range(15):
        pairs = [(i, k - i) for i in range(8) if 0 <= k - i < 8]
        out.append(f"  // column {k}: 2 x {len(pairs)} products")
        out.append(column_block2(k, pairs, pairs))
        out.append(f"  t1[{k}] = (uint32_t)acc1;")
        out.append(f"  t2[{k}] = (uint32_t)acc2;")
        out.append("  acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);")
        out.append("  acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);")
    out.append("  t1[15] = (uint32_t)acc1;")
    out.append("  t2[15] = (uint32_t)acc2;")
    out.append("  (void)c0; (void)c1; (void)e0; (void)e1;")
    out.append("}")
    out.append("")
    out.append("// 2*o + diagonal squares of one operand (the tail of a squaring)")
    out.append("__device__ __forceinline__ void sqr_tail(uint32_t t[16], const uint32_t o[16], const uint32_t* a) {")
    out.append("  uint32_t cy = 0;")
    out.append("#pragma unroll")
    out.append("  for (int i = 0; i < 8; ++i) {")
    out.append("    const uint64_t dd = (uint64_t)a[i] * a[i];")
    out.append("    const uint32_t s0 = (i == 0) ? (o[0] << 1) : __builtin_amdgcn_alignbit(o[2 * i], o[2 * i - 1], 31);")
    out.append("    const uint32_t s1 = __builtin_amdgcn_alignbit(o[2 * i + 1], o[2 * i], 31);")
    out.append("    t[2 * i] = __builtin_addc(s0, (uint32_t)dd, cy, &cy);")
    out.append("    t[2 * i + 1] = __builtin_addc(s1, (uint32_t)(dd >> 32), cy, &cy);")
    out.append("  }")
    out.append("}")
    out.append("")
    out.append("// two independent squarings, off-diagonal scans interleaved")
    out.append("__device__ __forceinline__ void sqr256_ps2(uint32_t t1[16], const uint32_t* a, uint32_t t2[16], const uint32_t* c) {")
    out.append("  const uint32_t* b = a;")
    out.append("  const uint32_t* d = c;")
    out.append("  uint32_t o1[16], o2[16];")
    out.append("  uint64_t acc1 = 0, acc2 = 0;")
    out.append("  uint32_t top1, top2;")
    out.append("  uint64_t c0, c1, e0, e1;")
    out.append("  o1[0] = 0;")
    out.append("  o2[0] = 0;")
    for k in range(1, 14):
        pairs = [(i, k - i) for i in range(8) if 0 <= k - i < 8 and i < k - i]
        out.append(f"  // column {k}: 2 x {len(pairs)} off-diagonal products")
        out.append(column_block2(k, pairs, pairs))
        out.append(f"  o1[{k}] = (uint32_t)acc1;")
        out.append(f"  o2[{k}] = (uint32_t)acc2;")
        out.append("  acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);")
        out.append("  acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);")
    out.append("  o1[14] = (uint32_t)acc1;")
    out.append("  o1[15] = (uint32_t)(acc1 >> 32);")
    out.append("  o2[14] = (uint32_t)acc2;")
    out.append("  o2[15] = (uint32_t)(acc2 >> 32);")
    out.append("  (void)c0; (void)c1; (void)e0; (void)e1;")
    out.append("  sqr_tail(t1, o1, a);")
    out.append("  sqr_tail(t2, o2, c);")
    out.append("}")
    out.append("")
    out.append("// a squaring (t1 = a^2) beside an independent product (t2 = c * d)")
    out.append("__device__ __forceinline__ void sqrmul256_ps2(uint32_t t1[16], const uint32_t* a, uint32_t t2[16], const uint32_t* c,")
    out.append("                                              const uint32_t* d) {")
    out.append("  const uint32_t* b = a;")
    out.append("  uint32_t o1[16];")
    out.append("  uint64_t acc1 = 0, acc2 = 0;")
    out.append("  uint32_t top1, top2;")
    out.append("  uint64_t c0, c1, e0, e1;")
    out.append("  o1[0] = 0;")
    for k in range(15):
        p1 = [(i, k - i) for i in range(8) if 0 <= k - i < 8 and i < k - i]
        p2 = [(i, k - i) for i in range(8) if 0 <= k - i < 8]
        out.append(f"  // column {k}: {len(p1)} off-diagonal + {len(p2)} products")
        out.append(column_block2(k, p1, p2))
        if 1 <= k <= 13:
            out.append(f"  o1[{k}] = (uint32_t)acc1;")
            out.append("  acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);")
        out.append(f"  t2[{k}] = (uint32_t)acc2;")
        out.append("  acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);")
    out.append("  o1[14] = (uint32_t)acc1;")
    out.append("  o1[15] = (uint32_t)(acc1 >> 32);")
    out.append("  t2[15] = (uint32_t)acc2;")
    out.append("  (void)c0; (void)c1; (void)e0; (void)e1;")
    out.append("  sqr_tail(t1, o1, a);")
    out.append("}")
    return out


def scan_block(pairs, mode):
    """asm for one column of the reduced scan (mul256_red_ps / sqr256_red_ps).

    pairs: [(x, y)] C expressions of the 32-bit limb operands of the column's
    products. mode:
      "acc"  -- acc is "+v" (C-level carry-in, as in column_block)
      "red0" -- low column 0: acc = h0 * 977 (no carry-in)
      "red"  -- low column j >= 1: acc = prevhi + init, init = (top_prev << 32) | h[j-1],
                then acc += h[j] * 977. Both sums stay below 2^43, so their
                carry-outs are discarded (written to %2 before any product).
    Operands: %0 acc, %1 top, %2..%4 carry pairs; then (red modes) the prefix
    operands; then the limb operands."""
    regs = {}
    for (x, y) in pairs:
        for nm in (x, y):
            regs.setdefault(nm, len(regs))
    lines = []
    if mode == "acc":
        pre_ins = []
    elif mode in ("red0", "red0e"):
        pre_ins = ['"v"(h[0])', '"s"(k977)']
        lines.append("v_mad_u64_u32 %0, %2, %5, %6, 0")
        if mode == "red0e":  # + the addend's limb 0 (the sum stays below 2^43)
            pre_ins.append('"v"(ej)')
            lines.append("v_mad_u64_u32 %0, %2, %7, 1, %0")
    else:
        pre_ins = ['"v"(prevhi)', '"v"(init)', '"v"(hj)', '"s"(k977)']
        lines.append("v_mad_u64_u32 %0, %2, %5, 1, %6")
        lines.append("v_mad_u64_u32 %0, %2, %7, %8, %0")
        if mode == "rede":  # + the addend's limb j
            pre_ins.append('"v"(ej)')
            lines.append("v_mad_u64_u32 %0, %2, %9, 1, %0")
    base = 5 + len(pre_ins)
    ref = lambda nm: f"%{base + regs[nm]}"
    m = len(pairs)
    seq = []
    for p in range(m):
        seq.append(("mad", p))
        if p - 2 >= 0:
            seq.append(("add", p - 2))
    for p in range(max(0, m - 2), m):
        seq.append(("add", p))
    emitted_mad = {}
    first_add = True
    for kind, p in seq:
        c = f"%{2 + p % 3}"
        if kind == "mad":
            x, y = pairs[p]
            lines.append(f"v_mad_u64_u32 %0, {c}, {ref(x)}, {ref(y)}, %0")
            emitted_mad[p] = len(lines) - 1
        else:
            dist = len(lines) - 1 - emitted_mad[p]
            if dist < 2:
                lines.append(f"s_nop {1 - dist}")
            if first_add:
                lines.append(f"v_addc_co_u32_e64 %1, {c}, 0, 0, {c}")
                first_add = False
            else:
                lines.append(f"v_addc_co_u32_e64 %1, {c}, %1, 0, {c}")
    asm = "\\n\\t".join(lines)
    accc = '"+v"(acc)' if mode == "acc" else '"=&v"(accn)'
    ins = ", ".join(pre_ins + [f'"v"({nm})' for nm in regs])
    return (f'  asm("{asm}"\n      : {accc}, "=&v"(top), "=&s"(c0), "=&s"(c1), "=&s"(c2)\n'
            f'      : {ins});')


def reduced_scan(name, cols, doc, addend=False):
    """A 256x256 product given as column pair lists cols[0..14], reduced mod p
    on the fly: columns 8..14 are scanned first (their carry-in from column 7
    is deferred), giving the high half h[0..7]; columns 0..7 then fold
    h * 2^256 == h * (2^32 + 977) into their accumulators (h[j] * 977 and
    h[j-1] enter column j). Output: r[0..7] and T < 2^38 with
    a * b == r + T * 2^256 (mod p)."""
    sig = "uint32_t r[8], uint64_t& T, const uint32_t* a, const uint32_t* b" + (", const uint32_t* e" if addend else "")
    out = [""] + ["// " + l for l in doc] + [
        f"__device__ __forceinline__ void {name}({sig}) {{",
        "  uint64_t acc = 0;",
        "  uint32_t top;",
        "  uint64_t c0, c1, c2;",
        "  uint32_t h[8], o[8];",
        "  const uint32_t k977 = 977u;"]
    if "sqr" in name:
        out += ["  (void)b;",
                "  // row i of the square multiplies a_i by X_i = a_i + 2 * sum_{j>i} a_j 2^(32(j-i)),",
                "  // whose limbs are a_i, e[i+1] = a_{i+1} << 1, then d[i+k] = (a_{i+k} << 1) | (a_{i+k-1} >> 31)",
                "  uint32_t e[8], d[9];",
                "#pragma unroll",
                "  for (int j = 1; j < 8; ++j) e[j] = a[j] << 1;",
                "#pragma unroll",
                "  for (int j = 2; j < 8; ++j) d[j] = __builtin_amdgcn_alignbit(a[j], a[j - 1], 31);",
                "  d[8] = a[7] >> 31;"]
    for k in range(8, 15):
        out.append(f"  // column {k}: {len(cols[k])} products")
        out.append(scan_block(cols[k], "acc"))
        out.append(f"  h[{k - 8}] = (uint32_t)acc;")
        out.append("  acc = (acc >> 32) | ((uint64_t)top << 32);")
    out.append("  h[7] = (uint32_t)acc;  // the high half is < 2^256: nothing above")
    for j in range(8):
        out.append(f"  // column {j}: {len(cols[j])} products + h[{j}] * 977" + (f" + h[{j - 1}]" if j else ""))
        out.append("  {")
        out.append("    uint64_t accn;")
        if addend:
            out.append(f"    const uint32_t ej = e[{j}];")
        if j:
            out.append("    const uint32_t prevhi = (uint32_t)(acc >> 32);")
            out.append(f"    const uint64_t init = ((uint64_t)top << 32) | h[{j - 1}];")
            out.append(f"    const uint32_t hj = h[{j}];")
            blk = scan_block(cols[j], "rede" if addend else "red")
        else:
            blk = scan_block(cols[j], "red0e" if addend else "red0")
        out.append("  " + blk.replace("\n", "\n  "))
        out.append("    acc = accn;")
        out.append("  }")
        out.append(f"  o[{j}] = (uint32_t)acc;")
    out.append("  T = (acc >> 32) + ((uint64_t)top << 32) + h[7];")
    out.append("  // r may alias a or b (fe_mul(x, x, y)): written only after the last column")
    out.append("#pragma unroll")
    out.append("  for (int j = 0; j < 8; ++j) r[j] = o[j];")
    out.append("  (void)c0; (void)c1; (void)c2;")
    out.append("}")
    return out


def reduced_functions():
    mul_cols = [[(f"a[{i}]", f"b[{k - i}]") for i in range(8) if 0 <= k - i < 8] for k in range(15)]
    sqr_cols = [[] for _ in range(16)]
    for i in range(8):
        sqr_cols[2 * i].append((f"a[{i}]", f"a[{i}]"))
        if i <= 6:
            sqr_cols[2 * i + 1].append((f"a[{i}]", f"e[{i + 1}]"))
        for j in range(i + 2, 9):
            sqr_cols[i + j].append((f"a[{i}]", f"d[{j}]"))
    assert not sqr_cols[15] and sum(map(len, sqr_cols)) == 43
    out = reduced_scan("mul256_red_ps", mul_cols, [
        "a * b mod p with the reduction folded into the product scan (HKV_MUL_RED):",
        "no separate 8-mad reduction chain, its limb moves or its two 8-limb",
        "add chains; a column's carry-in and h[j-1] enter through one mad (x 1)."])
    out += reduced_scan("mul256_red_add_ps", mul_cols, [
        "a * b + e mod p (e < 2^256): mul256_red_ps with the addend's limb j",
        "entering low column j through one more mad (x 1) — a product and an",
        "addition for one extra instruction per low column, no carry chain."], addend=True)
    out += reduced_scan("sqr256_red_ps", sqr_cols[:15], [
        "a^2 mod p as a column scan of 43 products (8 squares, 7 a_i * 2a_{i+1},",
        "28 a_i * (2a)_j limbs incl. the 1-bit limb 8) instead of 36 products plus",
        "a shift-and-add pass over 16 words, with the same folded reduction."])
    return out


def scan_block2(pairs1, pairs2, mode):
    """Two reduced-scan columns (scan_block) interleaved mad by mad, for the
    paired forms. %0 acc1, %1 top1, %2 acc2, %3 top2, %4 %5 carry pairs of
    stream 1, %6 %7 of stream 2, then the prefix operands of both streams
    (red modes), then the limb operands."""
    regs = {}
    for (x, y) in pairs1 + pairs2:
        for nm in (x, y):
            regs.setdefault(nm, len(regs))
    lines = []
    if mode == "acc":
        pre_ins = []
    elif mode == "red0":
        pre_ins = ['"v"(h1[0])', '"v"(h2[0])', '"s"(k977)']
        lines.append("v_mad_u64_u32 %0, %4, %8, %10, 0")
        lines.append("v_mad_u64_u32 %2, %6, %9, %10, 0")
    else:
        pre_ins = ['"v"(prevhi1)', '"v"(init1)', '"v"(hj1)', '"v"(prevhi2)', '"v"(init2)', '"v"(hj2)', '"s"(k977)']
        lines.append("v_mad_u64_u32 %0, %4, %8, 1, %9")
        lines.append("v_mad_u64_u32 %2, %6, %11, 1, %12")
        lines.append("v_mad_u64_u32 %0, %4, %10, %14, %0")
        lines.append("v_mad_u64_u32 %2, %6, %13, %14, %2")
    base = 8 + len(pre_ins)
    ref = lambda nm: f"%{base + regs[nm]}"
    streams = []
    for q, pairs in enumerate((pairs1, pairs2)):
        seq = []
        m = len(pairs)
        for p in range(m):
            seq.append(("mad", q, p, pairs[p]))
            if p - 1 >= 0:
                seq.append(("add", q, p - 1, None))
        if m:
            seq.append(("add", q, m - 1, None))
        streams.append(seq)
    merged = []
    for x in range(max(len(streams[0]), len(streams[1]))):
        for q in (0, 1):
            if x < len(streams[q]):
                merged.append(streams[q][x])
    emitted = {}
    first_add = [True, True]
    acc = ["%0", "%2"]
    top = ["%1", "%3"]
    for kind, q, p, pr in merged:
        c = f"%{4 + 2 * q + p % 2}"
        if kind == "mad":
            x, y = pr
            lines.append(f"v_mad_u64_u32 {acc[q]}, {c}, {ref(x)}, {ref(y)}, {acc[q]}")
            emitted[(q, p)] = len(lines) - 1
        else:
            dist = len(lines) - 1 - emitted[(q, p)]
            if dist < 2:
                lines.append(f"s_nop {1 - dist}")
            if first_add[q]:
                lines.append(f"v_addc_co_u32_e64 {top[q]}, {c}, 0, 0, {c}")
                first_add[q] = False
            else:
                lines.append(f"v_addc_co_u32_e64 {top[q]}, {c}, {top[q]}, 0, {c}")
    asm = "\\n\\t".join(lines)
    accc = '"+v"(acc1), "=&v"(top1), "+v"(acc2), "=&v"(top2)' if mode == "acc" else \
        '"=&v"(accn1), "=&v"(top1), "=&v"(accn2), "=&v"(top2)'
    ins = ", ".join(pre_ins + [f'"v"({nm})' for nm in regs])
    return (f'  asm("{asm}"\n      : {accc}, "=&s"(c0), "=&s"(c1), "=&s"(e0), "=&s"(e1)\n'
            f'      : {ins});')


def sqr_prep(src, e, d):
    return [f"  uint32_t {e}[8], {d}[9];",
            "#pragma unroll",
            f"  for (int j = 1; j < 8; ++j) {e}[j] = {src}[j] << 1;",
            "#pragma unroll",
            f"  for (int j = 2; j < 8; ++j) {d}[j] = __builtin_amdgcn_alignbit({src}[j], {src}[j - 1], 31);",
            f"  {d}[8] = {src}[7] >> 31;"]


def reduced_scan2(name, sig, cols1, cols2, preps, doc):
    out = [""] + ["// " + l for l in doc] + [
        f"__device__ __forceinline__ void {name}({sig}) {{",
        "  uint64_t acc1 = 0, acc2 = 0;",
        "  uint32_t top1, top2;",
        "  uint64_t c0, c1, e0, e1;",
        "  uint32_t h1[8], h2[8], o1[8], o2[8];",
        "  const uint32_t k977 = 977u;"]
    for pr in preps:
        out += sqr_prep(*pr)
    for k in range(8, 15):
        out.append(f"  // column {k}: {len(cols1[k])} + {len(cols2[k])} products")
        out.append(scan_block2(cols1[k], cols2[k], "acc"))
        out.append(f"  h1[{k - 8}] = (uint32_t)acc1;")
        out.append(f"  h2[{k - 8}] = (uint32_t)acc2;")
        out.append("  acc1 = (acc1 >> 32) | ((uint64_t)top1 << 32);")
        out.append("  acc2 = (acc2 >> 32) | ((uint64_t)top2 << 32);")
    out.append("  h1[7] = (uint32_t)acc1;")
    out.append("  h2[7] = (uint32_t)acc2;")
    for j in range(8):
        out.append(f"  // column {j}: {len(cols1[j])} + {len(cols2[j])} products + the folded high limbs")
        out.append("  {")
        out.append("    uint64_t accn1, accn2;")
        if j:
            for q in (1, 2):
                out.append(f"    const uint32_t prevhi{q} = (uint32_t)(acc{q} >> 32);")
                out.append(f"    const uint64_t init{q} = ((uint64_t)top{q} << 32) | h{q}[{j - 1}];")
                out.append(f"    const uint32_t hj{q} = h{q}[{j}];")
            blk = scan_block2(cols1[j], cols2[j], "red")
        else:
            blk = scan_block2(cols1[j], cols2[j], "red0")
        out.append("  " + blk.replace("\n", "\n  "))
        out.append("    acc1 = accn1;")
        out.append("    acc2 = accn2;")
        out.append("  }")
        out.append(f"  o1[{j}] = (uint32_t)acc1;")
        out.append(f"  o2[{j}] = (uint32_t)acc2;")
    out.append("  T1 = (acc1 >> 32) + ((uint64_t)top1 << 32) + h1[7];")
    out.append("  T2 = (acc2 >> 32) + ((uint64_t)top2 << 32) + h2[7];")
    out.append("#pragma unroll")
    out.append("  for (int j = 0; j < 8; ++j) { r1[j] = o1[j]; r2[j] = o2[j]; }")
    out.append("  (void)c0; (void)c1; (void)e0; (void)e1;")
    out.append("}")
    return out


def col_lists(kind, x, y=None):
    if kind == "mul":
        return [[(f"{x}[{i}]", f"{y}[{k - i}]") for i in range(8) if 0 <= k - i < 8] for k in range(15)]
    e, d = y
    cols = [[] for _ in range(16)]
    for i in range(8):
        cols[2 * i].append((f"{x}[{i}]", f"{x}[{i}]"))
        if i <= 6:
            cols[2 * i + 1].append((f"{x}[{i}]", f"{e}[{i + 1}]"))
        for j in range(i + 2, 9):
            cols[i + j].append((f"{x}[{i}]", f"{d}[{j}]"))
    return cols[:15]


def reduced_pair_functions():
    out = reduced_scan2(
        "mul256_red_ps2",
        "uint32_t r1[8], uint64_t& T1, const uint32_t* a, const uint32_t* b, uint32_t r2[8], uint64_t& T2, "
        "const uint32_t* c, const uint32_t* d",
        col_lists("mul", "a", "b"), col_lists("mul", "c", "d"), [],
        ["two independent folded-reduction products (mul256_red_ps) interleaved mad by mad"])
    out += reduced_scan2(
        "sqr256_red_ps2",
        "uint32_t r1[8], uint64_t& T1, const uint32_t* a, uint32_t r2[8], uint64_t& T2, const uint32_t* c",
        col_lists("sqr", "a", ("ea", "da")), col_lists("sqr", "c", ("ec", "dc")), [("a", "ea", "da"), ("c", "ec", "dc")],
        ["two independent folded-reduction squares (sqr256_red_ps) interleaved mad by mad"])
    out += reduced_scan2(
        "sqrmul256_red_ps2",
        "uint32_t r1[8], uint64_t& T1, const uint32_t* a, uint32_t r2[8], uint64_t& T2, const uint32_t* c, "
        "const uint32_t* d",
        col_lists("sqr", "a", ("ea", "da")), col_lists("mul", "c", "d"), [("a", "ea", "da")],
        ["a folded-reduction square beside an independent product, interleaved mad by mad"])
    return out


def row_functions():
    """Partial products of R rows of a (R limbs) by all 8 limbs of b: the
    lane-split products (hkv_field.h fe_mul_rows2 / fe_mul_rows4) give each
    lane of a pair or quad R = 4 or 2 rows of one 256 x 256 product, and
    the lanes' partials are summed across lanes (DPP) before one reduction."""
    out = [""]
    for R in (4, 2):
        n_out = R + 8
        out.append(f"// {R} x 8 limb product (rows a[0..{R - 1}] by b[0..7]) -> {n_out} limbs")
        out.append(f"__device__ __forceinline__ void mul{R}x8_ps(uint32_t t[{n_out}], const uint32_t* a, "
                   f"const uint32_t* b) {{")
        out.append("  uint64_t acc = 0;")
        out.append("  uint32_t top;")
        out.append("  uint64_t c0, c1, c2;")
        for k in range(R + 7):
            pairs = [(i, k - i) for i in range(R) if 0 <= k - i < 8]
            out.append(f"  // column {k}: {len(pairs)} products")
            out.append(column_block(k, pairs, "rows"))
            out.append(f"  t[{k}] = (uint32_t)acc;")
            out.append("  acc = (acc >> 32) | ((uint64_t)top << 32);")
        out.append(f"  t[{n_out - 1}] = (uint32_t)acc;")
        out.append("  (void)c0; (void)c1; (void)c2;")
        out.append("}")
    return out


def main():
    out = ["// GENERATED by tools/gen_mul_asm.py — do not edit.",
           "// 256x256 -> 512-bit product, product scanning in gfx950 inline asm",
           "// (one v_mad_u64_u32 + one v_addc_co_u32 per limb product).",
           "#pragma once",
           "#include <stdint.h>",
           "",
           "namespace hkv {",
           "",
           "__device__ __forceinline__ void mul256_ps(uint32_t t[16], const uint32_t* a, const uint32_t* b) {",
           "  uint64_t acc = 0;",
           "  uint32_t top;",
           "  uint64_t c0, c1, c2;"]
    for k in range(15):
        pairs = [(i, k - i) for i in range(8) if 0 <= k - i < 8]
        out.append(f"  // column {k}: {len(pairs)} products")
        out.append(column_block(k, pairs, "mul"))
        out.append(f"  t[{k}] = (uint32_t)acc;")
        out.append("  acc = (acc >> 32) | ((uint64_t)top << 32);")
    out.append("  t[15] = (uint32_t)acc;")
    out.append("  (void)c0; (void)c1; (void)c2;")
    out.append("}")
    out.append("")
    # squaring: off-diagonal product scan, then t = 2*o + diag in one carry chain
    out.append("// 256-bit square: product scan of the 28 off-diagonal products a_i*a_j (i<j),")
    out.append("// then t = 2*o + sum a_i^2 * 2^(64 i) in one shift-and-add pass.")
    out.append("__device__ __forceinline__ void sqr256_ps(uint32_t t[16], const uint32_t* a) {")
    out.append("  const uint32_t* b = a;")
    out.append("  uint32_t o[16];")
    out.append("  uint64_t acc = 0;")
    out.append("  uint32_t top;")
    out.append("  uint64_t c0, c1, c2;")
    out.append("  o[0] = 0;")
    for k in range(1, 14):
        pairs = [(i, k - i) for i in range(8) if 0 <= k - i < 8 and i < k - i]
        out.append(f"  // column {k}: {len(pairs)} off-diagonal products")
        out.append(column_block(k, pairs, "sqr"))
        out.append(f"  o[{k}] = (uint32_t)acc;")
        out.append("  acc = (acc >> 32) | ((uint64_t)top << 32);")
    out.append("  o[14] = (uint32_t)acc;")
    out.append("  o[15] = (uint32_t)(acc >> 32);")
    out.append("  (void)c0; (void)c1; (void)c2;")
    out.append("  // t = 2*o + diagonal squares (d_{2i}, d_{2i+1}) = a_i^2")
    out.append("  uint32_t cy = 0, d0, d1;")
    out.append("#pragma unroll")
    out.append("  for (int i = 0; i < 8; ++i) {")
    out.append("    const uint64_t d = (uint64_t)a[i] * a[i];")
    out.append("    d0 = (uint32_t)d;")
    out.append("    d1 = (uint32_t)(d >> 32);")
    out.append("    const uint32_t s0 = (i == 0) ? (o[0] << 1) : __builtin_amdgcn_alignbit(o[2 * i], o[2 * i - 1], 31);")
    out.append("    const uint32_t s1 = __builtin_amdgcn_alignbit(o[2 * i + 1], o[2 * i], 31);")
    out.append("    t[2 * i] = __builtin_addc(s0, d0, cy, &cy);")
    out.append("    t[2 * i + 1] = __builtin_addc(s1, d1, cy, &cy);")
    out.append("  }")
    out.append("}")
    out.extend(pair_functions())
    out.extend(row_functions())
    out.extend(reduced_functions())
    out.extend(reduced_pair_functions())
    out.append("")
    out.append("}  // namespace hkv")
    open(OUT, "w").write("\n".join(out) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
