"""Algorithmic work per verify, counted from the kernels' op sequence.

The roofline numerator: P = 32x32->64-bit limb products
(``v_mad_u64_u32``) per signature. Counts follow hkv_field.h / hkv_scalar.h /
hkv_group.h / hkv_kernels.hip op by op; degenerate-case branches (rare) and
the per-signature infinity-init mapping are excluded. The peak is the
measured ``v_mad_u64_u32`` issue rate (profiles/r01_ubench_int.json:
64 lane-products/clk/CU = half rate) x 256 CUs x 2.4 GHz.
"""
from __future__ import annotations

# limb products per primitive (hkv_mul_asm.h, HKV_MUL_RED: the reduction
# folded into the scan; the 7 carry-in mads by 1 per product are not limb
# products and are not counted)
MUL256 = 64          # 8x8 column scan
SQR256 = 43          # 8 squares + 7 a_i * 2a_{i+1} + 28 a_i * (2a)_j (incl. the 1-bit top limb)
FE_RED = 8 + 1       # h_j * 977 in the low columns + top fold (y = top*977)
FE_MUL = MUL256 + FE_RED
FE_SQR = SQR256 + FE_RED
FE_MUL_SMALL = 8 + 1
SC_RED = 8 * 4 + 5 * 4 + 4   # three folds by NC's low 128 bits
SC_MUL = MUL256 + SC_RED
SC_SQR = SQR256 + SC_RED

GEJ_DOUBLE = 3 * FE_MUL + 4 * FE_SQR + FE_MUL_SMALL           # a=0; the 1/2 scaling / 2^k are adds and shifts
GEJ_ADD_GE = 8 * FE_MUL + 3 * FE_SQR                          # mixed add
GEJ_ADD_ZINV = GEJ_ADD_GE + FE_MUL                            # + az = Z*Zg

QW = 4               # Booth radix 2^QW of the k1 / k2 windows (hkv_layout.h HKV_QW)
Q_WINDOWS = (130 + QW - 1) // QW     # 26 (radix 32) / 33 (radix 16)
Q_TABLE = 1 << (QW - 1)              # j*Q, j = 1..16 (radix 32) / 1..8
G_WINDOWS = 7        # radix-2^20 Booth over 140 bits (u1 halves)
DOUBLINGS = QW * (Q_WINDOWS - 2)   # the top two windows merged (HKV_TOP_MERGE)

SC_INV_LOW = 0x0BAAEDCE6AF48A03BBFD25E8CD036413F
BATCH_INV = 16       # signatures per s^-1 (hkv_layout.h)


YFREE = True         # full-grid batches verify y-free (hkv_layout.h HKV_YFREE)


def ecmult_products(qw: int = QW, beta_per_lookup: bool = False) -> int:
    """The ecmult stage: hkv_ecmult_kernel, plus (y-free) the finish and
    verdict kernels that complete u1*G + u2*Q and decide x(R) == r.
    qw / beta_per_lookup price the variants (the floor):
    radix-2^qw Q windows, and an (x, y)-only Q table whose lambda lookups
    form beta * x per addition instead of storing it."""
    q_table = 1 << (qw - 1)
    q_windows = (130 + qw - 1) // qw
    # radix 16: the top two windows run as one (HKV_TOP_MERGE: the halves are
    # < 2^128), their up to four additions counted as the two windows' two
    # each; radix 32's top window already holds bits 125..127 (no merge)
    doublings = qw * (q_windows - (2 if qw == 4 else 1))
    beta_t = 0 if beta_per_lookup else 1             # beta * x per table entry, or per lambda addition
    table = (GEJ_DOUBLE                      # 2Q
             + FE_SQR + 3 * FE_MUL           # Q' = (x Z^2, y Z^3)
             + (q_table - 2) * GEJ_ADD_GE    # 3Q .. q_table*Q
             + FE_MUL                        # Zg
             + beta_t * FE_MUL               # beta * x of the last entry
             + (q_table - 2) * ((4 + beta_t) * FE_MUL + FE_SQR)   # rescale entries 2..q_table-1 (+ rho step, beta)
             + ((3 + beta_t) * FE_MUL + FE_SQR))                 # rescale entry 1
    if not YFREE:
        ladder = doublings * GEJ_DOUBLE + 2 * q_windows * GEJ_ADD_GE + 2 * G_WINDOWS * GEJ_ADD_ZINV
        compare = 3 * FE_MUL + FE_SQR
        return table + ladder + compare
    to_ew = FE_MUL + FE_SQR                              # Q' = (x w, w^2) on E_w
    ladder = (doublings * GEJ_DOUBLE + 2 * q_windows * GEJ_ADD_GE + FE_MUL   # + Z = acc.z * Zg
              + (1 - beta_t) * q_windows * FE_MUL)       # beta * x per lambda addition
    g_sum = (2 * G_WINDOWS - 1) * GEJ_ADD_GE             # per-window tables, no doublings
    combine = 16 * FE_MUL + 6 * FE_SQR                   # num, num_{r+n}, den (hkv_finish_kernel)
    inv_chain = 255 * FE_SQR + 15 * FE_MUL               # fe_inv, one per BATCH_INV signatures
    verdict = 3 * FE_MUL + inv_chain // BATCH_INV + FE_MUL + FE_SQR   # y_c = num / den, y_c^2 == w
    return table + to_ew + ladder + g_sum + combine + verdict


def prologue_products() -> int:
    chain223 = 222 * FE_SQR + 11 * FE_MUL
    sqrt = 0 if YFREE else chain223 + (23 + 6 + 2) * FE_SQR + 2 * FE_MUL
    curve = FE_SQR + FE_MUL + FE_SQR                 # x^3 + 7, y^2 check
    x127 = (1 + 1 + 3 + 6 + 12 + 24 + 48 + 24 + 6 + 1) * SC_SQR + 10 * SC_MUL
    inv = x127 + 129 * SC_SQR + bin(SC_INV_LOW).count("1") * SC_MUL
    batch = BATCH_INV
    inv_per_sig = (inv + 3 * (batch - 1) * SC_MUL) // batch   # Montgomery's trick
    glv = 2 * MUL256 + 3 * SC_MUL
    return sqrt + curve + inv_per_sig + 2 * SC_MUL + glv


# --- the reference algorithm's work (the frozen roofline numerator) ---------
# P_alg is counted for the REFERENCE algorithm, not for this
# implementation, so it does not drift when the kernels change. libsecp256k1's
# secp256k1_ecmult for one point [dep; published algorithm]: GLV split of u2,
# wNAF w = 5 over both 129-bit halves (expected density 1/(w+1)), the 8-entry
# odd-multiples table of Q on a global Z (secp256k1_ecmult_odd_multiples_table
# + secp256k1_ge_table_set_globalz) plus its lambda image (beta * x), G and
# 2^128 G by precomputed w = 15 tables (ECMULT_WINDOW_SIZE default) added with
# secp256k1_gej_add_zinv_var, 129 doublings (secp256k1_gej_double: 3M + 4S),
# then the Jacobian x compare (1S + 1M). Field products are priced at this
# ISA's 32-bit limb-product counts as they stood when the numerator was
# frozen (round 1: 64 + 9 per multiply, 36 + 9 per square), not at the
# current kernels' counts above.
REF_FE_MUL = 64 + 9
REF_FE_SQR = 36 + 9
REF_BITS = 129                      # |k1|, |k2| < 2^129 after the GLV split
REF_WNAF_Q = 5
REF_WINDOW_G = 15
REF_Q_ADDS = 2 * REF_BITS / (REF_WNAF_Q + 1)     # 43
REF_G_ADDS = 2 * 128 / (REF_WINDOW_G + 1)        # 16
REF_TABLE = ((3 * REF_FE_MUL + 4 * REF_FE_SQR)            # 2Q
             + 7 * (8 * REF_FE_MUL + 3 * REF_FE_SQR)      # 3Q .. 15Q (odd multiples, mixed adds)
             + 7 * (4 * REF_FE_MUL + REF_FE_SQR)          # global-Z rescale
             + 8 * REF_FE_MUL)                            # lambda table: beta * x
REF_LADDER = (REF_BITS * (3 * REF_FE_MUL + 4 * REF_FE_SQR) + REF_Q_ADDS * (8 * REF_FE_MUL + 3 * REF_FE_SQR)
              + REF_G_ADDS * (9 * REF_FE_MUL + 3 * REF_FE_SQR))
REF_COMPARE = REF_FE_SQR + REF_FE_MUL
P_ALG_ECMULT = int(round(REF_TABLE + REF_LADDER + REF_COMPARE))
assert P_ALG_ECMULT == 103553, "the frozen numerator must not drift"

ECMULT_PRODUCTS_PER_VERIFY = ecmult_products()
PROLOGUE_PRODUCTS_PER_VERIFY = prologue_products()
PRODUCTS_PER_VERIFY = ECMULT_PRODUCTS_PER_VERIFY + PROLOGUE_PRODUCTS_PER_VERIFY

# v_mad_u64_u32 issue rate on gfx950 (lane-products / clk / CU): nominal half
# rate (64), and the rate measured by tools/ubench_int.hip
# (profiles/r01_ubench_int.json: 57.07 at the clock it ran at)
R_MUL = 64
R_MUL_MEASURED = 57.07
N_CU = 256
F_CLK_PEAK = 2.4e9
PEAK_PRODUCTS_PER_S = R_MUL * N_CU * F_CLK_PEAK

if __name__ == "__main__":
    print("P_alg(ecmult, reference algorithm)", P_ALG_ECMULT, "P_impl(ecmult)", ECMULT_PRODUCTS_PER_VERIFY)
    print("ecmult", ECMULT_PRODUCTS_PER_VERIFY, "prologue", PROLOGUE_PRODUCTS_PER_VERIFY,
          "total", PRODUCTS_PER_VERIFY, "peak/s %.3e" % PEAK_PRODUCTS_PER_S)
