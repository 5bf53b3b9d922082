"""Algorithmic work per verify, counted from the kernels' op sequence.

The roofline numerator: P = 32x32->64-bit limb products
(``v_mad_u64_u32``) per signature. Counts follow hkv_field.h / hkv_scalar.h /
hkv_group.h / hkv_kernels.hip op by op; degenerate-case branches (rare) and
the per-signature infinity-init mapping are excluded. The peak is the
measured ``v_mad_u64_u32`` issue rate (profiles/r01_ubench_int.json:
64 lane-products/clk/CU = half rate) x 256 CUs x 2.4 GHz.
"""
from __future__ import annotations

# limb products per primitive
MUL256 = 64          # 8x8 schoolbook rows
SQR256 = 28 + 8      # off-diagonal + diagonal
FE_RED = 8 + 1       # H*977 chain + top fold (y = top*977)
FE_MUL = MUL256 + FE_RED
FE_SQR = SQR256 + FE_RED
FE_MUL_SMALL = 8 + 1
SC_RED = 8 * 4 + 5 * 4 + 4   # three folds by NC's low 128 bits
SC_MUL = MUL256 + SC_RED
SC_SQR = SQR256 + SC_RED

GEJ_DOUBLE = 3 * FE_MUL + 4 * FE_SQR + FE_MUL_SMALL           # a=0, D = 4XB; 2^k scalings are shifts
GEJ_ADD_GE = 8 * FE_MUL + 3 * FE_SQR                          # mixed add
GEJ_ADD_ZINV = GEJ_ADD_GE + FE_MUL                            # + az = Z*Zg

Q_WINDOWS = 33       # radix-16 Booth over 132 bits
G_WINDOWS = 7        # radix-2^20 Booth over 140 bits (u1 halves)
DOUBLINGS = 4 * (Q_WINDOWS - 1)

SC_INV_LOW = 0x0BAAEDCE6AF48A03BBFD25E8CD036413F
BATCH_INV = 16       # signatures per s^-1 (hkv_layout.h)


def ecmult_products() -> int:
    table = (GEJ_DOUBLE                      # 2Q
             + FE_SQR + 3 * FE_MUL           # Q' = (x Z^2, y Z^3)
             + 6 * GEJ_ADD_GE                # 3Q .. 8Q
             + FE_MUL                        # Zg
             + FE_MUL                        # beta * x of entry 8
             + 6 * (5 * FE_MUL + FE_SQR)     # rescale entries 2..7 (+ rho step, beta)
             + (4 * FE_MUL + FE_SQR))        # rescale entry 1
    ladder = DOUBLINGS * GEJ_DOUBLE + 2 * Q_WINDOWS * GEJ_ADD_GE + 2 * G_WINDOWS * GEJ_ADD_ZINV
    compare = 3 * FE_MUL + FE_SQR
    return table + ladder + compare


def prologue_products() -> int:
    chain223 = 222 * FE_SQR + 11 * FE_MUL
    sqrt = chain223 + (23 + 6 + 2) * FE_SQR + 2 * FE_MUL
    curve = FE_SQR + FE_MUL + FE_SQR                 # x^3 + 7, y^2 check
    x127 = (1 + 1 + 3 + 6 + 12 + 24 + 48 + 24 + 6 + 1) * SC_SQR + 10 * SC_MUL
    inv = x127 + 129 * SC_SQR + bin(SC_INV_LOW).count("1") * SC_MUL
    batch = BATCH_INV
    inv_per_sig = (inv + 3 * (batch - 1) * SC_MUL) // batch   # Montgomery's trick
    glv = 2 * MUL256 + 3 * SC_MUL
    return sqrt + curve + inv_per_sig + 2 * SC_MUL + glv


ECMULT_PRODUCTS_PER_VERIFY = ecmult_products()
PROLOGUE_PRODUCTS_PER_VERIFY = prologue_products()
PRODUCTS_PER_VERIFY = ECMULT_PRODUCTS_PER_VERIFY + PROLOGUE_PRODUCTS_PER_VERIFY

# measured v_mad_u64_u32 issue rate on gfx950 (lane-products / clk / CU)
R_MUL = 64
N_CU = 256
F_CLK_PEAK = 2.4e9
PEAK_PRODUCTS_PER_S = R_MUL * N_CU * F_CLK_PEAK

if __name__ == "__main__":
    print("ecmult", ECMULT_PRODUCTS_PER_VERIFY, "prologue", PROLOGUE_PRODUCTS_PER_VERIFY,
          "total", PRODUCTS_PER_VERIFY, "peak/s %.3e" % PEAK_PRODUCTS_PER_S)
