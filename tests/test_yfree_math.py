"""The y-free verification identity used by the full-grid kernels
(hkv_kernels.hip §2b, hkv_finish_kernel / hkv_yverdict_kernel), checked on
the CPU with Python integers.

For a key Q = (x, y0) with w = x^3 + 7, Q' = (x w, w^2) lies on
E_w : y^2 = x^3 + 7 w^3 (the image of Q under (x, y) -> (y0^2 x, y0^3 y)),
so B' = u2 Q' maps back to B = u2 Q = (x'/w, y' y0 / w^2). Given A = u1 G and
B' in Jacobian coordinates, x(A + B) == r solves to y0 = num / den with the
kernel's num / den; the verdict is "y_c = num / den is a root of w with the
key's parity". A non-square w (a compressed key that does not parse) has no
root, so no r can pass.
"""
import random

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
     0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)


def inv(a):
    return pow(a, P - 2, P)


def add(p, q):
    """Affine addition for any y^2 = x^3 + b (the a = 0 formulas do not use b)."""
    if p is None:
        return q
    if q is None:
        return p
    (x1, y1), (x2, y2) = p, q
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * inv(2 * y1) % P
    else:
        lam = (y2 - y1) * inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def mul(k, p):
    r = None
    for bit in bin(k)[2:]:
        r = add(r, r)
        if bit == "1":
            r = add(r, p)
    return r


def jac(p, rng):
    z = rng.randrange(1, P)
    return p[0] * z * z % P, p[1] * pow(z, 3, P) % P, z


def num_den(A, Bp, w, rx):
    """hkv_finish_kernel's num / den (same operation order)."""
    XA, YA, ZA = A
    X, Y, Z = Bp
    ZA2 = ZA * ZA % P
    ZA3 = ZA2 * ZA % P
    Z2 = Z * Z % P
    Z3 = Z2 * Z % P
    Z2w = Z2 * w % P
    U1 = X * ZA2 % P
    t = XA * Z2w % P
    H = (U1 - t) % P
    S1 = (t + U1) % P
    T = Z2w * ZA2 % P
    S1 = (S1 + rx * T) % P
    HH = H * H % P
    a = Y * ZA3 % P
    b = YA * Z3 % P
    den = 2 * a * b * w % P
    num = (a * a + pow(w, 3, P) * b * b - HH * S1) % P
    return num, den, H


def test_yfree_identity_recovers_the_key_y():
    rng = random.Random(0x59465245)
    for _ in range(40):
        q = mul(rng.randrange(1, N), G)
        x, y0 = q
        w = (x ** 3 + 7) % P
        qp = (x * w % P, w * w % P)
        assert (qp[1] ** 2 - qp[0] ** 3 - 7 * w ** 3) % P == 0
        u1, u2 = rng.randrange(1, N), rng.randrange(1, N)
        a_pt, bp = mul(u1, G), mul(u2, qp)
        b_pt = mul(u2, q)
        assert b_pt == (bp[0] * inv(w) % P, bp[1] * y0 * inv(w * w) % P)
        rx = add(a_pt, b_pt)[0]
        num, den, h = num_den(jac(a_pt, rng), jac(bp, rng), w, rx)
        assert h != 0 and den != 0
        yc = num * inv(den) % P
        assert yc == y0
        # the other root fails the parity test; another r fails the root test
        assert (P - y0) % 2 != y0 % 2
        num2, den2, _ = num_den(jac(a_pt, rng), jac(bp, rng), w, (rx + 1) % P)
        yc2 = num2 * inv(den2) % P
        assert yc2 * yc2 % P != w


def test_yfree_rejects_non_square_keys():
    """x with x^3 + 7 a non-square: Q' = (x w, w^2) is a point of the twist
    E_w, the kernels still run, and no r yields a root of w."""
    rng = random.Random(5)
    found = 0
    while found < 8:
        x = rng.randrange(P)
        w = (x ** 3 + 7) % P
        if pow(w, (P - 1) // 2, P) == 1:
            continue
        found += 1
        qp = (x * w % P, w * w % P)
        u1, u2 = rng.randrange(1, N), rng.randrange(1, N)
        a_pt, bp = mul(u1, G), mul(u2, qp)
        if bp is None or a_pt[0] == bp[0] * inv(w) % P:
            continue  # the rare path decides these (its sqrt finds no root)
        for rx in (rng.randrange(N), 1, N - 1):
            num, den, _ = num_den(jac(a_pt, rng), jac(bp, rng), w, rx)
            yc = num * inv(den) % P
            assert yc * yc % P != w
