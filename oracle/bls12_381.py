"""BLS12-381 CPU restatement -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.  It restates, in plain Python big-int arithmetic, the parts of the un-vendored
dependency ``pairing = 0.14.2`` (reference ``Cargo.toml:28``) that hbbft's hot path reaches through
``threshold_crypto`` (reference ``Cargo.toml:35``, git, unpinned):

* Fq / Fq2 / Fq6 / Fq12 tower exactly as pairing 0.14 builds it
  (Fq2 = Fq[u]/(u^2+1), Fq6 = Fq2[v]/(v^3-(u+1)), Fq12 = Fq6[w]/(w^2-v));
* G1 (y^2 = x^3 + 4) and G2 (y^2 = x^3 + 4(u+1)) groups;
* the zcash/pairing compressed and uncompressed point encodings;
* the optimal-ate pairing (Miller loop over |x| = 0xd201000000010000, x negative) and the final
  exponentiation.  The pairing value is canonical (any correct optimal-ate pairing gives the same
  reduced value), so the verification bits this oracle produces do not depend on how pairing
  0.14 schedules its line functions.

Parity status: pinned by the BLS12-381 known answers of SURVEY.md App. A.2 (generator encodings,
r, cofactors), checked in ``tests/test_oracle_kat.py``, plus algebraic identities (bilinearity,
e^r = 1, subgroup orders).  The reference crates are not present in this container, so nothing
here was compared byte-for-byte against pairing 0.14 itself.

Representation: every field element is held in canonical (non-Montgomery) form as Python ints.
"""
from __future__ import annotations

# ---------------------------------------------------------------------------------------------
# Constants
# ---------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BLS_X = 0xD201000000010000  # |x|; x is negative
BLS_X_IS_NEGATIVE = True
H1 = 0x396C8C005555E1568C00AAAB0000AAAB
H2 = 0x5D543A95414E7F1091D50792876A202CD91DE4547085ABAA68A205B2E5A7DDFA628F1CB4D9E82EF21537E293A6691AE1616EC6E786F0C70CF1C38E31C7238E5
B1 = 4
MONT_R_FQ = 1 << 384
MONT_R_FR = 1 << 256
FQ_RINV = pow(MONT_R_FQ, -1, P)
FR_RINV = pow(MONT_R_FR, -1, R)


def fq_inv(a: int) -> int:
    return pow(a, P - 2, P)


def fq_sqrt(a: int):
    """Square root in Fq (p = 3 mod 4); None if a is a non-residue."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fq_is_lex_largest(y: int) -> bool:
    """pairing 0.14 'greatest' rule on Fq: y > -y on canonical representatives."""
    return y > (P - y) % P


# ---------------------------------------------------------------------------------------------
# Fq2 = Fq[u]/(u^2 + 1); elements are tuples (c0, c1)
# ---------------------------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = a0 * b0
    t1 = a1 * b1
    return ((t0 - t1) % P, ((a0 + a1) * (b0 + b1) - t0 - t1) % P)


def f2_sqr(a):
    a0, a1 = a
    return ((a0 + a1) * (a0 - a1) % P, 2 * a0 * a1 % P)


def f2_muls(a, s: int):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    a0, a1 = a
    t = fq_inv((a0 * a0 + a1 * a1) % P)
    return (a0 * t % P, (-a1) * t % P)


def f2_mul_xi(a):
    """Multiply by xi = u + 1 (the Fq6 non-residue)."""
    a0, a1 = a
    return ((a0 - a1) % P, (a0 + a1) % P)


def f2_is_zero(a):
    return a[0] % P == 0 and a[1] % P == 0


def f2_pow(a, e: int):
    r = F2_ONE
    for bit in bin(e)[2:]:
        r = f2_sqr(r)
        if bit == "1":
            r = f2_mul(r, a)
    return r


def f2_sqrt(a):
    """Some square root of a in Fq2, or None.  Which of the two roots is returned does not
    matter to callers: hash_g2 / decompression pick the root by the lexicographic rule."""
    a0, a1 = a[0] % P, a[1] % P
    if a1 == 0:
        s = fq_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fq_sqrt(-a0 % P)
        return (0, s) if s is not None else None
    alpha = fq_sqrt((a0 * a0 + a1 * a1) % P)
    if alpha is None:
        return None
    inv2 = (P + 1) // 2
    delta = (a0 + alpha) * inv2 % P
    x0 = fq_sqrt(delta)
    if x0 is None:
        delta = (a0 - alpha) * inv2 % P
        x0 = fq_sqrt(delta)
        if x0 is None:
            return None
    x1 = a1 * fq_inv(2 * x0 % P) % P
    r = (x0, x1)
    assert f2_sqr(r) == (a0, a1)
    return r


def f2_lex_gt(a, b) -> bool:
    """pairing 0.14 Ord for Fq2: compare c1 first, then c0 (canonical values)."""
    if a[1] != b[1]:
        return a[1] > b[1]
    return a[0] > b[0]


def f2_is_lex_largest(y) -> bool:
    return f2_lex_gt(y, f2_neg(y))


# ---------------------------------------------------------------------------------------------
# Fq6 = Fq2[v]/(v^3 - xi); elements are tuples of three Fq2
# ---------------------------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul_xi(t2))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a2, b0)), t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    """Multiply by v: (c0, c1, c2) * v = (xi * c2, c0, c1)."""
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_xi(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


# ---------------------------------------------------------------------------------------------
# Fq12 = Fq6[w]/(w^2 - v); elements are pairs of Fq6
# ---------------------------------------------------------------------------------------------
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), t0), t1)
    return (f6_add(t0, f6_mul_v(t1)), c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e: int):
    r = F12_ONE
    for bit in bin(e)[2:]:
        r = f12_sqr(r)
        if bit == "1":
            r = f12_mul(r, a)
    return r


def f12_eq(a, b) -> bool:
    return a == b


# Frobenius: Fq12 element viewed as sum_{i<6} g_i * W^i with W = w, g_i in Fq2 where
#   a = (a0, a1), a0 = (g0, g2, g4), a1 = (g1, g3, g5) since v = w^2.
# (g w^i)^p = conj(g) * gamma_i * w^i with gamma_i = xi^(i (p-1)/6).
_GAMMA1 = [f2_pow((1, 1), i * (P - 1) // 6) for i in range(6)]


def f12_frobenius(a):
    (g0, g2, g4), (g1, g3, g5) = a
    gs = [g0, g1, g2, g3, g4, g5]
    hs = [f2_mul(f2_conj(g), _GAMMA1[i]) for i, g in enumerate(gs)]
    return ((hs[0], hs[2], hs[4]), (hs[1], hs[3], hs[5]))


def f12_frobenius_n(a, n: int):
    for _ in range(n):
        a = f12_frobenius(a)
    return a


# ---------------------------------------------------------------------------------------------
# Curve groups.  Points are affine tuples (x, y) or None for the point at infinity.
# ---------------------------------------------------------------------------------------------
G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)
B2 = (4, 4)  # 4 (u + 1)


def g1_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * fq_inv(2 * y1 % P) % P
    else:
        lam = (y2 - y1) * fq_inv((x2 - x1) % P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_mul(pt, k: int):
    """Double-and-add (MSB first) with Jacobian internals for speed."""
    return _jac_to_aff1(_jac_mul1(_aff_to_jac1(pt), k))


def _aff_to_jac1(pt):
    return (0, 1, 0) if pt is None else (pt[0], pt[1], 1)


def _jac_to_aff1(j):
    X, Y, Z = j
    if Z % P == 0:
        return None
    zi = fq_inv(Z)
    zi2 = zi * zi % P
    return (X * zi2 % P, Y * zi2 * zi % P)


def _jac_dbl1(j):
    X, Y, Z = j
    if Z == 0 or Y == 0:
        return (0, 1, 0)
    A = X * X % P
    Bq = Y * Y % P
    C = Bq * Bq % P
    D = 2 * ((X + Bq) ** 2 - A - C) % P
    E = 3 * A % P
    X3 = (E * E - 2 * D) % P
    Y3 = (E * (D - X3) - 8 * C) % P
    Z3 = 2 * Y * Z % P
    return (X3, Y3, Z3)


def _jac_add1(j1, j2):
    X1, Y1, Z1 = j1
    X2, Y2, Z2 = j2
    if Z1 == 0:
        return j2
    if Z2 == 0:
        return j1
    Z1Z1 = Z1 * Z1 % P
    Z2Z2 = Z2 * Z2 % P
    U1 = X1 * Z2Z2 % P
    U2 = X2 * Z1Z1 % P
    S1 = Y1 * Z2 * Z2Z2 % P
    S2 = Y2 * Z1 * Z1Z1 % P
    if U1 == U2:
        if S1 == S2:
            return _jac_dbl1(j1)
        return (0, 1, 0)
    H = (U2 - U1) % P
    I = 4 * H * H % P
    J = H * I % P
    rr = 2 * (S2 - S1) % P
    V = U1 * I % P
    X3 = (rr * rr - J - 2 * V) % P
    Y3 = (rr * (V - X3) - 2 * S1 * J) % P
    Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % P
    return (X3, Y3, Z3)


def _jac_mul1(j, k: int):
    acc = (0, 1, 0)
    for bit in bin(k)[2:] if k > 0 else "":
        acc = _jac_dbl1(acc)
        if bit == "1":
            acc = _jac_add1(acc, j)
    return acc


def g2_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g2_neg(pt):
    return None if pt is None else (pt[0], f2_neg(pt[1]))


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if f2_add(y1, y2) == F2_ZERO:
            return None
        lam = f2_mul(f2_muls(f2_sqr(x1), 3), f2_inv(f2_muls(y1, 2)))
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    return (x3, f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1))


def _jac_dbl2(j):
    X, Y, Z = j
    if f2_is_zero(Z) or f2_is_zero(Y):
        return (F2_ZERO, F2_ONE, F2_ZERO)
    A = f2_sqr(X)
    Bq = f2_sqr(Y)
    C = f2_sqr(Bq)
    D = f2_muls(f2_sub(f2_sub(f2_sqr(f2_add(X, Bq)), A), C), 2)
    E = f2_muls(A, 3)
    X3 = f2_sub(f2_sqr(E), f2_muls(D, 2))
    Y3 = f2_sub(f2_mul(E, f2_sub(D, X3)), f2_muls(C, 8))
    Z3 = f2_muls(f2_mul(Y, Z), 2)
    return (X3, Y3, Z3)


def _jac_add2(j1, j2):
    X1, Y1, Z1 = j1
    X2, Y2, Z2 = j2
    if f2_is_zero(Z1):
        return j2
    if f2_is_zero(Z2):
        return j1
    Z1Z1 = f2_sqr(Z1)
    Z2Z2 = f2_sqr(Z2)
    U1 = f2_mul(X1, Z2Z2)
    U2 = f2_mul(X2, Z1Z1)
    S1 = f2_mul(f2_mul(Y1, Z2), Z2Z2)
    S2 = f2_mul(f2_mul(Y2, Z1), Z1Z1)
    if U1 == U2:
        if S1 == S2:
            return _jac_dbl2(j1)
        return (F2_ZERO, F2_ONE, F2_ZERO)
    H = f2_sub(U2, U1)
    I = f2_muls(f2_sqr(H), 4)
    J = f2_mul(H, I)
    rr = f2_muls(f2_sub(S2, S1), 2)
    V = f2_mul(U1, I)
    X3 = f2_sub(f2_sub(f2_sqr(rr), J), f2_muls(V, 2))
    Y3 = f2_sub(f2_mul(rr, f2_sub(V, X3)), f2_muls(f2_mul(S1, J), 2))
    Z3 = f2_mul(f2_sub(f2_sub(f2_sqr(f2_add(Z1, Z2)), Z1Z1), Z2Z2), H)
    return (X3, Y3, Z3)


def g2_mul(pt, k: int):
    if pt is None or k == 0:
        return None
    j = (pt[0], pt[1], F2_ONE)
    acc = (F2_ZERO, F2_ONE, F2_ZERO)
    for bit in bin(k)[2:]:
        acc = _jac_dbl2(acc)
        if bit == "1":
            acc = _jac_add2(acc, j)
    X, Y, Z = acc
    if f2_is_zero(Z):
        return None
    zi = f2_inv(Z)
    zi2 = f2_sqr(zi)
    return (f2_mul(X, zi2), f2_mul(f2_mul(Y, zi2), zi))


# ---------------------------------------------------------------------------------------------
# Encodings (zcash / pairing 0.14 format)
# ---------------------------------------------------------------------------------------------
FLAG_COMPRESSED = 0x80
FLAG_INFINITY = 0x40
FLAG_LARGEST = 0x20


def _be(x: int, n: int = 48) -> bytes:
    return x.to_bytes(n, "big")


def g1_compress(pt) -> bytes:
    if pt is None:
        out = bytearray(48)
        out[0] = FLAG_COMPRESSED | FLAG_INFINITY
        return bytes(out)
    x, y = pt
    out = bytearray(_be(x))
    out[0] |= FLAG_COMPRESSED
    if fq_is_lex_largest(y):
        out[0] |= FLAG_LARGEST
    return bytes(out)


def g1_uncompress_bytes(pt) -> bytes:
    """96-byte uncompressed G1 encoding: x || y big-endian (infinity flag 0x40)."""
    if pt is None:
        out = bytearray(96)
        out[0] = FLAG_INFINITY
        return bytes(out)
    return _be(pt[0]) + _be(pt[1])


def g1_decompress(data: bytes, subgroup_check: bool = True):
    """Inverse of g1_compress.  Raises ValueError on a malformed encoding (pairing 0.14
    ``G1Compressed::into_affine``: flag checks, x < p, point on curve, subgroup)."""
    if len(data) != 48:
        raise ValueError("length")
    flags = data[0]
    if not flags & FLAG_COMPRESSED:
        raise ValueError("not compressed")
    if flags & FLAG_INFINITY:
        if flags & FLAG_LARGEST or any(data[1:]) or (data[0] & 0x1F):
            raise ValueError("bad infinity")
        return None
    x = int.from_bytes(bytes([data[0] & 0x1F]) + data[1:], "big")
    if x >= P:
        raise ValueError("x not in field")
    y = fq_sqrt((x * x * x + B1) % P)
    if y is None:
        raise ValueError("not on curve")
    if fq_is_lex_largest(y) != bool(flags & FLAG_LARGEST):
        y = (-y) % P
    pt = (x, y)
    if subgroup_check and g1_mul(pt, R) is not None:
        raise ValueError("not in subgroup")
    return pt


def g2_compress(pt) -> bytes:
    if pt is None:
        out = bytearray(96)
        out[0] = FLAG_COMPRESSED | FLAG_INFINITY
        return bytes(out)
    x, y = pt
    out = bytearray(_be(x[1]) + _be(x[0]))
    out[0] |= FLAG_COMPRESSED
    if f2_is_lex_largest(y):
        out[0] |= FLAG_LARGEST
    return bytes(out)


def g2_uncompress_bytes(pt) -> bytes:
    """192-byte uncompressed G2 encoding: x.c1 || x.c0 || y.c1 || y.c0."""
    if pt is None:
        out = bytearray(192)
        out[0] = FLAG_INFINITY
        return bytes(out)
    x, y = pt
    return _be(x[1]) + _be(x[0]) + _be(y[1]) + _be(y[0])


def g2_decompress(data: bytes, subgroup_check: bool = True):
    if len(data) != 96:
        raise ValueError("length")
    flags = data[0]
    if not flags & FLAG_COMPRESSED:
        raise ValueError("not compressed")
    if flags & FLAG_INFINITY:
        if flags & FLAG_LARGEST or any(data[1:]) or (data[0] & 0x1F):
            raise ValueError("bad infinity")
        return None
    x1 = int.from_bytes(bytes([data[0] & 0x1F]) + data[1:48], "big")
    x0 = int.from_bytes(data[48:96], "big")
    if x0 >= P or x1 >= P:
        raise ValueError("x not in field")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise ValueError("not on curve")
    if f2_is_lex_largest(y) != bool(flags & FLAG_LARGEST):
        y = f2_neg(y)
    pt = (x, y)
    if subgroup_check and g2_mul(pt, R) is not None:
        raise ValueError("not in subgroup")
    return pt


# ---------------------------------------------------------------------------------------------
# Pairing (optimal ate).  Line functions are evaluated in Fq12 with the untwist
# (x', y') -> (x' / w^2, y' / w^3); each line is scaled by w^3, an Fq4 element, and vertical
# lines (Fq6 elements) are dropped: both vanish under the final exponentiation because
# (p^4 - 1) and (p^6 - 1) divide (p^12 - 1) / r.
# ---------------------------------------------------------------------------------------------
def _line_to_f12(c, cv, cvw):
    """Fq12 element c + cv * v + cvw * v*w (v = w^2) -> ((c, cv, 0), (0, cvw, 0))."""
    return ((c, cv, F2_ZERO), (F2_ZERO, cvw, F2_ZERO))


def _line(T, lam, P1):
    """l(P) * w^3 for the line through T (twist coords) with slope lam' (twist slope):
    l * w^3 = (lam' xT' - yT') - lam' xP * w^2 + yP * w^3."""
    xT, yT = T
    xP, yP = P1
    c = f2_sub(f2_mul(lam, xT), yT)
    cv = f2_neg(f2_muls(lam, xP))
    cvw = (yP % P, 0)
    return _line_to_f12(c, cv, cvw)


def miller_loop(P1, Q2):
    """f_{|x|,Q}(P), conjugated because x < 0.  P1 in G1, Q2 in G2 (affine, not infinity)."""
    if P1 is None or Q2 is None:
        return F12_ONE
    f = F12_ONE
    T = Q2
    for bit in bin(BLS_X)[3:]:
        # doubling step
        xT, yT = T
        lam = f2_mul(f2_muls(f2_sqr(xT), 3), f2_inv(f2_muls(yT, 2)))
        f = f12_mul(f12_sqr(f), _line(T, lam, P1))
        x3 = f2_sub(f2_sqr(lam), f2_muls(xT, 2))
        T = (x3, f2_sub(f2_mul(lam, f2_sub(xT, x3)), yT))
        if bit == "1":
            xT, yT = T
            xQ, yQ = Q2
            lam = f2_mul(f2_sub(yT, yQ), f2_inv(f2_sub(xT, xQ)))
            f = f12_mul(f, _line(T, lam, P1))
            x3 = f2_sub(f2_sub(f2_sqr(lam), xT), xQ)
            T = (x3, f2_sub(f2_mul(lam, f2_sub(xT, x3)), yT))
    if BLS_X_IS_NEGATIVE:
        f = f12_conj(f)
    return f


FINAL_EXP_HARD = (P**4 - P**2 + 1) // R


def final_exponentiation(f):
    """f^((p^12 - 1)/r): easy part (p^6 - 1)(p^2 + 1) by conjugation/Frobenius, hard part by
    plain square-and-multiply with (p^4 - p^2 + 1)/r (slow, transparent)."""
    t = f12_mul(f12_conj(f), f12_inv(f))  # f^(p^6 - 1)
    t = f12_mul(f12_frobenius_n(t, 2), t)  # ^(p^2 + 1)
    return f12_pow(t, FINAL_EXP_HARD)


def pairing(P1, Q2):
    return final_exponentiation(miller_loop(P1, Q2))


def pairing_product_is_one(pairs) -> bool:
    """prod_i e(P_i, Q_i) == 1 using one shared final exponentiation."""
    f = F12_ONE
    for P1, Q2 in pairs:
        f = f12_mul(f, miller_loop(P1, Q2))
    return final_exponentiation(f) == F12_ONE


# ---------------------------------------------------------------------------------------------
# Montgomery helpers (pairing 0.14 stores Fq/Fr in Montgomery form; Rand fills the raw repr)
# ---------------------------------------------------------------------------------------------
def fq_from_mont_repr(limbs_value: int) -> int:
    return limbs_value * FQ_RINV % P


def fr_from_mont_repr(limbs_value: int) -> int:
    return limbs_value * FR_RINV % R
