"""The kernels' field / curve / pairing / hash code (hbbft_amd/csrc/*.hpp, all __host__ __device__)
compiled for the CPU by g++ (tools/hostcheck) and compared with the oracle.  This pins the GPU
arithmetic without a GPU; the -m gpu tests then pin the kernels themselves."""
import ctypes
import hashlib
import os
import random
import subprocess

import pytest

from oracle import bls12_381 as bls
from oracle import threshold as tc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hc(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("hostcheck") / "libhostcheck.so")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-DHBX_DCHECK", "-shared", "-fPIC", "-o", out,
                           os.path.join(ROOT, "tools", "hostcheck", "hostcheck.cpp")])
    lib = ctypes.CDLL(out)
    lib.hc_sha256.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.hc_hash_g1_g2.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.hc_fq2d_mul.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    return lib


def _be(x, n=48):
    return x.to_bytes(n, "big")


def test_fq_mul_inv(hc):
    rnd = random.Random(1)
    for _ in range(50):
        a, b = rnd.randrange(bls.P), rnd.randrange(bls.P)
        out = ctypes.create_string_buffer(48)
        hc.hc_fq_mul(_be(a), _be(b), out)
        assert int.from_bytes(out.raw, "big") == a * b % bls.P
    for a in (1, 2, bls.P - 1, rnd.randrange(1, bls.P)):
        out = ctypes.create_string_buffer(48)
        hc.hc_fq_inv(_be(a), out)
        assert int.from_bytes(out.raw, "big") * a % bls.P == 1


def _limbs(x, n):
    return (ctypes.c_uint32 * n)(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)])


def test_binary_inversion_montgomery(hc):
    """fq_inv / fr_inv (binary extended Euclid + R^3 fix-up): Montgomery in, Montgomery out,
    for canonical and lazy-range (x + p) operands, the extremes, and 0 -> 0 (as x^(m-2))."""
    rnd = random.Random(11)
    for mod, n, bits, fn in ((bls.P, 12, 384, hc.hc_fq_inv_raw), (bls.R, 8, 256, hc.hc_fr_inv_raw)):
        R = 1 << bits
        xs = [0, 1, 2, mod - 1, mod - 2, (mod - 1) // 2] + [rnd.randrange(mod) for _ in range(200)]
        for x in xs:
            m = x * R % mod
            reps = [m] + ([m + mod] if mod == bls.P and m + mod < 2 * mod else [])
            for rep in reps:
                out = (ctypes.c_uint32 * n)()
                fn(_limbs(rep, n), out)
                got = sum(int(out[i]) << (32 * i) for i in range(n))
                want = 0 if x == 0 else pow(x, -1, mod) * R % mod
                assert got == want, (hex(x), hex(rep))


def test_fq_mul_lazy_range(hc):
    """The digit-sliced Montgomery product on lazy operands in [0, 2p]: r = a b / 2^384 mod p and
    r < 2p (the bound the tower relies on), including the extremes 0, p, 2p - 1 and 2p."""
    rnd = random.Random(7)
    P2 = 2 * bls.P
    edge = [0, 1, bls.P - 1, bls.P, bls.P + 1, P2 - 1, P2, (1 << 381) - 1]
    pairs = [(a, b) for a in edge for b in edge] + [(rnd.randrange(P2 + 1), rnd.randrange(P2 + 1)) for _ in range(400)]
    rinv = pow(1 << 384, -1, bls.P)
    for a, b in pairs:
        if a > P2 or b > P2:
            continue
        A = (ctypes.c_uint32 * 12)(*[(a >> (32 * i)) & 0xFFFFFFFF for i in range(12)])
        B = (ctypes.c_uint32 * 12)(*[(b >> (32 * i)) & 0xFFFFFFFF for i in range(12)])
        O = (ctypes.c_uint32 * 12)()
        hc.hc_fq_mul_raw(A, B, O)
        r = sum(int(O[i]) << (32 * i) for i in range(12))
        assert r < P2, (hex(a), hex(b))
        assert r % bls.P == a * b * rinv % bls.P, (hex(a), hex(b))


def test_fq_sqr_lazy_range(hc):
    """The dedicated square (105 + 196 digit products) equals the product of a with itself on lazy
    operands in [0, 2p], output < 2p."""
    rnd = random.Random(11)
    P2 = 2 * bls.P
    vals = [0, 1, 2, bls.P - 1, bls.P, bls.P + 1, P2 - 1, P2, (1 << 381) - 1, (1 << 380) + 12345]
    vals += [rnd.randrange(P2 + 1) for _ in range(600)]
    rinv = pow(1 << 384, -1, bls.P)
    for a in vals:
        A = (ctypes.c_uint32 * 12)(*[(a >> (32 * i)) & 0xFFFFFFFF for i in range(12)])
        O = (ctypes.c_uint32 * 12)()
        hc.hc_fq_sqr_raw(A, O)
        r = sum(int(O[i]) << (32 * i) for i in range(12))
        assert r < P2, hex(a)
        assert r % bls.P == a * a * rinv % bls.P, hex(a)


def test_point_roundtrips(hc):
    for k in (1, 2, 0xDEADBEEF, bls.R - 1):
        c1 = bls.g1_compress(bls.g1_mul(bls.G1_GEN, k))
        o1 = ctypes.create_string_buffer(48)
        assert hc.hc_g1_roundtrip(c1, o1) == 0 and o1.raw == c1
        c2 = bls.g2_compress(bls.g2_mul(bls.G2_GEN, k))
        o2 = ctypes.create_string_buffer(96)
        assert hc.hc_g2_roundtrip(c2, o2) == 0 and o2.raw == c2


def test_pairing_check(hc):
    a = 0x1234567890ABCDEF
    pa = bls.g1_compress(bls.g1_mul(bls.G1_GEN, a))
    g2 = bls.g2_compress(bls.G2_GEN)
    qa = bls.g2_compress(bls.g2_mul(bls.G2_GEN, a))
    ng1 = bls.g1_compress(bls.g1_neg(bls.G1_GEN))
    assert hc.hc_pairing_check2(pa, g2, ng1, qa) == 1          # e(aP,Q) e(-P,aQ) == 1
    qb = bls.g2_compress(bls.g2_mul(bls.G2_GEN, a + 1))
    assert hc.hc_pairing_check2(pa, g2, ng1, qb) == 0


def test_digit_tower_products(hc):
    """fieldd.hpp (the share check's signed 28-bit digit tower, R' = 2^392): Fq and fused Fq2
    products / squares equal the field's, including the extremes."""
    rnd = random.Random(21)
    P = bls.P
    vals = [0, 1, P - 1, P - 2, (P - 1) // 2] + [rnd.randrange(P) for _ in range(150)]
    for a in vals:
        b = rnd.choice(vals)
        out = ctypes.create_string_buffer(48)
        hc.hc_fqd_mul(_be(a), _be(b), out)
        assert int.from_bytes(out.raw, "big") == a * b % P
    for sq in (0, 1):
        for _ in range(150):
            a0, a1, b0, b1 = (rnd.choice(vals) for _ in range(4))
            if sq:
                b0, b1 = a0, a1
            out = ctypes.create_string_buffer(96)
            hc.hc_fq2d_mul(_be(a0) + _be(a1), _be(b0) + _be(b1), out, sq)
            assert int.from_bytes(out.raw[:48], "big") == (a0 * b0 - a1 * b1) % P
            assert int.from_bytes(out.raw[48:], "big") == (a0 * b1 + a1 * b0) % P


def test_fq4d_sqr_lazy(hc):
    """fieldd.hpp fq4d_sqr_lazy ((a + b Y)^2, Y^2 = xi, six convolutions and four reductions in one
    column loop: the Karabina and Granger-Scott squarings of the final exponentiation) equals the
    Fq4 square, with inputs at both ends of the normalised range (x - p, x + p; HBX_DCHECK on)."""
    rnd = random.Random(24)
    P = bls.P
    vals = [0, 1, P - 1, P - 2, (P - 1) // 2] + [rnd.randrange(P) for _ in range(60)]
    for trial in range(200):
        x = [rnd.choice(vals) for _ in range(4)]
        sh = [rnd.choice((-1, 0, 1)) if x[q] else rnd.choice((0, 1)) for q in range(4)]
        if trial < 16:  # every input at its largest
            x, sh = [P - 1] * 4, [1] * 4
        out = ctypes.create_string_buffer(192)
        hc.hc_fq4d_sqr_lazy(b"".join(_be(v) for v in x), (ctypes.c_int * 4)(*sh), out)
        a0, a1, b0, b1 = x
        # a^2 + xi b^2 and 2ab over Fq2 = Fq[u]/(u^2 + 1), xi = 1 + u
        a2 = ((a0 * a0 - a1 * a1), 2 * a0 * a1)
        b2 = ((b0 * b0 - b1 * b1), 2 * b0 * b1)
        want = [(a2[0] + b2[0] - b2[1]) % P, (a2[1] + b2[0] + b2[1]) % P,
                2 * (a0 * b0 - a1 * b1) % P, 2 * (a0 * b1 + a1 * b0) % P]
        got = [int.from_bytes(out.raw[48 * q:48 * q + 48], "big") for q in range(4)]
        assert got == want, (trial, x, sh)


def test_digit_tower_pairing_check(hc):
    """The share check's digit-form Miller loop and final exponentiation (pairingd.hpp, the code
    of k_verify_shares) give the same Fq12 elements as pairing.hpp's on the same prepared lines,
    for valid and invalid checks; host build with the operand-bound assertions (HBX_DCHECK)."""
    rnd = random.Random(22)
    chk = ctypes.c_int()
    for trial in range(6):
        a = rnd.randrange(1, bls.R)
        pa = bls.g1_compress(bls.g1_mul(bls.G1_GEN, a))
        qa = bls.g2_compress(bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R)))
        ng1 = bls.g1_compress(bls.g1_neg(bls.g1_mul(bls.G1_GEN, rnd.randrange(1, bls.R))))
        qb = bls.g2_compress(bls.g2_mul(bls.G2_GEN, a + (trial & 1)))
        assert hc.hc_miller2_digit_cmp(pa, qa, ng1, qb, ctypes.byref(chk)) == 3
    # a check that holds: e(aP, Q) e(-P, aQ) == 1
    a = rnd.randrange(1, bls.R)
    pa = bls.g1_compress(bls.g1_mul(bls.G1_GEN, a))
    g2 = bls.g2_compress(bls.G2_GEN)
    ng1 = bls.g1_compress(bls.g1_neg(bls.G1_GEN))
    qa = bls.g2_compress(bls.g2_mul(bls.G2_GEN, a))
    assert hc.hc_miller2_digit_cmp(pa, g2, ng1, qa, ctypes.byref(chk)) == 3 and chk.value == 1


def test_fe1_chain_matches_final_exponentiation(hc):
    """k_fe1's five-step final exponentiation (fe1d.hpp: the Fq12 values handed between kernels
    through packed slots, products streaming one operand from a slot) gives the same element as
    final_exponentiation_d, for checks that hold and checks that do not (HBX_DCHECK bounds on)."""
    rnd = random.Random(23)
    for trial in range(4):
        a = rnd.randrange(1, bls.R)
        pa = bls.g1_compress(bls.g1_mul(bls.G1_GEN, a))
        q = bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R))
        qa = bls.g2_compress(q)
        ng1 = bls.g1_compress(bls.g1_neg(bls.G1_GEN))
        qb = bls.g2_compress(bls.g2_mul(q, a + (trial & 1)))  # holds for even trials
        assert hc.hc_fe1_chain_cmp(pa, qa, ng1, qb) == (7 if trial % 2 == 0 else 3)


def test_fe1_step0_decides_t_one(hc):
    """a ciphertext with r = m = 3(x^2 - 1) makes W = H' and every honest share [m] pk_i,
    so the check's two Miller pairs are H''s lines at P and -P and t = 1 after the easy part; the
    compressed squarings of the chain would then all meet g3 = 0 (the fallback).  fe1_step0 reports
    t = 1 (k_fe1<0> decides the share valid there); an ordinary valid check is not t = 1."""
    m = 3 * (bls.BLS_X ** 2 - 1) % bls.R
    pk_m = bls.g1_mul(bls.G1_GEN, 0x5eed * m % bls.R)
    hp = bls.g2_compress(bls.g2_mul(bls.G2_GEN, 0xbeef))
    r = hc.hc_fe1_step0_one(bls.g1_compress(pk_m), hp, bls.g1_compress(bls.g1_neg(pk_m)), hp)
    assert r & 1 and r & 2  # t = 1, and the runs would degenerate
    a = 0x1234
    q = bls.g2_mul(bls.G2_GEN, 0x777)
    r = hc.hc_fe1_step0_one(bls.g1_compress(bls.g1_mul(bls.G1_GEN, a)), bls.g2_compress(q),
                            bls.g1_compress(bls.g1_neg(bls.G1_GEN)), bls.g2_compress(bls.g2_mul(q, a)))
    assert r == 4  # holds, decided by the whole chain


def test_sha256_and_hash_g1_g2(hc):
    for n in (0, 1, 55, 56, 64, 65, 200):
        m = bytes(range(n % 251))[:n] + bytes(max(0, n - 251))
        out = ctypes.create_string_buffer(32)
        hc.hc_sha256(m, len(m), out)
        assert out.raw == hashlib.sha256(m).digest()
    u = bls.g1_mul(bls.G1_GEN, 77)
    for v in (b"", b"x" * 64, b"y" * 65):
        out = ctypes.create_string_buffer(96)
        assert hc.hc_hash_g1_g2(bls.g1_compress(u), v, len(v), out) == 0
        assert out.raw == bls.g2_compress(tc.hash_g1_g2(u, v))


def test_sha3_256_and_digest_switch(hc):
    """Keccak-f[1600] SHA3-256 (the opt-in DIGEST) vs hashlib, every padding
    boundary of the 136-byte rate, and hash_g1_g2 under DIGEST = SHA3-256 vs the oracle."""
    hc.hc_sha3_256.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    hc.hc_sha3_256_2.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    hc.hc_hash_g1_g2_v.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p]
    rnd = random.Random(3)
    for n in (0, 1, 31, 135, 136, 137, 271, 272, 273, 1000):
        m = bytes(rnd.getrandbits(8) for _ in range(n))
        out = ctypes.create_string_buffer(32)
        hc.hc_sha3_256(m, len(m), out)
        assert out.raw == hashlib.sha3_256(m).digest(), n
        k = n // 3
        hc.hc_sha3_256_2(m[:k], k, m[k:], n - k, out)
        assert out.raw == hashlib.sha3_256(m).digest(), n
    u = bls.g1_mul(bls.G1_GEN, 91)
    for v in (b"", b"x" * 64, b"y" * 65, b"z" * 300):
        out = ctypes.create_string_buffer(96)
        assert hc.hc_hash_g1_g2_v(bls.g1_compress(u), v, len(v), 1, out) == 0
        assert out.raw == bls.g2_compress(tc.hash_g1_g2(u, v, "sha3_256"))


def test_g2_clear_cofactor_psi(hc):
    """h2 * P by the psi / GLS route equals the full 507-bit multiplication (pairing 0.14's
    scale_by_cofactor) for points of E'(Fq2) OUTSIDE G2."""
    rnd = random.Random(11)
    done = 0
    while done < 3:
        x = (rnd.randrange(bls.P), rnd.randrange(bls.P))
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is None:
            continue
        pt = (x, y)
        assert bls.g2_mul(pt, bls.R) is not None          # not in G2
        o1, o2 = ctypes.create_string_buffer(96), ctypes.create_string_buffer(96)
        assert hc.hc_g2_clear_cofactor(bls.g2_compress(pt), o1) == 0
        assert hc.hc_g2_mul_cofactor(bls.g2_compress(pt), o2) == 0
        assert o1.raw == o2.raw == bls.g2_compress(bls.g2_mul(pt, bls.H2))
        done += 1


def test_heff_scaled_hash_point(hc):
    """k_prepare_ct keeps Q = h_eff P = [3(x^2-1)] (h2 P) as H'; the checks scale their G1 side by
    m = 3(x^2-1) (k_scale_keys, G1_MGEN) and hbx_get_ct_hashes maps Q back to h2 P."""
    rnd = random.Random(12)
    m = 3 * (0xD201000000010000 ** 2 - 1)
    done = 0
    while done < 2:
        x = (rnd.randrange(bls.P), rnd.randrange(bls.P))
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is None:
            continue
        h = bls.g2_mul((x, y), bls.H2)
        q96, h96 = ctypes.create_string_buffer(96), ctypes.create_string_buffer(96)
        assert hc.hc_g2_heff(bls.g2_compress((x, y)), q96, h96) == 0
        assert q96.raw == bls.g2_compress(bls.g2_mul(h, m))
        assert h96.raw == bls.g2_compress(h)
        done += 1
    pk = bls.g1_mul(bls.G1_GEN, rnd.randrange(1, bls.R))
    out = ctypes.create_string_buffer(48)
    assert hc.hc_g1_scale_heff_m(bls.g1_compress(pk), out) == 0
    assert out.raw == bls.g1_compress(bls.g1_mul(pk, m))


def _slow_gcd_inputs(mod):
    """Inputs with long continued fractions against the modulus (x / m near 1/phi, and neighbours):
    the slowest gcds."""
    a, b = 1, 1
    while b < mod << 8:  # consecutive Fibonacci numbers: b / a -> phi to 2 x 392 bits
        a, b = b, a + b
    out = []
    for k in range(-40, 41):
        x = mod * a // b + k
        out += [x % mod, (mod - x) % mod, (2 * x) % mod]
    return [x for x in out if x]


def _hddivsteps_needed(x, m):
    """Steps the half-delta divstep recurrence (field.hpp binv_limbs) takes until g = 0."""
    delta, f, g, n = 1, m, x, 0  # 2 delta
    while g:
        if delta > 0 and g & 1:
            delta, f, g = 2 - delta, g, (g - f) // 2
        elif g & 1:
            delta, g = 2 + delta, (g + f) // 2
        else:
            delta, g = 2 + delta, g // 2
        n += 1
    return n


def test_hddivsteps_bound():
    """binv_limbs runs 31 batches of 30 half-delta divsteps at 381 bits (21 at 255 bits): the
    recurrence reaches g = 0 well inside that on random and slow-gcd inputs; the bound it relies on
    (floor((45907 b + 26313) / 19929), libsecp256k1's safegcd) is 886 / 590 steps."""
    rnd = random.Random(31)
    for mod, bits, batches in ((bls.P, 384, 31), (bls.R, 256, 21)):
        bound = (45907 * bits + 26313) // 19929
        assert bound <= 30 * batches - 30
        worst = max(_hddivsteps_needed(x, mod) for x in _slow_gcd_inputs(mod) + [rnd.randrange(1, mod) for _ in range(3000)])
        assert worst <= bound, (mod, worst, bound)


def _digits14(v):
    """v (any integer) as 14 normalised signed digits: digits 0..12 in [0, 2^28), digit 13 the rest."""
    ds = []
    for _ in range(13):
        ds.append(v & 0xFFFFFFF)
        v >>= 28
    return ds + [v]


def test_fqd_inv_digit_form(hc):
    """fieldd.hpp fqd_inv (divsteps on the 28-bit digits, the final exponentiation's and the Miller
    kernels' inversions since round 6) against Python's modular inverse: the input is x R' (R' =
    2^392) as any representative in (-2p, 3p), the output must be x^-1 R' mod p, normalised digits,
    value in (-p, 2p); x = 0 gives 0 with the zero flag."""
    rnd = random.Random(28)
    p, rr = bls.P, 1 << 392
    xs = [0, 1, 2, 3, p - 1, p - 2, (p + 1) // 2] + [rnd.randrange(p) for _ in range(400)] + _slow_gcd_inputs(p)[:200]
    for n, x in enumerate(xs):
        a = x * rr % p + p * rnd.choice((-2, -1, 0, 1, 2))  # any representative in (-2p, 3p)
        if a <= -2 * p or a >= 3 * p:
            a = x * rr % p
        ad = (ctypes.c_int32 * 14)(*[d if d < (1 << 31) else d - (1 << 32) for d in _digits14(a)])
        out = (ctypes.c_int32 * 14)()
        z = hc.hc_fqd_inv(ad, out)
        got = sum(int(out[i]) << (28 * i) for i in range(14))
        assert all(0 <= out[i] < (1 << 28) for i in range(13)), x
        assert -p < got < 2 * p, x
        if x == 0:
            assert z == 1 and got % p == 0
        else:
            assert z == 0 and got % p == pow(x, -1, p) * rr % p, (n, x)
    # the divsteps' slowest inputs as the canonical value the steps run on: out = a^-1 R'^2
    for a in _slow_gcd_inputs(p):
        ad = (ctypes.c_int32 * 14)(*[d if d < (1 << 31) else d - (1 << 32) for d in _digits14(a % p)])
        out = (ctypes.c_int32 * 14)()
        hc.hc_fqd_inv(ad, out)
        got = sum(int(out[i]) << (28 * i) for i in range(14))
        assert got % p == pow(a, -1, p) * rr * rr % p, a


def test_binv_divsteps(hc):
    """binv_limbs (batched Bernstein-Yang divsteps, every inversion of the kernels) against
    Python's modular inverse, mod p and mod r, on random and edge values (0 -> 0)."""
    rnd = random.Random(14)
    for mod, nl, which in ((bls.P, 12, 0), (bls.R, 8, 1)):
        vals = [0, 1, 2, 3, mod - 1, mod - 2, (mod + 1) // 2, 1 << 31, (1 << (32 * nl - 4)) % mod]
        vals += [rnd.randrange(mod) for _ in range(300)]
        vals += [rnd.randrange(1 << rnd.randrange(1, 40)) for _ in range(50)]  # short values
        vals += _slow_gcd_inputs(mod)
        vals += [rnd.randrange(mod) for _ in range(3000)]
        for x in vals:
            xa = (ctypes.c_uint32 * nl)(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(nl)])
            out = (ctypes.c_uint32 * nl)()
            hc.hc_binv(xa, which, out)
            got = sum(int(out[i]) << (32 * i) for i in range(nl))
            assert got == (pow(x, -1, mod) if x else 0), (which, x)


def test_lines_from_jacobian_point(hc):
    """k_prepare_lines makes H's lines from (X, Y) of its Jacobian form (a point of the isomorphic
    twist; no inversion in k_prepare_ct) and k_normalise_lines corrects them by Z: the 68 lines
    equal the affine point's, for any representative z."""
    rnd = random.Random(13)
    for s in (3, 0x1234567, bls.R - 5):
        q = bls.g2_compress(bls.g2_mul(bls.G2_GEN, s))
        z0, z1 = rnd.randrange(1, bls.P), rnd.randrange(bls.P)
        assert hc.hc_lines_jac_cmp(q, z0.to_bytes(48, "big"), z1.to_bytes(48, "big")) == 0
    # z = 1 is the affine case itself
    assert hc.hc_lines_jac_cmp(bls.g2_compress(bls.G2_GEN), (1).to_bytes(48, "big"), bytes(48)) == 0


def test_pairing_check_mixed_lines(hc):
    """Signature-share check shape: pair A over prepared lines, pair B's lines generated on the
    fly (un-normalised) from a varying G2 point."""
    a = 0xABCDEF0123
    pa = bls.g1_compress(bls.g1_mul(bls.G1_GEN, a))
    h = bls.g2_compress(bls.G2_GEN)
    ng1 = bls.g1_compress(bls.g1_neg(bls.G1_GEN))
    sig = bls.g2_compress(bls.g2_mul(bls.G2_GEN, a))
    assert hc.hc_pairing_check_mixed(pa, h, ng1, sig) == 1      # e(aP, Q) e(-P, aQ) == 1
    bad = bls.g2_compress(bls.g2_mul(bls.G2_GEN, a + 5))
    assert hc.hc_pairing_check_mixed(pa, h, ng1, bad) == 0


def test_digit_tower_mixed_check(hc):
    """The coin share check in the digit tower (pairingd.hpp miller_loop_mixed_d: lines of the
    signature share generated on the fly) equals pairing.hpp's element for element, valid and
    invalid shares."""
    rnd = random.Random(23)
    for trial in range(3):
        sk = rnd.randrange(1, bls.R)
        h = bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R))
        pk = bls.g1_compress(bls.g1_mul(bls.G1_GEN, sk))
        sig = bls.g2_compress(bls.g2_mul(h, sk + (trial == 2)))
        ng1 = bls.g1_compress(bls.g1_neg(bls.G1_GEN))
        want = 1 if trial < 2 else 0
        assert hc.hc_pairing_check_mixed_d(pk, bls.g2_compress(h), ng1, sig) == want + 6


def test_g1_mul_glv(hc):
    """k_combine's two-lane GLV scalar multiplication (k1 P + k2 phi(P)) against the oracle."""
    rnd = random.Random(7)
    pt = bls.g1_mul(bls.G1_GEN, 0xC0FFEE)
    comp = bls.g1_compress(pt)
    lam = 0xd201000000010000 ** 2 - 1
    for k in [0, 1, 2, lam - 1, lam, lam + 1, lam * lam, bls.R - 1] + [rnd.randrange(bls.R) for _ in range(8)]:
        out = ctypes.create_string_buffer(48)
        assert hc.hc_g1_mul_glv(comp, _be(k, 32), out) == 0
        assert out.raw == bls.g1_compress(bls.g1_mul(pt, k)), hex(k)


def _rand_curve_point_g1(rnd):
    while True:
        x = rnd.randrange(bls.P)
        y = bls.fq_sqrt((x * x * x + bls.B1) % bls.P)
        if y is not None:
            return (x, y)


def _rand_curve_point_g2(rnd):
    while True:
        x = (rnd.randrange(bls.P), rnd.randrange(bls.P))
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is not None:
            return (x, y)


def test_subgroup_checks_match_order_r(hc):
    """g1_is_torsion_free / g2_is_torsion_free (the endomorphism criteria the ciphertext decode
    uses) agree with the oracle's [r] P == O on subgroup points and on random curve points, which
    lie outside G1 / G2 (pairing 0.14's into_affine rejects those)."""
    rnd = random.Random(23)
    for k in (1, 5, bls.R - 1, rnd.randrange(1, bls.R)):
        p1 = bls.g1_mul(bls.G1_GEN, k)
        assert hc.hc_g1_torsion_free(_be(p1[0]), _be(p1[1])) == 1
        q = bls.g2_mul(bls.G2_GEN, k)
        assert hc.hc_g2_torsion_free(_be(q[0][1]) + _be(q[0][0]) + _be(q[1][1]) + _be(q[1][0])) == 1
    for _ in range(3):
        p1 = _rand_curve_point_g1(rnd)
        in_g1 = bls.g1_mul(p1, bls.R) is None
        assert hc.hc_g1_torsion_free(_be(p1[0]), _be(p1[1])) == int(in_g1)
        q = _rand_curve_point_g2(rnd)
        in_g2 = bls.g2_mul(q, bls.R) is None
        assert hc.hc_g2_torsion_free(_be(q[0][1]) + _be(q[0][0]) + _be(q[1][1]) + _be(q[1][0])) == int(in_g2)
    # a point of small order times a G1 point: on the curve, not in G1 (and the small-order points
    # themselves: their double-and-add meets the identity and +-P, the exact special cases)
    for _ in range(3):
        small = bls.g1_mul(_rand_curve_point_g1(rnd), bls.R)  # order divides h1
        if small is None:
            continue
        assert hc.hc_g1_torsion_free(_be(small[0]), _be(small[1])) == 0
        mixed = bls.g1_add(small, bls.g1_mul(bls.G1_GEN, 9))
        assert hc.hc_g1_torsion_free(_be(mixed[0]), _be(mixed[1])) == 0
    for k in (3, 11, 10177):  # points of order k | h1 (k prime): [h1 / k] of a random point
        h1 = 0x396C8C005555E1568C00AAAB0000AAAB
        q = bls.g1_mul(_rand_curve_point_g1(rnd), bls.R * (h1 // k))
        if q is not None:
            assert hc.hc_g1_torsion_free(_be(q[0]), _be(q[1])) == 0


def test_g2_membership_from_miller_T(hc):
    """The coin share checks take sigma's membership in G2 from their Miller loop's final
    T = [|x|] sigma (hbx_kernels.hip k_verify_sig_shares[2]); it must agree with the decode-time
    check (g2_is_torsion_free) on subgroup points, on points of E'(Fq2) outside G2, and on every
    decodable share of the coin fixtures (incl. their cofactor-torsion shares)."""
    import numpy as np

    hc.hc_g2_membership.argtypes = [ctypes.c_char_p]
    rnd = random.Random(5)
    seen = {0: 0, 3: 0}
    for _ in range(3):
        q = bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R))
        r = hc.hc_g2_membership(bls.g2_compress(q))
        assert r == 3
        seen[3] += 1
    k = 1
    while seen[0] < 3:  # points of the twist that are not cofactor-cleared: almost surely outside G2
        k += 1
        x = (k, 1)
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is None:
            continue
        r = hc.hc_g2_membership(bls.g2_compress((x, y)))
        assert r in (0, 3)
        seen[r] += 1
    for name in ("coin_n7", "coin_n128"):
        d = np.load(os.path.join(os.path.dirname(__file__), "golden", name + ".npz"), allow_pickle=False)
        sigs = d["sigs"].reshape(-1, 96)
        for s in sigs[:: max(1, len(sigs) // 400)]:
            r = hc.hc_g2_membership(s.tobytes())
            assert r in (-1, 0, 3), r
        st = d["expect_share_status"].reshape(-1)
        for s in sigs[st == 3]:  # UNDECODABLE shares: bad bytes or torsion; both checks reject alike
            assert hc.hc_g2_membership(s.tobytes()) in (-1, 0)


def test_g2_mul_u64_windows_match_naf(hc):
    """k_combine_sigs' 64-bit G2 multiplications by 4-bit windows, 12-limb (curve.hpp) and digit
    tower (g2d.hpp), equal the NAF ladder's."""
    hc.hc_g2_mul_u64_cmp.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    rnd = random.Random(9)
    q = bls.g2_compress(bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R)))
    for k in [0, 1, 2, 15, 16, 17, 0x10, 0xF000000000000000, 0xFFFFFFFFFFFFFFFF, 0xd201000000010000] + [rnd.getrandbits(64) for _ in range(6)]:
        assert hc.hc_g2_mul_u64_cmp(q, k) == 1, hex(k)


def test_g1_mul_u128_digit_tower(hc):
    """k_combine's GLV-half G1 multiplications in the digit tower (g1d.hpp g1d_mul_u128_w4) equal
    the 12-limb windowed ones, zero and single-window scalars included."""
    hc.hc_g1_mul_u128_cmp.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32)]
    rnd = random.Random(31)
    p = bls.g1_compress(bls.g1_mul(bls.G1_GEN, rnd.randrange(1, bls.R)))
    ks = [0, 1, 2, 15, 16, 17, 1 << 124, (1 << 128) - 1, 0xF << 124] + [rnd.getrandbits(128) for _ in range(6)]
    for k in ks:
        k4 = (ctypes.c_uint32 * 4)(*[(k >> (32 * i)) & 0xFFFFFFFF for i in range(4)])
        assert hc.hc_g1_mul_u128_cmp(p, k4) == 1, hex(k)


def test_g2d_add_special_cases(hc):
    """k_combine_sigs' digit-tower G2 addition (g2d.hpp g2d_add) equals curve.hpp g2_add on general
    Jacobian operands and on every special case (equal, opposite, identity operands), decided by
    exact tests mod p; and fqd_is_zero_mod on unnormalised multiples of p."""
    hc.hc_g2d_add_cases.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64]
    assert hc.hc_fqd_is_zero_mod() == 1
    rnd = random.Random(23)
    for z0 in (1, 3, 0xFFFFFFFF12345678):
        p = bls.g2_compress(bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R)))
        q = bls.g2_compress(bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R)))
        assert hc.hc_g2d_add_cases(p, q, z0) == 63


def test_miller_gen_matches_mixed(hc):
    """The two-lane coin check's inlined one-pair loop equals the mixed loop with pair A off."""
    hc.hc_miller_gen_cmp.argtypes = [ctypes.c_char_p, ctypes.c_int]
    rnd = random.Random(17)
    for _ in range(3):
        q = bls.g2_compress(bls.g2_mul(bls.G2_GEN, rnd.randrange(1, bls.R)))
        assert hc.hc_miller_gen_cmp(q, 0) == 1
        assert hc.hc_miller_gen_cmp(q, 1) == 1  # (qx, qy, bx, by) parked in the lane's slot


def test_digit_tower_square_roots(hc):
    """hash_g2_group's square roots with the digit-tower exponentiation equal field.hpp's."""
    hc.hc_sqrt_d_cmp.argtypes = [ctypes.c_char_p]
    rnd = random.Random(21)
    for _ in range(12):
        x = rnd.randrange(1, bls.P)
        assert hc.hc_sqrt_d_cmp(x.to_bytes(48, "big")) == 1
