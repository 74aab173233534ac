"""The input-triple lookup of broadcast.hpp k_rs_code_perm3, restated on the host: a byte's low six
bits through the 8-entry tables T0 (bits 0-2) and T1 (bits 3-5) of its own coefficient, and the
three inputs' two-bit tops regrouped as two 3-bit indices into the mixed tables
M1[a7 a6 | b6] = c_a (a_top << 6) ^ c_b (b6 << 6) and M2[b7 | c7 c6] = c_b (b7 << 7) ^ c_c (c_top << 6)
(built per pass in the kernel from the per-coefficient gf_ptab tables).  XOR of the eight lookups
must equal c_a a ^ c_b b ^ c_c c in GF(2^8) (oracle/rs_merkle.py gmul).  The GPU outputs
themselves: tests/test_gpu_broadcast.py."""
import random

from oracle import rs_merkle as rm


def ptab(c):
    t0 = [rm.gmul(c, i) for i in range(8)]
    t1 = [rm.gmul(c, i << 3) for i in range(8)]
    t2 = [rm.gmul(c, i << 6) for i in range(4)]
    return t0, t1, t2


def mixed(ta, tb, tc):
    m1 = [ta[2][j & 3] ^ (tb[2][1] if j & 4 else 0) for j in range(8)]
    m2 = [(tb[2][2] if j & 1 else 0) ^ tc[2][j >> 1] for j in range(8)]
    return m1, m2


def triple_lookup(a, b, c, ta, tb, tc, m1, m2):
    s1 = (a >> 6) | (((b >> 6) & 1) << 2)
    s2 = (b >> 7) | ((c >> 6) << 1)
    x = 0
    for v, t in ((a, ta), (b, tb), (c, tc)):
        x ^= t[0][v & 7] ^ t[1][(v >> 3) & 7]
    return x ^ m1[s1] ^ m2[s2]


def test_triple_lookup_is_the_gf_product_sum():
    rnd = random.Random(7)
    coefs = [(1, 1, 1), (0, 0, 0), (0x53, 0xCA, 0x01), (255, 2, 0)] + [tuple(rnd.randrange(256) for _ in range(3)) for _ in range(12)]
    for ca, cb, cc in coefs:
        ta, tb, tc = ptab(ca), ptab(cb), ptab(cc)
        m1, m2 = mixed(ta, tb, tc)
        samples = [(a, b, c) for a in (0, 1, 0x40, 0x80, 0xC0, 0xFF) for b in (0, 0x40, 0x80, 0xFF) for c in (0, 0x7F, 0xC0, 0xFF)]
        samples += [(rnd.randrange(256), rnd.randrange(256), rnd.randrange(256)) for _ in range(2000)]
        for a, b, c in samples:
            want = rm.gmul(ca, a) ^ rm.gmul(cb, b) ^ rm.gmul(cc, c)
            assert triple_lookup(a, b, c, ta, tb, tc, m1, m2) == want
