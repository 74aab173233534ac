"""Generate the committed golden fixtures for the threshold-decryption path.

    python tests/golden/make_golden.py [names...]   # default: all of FIXTURES below

Inputs are seeded (SURVEY.md §8(d) seeds 0x68626278_0000000{1..4}); every expected output comes
from the CPU restatement in ``oracle/`` (canonical pairing; digest variant recorded in the fixture
as ``digest``).  Each fixture is one HoneyBadger node-epoch (or a set of
proposer columns of one) as stack A of SURVEY.md §3 sees it:

* N nodes, f = (N-1)//3, t = f + 1 (messaging.rs:258, honey_badger.rs:328);
* ciphertexts PublicKey::encrypt(msg_j, r_j) (honey_badger.rs:116) of the master key;
* share matrix S[j][i] = sk_i * U_j (decrypt_share_no_verify, :403), with corruptions built like
  the reference's FaultyShareAdversary (tests/honey_badger.rs:99-106: the sender's valid share of
  a DIFFERENT ciphertext, "X marks the spot");
* expected: per-ciphertext HBX_CT_* status, per-share HBX_SHARE_* status (include/hbx.h),
  per-proposer combine status and plaintext (PublicKeySet::decrypt, :340), the hoisted
  H_j = hash_g1_g2(U_j, V_j), in plain mode and in own-share mode (node ``me`` computes its own
  share, whose check doubles as Ciphertext::verify);
* producer data: secret shares, r_j, messages and the untampered ciphertexts, for hbx_encrypt /
  hbx_decrypt_shares / hbx_public_keys parity.

Fixtures (BASELINE.json configs):
  hb_epoch_n4, hb_epoch_n7  every edge case: W of another ciphertext (ShareDecryptionFailed), U / W
                            off the subgroup (InvalidCiphertext), U = W = identity (valid), absent,
                            undecodable, off-subgroup and identity shares, a starved proposer
  hb_epoch_n10              config 1 (the simulation example's 10 nodes): mixed |v|, a few faults
  hb_epoch_n64              config 2: N = 64, 64 proposers x 64 shares, |v| = 1 KiB, 1 in 64
                            shares corrupted
  hb_cols_n256              config 3: N = 256, 4 proposer columns (t = 86), |v| = 1 MiB / 1 KiB /
                            64 B / 1 B, 1 in 64 shares corrupted
"""
from __future__ import annotations

import hashlib
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import threshold as tc  # noqa: E402
from oracle.chacha_rand04 import ChaChaRng04  # noqa: E402

SEED = 0x68626278
# include/hbx.h
SHARE_INVALID, SHARE_VALID, SHARE_ABSENT, SHARE_UNDECODABLE, SHARE_SKIPPED_CT = 0, 1, 2, 3, 4
CT_INVALID, CT_VALID, CT_UNDECODABLE = 0, 1, 3
E_NOT_ENOUGH, E_INVALID_CT = -3, -7

FIXTURES = {
    # name: (n, proposers, |v| pattern, edge cases, corrupt 1 in k (0 = the hand-placed ones only))
    "hb_epoch_n4": (4, 4, [1, 64, 65, 200], True, 0),
    "hb_epoch_n7": (7, 7, [1, 64, 65, 200], True, 0),
    "hb_epoch_n10": (10, 10, [100, 1024, 7, 65, 300], True, 0),
    "hb_epoch_n64": (64, 64, [1024], False, 64),
    "hb_cols_n256": (256, 4, [1 << 20, 1024, 64, 1], False, 64),
    # DIGEST = SHA3-256 (tiny-keccak threshold_crypto revisions; hbx_set_digest)
    "hb_epoch_n7_sha3": (7, 7, [1, 64, 65, 200], True, 0, "sha3_256"),
}


def off_subgroup_g1(seed: int):
    """A point on y^2 = x^3 + 4 that is not in G1."""
    x = seed
    while True:
        y = bls.fq_sqrt((x ** 3 + bls.B1) % bls.P)
        if y is not None and bls.g1_mul((x, y), bls.R) is not None:
            return (x, y)
        x += 1


def off_subgroup_g2(seed: int):
    """A point on y^2 = x^3 + 4(u + 1) that is not in G2."""
    x0 = seed
    while True:
        x = (x0, 1)
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is not None and bls.g2_mul((x, y), bls.R) is not None:
            return (x, y)
        x0 += 1


def _verify(args):
    pk, share, h, w = args
    return bls.pairing_product_is_one([(share, h), (bls.g1_neg(pk), w)])


def _sha(b: bytes) -> np.ndarray:
    return np.frombuffer(hashlib.sha256(b).digest(), dtype=np.uint8)


def make_epoch(n: int, p: int, v_lens, edge: bool, corrupt_every: int, pool, digest: str = "sha256"):
    f = (n - 1) // 3
    t = f + 1
    sks = tc.SecretKeySet.random(f, ChaChaRng04([SEED, 1]))
    pks = sks.public_keys()
    pk_shares = [pks.public_key_share(i) for i in range(n)]
    sk_shares = [sks.secret_key_share(i) for i in range(n)]
    data_rng = np.random.default_rng([SEED, 2, n])
    r_rng = ChaChaRng04([SEED, 3])
    msgs, rs, honest = [], [], []
    for j in range(p):
        ln = v_lens[j % len(v_lens)]
        msg = data_rng.integers(0, 256, size=ln, dtype=np.uint8).tobytes()
        r = tc.fr_rand(r_rng)
        honest.append(tc.encrypt(pks.public_key(), msg, r, digest))
        msgs.append(msg)
        rs.append(r)
    fake = tc.encrypt(pks.public_key(), b"X marks the spot", tc.fr_rand(r_rng), digest)  # tests/honey_badger.rs:90
    enc_u = [bls.g1_compress(c[0]) for c in honest]
    enc_w = [bls.g2_compress(c[2]) for c in honest]
    wire_u, wire_w = list(enc_u), list(enc_w)
    v_bytes = [bytes(c[1]) for c in honest]
    enc_ok = np.ones(p, dtype=bool)  # hbx_encrypt reproduces (u, v, w) of this proposer
    ident_ct = -1
    if edge:
        wire_w[0] = enc_w[1]                                   # ShareDecryptionFailed
        if p >= 7:
            wire_u[1] = bls.g1_compress(off_subgroup_g1(12345))  # InvalidCiphertext (U)
            wire_w[2] = bls.g2_compress(off_subgroup_g2(777))    # InvalidCiphertext (W)
            ident_ct = 3
        else:
            ident_ct = 1
        # U = W = identity: e(g1, O) = e(O, H) = 1 -> a valid ciphertext whose shares are O
        wire_u[ident_ct] = bls.g1_compress(None)
        wire_w[ident_ct] = bls.g2_compress(None)
        v_bytes[ident_ct] = data_rng.integers(0, 256, size=40, dtype=np.uint8).tobytes()
        enc_ok[ident_ct] = False
    # decoded ciphertexts (None = undecodable) and statuses
    cts, ct_status, hashes = [], [], []
    for j in range(p):
        try:
            u = bls.g1_decompress(wire_u[j])
            w = bls.g2_decompress(wire_w[j])
        except ValueError:
            cts.append(None)
            ct_status.append(CT_UNDECODABLE)
            hashes.append(None)
            continue
        ct = (u, v_bytes[j], w)
        h = tc.hash_g1_g2(u, v_bytes[j], digest)
        cts.append(ct)
        hashes.append(h)
        ct_status.append(CT_VALID if tc.ciphertext_verify(ct, hash_pt=h) else CT_INVALID)

    # share matrix
    shares = np.zeros((p, n, 48), dtype=np.uint8)
    present = np.ones((p, n), dtype=bool)
    share_pt = {}
    undecodable = set()
    crng = np.random.default_rng([SEED, 4, n])
    corrupt = (crng.integers(0, corrupt_every, size=(p, n)) == 0) if corrupt_every else np.zeros((p, n), bool)
    for j in range(p):
        u_pt = cts[j][0] if cts[j] is not None else honest[j][0]
        for i in range(n):
            s = bls.g1_mul(fake[0], sk_shares[i]) if corrupt[j, i] else bls.g1_mul(u_pt, sk_shares[i])
            share_pt[(j, i)] = s
    me = n - 2
    if edge:
        regular = [j for j in range(p) if ct_status[j] == CT_VALID and j != ident_ct]
        ja, jb = regular[0], regular[1 % len(regular)]
        starve = p - 1 if p >= 7 else None  # N = 4 keeps one proposer that decrypts
        # FaultyShareAdversary-style corruptions, an absent share, the identity and an off-subgroup point
        for (j, i) in [(ja, n - 1), (jb, 0)]:
            share_pt[(j, i)] = bls.g1_mul(fake[0], sk_shares[i])
            corrupt[j, i] = True
        present[ja, 0] = False
        share_pt[(jb, 1 % n)] = None                       # identity share: verifies false
        corrupt[jb, 1 % n] = True
        off = off_subgroup_g1(999)
        undecodable.add((ja, 1 % n))                       # x >= p (bad encoding)
        undecodable.add((jb, 2 % n))                       # on the curve, off the subgroup
        # starve the last proposer: t - 1 valid shares, the rest absent (own share rescues it)
        if starve is not None:
            for i in range(t - 1, n):
                present[starve, i] = False
            for i in range(n):
                undecodable.discard((starve, i))
    for (j, i), pt in share_pt.items():
        shares[j, i] = np.frombuffer(bls.g1_compress(pt), dtype=np.uint8)
    if edge:
        shares[ja, 1 % n] = 0xFF
        shares[ja, 1 % n, 0] = 0x9F
        shares[jb, 2 % n] = np.frombuffer(bls.g1_compress(off), dtype=np.uint8)

    # expected share statuses (plain mode), verified by the oracle where a check is due
    status = np.full((p, n), SHARE_ABSENT, dtype=np.uint8)
    jobs, where = [], []
    for j in range(p):
        for i in range(n):
            if not present[j, i]:
                continue
            if (j, i) in undecodable:
                status[j, i] = SHARE_UNDECODABLE
            elif ct_status[j] != CT_VALID:
                status[j, i] = SHARE_SKIPPED_CT
            else:
                jobs.append((pk_shares[i], share_pt[(j, i)], hashes[j], cts[j][2]))
                where.append((j, i))
    res = pool.map(_verify, jobs, chunksize=8) if pool is not None else list(map(_verify, jobs))
    for (j, i), ok in zip(where, res):
        status[j, i] = SHARE_VALID if ok else SHARE_INVALID
    # sanity: verification == "not corrupted" for the checked shares
    for (j, i), ok in zip(where, res):
        assert ok == (not corrupt[j, i]), (j, i)

    def combine(st, own):
        comb = np.zeros(p, dtype=np.int32)
        plains = []
        for j in range(p):
            if ct_status[j] != CT_VALID:
                comb[j] = E_INVALID_CT
                plains.append(b"")
                continue
            idx = [i for i in range(n) if st[j, i] == SHARE_VALID]
            if len(idx) < t:
                comb[j] = E_NOT_ENOUGH
                plains.append(b"")
                continue
            pts = [(i, (bls.g1_mul(cts[j][0], sk_shares[me]) if (own and i == me) else share_pt[(j, i)]))
                   for i in idx[:t]]
            pt = tc.decrypt(pks, pts, cts[j], digest)
            if j != ident_ct:
                assert pt == msgs[j]
            plains.append(pt)
        return comb, plains

    comb, plains = combine(status, False)
    status_own = status.copy()
    for j in range(p):
        status_own[j, me] = SHARE_VALID if ct_status[j] == CT_VALID else SHARE_SKIPPED_CT
    comb_own, plains_own = combine(status_own, True)

    v_off = np.zeros(p + 1, dtype=np.uint64)
    v_off[1:] = np.cumsum([len(v) for v in v_bytes])
    m_off = np.zeros(p + 1, dtype=np.uint64)
    m_off[1:] = np.cumsum([len(m) for m in msgs])
    small = int(v_off[-1]) <= 1 << 16

    def blob(pl, cs):
        out = np.zeros(int(v_off[-1]), dtype=np.uint8)
        for j in range(p):
            if cs[j] == 0:
                out[int(v_off[j]):int(v_off[j + 1])] = np.frombuffer(pl[j], dtype=np.uint8)
        return out

    d = dict(
        digest=np.array(digest), n=np.int64(n), t=np.int64(t),
        pk_comp=np.stack([np.frombuffer(bls.g1_compress(q), dtype=np.uint8) for q in pk_shares]),
        master_pk=np.frombuffer(bls.g1_compress(pks.public_key()), dtype=np.uint8),
        u=np.stack([np.frombuffer(x, dtype=np.uint8) for x in wire_u]),
        w=np.stack([np.frombuffer(x, dtype=np.uint8) for x in wire_w]),
        h=np.stack([np.frombuffer(bls.g2_compress(h), dtype=np.uint8) if h is not None else np.zeros(96, np.uint8)
                    for h in hashes]),
        v_blob=np.frombuffer(b"".join(v_bytes), dtype=np.uint8),
        v_off=v_off,
        shares=shares, present=present,
        expect_ct_status=np.array(ct_status, dtype=np.uint8),
        expect_ct_valid=np.array(ct_status, dtype=np.uint8) == CT_VALID,
        expect_share_status=status,
        expect_valid=status == SHARE_VALID,
        expect_status=comb,
        expect_plain_sha=np.stack([_sha(x) for x in plains]),
        own_me=np.int64(me),
        own_sk=np.frombuffer(sk_shares[me].to_bytes(32, "big"), dtype=np.uint8),
        expect_share_status_own=status_own,
        expect_valid_own=status_own == SHARE_VALID,
        expect_status_own=comb_own,
        expect_plain_sha_own=np.stack([_sha(x) for x in plains_own]),
        # producer side (hbx_public_keys / hbx_encrypt / hbx_decrypt_shares)
        sk_shares=np.stack([np.frombuffer(s.to_bytes(32, "big"), dtype=np.uint8) for s in sk_shares]),
        enc_r=np.stack([np.frombuffer(r.to_bytes(32, "big"), dtype=np.uint8) for r in rs]),
        enc_msg_blob=np.frombuffer(b"".join(msgs), dtype=np.uint8),
        enc_msg_off=m_off,
        enc_u=np.stack([np.frombuffer(x, dtype=np.uint8) for x in enc_u]),
        enc_w=np.stack([np.frombuffer(x, dtype=np.uint8) for x in enc_w]),
        enc_ok=enc_ok,
        corrupt=corrupt,
    )
    if small:
        d["expect_plain_blob"] = blob(plains, comb)
        d["expect_plain_blob_own"] = blob(plains_own, comb_own)
    return d


def main():
    names = sys.argv[1:] or list(FIXTURES)
    with mp.Pool(min(8, os.cpu_count() or 1)) as pool:
        for name in names:
            n, p, v_lens, edge, ce, *dg = FIXTURES[name]
            d = make_epoch(n, p, v_lens, edge, ce, pool, *dg)
            path = os.path.join(HERE, f"{name}.npz")
            np.savez_compressed(path, **d)
            st = d["expect_share_status"]
            print(path, "ct", d["expect_ct_status"].tolist()[:8], "combine", d["expect_status"].tolist()[:8],
                  "share statuses", {int(k): int((st == k).sum()) for k in np.unique(st)}, flush=True)


if __name__ == "__main__":
    main()
