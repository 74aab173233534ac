"""Generate the committed Common Coin fixtures with the oracle.

    python tests/golden/make_coin_golden.py      # coin_n4, coin_n7 (edge cases), coin_n128 (config 4)

One node's view of `count` concurrent coin instances (SURVEY.md §3 stack B): nonces formatted as
Nonce::new(invocation_id = master public key bytes, session, proposer, agreement_epoch = 2)
(src/agreement/mod.rs:155-165, messaging.rs:342-344), signature shares sig_i = sk_i * hash_g2(nonce)
(common_coin.rs:142), with faults: a share over a DIFFERENT nonce (valid signature, wrong message),
an undecodable encoding, an honest share plus a point of the cofactor part (on the curve, not in
G2: pairing's into_affine rejects it), an absent share, and one instance left with
fewer than t shares (NotEnoughShares).  coin_n128 is BASELINE config 4's shape (N = 128, t = 43)
for 4 instances (sessions 0/1, proposers 0, 1, 127) with 1 in 64 shares signed over another
nonce.  Expected: HBX_SHARE_* status per share (common_coin.rs:151), combined signature of the
first t valid shares in index order (:190), master verification (:196), parity (:173).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import threshold as tc  # noqa: E402
from oracle.chacha_rand04 import ChaChaRng04  # noqa: E402


SHARE_INVALID, SHARE_VALID, SHARE_ABSENT, SHARE_UNDECODABLE = 0, 1, 2, 3


def cofactor_point():
    """A nonzero point of E'(Fq2) killed by... nothing in G2: r * P for a random curve point P."""
    x0 = 5
    while True:
        x = (x0, 3)
        y = bls.f2_sqrt(bls.f2_add(bls.f2_mul(bls.f2_sqr(x), x), bls.B2))
        if y is not None:
            t = bls.g2_mul((x, y), bls.R)
            if t is not None:
                return t
        x0 += 1


def _verify(args):
    pk, sig, h = args
    return bls.pairing_product_is_one([(pk, h), (bls.g1_neg(bls.G1_GEN), sig)])


def make(n: int, pool=None, digest: str = "sha256"):
    f = (n - 1) // 3
    t = f + 1
    rng = ChaChaRng04([0x68626278, 0x10 + n])
    sks = tc.SecretKeySet.random(f, rng)
    pks = sks.public_keys()
    inv_id = tc.PublicKeySet.to_bytes(pks)
    big = n > 16
    specs = [(0, 0), (0, 1), (1, 0), (1, n - 1)] if big else [(0, 0), (0, 1), (1, 2)]  # (session, proposer)
    nonces = [tc.nonce_bytes(inv_id, s, p, 2) for s, p in specs]
    hs = [tc.hash_g2(x, digest) for x in nonces]
    count = len(nonces)
    sigs = np.zeros((count, n, 96), dtype=np.uint8)
    present = np.ones((count, n), dtype=bool)
    pts = {}
    for c in range(count):
        for i in range(n):
            pts[(c, i)] = tc.sign(sks.secret_key_share(i), nonces[c], hash_pt=hs[c])
    other = tc.hash_g2(b"some other nonce", digest)
    wrong = [(0, n - 1)]
    if big:
        crng = np.random.default_rng([0x68626278, 0x20 + n])
        wrong = [(c, i) for c in range(count) for i in range(n) if crng.integers(0, 64) == 0]
    for (c, i) in wrong:
        pts[(c, i)] = tc.sign(sks.secret_key_share(i), b"", hash_pt=other)   # a signature of another message
    for (c, i), p in pts.items():
        sigs[c, i] = np.frombuffer(bls.g2_compress(p), dtype=np.uint8)
    undecodable = set()
    if not big:
        sigs[1, 0] = 0xFF                               # undecodable (x >= p)
        sigs[1, 0, 0] = 0x9F
        torsion = bls.g2_add(pts[(0, 1)], cofactor_point())
        sigs[0, 1] = np.frombuffer(bls.g2_compress(torsion), dtype=np.uint8)  # honest + cofactor part
        undecodable = {(1, 0), (0, 1)}
        present[1, min(2, n - 1)] = False
        present[2, 1:] = False                          # starve instance 2: 1 share < t
    status = np.full((count, n), SHARE_ABSENT, dtype=np.uint8)
    jobs, where = [], []
    for c in range(count):
        for i in range(n):
            if not present[c, i]:
                continue
            if (c, i) in undecodable:
                status[c, i] = SHARE_UNDECODABLE
                continue
            jobs.append((pks.public_key_share(i), pts[(c, i)], hs[c]))
            where.append((c, i))
    res = pool.map(_verify, jobs, chunksize=8) if pool is not None else list(map(_verify, jobs))
    for (c, i), ok in zip(where, res):
        status[c, i] = SHARE_VALID if ok else SHARE_INVALID
        assert ok == ((c, i) not in wrong)
    expect_valid = status == SHARE_VALID
    comb_status = np.zeros(count, dtype=np.int32)
    sig_out = np.zeros((count, 96), dtype=np.uint8)
    master_ok = np.zeros(count, dtype=bool)
    parity = np.zeros(count, dtype=bool)
    for c in range(count):
        shares = [(i, pts[(c, i)]) for i in range(n) if expect_valid[c, i]]
        if len(shares) < t:
            comb_status[c] = -3
            continue
        sig = tc.combine_signatures(pks, shares)
        sig_out[c] = np.frombuffer(bls.g2_compress(sig), dtype=np.uint8)
        master_ok[c] = tc.verify_sig(pks.public_key(), sig, nonces[c], hash_pt=hs[c])
        parity[c] = tc.parity(sig)
    off = np.zeros(count + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(x) for x in nonces])
    return dict(
        digest=np.array(digest), n=np.int64(n), t=np.int64(t),
        pk_comp=np.stack([np.frombuffer(bls.g1_compress(pks.public_key_share(i)), dtype=np.uint8) for i in range(n)]),
        master_pk=np.frombuffer(bls.g1_compress(pks.public_key()), dtype=np.uint8),
        sk=np.stack([np.frombuffer(sks.secret_key_share(i).to_bytes(32, "big"), dtype=np.uint8) for i in range(n)]),
        nonce_blob=np.frombuffer(b"".join(nonces), dtype=np.uint8), nonce_off=off,
        h=np.stack([np.frombuffer(bls.g2_compress(h), dtype=np.uint8) for h in hs]),
        sigs=sigs, present=present, expect_valid=expect_valid, expect_share_status=status,
        expect_status=comb_status, expect_sig=sig_out,
        expect_master_ok=master_ok, expect_parity=parity,
    )


def main():
    specs = [(a.split("_")[0], "_".join(a.split("_")[1:]) or "sha256") for a in sys.argv[1:]] or \
        [("4", "sha256"), ("7", "sha256"), ("128", "sha256"), ("4", "sha3_256")]
    pool = mp.Pool(min(8, os.cpu_count() or 1))
    for ns, dg in specs:
        n = int(ns)
        d = make(n, pool, dg)
        path = os.path.join(HERE, f"coin_n{n}" + ("" if dg == "sha256" else "_sha3") + ".npz")
        np.savez_compressed(path, **d)
        print(path, "valid", int(d["expect_valid"].sum()), "status", d["expect_status"].tolist(),
              "master_ok", d["expect_master_ok"].tolist(), "parity", d["expect_parity"].astype(int).tolist())


if __name__ == "__main__":
    main()
