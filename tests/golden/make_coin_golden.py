"""Generate the committed Common Coin fixture (tests/golden/coin_n{4,7}.npz) with the oracle.

    python tests/golden/make_coin_golden.py

One node's view of `count` concurrent coin instances (SURVEY.md §3 stack B): nonces formatted as
Nonce::new(invocation_id = master public key bytes, session, proposer, agreement_epoch = 2)
(src/agreement/mod.rs:155-165, messaging.rs:342-344), signature shares sig_i = sk_i * hash_g2(nonce)
(common_coin.rs:142), with faults: a share over a DIFFERENT nonce (valid signature, wrong message),
an undecodable encoding, an absent share, and one instance left with fewer than t shares
(NotEnoughShares).  Expected: validity bits (common_coin.rs:151), combined signature of the first
t valid shares in index order (:190), master verification (:196), parity (:173).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import threshold as tc  # noqa: E402
from oracle.chacha_rand04 import ChaChaRng04  # noqa: E402


def make(n: int):
    f = (n - 1) // 3
    t = f + 1
    rng = ChaChaRng04([0x68626278, 0x10 + n])
    sks = tc.SecretKeySet.random(f, rng)
    pks = sks.public_keys()
    inv_id = tc.PublicKeySet.to_bytes(pks)
    specs = [(0, 0), (0, 1), (1, 2)]                    # (session, proposer)
    nonces = [tc.nonce_bytes(inv_id, s, p, 2) for s, p in specs]
    hs = [tc.hash_g2(x) for x in nonces]
    count = len(nonces)
    sigs = np.zeros((count, n, 96), dtype=np.uint8)
    present = np.ones((count, n), dtype=bool)
    pts = {}
    for c in range(count):
        for i in range(n):
            pts[(c, i)] = tc.sign(sks.secret_key_share(i), nonces[c], hash_pt=hs[c])
    other = tc.hash_g2(b"some other nonce")
    pts[(0, n - 1)] = tc.sign(sks.secret_key_share(n - 1), b"", hash_pt=other)   # wrong message
    for (c, i), p in pts.items():
        sigs[c, i] = np.frombuffer(bls.g2_compress(p), dtype=np.uint8)
    sigs[1, 0] = 0xFF                                   # undecodable (x >= p)
    sigs[1, 0, 0] = 0x9F
    present[1, min(2, n - 1)] = False
    present[2, 1:] = False                              # starve instance 2: 1 share < t
    expect_valid = np.zeros((count, n), dtype=bool)
    for c in range(count):
        for i in range(n):
            if present[c, i] and (c, i) != (1, 0):
                expect_valid[c, i] = tc.verify_sig(pks.public_key_share(i), pts[(c, i)], nonces[c], hash_pt=hs[c])
    status = np.zeros(count, dtype=np.int32)
    sig_out = np.zeros((count, 96), dtype=np.uint8)
    master_ok = np.zeros(count, dtype=bool)
    parity = np.zeros(count, dtype=bool)
    for c in range(count):
        shares = [(i, pts[(c, i)]) for i in range(n) if expect_valid[c, i]]
        if len(shares) < t:
            status[c] = -3
            continue
        sig = tc.combine_signatures(pks, shares)
        sig_out[c] = np.frombuffer(bls.g2_compress(sig), dtype=np.uint8)
        master_ok[c] = tc.verify_sig(pks.public_key(), sig, nonces[c], hash_pt=hs[c])
        parity[c] = tc.parity(sig)
    off = np.zeros(count + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(x) for x in nonces])
    return dict(
        n=np.int64(n), t=np.int64(t),
        pk_comp=np.stack([np.frombuffer(bls.g1_compress(pks.public_key_share(i)), dtype=np.uint8) for i in range(n)]),
        master_pk=np.frombuffer(bls.g1_compress(pks.public_key()), dtype=np.uint8),
        sk=np.stack([np.frombuffer(sks.secret_key_share(i).to_bytes(32, "big"), dtype=np.uint8) for i in range(n)]),
        nonce_blob=np.frombuffer(b"".join(nonces), dtype=np.uint8), nonce_off=off,
        h=np.stack([np.frombuffer(bls.g2_compress(h), dtype=np.uint8) for h in hs]),
        sigs=sigs, present=present, expect_valid=expect_valid, expect_status=status, expect_sig=sig_out,
        expect_master_ok=master_ok, expect_parity=parity,
    )


def main():
    for n in (4, 7):
        d = make(n)
        path = os.path.join(HERE, f"coin_n{n}.npz")
        np.savez_compressed(path, **d)
        print(path, "valid", int(d["expect_valid"].sum()), "status", d["expect_status"].tolist(),
              "master_ok", d["expect_master_ok"].tolist(), "parity", d["expect_parity"].astype(int).tolist())


if __name__ == "__main__":
    main()
