"""Generate the committed golden fixtures for the threshold-decryption path.

    python tests/golden/make_golden.py            # writes tests/golden/hb_epoch_n{4,7}.npz

Inputs are seeded (SURVEY.md §8(d) seeds 0x68626278_0000000{1..4}); expected outputs come from
the CPU restatement in ``oracle/`` (canonical pairing, SHA-256 digest variant).  Each fixture is
one HoneyBadger node-epoch as stack A of SURVEY.md §3 sees it:

* N nodes, f = (N-1)//3, t = f + 1 (messaging.rs:258, honey_badger.rs:328);
* one ciphertext per proposer j with |V_j| drawn from {1, 64, 65, 200} (covers the
  hash_g1_g2 "> 64 bytes => digest" branch); ciphertext 0 gets the W of ciphertext 1
  (Ciphertext::verify fails -> ShareDecryptionFailed, honey_badger.rs:371-373);
* share matrix S[j][i] = sk_i * U_j, with corruptions built like the reference's
  FaultyShareAdversary (tests/honey_badger.rs:99-106: a valid share of a DIFFERENT ciphertext),
  a few absent shares, one proposer left with fewer than t valid shares (NotEnoughShares) and
  one non-decodable share encoding;
* expected: ct validity, per-share validity, per-proposer status and plaintext.
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

SEED = 0x68626278
V_LENS = [1, 64, 65, 200]


def make_epoch(n: int):
    f = (n - 1) // 3
    t = f + 1
    key_rng = ChaChaRng04([SEED, 1])
    data_rng = ChaChaRng04([SEED, 2])
    r_rng = ChaChaRng04([SEED, 3])
    sks = tc.SecretKeySet.random(f, key_rng)
    pks = sks.public_keys()
    pk_shares = [pks.public_key_share(i) for i in range(n)]
    sk_shares = [sks.secret_key_share(i) for i in range(n)]
    p = n
    cts = []
    msgs = []
    for j in range(p):
        ln = V_LENS[j % len(V_LENS)]
        msg = bytes(data_rng.gen_u8() for _ in range(ln))
        r = tc.fr_rand(r_rng)
        cts.append(tc.encrypt(pks.public_key(), msg, r))
        msgs.append(msg)
    hashes = [tc.hash_g1_g2(u, v) for (u, v, _) in cts]
    # ciphertext 0 carries ciphertext 1's W -> invalid
    bad_cts = list(cts)
    if p > 1:
        bad_cts[0] = (cts[0][0], cts[0][1], cts[1][2])
    ct_valid = [tc.ciphertext_verify(bad_cts[j], hash_pt=hashes[j]) for j in range(p)]

    shares = np.zeros((p, n, 48), dtype=np.uint8)
    present = np.ones((p, n), dtype=bool)
    share_pts = {}
    for j in range(p):
        for i in range(n):
            s = tc.decrypt_share(sk_shares[i], bad_cts[j])
            share_pts[(j, i)] = s
    # FaultyShareAdversary-style corruptions: share of a different ciphertext
    corrupt = [(1 % p, n - 1), (2 % p, 0)]
    for (j, i) in corrupt:
        share_pts[(j, i)] = tc.decrypt_share(sk_shares[i], bad_cts[(j + 1) % p])
    # absent shares
    absent = [(1 % p, 0)]
    for (j, i) in absent:
        present[j, i] = False
    # starve the last proposer: only t-1 valid shares (rest absent)
    starve = p - 1
    for i in range(t - 1, n):
        present[starve, i] = False
    for (j, i), pt in share_pts.items():
        shares[j, i] = np.frombuffer(bls.g1_compress(pt), dtype=np.uint8)
    # one undecodable encoding (x >= p with the compression flag)
    bad_enc = (min(3, p - 1), 1 % n)
    shares[bad_enc[0], bad_enc[1]] = 0xFF
    shares[bad_enc[0], bad_enc[1], 0] = 0x9F

    expect_valid = np.zeros((p, n), dtype=bool)
    for j in range(p):
        if not ct_valid[j]:
            continue
        for i in range(n):
            if not present[j, i] or (j, i) == bad_enc:
                continue
            expect_valid[j, i] = tc.verify_decryption_share(pk_shares[i], share_pts[(j, i)], bad_cts[j],
                                                            hash_pt=hashes[j])
    status = np.zeros(p, dtype=np.int32)
    plains = []
    for j in range(p):
        if not ct_valid[j]:
            status[j] = -7
            plains.append(b"")
            continue
        idx = [i for i in range(n) if expect_valid[j, i]]
        if len(idx) < t:
            status[j] = -3
            plains.append(b"")
            continue
        pt = tc.decrypt(pks, [(i, share_pts[(j, i)]) for i in idx], bad_cts[j])
        assert pt == msgs[j]
        plains.append(pt)

    v_off = np.zeros(p + 1, dtype=np.uint64)
    v_off[1:] = np.cumsum([len(c[1]) for c in bad_cts])
    plain_blob = np.zeros(int(v_off[-1]), dtype=np.uint8)
    for j in range(p):
        if status[j] == 0:
            plain_blob[int(v_off[j]):int(v_off[j + 1])] = np.frombuffer(plains[j], dtype=np.uint8)

    # Own-share mode (hbx_set_own_share): node `me` uses its own share sk_me * U_j
    # (decrypt_share_no_verify, honey_badger.rs:403) whatever its row of the input holds; that
    # honest share verifies exactly when the ciphertext does.
    me = n - 2
    own_pts = dict(share_pts)
    for j in range(p):
        own_pts[(j, me)] = tc.decrypt_share(sk_shares[me], bad_cts[j])
    expect_valid_own = expect_valid.copy()
    for j in range(p):
        expect_valid_own[j, me] = bool(ct_valid[j])
    status_own = np.zeros(p, dtype=np.int32)
    plain_blob_own = np.zeros(int(v_off[-1]), dtype=np.uint8)
    for j in range(p):
        if not ct_valid[j]:
            status_own[j] = -7
            continue
        idx = [i for i in range(n) if expect_valid_own[j, i]]
        if len(idx) < t:
            status_own[j] = -3
            continue
        pt = tc.decrypt(pks, [(i, own_pts[(j, i)]) for i in idx], bad_cts[j])
        assert pt == msgs[j]
        plain_blob_own[int(v_off[j]):int(v_off[j + 1])] = np.frombuffer(pt, dtype=np.uint8)
    return dict(
        n=np.int64(n), t=np.int64(t),
        pk_comp=np.stack([np.frombuffer(bls.g1_compress(q), dtype=np.uint8) for q in pk_shares]),
        master_pk=np.frombuffer(bls.g1_compress(pks.public_key()), dtype=np.uint8),
        u=np.stack([np.frombuffer(bls.g1_compress(c[0]), dtype=np.uint8) for c in bad_cts]),
        w=np.stack([np.frombuffer(bls.g2_compress(c[2]), dtype=np.uint8) for c in bad_cts]),
        h=np.stack([np.frombuffer(bls.g2_compress(h), dtype=np.uint8) for h in hashes]),
        v_blob=np.frombuffer(b"".join(c[1] for c in bad_cts), dtype=np.uint8),
        v_off=v_off,
        shares=shares, present=present,
        expect_ct_valid=np.array(ct_valid, dtype=bool),
        expect_valid=expect_valid,
        expect_status=status,
        expect_plain_blob=plain_blob,
        own_me=np.int64(me),
        own_sk=np.frombuffer(sk_shares[me].to_bytes(32, "big"), dtype=np.uint8),
        expect_valid_own=expect_valid_own,
        expect_status_own=status_own,
        expect_plain_blob_own=plain_blob_own,
    )


def main():
    for n in (4, 7):
        d = make_epoch(n)
        path = os.path.join(HERE, f"hb_epoch_n{n}.npz")
        np.savez_compressed(path, **d)
        print(path, "ct_valid", d["expect_ct_valid"].astype(int).tolist(), "status", d["expect_status"].tolist(),
              "valid shares", int(d["expect_valid"].sum()))


if __name__ == "__main__":
    main()
