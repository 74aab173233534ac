"""Fixtures for the HoneyBadger epoch replay.

    python tests/golden/make_replay.py      # writes tests/golden/hb_replay_{a,b,c}.npz

One node-epoch of N = 7 nodes as node ``me`` receives it: DecryptionShare messages interleaved
with the CommonSubset output, including every fault path of honey_badger.rs's decryption sub-path:

* proposer 0: W of another ciphertext          -> ShareDecryptionFailed (:371-375)
* proposer 1: U off the G1 subgroup             -> InvalidCiphertext (:359-368)
* proposer 3: U = W = identity (a valid ciphertext: e(g1, O) = e(O, H) = 1; honest shares O)
* proposer 5: not in the CommonSubset output (its shares are stored, never verified)
* sender 6: FaultyShareAdversary shares (tests/honey_badger.rs:99-106: a share of a different
  ciphertext) to every proposer, some before and some after the ciphertexts are known
* sender 5: an undecodable share and an off-subgroup share (serde rejects both: no fault)
* sender 4: the identity as its share of proposer 6 (verifies false)
* sender 1: a wrong share of proposer 2 after the ciphertexts (fault at arrival), then the right
  one (a second message of the same pair)
* sender 9: not a validator -> Err(UnknownSender)
* scenario a: messages keep coming after the batch is output (ignored: past epoch);
  scenario b: proposer 6 never gets more than f shares -> no batch;
  scenario c: a Byzantine relayer sends two messages for one (proposer, sender) pair in each
  order before the ciphertexts are known: sender 3 to proposer 4 a valid then an invalid share
  (the invalid one replaces it unverified and is removed at the ciphertext: fault, no share),
  sender 0 to proposer 4 an invalid then a valid share (the valid one replaces it: no fault).

Expected FaultLog / errors / Batch come from the message-at-a-time restatement
``oracle/honey_badger.py`` (digest variant SHA-256), plus the expected engine
status of every message (HBX_SHARE_* / HBX_CT_*) for the CPU test of the replay logic.
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import honey_badger as ohb  # noqa: E402
from oracle import threshold as tc  # noqa: E402
from oracle.chacha_rand04 import ChaChaRng04  # noqa: E402

SEED = 0x68626278
N = 7
ME = 2
FAULT_CODES = {ohb.UNVERIFIED_DECRYPTION_SHARE_SENDER: 0, ohb.INVALID_CIPHERTEXT: 1, ohb.SHARE_DECRYPTION_FAILED: 2}
ERROR_CODES = {ohb.UNKNOWN_SENDER: 0}
NO_STATUS = 255
# include/hbx.h
SHARE_INVALID, SHARE_VALID, SHARE_UNDECODABLE, SHARE_SKIPPED_CT = 0, 1, 3, 4
CT_INVALID, CT_VALID, CT_UNDECODABLE = 0, 1, 3


def off_subgroup_g1(seed: int) -> bytes:
    """Compressed encoding of a point on y^2 = x^3 + 4 that is NOT in G1."""
    x = seed
    while True:
        y = bls.fq_sqrt((x ** 3 + bls.B1) % bls.P)
        if y is not None and bls.g1_mul((x, y), bls.R) is not None:
            return bls.g1_compress((x, y))
        x += 1


def keys():
    f = (N - 1) // 3
    sks = tc.SecretKeySet.random(f, ChaChaRng04([SEED, 1]))
    return sks, sks.public_keys()


def scenario(tag: str):
    sks, pks = keys()
    f = (N - 1) // 3
    sk = [sks.secret_key_share(i) for i in range(N)]
    data_rng = ChaChaRng04([SEED, 0x10 + ord(tag)])
    r_rng = ChaChaRng04([SEED, 0x20 + ord(tag)])
    msgs = [bytes(data_rng.gen_u8() for _ in range([5, 64, 65, 130, 1, 200, 33][j])) for j in range(N)]
    cts = [tc.encrypt(pks.public_key(), msgs[j], tc.fr_rand(r_rng)) for j in range(N)]
    fake = tc.encrypt(pks.public_key(), b"X marks the spot", tc.fr_rand(r_rng))  # tests/honey_badger.rs:90
    enc = lambda c: (bls.g1_compress(c[0]), bytes(c[1]), bls.g2_compress(c[2]))  # noqa: E731
    wire = {j: enc(cts[j]) for j in range(N)}
    # proposer 0: W of ciphertext 1; proposer 1: U off the subgroup; proposer 3: identity U and W
    wire[0] = (wire[0][0], wire[0][1], wire[1][2])
    wire[1] = (off_subgroup_g1(12345), wire[1][1], wire[1][2])
    v3 = bytes(data_rng.gen_u8() for _ in range(40))
    wire[3] = (bls.g1_compress(None), v3, bls.g2_compress(None))
    acs_set = [0, 1, 2, 3, 4, 6]
    u_pt = {j: ohb.decode_ciphertext(wire[j]) for j in range(N)}

    def honest(i, j):
        dec = u_pt[j]
        u = dec[0] if dec is not None else cts[j][0]
        return bls.g1_compress(bls.g1_mul(u, sk[i]))

    shares = []  # (sender, proposer, bytes)
    for j in range(N):
        for i in range(N):
            if i == ME:
                continue
            if i == 6:
                shares.append((i, j, bls.g1_compress(tc.decrypt_share(sk[i], fake))))
            elif i == 5 and j == 2:
                bad = bytearray(48)
                bad[0] = 0x9F
                bad[1:] = b"\xff" * 47
                shares.append((i, j, bytes(bad)))
            elif i == 5 and j == 4:
                shares.append((i, j, off_subgroup_g1(999)))
            elif i == 4 and j == 6:
                shares.append((i, j, bls.g1_compress(None)))
            else:
                shares.append((i, j, honest(i, j)))
    rnd = random.Random(SEED + ord(tag))
    rnd.shuffle(shares)
    if tag == "b":
        # starve proposer 6: only f - 1 honest shares besides ours (<= f shares in total)
        keep = 0
        out = []
        for (i, j, b) in shares:
            if j == 6 and i != 6:
                if keep >= f - 1:
                    continue
                keep += 1
            out.append((i, j, b))
        shares = out
    if tag == "c":
        # both pairs' messages go first (before the ciphertexts), in the two orders
        shares = [s for s in shares if (s[0], s[1]) not in ((3, 4), (0, 4))]
        bad34 = bls.g1_compress(bls.g1_mul(cts[4][0], sk[3] + 7))
        bad04 = bls.g1_compress(bls.g1_mul(cts[4][0], sk[0] + 5))
        shares = [(3, 4, honest(3, 4)), (0, 4, bad04), (3, 4, bad34), (0, 4, honest(0, 4))] + shares
    cut = 4 if tag == "a" else len(shares) // 3  # a: most shares arrive after the ciphertexts
    events = [("share", i, j, b) for (i, j, b) in shares[:cut]]
    events.append(("acs", {j: wire[j] for j in acs_set}))
    late = [("share", i, j, b) for (i, j, b) in shares[cut:]]
    # sender 1 first sends a wrong share of proposer 2 (after the ciphertexts), then the right one
    wrong = bls.g1_compress(bls.g1_mul(cts[2][0], sk[1] + 1))
    late.insert(1, ("share", 1, 2, wrong))
    late.insert(2, ("share", 9, 2, honest(3, 2)))  # unknown sender
    events += late
    if tag == "a":
        events.append(("share", 6, 4, bls.g1_compress(tc.decrypt_share(sk[6], fake))))
    node = ohb.EpochNode(N, ME, pks, sk[ME]).run(events)

    # expected engine statuses (what hbx_prepare_ciphertexts / hbx_verify_dec_shares report)
    ct_status = {}
    hashes = {}
    for j in acs_set:
        dec = ohb.decode_ciphertext(wire[j])
        if dec is None:
            ct_status[j] = CT_UNDECODABLE
            continue
        hashes[j] = tc.hash_g1_g2(dec[0], dec[1])
        ct_status[j] = CT_VALID if tc.ciphertext_verify(dec, hash_pt=hashes[j]) else CT_INVALID
    pk_share = [pks.public_key_share(i) for i in range(N)]
    ev_status = []
    for ev in events:
        st = NO_STATUS
        if ev[0] == "share" and ev[1] < N and ev[2] in ct_status:
            dec = ohb.decode_share(ev[3])
            if dec is None:
                st = SHARE_UNDECODABLE
            elif ct_status[ev[2]] != CT_VALID:
                st = SHARE_SKIPPED_CT
            else:
                ct = ohb.decode_ciphertext(wire[ev[2]])
                ok = tc.verify_decryption_share(pk_share[ev[1]], dec[1], ct, hash_pt=hashes[ev[2]])
                st = SHARE_VALID if ok else SHARE_INVALID
        ev_status.append(st)

    acs_ids = np.array(acs_set, dtype=np.int64)
    voff = np.zeros(len(acs_set) + 1, dtype=np.uint64)
    voff[1:] = np.cumsum([len(wire[j][1]) for j in acs_set])
    shares_ev = [ev for ev in events]
    kinds = np.array([0 if ev[0] == "share" else 1 for ev in shares_ev], dtype=np.int8)
    batch = node.batch or {}
    bprops = np.array(sorted(batch), dtype=np.int64)
    boff = np.zeros(len(bprops) + 1, dtype=np.uint64)
    boff[1:] = np.cumsum([len(batch[j]) for j in sorted(batch)])
    return dict(
        n=np.int64(N), me=np.int64(ME), t=np.int64(f + 1),
        pk_comp=np.stack([np.frombuffer(bls.g1_compress(q), dtype=np.uint8) for q in pk_share]),
        sk_me=np.frombuffer(sk[ME].to_bytes(32, "big"), dtype=np.uint8),
        ev_kind=kinds,
        ev_sender=np.array([ev[1] if ev[0] == "share" else -1 for ev in shares_ev], dtype=np.int64),
        ev_proposer=np.array([ev[2] if ev[0] == "share" else -1 for ev in shares_ev], dtype=np.int64),
        ev_share=np.stack([np.frombuffer(ev[3], dtype=np.uint8) if ev[0] == "share" else np.zeros(48, np.uint8)
                           for ev in shares_ev]),
        acs_proposers=acs_ids,
        acs_u=np.stack([np.frombuffer(wire[j][0], dtype=np.uint8) for j in acs_set]),
        acs_w=np.stack([np.frombuffer(wire[j][2], dtype=np.uint8) for j in acs_set]),
        acs_v_blob=np.frombuffer(b"".join(wire[j][1] for j in acs_set), dtype=np.uint8),
        acs_v_off=voff,
        expect_fault_node=np.array([a for a, _ in node.faults], dtype=np.int64),
        expect_fault_kind=np.array([FAULT_CODES[b] for _, b in node.faults], dtype=np.int64),
        expect_error_node=np.array([a for a, _ in node.errors], dtype=np.int64),
        expect_error_kind=np.array([ERROR_CODES[b] for _, b in node.errors], dtype=np.int64),
        expect_batch=np.bool_(node.batch is not None),
        expect_batch_proposers=bprops,
        expect_batch_blob=np.frombuffer(b"".join(batch[j] for j in sorted(batch)) or b"", dtype=np.uint8),
        expect_batch_off=boff,
        expect_ev_status=np.array(ev_status, dtype=np.uint8),
        expect_ct_status=np.array([ct_status[j] for j in acs_set], dtype=np.uint8),
    )


def load_events(d):
    """Rebuild the event list of a fixture (used by the tests)."""
    acs = {}
    off = d["acs_v_off"]
    for q, j in enumerate(d["acs_proposers"]):
        acs[int(j)] = (d["acs_u"][q].tobytes(), d["acs_v_blob"][int(off[q]):int(off[q + 1])].tobytes(),
                       d["acs_w"][q].tobytes())
    events = []
    for k in range(len(d["ev_kind"])):
        if d["ev_kind"][k] == 0:
            events.append(("share", int(d["ev_sender"][k]), int(d["ev_proposer"][k]), d["ev_share"][k].tobytes()))
        else:
            events.append(("acs", acs))
    return events


def main():
    for tag in ("a", "b", "c"):
        d = scenario(tag)
        path = os.path.join(HERE, f"hb_replay_{tag}.npz")
        np.savez_compressed(path, **d)
        print(path, "faults", list(zip(d["expect_fault_node"].tolist(), d["expect_fault_kind"].tolist())),
              "errors", d["expect_error_node"].tolist(), "batch", bool(d["expect_batch"]),
              d["expect_batch_proposers"].tolist())


if __name__ == "__main__":
    main()
