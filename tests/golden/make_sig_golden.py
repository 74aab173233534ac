"""Generate the committed PublicKey::verify fixture with the oracle.

    python tests/golden/make_sig_golden.py      # sigs_n16.npz

Dynamic HoneyBadger checks each signed vote with `pk.verify(&signed_vote.sig, bincode(vote))`
(src/dynamic_honey_badger/votes.rs:151-156) and each key-generation message with
`pk.verify(&sig, bincode(kg_msg))` (src/dynamic_honey_badger/dynamic_honey_badger.rs:395-410):
threshold_crypto PublicKey::verify(sig, msg) = e(pk, hash_g2(msg)) == e(g1, sig).  Every item
carries its own key, message and signature.  The messages here are byte strings of the lengths
bincode produces for those structs and beyond (0..300 B; both sides of the 64-byte boundary that
hash_g1_g2 has but hash_g2 does not), since the batch API takes the serialised bytes.
Cases: valid signatures; a signature over another message; a signature by another key; a
signature plus a point of the cofactor part (on the curve, not in G2); undecodable signature
bytes; a key off the G1 subgroup; an undecodable key; identity key with identity signature
(e(O, H) = 1 = e(g1, O): true); identity key with a real signature (false).
Expected: HBX_SHARE_VALID (1) / HBX_SHARE_INVALID (0) / HBX_SHARE_UNDECODABLE (3) per item.
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

sys.path.insert(0, HERE)
from make_coin_golden import cofactor_point  # noqa: E402
from make_golden import off_subgroup_g1  # noqa: E402

INVALID, VALID, UNDECODABLE = 0, 1, 3
IDENTITY_G1 = bytes([0xC0]) + bytes(47)
IDENTITY_G2 = bytes([0xC0]) + bytes(95)


def make(count: int = 16, digest: str = "sha256"):
    rng = ChaChaRng04([0x68626278, 0x51])
    sks = [tc.fr_rand(rng) for _ in range(count)]
    mrng = np.random.default_rng(0x5167)
    lens = [0, 1, 31, 63, 64, 65, 100, 300] + [int(mrng.integers(0, 300)) for _ in range(count - 8)]
    msgs = [mrng.integers(0, 256, size=ln, dtype=np.uint8).tobytes() for ln in lens]
    pk = [bls.g1_compress(bls.g1_mul(bls.G1_GEN, sk)) for sk in sks]
    sig = [bls.g2_compress(tc.sign(sk, m, digest)) for sk, m in zip(sks, msgs)]
    expect = [VALID] * count
    # faults
    sig[6] = bls.g2_compress(tc.sign(sks[6], msgs[6] + b"x", digest)); expect[6] = INVALID
    sig[7] = bls.g2_compress(tc.sign(sks[0], msgs[7], digest)); expect[7] = INVALID
    sig[8] = bls.g2_compress(bls.g2_add(tc.sign(sks[8], msgs[8], digest), cofactor_point())); expect[8] = UNDECODABLE
    bad = bytearray(sig[9]); bad[0] &= 0x1F; sig[9] = bytes(bad); expect[9] = UNDECODABLE   # compression flag cleared
    pk[10] = bls.g1_compress(off_subgroup_g1(4242)); expect[10] = UNDECODABLE
    bad = bytearray(pk[11]); bad[1:] = b"\xff" * 47; bad[0] = 0x9F; pk[11] = bytes(bad); expect[11] = UNDECODABLE
    pk[12] = IDENTITY_G1; sig[12] = IDENTITY_G2; expect[12] = VALID
    pk[13] = IDENTITY_G1; expect[13] = INVALID
    # the oracle's verdict on every decodable item agrees with the table above
    for i in range(count):
        if expect[i] == UNDECODABLE:  # pairing 0.14 into_affine rejects the key or the signature
            bad = 0
            for dec, b in ((bls.g1_decompress, pk[i]), (bls.g2_decompress, sig[i])):
                try:
                    dec(b)
                except ValueError:
                    bad += 1
            assert bad, i
            continue
        P = bls.g1_decompress(pk[i])
        S = bls.g2_decompress(sig[i])
        assert tc.verify_sig(P, S, msgs[i], digest) == (expect[i] == VALID), i
    off = np.zeros(count + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return dict(variant=np.array(f"digest={digest}"), count=np.int64(count),
                pk=np.frombuffer(b"".join(pk), dtype=np.uint8).reshape(count, 48),
                sig=np.frombuffer(b"".join(sig), dtype=np.uint8).reshape(count, 96),
                msg_blob=np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8), msg_off=off,
                expect=np.array(expect, dtype=np.uint8),
                h=np.stack([np.frombuffer(bls.g2_compress(tc.hash_g2(m, digest)), dtype=np.uint8) for m in msgs]))


def main():
    d = make()
    np.savez_compressed(os.path.join(HERE, "sigs_n16.npz"), **d)
    print("sigs_n16.npz", d["expect"].tolist())


if __name__ == "__main__":
    main()
