"""Fixture for BASELINE config C5: one Broadcast instance of a 1 MiB proposal at
N=128 (f=42, RS(44, 84), shard length 23,832 B), made by the oracle (oracle/rs_merkle.py, which
restates broadcast.rs:332-404 / :660-707, reed-solomon-erasure 3.1.0 and the merkle fork).

The payload is regenerated from its seed (numpy PCG64); the fixture holds digests of the outputs
(per-shard SHA-256, every tree node for both Merkle variants), the proofs of a few leaves in
hbx_merkle_validate_d's flat format, and the decode expectation with the last f shards missing.

    python tests/golden/make_c5_golden.py      # writes tests/golden/c5_broadcast.npz
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import rs_merkle as rm  # noqa: E402

SEED = 0x68626278_0000C5C5
N = 128
PLEN = 1 << 20
PROOF_LEAVES = [0, 1, 43, 44, 85, 86, 127]


def payload():
    return np.random.default_rng(SEED).integers(0, 256, size=PLEN, dtype=np.uint8).tobytes()


def flat_proofs(tree, leaves):
    P = len(PROOF_LEAVES)
    nodes = np.zeros((P, 17, 32), dtype=np.uint8)
    sibs = np.zeros((P, 16, 32), dtype=np.uint8)
    sides = np.zeros(P, dtype=np.int32)
    depth = np.zeros(P, dtype=np.int32)
    for j, leaf in enumerate(PROOF_LEAVES):
        p = tree.gen_proof(leaves[leaf])
        lem = p["lemma"]
        depth[j] = len(lem) - 1
        for lv, (h, sib) in enumerate(lem):
            nodes[j, lv] = np.frombuffer(h, dtype=np.uint8)
            if sib is not None:
                sibs[j, lv] = np.frombuffer(sib[1], dtype=np.uint8)
                if sib[0] == "L":
                    sides[j] |= 1 << lv
        assert rm.validate_broadcast_proof(p, leaf, N)
    return nodes, sibs, sides, depth


def main():
    value = payload()
    k, m = rm.coding_counts(N)
    f = rm.num_faulty(N)
    shards, leaves, tree = rm.send_shards(value, N)
    L = shards.shape[1]
    assert (k, m, L) == (44, 84, 23832)
    out = {
        "seed": np.uint64(SEED), "n": np.int32(N), "plen": np.int64(PLEN), "k": np.int32(k), "m": np.int32(m),
        "shard_len": np.int32(L),
        "payload_sha": np.frombuffer(hashlib.sha256(value).digest(), dtype=np.uint8),
        "shard_sha": np.stack([np.frombuffer(hashlib.sha256(shards[i].tobytes()).digest(), dtype=np.uint8)
                               for i in range(N)]),
        "proof_leaves": np.asarray(PROOF_LEAVES, dtype=np.uint32),
    }
    for variant in ("sha256", "sha3"):
        t = tree if variant == "sha256" else rm.MerkleTree(leaves, variant)
        flat = b"".join(h for lvl in t.levels for h in lvl)
        out[f"root_{variant}"] = np.frombuffer(t.root_hash(), dtype=np.uint8)
        out[f"nodes_sha_{variant}"] = np.frombuffer(hashlib.sha256(flat).digest(), dtype=np.uint8)
        out[f"node_count_{variant}"] = np.int32(len(flat) // 32)
        if variant == "sha256":
            nodes, sibs, sides, depth = flat_proofs(t, leaves)
            out.update(proof_nodes=nodes, proof_sibs=sibs, proof_sides=sides, proof_depth=depth)
    # decode with the last f shards missing (the C5 decode case) must give the payload back
    vals = [leaves[j] if j < N - f else None for j in range(N)]
    assert rm.decode_from_shards(vals, N, tree.root_hash()) == value
    np.savez_compressed(os.path.join(HERE, "c5_broadcast.npz"), **out)
    print("wrote c5_broadcast.npz", {kk: v.shape for kk, v in out.items() if hasattr(v, "shape")})


if __name__ == "__main__":
    main()
