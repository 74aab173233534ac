"""Pins the broadcast oracle (oracle/rs_merkle.py): reed-solomon-erasure 3.1.0's systematic
Vandermonde code, reconstruction from any k of n shards (first k present), the index-byte property
of SURVEY.md §0.7, merkle.rs proofs / validate / index, and the reference's own broadcast test
properties (tests/broadcast.rs:93-161: sizes 1..5 and beyond, equal-leaf payloads, silent-f
reconstruction)."""
import random

import numpy as np
import pytest

from oracle import rs_merkle as rm


def test_gf_tables():
    assert rm.gmul(2, 0x80) == 0x1D            # x * x^7 = x^8 = poly remainder
    for a in range(1, 256):
        assert rm.gmul(a, rm.ginv(a)) == 1
    assert rm.gexp(0, 0) == 1 and rm.gexp(0, 3) == 0 and rm.gexp(2, 8) == 0x1D


@pytest.mark.parametrize("k,m", [(2, 2), (3, 4), (5, 8), (44, 84)])
def test_systematic_and_any_k_reconstruct(k, m):
    rs = rm.ReedSolomon(k, m)
    assert [row[:k] for row in rs.matrix[:k]] == [[1 if i == j else 0 for j in range(k)] for i in range(k)]
    rnd = np.random.default_rng(k * 100 + m)
    data = np.zeros((k + m, 37), dtype=np.uint8)
    data[:k] = rnd.integers(0, 256, size=(k, 37), dtype=np.uint8)
    enc = rs.encode(data)
    assert (enc[:k] == data[:k]).all()
    for trial in range(3):
        keep = sorted(random.Random(trial).sample(range(k + m), k))
        shards = [enc[i].tobytes() if i in keep else None for i in range(k + m)]
        out = rs.reconstruct(shards)
        assert all(out[i] == enc[i].tobytes() for i in range(k + m))
    with pytest.raises(rm.TooFewShardsPresent):
        rs.reconstruct([enc[i].tobytes() if i < k - 1 else None for i in range(k + m)])


@pytest.mark.parametrize("n", [4, 7, 10, 128, 256])
def test_index_byte_property(n):
    """(0, 1, ..., k-1) encodes to (0, 1, ..., n-1): reconstructing the index-prefixed leaves
    restores the right index bytes."""
    k, m = rm.coding_counts(n)
    rs = rm.ReedSolomon(k, m)
    col = np.zeros((n, 1), dtype=np.uint8)
    col[:k, 0] = np.arange(k)
    assert (rs.encode(col)[:, 0] == np.arange(n) % 256).all()


def test_merkle_proofs_and_index():
    for count in range(1, 20):
        leaves = [bytes([i]) + b"leaf" for i in range(count)]
        tree = rm.MerkleTree(leaves)
        for i, leaf in enumerate(leaves):
            p = tree.gen_proof(leaf)
            assert rm.proof_validate(p, tree.root_hash())
            assert rm.proof_index(p, count) == i
            bad = dict(p, value=b"\xff" + leaf[1:])
            assert not rm.proof_validate(bad, tree.root_hash())
    # odd node promoted unchanged
    t3 = rm.MerkleTree([b"a", b"b", b"c"])
    assert t3.root_hash() == rm.hash_nodes(rm.hash_nodes(rm.hash_leaf(b"a"), rm.hash_leaf(b"b")), rm.hash_leaf(b"c"))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8, 13, 40])
@pytest.mark.parametrize("value", [b"Foo", b" " * 32, bytes(range(200))])
def test_broadcast_roundtrip_silent_f(n, value):
    """tests/broadcast.rs:93-161: every good node outputs the proposed value with f silent nodes."""
    f = rm.num_faulty(n)
    shards, leaves, tree = rm.send_shards(value, n)
    for i, leaf in enumerate(leaves):
        p = tree.gen_proof(leaf)
        assert rm.validate_broadcast_proof(p, i, n)
        assert not rm.validate_broadcast_proof(p, (i + 1) % n, n) or n == 1
    received = [leaves[i] if i < n - f else None for i in range(n)]   # last f silent
    assert rm.decode_from_shards(received, n, tree.root_hash()) == value
    if f and n > 3:
        assert rm.decode_from_shards(received, n, b"\0" * 32) is None
