"""The Broadcast path through the HOST-pointer entry points (the boundary a thin
Rust FFI drives from Vec<u8>): hbx_rs_encode, hbx_rs_reconstruct, hbx_merkle_build / _roots /
_proofs, hbx_merkle_validate and hbx_broadcast_decode[_leaves] called with plain numpy buffers --
no torch tensor anywhere -- against the committed C5 fixture (tests/golden/c5_broadcast.npz: a
1 MiB proposal at N = 128, RS(44, 84)) and the oracle (oracle/rs_merkle.py), byte for byte.

The sequence is the reference's: send_shards (broadcast.rs:341-401: frame, Coding::encode,
MerkleTree::from_vec, one gen_proof per node), validate_proof on every Value / Echo (:555-575) and
decode_from_shards with the last f shards missing (:660-707)."""
import hashlib
import os

import numpy as np
import pytest

from oracle import rs_merkle as rm

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _merkle(ctx, variant):
    from hbbft_amd.hbx import MERKLE_SHA3, MERKLE_SHA256

    ctx.set_merkle_digest(MERKLE_SHA3 if variant == "sha3" else MERKLE_SHA256)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sha256", "sha3"])
def test_c5_fixture_host_api(hbx_ctx, variant):
    g = np.load(os.path.join(GOLDEN, "c5_broadcast.npz"))
    n, k, m, L, plen = int(g["n"]), int(g["k"]), int(g["m"]), int(g["shard_len"]), int(g["plen"])
    value = np.random.default_rng(int(g["seed"])).integers(0, 256, size=plen, dtype=np.uint8).tobytes()
    assert hashlib.sha256(value).digest() == g["payload_sha"].tobytes()
    _merkle(hbx_ctx, variant)
    # send_shards: frame, then Coding::encode on the host buffer (broadcast.rs:341-367)
    framed = int(plen).to_bytes(4, "big") + value
    shards = np.zeros((1, n, L), dtype=np.uint8)
    shards.reshape(-1)[: len(framed)] = np.frombuffer(framed, dtype=np.uint8)
    shards[0, k:] = 0x5A  # parity rows are outputs: whatever they held is overwritten
    hbx_ctx.rs_encode(shards, k, m)
    got = np.stack([np.frombuffer(hashlib.sha256(shards[0, i].tobytes()).digest(), dtype=np.uint8) for i in range(n)])
    np.testing.assert_array_equal(got, g["shard_sha"])
    # MerkleTree::from_vec (broadcast.rs:381): the whole tree and the root
    nodes, roots = hbx_ctx.merkle_build(shards)
    assert roots[0].tobytes() == g[f"root_{variant}"].tobytes()
    assert nodes.shape[1] == int(g[f"node_count_{variant}"])
    assert hashlib.sha256(nodes.tobytes()).digest() == g[f"nodes_sha_{variant}"].tobytes()
    np.testing.assert_array_equal(hbx_ctx.merkle_roots(shards), roots)
    # one proof per node (gen_proof, broadcast.rs:389-401), validated as Value / Echo messages
    req = np.array([(0, j) for j in range(n)], dtype=np.uint32)
    nh, sh, sides, depth, proot = hbx_ctx.merkle_proofs(nodes, n, req)
    if variant == "sha256":
        fl = g["proof_leaves"].astype(np.int64)
        np.testing.assert_array_equal(depth[fl], g["proof_depth"])
        np.testing.assert_array_equal(sides[fl], g["proof_sides"])
        np.testing.assert_array_equal(nh[fl], g["proof_nodes"])
        np.testing.assert_array_equal(sh[fl], g["proof_sibs"])
    values = np.concatenate([np.arange(n, dtype=np.uint8)[:, None], shards[0]], axis=1)
    senders = np.arange(n, dtype=np.uint32)
    senders[5] = 6  # Echo from the wrong node (node_index(sender) != value[0])
    bad = values.copy()
    bad[9, 100] ^= 1  # a corrupted byte
    valid = hbx_ctx.merkle_validate(np.concatenate([values, bad[9:10]]), np.concatenate([nh, nh[9:10]]),
                                    np.concatenate([sh, sh[9:10]]), np.concatenate([sides, sides[9:10]]),
                                    np.concatenate([depth, depth[9:10]]), np.concatenate([proot, proot[9:10]]),
                                    np.concatenate([senders, senders[9:10]]), n)
    want = np.ones(n + 1, dtype=np.uint8)
    want[5] = 0
    want[n] = 0
    np.testing.assert_array_equal(valid, want)
    # decode_from_shards with the last f shards missing, then from the Echo proofs' leaf digests
    f = (n - 1) // 3
    present = np.ones((1, n), dtype=np.uint8)
    present[0, n - f:] = 0
    for leaves in (False, True):
        work = shards.copy()
        work[present == 0] = 0xA5
        lh = nh[np.arange(n), depth][None] if leaves else None  # the last lemma node = leaf digest
        out, out_len, st = hbx_ctx.broadcast_decode(work, present, roots, k, m, leaf_hash=lh)
        assert int(st[0]) == 0 and int(out_len[0]) == plen
        assert hashlib.sha256(out[0, :plen].tobytes()).digest() == g["payload_sha"].tobytes()
        np.testing.assert_array_equal(work, shards)  # the reconstructed rows, in place
    # a wrong root: ROOT_MISMATCH
    work = shards.copy()
    wrong = roots.copy()
    wrong[0, 0] ^= 1
    _, _, st = hbx_ctx.broadcast_decode(work, present, wrong, k, m)
    assert int(st[0]) == -10


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,L", [(2, 2, 9), (3, 4, 37), (44, 84, 1000), (86, 170, 2052)])
def test_rs_host_api_matches_oracle(hbx_ctx, k, m, L):
    """hbx_rs_encode / hbx_rs_reconstruct on numpy buffers against reed-solomon-erasure 3.1.0's
    restatement, incl. too few shards (TooFewShardsPresent -> HBX_E_TOO_FEW_SHARDS)."""
    n = k + m
    rs = rm.ReedSolomon(k, m)
    rng = np.random.default_rng(n * 31 + L)
    inst = 4
    shards = np.zeros((inst, n, L), dtype=np.uint8)
    shards[:, :k] = rng.integers(0, 256, size=(inst, k, L), dtype=np.uint8)
    hbx_ctx.rs_encode(shards, k, m)
    for i in range(inst):
        np.testing.assert_array_equal(shards[i], rs.encode(shards[i].copy()))
    present = np.ones((inst, n), dtype=np.uint8)
    for i, miss in enumerate([0, m, 1, m + 1]):
        present[i, rng.permutation(n)[:miss]] = 0
    work = shards.copy()
    work[present == 0] = 0
    st = hbx_ctx.rs_reconstruct(work, present, k, m)
    for i in range(inst):
        if present[i].sum() < k:
            assert st[i] == -9
        else:
            assert st[i] == 0
            np.testing.assert_array_equal(work[i], shards[i])


@pytest.mark.gpu
def test_host_api_rejects_bad_requests(hbx_ctx):
    """Argument checks of the host forms: a proof request outside the instances given, and a
    shard count that is not k + m."""
    from hbbft_amd.hbx import HbxError

    shards = np.zeros((1, 4, 8), dtype=np.uint8)
    nodes, _ = hbx_ctx.merkle_build(shards)
    with pytest.raises(HbxError):
        hbx_ctx.merkle_proofs(nodes, 4, np.array([[1, 0]], dtype=np.uint32))
    with pytest.raises(ValueError):
        hbx_ctx.broadcast_decode(shards, np.ones((1, 4), np.uint8), np.zeros((1, 32), np.uint8), 2, 3)
