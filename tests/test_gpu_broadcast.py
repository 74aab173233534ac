"""GPU parity for the Broadcast byte path against the
oracle (oracle/rs_merkle.py): RS parity bytes, reconstructed shards, Merkle roots, proof-validation
bits and decoded values must be identical.  Cases follow the reference's tests/broadcast.rs
(sizes 1..5 and larger, payloads b"Foo" and 32 spaces, f silent nodes) plus erasure patterns with
too few shards, corrupted proofs and a wrong root."""
import random

import numpy as np
import pytest

from oracle import rs_merkle as rm

torch = pytest.importorskip("torch")

HBX_E_TOO_FEW_SHARDS = -9
HBX_E_ROOT_MISMATCH = -10


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,L,inst", [(2, 2, 5, 3), (3, 4, 37, 2), (5, 8, 64, 4), (44, 84, 1000, 2), (86, 170, 33, 1),
                                          (1, 1, 4, 2), (2, 3, 8, 3), (86, 170, 516, 1), (44, 84, 23832, 2),
                                          (128, 128, 2052, 1), (3, 250, 4100, 1),
                                          # input-triple kernel: k % 3 = 1 and 0 with several triples, a
                                          # ragged last wave, more outputs than one tile
                                          (7, 9, 64, 2), (9, 12, 1024, 2), (43, 86, 4100, 1), (42, 100, 2052, 2)])
def test_rs_encode(hbx_ctx, k, m, L, inst):
    rng = np.random.default_rng(k * 1000 + L)
    data = np.zeros((inst, k + m, L), dtype=np.uint8)
    data[:, :k] = rng.integers(0, 256, size=(inst, k, L), dtype=np.uint8)
    d = dev(data)
    hbx_ctx.rs_encode_d(d, k, m)
    torch.cuda.synchronize()
    rs = rm.ReedSolomon(k, m)
    out = d.cpu().numpy()
    for i in range(inst):
        np.testing.assert_array_equal(out[i], rs.encode(data[i]))


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,L", [(2, 2, 9), (3, 4, 37), (44, 84, 257), (2, 2, 12), (44, 84, 1000), (44, 84, 23832),
                                   (86, 170, 2052), (43, 86, 1024), (9, 12, 64)])
def test_rs_reconstruct(hbx_ctx, k, m, L):
    n = k + m
    rs = rm.ReedSolomon(k, m)
    rng = np.random.default_rng(n + L)
    inst = 6
    full = np.zeros((inst, n, L), dtype=np.uint8)
    present = np.ones((inst, n), dtype=np.uint8)
    for i in range(inst):
        buf = np.zeros((n, L), dtype=np.uint8)
        buf[:k] = rng.integers(0, 256, size=(k, L), dtype=np.uint8)
        full[i] = rs.encode(buf)
        r = random.Random(i)
        nmiss = [0, m, m // 2, 1, m + 1, n][i]            # all present / max erasures / ... / too few
        for j in r.sample(range(n), min(nmiss, n)):
            present[i, j] = 0
    damaged = full.copy()
    damaged[present == 0] = 0xA5
    d = dev(damaged)
    st = torch.zeros(inst, dtype=torch.int32, device="cuda")
    hbx_ctx.rs_reconstruct_d(d, dev(present), st, k, m)
    torch.cuda.synchronize()
    out, st = d.cpu().numpy(), st.cpu().numpy()
    for i in range(inst):
        shards = [full[i, j].tobytes() if present[i, j] else None for j in range(n)]
        try:
            want = rs.reconstruct(shards)
        except rm.TooFewShardsPresent:
            assert st[i] == HBX_E_TOO_FEW_SHARDS
            continue
        assert st[i] == 0
        assert [out[i, j].tobytes() for j in range(n)] == want


@pytest.mark.gpu
@pytest.mark.parametrize("n,L", [(1, 3), (2, 7), (3, 1), (4, 5), (7, 64), (10, 65), (128, 300), (256, 4)])
def test_merkle_roots(hbx_ctx, n, L):
    rng = np.random.default_rng(n * 7 + L)
    inst = 3
    shards = rng.integers(0, 256, size=(inst, n, L), dtype=np.uint8)
    roots = torch.zeros((inst, 32), dtype=torch.uint8, device="cuda")
    hbx_ctx.merkle_roots_d(dev(shards), roots)
    torch.cuda.synchronize()
    for i in range(inst):
        leaves = [bytes([j & 0xFF]) + shards[i, j].tobytes() for j in range(n)]
        assert roots[i].cpu().numpy().tobytes() == rm.MerkleTree(leaves).root_hash()


def flatten(proofs, senders):
    P = len(proofs)
    vlen = len(proofs[0]["value"])
    vals = np.zeros((P, vlen), dtype=np.uint8)
    nodes = np.zeros((P, 17, 32), dtype=np.uint8)
    sibs = np.zeros((P, 16, 32), dtype=np.uint8)
    sides = np.zeros(P, dtype=np.uint32)
    depth = np.zeros(P, dtype=np.uint32)
    roots = np.zeros((P, 32), dtype=np.uint8)
    for j, p in enumerate(proofs):
        vals[j] = np.frombuffer(p["value"], dtype=np.uint8)
        lem = p["lemma"]
        depth[j] = len(lem) - 1
        for lv, (h, sib) in enumerate(lem):
            nodes[j, lv] = np.frombuffer(h, dtype=np.uint8)
            if sib is not None:
                sibs[j, lv] = np.frombuffer(sib[1], dtype=np.uint8)
                if sib[0] == "L":
                    sides[j] |= 1 << lv
        roots[j] = np.frombuffer(p["root_hash"], dtype=np.uint8)
    return vals, nodes, sibs, sides, depth, roots, np.asarray(senders, dtype=np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sha256", "sha3"])
@pytest.mark.parametrize("n,size", [(4, 768), (7, 768), (13, 768), (128, 768), (13, 200_003), (128, 1_048_576)])
def test_merkle_validate(hbx_ctx, n, size, variant):
    """validate_proof over a batch; values longer than 256 B take the leaf-kernel path (their
    digests hashed first by k_merkle_leaves_sha256 / _sha3), shorter ones the one-lane path."""
    _set_merkle(hbx_ctx, variant)
    value = (bytes(range(256)) * (size // 256 + 1))[:size]
    _, leaves, tree = rm.send_shards(value, n, variant)
    proofs, senders = [], []
    for i, leaf in enumerate(leaves):
        p = tree.gen_proof(leaf)
        proofs.append(p)
        senders.append(i)
        if i % 3 == 0:                       # wrong sender (node_index check)
            proofs.append(p)
            senders.append((i + 1) % n)
        if i % 4 == 1:                       # corrupted value byte (last, then middle)
            proofs.append(dict(p, value=p["value"][:-1] + bytes([p["value"][-1] ^ 1])))
            senders.append(i)
            mid = len(p["value"]) // 2
            proofs.append(dict(p, value=p["value"][:mid] + bytes([p["value"][mid] ^ 0x10]) + p["value"][mid + 1:]))
            senders.append(i)
        if i % 5 == 2 and len(p["lemma"]) > 1:  # corrupted sibling hash
            lem = list(p["lemma"])
            h, (side, sh) = lem[0]
            lem[0] = (h, (side, bytes([sh[0] ^ 0x80]) + sh[1:]))
            proofs.append(dict(p, lemma=lem))
            senders.append(i)
        if i % 7 == 3:                       # proof for another root
            proofs.append(dict(p, root_hash=b"\x11" * 32))
            senders.append(i)
    arrs = flatten(proofs, senders)
    valid = torch.zeros(len(proofs), dtype=torch.uint8, device="cuda")
    hbx_ctx.merkle_validate_d(*[dev(a) for a in arrs], n, valid)
    torch.cuda.synchronize()
    want = [rm.validate_broadcast_proof(p, s, n, variant) for p, s in zip(proofs, senders)]
    assert valid.cpu().numpy().astype(bool).tolist() == want
    assert sum(want) == n


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8, 13, 40, 128])
@pytest.mark.parametrize("value", [b"Foo", b" " * 32, bytes(range(256)) * 5])
def test_broadcast_decode(hbx_ctx, n, value):
    f = rm.num_faulty(n)
    k, m = rm.coding_counts(n)
    shards, leaves, tree = rm.send_shards(value, n)
    L = shards.shape[1]
    inst = 3   # 0: f silent (the last f), 1: wrong root, 2: one too many missing (when m > 0)
    buf = np.stack([shards] * inst)
    present = np.ones((inst, n), dtype=np.uint8)
    present[0, n - f:] = 0
    present[1, : f] = 0
    if m > 0:
        present[2, : m + 1] = 0
    buf[present == 0] = 0
    roots = np.stack([np.frombuffer(tree.root_hash(), dtype=np.uint8)] * inst).copy()
    roots[1, 0] ^= 1
    out = torch.zeros((inst, k * L), dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(inst, dtype=torch.int64, device="cuda")
    st = torch.zeros(inst, dtype=torch.int32, device="cuda")
    hbx_ctx.broadcast_decode_d(dev(buf), dev(present), dev(roots), k, m, out, out_len, st)
    torch.cuda.synchronize()
    st, out_len, out = st.cpu().numpy(), out_len.cpu().numpy(), out.cpu().numpy()
    for i in range(inst):
        vals = [leaves[j] if present[i, j] else None for j in range(n)]
        want = rm.decode_from_shards(vals, n, roots[i].tobytes())
        if want is None:
            assert st[i] in (HBX_E_TOO_FEW_SHARDS, HBX_E_ROOT_MISMATCH), (i, st[i])
        else:
            assert st[i] == 0, (i, st[i])
            assert out[i, : out_len[i]].tobytes() == want
    assert st[0] == 0 and out[0, : out_len[0]].tobytes() == value


# ---- Merkle tree build + gen_proof and the SHA3
# variant (HBX_MERKLE_SHA3: later hbbft's src/broadcast/merkle.rs; north_star "SHA3 Merkle") ----
def _set_merkle(ctx, variant):
    from hbbft_amd.hbx import MERKLE_SHA3, MERKLE_SHA256

    ctx.set_merkle_digest(MERKLE_SHA3 if variant == "sha3" else MERKLE_SHA256)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sha256", "sha3"])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 13, 128, 256])
def test_merkle_build_and_gen_proof(hbx_ctx, n, variant):
    """Every level of the tree, and gen_proof for every leaf, byte-identical with the oracle's
    MerkleTree / gen_proof (odd node promoted; proofs in hbx_merkle_validate_d's format), and every
    generated proof validates."""
    _set_merkle(hbx_ctx, variant)
    rng = np.random.default_rng(n * 31 + len(variant))
    inst, L = 2, 37
    shards = rng.integers(0, 256, size=(inst, n, L), dtype=np.uint8)
    cnt = hbx_ctx.merkle_node_count(n)
    nodes = torch.zeros((inst, cnt, 32), dtype=torch.uint8, device="cuda")
    roots = torch.zeros((inst, 32), dtype=torch.uint8, device="cuda")
    hbx_ctx.merkle_build_d(dev(shards), nodes, roots)
    req = np.array([(i, j) for i in range(inst) for j in range(n)], dtype=np.uint32)
    P = len(req)
    nh = torch.zeros((P, 17, 32), dtype=torch.uint8, device="cuda")
    sh = torch.zeros((P, 16, 32), dtype=torch.uint8, device="cuda")
    sides = torch.zeros(P, dtype=torch.int32, device="cuda")
    depth = torch.zeros(P, dtype=torch.int32, device="cuda")
    proot = torch.zeros((P, 32), dtype=torch.uint8, device="cuda")
    hbx_ctx.merkle_proofs_d(nodes, n, dev(req), nh, sh, sides, depth, proot)
    torch.cuda.synchronize()
    nodes, roots = nodes.cpu().numpy(), roots.cpu().numpy()
    proofs, senders = [], []
    for i in range(inst):
        leaves = [bytes([j & 0xFF]) + shards[i, j].tobytes() for j in range(n)]
        tree = rm.MerkleTree(leaves, variant)
        flat = [h for lvl in tree.levels for h in lvl]
        assert len(flat) == cnt
        assert [bytes(x) for x in nodes[i]] == flat
        assert roots[i].tobytes() == tree.root_hash()
        for j in range(n):
            proofs.append(tree.gen_proof(leaves[j]))
            senders.append(j)
    want = flatten(proofs, senders)
    _, w_nodes, w_sibs, w_sides, w_depth, w_roots, _ = want
    np.testing.assert_array_equal(depth.cpu().numpy(), w_depth.astype(np.int32))
    np.testing.assert_array_equal(sides.cpu().numpy(), w_sides.astype(np.int32))
    np.testing.assert_array_equal(proot.cpu().numpy(), w_roots)
    got_n, got_s = nh.cpu().numpy(), sh.cpu().numpy()
    for q in range(P):
        d = int(w_depth[q])
        np.testing.assert_array_equal(got_n[q, :d + 1], w_nodes[q, :d + 1])
        np.testing.assert_array_equal(got_s[q, :d], w_sibs[q, :d])
    valid = torch.zeros(P, dtype=torch.uint8, device="cuda")
    hbx_ctx.merkle_validate_d(dev(want[0]), nh, sh, sides, depth, proot, dev(want[6]), n, valid)
    torch.cuda.synchronize()
    assert valid.cpu().numpy().all()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 13])
def test_merkle_sha3_validate_and_decode(hbx_ctx, n):
    """The SHA3 variant through validate_proof (bad sender / value / root rejected) and
    decode_from_shards (f silent, wrong root)."""
    _set_merkle(hbx_ctx, "sha3")
    value = bytes(range(256)) * 2
    shards, leaves, tree = rm.send_shards(value, n, "sha3")
    proofs, senders = [], []
    for i, leaf in enumerate(leaves):
        p = tree.gen_proof(leaf)
        proofs += [p, p, dict(p, value=p["value"][:-1] + bytes([p["value"][-1] ^ 1])), dict(p, root_hash=b"\x11" * 32)]
        senders += [i, (i + 1) % n, i, i]
    arrs = flatten(proofs, senders)
    valid = torch.zeros(len(proofs), dtype=torch.uint8, device="cuda")
    hbx_ctx.merkle_validate_d(*[dev(a) for a in arrs], n, valid)
    torch.cuda.synchronize()
    want = [rm.validate_broadcast_proof(p, s, n, "sha3") for p, s in zip(proofs, senders)]
    assert valid.cpu().numpy().astype(bool).tolist() == want and sum(want) == n
    f = rm.num_faulty(n)
    k, m = rm.coding_counts(n)
    L = shards.shape[1]
    buf = np.stack([shards] * 2)
    present = np.ones((2, n), dtype=np.uint8)
    present[:, n - f:] = 0
    buf[present == 0] = 0
    roots = np.stack([np.frombuffer(tree.root_hash(), dtype=np.uint8)] * 2).copy()
    roots[1, 3] ^= 1
    out = torch.zeros((2, k * L), dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(2, dtype=torch.int64, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    hbx_ctx.broadcast_decode_d(dev(buf), dev(present), dev(roots), k, m, out, out_len, st)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert st[0] == 0 and out[0, : int(out_len[0])].cpu().numpy().tobytes() == value
    assert st[1] == HBX_E_ROOT_MISMATCH


# ---- BASELINE config C5: one 1 MiB proposal at N=128 against the committed
# fixture tests/golden/c5_broadcast.npz (tests/golden/make_c5_golden.py) ----
@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["sha256", "sha3"])
def test_c5_fixture(hbx_ctx, variant):
    import hashlib
    import os

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "c5_broadcast.npz"))
    n, k, m, L, plen = int(g["n"]), int(g["k"]), int(g["m"]), int(g["shard_len"]), int(g["plen"])
    value = np.random.default_rng(int(g["seed"])).integers(0, 256, size=plen, dtype=np.uint8).tobytes()
    assert hashlib.sha256(value).digest() == g["payload_sha"].tobytes()
    _set_merkle(hbx_ctx, variant)
    # send_shards: frame, RS encode (broadcast.rs:341-367)
    framed = int(plen).to_bytes(4, "big") + value
    buf = np.zeros((1, n, L), dtype=np.uint8)
    buf.reshape(-1)[: len(framed)] = np.frombuffer(framed, dtype=np.uint8)
    d = dev(buf)
    hbx_ctx.rs_encode_d(d, k, m)
    torch.cuda.synchronize()
    shards = d.cpu().numpy()[0]
    got = np.stack([np.frombuffer(hashlib.sha256(shards[i].tobytes()).digest(), dtype=np.uint8) for i in range(n)])
    np.testing.assert_array_equal(got, g["shard_sha"])
    # Merkle tree (broadcast.rs:381): every node, root, and the proofs of the fixture's leaves
    cnt = hbx_ctx.merkle_node_count(n)
    assert cnt == int(g[f"node_count_{variant}"])
    nodes = torch.zeros((1, cnt, 32), dtype=torch.uint8, device="cuda")
    roots = torch.zeros((1, 32), dtype=torch.uint8, device="cuda")
    hbx_ctx.merkle_build_d(d, nodes, roots)
    torch.cuda.synchronize()
    assert roots.cpu().numpy()[0].tobytes() == g[f"root_{variant}"].tobytes()
    assert hashlib.sha256(nodes.cpu().numpy().tobytes()).digest() == g[f"nodes_sha_{variant}"].tobytes()
    if variant == "sha256":
        req = np.array([(0, j) for j in g["proof_leaves"]], dtype=np.uint32)
        P = len(req)
        nh = torch.zeros((P, 17, 32), dtype=torch.uint8, device="cuda")
        sh = torch.zeros((P, 16, 32), dtype=torch.uint8, device="cuda")
        sides = torch.zeros(P, dtype=torch.int32, device="cuda")
        depth = torch.zeros(P, dtype=torch.int32, device="cuda")
        proot = torch.zeros((P, 32), dtype=torch.uint8, device="cuda")
        hbx_ctx.merkle_proofs_d(nodes, n, dev(req), nh, sh, sides, depth, proot)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(depth.cpu().numpy(), g["proof_depth"])
        np.testing.assert_array_equal(sides.cpu().numpy(), g["proof_sides"])
        np.testing.assert_array_equal(nh.cpu().numpy(), g["proof_nodes"])
        np.testing.assert_array_equal(sh.cpu().numpy(), g["proof_sibs"])
    # decode_from_shards with the last f shards missing (broadcast.rs:660-707)
    f = (n - 1) // 3
    present = np.ones((1, n), dtype=np.uint8)
    present[0, n - f:] = 0
    work = shards[None].copy()
    work[present == 0] = 0xA5
    out = torch.zeros((1, k * L), dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    hbx_ctx.broadcast_decode_d(dev(work), dev(present), dev(g[f"root_{variant}"][None].copy()), k, m, out, out_len, st)
    torch.cuda.synchronize()
    assert int(st.cpu()[0]) == 0 and int(out_len.cpu()[0]) == plen
    assert hashlib.sha256(out.cpu().numpy()[0, :plen].tobytes()).digest() == g["payload_sha"].tobytes()


@pytest.mark.gpu
def test_broadcast_decode_oversized_header(hbx_ctx):
    """A Byzantine proposer's length header larger than the payload: glue_shards takes the bytes
    there are (broadcast.rs:697-707), and an output row shorter than k L - 4 is rejected
    (the header must never write past the caller's row)."""
    from hbbft_amd.hbx import HbxError

    n = 7
    k, m = rm.coding_counts(n)
    buf = rm.frame_shards(b"payload of a faulty proposer" * 3, n)
    buf[0, :4] = 0xFF  # BE length 2^32 - 1
    buf = rm.ReedSolomon(k, m).encode(buf)
    leaves = [bytes([i]) + buf[i].tobytes() for i in range(n)]
    tree = rm.MerkleTree(leaves)
    L = buf.shape[1]
    want = rm.decode_from_shards(leaves, n, tree.root_hash())
    assert want is not None and len(want) == k * L - 4
    present = np.ones((1, n), dtype=np.uint8)
    root = np.frombuffer(tree.root_hash(), dtype=np.uint8)[None].copy()
    out = torch.zeros((1, k * L), dtype=torch.uint8, device="cuda")
    out_len = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    hbx_ctx.broadcast_decode_d(dev(buf[None]), dev(present), dev(root), k, m, out, out_len, st)
    torch.cuda.synchronize()
    assert int(st[0]) == 0 and int(out_len[0]) == k * L - 4
    assert out[0, : k * L - 4].cpu().numpy().tobytes() == want
    short = torch.zeros((1, k * L - 5), dtype=torch.uint8, device="cuda")
    with pytest.raises(HbxError):
        hbx_ctx.broadcast_decode_d(dev(buf[None]), dev(present), dev(root), k, m, short, out_len, st)
