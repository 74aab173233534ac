"""Multi-rank Common Coin and Broadcast rounds ("Coin: shard by instance.
Broadcast: shard by instance (proposer)").  Each rank owns a contiguous range of
instances (``shard.instance_range``), fills a fixed-size result slab (``shard.coin_layout`` /
``shard.broadcast_layout``) with its instances' results, and one all-gather gives every rank the
round's whole result.

* CPU (gloo, world 2 and 3): slabs filled with the coin fixtures' expectations and with the
  oracle's broadcast results assemble to the full round;
* GPU: each rank's slice run through the engine on its own (as that rank's GPU would: nonces,
  signature shares, combines; or encode, Merkle roots, decode), slabs assembled as the all-gather
  would, against the fixtures / the oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

GOLD = os.path.join(os.path.dirname(__file__), "golden")
COIN_FIX = ["coin_n7", "coin_n128"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _coin(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))


def coin_slab(d, world, rank, results=None):
    """The slab of rank ``rank``: its instances' (share status, sig, combine status, master ok,
    parity), from ``results`` (the engine's) or the fixture's expectations."""
    from hbbft_amd import shard

    count, n = d["sigs"].shape[:2]
    lo, hi = shard.instance_range(count, world, rank)
    lay = shard.coin_layout(count, n, world)
    slab = np.zeros(lay.size, dtype=np.uint8)
    r = results or {"share_status": d["expect_share_status"][lo:hi], "sig": d["expect_sig"][lo:hi],
                    "comb_status": d["expect_status"][lo:hi], "master_ok": d["expect_master_ok"][lo:hi],
                    "parity": d["expect_parity"][lo:hi]}
    for name, v in r.items():
        lay.view(slab, name, hi - lo)[...] = np.asarray(v)
    return slab


def check_coin(d, full):
    np.testing.assert_array_equal(full["share_status"], d["expect_share_status"])
    np.testing.assert_array_equal(full["sig"], d["expect_sig"])
    np.testing.assert_array_equal(full["comb_status"], d["expect_status"])
    np.testing.assert_array_equal(full["master_ok"].astype(bool), d["expect_master_ok"])
    np.testing.assert_array_equal(full["parity"].astype(bool), d["expect_parity"])


def broadcast_round(n, count, seed, variant="sha256"):
    """Oracle results of ``count`` proposals at N = n: root, decode status (all f last shards
    missing) and output length per instance."""
    from oracle import broadcast as ob
    from oracle import rs_merkle as rm

    rng = np.random.default_rng(seed)
    f = rm.num_faulty(n)
    vals, roots, lens, shards = [], [], [], []
    for i in range(count):
        v = rng.integers(0, 256, size=int(rng.integers(1, 3000)), dtype=np.uint8).tobytes()
        sh, leaves, tree = rm.send_shards(v, n, variant)
        vals.append(v)
        shards.append(sh)
        roots.append(np.frombuffer(tree.root_hash(), dtype=np.uint8))
        present = [leaf if j < n - f else None for j, leaf in enumerate(leaves)]
        out = ob.decode_from_shards(present, n, tree.root_hash(), variant)
        assert out == v
        lens.append(len(out))
    return vals, shards, np.stack(roots), np.array(lens, dtype=np.int64)


def bc_slab(roots, status, lens, count, world, rank):
    from hbbft_amd import shard

    lo, hi = shard.instance_range(count, world, rank)
    lay = shard.broadcast_layout(count, world)
    slab = np.zeros(lay.size, dtype=np.uint8)
    lay.view(slab, "root", hi - lo)[...] = roots
    lay.view(slab, "decode_status", hi - lo)[...] = status
    lay.view(slab, "out_len", hi - lo)[...] = lens
    return slab


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hbbft_amd import shard

    ok = True
    for name in COIN_FIX:
        d = _coin(name)
        count, n = d["sigs"].shape[:2]
        g = shard.all_gather_slabs(torch.from_numpy(coin_slab(d, world, rank)), world)
        full = shard.assemble_fields(g.numpy(), shard.coin_layout(count, n, world), count, world)
        try:
            check_coin(d, full)
        except AssertionError:
            ok = False
    n, count = 7, 5
    _, _, roots, lens = broadcast_round(n, count, 11)
    lo, hi = shard.instance_range(count, world, rank)
    slab = bc_slab(roots[lo:hi], np.zeros(hi - lo, np.int32), lens[lo:hi], count, world, rank)
    g = shard.all_gather_slabs(torch.from_numpy(slab), world)
    full = shard.assemble_fields(g.numpy(), shard.broadcast_layout(count, world), count, world)
    ok = ok and (full["root"] == roots).all() and (full["out_len"] == lens).all() and (full["decode_status"] == 0).all()
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_gather_coin_and_broadcast_rounds(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def test_slab_layout_views():
    from hbbft_amd import shard

    lay = shard.coin_layout(5, 7, 2)  # 3 instances per rank at most
    assert lay.size % 8 == 0
    buf = np.zeros(lay.size, dtype=np.uint8)
    lay.view(buf, "comb_status", 2)[...] = [-3, 7]
    lay.view(buf, "sig", 2)[1, 95] = 9
    assert list(lay.view(buf, "comb_status")) == [-3, 7, 0]
    assert lay.view(buf, "sig")[1, 95] == 9 and lay.view(buf, "parity").shape == (3,)


# ---- GPU --------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", COIN_FIX)
def test_gpu_coin_shard_slices(hbx_ctx, name, world):
    from hbbft_amd import shard

    d = _coin(name)
    count, n = d["sigs"].shape[:2]
    assert (hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]]) == 0).all()
    dev = torch.device("cuda", 0)
    off = d["nonce_off"].astype(np.int64)
    nonces = [d["nonce_blob"][off[j]:off[j + 1]].tobytes() for j in range(count)]
    slabs = []
    for r in range(world):
        lo, hi = shard.instance_range(count, world, r)
        c = hi - lo
        hbx_ctx.prepare_nonces(nonces[lo:hi])
        d_st = torch.zeros((c, n), dtype=torch.uint8, device=dev)
        hbx_ctx.verify_sig_shares_d(torch.from_numpy(np.ascontiguousarray(d["sigs"][lo:hi])).to(dev),
                                    torch.from_numpy(np.ascontiguousarray(d["present"][lo:hi]).astype(np.uint8)).to(dev),
                                    d_st)
        d_sig = torch.zeros((c, 96), dtype=torch.uint8, device=dev)
        d_cs = torch.zeros(c, dtype=torch.int32, device=dev)
        d_ok = torch.zeros(c, dtype=torch.uint8, device=dev)
        d_par = torch.zeros(c, dtype=torch.uint8, device=dev)
        hbx_ctx.combine_signatures_d(d["master_pk"].tobytes(), int(d["t"]), None, d_sig, d_cs, d_ok, d_par)
        torch.cuda.synchronize(dev)
        res = {"share_status": d_st.cpu().numpy(), "sig": d_sig.cpu().numpy(), "comb_status": d_cs.cpu().numpy(),
               "master_ok": d_ok.cpu().numpy(), "parity": d_par.cpu().numpy()}
        slabs.append(coin_slab(d, world, r, res))
    full = shard.assemble_fields(np.stack(slabs), shard.coin_layout(count, n, world), count, world)
    # statuses where the combine failed carry no signature bytes in the fixture
    check_coin(d, full)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_broadcast_shard_slices(hbx_ctx, world):
    from hbbft_amd import shard
    from oracle import rs_merkle as rm

    n, count = 16, 6
    vals, shards, roots, lens = broadcast_round(n, count, 23)
    k, m = rm.coding_counts(n)
    f = rm.num_faulty(n)
    dev = torch.device("cuda", 0)
    hbx_ctx.set_merkle_digest(0)
    slabs = []
    for r in range(world):
        lo, hi = shard.instance_range(count, world, r)
        c = hi - lo
        L = max(shards[i].shape[1] for i in range(lo, hi))
        buf = np.zeros((c, n, L), dtype=np.uint8)
        groups = {}
        for q, i in enumerate(range(lo, hi)):
            groups.setdefault(shards[i].shape[1], []).append(q)
        st = np.zeros(c, dtype=np.int32)
        ln = np.zeros(c, dtype=np.int64)
        rt = np.zeros((c, 32), dtype=np.uint8)
        for Li, qs in groups.items():  # one engine call per shard length, as the replay does
            data = np.zeros((len(qs), n, Li), dtype=np.uint8)
            for a, q in enumerate(qs):
                data[a, :k] = shards[lo + q][:k]
            d_sh = torch.from_numpy(data).to(dev)
            hbx_ctx.rs_encode_d(d_sh, k, m)
            d_rt = torch.zeros((len(qs), 32), dtype=torch.uint8, device=dev)
            hbx_ctx.merkle_roots_d(d_sh, d_rt)
            present = np.ones((len(qs), n), dtype=np.uint8)
            present[:, n - f:] = 0
            d_out = torch.zeros((len(qs), k * Li), dtype=torch.uint8, device=dev)
            d_len = torch.zeros(len(qs), dtype=torch.int64, device=dev)
            d_st = torch.zeros(len(qs), dtype=torch.int32, device=dev)
            hbx_ctx.broadcast_decode_d(d_sh, torch.from_numpy(present).to(dev), d_rt, k, m, d_out, d_len, d_st)
            torch.cuda.synchronize(dev)
            for a, q in enumerate(qs):
                st[q] = d_st[a].item()
                ln[q] = d_len[a].item()
                rt[q] = d_rt[a].cpu().numpy()
                assert d_out[a, :ln[q]].cpu().numpy().tobytes() == vals[lo + q]
        del buf
        slabs.append(bc_slab(rt, st, ln, count, world, r))
    full = shard.assemble_fields(np.stack(slabs), shard.broadcast_layout(count, world), count, world)
    np.testing.assert_array_equal(full["root"], roots)
    np.testing.assert_array_equal(full["out_len"], lens)
    assert (full["decode_status"] == 0).all()
