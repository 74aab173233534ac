"""Multi-rank epoch sharding on CPU (gloo): each rank owns a block of proposer columns of the
N = 64 fixture (tests/golden/hb_epoch_n64.npz, BASELINE config 2), fills its result slab with that
slice's per-share / per-ciphertext / combine statuses (the oracle's results for the slice, which
is what the engine returns for it: test_gpu_shard_slices checks that on the GPU), and one
all-gather assembles the node's full epoch result.  World sizes 2 and 3 (N not
divisible by the world size)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

FIX = os.path.join(os.path.dirname(__file__), "golden", "hb_epoch_n64.npz")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def slab_for_slice(d, n, world, rank, share_status=None, ct_status=None, comb_status=None):
    from hbbft_amd import shard

    lo, hi = shard.proposer_range(n, world, rank)
    pj = hi - lo
    lay = shard.slab_layout(n, shard.max_columns(n, world))
    slab = np.zeros(lay["size"], dtype=np.uint8)
    ss = d["expect_share_status"][lo:hi] if share_status is None else share_status
    cs = d["expect_ct_status"][lo:hi] if ct_status is None else ct_status
    st = d["expect_status"][lo:hi] if comb_status is None else comb_status
    slab[lay["valid"][0]:lay["valid"][0] + pj * n] = np.asarray(ss, dtype=np.uint8).reshape(-1)
    slab[lay["ct_valid"][0]:lay["ct_valid"][0] + pj] = cs
    slab[lay["status"][0]:lay["status"][0] + 4 * pj] = np.asarray(st, dtype=np.int32).view(np.uint8)
    return slab


def plain_slab(n, world, rank, lens, pb, seed=3):
    """A slab with only the plaintext region filled: proposer j's plaintext = bytes of a seeded
    stream of length lens[j] (what the rank's decryption writes there)."""
    from hbbft_amd import shard

    lay = shard.slab_layout(n, shard.max_columns(n, world), pb)
    slab = np.zeros(lay["size"], dtype=np.uint8)
    lo, hi = shard.proposer_range(n, world, rank)
    pos = lay["plain"][0]
    for j in range(lo, hi):
        slab[pos:pos + lens[j]] = np.random.default_rng(seed + j).integers(0, 256, size=lens[j], dtype=np.uint8)
        pos += lens[j]
    return slab


def _plain_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hbbft_amd import shard

    n = 10
    lens = [5 + 7 * j for j in range(n)]
    pb = max(sum(lens[lo:hi]) for lo, hi in (shard.proposer_range(n, world, r) for r in range(world)))
    g = shard.all_gather_slabs(torch.from_numpy(plain_slab(n, world, rank, lens, pb)), world)
    got = shard.assemble_plaintexts(g.numpy(), n, world, lens, pb)
    want = [np.random.default_rng(3 + j).integers(0, 256, size=lens[j], dtype=np.uint8).tobytes() for j in range(n)]
    ss, cs, st = shard.assemble(g.numpy(), n, world)  # the status fields still assemble with the plaintext region
    q.put((rank, got == want and ss.shape == (n, n)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_gather_plaintexts(world):
    """The combined outputs of stack A -- every proposer's plaintext -- travel in the same
    all-gather as the statuses (north_star: "validity bitmaps and combined outputs")."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plain_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _keys_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hbbft_amd import shard

    d = dict(np.load(FIX, allow_pickle=False))
    n = int(d["n"])
    mine = rank == 0
    pk, mpk, sk, t = shard.broadcast_key_material(d["pk_comp"] if mine else np.zeros((n, 48), np.uint8),
                                                  d["master_pk"].tobytes() if mine else bytes(48),
                                                  d["own_sk"].tobytes() if mine else bytes(32),
                                                  int(d["t"]) if mine else 0, n, world, torch.device("cpu"))
    ok = (pk == d["pk_comp"]).all() and mpk == d["master_pk"].tobytes() and sk == d["own_sk"].tobytes() and t == int(d["t"])
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_key_material_broadcast(world):
    """One broadcast per era gives every rank the node's key material (pk shares, master key,
    own secret share, threshold) of rank 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_keys_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hbbft_amd import shard

    d = dict(np.load(FIX, allow_pickle=False))
    n = int(d["n"])
    slab = torch.from_numpy(slab_for_slice(d, n, world, rank))
    g = shard.all_gather_slabs(slab, world)
    ss, cs, st = shard.assemble(g.numpy(), n, world)
    ok = ((ss == d["expect_share_status"]).all() and (cs == d["expect_ct_status"]).all()
          and (st == d["expect_status"]).all())
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_gather_fixture_epoch(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def test_proposer_ranges_cover():
    from hbbft_amd import shard

    for n in (1, 7, 64, 256):
        for world in (1, 2, 3, 8):
            rs = [shard.proposer_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) == shard.max_columns(n, world)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [3, 8])
def test_gpu_shard_slices(hbx_ctx, world):
    """The sharded result path with the HIP engine: each rank's proposer slice of the N = 64 epoch
    is run through hbx_decrypt_epoch_d on its own (as that rank's GPU would), the slabs are
    assembled as the all-gather would, and the node's epoch result equals the full fixture."""
    from hbbft_amd import shard

    d = dict(np.load(FIX, allow_pickle=False))
    n = int(d["n"])
    assert (hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]]) == 0).all()
    dev = torch.device("cuda", 0)
    slabs = []
    for r in range(world):
        lo, hi = shard.proposer_range(n, world, r)
        pj = hi - lo
        off = d["v_off"][lo:hi + 1].astype(np.int64)
        off0 = off - off[0]
        t_u = torch.from_numpy(np.ascontiguousarray(d["u"][lo:hi])).to(dev)
        t_w = torch.from_numpy(np.ascontiguousarray(d["w"][lo:hi])).to(dev)
        t_v = torch.from_numpy(np.ascontiguousarray(d["v_blob"][off[0]:off[-1]])).to(dev)
        t_off = torch.from_numpy(off0).to(dev)
        t_sh = torch.from_numpy(np.ascontiguousarray(d["shares"][lo:hi])).to(dev)
        t_pr = torch.from_numpy(np.ascontiguousarray(d["present"][lo:hi]).astype(np.uint8)).to(dev)
        t_out = torch.zeros(max(int(off0[-1]), 1), dtype=torch.uint8, device=dev)
        t_valid = torch.zeros(pj * n, dtype=torch.uint8, device=dev)
        t_ct = torch.zeros(pj, dtype=torch.uint8, device=dev)
        t_st = torch.zeros(pj, dtype=torch.int32, device=dev)
        hbx_ctx.decrypt_epoch_d(t_u, t_v, t_off, t_w, pj, int(np.max(np.diff(off0))), t_sh, n, int(d["t"]), t_out,
                                d_valid=t_valid, d_ct_valid=t_ct, d_status=t_st, d_present=t_pr)
        slabs.append(slab_for_slice(d, n, world, r, t_valid.cpu().numpy().reshape(pj, n), t_ct.cpu().numpy(),
                                    t_st.cpu().numpy()))
    ss, cs, st = shard.assemble(np.stack(slabs), n, world)
    np.testing.assert_array_equal(ss, d["expect_share_status"])
    np.testing.assert_array_equal(cs, d["expect_ct_status"])
    np.testing.assert_array_equal(st, d["expect_status"])


@pytest.mark.gpu
def test_gpu_rccl_gather_world1(hbx_ctx):
    """The all-gather of shard.py on RCCL (backend "nccl") with the slab on the GPU: a world of one
    rank (the one GPU of a test box) gathers the N = 64 epoch's result slab computed by the engine,
    through dist.all_gather_into_tensor itself (not the world == 1 shortcut)."""
    from hbbft_amd import shard

    d = dict(np.load(FIX, allow_pickle=False))
    n = int(d["n"])
    assert (hbx_ctx.set_pk_shares([row.tobytes() for row in d["pk_comp"]]) == 0).all()
    dev = torch.device("cuda", 0)
    off = d["v_off"].astype(np.int64)
    t_valid = torch.zeros(n * n, dtype=torch.uint8, device=dev)
    t_ct = torch.zeros(n, dtype=torch.uint8, device=dev)
    t_st = torch.zeros(n, dtype=torch.int32, device=dev)
    hbx_ctx.decrypt_epoch_d(torch.from_numpy(d["u"]).to(dev), torch.from_numpy(d["v_blob"]).to(dev),
                            torch.from_numpy(off).to(dev), torch.from_numpy(d["w"]).to(dev), n,
                            int(np.max(np.diff(off))), torch.from_numpy(d["shares"]).to(dev), n, int(d["t"]),
                            torch.zeros(max(int(off[-1]), 1), dtype=torch.uint8, device=dev), d_valid=t_valid,
                            d_ct_valid=t_ct, d_status=t_st,
                            d_present=torch.from_numpy(d["present"].astype(np.uint8)).to(dev))
    lay = shard.slab_layout(n, n)
    slab = torch.zeros(lay["size"], dtype=torch.uint8, device=dev)
    slab[lay["valid"][0]:lay["valid"][1]] = t_valid
    slab[lay["ct_valid"][0]:lay["ct_valid"][1]] = t_ct
    slab[lay["status"][0]:lay["status"][1]] = t_st.view(torch.uint8)
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        out = torch.empty_like(slab)
        dist.all_gather_into_tensor(out, slab)
        torch.cuda.synchronize(dev)
    finally:
        dist.destroy_process_group()
    ss, cs, st = shard.assemble(out.cpu().numpy().reshape(1, -1), n, 1)
    np.testing.assert_array_equal(ss, d["expect_share_status"])
    np.testing.assert_array_equal(cs, d["expect_ct_status"])
    np.testing.assert_array_equal(st, d["expect_status"])
