"""Multi-rank epoch sharding on CPU (gloo, world_size 2): each rank fills its proposer-column
slab, one all-gather assembles the node's full epoch result."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hbbft_amd import shard

    lo, hi = shard.proposer_range(n, world, rank)
    pj = hi - lo
    lay = shard.slab_layout(n, pj)
    slab = torch.zeros(lay["size"], dtype=torch.uint8)
    full_valid = (np.arange(n * n).reshape(n, n) % 5) != 0
    slab[lay["valid"][0]:lay["valid"][1]] = torch.from_numpy(full_valid[lo:hi].astype(np.uint8).reshape(-1))
    slab[lay["ct_valid"][0]:lay["ct_valid"][1]] = 1
    st = np.arange(lo, hi, dtype=np.int32) * -1
    slab[lay["status"][0]:lay["status"][1]] = torch.from_numpy(st.view(np.uint8))
    g = shard.all_gather_slabs(slab, world)
    valid, ctv, status = shard.assemble(g.numpy(), n, world)
    ok = (valid == full_valid).all() and ctv.all() and (status == -np.arange(n)).all()
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_two_rank_gather():
    world, n = 2, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
