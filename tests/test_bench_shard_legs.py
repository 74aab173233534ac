"""The bench's multi-GPU legs for stacks B and C (bench.py sharded_c4 / sharded_c5: instance
sharding + one all-gather of result slabs) run on the GPU with a world of one
rank over RCCL (the one GPU of a test box; the driver runs the N-GPU case), with their own checks
of the gathered round result."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_sharded_legs_world1(hbx_ctx):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench
    from hbbft_amd.hbx import Context

    dev = torch.device("cuda", 0)
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        args = bench.parse_args_for_test(["--steps", "1"])
        c4 = bench.sharded_c4(args, dev, torch, Context, 1, 0)
        c5 = bench.sharded_c5(args, dev, torch, Context, 1, 0)
    finally:
        dist.destroy_process_group()
    assert c4["instances_per_gpu"] == 256 and c4["value"] > 0
    assert c5["instances_per_gpu"] == 128 and c5["value"] > 0
