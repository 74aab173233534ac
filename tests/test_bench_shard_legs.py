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


@pytest.mark.gpu
def test_strong_epoch_slab_world1():
    """Stack A's strong-mode slab path (statuses + the plaintexts written straight into the
    gathered slab, then assembled and compared with every contribution) at a world of one rank:
    bench.py --strong-at-1 runs exactly the code --gpus G runs per rank."""
    import json
    import subprocess

    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--strong-at-1", "--steps", "1", "--warmup", "0",
                          "--configs=", "--no-cpu-baseline", "--in-flight", "1", "--n", "64"],
                         capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["config"]["parallelism"] == "proposer-column x1" and line["value"] > 0
