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


# ---- the same legs at world 2 and 3 on the CPU (gloo), with a stand-in engine ------------------
class _FakeEngine:
    """CPU stand-in for hbbft_amd.hbx.Context in bench.sharded_c4 / sharded_c5 (tests only): the
    coin calls are keyed hashes (a share verifies iff it is the signer's hash of the nonce), the
    Broadcast calls are the oracle's reed-solomon-erasure / Merkle restatement.  What is under test
    is the legs' own control flow -- instance slicing per rank, the slab layout, the gloo
    all-gather, assembly and the gathered-result checks -- which the 8-GPU run executes unchanged."""

    def __init__(self, device=0):
        self.pk = None
        self.nonces = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    @staticmethod
    def _h(*parts, size=32):
        import hashlib

        out = b""
        ctr = 0
        while len(out) < size:
            out += hashlib.sha256(b"".join(parts) + bytes([ctr])).digest()
            ctr += 1
        return out[:size]

    # coin
    def public_keys(self, sk32):
        import numpy as np

        return np.stack([np.frombuffer(self._h(bytes(r), size=48), np.uint8) for r in np.asarray(sk32)])

    def set_pk_shares(self, pk):
        import numpy as np

        self.pk = [bytes(p) for p in pk]
        return np.zeros(len(pk), dtype=np.int32)

    def prepare_nonces(self, nonces, hashes=True):
        self.nonces = [bytes(x) for x in nonces]

    def _sig(self, pk, nonce):
        return self._h(pk, nonce, size=96)

    def sign(self, sk32):
        import numpy as np

        pks = [bytes(p) for p in self.public_keys(sk32)]
        return np.stack([np.stack([np.frombuffer(self._sig(pk, x), np.uint8) for pk in pks]) for x in self.nonces])

    def verify_sig_shares_d(self, d_sigs, d_present=None, d_status=None):
        import numpy as np
        import torch

        sigs = d_sigs.cpu().numpy()
        st = np.array([[sigs[c, i].tobytes() == self._sig(self.pk[i], self.nonces[c]) for i in range(sigs.shape[1])]
                       for c in range(sigs.shape[0])], dtype=np.uint8)
        d_status.copy_(torch.from_numpy(st))
        self._status = st

    def combine_signatures_d(self, master_pk48, t, d_use, d_sig, d_status, d_ok, d_parity):
        import torch

        enough = torch.from_numpy((self._status.sum(axis=1) >= t).astype("uint8"))
        d_status.copy_(torch.where(enough.bool(), 0, -3).to(d_status.dtype))
        d_ok.copy_(enough)
        d_parity.zero_()

    # broadcast
    def set_merkle_digest(self, v):
        assert v == 0

    def rs_encode_d(self, shards, k, m):
        import torch

        from oracle import rs_merkle as rm

        a = shards.cpu().numpy()
        for i in range(a.shape[0]):
            a[i] = rm.ReedSolomon(k, m).encode(a[i].copy())
        shards.copy_(torch.from_numpy(a))

    def merkle_roots_d(self, shards, roots):
        import numpy as np
        import torch

        from oracle import rs_merkle as rm

        a = shards.cpu().numpy()
        r = [np.frombuffer(rm.MerkleTree([bytes([j]) + a[i, j].tobytes() for j in range(a.shape[1])]).root_hash(),
                           np.uint8) for i in range(a.shape[0])]
        roots.copy_(torch.from_numpy(np.stack(r)))

    def broadcast_decode_d(self, work, present, roots, k, m, out, out_len, status):
        import numpy as np
        import torch

        from oracle import rs_merkle as rm

        w, p, r = work.cpu().numpy(), present.cpu().numpy(), roots.cpu().numpy()
        o = np.zeros(out.shape, dtype=np.uint8)
        ln = np.zeros(w.shape[0], dtype=np.int64)
        st = np.zeros(w.shape[0], dtype=np.int32)
        n = k + m
        for i in range(w.shape[0]):
            leaves = [bytes([j]) + w[i, j].tobytes() if p[i, j] else None for j in range(n)]
            v = rm.decode_from_shards(leaves, n, r[i].tobytes())
            if v is None:
                st[i] = -10
            else:
                o[i, :len(v)] = np.frombuffer(v, np.uint8)
                ln[i] = len(v)
        out.copy_(torch.from_numpy(o))
        out_len.copy_(torch.from_numpy(ln).to(out_len.dtype))
        status.copy_(torch.from_numpy(st).to(status.dtype))


class _FakeEpoch:
    """Stand-in for bench._WeakEpoch: a step is a small CPU computation, the check its result."""

    steps_run = 0

    def __init__(self, rank):
        self.units = 64
        self.acc = rank

    def step(self):
        _FakeEpoch.steps_run += 1
        self.acc = (self.acc * 31 + 7) % 1000003

    def check(self):
        return self.acc >= 0


def _legs_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench

    try:
        args = bench.parse_args_for_test(["--steps", "1"])
        dev = torch.device("cpu")
        c4 = bench.sharded_c4(args, dev, torch, _FakeEngine, world, rank, n=7, inst=8)
        c5 = bench.sharded_c5(args, dev, torch, _FakeEngine, world, rank, n=7, inst=5, plen=300)
        # the weak node-rate sub-object and the slab gather's own time (bench.main at --gpus G > 1)
        wk = bench.weak_epochs(args, dev, torch, world, rank, lambda: _FakeEpoch(rank))
        gms = bench.gather_ms(torch, dev, world, torch.full((40,), rank, dtype=torch.uint8), reps=3)
        ok = c4["ms_per_round"] > 0 and c5["ms_per_round"] > 0 and gms > 0
        ok = ok and wk["scaling"] == "weak" and wk["epochs"] == world * 2 and wk["value"] > 0
        ok = ok and _FakeEpoch.steps_run == 3  # one untimed + steps (max(1, 2))
        q.put((rank, c4["instances_per_gpu"], c5["instances_per_gpu"], ok, None))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        import traceback

        q.put((rank, -1, -1, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_legs_gloo(world):
    """bench.sharded_c4 / sharded_c5 at world 2 and 3 over gloo on the CPU (uneven instance splits:
    8 coin instances, 5 proposals), each leg's gathered-result assertions included; and the weak
    node-rate sub-object (bench.weak_epochs: whole epochs per rank, verdicts all-gathered) and the
    slab gather's own time (bench.gather_ms) that bench.main adds at --gpus G > 1."""
    import torch.multiprocessing as mp

    from hbbft_amd import shard

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_legs_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, c4, c5, ok, err in res:
        assert err is None, err
        assert ok
        lo, hi = shard.instance_range(8, world, rank)
        assert c4 == hi - lo
        lo, hi = shard.instance_range(5, world, rank)
        assert c5 == hi - lo
