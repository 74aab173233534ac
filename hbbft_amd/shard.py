"""Multi-GPU sharding of one epoch's verification work.

One process per GPU.  Verifications are independent, so the N x N share matrix is split by
proposer column: rank g owns proposers [g N/G, (g+1) N/G) together with their ciphertexts, hoisted
hashes, prepared lines and combines; key material is replicated.  Nothing crosses GPUs while the
kernels run.  Afterwards ONE all-gather (RCCL over xGMI on GPUs, gloo in the CPU tests) assembles
every rank's fixed-size result slab -- validity bytes, ciphertext bits, per-proposer status -- so
each rank holds the node's complete epoch result, the input the reference's fault-log and
decryption logic consumes (honey_badger.rs:422-461, :315-349).
"""
from __future__ import annotations

import numpy as np


def proposer_range(n: int, world: int, rank: int):
    """[lo, hi) of the proposer columns rank ``rank`` owns."""
    if n % world:
        raise ValueError(f"N={n} does not divide over {world} ranks")
    return rank * n // world, (rank + 1) * n // world


def slab_layout(n: int, pj: int):
    """Byte offsets of one rank's result slab: valid[pj*n] | ct_valid[pj] | status int32[pj]."""
    a = pj * n
    b = a + pj
    return {"valid": (0, a), "ct_valid": (a, b), "status": (b, b + 4 * pj), "size": b + 4 * pj}


def all_gather_slabs(slab, world: int):
    """All-gather equal-size uint8 slabs (torch tensors, any device) -> [world, size]."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return slab.view(1, -1)
    out = torch.empty(world * slab.numel(), dtype=slab.dtype, device=slab.device)
    if slab.device.type == "cuda":
        dist.all_gather_into_tensor(out, slab)
    else:  # gloo
        parts = list(out.view(world, -1).unbind(0))
        dist.all_gather(parts, slab)
    return out.view(world, -1)


def assemble(gathered: np.ndarray, n: int, world: int):
    """Gathered slabs -> (valid[n, n] bool, ct_valid[n] bool, status[n] int32) in proposer order."""
    pj = n // world
    lay = slab_layout(n, pj)
    g = np.asarray(gathered, dtype=np.uint8).reshape(world, lay["size"])
    valid = np.concatenate([g[r, lay["valid"][0]:lay["valid"][1]].reshape(pj, n) for r in range(world)]).astype(bool)
    ctv = np.concatenate([g[r, lay["ct_valid"][0]:lay["ct_valid"][1]] for r in range(world)]).astype(bool)
    st = np.concatenate([g[r, lay["status"][0]:lay["status"][1]].copy().view(np.int32) for r in range(world)])
    return valid, ctv, st
