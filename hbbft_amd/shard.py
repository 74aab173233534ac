"""Multi-GPU sharding of one epoch's verification work.

One process per GPU.  Verifications are independent, so the N x N share matrix is split by
proposer column: rank g owns a contiguous block of proposers together with their ciphertexts,
hoisted hashes, prepared lines and combines; key material is replicated.  Nothing crosses GPUs
while the kernels run.  Afterwards ONE all-gather (RCCL over xGMI on GPUs, gloo in the CPU tests)
assembles every rank's fixed-size result slab -- per-share HBX_SHARE_* status bytes, per-ciphertext
HBX_CT_* bytes, per-proposer combine status -- so each rank holds the node's complete epoch result,
the input the reference's fault-log and decryption logic consumes (honey_badger.rs:422-461,
:315-349; hbbft_amd/honey_badger.py).  Plaintexts stay on the GPU that decrypted them.
"""
from __future__ import annotations

import numpy as np


def proposer_range(n: int, world: int, rank: int):
    """[lo, hi) of the proposer columns rank ``rank`` owns: contiguous blocks, the first n % world
    ranks one column more (any N over any number of ranks)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def max_columns(n: int, world: int) -> int:
    return -(-n // world)


def slab_layout(n: int, pj: int):
    """Byte offsets of one rank's result slab for up to ``pj`` proposer columns:
    share status [pj*n] | ct status [pj] | combine status int32 [pj].  Every rank uses the
    layout of max_columns(n, world) so the slabs have equal size for one all-gather."""
    a = pj * n
    b = a + pj
    c = (b + 3) // 4 * 4
    return {"valid": (0, a), "ct_valid": (a, b), "status": (c, c + 4 * pj), "size": c + 4 * pj}


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
    """Gathered slabs -> (share status uint8[n, n], ct status uint8[n], combine status int32[n]) in
    proposer order."""
    pm = max_columns(n, world)
    lay = slab_layout(n, pm)
    g = np.asarray(gathered, dtype=np.uint8).reshape(world, lay["size"])
    sv, cv, st = [], [], []
    for r in range(world):
        lo, hi = proposer_range(n, world, r)
        pj = hi - lo
        sv.append(g[r, lay["valid"][0]:lay["valid"][0] + pj * n].reshape(pj, n))
        cv.append(g[r, lay["ct_valid"][0]:lay["ct_valid"][0] + pj])
        st.append(g[r, lay["status"][0]:lay["status"][0] + 4 * pj].copy().view(np.int32))
    return np.concatenate(sv), np.concatenate(cv), np.concatenate(st)
