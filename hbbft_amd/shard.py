"""Multi-GPU sharding of one epoch's verification work.

One process per GPU.  Verifications are independent, so the N x N share matrix is split by
proposer column: rank g owns a contiguous block of proposers together with their ciphertexts,
hoisted hashes, prepared lines and combines; key material is replicated.  Nothing crosses GPUs
while the kernels run.  Afterwards ONE all-gather (RCCL over xGMI on GPUs, gloo in the CPU tests)
assembles every rank's fixed-size result slab -- per-share HBX_SHARE_* status bytes, per-ciphertext
HBX_CT_* bytes, per-proposer combine status and the decrypted plaintexts (the rank's decryption
output buffer is the slab's plaintext region, so gathering them costs no copy) -- so each rank holds
the node's complete epoch result and every contribution, the input the reference's fault-log and
decryption logic consumes (honey_badger.rs:422-461, :315-349; hbbft_amd/honey_badger.py).
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


def slab_layout(n: int, pj: int, plain_bytes: int = 0):
    """Byte offsets of one rank's result slab for up to ``pj`` proposer columns:
    share status [pj*n] | ct status [pj] | combine status int32 [pj] | plaintexts [plain_bytes].
    The plaintext region is the rank's decryption output blob itself (its proposers' plaintexts
    back to back at their ciphertexts' V offsets; hbx_decrypt_epoch_d writes it in place), sized
    for the largest rank's blob.  Every rank uses the layout of max_columns(n, world) so the slabs
    have equal size for one all-gather."""
    a = pj * n
    b = a + pj
    c = (b + 3) // 4 * 4
    d = c + 4 * pj
    lay = {"valid": (0, a), "ct_valid": (a, b), "status": (c, d), "size": d}
    if plain_bytes:
        e = (d + 7) // 8 * 8
        lay["plain"] = (e, e + plain_bytes)
        lay["size"] = (e + plain_bytes + 7) // 8 * 8
    return lay


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


def assemble_plaintexts(gathered: np.ndarray, n: int, world: int, lens, plain_bytes: int):
    """Gathered slabs -> every proposer's plaintext (bytes), in proposer order: rank r's blob
    holds its proposers' plaintexts back to back, lengths ``lens[j]`` (the ciphertexts' |V|,
    known to every node)."""
    pm = max_columns(n, world)
    lay = slab_layout(n, pm, plain_bytes)
    g = np.asarray(gathered, dtype=np.uint8).reshape(world, lay["size"])
    out = []
    for r in range(world):
        lo, hi = proposer_range(n, world, r)
        pos = lay["plain"][0]
        for j in range(lo, hi):
            out.append(g[r, pos:pos + int(lens[j])].tobytes())
            pos += int(lens[j])
    return out


def broadcast_key_material(pk_comp, master_pk48: bytes, own_sk32: bytes, t: int, n: int, world: int, device,
                           src: int = 0):
    """Once per era (a key change is a new era, dynamic_honey_badger.rs): the node's key material
    -- the N compressed public key shares (NetworkInfo, messaging.rs:251-254), the master public
    key, this node's secret key share and the threshold -- from rank ``src`` to every rank in ONE
    broadcast (RCCL on GPUs, gloo in the CPU tests), instead of each rank deriving it.  Other ranks
    pass anything for the values (only ``n`` must agree).  Returns (pk_comp uint8[n, 48],
    master_pk48, own_sk32, t)."""
    import torch
    import torch.distributed as dist

    size = 4 + 48 + 32 + 48 * n
    buf = np.zeros(size, dtype=np.uint8)
    if world == 1 or dist.get_rank() == src:
        buf[:4] = np.frombuffer(np.uint32(t).tobytes(), dtype=np.uint8)
        buf[4:52] = np.frombuffer(bytes(master_pk48), dtype=np.uint8)
        buf[52:84] = np.frombuffer(bytes(own_sk32), dtype=np.uint8)
        buf[84:] = np.asarray(pk_comp, dtype=np.uint8).reshape(-1)
    if world > 1:
        tb = torch.from_numpy(buf).to(device)
        dist.broadcast(tb, src)
        buf = tb.cpu().numpy()
    return (buf[84:].reshape(n, 48).copy(), buf[4:52].tobytes(), buf[52:84].tobytes(),
            int(buf[:4].copy().view(np.uint32)[0]))


def assemble(gathered: np.ndarray, n: int, world: int):
    """Gathered slabs -> (share status uint8[n, n], ct status uint8[n], combine status int32[n]) in
    proposer order."""
    pm = max_columns(n, world)
    lay = slab_layout(n, pm)
    g = np.asarray(gathered, dtype=np.uint8).reshape(world, -1)[:, :lay["size"]]
    sv, cv, st = [], [], []
    for r in range(world):
        lo, hi = proposer_range(n, world, r)
        pj = hi - lo
        sv.append(g[r, lay["valid"][0]:lay["valid"][0] + pj * n].reshape(pj, n))
        cv.append(g[r, lay["ct_valid"][0]:lay["ct_valid"][0] + pj])
        st.append(g[r, lay["status"][0]:lay["status"][0] + 4 * pj].copy().view(np.int32))
    return np.concatenate(sv), np.concatenate(cv), np.concatenate(st)


# ---------------------------------------------------------------------------------------------
# Common Coin and Broadcast rounds: sharded by instance ("Coin: shard by
# instance.  Broadcast: shard by instance (proposer)").  Rank g owns the contiguous instance range
# instance_range(count, world, g) -- its nonces (hash_g2, lines), signature shares, combines, or
# its proposals (encode, Merkle trees, Echo validation, decodes).  One all-gather of a fixed-size
# slab per rank then gives every rank the whole round's result: per-share status bytes, combined
# signatures with their master-check and parity bits (coin), or the roots, decode statuses and
# output lengths (broadcast); payload bytes stay on the owning GPU.
# ---------------------------------------------------------------------------------------------
instance_range = proposer_range


class SlabLayout:
    """Named fields of one rank's result slab at 8-byte aligned offsets: [(name, numpy dtype,
    shape)], shapes for the largest rank's instance count so that all slabs have one size."""

    def __init__(self, fields):
        self.fields = {}
        pos = 0
        for name, dt, shape in fields:
            dt = np.dtype(dt)
            pos = (pos + 7) // 8 * 8
            nbytes = int(np.prod(shape)) * dt.itemsize
            self.fields[name] = (pos, dt, tuple(shape), nbytes)
            pos += nbytes
        self.size = (pos + 7) // 8 * 8

    def view(self, buf, name, rows=None):
        """Typed view of field ``name`` in a uint8 buffer (numpy array or torch tensor), optionally
        only its first ``rows`` rows."""
        off, dt, shape, nbytes = self.fields[name]
        part = buf[off:off + nbytes]
        if hasattr(part, "view") and not isinstance(part, np.ndarray):  # torch
            import torch

            tdt = {np.dtype(np.uint8): torch.uint8, np.dtype(np.int32): torch.int32,
                   np.dtype(np.int64): torch.int64}[dt]
            v = part.view(tdt).view(shape)
        else:
            v = part.view(dt).reshape(shape)
        return v if rows is None else v[:rows]


def coin_layout(count: int, n: int, world: int) -> SlabLayout:
    im = max_columns(count, world)
    return SlabLayout([("share_status", np.uint8, (im, n)), ("sig", np.uint8, (im, 96)),
                       ("comb_status", np.int32, (im,)), ("master_ok", np.uint8, (im,)),
                       ("parity", np.uint8, (im,))])


def broadcast_layout(count: int, world: int) -> SlabLayout:
    im = max_columns(count, world)
    return SlabLayout([("root", np.uint8, (im, 32)), ("decode_status", np.int32, (im,)),
                       ("out_len", np.int64, (im,))])


def assemble_fields(gathered, layout: SlabLayout, count: int, world: int):
    """Gathered slabs [world, size] -> {field: array over all ``count`` instances in order}."""
    g = np.asarray(gathered, dtype=np.uint8).reshape(world, layout.size)
    out = {}
    for name in layout.fields:
        parts = []
        for r in range(world):
            lo, hi = instance_range(count, world, r)
            parts.append(np.array(layout.view(g[r], name, hi - lo)))
        out[name] = np.concatenate(parts)
    return out
