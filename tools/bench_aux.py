"""Secondary measurements at SURVEY.md §8 configs C4 (Common Coin) and C5 (Broadcast) on one GPU.

    python tools/bench_aux.py [--steps 5]

Prints one JSON line per config.  Not the driver's bench line (bench.py measures the headline
N=256 decryption epoch); these put numbers and rooflines on the other two stacks.

C4: N=128 validators, 256 ABA instances (sessions {0,1} x proposers 0..127, agreement epoch 2);
    32,768 signature-share verifications (common_coin.rs:151) + 256 combine_signatures + master
    verifications + parities (:190, :196, :173).  1 in 64 shares replaced by another instance's
    share of the same signer (must verify false).
C5: N=128 (f=42), RS(k=44, m=84), 128 broadcast instances of a 1 MiB proposal each:
    encode (broadcast.rs:366) + Merkle roots (:381) + decode with the last 42 shards missing
    (reconstruct + rebuild + root check + glue, :660-707).  Output == input payload is checked.
    RS is reported as HBM GB/s (k L read + m L written per instance), Merkle as hashed GB/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def coin(ctx, steps):
    import torch  # noqa: F401  (device init through the binding)
    from hbbft_amd import netinfo

    n, inst = 128, 256
    sks, sk_shares, master_sk = netinfo.generate_keys(n)
    t = sks.threshold + 1
    pk = ctx.public_keys(sk_shares)
    master_pk = ctx.public_keys(master_sk)[0].tobytes()
    assert (ctx.set_pk_shares([r.tobytes() for r in pk]) == 0).all()
    inv_id = "[" + ", ".join(str(b) for b in master_pk) + "]"
    nonces = [f"Nonce for Honey Badger {inv_id}@{s}:2:{j}".encode() for s in (0, 1) for j in range(n)]
    ctx.prepare_nonces(nonces)
    sigs = ctx.sign(sk_shares)  # (inst, n, 96)
    rng = np.random.default_rng(0x68626278_00000005)
    corrupt = rng.integers(0, 64, size=(inst, n)) == 0
    bad = sigs.copy()
    ii = np.nonzero(corrupt)
    bad[ii[0], ii[1]] = sigs[(ii[0] + 1) % inst, ii[1]]
    times = {"prepare_nonces": [], "verify_sig_shares": [], "combine_signatures": []}
    ctx.set_timing(True)
    for _ in range(steps):
        t0 = time.perf_counter()
        ctx.prepare_nonces(nonces)
        t1 = time.perf_counter()
        valid = ctx.verify_sig_shares(bad)
        t2 = time.perf_counter()
        sig, st, ok, par = ctx.combine_signatures(master_pk, t)
        t3 = time.perf_counter()
        times["prepare_nonces"].append(t1 - t0)
        times["verify_sig_shares"].append(t2 - t1)
        times["combine_signatures"].append(t3 - t2)
    kern = {}
    for name in ("hash_nonces", "verify_sig", "combine_sigs"):
        ms_, cnt_ = ctx.kernel_time(name)
        kern[name] = round(ms_ / max(cnt_, 1), 3)
    k_ms, k_cnt = ctx.kernel_time("verify_sig")
    ctx.set_timing(False)
    assert (valid == ~corrupt).all(), "signature-share validity"
    assert (st == 0).all() and ok.all(), "combine / master verification"
    wall = {k: round(1e3 * float(np.mean(v)), 3) for k, v in times.items()}
    kms = k_ms / max(k_cnt, 1)
    return {"config": "C4 CommonCoin N=128 x 256 instances", "sig_share_verifies": inst * n,
            "verify_sig_kernel_ms": round(kms, 3), "sig_share_verifies_per_s_kernel": round(inst * n / (kms * 1e-3), 1),
            # tools/opcount: mixed Miller loop 9,631 + final exponentiation 7,657 Fq-mul per check,
            # 288 MAD each; peak 27.27 T MAD/s (tools/microbench/mad_rate.hip).  32,768 checks are
            # 512 waves: half the SIMDs at one wave each.
            "verify_sig_roofline": {"bound": "valu-int (v_mad_u64_u32)",
                                    "achieved_Tmad_s": round(inst * n * 17288 * 288 / (kms * 1e-3) / 1e12, 3),
                                    "peak_Tmad_s": 27.27,
                                    "frac": round(inst * n * 17288 * 288 / (kms * 1e-3) / 1e12 / 27.27, 4)},
            "coin_round_ms_wall": round(sum(wall.values()), 3), "wall_ms": wall, "kernel_ms": kern,
            "note": "host API (PCIe staging of 3.1 MB of shares included in wall times)"}


def broadcast(ctx, steps):
    import torch

    n, f = 128, 42
    k, m = n - 2 * f, 2 * f
    inst, plen = 128, 1 << 20
    L = (plen + 4 + k - 1) // k
    rng = np.random.default_rng(0x68626278_00000006)
    payload = rng.integers(0, 256, size=(inst, plen), dtype=np.uint8)
    frame = np.zeros((inst, k * L), dtype=np.uint8)
    frame[:, :4] = np.frombuffer(np.uint32(plen).byteswap().tobytes(), dtype=np.uint8)
    frame[:, 4:4 + plen] = payload
    host = np.zeros((inst, n, L), dtype=np.uint8)
    host[:, :k] = frame.reshape(inst, k, L)
    dev = torch.device("cuda", 0)
    shards = torch.from_numpy(host).to(dev)
    roots = torch.zeros((inst, 32), dtype=torch.uint8, device=dev)
    present = torch.ones((inst, n), dtype=torch.uint8, device=dev)
    present[:, n - f:] = 0
    out = torch.zeros((inst, k * L), dtype=torch.uint8, device=dev)
    out_len = torch.zeros(inst, dtype=torch.int64, device=dev)
    status = torch.zeros(inst, dtype=torch.int32, device=dev)
    work = torch.empty_like(shards)
    stream = torch.cuda.Stream(dev)  # events must be recorded on the stream the kernels run on
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    res = {"encode": [], "roots": [], "decode": []}
    ctx.set_timing(True)
    for s in range(steps + 1):
        if s == 1:
            ctx.set_timing(True)  # drop the warm-up step's kernel times
        ev[0].record(stream)
        ctx.rs_encode_d(shards, k, m, stream=sh)
        ev[1].record(stream)
        ctx.merkle_roots_d(shards, roots, stream=sh)
        ev[2].record(stream)
        work.copy_(shards)
        work[:, n - f:] = 0xA5  # erased shards
        ev[3].record(stream)
        ctx.broadcast_decode_d(work, present, roots, k, m, out, out_len, status, stream=sh)
        e4 = torch.cuda.Event(enable_timing=True)
        e4.record(stream)
        torch.cuda.synchronize()
        if s:
            res["encode"].append(ev[0].elapsed_time(ev[1]))
            res["roots"].append(ev[1].elapsed_time(ev[2]))
            res["decode"].append(ev[3].elapsed_time(e4))
    rs_ms, rs_cnt = ctx.kernel_time("rs_code")
    ml_ms, ml_cnt = ctx.kernel_time("merkle_leaves")
    ctx.set_timing(False)
    assert (status.cpu().numpy() == 0).all(), "decode status"
    assert (out_len.cpu().numpy() == plen).all()
    assert np.array_equal(out[:, :plen].cpu().numpy(), payload), "decoded payload"
    ms = {key: float(np.mean(v)) for key, v in res.items()}
    rs_bytes = inst * (k + m) * L
    leaf_bytes = inst * n * (L + 1)
    # per step: 1 encode launch (m rows) + 2 reconstruct launches (missing data rows, then missing
    # parity rows; here the last f shards are parity: 0 + f rows).
    enc_ms = ms["encode"]
    dwords = inst * (L // 4)
    # byte-permute kernel: per (output row, input row, dword) 3 v_perm_b32 + 1.5 xor (v_xor3)
    enc_valu = dwords * m * k * 4.5
    valu_peak = 256 * 4 * 16 * 2.4e9  # 32-bit lane-ops/s (256 CUs x 4 SIMD16 x 2.4 GHz)
    return {"config": "C5 Broadcast N=128 RS(44,84) x 128 instances of 1 MiB", "shard_len": L,
            "ms": {key: round(v, 3) for key, v in ms.items()},
            "rs_encode_hbm_GBps": round(rs_bytes / (enc_ms * 1e-3) / 1e9, 1),
            "rs_encode_valu_frac": round(enc_valu / (enc_ms * 1e-3) / valu_peak, 3),
            "rs_encode_valu_floor_ms": round(enc_valu / valu_peak * 1e3, 3),
            "rs_kernel_ms_per_launch": round(rs_ms / max(rs_cnt, 1), 4),
            "merkle_leaves_kernel_ms": round(ml_ms / max(ml_cnt, 1), 4),
            "merkle_hashed_GBps": round(leaf_bytes / (ms["roots"] * 1e-3) / 1e9, 1),
            "hbm_peak_GBps": 8000,
            "decode_note": "reconstruct 42 missing shards + rebuild tree + root check + glue per instance"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--only", default="", choices=["", "c4", "c5"])
    args = ap.parse_args()
    import torch

    torch.cuda.set_device(0)
    from hbbft_amd.hbx import Context

    with Context(0) as ctx:
        if args.only in ("", "c5"):
            print(json.dumps(broadcast(ctx, args.steps)), flush=True)
        if args.only in ("", "c4"):
            print(json.dumps(coin(ctx, args.steps)), flush=True)


if __name__ == "__main__":
    main()
