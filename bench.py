"""Benchmark: one HoneyBadger node-epoch of threshold-decryption crypto at N=256 on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 256] [--vlen 1024] [--no-cpu-baseline]

A *step* is the crypto of one HoneyBadger epoch as one node sees it (SURVEY.md §3 stack A,
BASELINE.json configs[2]): for every one of the N accepted proposals
  * ``Ciphertext::verify`` + the hoisted ``hash_g1_g2(U_j, V_j)``  (honey_badger.rs:371),
  * ``verify_decryption_share`` for all N senders                  (honey_badger.rs:229, :422-444),
  * ``PublicKeySet::decrypt`` with the first f+1 valid shares      (honey_badger.rs:340),
i.e. 65,536 share verifications + 256 ciphertext checks + 256 Lagrange combines (t = 86) + the
hash_bytes keystream XOR, through the C ABI of libhbx.so on device-resident inputs.

Multi-GPU (``torchrun``), two modes:
  * ``--scaling strong`` (default; BASELINE config 3): ONE N=256 epoch sharded by proposer column
    (rank g owns proposers [g P/G, (g+1) P/G) with their ciphertexts and share columns; keys are
    replicated); after the combine one RCCL all-gather assembles the per-share status bytes,
    ciphertext statuses and per-proposer combine statuses.  value = N^2 verifies / epoch time.
  * ``--scaling weak``: every rank runs one full node-epoch (G epochs in flight, as a node
    pipelining epochs or G co-hosted validators would); no collective on the data path.
    value = G x N^2 verifies / max-over-ranks time.

Inputs (synthetic, seeded): keys from ``hbbft_amd.netinfo.generate_keys``; 1 KiB random
contributions; U/V/W made by ``hbx_encrypt`` and shares by ``hbx_decrypt_shares`` on the GPU; 1 in
64 shares replaced by the same sender's share of a DIFFERENT ciphertext (the reference's
FaultyShareAdversary, tests/honey_badger.rs:99-106).  After the timed steps the validity matrix
must equal "not corrupted" and every plaintext must equal its contribution, or the bench fails.

Roofline: the dominant kernel is the share verification (k_verify_shares).  Its algorithmic work
is 15,057 Fq multiplications per share (tools/opcount: 2-pair Miller loop 7,400 + final
exponentiation 7,657; the 486 of the share's decode run in k_prepare_ct / k_decompress_shares) x 288 32-bit
multiply-adds each; its launch time is measured with HIP events recorded on the stream it runs on.  The bound is integer VALU (v_mad_u64_u32), not HBM
or MFMA; the peak is the measured chip rate from tools/microbench.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Algorithmic work per unit (tools/opcount/opcount.cpp)
FQMUL_PER_SHARE_VERIFY = 15057  # opcount: miller_loop2 7400 + final_exp 7657 (decode excluded)
MADS_PER_FQMUL = 288
# Chip peak of 32x32->64-bit integer multiply-add (v_mad_u64_u32), measured by
# tools/microbench/mad_rate.hip on MI355X (profiles/r01_mad_rate.txt): tera-MAD/s.
PEAK_TMAD_S = float(os.environ.get("HBX_PEAK_TMAD_S", "27.27"))
# HBM traffic of one k_verify_shares launch at N=256 (all 256 proposers on one GPU), from
# rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes (tools/gpu_round.sh PMC=1,
# profiles/r02m_pmc_hbm.txt, the digit-tower kernel with the h_eff-scaled keys): 5.048e6 KB +
# 8.592e6 KB per launch.  The accesses are the kernel's scratch
# traffic (95 spilled VGPRs in the Miller loop, Fq12 operands of the out-of-line Fq12 products of
# the final exponentiation), a width the guide leaves uncalibrated, so the raw counter bytes are
# reported without the x2 streaming-read correction.  Algorithmic bytes per launch are ~12 MB
# (shares 48 B + pk + 30 KB of digit-form lines per proposer + 1 B out): the kernel is VALU-bound
# and the traffic (~0.56 TB/s) is not its bound.
TRAFFIC_N256_BYTES = (5.069e6 + 8.579e6) * 1024
TRAFFIC_SOURCE = "profiles/r02y_pmc_hbm.txt (PMC FETCH_SIZE+WRITE_SIZE, digit-tower kernel)"
# The benchmarked node is validator 0: its own decryption shares are computed locally
# (hbx_set_own_share), and its own share's check doubles as Ciphertext::verify.
OWN_INDEX = 0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=256, help="validators N (shares per ciphertext)")
    ap.add_argument("--vlen", type=int, default=1024, help="contribution bytes per proposer")
    ap.add_argument("--corrupt-every", type=int, default=64)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-own-share", action="store_true",
                    help="run Ciphertext::verify as separate checks instead of through the node's own share")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--verify-lanes", type=int, default=0, choices=(0, 1, 3),
                    help="lanes per decryption-share check (0: auto by occupancy)")
    ap.add_argument("--in-flight", type=int, default=2,
                    help="also time this many consecutive epochs in flight at once (one context and stream "
                         "each, as HoneyBadger's max_future_epochs allows); reported beside the headline")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="single-GPU rehearsal of strong scaling: run only rank 0's proposer slice of a G-way "
                         "sharded epoch (the per-GPU work of --scaling strong at --gpus G, minus the all-gather)")
    return ap.parse_args()


def make_epoch(ctx, n: int, lo: int, hi: int, vlen: int, corrupt_every: int):
    """Synthetic inputs of proposers [lo, hi) of one epoch, built on the GPU (hbx producer API)."""
    from hbbft_amd import netinfo

    sks, sk_shares, master_sk = netinfo.generate_keys(n)
    pk_shares = ctx.public_keys(sk_shares)
    master_pk = ctx.public_keys(master_sk)[0].tobytes()
    rng = np.random.default_rng(0x68626278_00000002)
    msgs_all = [rng.integers(0, 256, size=vlen, dtype=np.uint8).tobytes() for _ in range(n)]
    r_all = netinfo.scalars_to_be32(netinfo.random_scalars(np.random.default_rng(0x68626278_00000003), n + 1))
    pj = hi - lo
    # own proposers plus one foreign ciphertext (index n) whose shares serve as corruptions
    idx = list(range(lo, hi)) + [n]
    foreign_msg = b"foreign ciphertext"
    msgs = [msgs_all[j] for j in range(lo, hi)] + [foreign_msg]
    cts = ctx.encrypt(master_pk, msgs, r_all[idx])
    u48 = np.stack([np.frombuffer(c[0], dtype=np.uint8) for c in cts])
    shares = ctx.decrypt_shares(sk_shares, u48)  # (pj + 1, n, 48)
    crng = np.random.default_rng(0x68626278_00000004)
    corrupt = crng.integers(0, corrupt_every, size=(n, n)) == 0  # global (proposer, sender) pattern
    corrupt[:, OWN_INDEX] = False  # this node's own share is computed locally, never received
    corrupt = corrupt[lo:hi]
    sh = shares[:pj].copy()
    ii = np.nonzero(corrupt)
    sh[ii[0], ii[1]] = shares[pj, ii[1]]
    return dict(pk_shares=pk_shares, cts=cts[:pj], msgs=msgs[:pj], shares=sh, corrupt=corrupt, t=sks.threshold + 1,
                own_sk=sk_shares[OWN_INDEX].tobytes())


def host_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "nproc": os.cpu_count()}


def cpu_baseline(ep, seconds: float, threads: int):
    """CPU baseline ("port", tools/cpu_baseline/cpu_port.cpp, g++ -O3), both rows of BASELINE.md §2
    on `threads` std::threads over a bounded sample of this workload's shares, each checked against
    the expected bits:
      (a) reference shape (honey_badger.rs:229 as threshold_crypto runs it): hash_g1_g2 recomputed
          per share with pairing 0.14's 507-bit cofactor multiplication, two full pairings with
          separate final exponentiations;
      (b) hoisted + fused: hash_g1_g2 and the Miller lines of H_j, W_j once per proposer, then one
          two-pair Miller loop and ONE final exponentiation per share.
    `value` is row (b), the faster CPU formulation."""
    import ctypes

    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libcpu_port.so"))
    P = ctypes.c_void_p
    lib.cpu_verify_dec_shares.argtypes = [P, ctypes.c_uint32, P, P, P, P, P, P, ctypes.c_uint32, ctypes.c_int, P]
    lib.cpu_verify_dec_shares_fused.argtypes = [P, ctypes.c_uint32, P, P, P, P, P, ctypes.c_uint32, P,
                                                ctypes.c_uint32, ctypes.c_int, P]
    cts = ep["cts"]
    n = len(ep["pk_shares"])
    p = len(cts)
    pk = np.ascontiguousarray(ep["pk_shares"], dtype=np.uint8)
    u = np.stack([np.frombuffer(c[0], dtype=np.uint8) for c in cts])
    w = np.stack([np.frombuffer(c[2], dtype=np.uint8) for c in cts])
    off = np.zeros(p + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(c[1]) for c in cts])
    v = np.frombuffer(b"".join(c[1] for c in cts), dtype=np.uint8).copy()
    sh = np.ascontiguousarray(ep["shares"], dtype=np.uint8)

    def run(njobs, nthreads, start, fused, nprop=None):
        k = np.arange(start, start + njobs, dtype=np.uint64)
        pp = p if nprop is None else nprop
        jobs = np.stack([(k * 7919) % pp, (k * 104729 + 3) % n], axis=1).astype(np.uint32)
        out = np.zeros(njobs, dtype=np.uint8)
        t0 = time.perf_counter()
        if fused:
            lib.cpu_verify_dec_shares_fused(pk.ctypes.data, n, u.ctypes.data, v.ctypes.data, off.ctypes.data,
                                            w.ctypes.data, sh.ctypes.data, p, jobs.ctypes.data, njobs, nthreads,
                                            out.ctypes.data)
        else:
            lib.cpu_verify_dec_shares(pk.ctypes.data, n, u.ctypes.data, v.ctypes.data, off.ctypes.data,
                                      w.ctypes.data, sh.ctypes.data, jobs.ctypes.data, njobs, nthreads, out.ctypes.data)
        dt = time.perf_counter() - t0
        expect = ~ep["corrupt"][jobs[:, 0], jobs[:, 1]]
        assert (out.astype(bool) == expect).all(), "CPU port disagrees with the expected validity"
        return dt

    # (a) reference shape
    t1 = run(2, 1, 0, False) / 2
    na = max(threads, int(seconds / 2 * threads / t1))
    da = run(na, threads, 2, False)
    # (b) hoisted + fused: a sample of whole proposer columns (the per-proposer preparation is part
    # of the work and amortises over its n shares, as it does in an epoch)
    tb1 = run(n, 1, 0, True, nprop=1) / n
    cols = max(1, min(p, int(seconds / 2 * threads / (tb1 * n))))
    nb = cols * n
    kk = np.arange(nb, dtype=np.uint64)
    jobs = np.stack([kk // n, kk % n], axis=1).astype(np.uint32)
    out = np.zeros(nb, dtype=np.uint8)
    t0 = time.perf_counter()
    lib.cpu_verify_dec_shares_fused(pk.ctypes.data, n, u.ctypes.data, v.ctypes.data, off.ctypes.data, w.ctypes.data,
                                    sh.ctypes.data, p, jobs.ctypes.data, nb, threads, out.ctypes.data)
    db = time.perf_counter() - t0
    assert (out.astype(bool) == ~ep["corrupt"][jobs[:, 0], jobs[:, 1]]).all(), "fused CPU port disagrees"
    host = host_info()
    return dict(value=round(nb / db, 1), unit="share verifies/s", cores=threads, kind="port",
                host=host,
                rows={"a_reference_shape": {"value": round(na / da, 1), "single_thread": round(1.0 / t1, 2),
                                            "sample": f"{na} shares in {da:.1f} s"},
                      "b_hoisted_fused": {"value": round(nb / db, 1), "single_thread": round(1.0 / tb1, 2),
                                          "sample": f"{cols} proposer columns x {n} shares in {db:.1f} s"}},
                sample=f"tools/cpu_baseline/cpu_port.cpp (g++ -O3, {threads} std::threads on {host['model']}, "
                       f"nproc {host['nproc']}): (b) hash_g1_g2 + lines hoisted per proposer, one 2-pair Miller "
                       f"loop + one final exponentiation per share, {cols} whole proposer columns of the N={n} "
                       f"epoch in {db:.1f} s; (a) the reference's per-share shape {na / da:.0f}/s; a restatement, "
                       f"not the reference binary (no Rust toolchain)")


def in_flight(args, ep, dev, torch, Context, inputs, pj, maxv, n, t, off, verifies):
    """Throughput with `args.in_flight` consecutive epochs overlapping: epoch k on context k mod F
    (own buffers and stream), issued back to back, so one epoch's latency-bound stages (hash-to-G2,
    lines, combine) run beside another's share checks.  The headline `value` stays one epoch at a
    time; this is the node's rate when future-epoch messages are already queued."""
    F = args.in_flight
    d_u, d_v, d_off, d_w, d_shares = inputs
    lanes = []
    for _ in range(F):
        c = Context(dev.index or 0)
        c.set_verify_lanes(args.verify_lanes)
        assert (c.set_pk_shares([row.tobytes() for row in ep["pk_shares"]]) == 0).all()
        if not args.no_own_share:
            c.set_own_share(OWN_INDEX, ep["own_sk"])
        st = torch.cuda.Stream(dev)
        outs = (torch.zeros(int(off[-1]), dtype=torch.uint8, device=dev), torch.zeros(pj * n, dtype=torch.uint8, device=dev),
                torch.zeros(pj, dtype=torch.uint8, device=dev), torch.zeros(pj, dtype=torch.int32, device=dev))
        lanes.append((c, st, outs))
    torch.cuda.synchronize(dev)

    def issue(k):
        c, st, (o, v, cv, stt) = lanes[k % F]
        c.decrypt_epoch_d(d_u, d_v, d_off, d_w, pj, maxv, d_shares, n, t, o, d_valid=v, d_ct_valid=cv, d_status=stt,
                          stream=st.cuda_stream)

    for k in range(F):
        issue(k)
    torch.cuda.synchronize(dev)
    epochs = F * max(args.steps, 2)
    t0 = time.perf_counter()
    for k in range(epochs):
        issue(k)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    for c, _, (o, v, cv, stt) in lanes:
        assert (stt.cpu().numpy() == 0).all() and (cv.cpu().numpy() == 1).all(), "in-flight epoch status"
        assert ((v.cpu().numpy().reshape(pj, n) == 1) == ~ep["corrupt"]).all(), "in-flight validity"
        out = o.cpu().numpy()
        assert all(out[off[j]:off[j + 1]].tobytes() == ep["msgs"][j] for j in range(pj)), "in-flight plaintexts"
        c.close()
    return {"epochs": epochs, "in_flight": F, "ms_per_epoch": round(elapsed / epochs * 1e3, 3),
            "value": round(verifies * epochs / elapsed, 1), "unit": "share verifies/s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from hbbft_amd import shard
    from hbbft_amd.hbx import Context

    n = args.n
    strong = args.scaling == "strong" and world > 1
    if strong:
        lo, hi = shard.proposer_range(n, world, rank)
    elif args.shard_of > 1 and world == 1:
        lo, hi = shard.proposer_range(n, args.shard_of, 0)
    else:
        lo, hi = 0, n
    pj = hi - lo
    ctx = Context(local)
    ctx.set_verify_lanes(args.verify_lanes)
    ep = make_epoch(ctx, n, lo, hi, args.vlen, args.corrupt_every)
    st = ctx.set_pk_shares([row.tobytes() for row in ep["pk_shares"]])
    assert (st == 0).all()
    if not args.no_own_share:
        ctx.set_own_share(OWN_INDEX, ep["own_sk"])

    # a dedicated stream for the epoch calls; the HIP events that time the epoch and the kernels are
    # recorded on the stream the kernels run on
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    assert sh != 0
    cts = ep["cts"]
    d_u = torch.from_numpy(np.stack([np.frombuffer(c[0], dtype=np.uint8) for c in cts])).to(dev)
    d_w = torch.from_numpy(np.stack([np.frombuffer(c[2], dtype=np.uint8) for c in cts])).to(dev)
    off = np.zeros(pj + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(c[1]) for c in cts])
    d_off = torch.from_numpy(off).to(dev)
    d_v = torch.from_numpy(np.frombuffer(b"".join(c[1] for c in cts), dtype=np.uint8).copy()).to(dev)
    d_shares = torch.from_numpy(ep["shares"]).to(dev)
    d_out = torch.zeros(int(off[-1]), dtype=torch.uint8, device=dev)
    # result slab gathered across ranks: [share status pj*n | ct status pj | combine status pj*4],
    # laid out for the largest column block so every rank's slab has the same size
    lay = shard.slab_layout(n, shard.max_columns(n, world) if strong else pj)
    slab = torch.zeros(lay["size"], dtype=torch.uint8, device=dev)
    d_valid = slab[lay["valid"][0]:lay["valid"][0] + pj * n]
    d_ct_valid = slab[lay["ct_valid"][0]:lay["ct_valid"][0] + pj]
    d_status = slab[lay["status"][0]:lay["status"][0] + 4 * pj].view(torch.int32)
    gathered = [None]
    t = ep["t"]
    maxv = int(np.max(np.diff(off)))

    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]

    def step(events=None):
        if events:
            events[0].record(stream)
        # one call per node-epoch (hbx_decrypt_epoch_d): hash_g1_g2 + lines, share checks (the
        # node's own share check is Ciphertext::verify), combine + decrypt
        ctx.decrypt_epoch_d(d_u, d_v, d_off, d_w, pj, maxv, d_shares, n, t, d_out, d_valid=d_valid,
                            d_ct_valid=d_ct_valid, d_status=d_status, stream=sh)
        if events:
            events[1].record(stream)
        if strong:
            gathered[0] = shard.all_gather_slabs(slab, world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(ev[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # correctness of the last step (size-independent properties)
    valid = d_valid.cpu().numpy().reshape(pj, n).astype(bool)
    expect = ~ep["corrupt"]
    assert (d_ct_valid.cpu().numpy() == 1).all(), "a valid ciphertext failed Ciphertext::verify"
    assert (valid == expect).all(), f"validity mismatch at {int((valid != expect).sum())} positions"
    assert (d_status.cpu().numpy() == 0).all(), "combine status"
    out = d_out.cpu().numpy()
    for j in range(pj):
        assert out[off[j]:off[j + 1]].tobytes() == ep["msgs"][j], f"plaintext {lo + j} differs"
    if strong:
        gv, gct, gst = shard.assemble(gathered[0].cpu().numpy(), n, world)
        full = np.random.default_rng(0x68626278_00000004).integers(0, args.corrupt_every, size=(n, n)) == 0
        full[:, OWN_INDEX] = False
        assert ((gv == 1) == ~full).all() and (gct == 1).all() and (gst == 0).all(), "gathered epoch result"

    ms_epoch_ev = np.mean([ev[k][0].elapsed_time(ev[k][1]) for k in range(args.steps)])
    ms_step = elapsed / args.steps * 1e3
    verifies = n * n * (1 if strong else world) if args.shard_of <= 1 else pj * n
    value = verifies * args.steps / elapsed
    shares_here = pj * n
    kern = {}
    for name in ("prepare_ct", "prepare_lines", "ct_checks", "verify_shares", "combine"):
        tot, cnt = ctx.kernel_time(name)
        kern[name] = round(tot / max(cnt, 1), 3)
    ctx.set_timing(False)
    # average launch duration of the dominant kernel, HIP events on its own stream
    ms_kernel = kern["verify_shares"]
    achieved = shares_here * FQMUL_PER_SHARE_VERIFY * MADS_PER_FQMUL / (ms_kernel * 1e-3) / 1e12
    res = {
        "metric": "BLS12-381 share verifies/sec (node) at N=256; crypto ms per HB epoch",
        "value": round(value, 1),
        "unit": "share verifies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "i32 (Fq as 14 signed 28-bit digits, R = 2^392, in the share check; 12 x u32 limbs elsewhere)",
        "data": "synthetic (seeded keys, 1 KiB random contributions, GPU-made ciphertexts/shares, 1/64 foreign-ciphertext shares)",
        "config": {"workload": f"HoneyBadger node-epoch N={n}: {n * n} decryption-share verifies + {n} Ciphertext::verify + "
                               f"{n} combines (t={t}) + decrypt, |v|={args.vlen} B"
                               + ("" if strong or world == 1 else f"; {world} epochs in flight, one per GPU"),
                   "n": n, "t": t, "proposers_per_gpu": pj,
                   "parallelism": (f"proposer-column x{world}" if strong else
                                   f"rehearsal: rank 0 slice of proposer-column x{args.shard_of}" if args.shard_of > 1
                                   else f"epoch-per-gpu x{world}")},
        "epoch_ms_hip_events": round(float(ms_epoch_ev), 3),
        "kernels_ms": kern,
        "roofline": {"bound": "valu-int (v_mad_u64_u32)", "achieved": round(achieved, 3), "peak": PEAK_TMAD_S,
                     "unit": "Tmad/s", "frac": round(achieved / PEAK_TMAD_S, 4),
                     "traffic": TRAFFIC_N256_BYTES if (n == 256 and pj == 256) else None,
                     "traffic_note": "bytes/launch from " + TRAFFIC_SOURCE + " (scratch at Fq12 calls); algorithmic ~1e7",
                     "kernel": "k_verify_shares", "kernel_ms": ms_kernel,
                     "work": f"{shares_here} shares x {FQMUL_PER_SHARE_VERIFY} Fq-mul x {MADS_PER_FQMUL} MAD"},
        "check": "validity bitmap == not-corrupted; plaintexts == contributions",
    }
    if world == 1 and args.in_flight > 1:
        res["epochs_in_flight"] = in_flight(args, ep, dev, torch, Context, (d_u, d_v, d_off, d_w, d_shares), pj, maxv,
                                            n, t, off, verifies)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(ep, args.cpu_seconds, min(16, os.cpu_count() or 1))
    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
