"""Benchmark: one HoneyBadger node-epoch of threshold-decryption crypto at N=256 on MI355X, plus the
other BASELINE.json configs as sub-objects of the same JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 256] [--vlen 1024] [--no-cpu-baseline]
                    [--configs C1,C2,C4,C5]

A *step* is the crypto of one HoneyBadger epoch as one node sees it (SURVEY.md §3 stack A,
BASELINE.json configs[2]): for every one of the N accepted proposals
  * ``Ciphertext::verify`` + the hoisted ``hash_g1_g2(U_j, V_j)``  (honey_badger.rs:371),
  * ``verify_decryption_share`` for all N senders                  (honey_badger.rs:229, :422-444),
  * ``PublicKeySet::decrypt`` with the first f+1 valid shares      (honey_badger.rs:340),
i.e. 65,536 share verifications + 256 ciphertext checks + 256 Lagrange combines (t = 86) + the
hash_bytes keystream XOR, through the C ABI of libhbx.so on device-resident inputs.

``configs`` (single GPU, rank 0 only): C1 (the N=10 node-epoch of the simulation example, BASELINE
config 0, in ms), C2 (an N=64 epoch, BASELINE config 1), C4 (Common Coin,
256 instances at N=128, config 3) and C5 (Broadcast, 128 x 1 MiB proposals at N=128, both Merkle
digests, config 4), each with its own value, roofline and CPU baseline.

Multi-GPU (``torchrun``), two modes:
  * ``--scaling strong`` (default; BASELINE config 3): ONE N=256 epoch sharded by proposer column
    (rank g owns proposers [g P/G, (g+1) P/G) with their ciphertexts and share columns; keys are
    replicated); after the combine one RCCL all-gather assembles the per-share status bytes,
    ciphertext statuses, per-proposer combine statuses and the plaintexts.  value = N^2 verifies / epoch time.
  * ``--scaling weak``: every rank runs one full node-epoch (G epochs in flight, as a node
    pipelining epochs or G co-hosted validators would); no collective on the data path.
    value = G x N^2 verifies / max-over-ranks time.

Inputs (synthetic, seeded): keys from ``hbbft_amd.netinfo.generate_keys``; 1 KiB random
contributions; U/V/W made by ``hbx_encrypt`` and shares by ``hbx_decrypt_shares`` on the GPU; 1 in
64 shares replaced by the same sender's share of a DIFFERENT ciphertext (the reference's
FaultyShareAdversary, tests/honey_badger.rs:99-106).  After the timed steps the validity matrix
must equal "not corrupted" and every plaintext must equal its contribution, or the bench fails.

Roofline: the dominant kernel is the share verification (k_verify_shares / k_verify_shares2).  Its
algorithmic work is FROZEN at SURVEY.md §8(d)'s unit V_dec = 16,500 Fq multiplications per share
(2 precomputed-line Miller loops + 1 cyclotomic final exponentiation + 1 inversion) x 288 32-bit
multiply-adds each; the current code's own count (tools/opcount) is reported beside it.  Its launch
time is measured with HIP events recorded on the stream it runs on.  The bound is integer VALU
(v_mad_u64_u32), not HBM or MFMA; the peak is the measured chip rate.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Frozen algorithmic work units (DESIGN.md §4 "Work units")
VDEC_FQMUL = 16500     # one decryption-share verify
VSIG_FQMUL = 20000     # one coin signature-share verify (sigma's lines generated in the loop)
G1_MUL_FQMUL = 4100    # one G1 double-and-add scalar multiplication (C_t = t x 4.1k)
MADS_PER_FQMUL = 288   # 2 x 12^2 (32-bit schoolbook Montgomery product)
# Current code's own count (tools/opcount/opcount.cpp over the kernels' code), reported beside
OPCOUNT_VDEC = 15057   # two-pair Miller loop 7,400 + final exponentiation 7,657
OPCOUNT_VSIG = 17288   # mixed Miller loop 9,631 + final exponentiation 7,657
# Chip peak of 32x32->64-bit integer multiply-add (v_mad_u64_u32), measured by
# tools/microbench/mad_rate.hip on MI355X (profiles/r01_mad_rate.txt): tera-MAD/s.
PEAK_TMAD_S = float(os.environ.get("HBX_PEAK_TMAD_S", "27.27"))
# 32-bit VALU lane-op peak (256 CUs x 4 SIMD x 16 lanes x 2.4 GHz) for the byte kernels
PEAK_VALU_OPS = 256 * 4 * 16 * 2.4e9
HBM_PEAK_GBPS = 8000.0
# HBM traffic of one share-check launch at N=256, from a PMC pass (rocprofv3 --pmc FETCH_SIZE and
# WRITE_SIZE in separate passes, tools/gpu_final.sh via tools/gpu_prof.sh): the newest profiles/*_pmc_hbm.json
# carries the kernel, the bytes per launch and the commit the pass was taken at.
OWN_INDEX = 0  # the benchmarked node is validator 0 (own share computed locally, hbx_set_own_share)


def parse(argv=None):
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
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget per config")
    ap.add_argument("--verify-lanes", type=int, default=0, choices=(0, 1, 2, 3, 6, 7),
                    help="lanes per decryption-share check (0: auto by occupancy)")
    ap.add_argument("--combine-lanes", type=int, default=0, choices=(0, 1, 4),
                    help="lanes per Lagrange term in the combine (0: auto by occupancy)")
    ap.add_argument("--in-flight", type=int, default=2,
                    help="also time this many consecutive epochs in flight at once (one context and stream "
                         "each, as HoneyBadger's max_future_epochs allows); reported beside the headline")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="single-GPU rehearsal of strong scaling: run only rank 0's proposer slice of a G-way "
                         "sharded epoch (the per-GPU work of --scaling strong at --gpus G, minus the all-gather)")
    ap.add_argument("--strong-at-1", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-node-rate", dest="node_rate", action="store_false",
                    help="at --gpus G > 1 (strong), skip the weak sub-object (G whole epochs in flight)")  # tests: the strong-mode slab path at world 1
    ap.add_argument("--configs", default="C1,C2,C4,C5",
                    help="secondary BASELINE configs in the same line ('' for none); at --gpus > 1 (strong) C4 "
                         "and C5 run sharded by instance")
    return ap.parse_args(argv)


def parse_args_for_test(argv):
    return parse(argv)


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
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    return {"model": model, "nproc": os.cpu_count(), "affinity": usable}


def all_cores() -> int:
    """Row (b) threads: every host core, os.cpu_count()."""
    return max(1, os.cpu_count() or 1)


def usable_cores() -> int:
    """CPUs this process may actually run on at once: the cgroup quota when there is one, else the
    affinity mask (the `cores` every cpu_baseline reports)."""
    qc = quota_cores()
    if qc:
        return qc
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return all_cores()


def quota_cores():
    """CPUs the process may actually run on at once: the cgroup v2 cpu.max quota (the GPU box
    grants a share of the machine), or None when there is no quota below os.cpu_count()."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
        if q == "max":
            return None
        c = max(1, int(int(q) / int(period)))
        return c if c < all_cores() else None
    except (OSError, ValueError):
        return None


def hbx_build_info():
    """Provenance of the loaded libhbx.so (hbbft_amd/hbx.py build_info: compiled-in source hash vs
    the tree's)."""
    from hbbft_amd import hbx

    return hbx.build_info()


def traffic_record(kind="hbm"):
    """Newest PMC record for the share check (profiles/*_pmc_hbm.json) or the coin's two-lane
    signature-share check (kind "coin": profiles/*_pmc_coin.json), or None."""
    import glob

    recs = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{kind}.json")))
    if not recs:
        return None
    with open(recs[-1]) as fh:
        rec = json.load(fh)
    rec["source"] = os.path.relpath(recs[-1], ROOT)
    return rec


def c5_traffic():
    """Newest PMC records of the C5 kernels (profiles/*_pmc_c5.jsonl): {kernel: record}."""
    import glob

    recs = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_c5.jsonl")))
    if not recs:
        return {}
    out = {}
    with open(recs[-1]) as fh:
        for line in fh:
            if line.strip():
                r = json.loads(line)
                r["source"] = os.path.relpath(recs[-1], ROOT)
                out[r["kernel"]] = r
    return out


def cpu_lib():
    import ctypes

    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libcpu_port.so"))
    P, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.cpu_verify_dec_shares.argtypes = [P, u32, P, P, P, P, P, P, u32, i32, P]
    lib.cpu_verify_dec_shares_fused.argtypes = [P, u32, P, P, P, P, P, u32, P, u32, i32, P]
    lib.cpu_verify_sig_shares.argtypes = [P, u32, P, P, u32, P, P, u32, i32, i32, P]
    lib.cpu_combine_sigs.argtypes = [P, P, u32, u32, u32, P, P, P, i32, P, P]
    lib.cpu_rs_encode.argtypes = [P, u32, u32, u32, u32, i32]
    lib.cpu_rs_reconstruct.argtypes = [P, P, u32, u32, u32, u32, i32, P]
    lib.cpu_combine_decrypt.argtypes = [P, P, u32, u32, u32, P, P, i32, P, P]
    return lib


# ----------------------------------------------------------------------------------------------
# Stack A: HoneyBadger threshold decryption (C2, C3)
# ----------------------------------------------------------------------------------------------
def epoch_contributions(n: int, vlen: int):
    """The N contributions of the synthetic epoch (seeded; every rank can regenerate them)."""
    rng = np.random.default_rng(0x68626278_00000002)
    return [rng.integers(0, 256, size=vlen, dtype=np.uint8).tobytes() for _ in range(n)]


def make_epoch(ctx, n: int, lo: int, hi: int, vlen: int, corrupt_every: int):
    """Synthetic inputs of proposers [lo, hi) of one epoch, built on the GPU (hbx producer API)."""
    from hbbft_amd import netinfo

    sks, sk_shares, master_sk = netinfo.generate_keys(n)
    pk_shares = ctx.public_keys(sk_shares)
    master_pk = ctx.public_keys(master_sk)[0].tobytes()
    msgs_all = epoch_contributions(n, vlen)
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
                own_sk=sk_shares[OWN_INDEX].tobytes(), master_pk=master_pk)


def cpu_baseline_dec(ep, seconds: float):
    """CPU baseline ("port", tools/cpu_baseline/cpu_port.cpp, g++ -O3) of the decryption-share
    checks, both rows of BASELINE.md §2 over a bounded sample of this workload's shares, each
    checked against the expected bits:
      (a) 1 thread, the reference's shape (honey_badger.rs:229 as threshold_crypto runs it):
          hash_g1_g2 recomputed per share with pairing 0.14's 507-bit cofactor multiplication, two
          full pairings with separate final exponentiations;
      (b) all host cores (os.cpu_count() std::threads), hoisted + fused: hash_g1_g2 and the Miller
          lines of H_j, W_j once per proposer, then one two-pair Miller loop and ONE final
          exponentiation per share.
    `value` is row (b)."""
    lib = cpu_lib()
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
    threads = all_cores()

    def run(jobs, nthreads, fused):
        out = np.zeros(len(jobs), dtype=np.uint8)
        t0 = time.perf_counter()
        if fused:
            lib.cpu_verify_dec_shares_fused(pk.ctypes.data, n, u.ctypes.data, v.ctypes.data, off.ctypes.data,
                                            w.ctypes.data, sh.ctypes.data, p, jobs.ctypes.data, len(jobs), nthreads,
                                            out.ctypes.data)
        else:
            lib.cpu_verify_dec_shares(pk.ctypes.data, n, u.ctypes.data, v.ctypes.data, off.ctypes.data,
                                      w.ctypes.data, sh.ctypes.data, jobs.ctypes.data, len(jobs), nthreads,
                                      out.ctypes.data)
        dt = time.perf_counter() - t0
        assert (out.astype(bool) == ~ep["corrupt"][jobs[:, 0], jobs[:, 1]]).all(), "CPU port disagrees"
        return dt

    def scattered(count, start):
        k = np.arange(start, start + count, dtype=np.uint64)
        return np.stack([(k * 7919) % p, (k * 104729 + 3) % n], axis=1).astype(np.uint32)

    # (a) reference shape, one thread
    t1 = run(scattered(2, 0), 1, False) / 2
    na = max(2, int(seconds / 2 / t1))
    da = run(scattered(na, 2), 1, False)
    # (b) hoisted + fused, all cores, whole proposer columns (the per-proposer preparation is part
    # of the work and amortises over its n shares, as it does in an epoch)
    col = np.stack([np.zeros(n, np.uint64), np.arange(n, dtype=np.uint64)], axis=1).astype(np.uint32)
    tb1 = run(col, 1, True) / n
    cols = max(1, min(p, int(seconds / 2 * min(threads, 64) / (tb1 * n))))
    kk = np.arange(cols * n, dtype=np.uint64)
    jobs = np.stack([kk // n, kk % n], axis=1).astype(np.uint32)
    db = run(jobs, threads, True)
    host = host_info()
    rows = {"a_reference_shape_1thread": {"value": round(na / da, 1), "cores": 1,
                                          "sample": f"{na} shares in {da:.1f} s"},
            "b_hoisted_fused_all_cores": {"value": round(len(jobs) / db, 1), "cores": threads,
                                          "single_thread": round(1.0 / tb1, 2),
                                          "sample": f"{cols} proposer columns x {n} shares in {db:.1f} s"}}
    qc = quota_cores()
    if qc:  # the same sample on as many threads as the cgroup quota lets run at once
        dq = run(jobs, qc, True)
        rows["b_hoisted_fused_quota_cores"] = {"value": round(len(jobs) / dq, 1), "cores": qc,
                                               "sample": f"same sample in {dq:.1f} s; cgroup cpu.max allows {qc} CPUs"}
    # value = the row on the CPUs the process may use (the quota row when the box sets one): an
    # oversubscribed all-cores row can be timed but does not say what those CPUs sustain
    best = "b_hoisted_fused_quota_cores" if qc else "b_hoisted_fused_all_cores"
    # PublicKeySet::decrypt (honey_badger.rs:340) of a sample of proposers on the best row's threads:
    # Lagrange combine of the first t valid shares + hash_bytes keystream XOR, checked against the
    # contributions; the epoch row adds the share checks of the whole epoch at the best rate
    bt = rows[best]["cores"]
    pc = max(1, min(p, 2 * bt))
    valid = np.ascontiguousarray(~ep["corrupt"], dtype=np.uint8)
    outp = np.zeros_like(v)
    stc = np.zeros(p, dtype=np.int32)
    t0 = time.perf_counter()
    lib.cpu_combine_decrypt(sh.ctypes.data, valid.ctypes.data, n, pc, ep["t"], v.ctypes.data, off.ctypes.data, bt,
                            outp.ctypes.data, stc.ctypes.data)
    dc = time.perf_counter() - t0
    assert (stc[:pc] == 0).all() and all(outp[off[j]:off[j + 1]].tobytes() == ep["msgs"][j] for j in range(pc)), \
        "CPU combine / decrypt"
    comb_ms = dc / pc * p * 1e3
    rows["c_combine_decrypt"] = {"ms_per_epoch": round(comb_ms, 1), "cores": bt, "t": int(ep["t"]),
                                 "sample": f"{pc} proposers in {dc:.2f} s, scaled to {p}"}
    rows["epoch_verify_plus_combine"] = {"ms_per_epoch": round(p * n / rows[best]["value"] * 1e3 + comb_ms, 1),
                                         "cores": bt, "note": f"{p * n} checks at row {best} + row c_combine_decrypt"}
    return dict(value=rows[best]["value"], unit="share verifies/s", cores=rows[best]["cores"], kind="port",
                host=host, best_row=best, cgroup_cpus=qc,
                rows=rows,
                sample=f"tools/cpu_baseline/cpu_port.cpp (g++ -O3) on {host['model']} (nproc {host['nproc']}, "
                       f"affinity {host['affinity']}, cgroup quota {qc or 'none'} CPUs): value = row {best}; (b) "
                       f"hash_g1_g2 + lines hoisted per proposer, one 2-pair Miller loop + one final exponentiation "
                       f"per share, {cols} whole proposer columns of the N={n} epoch; (a) 1 thread, the reference's "
                       f"per-share shape, {na} shares; a restatement, not the reference binary (no Rust toolchain)")


class EpochBench:
    """One node-epoch (or a proposer slice of one) on device-resident inputs, timed per step."""

    def __init__(self, ctx, ep, dev, stream, torch, verify_lanes, own: bool, combine_lanes: int = 0):
        self.ctx, self.ep, self.dev, self.stream, self.torch = ctx, ep, dev, stream, torch
        ctx.set_verify_lanes(verify_lanes)
        ctx.set_combine_lanes(combine_lanes)
        assert (ctx.set_pk_shares([row.tobytes() for row in ep["pk_shares"]]) == 0).all()
        if own:
            ctx.set_own_share(OWN_INDEX, ep["own_sk"])
        cts = ep["cts"]
        self.n = len(ep["pk_shares"])
        self.pj = len(cts)
        self.t = ep["t"]
        self.d_u = torch.from_numpy(np.stack([np.frombuffer(c[0], dtype=np.uint8) for c in cts])).to(dev)
        self.d_w = torch.from_numpy(np.stack([np.frombuffer(c[2], dtype=np.uint8) for c in cts])).to(dev)
        off = np.zeros(self.pj + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(c[1]) for c in cts])
        self.off = off
        self.d_off = torch.from_numpy(off).to(dev)
        self.d_v = torch.from_numpy(np.frombuffer(b"".join(c[1] for c in cts), dtype=np.uint8).copy()).to(dev)
        self.d_shares = torch.from_numpy(ep["shares"]).to(dev)
        self.d_out = torch.zeros(int(off[-1]), dtype=torch.uint8, device=dev)
        self.maxv = int(np.max(np.diff(off)))

    def bind_outputs(self, d_valid, d_ct_valid, d_status, d_out=None):
        self.d_valid, self.d_ct_valid, self.d_status = d_valid, d_ct_valid, d_status
        if d_out is not None:  # the plaintexts straight into the gathered slab
            assert d_out.numel() >= int(self.off[-1])
            self.d_out = d_out

    def step(self, events=None):
        if events:
            events[0].record(self.stream)
        # one call per node-epoch (hbx_decrypt_epoch_d): hash_g1_g2 + lines, share checks (the
        # node's own share check is Ciphertext::verify), combine + decrypt
        self.ctx.decrypt_epoch_d(self.d_u, self.d_v, self.d_off, self.d_w, self.pj, self.maxv, self.d_shares, self.n,
                                 self.t, self.d_out, d_valid=self.d_valid, d_ct_valid=self.d_ct_valid,
                                 d_status=self.d_status, stream=self.stream.cuda_stream)
        if events:
            events[1].record(self.stream)

    def check(self, lo):
        valid = self.d_valid.cpu().numpy().reshape(self.pj, self.n).astype(bool)
        expect = ~self.ep["corrupt"]
        assert (self.d_ct_valid.cpu().numpy() == 1).all(), "a valid ciphertext failed Ciphertext::verify"
        assert (valid == expect).all(), f"validity mismatch at {int((valid != expect).sum())} positions"
        assert (self.d_status.cpu().numpy() == 0).all(), "combine status"
        out = self.d_out.cpu().numpy()
        for j in range(self.pj):
            assert out[self.off[j]:self.off[j + 1]].tobytes() == self.ep["msgs"][j], f"plaintext {lo + j} differs"

    def kernel_ms(self):
        kern = {}
        for name in ("prepare_ct", "prepare_lines", "ct_checks", "verify_shares", "combine"):
            tot, cnt = self.ctx.kernel_time(name)
            kern[name] = round(tot / max(cnt, 1), 3)
        return kern


def verify_roofline(shares: int, ms_kernel: float, kernel: str, traffic=None):
    achieved = shares * VDEC_FQMUL * MADS_PER_FQMUL / (ms_kernel * 1e-3) / 1e12
    achieved_op = shares * OPCOUNT_VDEC * MADS_PER_FQMUL / (ms_kernel * 1e-3) / 1e12
    r = {"bound": "valu-int (v_mad_u64_u32)", "achieved": round(achieved, 3), "peak": PEAK_TMAD_S,
         "unit": "Tmad/s", "frac": round(achieved / PEAK_TMAD_S, 4), "traffic": None,
         "kernel": kernel, "kernel_ms": ms_kernel,
         "work": f"{shares} shares x {VDEC_FQMUL} Fq-mul (frozen unit V_dec, SURVEY.md §8(d)) x {MADS_PER_FQMUL} MAD",
         "opcount": {"fqmul_per_share": OPCOUNT_VDEC, "achieved": round(achieved_op, 3),
                     "frac": round(achieved_op / PEAK_TMAD_S, 4),
                     "note": "the current code's own Fq-mul count (tools/opcount), reported beside the frozen unit"}}
    if traffic:
        r["traffic"] = traffic["bytes_per_launch"]
        r["traffic_note"] = (f"PMC FETCH_SIZE (x2, gfx950) + WRITE_SIZE per share-check region at N=256, summed over "
                             f"{traffic['kernel']} ({traffic['source']}, commit {traffic.get('commit', '?')}); "
                             f"algorithmic ~1.2e7 B of inputs + 3 Fq12 slots per check written and read "
                             f"(~0.5e9 B at N=256)")
    return r


def in_flight(args, eb: EpochBench, dev, torch, Context, verifies):
    """Throughput with `args.in_flight` consecutive epochs overlapping: epoch k on context k mod F
    (own buffers and stream), issued back to back, so one epoch's latency-bound stages (hash-to-G2,
    lines, combine) run beside another's share checks.  The headline `value` stays one epoch at a
    time; this is the node's rate when future-epoch messages are already queued."""
    F = args.in_flight
    ep, pj, n, off = eb.ep, eb.pj, eb.n, eb.off
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
        c.decrypt_epoch_d(eb.d_u, eb.d_v, eb.d_off, eb.d_w, pj, eb.maxv, eb.d_shares, n, eb.t, o, d_valid=v,
                          d_ct_valid=cv, d_status=stt, stream=st.cuda_stream)

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


def config_c1(args, dev, torch, Context):
    """BASELINE config 0 (``examples/simulation.rs``, 10 nodes): the crypto of one node-epoch at
    N=10 -- 10 Ciphertext::verify, 90 decryption-share verifies, 10 combines (t=4) + decrypt -- on
    one GPU (one hbx_decrypt_epoch_d call) and on one CPU thread in the reference's shape (the
    simulator runs every node as a single-threaded state machine).  The network simulation itself
    (message delays, bandwidth) is out of scope."""
    n = 10
    stream = torch.cuda.Stream(dev)
    with Context(dev.index or 0) as ctx:
        ep = make_epoch(ctx, n, 0, n, args.vlen, args.corrupt_every)
        eb = EpochBench(ctx, ep, dev, stream, torch, args.verify_lanes, not args.no_own_share)
        eb.bind_outputs(torch.zeros(n * n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev),
                        torch.zeros(n, dtype=torch.int32, device=dev))
        for _ in range(max(args.warmup, 1)):
            eb.step()
        torch.cuda.synchronize(dev)
        steps = max(args.steps, 10)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
        wall = []
        for k in range(steps):
            t0 = time.perf_counter()
            eb.step(ev[k])
            torch.cuda.synchronize(dev)
            wall.append(time.perf_counter() - t0)
        eb.check(0)
        flight = in_flight(args, eb, dev, torch, Context, n * n) if args.in_flight > 1 else None
    res = {"workload": f"node-epoch crypto at N={n} (simulation example's 10 nodes): {n} Ciphertext::verify + "
                       f"{n * (n - 1)} decryption-share verifies + {n} combines (t={ep['t']}) + decrypt, |v|={args.vlen} B",
           "value": round(1e3 * float(np.mean(wall)), 3), "unit": "ms per node-epoch (wall, one call, synchronised)",
           "higher_is_better": False,
           "epoch_ms_hip_events": round(float(np.mean([e[0].elapsed_time(e[1]) for e in ev])), 3),
           "note": "latency-bound: 100 checks occupy 100 lanes; the chain of dependent stages sets the time"}
    if flight:
        res["epochs_in_flight"] = flight
    if not args.no_cpu_baseline:
        lib = cpu_lib()
        cts = ep["cts"]
        pk = np.ascontiguousarray(ep["pk_shares"], dtype=np.uint8)
        u = np.stack([np.frombuffer(c[0], dtype=np.uint8) for c in cts])
        w = np.stack([np.frombuffer(c[2], dtype=np.uint8) for c in cts])
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(c[1]) for c in cts])
        v = np.frombuffer(b"".join(c[1] for c in cts), dtype=np.uint8).copy()
        sh = np.ascontiguousarray(ep["shares"], dtype=np.uint8)
        kk = np.arange(n * n, dtype=np.uint64)
        jobs = np.stack([kk // n, kk % n], axis=1).astype(np.uint32)
        out = np.zeros(len(jobs), dtype=np.uint8)
        t0 = time.perf_counter()
        lib.cpu_verify_dec_shares(pk.ctypes.data, n, u.ctypes.data, v.ctypes.data, off.ctypes.data, w.ctypes.data,
                                  sh.ctypes.data, jobs.ctypes.data, len(jobs), 1, out.ctypes.data)
        dv = time.perf_counter() - t0
        assert (out.astype(bool) == ~ep["corrupt"].reshape(-1)).all(), "CPU C1 checks"
        plain = np.zeros_like(v)
        st = np.zeros(n, dtype=np.int32)
        t0 = time.perf_counter()
        lib.cpu_combine_decrypt(sh.ctypes.data, out.ctypes.data, n, n, ep["t"], v.ctypes.data, off.ctypes.data, 1,
                                plain.ctypes.data, st.ctypes.data)
        dc = time.perf_counter() - t0
        assert (st == 0).all() and all(plain[off[j]:off[j + 1]].tobytes() == ep["msgs"][j] for j in range(n)), "CPU C1 decrypt"
        host = host_info()
        res["cpu_baseline"] = {"value": round((dv + dc) * 1e3, 1), "unit": "ms per node-epoch", "cores": 1, "kind": "port",
                               "higher_is_better": False, "host": host,
                               "rows": {"checks_ms": round(dv * 1e3, 1), "combine_decrypt_ms": round(dc * 1e3, 1)},
                               "sample": f"the whole N={n} node-epoch on 1 thread, reference shape (per-share hash_g1_g2 "
                                         f"+ two pairings; {n * n} two-pairing checks: the {n} Ciphertext::verify have the "
                                         f"shape of a share check) + {n} combines; tools/cpu_baseline/cpu_port.cpp on "
                                         f"{host['model']}"}
    return res


def config_c2(args, dev, torch, Context):
    """BASELINE config 1: N=64, 4,096 decryption-share verifies + 64 combines (t=22) on one GPU."""
    n = 64
    stream = torch.cuda.Stream(dev)
    with Context(dev.index or 0) as ctx:
        ep = make_epoch(ctx, n, 0, n, args.vlen, args.corrupt_every)
        eb = EpochBench(ctx, ep, dev, stream, torch, args.verify_lanes, not args.no_own_share)
        eb.bind_outputs(torch.zeros(n * n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev),
                        torch.zeros(n, dtype=torch.int32, device=dev))
        for _ in range(max(args.warmup, 1)):
            eb.step()
        torch.cuda.synchronize(dev)
        steps = max(args.steps, 5)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
        ctx.set_timing(True)
        t0 = time.perf_counter()
        for k in range(steps):
            eb.step(ev[k])
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        eb.check(0)
        kern = eb.kernel_ms()
        ctx.set_timing(False)
        lanes = ctx.verify_lanes_used()
        # latency-bound at N=64: the node's rate with epochs overlapping (HoneyBadger's future epochs)
        flight = in_flight(args, eb, dev, torch, Context, n * n) if args.in_flight > 1 else None
    ms = elapsed / steps * 1e3
    res = {"workload": f"HoneyBadger node-epoch N={n}: {n * n} decryption-share verifies + {n} Ciphertext::verify + "
                       f"{n} combines (t={ep['t']}) + decrypt, |v|={args.vlen} B",
           "value": round(n * n / (elapsed / steps), 1), "unit": "share verifies/s", "ms_per_epoch": round(ms, 3),
           "epoch_ms_hip_events": round(float(np.mean([e[0].elapsed_time(e[1]) for e in ev])), 3),
           "kernels_ms": kern,
           "verify_lanes": lanes,
           "roofline": verify_roofline(n * n, kern["verify_shares"], f"k_verify_shares{lanes if lanes > 1 else ''} "
                                       "(auto: 64 x 64 checks fill 1/16 of the chip one lane per check)"),
           "note": "latency-bound: 4,096 checks leave most SIMDs idle; the per-proposer chains set the time"}
    if flight:
        res["epochs_in_flight"] = flight
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_dec(ep, args.cpu_seconds)
    return res


# ----------------------------------------------------------------------------------------------
# Stack B: Common Coin (C4)
# ----------------------------------------------------------------------------------------------
def config_c4(args, dev, torch, Context):
    """BASELINE config 3: CommonCoin for 256 concurrent ABA instances at N=128 (sessions {0,1} x
    proposers 0..127, agreement epoch 2; nonces as agreement/mod.rs:155-165): 32,768 signature-share
    verifies (common_coin.rs:151) + 256 combine_signatures + master verifications + parities (:190,
    :196, :173).  1 in 64 shares replaced by another instance's share of the same signer."""
    from hbbft_amd import netinfo

    n, inst = 128, 256
    with Context(dev.index or 0) as ctx:
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
        steps = max(args.steps, 3)
        wall = []
        # the round on HBM-resident buffers (hbx_verify_sig_shares_d / hbx_combine_signatures_d):
        # the shares are already on the device, as they would be after the transport's copy
        d_bad = torch.from_numpy(bad).to(dev)
        d_vst = torch.zeros((inst, n), dtype=torch.uint8, device=dev)
        d_sig = torch.zeros((inst, 96), dtype=torch.uint8, device=dev)
        d_st = torch.zeros(inst, dtype=torch.int32, device=dev)
        d_ok = torch.zeros(inst, dtype=torch.uint8, device=dev)
        d_par = torch.zeros(inst, dtype=torch.uint8, device=dev)

        def round_():
            ctx.prepare_nonces(nonces, hashes=False)
            ctx.verify_sig_shares_d(d_bad, None, d_vst)
            ctx.combine_signatures_d(master_pk, t, None, d_sig, d_st, d_ok, d_par)

        round_()  # warm-up round
        torch.cuda.synchronize(dev)
        ctx.set_timing(True)
        for _ in range(steps):
            t0 = time.perf_counter()
            round_()
            torch.cuda.synchronize(dev)
            wall.append(time.perf_counter() - t0)
        kern = {}
        for name in ("hash_nonces", "prepare_lines", "decode_sigs", "verify_sig", "combine_sigs"):
            ms_, cnt_ = ctx.kernel_time(name)
            kern[name] = round(ms_ / max(cnt_, 1), 3) if cnt_ else 0.0
        ctx.set_timing(False)
        lanes = ctx.coin_lanes_used()
        valid = d_vst.cpu().numpy() == 1
        st, ok = d_st.cpu().numpy(), d_ok.cpu().numpy().astype(bool)
        flight = c4_in_flight(args, dev, torch, Context, pk, master_pk, nonces, d_bad, corrupt, t, steps)
    assert (valid == ~corrupt).all(), "signature-share validity"
    assert (st == 0).all() and ok.all(), "combine / master verification"
    kms = kern["verify_sig"]
    achieved = inst * n * VSIG_FQMUL * MADS_PER_FQMUL / (kms * 1e-3) / 1e12
    achieved_op = inst * n * OPCOUNT_VSIG * MADS_PER_FQMUL / (kms * 1e-3) / 1e12
    round_kernels = sum(kern.values())
    res = {"workload": f"CommonCoin N={n} x {inst} instances: {inst * n} signature-share verifies + {inst} "
                       f"combine_signatures (t={t}) + master verifies + parities",
           "value": round(inst * n / (round_kernels * 1e-3), 1),
           "unit": "sig shares/s through the whole coin round (hash_g2 of the nonces + share decode + share "
                   "checks + combine + master verify + parity; sum of the round's kernel times, HIP events)",
           "verify_value": round(inst * n / (kms * 1e-3), 1),
           "verify_unit": "sig-share verifies/s (the share-check kernels alone)",
           "round_ms_kernels": round(round_kernels, 3),
           "rounds_in_flight": flight,
           "round_ms_wall": round(1e3 * float(np.mean(wall)), 3),
           "wall_note": "device API (hbx_verify_sig_shares_d / hbx_combine_signatures_d) on HBM-resident shares; "
                        "hbx_prepare_nonces uploads the 256 nonces and synchronises",
           "kernels_ms": kern, "coin_lanes": lanes,
           "roofline": {"bound": "valu-int (v_mad_u64_u32)", "achieved": round(achieved, 3), "peak": PEAK_TMAD_S,
                        "unit": "Tmad/s", "frac": round(achieved / PEAK_TMAD_S, 4), "traffic": None,
                        "kernel": ("k_verify_sig_shares2 (two lanes per check: 512 one-lane waves would fill half the chip)"
                                   if lanes == 2 else "k_verify_sig_shares (one lane per check)"),
                        "kernel_ms": kms,
                        "work": f"{inst * n} checks x {VSIG_FQMUL} Fq-mul (frozen unit V_sig) x {MADS_PER_FQMUL} MAD",
                        "opcount": {"fqmul_per_check": OPCOUNT_VSIG, "frac": round(achieved_op / PEAK_TMAD_S, 4)}}}
    coin_pmc = traffic_record("coin") if lanes == 2 else None
    if coin_pmc:
        res["roofline"]["traffic"] = coin_pmc["bytes_per_launch"]
        res["roofline"]["traffic_note"] = (
            f"PMC FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch of {coin_pmc['kernel']} at this workload "
            f"({coin_pmc['source']}, commit {coin_pmc.get('commit', '?')}); algorithmic: the keys, H', the "
            f"decoded shares and one Fq12 per check written to and read from the pair's global slot (~0.05e9 B)")
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_coin(pk, nonces, bad, corrupt, master_pk, t, args.cpu_seconds)
    return res


def c4_in_flight(args, dev, torch, Context, pk, master_pk, nonces, d_bad, corrupt, t, steps):
    """C4 rounds with `args.in_flight` rounds overlapping: round k on context k mod F (own nonce
    hashes, statuses and stream), so one round's hash_g2 (64 waves: a latency chain) and combine run
    beside another round's share checks.  The host waits for round k - F before reusing its context.
    Same inputs every round; every round's statuses and combines are checked."""
    F = args.in_flight
    if F < 2:
        return None
    inst, n = d_bad.shape[:2]
    flights = []
    for _ in range(F):
        c = Context(dev.index or 0)
        assert (c.set_pk_shares([r.tobytes() for r in pk]) == 0).all()
        st = torch.cuda.Stream(dev)
        bufs = (torch.zeros((inst, n), dtype=torch.uint8, device=dev), torch.zeros((inst, 96), dtype=torch.uint8, device=dev),
                torch.zeros(inst, dtype=torch.int32, device=dev), torch.zeros(inst, dtype=torch.uint8, device=dev),
                torch.zeros(inst, dtype=torch.uint8, device=dev))
        flights.append((c, st, bufs))
    torch.cuda.synchronize(dev)

    def issue(k):
        c, st, (v, sig, stt, ok, par) = flights[k % F]
        st.synchronize()  # round k - F on this context is done: its buffers may be reused
        c.prepare_nonces(nonces, hashes=False)
        c.verify_sig_shares_d(d_bad, None, v, stream=st.cuda_stream)
        c.combine_signatures_d(master_pk, t, None, sig, stt, ok, par, stream=st.cuda_stream)

    for k in range(F):
        issue(k)
    torch.cuda.synchronize(dev)
    rounds = F * max(steps, 2)
    t0 = time.perf_counter()
    for k in range(rounds):
        issue(k)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    for c, _, (v, sig, stt, ok, par) in flights:
        assert ((v.cpu().numpy() == 1) == ~corrupt).all(), "in-flight coin validity"
        assert (stt.cpu().numpy() == 0).all() and (ok.cpu().numpy() == 1).all(), "in-flight combine"
        c.close()
    return {"rounds": rounds, "in_flight": F, "ms_per_round": round(elapsed / rounds * 1e3, 3),
            "value": round(inst * n * rounds / elapsed, 1), "unit": "sig shares/s (wall clock, rounds overlapping)"}


def cpu_baseline_coin(pk, nonces, sigs, corrupt, master_pk, t, seconds):
    lib = cpu_lib()
    inst, n = sigs.shape[:2]
    pk = np.ascontiguousarray(pk, dtype=np.uint8)
    blob = np.frombuffer(b"".join(nonces), dtype=np.uint8).copy()
    off = np.zeros(inst + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(x) for x in nonces])
    sig = np.ascontiguousarray(sigs, dtype=np.uint8)
    threads = all_cores()

    def run(jobs, nthreads, fused):
        out = np.zeros(len(jobs), dtype=np.uint8)
        t0 = time.perf_counter()
        lib.cpu_verify_sig_shares(pk.ctypes.data, n, blob.ctypes.data, off.ctypes.data, inst, sig.ctypes.data,
                                  jobs.ctypes.data, len(jobs), nthreads, fused, out.ctypes.data)
        dt = time.perf_counter() - t0
        assert (out.astype(bool) == ~corrupt[jobs[:, 0], jobs[:, 1]]).all(), "CPU coin port disagrees"
        return dt

    def scattered(count, start):
        k = np.arange(start, start + count, dtype=np.uint64)
        return np.stack([(k * 7919) % inst, (k * 104729 + 3) % n], axis=1).astype(np.uint32)

    t1 = run(scattered(2, 0), 1, 0) / 2
    na = max(2, int(seconds / 2 / t1))
    da = run(scattered(na, 2), 1, 0)
    one = np.stack([np.zeros(n, np.uint64), np.arange(n, dtype=np.uint64)], axis=1).astype(np.uint32)
    tb1 = run(one, 1, 1) / n
    rows = max(1, min(inst, int(seconds / 2 * min(threads, 64) / (tb1 * n))))
    kk = np.arange(rows * n, dtype=np.uint64)
    jobs = np.stack([kk // n, kk % n], axis=1).astype(np.uint32)
    db = run(jobs, threads, 1)
    brow = {"b_hoisted_fused_all_cores": (len(jobs) / db, threads)}
    qc = quota_cores()
    if qc:
        dq = run(jobs, qc, 1)
        brow["b_hoisted_fused_quota_cores"] = (len(jobs) / dq, qc)
    best = "b_hoisted_fused_quota_cores" if qc else "b_hoisted_fused_all_cores"  # as cpu_baseline_dec
    threads_c = brow[best][1]
    # combine_signatures + master verify + parity of the sampled instances, best row's threads
    valid = np.ascontiguousarray(~corrupt, dtype=np.uint8)
    ok = np.zeros(inst, dtype=np.uint8)
    par = np.zeros(inst, dtype=np.uint8)
    mpk = np.frombuffer(master_pk, dtype=np.uint8).copy()
    t0 = time.perf_counter()
    lib.cpu_combine_sigs(sig.ctypes.data, valid.ctypes.data, n, rows, t, mpk.ctypes.data, blob.ctypes.data,
                         off.ctypes.data, threads_c, ok.ctypes.data, par.ctypes.data)
    dc = time.perf_counter() - t0
    assert ok[:rows].all(), "CPU combine / master verification"
    host = host_info()
    out_rows = {"a_reference_shape_1thread": {"value": round(na / da, 1), "cores": 1,
                                              "sample": f"{na} shares in {da:.1f} s"},
                "b_hoisted_fused_all_cores": {"value": round(len(jobs) / db, 1), "cores": threads,
                                              "single_thread": round(1.0 / tb1, 2),
                                              "sample": f"{rows} instances x {n} shares in {db:.1f} s"},
                "combine_master_parity": {"ms_per_256_instances": round(dc / rows * 256 * 1e3, 1), "cores": threads_c,
                                          "sample": f"{rows} instances in {dc:.2f} s"}}
    if qc:
        out_rows["b_hoisted_fused_quota_cores"] = {"value": round(brow["b_hoisted_fused_quota_cores"][0], 1),
                                                   "cores": qc, "sample": f"same sample; cgroup cpu.max allows {qc} CPUs"}
    out_rows["round_verify_plus_combine"] = {"ms_per_round": round((inst * n / brow[best][0] + dc / rows * inst) * 1e3, 1),
                                             "cores": threads_c}
    return dict(value=round(brow[best][0], 1), unit="sig-share verifies/s", cores=brow[best][1], kind="port",
                host=host, best_row=best, cgroup_cpus=qc, rows=out_rows,
                sample=f"tools/cpu_baseline/cpu_port.cpp (g++ -O3) on {host['model']}: value = row {best}; (a) 1 thread, hash_g2 per "
                       f"share with pairing 0.14's cofactor multiplication + two pairings; (b) {threads} threads, "
                       f"H lines per instance + one mixed Miller loop + one final exponentiation per share; a "
                       f"restatement, not the reference binary")


# ----------------------------------------------------------------------------------------------
# Stack C: Broadcast (C5)
# ----------------------------------------------------------------------------------------------
def config_c5(args, dev, torch, Context):
    """BASELINE config 4: Broadcast at N=128 (f=42), RS(k=44, m=84), 128 instances of a 1 MiB
    proposal each: encode (broadcast.rs:366) + Merkle roots (:381) + decode with the last 42 shards
    missing (reconstruct + rebuild + root check + glue, :660-707), for both Merkle digests
    (SHA-256 as the reference's merkle/ring, and the SHA3 variant north_star names).  Output ==
    input payload is checked."""
    from hbbft_amd.hbx import MERKLE_SHA3, MERKLE_SHA256

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
    shards = torch.from_numpy(host).to(dev)
    roots = torch.zeros((inst, 32), dtype=torch.uint8, device=dev)
    present = torch.ones((inst, n), dtype=torch.uint8, device=dev)
    present[:, n - f:] = 0
    out = torch.zeros((inst, k * L), dtype=torch.uint8, device=dev)
    out_len = torch.zeros(inst, dtype=torch.int64, device=dev)
    status = torch.zeros(inst, dtype=torch.int32, device=dev)
    work = torch.empty_like(shards)
    stream = torch.cuda.Stream(dev)  # events must be recorded on the stream the kernels run on
    sh = stream.cuda_stream
    steps = max(args.steps, 3)
    variants = {}
    roots_by = {}
    with Context(dev.index or 0) as ctx, torch.cuda.stream(stream):
        for name, var in (("sha256", MERKLE_SHA256), ("sha3", MERKLE_SHA3)):
            ctx.set_merkle_digest(var)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            res = {"encode": [], "roots": [], "decode": [], "step": []}
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
                ev[4].record(stream)
                torch.cuda.synchronize(dev)
                if s:
                    res["encode"].append(ev[0].elapsed_time(ev[1]))
                    res["roots"].append(ev[1].elapsed_time(ev[2]))
                    res["decode"].append(ev[3].elapsed_time(ev[4]))
                    res["step"].append(ev[0].elapsed_time(ev[2]) + ev[3].elapsed_time(ev[4]))
            rs_ms, rs_cnt = ctx.kernel_time("rs_code")
            ml_ms, ml_cnt = ctx.kernel_time("merkle_leaves")
            ctx.set_timing(False)
            assert (status.cpu().numpy() == 0).all(), "decode status"
            assert (out_len.cpu().numpy() == plen).all()
            assert np.array_equal(out[:, :plen].cpu().numpy(), payload), "decoded payload"
            # the same decode with the f erasures spread over data and parity shards (about a third
            # of them data shards: the reconstruct solves for those), beside the parity-only pattern
            spread = np.unique(np.linspace(0, n - 1, f).round().astype(np.int64))
            present_mix = torch.ones((inst, n), dtype=torch.uint8, device=dev)
            present_mix[:, torch.from_numpy(spread).to(dev)] = 0
            mix_ms = []
            for s in range(steps + 1):
                work.copy_(shards)
                work[present_mix == 0] = 0xA5
                ev[3].record(stream)
                ctx.broadcast_decode_d(work, present_mix, roots, k, m, out, out_len, status, stream=sh)
                ev[4].record(stream)
                torch.cuda.synchronize(dev)
                if s:
                    mix_ms.append(ev[3].elapsed_time(ev[4]))
            assert (status.cpu().numpy() == 0).all(), "decode status (spread erasures)"
            assert np.array_equal(out[:, :plen].cpu().numpy(), payload), "decoded payload (spread erasures)"
            res["decode_spread"] = mix_ms
            res["erased_data_spread"] = [int((spread < k).sum())]
            roots_by[name] = roots.cpu().numpy().copy()
            erased_data = res.pop("erased_data_spread")[0]
            ms = {key: float(np.mean(v)) for key, v in res.items()}
            leaf_bytes = inst * n * (L + 1)
            pmc = c5_traffic()
            kleaf = "k_merkle_leaves" + ("_sha256" if name == "sha256" else "_sha3")
            rs_bytes = inst * (k + m) * L  # k L read + m L written per instance
            ml = ml_ms / max(ml_cnt, 1)
            variants[name] = {
                "value": round(inst * plen / (ms["step"] * 1e-3) / 1e9, 2),
                "unit": "GB/s of proposals (encode + Merkle roots + decode with 42 missing)",
                "ms": {key: round(v, 3) for key, v in ms.items()},
                "decode_spread_note": (f"decode_spread: the {f} erasures at evenly spaced shard indices, {erased_data} of them "
                                       f"data shards (decode: the last {f}, parity only); not in the step"),
                "merkle_leaves_kernel_ms": round(ml, 4),
                "merkle_leaves_GBps": round(leaf_bytes / (ml * 1e-3) / 1e9, 1),
                "roofline": {"bound": "hbm", "achieved": round(leaf_bytes / (ml * 1e-3) / 1e9, 1),
                             "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(leaf_bytes / (ml * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                             "traffic": pmc.get(kleaf, {}).get("bytes_per_launch"), "kernel": kleaf,
                             "traffic_note": (f"PMC FETCH_SIZE (x2) + WRITE_SIZE per launch, {pmc[kleaf]['source']}"
                                              if kleaf in pmc else None),
                             "work": f"{inst} x {n} leaves of {L + 1} B hashed per launch"},
            }
            variants[name]["node_epoch"] = echo_epoch(ctx, torch, dev, stream, shards, roots, present, k, m, steps)
            if name == "sha256":
                enc = ms["encode"]
                dwords = inst * (L // 4)
                enc_valu = dwords * m * k * 4.0  # k_rs_code_perm3: 8 v_perm_b32 + 4 v_bitop3 per (out, input triple, dword)
                krs = "k_rs_code_perm3"
                variants["rs_encode"] = {
                    "ms": round(enc, 4), "kernel_ms_per_launch": round(rs_ms / max(rs_cnt, 1), 4),
                    "roofline": {"bound": "valu (v_perm_b32 table lookups)", "achieved": round(rs_bytes / (enc * 1e-3) / 1e9, 1),
                                 "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(rs_bytes / (enc * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                                 "valu_frac": round(enc_valu / (enc * 1e-3) / PEAK_VALU_OPS, 3),
                                 "valu_floor_ms": round(enc_valu / PEAK_VALU_OPS * 1e3, 3),
                                 "traffic": pmc.get(krs, {}).get("bytes_per_launch"),
                                 "traffic_note": ("PMC per launch averaged over the run's encode AND reconstruct "
                                                  f"launches ({pmc[krs]['launches'][0]}), "
                                                  f"{pmc[krs]['source']}" if krs in pmc else None),
                                 "kernel": krs,
                                 "work": f"{inst} x ({k} L read + {m} L written), L = {L}"}}
    sub = {"workload": f"Broadcast N={n} RS({k},{m}) x {inst} instances of a 1 MiB proposal (shard {L} B)",
           "value": variants["sha256"]["value"], "unit": variants["sha256"]["unit"],
           "merkle_sha256": variants["sha256"], "merkle_sha3": variants["sha3"], "rs_encode": variants["rs_encode"]}
    if args.in_flight > 1:
        sub["steps_in_flight"] = c5_in_flight(args, dev, torch, Context, shards, present, k, m, f, plen, payload, steps)
    if not args.no_cpu_baseline:
        sub["cpu_baseline"] = cpu_baseline_broadcast(host, k, m, L, payload, roots_by, args.cpu_seconds)
    return sub


def c5_in_flight(args, dev, torch, Context, shards0, present, k, m, f, plen, payload, steps):
    """C5 steps (encode + roots + decode, SHA-256 tree) with `args.in_flight` steps overlapping:
    step s on context s mod F with its own shard, work and output buffers and stream, issued back
    to back -- the leaf hashing's serial chains fill a quarter of the SIMDs, so the next batch of
    proposals' coding and hashing run beside it (Broadcast instances of later epochs).  The
    headline stays one step at a time."""
    from hbbft_amd.hbx import MERKLE_SHA256

    F = args.in_flight
    inst, n, L = shards0.shape
    lanes = []
    for _ in range(F):
        c = Context(dev.index or 0)
        c.set_merkle_digest(MERKLE_SHA256)
        st = torch.cuda.Stream(dev)
        bufs = (shards0.clone(), torch.empty_like(shards0), torch.zeros((inst, 32), dtype=torch.uint8, device=dev),
                torch.zeros((inst, k * L), dtype=torch.uint8, device=dev), torch.zeros(inst, dtype=torch.int64, device=dev),
                torch.zeros(inst, dtype=torch.int32, device=dev))
        lanes.append((c, st, bufs))
    torch.cuda.synchronize(dev)

    def issue(q):
        c, st, (sh_, work, roots, out, out_len, status) = lanes[q % F]
        with torch.cuda.stream(st):
            c.rs_encode_d(sh_, k, m, stream=st.cuda_stream)
            c.merkle_roots_d(sh_, roots, stream=st.cuda_stream)
            work.copy_(sh_)
            work[:, n - f:] = 0xA5
            c.broadcast_decode_d(work, present, roots, k, m, out, out_len, status, stream=st.cuda_stream)

    for q in range(F):
        issue(q)
    torch.cuda.synchronize(dev)
    total = F * max(steps, 2)
    t0 = time.perf_counter()
    for q in range(total):
        issue(q)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    for c, _, (_, _, _, out, out_len, status) in lanes:
        assert (status.cpu().numpy() == 0).all() and (out_len.cpu().numpy() == plen).all(), "in-flight decode status"
        assert np.array_equal(out[:, :plen].cpu().numpy(), payload), "in-flight decoded payload"
        c.close()
    return {"steps": total, "in_flight": F, "ms_per_step": round(elapsed / total * 1e3, 3),
            "value": round(inst * plen * total / elapsed / 1e9, 2),
            "unit": "GB/s of proposals (wall clock, steps overlapping; SHA-256 tree)"}


def echo_epoch(ctx, torch, dev, stream, shards, roots, present, k, m, steps):
    """One node's Broadcast crypto for a whole epoch (row f3, hbbft_amd/broadcast.py): validate the
    Echo proof of every (instance, sender) pair -- validate_proof at broadcast.rs:451, one
    hbx_merkle_validate_d call -- then decode every instance from its validated Echo values with
    the proofs' leaf digests (hbx_broadcast_decode_leaves_d, compute_output :521-551).  The proofs
    are MerkleTree::gen_proof outputs of the encoded shards (hbx_merkle_build_d +
    hbx_merkle_proofs_d, not timed)."""
    inst, n, L = shards.shape
    sh = stream.cuda_stream
    cnt = ctx.merkle_node_count(n)
    nodes = torch.zeros((inst, cnt, 32), dtype=torch.uint8, device=dev)
    ctx.merkle_build_d(shards, nodes, stream=sh)
    P = inst * n
    req = torch.stack([torch.arange(inst, device=dev).repeat_interleave(n), torch.arange(n, device=dev).repeat(inst)],
                      dim=1).to(torch.int32).contiguous()
    nh = torch.zeros((P, 17, 32), dtype=torch.uint8, device=dev)
    sb = torch.zeros((P, 16, 32), dtype=torch.uint8, device=dev)
    sides = torch.zeros(P, dtype=torch.int32, device=dev)
    depth = torch.zeros(P, dtype=torch.int32, device=dev)
    proot = torch.zeros((P, 32), dtype=torch.uint8, device=dev)
    ctx.merkle_proofs_d(nodes, n, req, nh, sb, sides, depth, proot, stream=sh)
    values = torch.empty((P, L + 1), dtype=torch.uint8, device=dev)  # index byte || shard
    values[:, 0] = torch.arange(n, device=dev).repeat(inst).to(torch.uint8)
    values[:, 1:] = shards.reshape(P, L)
    sender = torch.arange(n, device=dev).repeat(inst).to(torch.int32)
    valid = torch.zeros(P, dtype=torch.uint8, device=dev)
    leaf = nh.gather(1, depth.long().view(P, 1, 1).expand(P, 1, 32)).view(inst, n, 32).contiguous()
    work = torch.empty_like(shards)
    out = torch.zeros((inst, k * L), dtype=torch.uint8, device=dev)
    out_len = torch.zeros(inst, dtype=torch.int64, device=dev)
    status = torch.zeros(inst, dtype=torch.int32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    tv, td = [], []
    for s in range(steps + 1):
        ev[0].record(stream)
        ctx.merkle_validate_d(values, nh, sb, sides, depth, proot, sender, n, valid, stream=sh)
        ev[1].record(stream)
        work.copy_(shards)
        work[present == 0] = 0xA5
        ev[2].record(stream)
        ctx.broadcast_decode_leaves_d(work, present, leaf, roots, k, m, out, out_len, status, stream=sh)
        ev[3].record(stream)
        torch.cuda.synchronize(dev)
        if s:
            tv.append(ev[0].elapsed_time(ev[1]))
            td.append(ev[2].elapsed_time(ev[3]))
    assert bool((valid == 1).all()), "an honest Echo proof failed validate_proof"
    assert bool((status == 0).all()), "decode of the validated Echo values"
    vms, dms = float(np.mean(tv)), float(np.mean(td))
    vbytes = P * (L + 1)
    return {"echo_proofs": P, "validate_ms": round(vms, 3), "decode_leaves_ms": round(dms, 3),
            "ms": round(vms + dms, 3), "validate_GBps_hashed": round(vbytes / (vms * 1e-3) / 1e9, 1),
            "note": f"{P} Echo proofs of {L + 1} B validated in one call + {inst} decodes from the validated "
                    f"values with their leaf digests ({m - (n - int(present[0].sum().item()))} of {m} spare shards "
                    f"present per instance)"}


def _tree_root(leaf_hashes, node):
    level = list(leaf_hashes)
    while len(level) > 1:
        nxt = [node(level[i], level[i + 1]) for i in range(0, len(level) - 1, 2)]
        if len(level) % 2:
            nxt.append(level[-1])
        level = nxt
    return level[0]


def cpu_merkle_root(shards, variant):
    """merkle (afck) over index-prefixed leaves with OpenSSL's SHA-256 (hashlib; ring uses the same
    SHA extensions on this CPU), or the SHA3 variant."""
    n = shards.shape[0]
    if variant == "sha256":
        leaf = lambda i: hashlib.sha256(b"\x00" + bytes([i & 0xFF]) + shards[i].tobytes()).digest()  # noqa: E731
        node = lambda a, b: hashlib.sha256(b"\x01" + a + b).digest()  # noqa: E731
    else:
        leaf = lambda i: hashlib.sha3_256(bytes([i & 0xFF]) + shards[i].tobytes()).digest()  # noqa: E731
        node = lambda a, b: hashlib.sha3_256(a + b).digest()  # noqa: E731
    return _tree_root([leaf(i) for i in range(n)], node)


def _tree_levels(leaf_hashes, node):
    levels = [list(leaf_hashes)]
    while len(levels[-1]) > 1:
        lv = levels[-1]
        nxt = [node(lv[i], lv[i + 1]) for i in range(0, len(lv) - 1, 2)]
        if len(lv) % 2:
            nxt.append(lv[-1])
        levels.append(nxt)
    return levels


def cpu_proofs(shards):
    """Proofs (index, shard, sibling path, root) of every leaf of one SHA-256 tree, as
    MerkleTree::gen_proof gives them (an unpaired last node moves up unchanged: no sibling)."""
    n = shards.shape[0]
    leaf = [hashlib.sha256(b"\x00" + bytes([i & 0xFF]) + shards[i].tobytes()).digest() for i in range(n)]
    levels = _tree_levels(leaf, lambda a, b: hashlib.sha256(b"\x01" + a + b).digest())
    out = []
    for i in range(n):
        path, q = [], i
        for lv in levels[:-1]:
            sib = q ^ 1
            if sib < len(lv):
                path.append((q & 1, lv[sib]))
            q >>= 1
        out.append((i, shards[i].tobytes(), path))
    return out, levels[-1][0]


def cpu_validate(proofs, root):
    """Proof::validate (broadcast.rs:451) of each proof: leaf hash, then one node hash per sibling."""
    ok = 0
    for i, value, path in proofs:
        h = hashlib.sha256(b"\x00" + bytes([i & 0xFF]) + value).digest()
        for right, sib in path:
            h = hashlib.sha256(b"\x01" + (sib + h if right else h + sib)).digest()
        ok += h == root
    return ok


def cpu_baseline_broadcast(host_shards, k, m, L, payload, roots_by, seconds):
    """C5 on host cores: reed-solomon-erasure's table-driven encode / reconstruct
    (tools/cpu_baseline/cpu_port.cpp) and the Merkle trees with OpenSSL's SHA-256 / SHA3-256
    (hashlib).  (a) one thread, per instance; (b) the usable cores over instances (RS: std::threads;
    Merkle: a thread pool, hashlib releases the GIL on these buffer sizes)."""
    lib = cpu_lib()
    inst, n = host_shards.shape[:2]
    threads = usable_cores()  # the CPUs this process may use (cgroup quota), as stacks A and B
    # (a) one instance, one thread
    one = host_shards[:1].copy()
    t0 = time.perf_counter()
    lib.cpu_rs_encode(one.ctypes.data, 1, k, m, L, 1)
    enc1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    r256 = cpu_merkle_root(one[0], "sha256")
    mk1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    r3 = cpu_merkle_root(one[0], "sha3")
    mk3 = time.perf_counter() - t0
    assert r256 == roots_by["sha256"][0].tobytes() and r3 == roots_by["sha3"][0].tobytes(), "CPU Merkle roots"
    pres = np.ones((1, n), dtype=np.uint8)
    pres[0, n - (n - k) // 2:] = 0  # the last f missing
    work = one.copy()
    work[pres == 0] = 0
    st = np.zeros(1, dtype=np.int32)
    t0 = time.perf_counter()
    lib.cpu_rs_reconstruct(work.ctypes.data, pres.ctypes.data, 1, k, m, L, 1, st.ctypes.data)
    rec1 = time.perf_counter() - t0
    dec_root = cpu_merkle_root(work[0], "sha256")
    assert st[0] == 0 and dec_root == r256 and np.array_equal(work, one), "CPU reconstruct"
    glued = work[0, :k].reshape(-1)[4:4 + payload.shape[1]]
    assert np.array_equal(glued, payload[0]), "CPU glue"
    dec1 = time.perf_counter() - t0
    # (b) a bounded sample of instances on all cores
    cnt = max(1, min(inst, int(seconds / 2 * min(threads, 64) / max(enc1 + mk1 + dec1, 1e-3))))
    many = host_shards[:cnt].copy()
    t0 = time.perf_counter()
    lib.cpu_rs_encode(many.ctypes.data, cnt, k, m, L, threads)
    encb = time.perf_counter() - t0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as pool:
        rts = list(pool.map(lambda j: cpu_merkle_root(many[j], "sha256"), range(cnt)))
    mkb = time.perf_counter() - t0
    assert all(rts[j] == roots_by["sha256"][j].tobytes() for j in range(cnt)), "CPU Merkle roots (b)"
    # reconstruct with the last f shards missing, all cores
    presb = np.ones((cnt, n), dtype=np.uint8)
    presb[:, n - (n - k) // 2:] = 0
    workb = many.copy()
    workb[presb == 0] = 0
    stb = np.zeros(cnt, dtype=np.int32)
    t0 = time.perf_counter()
    lib.cpu_rs_reconstruct(workb.ctypes.data, presb.ctypes.data, cnt, k, m, L, threads, stb.ctypes.data)
    recb = time.perf_counter() - t0
    assert (stb == 0).all() and np.array_equal(workb, many), "CPU reconstruct (b)"
    del workb
    # Echo branch verification: every (instance, sender) proof of the sample, all cores
    pr = [cpu_proofs(many[j]) for j in range(cnt)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as pool:
        oks = list(pool.map(lambda j: cpu_validate(pr[j][0], pr[j][1]), range(cnt)))
    vb = time.perf_counter() - t0
    assert sum(oks) == cnt * n, "CPU Proof::validate"
    del pr
    prop = payload.shape[1]
    host = host_info()
    gbps = lambda b, s: round(b / s / 1e9, 3)  # noqa: E731
    return dict(value=gbps(cnt * prop, encb + mkb), unit="GB/s of proposals (encode + SHA-256 Merkle roots)",
                cores=threads, kind="port", host=host,
                rows={"a_1thread": {"rs_encode_GBps_hbm_equiv": gbps((k + m) * L, enc1),
                                    "merkle_sha256_GBps": gbps(n * (L + 1), mk1),
                                    "merkle_sha3_GBps": gbps(n * (L + 1), mk3),
                                    "decode_ms_per_instance": round(dec1 * 1e3, 1),
                                    "ms_per_instance_encode_roots_decode": round((enc1 + mk1 + dec1) * 1e3, 1)},
                      "b_usable_cores": {"rs_encode_GBps_hbm_equiv": gbps(cnt * (k + m) * L, encb),
                                      "merkle_sha256_GBps": gbps(cnt * n * (L + 1), mkb),
                                      "rs_reconstruct_GBps_hbm_equiv": gbps(cnt * (k + m) * L, recb),
                                      "reconstruct_ms_per_instance": round(recb / cnt * 1e3, 2),
                                      "branch_verify_GBps_hashed": gbps(cnt * n * (L + 1), vb),
                                      "branch_verify_proofs_per_s": round(cnt * n / vb, 1),
                                      "sample": f"{cnt} instances on {threads} threads ({cnt * n} Echo proofs)"}},
                cgroup_cpus=quota_cores(),
                sample=f"value = row b_usable_cores ({threads} threads = the CPUs this process may use; nproc "
                       f"{host['nproc']}): RS encode by tools/cpu_baseline/cpu_port.cpp, reed-solomon-erasure "
                       f"3.1.0's MUL_TABLE shape (g++ -O3); Merkle roots by Python hashlib (OpenSSL SHA-256 / "
                       f"SHA3-256, the leaf and node digests the merkle crate's afck variant computes) on a thread "
                       f"pool, not the port; {host['model']}; a restatement, not the reference binary")


# ----------------------------------------------------------------------------------------------
# Stacks B and C across GPUs: instance sharding + one all-gather of result slabs
# ----------------------------------------------------------------------------------------------
def _sync(torch, dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _timed_steps(torch, dist, dev, world, steps, fn):
    """Barrier + synchronize on both sides of ``steps`` calls of fn; max over ranks (seconds).
    (``dev`` may be the CPU: tests/test_bench_shard_legs.py runs the legs over gloo.)"""
    group = dist.is_available() and dist.is_initialized()  # (not at a world of one without a group)
    fn()
    _sync(torch, dev)
    if group:
        dist.barrier()
    _sync(torch, dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    _sync(torch, dev)
    if group:
        dist.barrier()
    _sync(torch, dev)
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if group:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def sharded_c4(args, dev, torch, Context, world, rank, n=128, inst=256):
    """C4 across ``world`` GPUs: rank g owns instances instance_range(256, world, g) -- their nonces,
    the 128 signature shares of each, the combines; one all-gather of (share status, signature,
    combine status, master-ok, parity) slabs gives every rank the round's result.  (``n`` / ``inst``
    smaller and ``Context`` a stand-in: the CPU gloo test of this leg's control flow.)"""
    import torch.distributed as dist

    from hbbft_amd import netinfo, shard

    lo, hi = shard.instance_range(inst, world, rank)
    c = hi - lo
    lay = shard.coin_layout(inst, n, world)
    with Context(dev.index or 0) as ctx:
        sks, sk_shares, master_sk = netinfo.generate_keys(n)
        t = sks.threshold + 1
        pk = ctx.public_keys(sk_shares)
        master_pk = ctx.public_keys(master_sk)[0].tobytes()
        assert (ctx.set_pk_shares([r.tobytes() for r in pk]) == 0).all()
        inv_id = "[" + ", ".join(str(b) for b in master_pk) + "]"
        nonces = [f"Nonce for Honey Badger {inv_id}@{s}:2:{j}".encode() for s in (0, 1) for j in range(n)][lo:hi]
        ctx.prepare_nonces(nonces)
        sigs = ctx.sign(sk_shares)
        corrupt = (np.random.default_rng(0x68626278_00000005).integers(0, 64, size=(inst, n)) == 0)
        bad = sigs.copy()
        ii = np.nonzero(corrupt[lo:hi])
        bad[ii[0], ii[1]] = sigs[(ii[0] + 1) % c, ii[1]]  # another instance's share of the same signer
        expect = corrupt  # every rank substitutes within its own slice (c > 1 at 256 instances)
        slab = torch.zeros(lay.size, dtype=torch.uint8, device=dev)
        d_bad = torch.from_numpy(bad).to(dev)
        v = {name: lay.view(slab, name, c) for name in lay.fields}
        gathered = [None]

        def step():
            ctx.prepare_nonces(nonces, hashes=False)
            ctx.verify_sig_shares_d(d_bad, None, v["share_status"])
            ctx.combine_signatures_d(master_pk, t, None, v["sig"], v["comb_status"], v["master_ok"], v["parity"])
            gathered[0] = shard.all_gather_slabs(slab, world)

        steps = max(args.steps, 3)
        el = _timed_steps(torch, dist, dev, world, steps, step)
        full = shard.assemble_fields(gathered[0].cpu().numpy(), lay, inst, world)
    assert ((full["share_status"] == 1) == ~expect).all(), "gathered signature-share statuses"
    assert (full["comb_status"] == 0).all() and (full["master_ok"] == 1).all(), "gathered combines"
    return {"workload": f"CommonCoin N={n} x {inst} instances sharded by instance over {world} GPUs "
                        f"(+ one all-gather of {lay.size} B result slabs)",
            "value": round(inst * n * steps / el, 1), "unit": "sig-share verifies/s (whole job, wall)",
            "ms_per_round": round(el / steps * 1e3, 3), "instances_per_gpu": c, "scaling": "strong"}


def sharded_c5(args, dev, torch, Context, world, rank, n=128, inst=128, plen=1 << 20):
    """C5 across ``world`` GPUs: rank g owns proposals instance_range(128, world, g): encode, SHA-256
    Merkle roots and the decode with the last 42 shards missing; one all-gather of (root, decode
    status, output length) slabs; payloads stay on the owning GPU.  (Smaller shapes and a stand-in
    ``Context``: the CPU gloo test of this leg.)"""
    import torch.distributed as dist

    from hbbft_amd import shard

    f = (n - 1) // 3
    k, m = n - 2 * f, 2 * f
    L = (plen + 4 + k - 1) // k
    lo, hi = shard.instance_range(inst, world, rank)
    c = hi - lo
    rng = np.random.default_rng(0x68626278_00000006)
    payload = rng.integers(0, 256, size=(inst, plen), dtype=np.uint8)[lo:hi]
    frame = np.zeros((c, k * L), dtype=np.uint8)
    frame[:, :4] = np.frombuffer(np.uint32(plen).byteswap().tobytes(), dtype=np.uint8)
    frame[:, 4:4 + plen] = payload
    host = np.zeros((c, n, L), dtype=np.uint8)
    host[:, :k] = frame.reshape(c, k, L)
    shards = torch.from_numpy(host).to(dev)
    present = torch.ones((c, n), dtype=torch.uint8, device=dev)
    present[:, n - f:] = 0
    out = torch.zeros((c, k * L), dtype=torch.uint8, device=dev)
    work = torch.empty_like(shards)
    lay = shard.broadcast_layout(inst, world)
    slab = torch.zeros(lay.size, dtype=torch.uint8, device=dev)
    v = {name: lay.view(slab, name, c) for name in lay.fields}
    gathered = [None]
    with Context(dev.index or 0) as ctx:
        ctx.set_merkle_digest(0)

        def step():
            ctx.rs_encode_d(shards, k, m)
            ctx.merkle_roots_d(shards, v["root"])
            work.copy_(shards)
            work[:, n - f:] = 0xA5
            ctx.broadcast_decode_d(work, present, v["root"], k, m, out, v["out_len"], v["decode_status"])
            gathered[0] = shard.all_gather_slabs(slab, world)

        steps = max(args.steps, 3)
        el = _timed_steps(torch, dist, dev, world, steps, step)
        full = shard.assemble_fields(gathered[0].cpu().numpy(), lay, inst, world)
        assert np.array_equal(out[:, :plen].cpu().numpy(), payload), "decoded payload"
    assert (full["decode_status"] == 0).all() and (full["out_len"] == plen).all(), "gathered decodes"
    return {"workload": f"Broadcast N={n} RS({k},{m}) x {inst} {plen} B proposals sharded by instance over {world} "
                        f"GPUs (encode + SHA-256 roots + decode, + one all-gather of {lay.size} B slabs)",
            "value": round(inst * plen * steps / el / 1e9, 2), "unit": "GB/s of proposals (whole job, wall)",
            "ms_per_round": round(el / steps * 1e3, 3), "instances_per_gpu": c, "scaling": "strong"}


def weak_epochs(args, dev, torch, world, rank, make_bench):
    """The node's rate beside the latency-bound strong split: every rank runs
    WHOLE node-epochs of its own -- G epochs in flight across the node, as HoneyBadger keeps up to
    max_future_epochs = 3 future epochs open (dynamic_honey_badger/builder.rs:18-27) -- timed with a
    barrier + synchronize on both sides, max over ranks; every rank checks its last epoch and the
    verdicts are all-gathered (one byte per rank).  ``make_bench()`` returns an object with
    ``step()``, ``check()`` and ``units`` (share verifies per step); a stand-in in the gloo test."""
    import torch.distributed as dist

    eb = make_bench()
    steps = max(args.steps, 2)
    el = _timed_steps(torch, dist, dev, world, steps, eb.step)
    ok = torch.tensor([1 if eb.check() else 0], dtype=torch.uint8, device=dev)
    oks = torch.empty(world, dtype=torch.uint8, device=dev)
    if world > 1:
        if dev.type == "cuda":
            dist.all_gather_into_tensor(oks, ok)
        else:
            dist.all_gather(list(oks.view(world, 1).unbind(0)), ok)
    else:
        oks.copy_(ok)
    assert bool((oks == 1).all()), "weak leg: a rank's epoch failed its check"
    return {"workload": f"{world} whole node-epochs in flight, one per GPU (each {eb.units} share verifies, "
                        f"checked on every rank)",
            "value": round(world * eb.units * steps / el, 1), "unit": "share verifies/s (whole job, wall)",
            "ms_per_epoch": round(el / steps * 1e3, 3), "epochs": world * steps, "scaling": "weak"}


def gather_ms(torch, dev, world, slab, reps=10):
    """The result slab's all-gather alone (RCCL over xGMI on GPUs): barrier-bracketed, max over
    ranks, per gather."""
    import torch.distributed as dist

    from hbbft_amd import shard

    el = _timed_steps(torch, dist, dev, world, reps, lambda: shard.all_gather_slabs(slab, world))
    return round(el / reps * 1e3, 4)


class _WeakEpoch:
    """A whole node-epoch on this rank's GPU for weak_epochs (its own context and stream)."""

    def __init__(self, args, dev, torch, Context, n):
        self.torch = torch
        self.ctx = Context(dev.index or 0)
        self.ep = make_epoch(self.ctx, n, 0, n, args.vlen, args.corrupt_every)
        self.stream = torch.cuda.Stream(dev)
        self.eb = EpochBench(self.ctx, self.ep, dev, self.stream, torch, args.verify_lanes, not args.no_own_share,
                             args.combine_lanes)
        self.eb.bind_outputs(torch.zeros(n * n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8, device=dev),
                             torch.zeros(n, dtype=torch.int32, device=dev))
        self.units = n * n

    def step(self):
        self.eb.step()

    def check(self):
        self.torch.cuda.synchronize()
        self.eb.check(0)  # raises on any difference
        self.ctx.close()
        return True


# ----------------------------------------------------------------------------------------------
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
    strong = args.scaling == "strong" and (world > 1 or args.strong_at_1)
    if strong:
        lo, hi = shard.proposer_range(n, world, rank)
    elif args.shard_of > 1 and world == 1:
        lo, hi = shard.proposer_range(n, args.shard_of, 0)
    else:
        lo, hi = 0, n
    pj = hi - lo
    ctx = Context(local)
    ep = make_epoch(ctx, n, lo, hi, args.vlen, args.corrupt_every)
    key_ms = None
    if world > 1:
        # the node's key material reaches every rank in one broadcast per era from rank 0 (each
        # rank synthesised the epoch's inputs itself; the engine is set up from what it received)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        pk, _mpk, own_sk, t_b = shard.broadcast_key_material(ep["pk_shares"], ep["master_pk"], ep["own_sk"], ep["t"], n,
                                                             world, dev)
        key_ms = round((time.perf_counter() - t0) * 1e3, 3)
        assert (pk == ep["pk_shares"]).all() and own_sk == ep["own_sk"] and t_b == ep["t"], "era key broadcast"
        ep["pk_shares"], ep["own_sk"], ep["t"] = pk, own_sk, t_b
    # a dedicated stream for the epoch calls; the HIP events that time the epoch and the kernels are
    # recorded on the stream the kernels run on
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0
    eb = EpochBench(ctx, ep, dev, stream, torch, args.verify_lanes, not args.no_own_share, args.combine_lanes)
    # result slab gathered across ranks: [share status pj*n | ct status pj | combine status pj*4],
    # laid out for the largest column block so every rank's slab has the same size
    # ... and, at --gpus > 1, the plaintexts (the combined outputs): the rank's decryption blob IS
    # the slab's plaintext region, sized for the largest rank's proposers
    pb = shard.max_columns(n, world) * args.vlen if strong else 0
    lay = shard.slab_layout(n, shard.max_columns(n, world) if strong else pj, pb)
    slab = torch.zeros(lay["size"], dtype=torch.uint8, device=dev)
    eb.bind_outputs(slab[lay["valid"][0]:lay["valid"][0] + pj * n], slab[lay["ct_valid"][0]:lay["ct_valid"][0] + pj],
                    slab[lay["status"][0]:lay["status"][0] + 4 * pj].view(torch.int32),
                    slab[lay["plain"][0]:lay["plain"][1]] if pb else None)
    gathered = [None]
    t = ep["t"]
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]

    def step(events=None):
        eb.step(events)
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
    eb.check(lo)
    if strong:
        gv, gct, gst = shard.assemble(gathered[0].cpu().numpy(), n, world)
        full = np.random.default_rng(0x68626278_00000004).integers(0, args.corrupt_every, size=(n, n)) == 0
        full[:, OWN_INDEX] = False
        assert ((gv == 1) == ~full).all() and (gct == 1).all() and (gst == 0).all(), "gathered epoch result"
        plains = shard.assemble_plaintexts(gathered[0].cpu().numpy(), n, world, [args.vlen] * n, pb)
        assert plains == epoch_contributions(n, args.vlen), "gathered plaintexts"

    ms_epoch_ev = np.mean([ev[k][0].elapsed_time(ev[k][1]) for k in range(args.steps)])
    ms_step = elapsed / args.steps * 1e3
    verifies = n * n * (1 if strong else world) if args.shard_of <= 1 else pj * n
    value = verifies * args.steps / elapsed
    kern = eb.kernel_ms()
    ctx.set_timing(False)
    lanes = ctx.verify_lanes_used()
    kname = {1: "k_verify_shares_ml + k_fe1<0,1,3,5> (+ k_verify_shares for fallback lanes; one timed region)",
             2: "k_verify_shares2", 3: "k_verify_shares3", 6: "k_verify_shares6",
             7: "k_verify_shares (single kernel)"}.get(lanes, "k_verify_shares")
    traffic = traffic_record() if (n == 256 and pj == 256) else None
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
        "verify_lanes": lanes,
        "roofline": verify_roofline(pj * n, kern["verify_shares"], kname, traffic),
        "check": "validity bitmap == not-corrupted; plaintexts == contributions",
        "build": hbx_build_info(),
    }
    if key_ms is not None:
        res["era_key_broadcast_ms"] = key_ms
    if strong:
        # the gather of this epoch's result slab on its own (it is inside every timed step above)
        res["all_gather"] = {"ms": gather_ms(torch, dev, world, slab), "bytes_per_rank": int(lay["size"]),
                             "fields": "share status bytes (HBX_SHARE_*: the reference logs a FaultKind per share), "
                                       "ct status, combine status, plaintexts"}
    if world > 1 and strong and args.node_rate:
        # the node's rate with G whole epochs in flight, in the same line as the strong split
        res["node_rate"] = weak_epochs(args, dev, torch, world, rank, lambda: _WeakEpoch(args, dev, torch, Context, n))
    if world == 1 and args.in_flight > 1:
        res["epochs_in_flight"] = in_flight(args, eb, dev, torch, Context, verifies)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_dec(ep, args.cpu_seconds)
    ctx.close()
    if rank == 0 and world == 1 and args.shard_of <= 1 and args.configs:
        cfgs = {}
        for name in [c.strip().upper() for c in args.configs.split(",") if c.strip()]:
            fn = {"C1": config_c1, "C2": config_c2, "C4": config_c4, "C5": config_c5}.get(name)
            if fn is None:
                raise SystemExit(f"unknown config {name}")
            cfgs[name] = fn(args, dev, torch, Context)
        res["configs"] = cfgs
    if world > 1 and strong and args.configs:
        cfgs = {}
        for name in [c.strip().upper() for c in args.configs.split(",") if c.strip()]:
            fn = {"C4": sharded_c4, "C5": sharded_c5}.get(name)
            if fn is not None:  # C2 is a single-GPU config (BASELINE: "on 1 MI355X")
                cfgs[name] = fn(args, dev, torch, Context, world, rank)
        res["configs"] = cfgs
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
