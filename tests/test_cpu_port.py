"""The CPU baseline port (tools/cpu_baseline/cpu_port.cpp, bench.py's cpu_baseline leg) computes the
same verify_decryption_share bits as the oracle fixtures: it times the real algorithm, not a stub."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def port(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cpuport") / "libcpu_port.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-o", out,
                           os.path.join(ROOT, "tools", "cpu_baseline", "cpu_port.cpp")])
    lib = ctypes.CDLL(out)
    P = ctypes.c_void_p
    lib.cpu_verify_dec_shares.argtypes = [P, ctypes.c_uint32, P, P, P, P, P, P, ctypes.c_uint32, ctypes.c_int, P]
    return lib


@pytest.mark.parametrize("n", [4, 7])
def test_port_matches_fixture(port, n):
    d = dict(np.load(os.path.join(ROOT, "tests", "golden", f"hb_epoch_n{n}.npz"), allow_pickle=False))
    p = len(d["v_off"]) - 1
    nn = d["shares"].shape[1]
    # shares that reach a verification (not absent, decodable, ciphertext valid)
    jobs = [(j, i) for j in range(p) for i in range(nn) if d["expect_share_status"][j, i] in (0, 1)]
    assert jobs
    J = np.array(jobs, dtype=np.uint32)
    out = np.zeros(len(jobs), dtype=np.uint8)
    arrs = [np.ascontiguousarray(d[k], dtype=np.uint8) for k in ("pk_comp", "u", "v_blob", "w", "shares")]
    off = np.ascontiguousarray(d["v_off"], dtype=np.uint64)
    port.cpu_verify_dec_shares(arrs[0].ctypes.data, nn, arrs[1].ctypes.data, arrs[2].ctypes.data, off.ctypes.data,
                               arrs[3].ctypes.data, arrs[4].ctypes.data, J.ctypes.data, len(jobs), 2, out.ctypes.data)
    expect = np.array([d["expect_valid"][j, i] for j, i in jobs])
    np.testing.assert_array_equal(out.astype(bool), expect)


@pytest.mark.parametrize("n", [4, 7, 10])
def test_fused_port_matches_fixture(port, n):
    """CPU baseline row (b): hoisted hash_g1_g2 + one two-pair Miller loop + one final
    exponentiation per share gives the fixture's bits."""
    port.cpu_verify_dec_shares_fused.argtypes = [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 5 + \
        [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
    d = dict(np.load(os.path.join(ROOT, "tests", "golden", f"hb_epoch_n{n}.npz"), allow_pickle=False))
    p = len(d["v_off"]) - 1
    nn = d["shares"].shape[1]
    jobs = [(j, i) for j in range(p) for i in range(nn) if d["expect_share_status"][j, i] in (0, 1)]
    J = np.array(jobs, dtype=np.uint32)
    out = np.zeros(len(jobs), dtype=np.uint8)
    arrs = [np.ascontiguousarray(d[k], dtype=np.uint8) for k in ("pk_comp", "u", "v_blob", "w", "shares")]
    off = np.ascontiguousarray(d["v_off"], dtype=np.uint64)
    port.cpu_verify_dec_shares_fused(arrs[0].ctypes.data, nn, arrs[1].ctypes.data, arrs[2].ctypes.data,
                                     off.ctypes.data, arrs[3].ctypes.data, arrs[4].ctypes.data, p, J.ctypes.data,
                                     len(jobs), 3, out.ctypes.data)
    expect = np.array([d["expect_valid"][j, i] for j, i in jobs])
    np.testing.assert_array_equal(out.astype(bool), expect)


def _coin_args(port):
    P, u32 = ctypes.c_void_p, ctypes.c_uint32
    port.cpu_verify_sig_shares.argtypes = [P, u32, P, P, u32, P, P, u32, ctypes.c_int, ctypes.c_int, P]
    port.cpu_combine_sigs.argtypes = [P, P, u32, u32, u32, P, P, P, ctypes.c_int, P, P]


@pytest.mark.parametrize("fused", [0, 1])
def test_coin_port_matches_fixture(port, fused):
    """CPU baseline row C4: PublicKeyShare::verify bits (both shapes), then the combine, master
    check and parity of the fixture."""
    _coin_args(port)
    d = dict(np.load(os.path.join(ROOT, "tests", "golden", "coin_n7.npz"), allow_pickle=False))
    inst, n = d["sigs"].shape[:2]
    st = d["expect_share_status"]
    jobs = [(j, i) for j in range(inst) for i in range(n) if st[j, i] in (0, 1)]
    J = np.array(jobs, dtype=np.uint32)
    out = np.zeros(len(jobs), dtype=np.uint8)
    pk = np.ascontiguousarray(d["pk_comp"], dtype=np.uint8)
    blob = np.ascontiguousarray(d["nonce_blob"], dtype=np.uint8)
    off = np.ascontiguousarray(d["nonce_off"], dtype=np.uint64)
    sig = np.ascontiguousarray(d["sigs"], dtype=np.uint8)
    port.cpu_verify_sig_shares(pk.ctypes.data, n, blob.ctypes.data, off.ctypes.data, inst, sig.ctypes.data,
                               J.ctypes.data, len(jobs), 2, fused, out.ctypes.data)
    np.testing.assert_array_equal(out.astype(bool), np.array([d["expect_valid"][j, i] for j, i in jobs]))
    valid = np.ascontiguousarray(st == 1, dtype=np.uint8)
    ok = np.zeros(inst, dtype=np.uint8)
    par = np.zeros(inst, dtype=np.uint8)
    mpk = np.ascontiguousarray(d["master_pk"], dtype=np.uint8)
    assert port.cpu_combine_sigs(sig.ctypes.data, valid.ctypes.data, n, inst, int(d["t"]), mpk.ctypes.data,
                                 blob.ctypes.data, off.ctypes.data, 2, ok.ctypes.data, par.ctypes.data) == 0
    good = d["expect_status"] == 0
    np.testing.assert_array_equal(ok.astype(bool)[good], d["expect_master_ok"][good])
    np.testing.assert_array_equal(par.astype(bool)[good], d["expect_parity"][good])


@pytest.mark.parametrize("n", [4, 13, 40])
def test_rs_port_matches_oracle(port, n):
    """CPU baseline row C5: reed-solomon-erasure's encode and reconstruct (first k present rows)."""
    from oracle import rs_merkle as rm

    P, u32 = ctypes.c_void_p, ctypes.c_uint32
    port.cpu_rs_encode.argtypes = [P, u32, u32, u32, u32, ctypes.c_int]
    port.cpu_rs_reconstruct.argtypes = [P, P, u32, u32, u32, u32, ctypes.c_int, P]
    k, m = rm.coding_counts(n)
    rng = np.random.default_rng(n)
    inst, L = 3, 37
    buf = np.zeros((inst, n, L), dtype=np.uint8)
    buf[:, :k] = rng.integers(0, 256, size=(inst, k, L), dtype=np.uint8)
    want = np.stack([rm.ReedSolomon(k, m).encode(buf[j]) for j in range(inst)])
    port.cpu_rs_encode(buf.ctypes.data, inst, k, m, L, 2)
    np.testing.assert_array_equal(buf, want)
    present = np.ones((inst, n), dtype=np.uint8)
    present[0, n - m:] = 0            # parity missing
    present[1, :m] = 0                # data missing
    present[2, rng.permutation(n)[:m]] = 0
    work = buf.copy()
    work[present == 0] = 0
    status = np.zeros(inst, dtype=np.int32)
    port.cpu_rs_reconstruct(work.ctypes.data, present.ctypes.data, inst, k, m, L, 2, status.ctypes.data)
    assert (status == 0).all()
    np.testing.assert_array_equal(work, want)


@pytest.mark.parametrize("n", [4, 7, 10])
def test_combine_decrypt_port_matches_fixture(port, n):
    """CPU baseline row C3 (verify + combine): PublicKeySet::decrypt over the first t valid shares
    gives the fixture's plaintexts and NotEnoughShares statuses."""
    P, u32 = ctypes.c_void_p, ctypes.c_uint32
    port.cpu_combine_decrypt.argtypes = [P, P, u32, u32, u32, P, P, ctypes.c_int, P, P]
    d = dict(np.load(os.path.join(ROOT, "tests", "golden", f"hb_epoch_n{n}.npz"), allow_pickle=False))
    p = len(d["v_off"]) - 1
    nn = d["shares"].shape[1]
    sh = np.ascontiguousarray(d["shares"], dtype=np.uint8)
    valid = np.ascontiguousarray(d["expect_valid"], dtype=np.uint8)
    v = np.ascontiguousarray(d["v_blob"], dtype=np.uint8)
    off = np.ascontiguousarray(d["v_off"], dtype=np.uint64)
    out = np.zeros_like(v)
    st = np.zeros(p, dtype=np.int32)
    assert port.cpu_combine_decrypt(sh.ctypes.data, valid.ctypes.data, nn, p, int(d["t"]), v.ctypes.data,
                                    off.ctypes.data, 2, out.ctypes.data, st.ctypes.data) == 0
    ok = d["expect_ct_valid"].astype(bool)
    np.testing.assert_array_equal(st[ok], d["expect_status"][ok])
    for j in range(p):
        if ok[j] and d["expect_status"][j] == 0:
            a, b = int(off[j]), int(off[j + 1])
            assert out[a:b].tobytes() == d["expect_plain_blob"][a:b].tobytes(), j
