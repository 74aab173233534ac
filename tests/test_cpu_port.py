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
