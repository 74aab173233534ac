"""ctypes binding of the C ABI in ``include/hbx.h`` (``hbbft_amd/libhbx.so``).

This is plumbing for tests, the bench and Python callers; the product is the C ABI itself.
There is deliberately no CPU fallback: if ``libhbx.so`` is missing or no HIP device is present,
construction fails with an exception naming what is missing.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# HBX_LIB_PATH: an alternative in-tree build of the same library (kernel variants under test)
LIB_PATH = os.environ.get("HBX_LIB_PATH") or os.path.join(_HERE, "libhbx.so")

HBX_OK = 0
HBX_E_INVALID_ARG = -1
HBX_E_DEVICE = -2
HBX_E_NOT_ENOUGH_SHARES = -3
HBX_E_DUPLICATE_ENTRY = -4
HBX_E_NO_KEYS = -5
HBX_E_NO_CIPHERTEXTS = -6
HBX_E_INVALID_CIPHERTEXT = -7
HBX_E_OUT_OF_MEMORY = -8
HBX_E_TOO_FEW_SHARDS = -9
HBX_E_ROOT_MISMATCH = -10
HBX_E_NO_PAYLOAD = -11

# Every symbol include/hbx.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "hbx_ctx_create",
    "hbx_ctx_destroy",
    "hbx_last_error",
    "hbx_version",
    "hbx_set_pk_shares",
    "hbx_set_own_share",
    "hbx_prepare_ciphertexts",
    "hbx_verify_dec_shares",
    "hbx_combine_decrypt",
    "hbx_prepare_ciphertexts_d",
    "hbx_verify_dec_shares_d",
    "hbx_combine_decrypt_d",
    "hbx_get_ct_valid_d",
    "hbx_decrypt_epoch_d",
    "hbx_public_keys",
    "hbx_encrypt",
    "hbx_decrypt_shares",
    "hbx_prepare_nonces",
    "hbx_sign",
    "hbx_verify_sig_shares",
    "hbx_combine_signatures",
    "hbx_verify_sig_shares_d",
    "hbx_combine_signatures_d",
    "hbx_get_coin_lanes_used",
    "hbx_verify_sigs",
    "hbx_bivar_rows",
    "hbx_bivar_check_acks",
    "hbx_rs_encode_d",
    "hbx_rs_reconstruct_d",
    "hbx_merkle_roots_d",
    "hbx_merkle_validate_d",
    "hbx_broadcast_decode_d",
    "hbx_broadcast_decode_leaves_d",
    "hbx_set_timing",
    "hbx_kernel_time",
    "hbx_get_share_status",
    "hbx_get_ct_status",
    "hbx_get_sig_share_status",
    "hbx_get_ct_hashes",
    "hbx_set_digest",
    "hbx_set_merkle_digest",
    "hbx_set_verify_lanes",
    "hbx_get_verify_lanes_used",
    "hbx_set_combine_lanes",
    "hbx_debug_force_fallback",
    "hbx_get_fallback_lanes",
    "hbx_build_id",
    "hbx_merkle_node_count",
    "hbx_merkle_build_d",
    "hbx_merkle_proofs_d",
    "hbx_rs_encode",
    "hbx_rs_reconstruct",
    "hbx_merkle_roots",
    "hbx_merkle_build",
    "hbx_merkle_proofs",
    "hbx_merkle_validate",
    "hbx_broadcast_decode",
    "hbx_broadcast_decode_leaves",
)

DIGEST_SHA256 = 0
DIGEST_SHA3_256 = 1
MERKLE_SHA256 = 0
MERKLE_SHA3 = 1

# Per-share / per-ciphertext status bytes (include/hbx.h HBX_SHARE_*, HBX_CT_*)
SHARE_INVALID = 0
SHARE_VALID = 1
SHARE_ABSENT = 2
SHARE_UNDECODABLE = 3
SHARE_SKIPPED_CT = 4
SHARE_UNKNOWN_SENDER = 5
CT_INVALID = 0
CT_VALID = 1
CT_UNDECODABLE = 3

# kernel ids of hbx_kernel_time (include/hbx.h)
KERNELS = {"prepare_ct": 0, "prepare_lines": 1, "ct_checks": 2, "verify_shares": 3, "combine": 4,
           "verify_sig": 5, "combine_sigs": 6, "rs_code": 7, "merkle_leaves": 8, "hash_nonces": 9,
           "decode_sigs": 10}

_lib = None


class HbxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hbx error {code}: {msg}")
        self.code = code


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libhbx.so (raises OSError with the path if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same SONAME as
    # /opt/rocm's, which libhbx.so links).  Whichever loads first serves both; if libhbx.so came
    # first, torch later finds "No HIP GPUs".  So torch (the device-memory plumbing of the _d
    # calls) is imported before the library whenever it is installed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    u8p = ctypes.POINTER(ctypes.c_uint8)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    i32p = ctypes.POINTER(ctypes.c_int32)
    u32 = ctypes.c_uint32
    lib.hbx_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
    lib.hbx_ctx_destroy.argtypes = [P]
    lib.hbx_last_error.argtypes = [P]
    lib.hbx_last_error.restype = ctypes.c_char_p
    lib.hbx_version.restype = ctypes.c_char_p
    lib.hbx_build_id.restype = ctypes.c_char_p
    lib.hbx_set_pk_shares.argtypes = [P, u8p, u32, i32p]
    lib.hbx_set_own_share.argtypes = [P, u32, u8p]
    lib.hbx_prepare_ciphertexts.argtypes = [P, u8p, u8p, u64p, u8p, u32, u8p]
    lib.hbx_verify_dec_shares.argtypes = [P, u8p, u8p, u32, u32, u8p]
    lib.hbx_combine_decrypt.argtypes = [P, u32, u8p, i32p]
    lib.hbx_prepare_ciphertexts_d.argtypes = [P, P, P, P, P, u32, ctypes.c_uint64, P, P]
    lib.hbx_verify_dec_shares_d.argtypes = [P, P, P, u32, u32, P, P]
    lib.hbx_combine_decrypt_d.argtypes = [P, u32, P, P, P]
    lib.hbx_get_ct_valid_d.argtypes = [P, P, P]
    lib.hbx_decrypt_epoch_d.argtypes = [P, P, P, P, P, u32, ctypes.c_uint64, P, P, u32, u32, P, P, P, P, P]
    lib.hbx_prepare_nonces.argtypes = [P, u8p, u64p, u32, u8p]
    lib.hbx_sign.argtypes = [P, u8p, u32, u8p]
    lib.hbx_verify_sig_shares.argtypes = [P, u8p, u8p, u32, u32, u8p]
    lib.hbx_combine_signatures.argtypes = [P, u8p, u32, u8p, i32p, u8p, u8p]
    lib.hbx_verify_sig_shares_d.argtypes = [P, P, P, u32, u32, P, P]
    lib.hbx_combine_signatures_d.argtypes = [P, u8p, u32, P, P, P, P, P, P]
    lib.hbx_get_coin_lanes_used.argtypes = [P]
    lib.hbx_verify_sigs.argtypes = [P, u8p, u8p, u64p, u8p, u32, u8p]
    lib.hbx_bivar_rows.argtypes = [P, u8p, u32, u32, ctypes.c_uint64, u8p, u8p]
    lib.hbx_bivar_check_acks.argtypes = [P, u8p, u32, u32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32), u64p,
                                         u8p, u32, u8p]
    lib.hbx_rs_encode_d.argtypes = [P, P, u32, u32, u32, u32, P]
    lib.hbx_rs_reconstruct_d.argtypes = [P, P, P, u32, u32, u32, u32, P, P]
    lib.hbx_merkle_roots_d.argtypes = [P, P, u32, u32, u32, P, P]
    lib.hbx_merkle_validate_d.argtypes = [P, P, u32, P, P, P, P, P, P, u32, u32, P, P]
    lib.hbx_broadcast_decode_d.argtypes = [P, P, P, P, u32, u32, u32, u32, P, ctypes.c_uint64, P, P, P]
    lib.hbx_broadcast_decode_leaves_d.argtypes = [P, P, P, P, P, u32, u32, u32, u32, P, ctypes.c_uint64, P, P, P]
    lib.hbx_public_keys.argtypes = [P, u8p, u32, u8p]
    lib.hbx_encrypt.argtypes = [P, u8p, u8p, u64p, u32, u8p, u8p, u8p, u8p]
    lib.hbx_decrypt_shares.argtypes = [P, u8p, u32, u8p, u32, u8p]
    lib.hbx_set_timing.argtypes = [P, ctypes.c_int]
    lib.hbx_kernel_time.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
    lib.hbx_set_digest.argtypes = [P, ctypes.c_int]
    lib.hbx_set_merkle_digest.argtypes = [P, ctypes.c_int]
    lib.hbx_set_verify_lanes.argtypes = [P, ctypes.c_int]
    lib.hbx_get_verify_lanes_used.argtypes = [P]
    lib.hbx_set_combine_lanes.argtypes = [P, ctypes.c_int]
    lib.hbx_debug_force_fallback.argtypes = [P, u32]
    lib.hbx_get_fallback_lanes.argtypes = [P]
    lib.hbx_get_fallback_lanes.restype = ctypes.c_int64
    lib.hbx_merkle_node_count.argtypes = [u32]
    lib.hbx_merkle_node_count.restype = u32
    lib.hbx_merkle_build_d.argtypes = [P, P, u32, u32, u32, P, P, P]
    lib.hbx_merkle_proofs_d.argtypes = [P, P, u32, P, u32, P, P, P, P, P, P]
    # host-pointer Broadcast calls (numpy buffers; what a Rust FFI calls from Vec<u8>)
    lib.hbx_rs_encode.argtypes = [P, P, u32, u32, u32, u32]
    lib.hbx_rs_reconstruct.argtypes = [P, P, P, u32, u32, u32, u32, P]
    lib.hbx_merkle_roots.argtypes = [P, P, u32, u32, u32, P]
    lib.hbx_merkle_build.argtypes = [P, P, u32, u32, u32, P, P]
    lib.hbx_merkle_proofs.argtypes = [P, P, u32, u32, P, u32, P, P, P, P, P]
    lib.hbx_merkle_validate.argtypes = [P, P, u32, P, P, P, P, P, P, u32, u32, P]
    lib.hbx_broadcast_decode.argtypes = [P, P, P, P, u32, u32, u32, u32, P, ctypes.c_uint64, P, P]
    lib.hbx_broadcast_decode_leaves.argtypes = [P, P, P, P, P, u32, u32, u32, u32, P, ctypes.c_uint64, P, P]
    for name in ("hbx_get_share_status", "hbx_get_ct_status", "hbx_get_sig_share_status", "hbx_get_ct_hashes"):
        getattr(lib, name).argtypes = [P, u8p, ctypes.c_size_t]
    _lib = lib
    return lib


def build_info() -> dict:
    """Provenance of the loaded library: the source hash it was built from (hbx_build_id), the hash
    of the sources in this tree (hbbft_amd/buildinfo.py) and whether they match."""
    from . import buildinfo

    lib = load_library()
    built = lib.hbx_build_id().decode()
    tree = buildinfo.source_hash()
    return {"lib_source_sha256": built, "tree_source_sha256": tree, "match": built == tree,
            "lib": os.path.relpath(LIB_PATH, buildinfo.ROOT)}


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def pack_bits(bools) -> np.ndarray:
    a = np.asarray(bools, dtype=np.uint8).reshape(-1)
    return np.packbits(a, bitorder="little")


def unpack_bits(bits: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(np.asarray(bits, dtype=np.uint8), bitorder="little")[:n].astype(bool)


class Context:
    """One hbx context bound to a HIP device (``hbx_ctx_create``)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.hbx_ctx_create(device, ctypes.byref(h))
        if rc != HBX_OK:
            raise HbxError(rc, f"hbx_ctx_create(device={device}) failed: no usable HIP device?")
        self.h = h
        self.device = device
        self._v_off = None  # offsets of the prepared ciphertexts' V blob (host) ...
        self._d_off = None  # ... or the caller's device tensor of them (device API)

    def close(self):
        if getattr(self, "h", None):
            self.lib.hbx_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != HBX_OK:
            raise HbxError(rc, self.lib.hbx_last_error(self.h).decode())

    def set_digest(self, variant: int):
        """hbx_set_digest: DIGEST_SHA256 (default) or DIGEST_SHA3_256 for hash_g2 / hash_g1_g2 / hash_bytes."""
        self._check(self.lib.hbx_set_digest(self.h, variant))

    def set_verify_lanes(self, lanes: int):
        """hbx_set_verify_lanes: 0 auto (default), 1, 2, 3, 6 or 7 (one lane, single kernel) per check."""
        self._check(self.lib.hbx_set_verify_lanes(self.h, lanes))

    def verify_lanes_used(self) -> int:
        """hbx_get_verify_lanes_used: lanes per check of the last decryption-share launch."""
        return int(self.lib.hbx_get_verify_lanes_used(self.h))

    def debug_force_fallback(self, every: int):
        """hbx_debug_force_fallback (tests only): route every ``every``-th sender's one-lane check
        through the single-kernel fallback (0 = off)."""
        self._check(self.lib.hbx_debug_force_fallback(self.h, every))

    def fallback_lanes(self) -> int:
        """hbx_get_fallback_lanes: lanes of the last one-lane launch the fallback check decided."""
        v = int(self.lib.hbx_get_fallback_lanes(self.h))
        if v < 0:
            self._check(v)
        return v

    def set_combine_lanes(self, lanes: int):
        """hbx_set_combine_lanes: 0 auto (default), 1 (a lane per Lagrange term) or 4 (a quad per term)."""
        self._check(self.lib.hbx_set_combine_lanes(self.h, lanes))

    def set_merkle_digest(self, variant: int):
        """hbx_set_merkle_digest: MERKLE_SHA256 (default, afck merkle) or MERKLE_SHA3."""
        self._check(self.lib.hbx_set_merkle_digest(self.h, variant))

    # -- instrumentation -----------------------------------------------------------------------
    def set_timing(self, on: bool = True):
        """Bracket every launch of the timed kernels with HIP events on their stream."""
        self._check(self.lib.hbx_set_timing(self.h, 1 if on else 0))

    def kernel_time(self, name: str):
        """(total_ms, launches) of a timed kernel since the last set_timing call."""
        ms = ctypes.c_double()
        cnt = ctypes.c_uint32()
        self._check(self.lib.hbx_kernel_time(self.h, KERNELS[name], ctypes.byref(ms), ctypes.byref(cnt)))
        return ms.value, cnt.value

    # -- host API ------------------------------------------------------------------------------
    def set_pk_shares(self, pk_comp: Sequence[bytes]) -> np.ndarray:
        n = len(pk_comp)
        buf = np.frombuffer(b"".join(pk_comp), dtype=np.uint8).copy()
        st = np.zeros(n, dtype=np.int32)
        self._check(self.lib.hbx_set_pk_shares(self.h, _u8(buf), n, st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return st

    def prepare_ciphertexts(self, cts) -> np.ndarray:
        """cts: list of (u_comp48, v_bytes, w_comp96).  Returns bool[p] = Ciphertext::verify."""
        p = len(cts)
        u = np.frombuffer(b"".join(c[0] for c in cts), dtype=np.uint8).copy()
        w = np.frombuffer(b"".join(c[2] for c in cts), dtype=np.uint8).copy()
        off = np.zeros(p + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(c[1]) for c in cts])
        vb = np.frombuffer(b"".join(c[1] for c in cts) or b"\0", dtype=np.uint8).copy()
        bits = np.zeros((p + 7) // 8, dtype=np.uint8)
        self._check(self.lib.hbx_prepare_ciphertexts(
            self.h, _u8(u), _u8(vb), off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), _u8(w), p, _u8(bits)))
        self._v_off = off
        return unpack_bits(bits, p)

    def verify_dec_shares(self, shares: np.ndarray, present: Optional[np.ndarray] = None) -> np.ndarray:
        """shares: uint8[p, n, 48].  Returns bool[p, n]."""
        shares = np.ascontiguousarray(shares, dtype=np.uint8)
        p, n, _ = shares.shape
        pres = None if present is None else pack_bits(np.asarray(present, dtype=bool).reshape(-1))
        bits = np.zeros((p * n + 7) // 8, dtype=np.uint8)
        self._check(self.lib.hbx_verify_dec_shares(
            self.h, _u8(shares), None if pres is None else _u8(pres), n, p, _u8(bits)))
        return unpack_bits(bits, p * n).reshape(p, n)

    def combine_decrypt(self, t: int):
        """Returns (list of plaintext bytes or None, status int32[p])."""
        off = self._v_off
        if off is None:  # prepared through the device API: the caller's offsets tensor
            off = self._d_off.detach().cpu().numpy().astype(np.uint64)
        p = len(off) - 1
        out = np.zeros(max(int(off[-1]), 1), dtype=np.uint8)
        st = np.zeros(p, dtype=np.int32)
        self._check(self.lib.hbx_combine_decrypt(self.h, t, _u8(out), st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        res = []
        for j in range(p):
            res.append(out[int(off[j]):int(off[j + 1])].tobytes() if st[j] == HBX_OK else None)
        return res, st

    def share_status(self, p: int, n: int) -> np.ndarray:
        """HBX_SHARE_* byte of every share of the last verification -> uint8[p, n]."""
        out = np.zeros(p * n, dtype=np.uint8)
        self._check(self.lib.hbx_get_share_status(self.h, _u8(out), out.size))
        return out.reshape(p, n)

    def ct_status(self, p: int) -> np.ndarray:
        """HBX_CT_* byte of every prepared ciphertext -> uint8[p]."""
        out = np.zeros(p, dtype=np.uint8)
        self._check(self.lib.hbx_get_ct_status(self.h, _u8(out), out.size))
        return out

    def ct_hashes(self, p: int) -> np.ndarray:
        """Compressed H_j = hash_g1_g2(U_j, V_j) of the prepared ciphertexts -> uint8[p, 96]."""
        out = np.zeros(p * 96, dtype=np.uint8)
        self._check(self.lib.hbx_get_ct_hashes(self.h, _u8(out), p))
        return out.reshape(p, 96)

    def sig_share_status(self, count: int, n: int) -> np.ndarray:
        """HBX_SHARE_* byte of every signature share of the last hbx_verify_sig_shares."""
        out = np.zeros(count * n, dtype=np.uint8)
        self._check(self.lib.hbx_get_sig_share_status(self.h, _u8(out), out.size))
        return out.reshape(count, n)

    # -- producer side -------------------------------------------------------
    def public_keys(self, sk32: np.ndarray) -> np.ndarray:
        """sk32: uint8[n, 32] big-endian canonical scalars -> uint8[n, 48] compressed g1 * sk."""
        sk32 = np.ascontiguousarray(sk32, dtype=np.uint8)
        n = sk32.shape[0]
        out = np.zeros((n, 48), dtype=np.uint8)
        self._check(self.lib.hbx_public_keys(self.h, _u8(sk32), n, _u8(out)))
        return out

    def encrypt(self, pk48: bytes, msgs: Sequence[bytes], r32: np.ndarray):
        """PublicKey::encrypt for each message with randomness r32[j] -> list of (u48, v, w96)."""
        p = len(msgs)
        off = np.zeros(p + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(m) for m in msgs])
        mb = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
        vb = np.zeros_like(mb)
        u = np.zeros((p, 48), dtype=np.uint8)
        w = np.zeros((p, 96), dtype=np.uint8)
        pk = np.frombuffer(bytes(pk48), dtype=np.uint8).copy()
        r32 = np.ascontiguousarray(r32, dtype=np.uint8)
        self._check(self.lib.hbx_encrypt(self.h, _u8(pk), _u8(mb), off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                         p, _u8(r32), _u8(u), _u8(vb), _u8(w)))
        return [(u[j].tobytes(), vb[int(off[j]):int(off[j + 1])].tobytes(), w[j].tobytes()) for j in range(p)]

    def decrypt_shares(self, sk32: np.ndarray, u48: np.ndarray) -> np.ndarray:
        """shares[j, i] = sk_i * U_j compressed -> uint8[p, n, 48]."""
        sk32 = np.ascontiguousarray(sk32, dtype=np.uint8)
        u48 = np.ascontiguousarray(u48, dtype=np.uint8)
        n, p = sk32.shape[0], u48.shape[0]
        out = np.zeros((p, n, 48), dtype=np.uint8)
        self._check(self.lib.hbx_decrypt_shares(self.h, _u8(sk32), n, _u8(u48), p, _u8(out)))
        return out

    def set_own_share(self, me: int, sk32=None):
        """hbx_set_own_share: this node's index and 32-byte big-endian secret share (None clears)."""
        if sk32 is None:
            self._check(self.lib.hbx_set_own_share(self.h, 0, None))
            return
        sk = np.frombuffer(bytes(sk32), dtype=np.uint8).copy()
        assert sk.size == 32
        self._check(self.lib.hbx_set_own_share(self.h, me, _u8(sk)))

    # -- device API (torch tensors as HBM buffers; torch is plumbing only) -----------------------
    # stream=None enqueues on torch's current stream of the context's device (the C ABI's NULL is
    # the HIP null stream, which is what torch's default stream is), so the calls are ordered
    # with the tensor uploads and reads the caller did on that stream.
    def _stream(self, stream):
        if stream is not None:
            return stream
        import torch

        return torch.cuda.current_stream(self.device).cuda_stream

    def prepare_ciphertexts_d(self, d_u, d_v, d_off, d_w, p: int, max_v_len: int, d_ct_valid=None, stream=None):
        # the host combine_decrypt sizes its output from these offsets (read back when needed)
        self._v_off, self._d_off = None, d_off
        self._check(self.lib.hbx_prepare_ciphertexts_d(
            self.h, d_u.data_ptr(), d_v.data_ptr(), d_off.data_ptr(), d_w.data_ptr(), p, max_v_len,
            None if d_ct_valid is None else d_ct_valid.data_ptr(), self._stream(stream)))

    def verify_dec_shares_d(self, d_shares, n: int, p: int, d_valid=None, d_present=None, stream=None):
        self._check(self.lib.hbx_verify_dec_shares_d(
            self.h, d_shares.data_ptr(), None if d_present is None else d_present.data_ptr(), n, p,
            None if d_valid is None else d_valid.data_ptr(), self._stream(stream)))

    # -- common coin ------------------------------------------------------------------------------
    def prepare_nonces(self, nonces: Sequence[bytes], hashes: bool = True) -> Optional[np.ndarray]:
        """hash_g2 of every nonce; returns uint8[count, 96] compressed points, or None with
        ``hashes=False`` -- then the call returns after its uploads, the share checks and the
        combine do not wait for the true H (only hbx_sign does), and the hashing runs on."""
        count = len(nonces)
        off = np.zeros(count + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(x) for x in nonces])
        blob = np.frombuffer(b"".join(nonces) or b"\0", dtype=np.uint8).copy()
        h = np.zeros((count, 96), dtype=np.uint8) if hashes else None
        self._check(self.lib.hbx_prepare_nonces(self.h, _u8(blob), off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                count, _u8(h) if hashes else None))
        self._coin_count = count
        return h

    def sign(self, sk32: np.ndarray) -> np.ndarray:
        """uint8[n, 32] scalars -> uint8[count, n, 96] signature shares of the prepared nonces."""
        sk32 = np.ascontiguousarray(sk32, dtype=np.uint8)
        n = sk32.shape[0]
        out = np.zeros((self._coin_count, n, 96), dtype=np.uint8)
        self._check(self.lib.hbx_sign(self.h, _u8(sk32), n, _u8(out)))
        return out

    def verify_sig_shares(self, sigs: np.ndarray, present: Optional[np.ndarray] = None) -> np.ndarray:
        """sigs: uint8[count, n, 96] -> bool[count, n]."""
        sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
        count, n, _ = sigs.shape
        pres = None if present is None else pack_bits(np.asarray(present, dtype=bool).reshape(-1))
        bits = np.zeros((count * n + 7) // 8, dtype=np.uint8)
        self._check(self.lib.hbx_verify_sig_shares(self.h, _u8(sigs), None if pres is None else _u8(pres), n, count,
                                                   _u8(bits)))
        return unpack_bits(bits, count * n).reshape(count, n)

    def coin_lanes_used(self) -> int:
        """hbx_get_coin_lanes_used: lanes per check of the last signature-share verification."""
        return int(self.lib.hbx_get_coin_lanes_used(self.h))

    def verify_sig_shares_d(self, d_sigs, d_present=None, d_status=None, stream=None):
        """d_sigs: uint8[count, n, 96] device tensor; d_present / d_status: uint8[count, n] (or None)."""
        import torch

        count, n, w = d_sigs.shape
        if w != 96 or d_sigs.dtype != torch.uint8 or not d_sigs.is_contiguous():
            raise ValueError("verify_sig_shares_d: d_sigs must be contiguous uint8[count, n, 96]")
        for x in (d_present, d_status):
            if x is not None and (tuple(x.shape) != (count, n) or x.dtype != torch.uint8 or not x.is_contiguous()):
                raise ValueError(f"verify_sig_shares_d: present/status must be contiguous uint8[{count}, {n}]")
        opt = lambda x: None if x is None else x.data_ptr()  # noqa: E731
        self._check(self.lib.hbx_verify_sig_shares_d(self.h, d_sigs.data_ptr(), opt(d_present), n, count,
                                                     opt(d_status), self._stream(stream)))

    def combine_signatures_d(self, master_pk48: bytes, t: int, d_use=None, d_sig=None, d_status=None, d_ok=None,
                             d_parity=None, stream=None):
        """hbx_combine_signatures_d: d_use uint8[count, n] (or None: every valid share)."""
        mpk = np.frombuffer(bytes(master_pk48), dtype=np.uint8).copy()
        opt = lambda x: None if x is None else x.data_ptr()  # noqa: E731
        self._check(self.lib.hbx_combine_signatures_d(self.h, _u8(mpk), t, opt(d_use), opt(d_sig), opt(d_status),
                                                      opt(d_ok), opt(d_parity), self._stream(stream)))

    def combine_signatures(self, master_pk48: bytes, t: int):
        """-> (sig uint8[count, 96], status int32[count], master_ok bool[count], parity bool[count])."""
        count = self._coin_count
        sig = np.zeros((count, 96), dtype=np.uint8)
        st = np.zeros(count, dtype=np.int32)
        ok = np.zeros((count + 7) // 8, dtype=np.uint8)
        par = np.zeros((count + 7) // 8, dtype=np.uint8)
        mpk = np.frombuffer(bytes(master_pk48), dtype=np.uint8).copy()
        self._check(self.lib.hbx_combine_signatures(self.h, _u8(mpk), t, _u8(sig),
                                                    st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _u8(ok), _u8(par)))
        return sig, st, unpack_bits(ok, count), unpack_bits(par, count)

    def verify_sigs(self, pk48: np.ndarray, msgs, sig96: np.ndarray) -> np.ndarray:
        """PublicKey::verify(sig_i, msg_i) for independent items (DHB votes, key-generation
        messages): pk48 uint8[count, 48], msgs = list of bytes, sig96 uint8[count, 96] ->
        HBX_SHARE_* status uint8[count] (VALID / INVALID / UNDECODABLE)."""
        pk48 = np.ascontiguousarray(pk48, dtype=np.uint8)
        sig96 = np.ascontiguousarray(sig96, dtype=np.uint8)
        count = pk48.shape[0]
        if len(msgs) != count or sig96.shape[0] != count:
            raise ValueError("verify_sigs: pk48, msgs and sig96 must have the same count")
        off = np.zeros(count + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(m) for m in msgs])
        blob = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
        out = np.zeros(count, dtype=np.uint8)
        self._check(self.lib.hbx_verify_sigs(self.h, _u8(pk48), _u8(blob),
                                             off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), _u8(sig96), count,
                                             _u8(out)))
        return out

    def bivar_rows(self, commits: np.ndarray, t: int, x: int):
        """BivarCommitment::row(x) of p commitments uint8[p, (t+1)(t+2)/2, 48] ->
        (rows uint8[p, t + 1, 48], status uint8[p])."""
        commits = np.ascontiguousarray(commits, dtype=np.uint8)
        p = commits.shape[0]
        rows = np.zeros((p, t + 1, 48), dtype=np.uint8)
        st = np.zeros(p, dtype=np.uint8)
        self._check(self.lib.hbx_bivar_rows(self.h, _u8(commits), p, t, x, _u8(rows), _u8(st)))
        return rows, st

    def bivar_check_acks(self, commits: np.ndarray, t: int, x: int, proposer, y, vals32: np.ndarray) -> np.ndarray:
        """handle_ack's check commit[proposer].evaluate(x, y) == g1 * val -> HBX_SHARE_* uint8[count]."""
        commits = np.ascontiguousarray(commits, dtype=np.uint8)
        pr = np.ascontiguousarray(proposer, dtype=np.uint32)
        yy = np.ascontiguousarray(y, dtype=np.uint64)
        vals32 = np.ascontiguousarray(vals32, dtype=np.uint8)
        out = np.zeros(len(pr), dtype=np.uint8)
        self._check(self.lib.hbx_bivar_check_acks(self.h, _u8(commits), commits.shape[0], t, x,
                                                  pr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                  yy.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), _u8(vals32),
                                                  len(pr), _u8(out)))
        return out

    # -- broadcast (torch tensors as HBM buffers) ------------------------------------------------
    def rs_encode_d(self, d_shards, k: int, m: int, stream=None):
        """d_shards: uint8[inst, k + m, L] (parity rows overwritten)."""
        inst, n, L = d_shards.shape
        if n != k + m:
            raise ValueError(f"rs_encode_d: {n} shards per instance != k + m = {k + m}")
        self._check(self.lib.hbx_rs_encode_d(self.h, d_shards.data_ptr(), inst, k, m, L, self._stream(stream)))

    def rs_reconstruct_d(self, d_shards, d_present, d_status, k: int, m: int, stream=None):
        inst, n, L = d_shards.shape
        if n != k + m:
            raise ValueError(f"rs_reconstruct_d: {n} shards per instance != k + m = {k + m}")
        self._check(self.lib.hbx_rs_reconstruct_d(self.h, d_shards.data_ptr(), d_present.data_ptr(), inst, k, m, L,
                                                  d_status.data_ptr(), self._stream(stream)))

    def merkle_roots_d(self, d_shards, d_roots, stream=None):
        inst, n, L = d_shards.shape
        self._check(self.lib.hbx_merkle_roots_d(self.h, d_shards.data_ptr(), inst, n, L, d_roots.data_ptr(), self._stream(stream)))

    def merkle_validate_d(self, d_values, d_nodes, d_sibs, d_sides, d_depth, d_root, d_sender, count: int, d_valid,
                          stream=None):
        nproofs, vlen = d_values.shape
        self._check(self.lib.hbx_merkle_validate_d(
            self.h, d_values.data_ptr(), vlen, d_nodes.data_ptr(), d_sibs.data_ptr(), d_sides.data_ptr(),
            d_depth.data_ptr(), d_root.data_ptr(), d_sender.data_ptr(), count, nproofs, d_valid.data_ptr(), self._stream(stream)))

    # -- Broadcast on host buffers (numpy; no device memory on the caller's side) ----------------
    @staticmethod
    def _host(a, dtype, shape=None, writable=False):
        """A C-contiguous numpy array of `dtype` (and `shape`), in place when it already is one."""
        if not isinstance(a, np.ndarray) or a.dtype != dtype or not a.flags["C_CONTIGUOUS"]:
            if writable:
                raise ValueError(f"need a C-contiguous {np.dtype(dtype)} numpy array (written in place)")
            a = np.ascontiguousarray(a, dtype=dtype)
        if shape is not None and tuple(a.shape) != tuple(shape):
            raise ValueError(f"expected shape {tuple(shape)}, got {tuple(a.shape)}")
        return a

    def rs_encode(self, shards: np.ndarray, k: int, m: int):
        """hbx_rs_encode: shards uint8[inst, k + m, L] on the host, parity rows written in place."""
        shards = self._host(shards, np.uint8, writable=True)
        inst, n, L = shards.shape
        if n != k + m:  # the library copies (k + m) L bytes per instance each way
            raise ValueError(f"rs_encode: {n} shards per instance != k + m = {k + m}")
        self._check(self.lib.hbx_rs_encode(self.h, shards.ctypes.data, inst, k, m, L))

    def rs_reconstruct(self, shards: np.ndarray, present, k: int, m: int) -> np.ndarray:
        """hbx_rs_reconstruct: shards rebuilt in place; returns status int32[inst]."""
        shards = self._host(shards, np.uint8, writable=True)
        inst, n, L = shards.shape
        if n != k + m:  # the library copies (k + m) L bytes per instance each way
            raise ValueError(f"rs_reconstruct: {n} shards per instance != k + m = {k + m}")
        pres = self._host(present, np.uint8, (inst, n))
        st = np.zeros(inst, dtype=np.int32)
        self._check(self.lib.hbx_rs_reconstruct(self.h, shards.ctypes.data, pres.ctypes.data, inst, k, m, L,
                                                st.ctypes.data))
        return st

    def merkle_roots(self, shards) -> np.ndarray:
        shards = self._host(shards, np.uint8)
        inst, n, L = shards.shape
        roots = np.zeros((inst, 32), dtype=np.uint8)
        self._check(self.lib.hbx_merkle_roots(self.h, shards.ctypes.data, inst, n, L, roots.ctypes.data))
        return roots

    def merkle_build(self, shards):
        """hbx_merkle_build -> (nodes uint8[inst, node_count(n), 32], roots uint8[inst, 32])."""
        shards = self._host(shards, np.uint8)
        inst, n, L = shards.shape
        nodes = np.zeros((inst, self.merkle_node_count(n), 32), dtype=np.uint8)
        roots = np.zeros((inst, 32), dtype=np.uint8)
        self._check(self.lib.hbx_merkle_build(self.h, shards.ctypes.data, inst, n, L, nodes.ctypes.data,
                                              roots.ctypes.data))
        return nodes, roots

    def merkle_proofs(self, nodes, n: int, req):
        """hbx_merkle_proofs: req uint32[count, 2] = (instance, leaf) -> (node_hash, sib_hash, sides,
        depth, root) as hbx_merkle_validate takes them."""
        nodes = self._host(nodes, np.uint8)
        inst = nodes.shape[0]
        req = self._host(req, np.uint32)
        if req.ndim != 2 or req.shape[1] != 2:  # the library reads req[2 q], req[2 q + 1] for q < count
            raise ValueError(f"merkle_proofs: req must be uint32[count, 2] (instance, leaf), got shape {req.shape}")
        count = req.shape[0]
        nh = np.zeros((count, 17, 32), dtype=np.uint8)
        sh = np.zeros((count, 16, 32), dtype=np.uint8)
        sides = np.zeros(count, dtype=np.uint32)
        depth = np.zeros(count, dtype=np.uint32)
        root = np.zeros((count, 32), dtype=np.uint8)
        self._check(self.lib.hbx_merkle_proofs(self.h, nodes.ctypes.data, inst, n, req.ctypes.data, count,
                                               nh.ctypes.data, sh.ctypes.data, sides.ctypes.data, depth.ctypes.data,
                                               root.ctypes.data))
        return nh, sh, sides, depth, root

    def merkle_validate(self, values, nodes, sibs, sides, depth, root, sender, count: int) -> np.ndarray:
        """hbx_merkle_validate: returns valid uint8[nproofs]."""
        values = self._host(values, np.uint8)
        nproofs, vlen = values.shape
        args = [self._host(nodes, np.uint8, (nproofs, 17, 32)), self._host(sibs, np.uint8, (nproofs, 16, 32)),
                self._host(sides, np.uint32, (nproofs,)), self._host(depth, np.uint32, (nproofs,)),
                self._host(root, np.uint8, (nproofs, 32)), self._host(sender, np.uint32, (nproofs,))]
        valid = np.zeros(nproofs, dtype=np.uint8)
        self._check(self.lib.hbx_merkle_validate(self.h, values.ctypes.data, vlen, *[a.ctypes.data for a in args],
                                                 count, nproofs, valid.ctypes.data))
        return valid

    def broadcast_decode(self, shards, present, root, k: int, m: int, leaf_hash=None):
        """hbx_broadcast_decode[_leaves]: shards rebuilt in place -> (out uint8[inst, k L], out_len
        uint64[inst], status int32[inst])."""
        shards = self._host(shards, np.uint8, writable=True)
        inst, n, L = shards.shape
        if n != k + m:
            raise ValueError(f"broadcast_decode: {n} shards per instance != k + m = {k + m}")
        pres = self._host(present, np.uint8, (inst, n))
        root = self._host(root, np.uint8, (inst, 32))
        stride = max(k * L, 1)
        out = np.zeros((inst, stride), dtype=np.uint8)
        out_len = np.zeros(inst, dtype=np.uint64)
        st = np.zeros(inst, dtype=np.int32)
        if leaf_hash is None:
            self._check(self.lib.hbx_broadcast_decode(self.h, shards.ctypes.data, pres.ctypes.data, root.ctypes.data,
                                                      inst, k, m, L, out.ctypes.data, stride, out_len.ctypes.data,
                                                      st.ctypes.data))
        else:
            lh = self._host(leaf_hash, np.uint8, (inst, n, 32))
            self._check(self.lib.hbx_broadcast_decode_leaves(self.h, shards.ctypes.data, pres.ctypes.data,
                                                             lh.ctypes.data, root.ctypes.data, inst, k, m, L,
                                                             out.ctypes.data, stride, out_len.ctypes.data,
                                                             st.ctypes.data))
        return out, out_len, st

    def merkle_node_count(self, n: int) -> int:
        return int(self.lib.hbx_merkle_node_count(n))

    def merkle_build_d(self, d_shards, d_nodes, d_roots=None, stream=None):
        inst, n, L = d_shards.shape
        self._check(self.lib.hbx_merkle_build_d(self.h, d_shards.data_ptr(), inst, n, L, d_nodes.data_ptr(),
                                                None if d_roots is None else d_roots.data_ptr(), self._stream(stream)))

    def merkle_proofs_d(self, d_nodes, n: int, d_req, d_node_hash, d_sib_hash, d_sides, d_depth, d_root, stream=None):
        count = d_req.shape[0]
        self._check(self.lib.hbx_merkle_proofs_d(self.h, d_nodes.data_ptr(), n, d_req.data_ptr(), count,
                                                 d_node_hash.data_ptr(), d_sib_hash.data_ptr(), d_sides.data_ptr(),
                                                 d_depth.data_ptr(), d_root.data_ptr(), self._stream(stream)))

    def broadcast_decode_d(self, d_shards, d_present, d_root, k: int, m: int, d_out, d_out_len, d_status, stream=None):
        inst, n, L = d_shards.shape
        self._check(self.lib.hbx_broadcast_decode_d(
            self.h, d_shards.data_ptr(), d_present.data_ptr(), d_root.data_ptr(), inst, k, m, L, d_out.data_ptr(),
            d_out.shape[1], d_out_len.data_ptr(), d_status.data_ptr(), self._stream(stream)))

    def broadcast_decode_leaves_d(self, d_shards, d_present, d_leaf_hash, d_root, k: int, m: int, d_out, d_out_len,
                                  d_status, stream=None):
        """hbx_broadcast_decode_leaves_d: d_leaf_hash uint8[inst, k + m, 32] = the present shards'
        leaf digests from their validated Echo proofs."""
        import torch

        inst, n, L = d_shards.shape
        # k_import_leaf_hashes reads inst * (k + m) * 32 bytes from this pointer, and the root check
        # trusts them: the layout must be exactly that
        if n != k + m:
            raise ValueError(f"broadcast_decode_leaves_d: {n} shards per instance != k + m = {k + m}")
        if (tuple(d_leaf_hash.shape) != (inst, n, 32) or d_leaf_hash.dtype != torch.uint8
                or not d_leaf_hash.is_contiguous()):
            raise ValueError(f"broadcast_decode_leaves_d: d_leaf_hash must be contiguous uint8[{inst}, {n}, 32], "
                             f"got {d_leaf_hash.dtype}{list(d_leaf_hash.shape)}")
        self._check(self.lib.hbx_broadcast_decode_leaves_d(
            self.h, d_shards.data_ptr(), d_present.data_ptr(), d_leaf_hash.data_ptr(), d_root.data_ptr(), inst, k, m,
            L, d_out.data_ptr(), d_out.shape[1], d_out_len.data_ptr(), d_status.data_ptr(), self._stream(stream)))

    def get_ct_valid_d(self, d_ct_valid, stream=None):
        self._check(self.lib.hbx_get_ct_valid_d(self.h, d_ct_valid.data_ptr(), self._stream(stream)))

    def combine_decrypt_d(self, t: int, d_out, d_status=None, stream=None):
        self._check(self.lib.hbx_combine_decrypt_d(
            self.h, t, d_out.data_ptr(), None if d_status is None else d_status.data_ptr(), self._stream(stream)))

    def decrypt_epoch_d(self, d_u, d_v, d_off, d_w, p: int, max_v_len: int, d_shares, n: int, t: int, d_out,
                        d_valid=None, d_ct_valid=None, d_status=None, d_present=None, stream=None):
        """One node-epoch (hbx_decrypt_epoch_d): prepare + share checks (with Ciphertext::verify) +
        combine + decrypt; same results as the three-call sequence."""
        opt = lambda x: None if x is None else x.data_ptr()  # noqa: E731
        self._v_off, self._d_off = None, d_off
        self._check(self.lib.hbx_decrypt_epoch_d(
            self.h, d_u.data_ptr(), d_v.data_ptr(), d_off.data_ptr(), d_w.data_ptr(), p, max_v_len,
            d_shares.data_ptr(), opt(d_present), n, t, opt(d_valid), opt(d_ct_valid), d_out.data_ptr(),
            opt(d_status), self._stream(stream)))
