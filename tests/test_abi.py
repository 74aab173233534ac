"""The C-ABI library (hbbft_amd/libhbx.so) loads and exports every symbol include/hbx.h declares.
No compute call is made here (no GPU in the CPU suite)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hbx.h")
LIB = os.path.join(ROOT, "hbbft_amd", "libhbx.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hbx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared_functions()
    from hbbft_amd import hbx

    assert names == sorted(hbx.EXPORTS)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhbx.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    lib.hbx_version.restype = ctypes.c_char_p
    assert lib.hbx_version().decode().startswith("hbx ")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhbx.so not built")
def test_no_silent_cpu_fallback_without_device():
    """Without a HIP device the product must fail loudly, never compute on the CPU."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from hbbft_amd.hbx import Context, HbxError

    with pytest.raises(HbxError):
        Context(0)


def test_shard_layout():
    from hbbft_amd import shard

    assert shard.proposer_range(256, 8, 3) == (96, 128)
    # N % G != 0: balanced contiguous ranges covering every proposer once
    assert [shard.proposer_range(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    with pytest.raises(ValueError):
        shard.proposer_range(10, 4, 4)
    lay = shard.slab_layout(256, 32)
    assert lay["size"] == 256 * 32 + 32 + 128


@pytest.mark.skipif(not os.path.exists(LIB), reason="libhbx.so not built")
def test_library_was_built_from_these_sources():
    """Provenance: the shipped library carries the SHA-256 of the sources it was
    built from (hbx_build_id, compiled in by tools/build.py); it must be this tree's."""
    from hbbft_amd import buildinfo

    lib = ctypes.CDLL(LIB)
    lib.hbx_build_id.restype = ctypes.c_char_p
    assert lib.hbx_build_id().decode() == buildinfo.source_hash()


class _NoLib:
    """Stands in for a Context's library: any call is a test failure (the guards must fire first)."""

    def __getattr__(self, name):
        raise AssertionError(f"{name} reached the library with mismatched arguments")


def _bare_context():
    from hbbft_amd import hbx

    ctx = object.__new__(hbx.Context)  # no device: only the argument checks run
    ctx.lib, ctx.h = _NoLib(), None
    return ctx


@pytest.mark.parametrize("k,m", [(3, 2), (2, 2), (4, 3)])
def test_rs_host_forms_reject_shard_count_mismatch(k, m):
    """hbx_rs_encode / hbx_rs_reconstruct copy (k + m) L bytes per instance each way, so
    a buffer with n != k + m shards must be refused before the call (a ValueError, not an assert)."""
    import numpy as np

    ctx = _bare_context()
    shards = np.zeros((1, 5, 8), dtype=np.uint8)
    if k + m == 5:
        pytest.skip("matching shape")
    with pytest.raises(ValueError, match="k \\+ m"):
        ctx.rs_encode(shards, k, m)
    with pytest.raises(ValueError, match="k \\+ m"):
        ctx.rs_reconstruct(shards, np.ones((1, 5), dtype=np.uint8), k, m)


@pytest.mark.parametrize("shape", [(6,), (3, 3), (2, 2, 2)])
def test_merkle_proofs_rejects_malformed_requests(shape):
    """hbx_merkle_proofs reads req[2 q], req[2 q + 1] for q < count; only uint32[count, 2]
    is accepted."""
    import numpy as np

    ctx = _bare_context()
    nodes = np.zeros((1, 7, 32), dtype=np.uint8)
    with pytest.raises(ValueError, match="count, 2"):
        ctx.merkle_proofs(nodes, 4, np.zeros(shape, dtype=np.uint32))
