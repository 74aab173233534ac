"""Build provenance of libhbx.so.

``source_hash()`` is a SHA-256 over the sources a libhbx.so build reads: the HIP sources and headers
under ``hbbft_amd/csrc`` (not the generated ``_kdecl.hpp``), ``include/hbx.h`` and
``tools/build.py`` (which holds the compile flags).  ``tools/build.py`` compiles the hash into the
library (``hbx_build_id``) and rebuilds when the library's hash differs from the tree's, so a
pushed binary that does not match its sources is never reused; the bench line reports both
hashes."""
from __future__ import annotations

import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files(root: str = ROOT):
    csrc = os.path.join(root, "hbbft_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")))
    files = [f for f in files if os.path.basename(f) != "_kdecl.hpp"]
    return files + [os.path.join(root, "include", "hbx.h"), os.path.join(root, "tools", "build.py")]


def source_hash(root: str = ROOT):
    """Hex SHA-256 of the library's sources, or None when they are not all present."""
    h = hashlib.sha256()
    for f in source_files(root):
        if not os.path.exists(f):
            return None
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()
