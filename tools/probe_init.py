"""Probe: libhbx.so loaded (HIP initialised) BEFORE torch is imported, then torch uses the GPU."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from hbbft_amd import hbx  # noqa: E402

order = sys.argv[1] if len(sys.argv) > 1 else "lib-first"
if order == "torch-first":
    import torch  # noqa: F401
ctx = hbx.Context(0)
print("ctx ok", flush=True)
import torch  # noqa: E402

print("is_available", torch.cuda.is_available(), flush=True)
x = torch.zeros(4, device="cuda")
print("tensor ok", x.sum().item(), flush=True)
