"""Run one transformer GEMM shape a few times (for rocprofv3 --pmc passes):
python scripts/gemm_pmc.py M N K a_kcontig b_kcontig [reps] [tile splits]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "e2e-parking-carla_amd"))
import torch  # noqa: E402

from e2ep_amd import _lib, nn_ops  # noqa: E402

M, N, K, ak, bk = (int(v) for v in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
if len(sys.argv) > 8:
    _lib.call("e2ep_gemm_force", int(sys.argv[7]), int(sys.argv[8]), 0)
A = torch.randn((M, K) if ak else (K, M), device="cuda")
B = torch.randn((N, K) if bk else (K, N), device="cuda")
out = torch.empty(M, N, device="cuda")
for _ in range(reps):
    nn_ops.gemm(A, ak, B, bk, M, N, K, out=out)
torch.cuda.synchronize()
print("done")
