"""Run one tiled-GEMM (or library) shape repeatedly -- a target for rocprofv3 counter passes.

    python tools/prof_gemm_one.py --shape gate_up --M 8192 --cfg 3 --iters 20 [--library]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_sse_for_llm_response_amd import ops  # noqa: E402
from distributed_sse_for_llm_response_amd.ops import reference as R  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="gate_up")
ap.add_argument("--M", type=int, default=8192)
ap.add_argument("--cfg", default="3")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--library", action="store_true")
a = ap.parse_args()
os.environ["DSSE_KERNEL_CFG"] = f"gemm_impl=4,t_cfg={a.cfg}"
ops.load_library(required=True)
ops.refresh_env()
N, K = SHAPES[a.shape]
g = torch.Generator().manual_seed(0)
dev = torch.device("cuda", 0)
w = ((torch.rand(N, K, generator=g) * 2 - 1) / 64).bfloat16().to(dev)
wt = R.tile_weight(w)
x = (torch.rand(a.M, K, generator=g) * 2 - 1).bfloat16().to(dev)
out = torch.empty(a.M, N, device=dev, dtype=torch.bfloat16)
for _ in range(a.iters):
    if a.library:
        torch.matmul(x, w.t(), out=out)
    else:
        ops.gemm_out(x, wt, out)
torch.cuda.synchronize()
print("done", flush=True)
