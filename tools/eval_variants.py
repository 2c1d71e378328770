"""Repeated, interleaved timing of eval variants (plain vs non-temporal)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
from ska_sdp_screen_fitting_amd import geometry, get_context  # noqa: E402
from ska_sdp_screen_fitting_amd._lib import (SF_EVAL_FAST_SINCOS,  # noqa: E402
                                             SF_EVAL_NT_STORES)

dev = torch.device("cuda", 0)
ctx = get_context(0)
stream = torch.cuda.current_stream(dev)
ctx.set_stream(stream.cuda_stream)
rng = np.random.default_rng(0)
D, N = int(sys.argv[1]) if len(sys.argv) > 1 else 20, 256
S = 102400
pp = np.stack([rng.uniform(-3000, 3000, D), rng.uniform(-3000, 3000, D), np.zeros(D)], 1)
ctx.set_basis(pp)
x = np.linspace(-2000, 2000, N)
ctx.set_grid(x, x)
coef = torch.from_numpy(rng.normal(0, 0.01, (S, D))).to(dev)
ring = 16384
out = torch.empty((ring, 4, N, N), dtype=torch.float32, device=dev)
variants = {"fast": 1 | SF_EVAL_FAST_SINCOS,
            "fast+nt": 1 | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES}
res = {k: [] for k in variants}
for rep in range(6):
    for k, fl in variants.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ctx.eval(coef, S, out, ring, fl)
        e1.record(stream)
        torch.cuda.synchronize()
        if rep:
            res[k].append(e0.elapsed_time(e1))
for k, v in res.items():
    ms = float(np.median(v))
    print(f"D={D} {k:8s}: median {ms:.2f} ms  min {min(v):.2f}  "
          f"{S * (16 * N * N + 8 * D) / ms / 1e6:.1f} GB/s", flush=True)
