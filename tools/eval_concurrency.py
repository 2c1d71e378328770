"""Does splitting one evaluation into concurrent launches on several HIP
streams (separate output windows) change the achieved store bandwidth?
Dev experiment: 102,400 slots at 256^2, D = 20, fp32-sincos + NT stores."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
from ska_sdp_screen_fitting_amd import get_context  # noqa: E402
from ska_sdp_screen_fitting_amd._lib import (  # noqa: E402
    SF_EVAL_FAST_SINCOS, SF_EVAL_NAN_SCRUB, SF_EVAL_NT_STORES)

dev = torch.device("cuda", 0)
ctx = get_context(0)
D, N, S = 20, 256, 102400
rng = np.random.default_rng(0)
pp = np.stack([rng.uniform(-3000, 3000, D), rng.uniform(-3000, 3000, D), np.zeros(D)], 1)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
ctx.set_basis(pp)
x = np.linspace(-2000, 2000, N)
ctx.set_grid(x, x)
coef = torch.from_numpy(rng.normal(0, 0.01, (S, D))).to(dev)
ring = 16384
out = torch.empty((ring, 4, N, N), dtype=torch.float32, device=dev)
fl = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES
streams = [torch.cuda.Stream(dev) for _ in range(4)]


def run(k):
    """k concurrent launches, each S/k slots into its own ring window."""
    main = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()
    ev.record(main)
    part, rpart = S // k, ring // k
    for j in range(k):
        st = streams[j]
        st.wait_event(ev)
        ctx.set_stream(st.cuda_stream)
        ctx.eval(coef[j * part:(j + 1) * part], part, out[j * rpart:(j + 1) * rpart], rpart, fl)
    for j in range(k):
        e = torch.cuda.Event()
        e.record(streams[j])
        main.wait_event(e)


res = {k: [] for k in (1, 2, 3, 4)}
for rep in range(8):
    for k in res:
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        run(k)
        e1.record()
        torch.cuda.synchronize()
        if rep:
            res[k].append(e0.elapsed_time(e1))
for k, v in res.items():
    ms = float(np.median(v))
    gbs = S * (16 * N * N + 8 * D) / ms / 1e6
    print(f"{k} concurrent launches: median {ms:.3f} ms  {gbs:.1f} GB/s  frac {gbs / 8000:.3f}")
