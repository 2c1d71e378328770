"""How much of the fit pass the flagged-direction slots cost: the batched
fit (sf_kl_fit, phase, niter 2) of one config-5-shaped block (D = 50) with
the workload's 1 % zero weights and 0.5 % outliers, without the zero
weights, and without either -- each timed with HIP events over 3 calls.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python tools/fit_flag_share.py [A T F D]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
from ska_sdp_screen_fitting_amd import geometry, get_context  # noqa: E402
from ska_sdp_screen_fitting_amd.stationscreen import station_orders  # noqa: E402
from ska_sdp_screen_fitting_amd.synthetic import make_solutions  # noqa: E402

A, T, F, D = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (64, 400, 64, 50)))
dev = torch.device("cuda", 0)
ctx = get_context(0)
stream = torch.cuda.current_stream(dev)
ctx.set_stream(stream.cuda_stream)
for flag_frac, outlier_frac in ((0.01, 0.005), (0.0, 0.005), (0.0, 0.0)):
    s = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D, flag_frac=flag_frac,
                       outlier_frac=outlier_frac)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    ctx.set_basis(pp)
    st = station_orders(s.ant_pos, 0, min(20, D - 1))
    ph = torch.from_numpy(s.val).to(dev)
    wt = torch.from_numpy(s.weight).to(dev)
    coef = torch.empty_like(ph)
    ms = []
    for rep in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ctx.fit(ph, wt, T, F, A, st, ref_ant=0, coef=coef)
        e1.record(stream)
        torch.cuda.synchronize()
        if rep:
            ms.append(e0.elapsed_time(e1))
    fs = ctx.fit_stats()
    print(f"flags {flag_frac} outliers {outlier_frac}: {T * F * A} slots, fit "
          f"{np.mean(ms):.1f} ms, masks {fs['n_masks']}", flush=True)
