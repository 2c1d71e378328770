"""Where the fit pass's time goes: the batched KL fit (sf_kl_fit, phase,
adjust_order) of a bench workload with niter 1 (pass 0 without the outlier
flagging) and niter 2 (the bench's), each timed with HIP events over 3 calls,
then the bench's fit with SF_OPT_FIT_SUBSET_DELETION off / on (alternating);
run under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python tools/fit_pass_split.py [workload] [times]
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
sys.path.insert(0, REPO)
from bench import WORKLOADS  # noqa: E402
from ska_sdp_screen_fitting_amd import get_context  # noqa: E402
from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_SUBSET_DELETION  # noqa: E402
from ska_sdp_screen_fitting_amd.distributed import setup_shard  # noqa: E402
from ska_sdp_screen_fitting_amd.synthetic import (FIELD_DEC_DEG, FIELD_RA_DEG,  # noqa: E402
                                                  FIELD_WIDTH_DEG, make_solutions)

wl = sys.argv[1] if len(sys.argv) > 1 else "config4"
A, T, F, D, N, cell = WORKLOADS[wl]
if len(sys.argv) > 2:
    T = int(sys.argv[2])
if wl == "config5":
    A = 64  # one GPU's shard of the 512 stations
sol = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D, ant_offset=0, n_ant_total=A)
setup = setup_shard(sol, 0, A, FIELD_RA_DEG, FIELD_DEC_DEG, FIELD_WIDTH_DEG, cell, device="cpu")
dev = torch.device("cuda", 0)
ctx = get_context(0)
stream = torch.cuda.current_stream(dev)
ctx.set_stream(stream.cuda_stream)
ctx.set_basis(setup["piercepoints"], 100, 5.0 / 3.0)
phase = torch.from_numpy(sol.val).to(dev)
weight = torch.from_numpy(sol.weight).to(dev)
refph = setup["ref_phase"].to(dev).contiguous()
coef = torch.empty_like(phase)
resid = torch.empty_like(phase)
w_out = torch.empty_like(weight)
order_out = torch.empty((T, F, A), dtype=torch.int32, device=dev)
runs = [(1, True, 0), (2, False, 0), (2, True, 0)] + [(2, True, v) for v in (0, 1, 0, 1)]
for niter, adjust, dele in runs:
    ctx.set_option(SF_OPT_FIT_SUBSET_DELETION, dele)
    def run():
        ctx.fit(phase, weight, T, F, A, setup["st_order"], niter=niter, nsigma=5.0,
                adjust_order=adjust, ref_ant=setup["ref_ant"], coef=coef, resid=resid,
                w_out=w_out, order_out=order_out, ant_offset=setup["ant_offset"],
                ref_phase=refph)
    run()
    torch.cuda.synchronize()
    ms = []
    for _ in range(3):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run()
        e1.record(stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    print(f"{wl} S={T * F * A} niter={niter} adjust_order={adjust} deletion={dele}: "
          f"{np.median(ms):.2f} ms  {ctx.fit_stats()}", flush=True)
