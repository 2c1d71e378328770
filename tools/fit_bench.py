"""Time the batched KL fit (sf_kl_fit, phase, niter 2, adjust_order) alone on
one GPU for a few (D, slots) shapes and print a digest of its outputs, so
two builds can be compared for speed and for bit-identical results.

    python tools/fit_bench.py [D:A:T:F ...]
"""
import hashlib
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
from ska_sdp_screen_fitting_amd import geometry, get_context  # noqa: E402
from ska_sdp_screen_fitting_amd._lib import SF_OPT_FIT_PACK  # noqa: E402
from ska_sdp_screen_fitting_amd.stationscreen import station_orders  # noqa: E402
from ska_sdp_screen_fitting_amd.synthetic import make_solutions  # noqa: E402

dev = torch.device("cuda", 0)
ctx = get_context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
shapes = sys.argv[1:] or ["20:64:100:16", "50:64:100:4", "50:64:200:16"]
for sh in shapes:
    D, A, T, F = (int(v) for v in sh.split(":"))
    s = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    st = station_orders(s.ant_pos, 0, min(20, D - 1))
    ctx.set_basis(pp)
    ph = torch.from_numpy(s.val).to(dev)
    wt = torch.from_numpy(s.weight).to(dev)
    coef = torch.empty_like(ph)
    order = torch.empty((T, F, A), dtype=torch.int32, device=dev)
    w_out = torch.empty_like(wt)

    def run():
        ctx.fit(ph, wt, T, F, A, st, ref_ant=0, coef=coef, order_out=order,
                w_out=w_out, adjust_order=True, niter=2)

    for pack in (1, 0):
        ctx.set_option(SF_OPT_FIT_PACK, pack)
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ms = float(np.median(ts)) * 1e3
        h = hashlib.sha1()
        for t in (coef, order, w_out):
            h.update(t.cpu().numpy().tobytes())
        S = T * F * A
        print(f"D={D} S={S} pack={pack}: {ms:9.2f} ms  "
              f"{S / ms * 1e3 / 1e6:7.2f} M slots/s  {ctx.fit_stats()}  "
              f"digest {h.hexdigest()[:16]}", flush=True)
    ctx.set_option(SF_OPT_FIT_PACK, 1)
