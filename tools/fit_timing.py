"""Timing experiments for the fit / eval kernels on one GPU (dev tool)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
from ska_sdp_screen_fitting_amd import geometry, get_context  # noqa: E402
from ska_sdp_screen_fitting_amd._lib import SF_EVAL_FAST_SINCOS, SF_EVAL_NT_STORES  # noqa: E402
from ska_sdp_screen_fitting_amd.stationscreen import station_orders  # noqa: E402
from ska_sdp_screen_fitting_amd.synthetic import make_solutions  # noqa: E402


def timeit(fn, n=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    A, T, F, D = 64, 100, 16, 20
    for label, kw in (("clean", dict(flag_frac=0.0, outlier_frac=0.0)),
                      ("flags1%", dict(flag_frac=0.01, outlier_frac=0.0)),
                      ("outl0.5%", dict(flag_frac=0.0, outlier_frac=0.005)),
                      ("default", dict())):
        s = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D, **kw)
        pp, mra, mdec = geometry.piercepoints(s.dir_radec)
        st = station_orders(s.ant_pos, 0, 19)
        ctx.set_basis(pp)
        ph = torch.from_numpy(s.val).to(dev)
        wt = torch.from_numpy(s.weight).to(dev)
        coef = torch.empty_like(ph)
        order = torch.empty((T, F, A), dtype=torch.int32, device=dev)
        w_out = torch.empty_like(wt)
        for adj, niter in ((True, 2), (False, 1)):
            ms = timeit(lambda: ctx.fit(ph, wt, T, F, A, st, ref_ant=0, coef=coef,
                                        order_out=order, w_out=w_out,
                                        adjust_order=adj, niter=niter))
            o = order.cpu().numpy()
            nflag = int((w_out.cpu().numpy() == 0).sum())
            print(f"fit {label:9s} adjust={adj} niter={niter}: {ms:8.2f} ms  "
                  f"orders {np.bincount(o.ravel())[-6:]} flagged {nflag} "
                  f"{ctx.fit_stats()}", flush=True)
    x, y = geometry.grid_coords(126.23, 64.5, 3.3300000000000054, 0.01301, mra, mdec)
    ctx.set_grid(x, y)
    S = T * F * A
    ring = 16384
    out = torch.empty((ring, 4, 256, 256), dtype=torch.float32, device=dev)
    for flags, name in ((1, "fp64 sincos+scrub"), (0, "fp64 sincos"),
                        (1 | SF_EVAL_FAST_SINCOS, "fast sincos+scrub"),
                        (1 | SF_EVAL_FAST_SINCOS | SF_EVAL_NT_STORES, "fast+scrub+nt")):
        ms = timeit(lambda: ctx.eval(coef, S, out, ring, flags))
        gbs = S * (16 * 65536 + 160) / (ms * 1e-3) / 1e9
        print(f"eval {name:18s}: {ms:8.2f} ms  {gbs:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
