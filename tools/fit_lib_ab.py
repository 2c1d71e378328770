"""A/B of two libscreenfit builds on the batched KL fit (sf_kl_fit, phase,
niter 2, adjust_order): the fit of one block timed with HIP events (median
of 3 calls after one warm-up), alternating the builds, and (blocks of <= 2 M
slots) the outputs of the two compared -- orders and flagged weights bit for bit, coefficients as the
largest difference relative to max(1, |coef|max).  Each build runs in its own
child process (SCREENFIT_LIB); the outputs go through .npy files under
OUTDIR.

    python tools/fit_lib_ab.py OUTDIR LIB_A LIB_B [D:A:T:F ...] [--rounds 2]

A LIB may carry library options, LIB@OPT=VALUE[,OPT=VALUE] (sf_set_option
ids, e.g. lib.so@18=2: SF_OPT_FIT_SUBSET_DELETION 2), so one build can be
A/B'd against itself.  A shape gain:D:A:T:F is the gain step's two fits as
bench.py --screen gain runs them: the phase fit, then the XX / YY amplitude
fit stacked along the station axis (niter 3, block sigma, no reference); its
outputs compared are the amplitude fit's.
"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out, shape, keep, opts):
    sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
    import torch
    from ska_sdp_screen_fitting_amd import geometry, get_context
    from ska_sdp_screen_fitting_amd._lib import SF_SCREEN_AMPLITUDE, library_identity
    from ska_sdp_screen_fitting_amd.stationscreen import station_orders
    from ska_sdp_screen_fitting_amd.synthetic import make_amplitudes, make_solutions

    gain = shape.startswith("gain:")
    D, A, T, F = (int(v) for v in shape.split(":")[-4:])
    dev = torch.device("cuda", 0)
    ctx = get_context(0)
    for k, v in opts:
        ctx.set_option(k, v)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    s = make_solutions(n_ant=A, n_time=T, n_freq=F, n_dir=D)
    pp, _, _ = geometry.piercepoints(s.dir_radec)
    st = station_orders(s.ant_pos, 0, min(20, D - 1))
    ctx.set_basis(pp)
    ph = torch.from_numpy(s.val).to(dev)
    wt = torch.from_numpy(s.weight).to(dev)
    coef = torch.empty_like(ph)
    order = torch.empty((T, F, A), dtype=torch.int32, device=dev)
    w_out = torch.empty_like(wt)

    if gain:
        make_amplitudes(s)
        va = torch.from_numpy(np.ascontiguousarray(
            np.concatenate([s.amp_val[..., p] for p in range(2)], axis=2))).to(dev)
        wa = torch.from_numpy(np.ascontiguousarray(
            np.concatenate([s.meta["amp_weight"][..., p] for p in range(2)], axis=2))).to(dev)
        amp_order = min(12, max(3, int(np.round(D / 2))))
        coef_a = torch.empty_like(va)
        w_a = torch.empty_like(wa)
        order_a = torch.empty((T, F, 2 * A), dtype=torch.int32, device=dev)

    def run():
        ctx.fit(ph, wt, T, F, A, st, ref_ant=0, coef=coef, order_out=order,
                w_out=w_out, adjust_order=True, niter=2)
        if gain:
            ctx.fit(va, wa, T, F, 2 * A, [amp_order] * (2 * A),
                    screen_type=SF_SCREEN_AMPLITUDE, niter=3, nsigma=5.0,
                    adjust_order=True, ref_ant=-1, coef=coef_a, w_out=w_a,
                    order_out=order_a)

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
    if keep:
        o, w, c = (order_a, w_a, coef_a) if gain else (order, w_out, coef)
        np.save(out + "_order.npy", o.cpu().numpy())
        np.save(out + "_w.npy", w.cpu().numpy())
        np.save(out + "_coef.npy", c.cpu().numpy())
    print(json.dumps({"shape": shape, "slots": T * F * A, "ms": float(np.median(ms)),
                      "ms_all": ms, "fit_stats": str(ctx.fit_stats()),
                      "library": library_identity()["sha16"], "opts": opts}), flush=True)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = 2
    if "--rounds" in sys.argv:
        rounds = int(sys.argv[sys.argv.index("--rounds") + 1])
        args = [a for a in args if a != str(rounds)]
    outdir, libs, shapes = args[0], args[1:3], args[3:] or ["50:64:400:16"]
    os.makedirs(outdir, exist_ok=True)
    res = {"libs": libs, "runs": [], "compare": {}}
    for shape in shapes:
        tag = shape.replace(":", "_")
        D, A, T, F = (int(v) for v in shape.split(":")[-4:])
        small = T * F * A <= 2_000_000  # outputs compared (kept on disk) only then
        for rnd in range(rounds):
            for li, lib in enumerate(libs):
                out = os.path.join(outdir, f"{tag}_{li}")
                path, _, opts = lib.partition("@")
                env = dict(os.environ, SCREENFIT_LIB=os.path.abspath(path))
                keep = "1" if rnd == 0 and small else "0"
                p = subprocess.run([sys.executable, "-u", __file__, "--child", out, shape,
                                    keep, opts], env=env, capture_output=True, text=True,
                                   timeout=600)
                if p.returncode != 0:
                    print(p.stdout, p.stderr, file=sys.stderr)
                    raise SystemExit(f"child failed: {lib} {shape}")
                r = json.loads(p.stdout.strip().splitlines()[-1])
                r["lib"] = li
                r["round"] = rnd
                res["runs"].append(r)
                print(json.dumps(r), flush=True)
        if not small:
            continue
        a = [np.load(os.path.join(outdir, f"{tag}_{li}_{k}.npy"))
             for li in range(2) for k in ("order", "w", "coef")]
        oa, wa, ca, ob, wb, cb = a
        scale = max(1.0, float(np.nanmax(np.abs(ca))))
        res["compare"][shape] = {
            "orders_equal": bool(np.array_equal(oa, ob)),
            "orders_differ": int((oa != ob).sum()),
            "weights_equal": bool(np.array_equal(wa, wb)),
            "weights_differ": int((wa != wb).sum()),
            "coef_max_rel": float(np.nanmax(np.abs(ca - cb)) / scale),
            "coef_bit_equal": bool(np.array_equal(ca.view(np.uint64), cb.view(np.uint64))),
        }
        for li in range(2):
            for k in ("order", "w", "coef"):
                os.remove(os.path.join(outdir, f"{tag}_{li}_{k}.npy"))
        print(json.dumps({shape: res["compare"][shape]}), flush=True)
    with open(os.path.join(outdir, "fit_lib_ab.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        opts = [tuple(int(x) for x in kv.split("=")) for kv in sys.argv[5].split(",") if kv]
        child(sys.argv[2], sys.argv[3], sys.argv[4] == "1", opts)
    else:
        main()
