"""Interleaved timing of the evaluation kernels (sf_kl_eval variants) on one
GPU, plus a bitwise cross-check of their outputs.

    python tools/eval_variants.py [--variants tile+nt,lds16+nt] D:N [D:N ...]

Every repetition runs every (shape, variant) pair once, so box-to-box and
drift effects hit all of them alike.
"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
from ska_sdp_screen_fitting_amd import get_context  # noqa: E402
from ska_sdp_screen_fitting_amd._lib import (  # noqa: E402
    SF_EVAL_FAST_SINCOS, SF_EVAL_KERNEL_AUTO, SF_EVAL_KERNEL_LDS4,
    SF_EVAL_KERNEL_LDS8, SF_EVAL_KERNEL_LDS8H, SF_EVAL_KERNEL_LDS16,
    SF_EVAL_KERNEL_LDS16H, SF_EVAL_KERNEL_SHB, SF_EVAL_KERNEL_TILE, SF_EVAL_KERNEL_TILE3,
    SF_EVAL_NAN_SCRUB, SF_EVAL_NT_STORES, SF_OPT_EVAL_KERNEL,
    SF_OPT_EVAL_GROUPS, SF_OPT_EVAL_KS_PAD, SF_OPT_EVAL_SLEEP,
    SF_OPT_EVAL_XCD_MAP, SF_OPT_EVAL_BANDS, SF_OPT_EVAL_INT, SF_OPT_EVAL_WG_WAVES)

KERNELS = {"auto": SF_EVAL_KERNEL_AUTO, "tile": SF_EVAL_KERNEL_TILE,
           "tile3": SF_EVAL_KERNEL_TILE3,
           "lds4": SF_EVAL_KERNEL_LDS4, "lds8": SF_EVAL_KERNEL_LDS8,
           "lds16": SF_EVAL_KERNEL_LDS16, "lds8h": SF_EVAL_KERNEL_LDS8H,
           "lds16h": SF_EVAL_KERNEL_LDS16H, "shb": SF_EVAL_KERNEL_SHB}

ap = argparse.ArgumentParser()
ap.add_argument("shapes", nargs="*", default=["20:256"])
ap.add_argument("--variants", default=",".join(
    f"{k}+nt" for k in KERNELS))
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--slots", type=int, default=102400,
                help="slots per launch at 256^2 (scaled by 256^2/N^2)")
ap.add_argument("--no-check", action="store_true",
                help="skip the bitwise cross-check (energy-diagnostic builds)")
ap.add_argument("--gain", action="store_true",
                help="gain screens (sf_kl_eval_gain: phase + XX / YY log-amplitude "
                     "coefficients, three contractions, four distinct planes)")
args = ap.parse_args()

dev = torch.device("cuda", 0)
ctx = get_context(0)
stream = torch.cuda.current_stream(dev)
ctx.set_stream(stream.cuda_stream)
base = SF_EVAL_NAN_SCRUB | SF_EVAL_FAST_SINCOS
variants = {}
for v in args.variants.split(","):
    # kernel[+nt][+padN][+sleepN][+xi|+xc][+gN][+bN]; the XCD map is the
    # library's auto choice unless +xi (interleaved) / +xc (contiguous);
    # +int0: the fp64 contraction where the integer-digit one would apply
    k, *mods = v.split("+")
    fl, pad, sleep, xi, grp, bands, ival, wgw = base, 0, 0, -1, 0, 0, -1, 0
    for m in mods:
        if m == "nt":
            fl |= SF_EVAL_NT_STORES
        elif m.startswith("pad"):
            pad = int(m[3:])
        elif m.startswith("sleep"):
            sleep = int(m[5:])
        elif m == "xi":
            xi = 1
        elif m == "xc":
            xi = 0
        elif m == "int0":
            ival = 0
        elif m.startswith("w"):
            wgw = int(m[1:])
        elif m.startswith("b"):
            bands = int(m[1:])
        elif m.startswith("g"):
            grp = int(m[1:])
        else:
            raise SystemExit(f"unknown variant modifier {m}")
    variants[v] = (KERNELS[k], fl, (pad, sleep, xi, grp, bands, ival, wgw))


def use(kv, opts=(0, 0, -1, 0, 0, -1, 0)):
    pad, sleep, xi, grp, bands, ival, wgw = opts
    ctx.set_option(SF_OPT_EVAL_INT, ival)
    ctx.set_option(SF_OPT_EVAL_WG_WAVES, wgw)
    ctx.set_option(SF_OPT_EVAL_BANDS, bands)
    ctx.set_option(SF_OPT_EVAL_GROUPS, grp)
    ctx.set_option(SF_OPT_EVAL_KERNEL, kv)
    ctx.set_option(SF_OPT_EVAL_KS_PAD, pad)
    ctx.set_option(SF_OPT_EVAL_SLEEP, sleep)
    ctx.set_option(SF_OPT_EVAL_XCD_MAP, xi)

ring_bytes = 16 * 2 ** 30
out_flat = torch.empty(ring_bytes // 4, dtype=torch.float32, device=dev)
shapes = []
for sh in args.shapes:
    D, N = (int(x) for x in sh.split(":"))
    rng = np.random.default_rng(D * 1000 + N)
    pp = np.stack([rng.uniform(-3000, 3000, D), rng.uniform(-3000, 3000, D),
                   np.zeros(D)], 1)
    S = args.slots * (256 * 256) // (N * N)
    coef = torch.from_numpy(rng.normal(0, 0.01, (S, D))).to(dev)
    if args.gain:
        amps = tuple(torch.from_numpy(rng.normal(0, 0.002, (S, D))).to(dev)
                     for _ in range(2))
        coef = (coef,) + amps
    shapes.append((D, N, S, pp, coef))


def run_eval(coef, S, out, ring, fl):
    if args.gain:
        ctx.eval_gain(coef[0], coef[1], coef[2], S, out, ring, fl)
    else:
        ctx.eval(coef, S, out, ring, fl)


def select(D, N, pp):
    ctx.set_basis(pp)
    x = np.linspace(-2000, 2000, N)
    ctx.set_grid(x, x)


# bitwise cross-check on a small ragged batch with a NaN coefficient
for D, N, S, pp, coef in ([] if args.no_check else shapes):
    select(D, N, pp)
    Sc = 37
    if args.gain:
        cchk = tuple(c[:Sc].clone() for c in coef)
        cchk[0][5, min(3, D - 1)] = float("nan")
        cchk[1][7, 0] = float("nan")
    else:
        cchk = coef[:Sc].clone()
        cchk[5, min(3, D - 1)] = float("nan")
    refs = {}
    for name, (kv, fl, opts) in variants.items():
        use(kv, opts)
        o = torch.full((Sc, 4, N, N), -7.0, dtype=torch.float32, device=dev)
        run_eval(cchk, Sc, o, Sc, fl)
        torch.cuda.synchronize()
        # the two contractions (integer digits / fp64) are compared within
        # themselves: they agree to ~1e-7, not bitwise
        if opts[5] not in refs:
            refs[opts[5]] = (o, name)
            continue
        ref, rname = refs[opts[5]]
        if not torch.equal(o.view(torch.int32), ref.view(torch.int32)):
            print(f"check D={D} N={N} {name}: DIFFERENT from {rname} "
                  f"(max |d| {float((o - ref).abs().max()):.3g})", flush=True)
            sys.exit(1)
    print(f"check D={D} N={N}: all variants bitwise equal", flush=True)

res = {}
for rep in range(args.reps):
    for D, N, S, pp, coef in shapes:
        select(D, N, pp)
        ring = ring_bytes // (16 * N * N)
        out = out_flat[: ring * 4 * N * N].view(ring, 4, N, N)
        use(SF_EVAL_KERNEL_AUTO)
        run_eval(coef, S, out, ring, base)  # untimed: re-warm after select()
        for name, (kv, fl, opts) in variants.items():
            use(kv, opts)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            run_eval(coef, S, out, ring, fl)
            e1.record(stream)
            torch.cuda.synchronize()
            if rep:
                res.setdefault((D, N, S, name), []).append(e0.elapsed_time(e1))
for (D, N, S, name), v in res.items():
    ms = float(np.median(v))
    gbs = S * (16 * N * N + (24 if args.gain else 8) * D) / ms / 1e6
    print(f"D={D:2d} N={N} {name:10s}: median {ms:.3f} ms  min {min(v):.3f}  "
          f"{gbs:.1f} GB/s  frac {gbs / 8000:.3f}", flush=True)
