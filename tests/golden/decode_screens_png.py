#!/usr/bin/env python3
"""Decode the reference's own rendering of its config-1 screens into a fixture.

``/root/reference/resources/screens_.png`` (871 x 427 RGBA) is the figure the
reference's ``scripts/analyze_screens.py:97-223`` draws from its own outputs
``kl_0.fits`` and ``tessellated_0.fits`` (the reference test's fields:
bounds [124.565, 66.165, 127.895, 62.835], cell 0.2 deg -> 17^2,
tessellated with ``smooth_deg=0.1`` = 0.5 px): two ``imshow`` panels of
``cube[time=0, freq=3, antenna=1, polarization_idx=1]`` (Im XX), viridis,
``vmin`` / ``vmax`` from ``get_boundaries`` (:13-66), with the patch markers
drawn over them.

Every data pixel of a 17 x 17 panel is a ~22 x 22 block of one colour
(nearest-neighbour upsampling); the block's most frequent colour (the
scatter markers cover less than half of any block's centre) is stored, per
pixel, as RGB bytes together with matplotlib's 8-bit viridis table, so the
tests can check "value -> colour" without matplotlib:
idx = min(floor((v - vmin) / (vmax - vmin) * 256), 255), colour = lut[idx]
(matplotlib Normalize + Colormap; two pairs of viridis entries, 104 / 105
and 137 / 138, share their bytes, so the comparison is on colours).

The panel frames are found from the axis spines (rows / columns of dark
pixels spanning the panel).  Every decoded block colour is an exact viridis
entry (checked here).

This is test infrastructure: it reads ``/root/reference`` (this container
only) and writes ``tests/golden/screens_png.npz`` (data).  Use:

    python3 tests/golden/decode_screens_png.py
"""

import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
PNG = "/root/reference/resources/screens_.png"
N = 17                      # 0.2 deg cells over the 3.33 deg field
SELECT = (0, 3, 1, 1)       # analyze_screens.plot_screens defaults (:102-105)


def viridis_lut():
    import matplotlib
    lut = matplotlib.colormaps["viridis"](np.arange(256), bytes=True)[:, :3]
    return np.asarray(lut, np.uint8)


def spines(img):
    """Rows and columns of the axes frames: dark, opaque, > 300 px long."""
    rgb = img[..., :3].astype(int)
    dark = (rgb.sum(-1) < 150) & (img[..., 3] > 200)
    rows = np.nonzero(dark.sum(1) > 300)[0]
    cols = np.nonzero(dark.sum(0) > 300)[0]
    assert len(rows) == 2 and len(cols) == 4, (rows, cols)
    return rows, cols


def decode_panel(img, x0, x1, y0, y1, half=7):
    """Block colour per data pixel: the most frequent RGB of the
    (2 half + 1)^2 screen pixels about the block centre.  The spines sit on
    the axes limits -0.5 and 16.5, so pixel i spans [x0 + i w, x0 + (i+1) w]."""
    rgb = img[..., :3]
    out = np.zeros((N, N, 3), np.uint8)
    purity = np.zeros((N, N))
    for r in range(N):
        yc = int(y0 + (r + 0.5) * (y1 - y0) / N)
        for c in range(N):
            xc = int(x0 + (c + 0.5) * (x1 - x0) / N)
            blk = rgb[yc - half:yc + half + 1, xc - half:xc + half + 1].reshape(-1, 3)
            cols, cnt = np.unique(blk, axis=0, return_counts=True)
            k = int(np.argmax(cnt))
            out[r, c] = cols[k]
            purity[r, c] = cnt[k] / len(blk)
    return out, purity


def main():
    img = np.array(Image.open(PNG))
    assert img.shape == (427, 871, 4), img.shape
    rows, cols = spines(img)
    lut = viridis_lut()
    panels = {}
    for name, (xa, xb) in (("kl", cols[0:2]), ("vor", cols[2:4])):
        rgb, purity = decode_panel(img, xa, xb, rows[0], rows[1])
        # every block colour is an exact viridis entry
        d = np.abs(rgb[:, :, None, :].astype(int) - lut[None, None].astype(int)).sum(-1)
        assert int(d.min(-1).max()) == 0, name
        assert purity.min() > 0.5, (name, purity.min())
        panels[name] = rgb
        print(name, "frame x", (int(xa), int(xb)), "y", tuple(int(v) for v in rows),
              "min purity", round(float(purity.min()), 3))
    np.savez_compressed(os.path.join(HERE, "screens_png.npz"),
                        kl_rgb=panels["kl"], vor_rgb=panels["vor"], lut=lut,
                        select=np.array(SELECT), grid=np.array(N),
                        frame_rows=rows, frame_cols=cols)
    print("wrote", os.path.join(HERE, "screens_png.npz"))


if __name__ == "__main__":
    main()
