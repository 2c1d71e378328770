#!/usr/bin/env python3
"""Which tessellated-label pixels depend on the GEOS ring convention.

The reference rasterizes each Voronoi cell with Pillow from the exterior ring
shapely.ops.polygonize returns (voronoi_screen.py:311-340,
processing_utils.py:313-329).  Pillow's outline -- and so which pixels reach
the exact border test -- depends on the ring's start vertex and direction,
and shared-edge pixels on the painting order.  This build follows the ring
convention of the GEOS Polygonizer algorithm (clockwise shells, start at the
lowest-index directed edge, polygonize order; voronoi_screen._rings, restated
as a graph walk in oracle/voronoi.geos_polygonize).  Since GEOS itself is not
importable here, this tool lists, per cell size of the configs, the pixels
whose label would change under any other convention:

* orientation: the cell's ring reversed, same start vertex;
* start vertex: every other start vertex of the cell, same direction;
* both: every (start, direction) pair;

one cell at a time (the other cells keep the GEOS convention), plus the
count of pixels claimed by two cells (painting order).

    python tools/tess_ring_conventions.py > profiles/round3_tess_ring_conventions.txt
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))

from ska_sdp_screen_fitting_amd import voronoi_screen as vs  # noqa: E402

FIELD = dict(rad=126.23, dec=64.50, width=3.3300000000000054)
CELLS = (0.2, 0.1, 0.05, 0.02602)


def main():
    g = np.load(os.path.join(REPO, "tests", "golden", "fixture_kl.npz"))
    pos = vs.read_patch_positions(os.path.join(REPO, "tests", "golden", "skymodel.txt"))
    radec = np.array([pos[str(d).strip("[]")] for d in g["dir_names"]])
    print("cell_deg grid  claimed_twice  pixels that move with: orientation | "
          "start vertex | either  (row, col: geos label -> other labels)")
    for cell in CELLS:
        rings, xy, n, order = vs._rings(radec, FIELD["rad"], FIELD["dec"],
                                        FIELD["width"], cell)
        base = vs.paint_cells(rings, n, order)
        claims = sum(vs.rasterize_cell(r, n).astype(int) for r in rings)
        moved = {"orientation": {}, "start": {}}
        for i, ring in enumerate(rings):
            pts = ring[:-1]
            variants = []
            for k in range(len(pts)):
                for rev in (False, True):
                    if k == 0 and not rev:
                        continue
                    p = pts[k:] + pts[:k]
                    if rev:
                        p = [p[0]] + p[1:][::-1]
                    kind = "orientation" if (k == 0 and rev) else "start"
                    variants.append((kind, p + [p[0]]))
            for kind, alt in variants:
                rr = list(rings)
                rr[i] = alt
                lab = vs.paint_cells(rr, n, order)
                for r, c in np.argwhere(lab != base):
                    moved[kind].setdefault((int(r), int(c)), set()).add(int(lab[r, c]))
        either = set(moved["orientation"]) | set(moved["start"])
        print(f"{cell:<8} {n:>3}^2  {int((claims > 1).sum()):>3}  "
              f"{len(moved['orientation'])} | {len(moved['start'])} | {len(either)} "
              f"of {n * n}")
        for key in sorted(either):
            tags = [k for k in ("orientation", "start") if key in moved[k]]
            alts = sorted(set().union(*(moved[k][key] for k in tags)))
            print(f"    {key}: {int(base[key])} -> {alts}  ({', '.join(tags)})")


if __name__ == "__main__":
    main()
