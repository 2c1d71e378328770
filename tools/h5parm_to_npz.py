#!/usr/bin/env python3
"""Convert an H5parm (needs h5py) into the .npz the GPU box reads.

    python tools/h5parm_to_npz.py solutions.h5 solutions.npz [sol000] [phase000]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "ska-sdp-screen-fitting_amd"))
from ska_sdp_screen_fitting_amd.h5parm import H5parm  # noqa: E402


def main(src, dst, solset="sol000", soltab="phase000"):
    h = H5parm(src)
    ss = h.get_solset(solset)
    st = ss.get_soltab(soltab)
    axes = st.get_axes_names()
    order = [axes.index(a) for a in ("time", "freq", "ant", "dir")]
    ants, srcs = ss.get_ant(), ss.get_source()
    np.savez(dst, val=np.transpose(st.val, order), weight=np.transpose(st.weight, order),
             times=st.time, freqs=st.freq, ant_names=np.array(st.ant),
             dir_names=np.array(st.dir),
             ant_pos=np.array([ants[a] for a in st.ant], np.float32),
             dir_radec=np.array([srcs[d] for d in st.dir], np.float32),
             solset=solset, soltab=soltab)


if __name__ == "__main__":
    main(*sys.argv[1:])
