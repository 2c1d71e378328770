#!/opt/conda/bin/python3.9
"""Acceptance of files written by ska_sdp_screen_fitting_amd.hdf5.Writer /
H5parm.save by libhdf5 itself (h5py 3.3 in the reference's interpreter).

Step 1 (any interpreter with the package):  python  check_writer_with_h5py.py write DIR
Step 2 (h5py interpreter):                  python3.9 check_writer_with_h5py.py check DIR
The output of step 2 is kept in writer_h5py_check.txt.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def write(d):
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    sys.path.insert(0, os.path.join(HERE, "..", "..", "..", "ska-sdp-screen-fitting_amd"))
    from test_hdf5 import _screen_h5parm
    from ska_sdp_screen_fitting_amd import hdf5
    g, h5 = _screen_h5parm()
    h5.save(os.path.join(d, "screen.h5"))
    w = hdf5.Writer()
    for k in range(100):
        w.dataset(f"/grp/d{k:03d}", np.full(k % 5 + 1, k, np.int64))
    w.dataset("/grp/f2", np.arange(7, dtype=np.float16))
    w.dataset("/scalar", np.float32(3.5))
    w.group_attrs("/", {"top": np.int32(-7)})
    w.save(os.path.join(d, "many.h5"))
    np.savez(os.path.join(d, "expect.npz"), coef=g["coef"],
             w=g["w_out"].astype(np.float16), pp=g["piercepoints"])


def check(d):
    import h5py
    e = np.load(os.path.join(d, "expect.npz"))
    out = {"h5py": h5py.__version__, "hdf5": h5py.version.hdf5_version}
    with h5py.File(os.path.join(d, "screen.h5"), "r") as f:
        names = []
        f.visit(names.append)
        st = f["sol000/phase_screen000"]
        out["screen_members"] = sorted(names)
        out["val_equal"] = bool(np.array_equal(st["val"][()], e["coef"]))
        out["weight_f16_equal"] = bool(np.array_equal(st["weight"][()], e["w"]))
        out["piercepoint_equal"] = bool(np.array_equal(st["piercepoint"][()], e["pp"]))
        out["screen_attrs"] = {k: (v.decode() if isinstance(v, bytes) else float(v))
                               for k, v in st.attrs.items()}
        out["antenna_dtype"] = str(f["sol000/antenna"].dtype)
    with h5py.File(os.path.join(d, "many.h5"), "r") as f:
        out["many_members"] = len(f["grp"])
        out["many_equal"] = all(np.array_equal(f[f"grp/d{k:03d}"][()], np.full(k % 5 + 1, k))
                                for k in range(100))
        out["scalar_shape"] = list(f["scalar"].shape)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    {"write": write, "check": check}[sys.argv[1]](sys.argv[2])
