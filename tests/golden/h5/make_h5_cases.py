#!/opt/conda/bin/python3.9
"""HDF5 layout cases for the H5parm reader (ska_sdp_screen_fitting_amd/hdf5.py),
written with h5py 3.3 (the reference's interpreter) and read back by h5py to
produce the expected arrays (expected.npz):

* dp3_like.h5  -- the reference fixture's solution arrays (from
  ../fixture_kl.npz) laid out as DP3 writes an H5parm: superblock v0,
  contiguous datasets, compound antenna / source tables, fixed-string
  TITLE / AXES / h5parm_version attributes;
* cases_v0.h5  -- superblock v0 (libver earliest, as PyTables writes): val /
  weight CHUNKED + gzip + shuffle (+ fletcher32 on a float16 weight, as
  losoto writes), big-endian axes, a chunked compound table, variable-length
  string attributes, scalar / array numeric attributes, and a group with 40
  members (multi-node symbol-table B-tree);
* cases_latest.h5 -- superblock v3 / v2 object headers (libver latest): link
  messages, compact and contiguous layouts, v3 attribute messages.

Usage:  /opt/conda/bin/python3.9 tests/golden/h5/make_h5_cases.py
"""
import os

import h5py
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _collect(path, tag, exp):
    with h5py.File(path, "r") as f:
        def visit(name, obj):
            if isinstance(obj, h5py.Dataset):
                v = obj[()]
                if v.dtype.names:  # compound: one plain array per field
                    for fld in v.dtype.names:
                        exp[f"{tag}:{name}#{fld}"] = np.ascontiguousarray(v[fld])
                else:
                    exp[f"{tag}:{name}"] = v
            for k, v in obj.attrs.items():
                exp[f"{tag}@{name}@{k}"] = np.array(v)
        f.visititems(visit)


def dp3_like(path):
    z = np.load(os.path.join(HERE, "..", "fixture_kl.npz"))
    with h5py.File(path, "w", libver="earliest") as f:
        ss = f.create_group("sol000")
        ss.attrs["h5parm_version"] = np.bytes_("1.0")
        ant = np.zeros(len(z["ant_names"]), dtype=[("name", "S16"),
                                                   ("position", "<f4", (3,))])
        ant["name"] = z["ant_names"].astype("S16")
        ant["position"] = z["ant_pos"]
        ss.create_dataset("antenna", data=ant)
        src = np.zeros(len(z["dir_names"]), dtype=[("name", "S128"),
                                                   ("dir", "<f4", (2,))])
        src["name"] = z["dir_names"].astype("S128")
        src["dir"] = z["dir_radec"]
        ss.create_dataset("source", data=src)
        st = ss.create_group("phase000")
        st.attrs["TITLE"] = np.bytes_("phase")
        st.attrs["h5parm_version"] = np.bytes_("1.0")
        st.create_dataset("ant", data=z["ant_names"].astype("S9"))
        st.create_dataset("dir", data=z["dir_names"].astype("S128"))
        st.create_dataset("freq", data=z["freqs"])
        st.create_dataset("time", data=z["times"])
        for name in ("val", "weight"):
            d = st.create_dataset(name, data=z[name])
            d.attrs["AXES"] = np.bytes_("time,freq,ant,dir")


def cases_v0(path, rng):
    with h5py.File(path, "w", libver="earliest") as f:
        ss = f.create_group("sol000")
        ss.attrs["h5parm_version"] = np.bytes_("1.0")
        ant = np.zeros(5, dtype=[("name", "S16"), ("position", "<f4", (3,))])
        ant["name"] = [b"CS%03dHBA0" % k for k in range(5)]
        ant["position"] = rng.normal(size=(5, 3)) * 1e6
        ss.create_dataset("antenna", data=ant, chunks=(2,))
        src = np.zeros(3, dtype=[("name", "S128"), ("dir", "<f4", (2,))])
        src["name"] = [b"[Patch_%d]" % k for k in range(3)]
        src["dir"] = rng.random((3, 2))
        ss.create_dataset("source", data=src)
        st = ss.create_group("amplitude000")
        st.attrs["TITLE"] = np.bytes_("amplitude")
        st.attrs["vlen_note"] = "variable length text"
        st.attrs["scalar_f"] = 2.5
        st.attrs["arr_i"] = np.arange(4, dtype=np.int32)
        val = 1.0 + 0.1 * rng.normal(size=(6, 4, 5, 3, 2))
        w = (rng.random((6, 4, 5, 3, 2)) > 0.1).astype(np.float16)
        d = st.create_dataset("val", data=val, chunks=(4, 3, 5, 3, 2),
                              compression="gzip", shuffle=True)
        d.attrs["AXES"] = np.bytes_("time,freq,ant,dir,pol")
        d = st.create_dataset("weight", data=w, chunks=(3, 4, 5, 3, 1),
                              compression="gzip", shuffle=True, fletcher32=True)
        d.attrs["AXES"] = np.bytes_("time,freq,ant,dir,pol")
        st.create_dataset("time", data=np.arange(6) * 8.0 + 5e9, dtype=">f8")
        st.create_dataset("freq", data=np.arange(4) * 1e6 + 1.2e8, dtype=">f8")
        st.create_dataset("ant", data=ant["name"].astype("S9"))
        st.create_dataset("dir", data=src["name"])
        st.create_dataset("pol", data=np.array([b"XX", b"YY"]))
        big = f.create_group("many")
        for k in range(40):
            big.create_dataset(f"d{k:02d}", data=np.full(3, k, np.int16))


def cases_latest(path, rng):
    with h5py.File(path, "w", libver="latest") as f:
        g = f.create_group("sol000/phase000")
        g.attrs["TITLE"] = np.bytes_("phase")
        g.attrs["note"] = "latest format"
        g.create_dataset("val", data=rng.normal(size=(4, 2, 3, 5)))
        g.create_dataset("small", data=np.arange(6, dtype="<i4"))
        g.create_dataset("w", data=rng.random((4, 2, 3, 5)).astype("<f4"))


def main():
    rng = np.random.default_rng(11)
    exp = {}
    for name, fn in (("dp3_like", dp3_like), ("cases_v0", cases_v0),
                     ("cases_latest", cases_latest)):
        path = os.path.join(HERE, name + ".h5")
        if fn is dp3_like:
            fn(path)
        else:
            fn(path, rng)
        if fn is not dp3_like:  # dp3_like is checked against fixture_kl.npz
            _collect(path, name, exp)
    exp = {k: (v.astype("U") if v.dtype == object else v) for k, v in exp.items()}
    np.savez_compressed(os.path.join(HERE, "expected.npz"), **exp)
    print(len(exp), "expected arrays")


if __name__ == "__main__":
    main()
