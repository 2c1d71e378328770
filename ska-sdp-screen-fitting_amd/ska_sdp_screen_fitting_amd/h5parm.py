"""The subset of the H5parm solution-file API the KL path uses.

Mirrors, for the drop-in, the reference's ``utils/h5parm.py`` objects as far
as ``make_aterm_image`` / ``KLScreen.fit`` / ``stationscreen.run`` touch them
(``H5parm.get_solset`` :78-457, ``Solset.get_soltab/get_source/get_ant/
make_soltab`` :460-799, ``Soltab`` axis access :1306-1324).

Storage backends:

* ``.h5`` / ``.h5parm`` through the built-in read-only HDF5 reader
  (``hdf5.py``; neither PyTables nor h5py is needed) -- the LoSoTo / DP3
  layout: ``/<solset>/<soltab>/{val,weight,<axis>}`` with an ``AXES``
  attribute, ``TITLE`` = soltab type, ``/<solset>/antenna`` and
  ``/<solset>/source`` compound tables;
* ``.npz`` produced by ``tools/h5parm_to_npz.py``:
  keys ``val weight times freqs dir_names ant_names dir_radec ant_pos``
  (+ optional ``soltab``/``solset`` names and ``pol``/``amp_*`` arrays).

Unlike the reference, an H5parm opened for the KL fit is never mutated: the
fitted screen soltabs live in memory (the reference writes them into the
input file, kl_screen.py:66, and on re-runs reads back a stale table because
``remove_soltabs`` silently fails, processing_utils.py:590-596).
"""

import os

import numpy as np


class Soltab:
    """One solution table: values ``val[axes...]`` and ``weight``."""

    def __init__(self, name, soltype, axes_names, axes_vals, val, weight,
                 solset=None, attrs=None):
        self.name = name
        self.soltype = soltype
        self._axes_names = list(axes_names)
        self._axes = {a: v for a, v in zip(axes_names, axes_vals)}
        self.val = val
        self.weight = weight
        self._solset = solset
        self.attrs = dict(attrs or {})
        self.piercepoint = None

    # reference: Soltab.get_type / get_axes_names / get_solset / __getattr__
    def get_type(self):
        return self.soltype

    def get_axes_names(self):
        return list(self._axes_names)

    def get_solset(self):
        return self._solset

    def __getattr__(self, axis):
        axes = self.__dict__.get("_axes", {})
        if axis in axes:
            return axes[axis]
        raise AttributeError(axis)

    def get_values(self, weight=False):
        return self.weight if weight else self.val


class Solset:
    """A set of soltabs plus the antenna and source tables."""

    def __init__(self, name, ant_names, ant_pos, dir_names, dir_radec):
        self.name = name
        self.soltabs = {}
        self._ants = {n: np.asarray(p, np.float32) for n, p in zip(ant_names, ant_pos)}
        self._sources = {n: np.asarray(p, np.float32)
                         for n, p in zip(dir_names, dir_radec)}

    def get_ant(self):
        return dict(self._ants)

    def get_source(self):
        return dict(self._sources)

    def get_soltab(self, name):
        if name not in self.soltabs:
            raise KeyError(f"soltab {name!r} not in solset {self.name!r}")
        return self.soltabs[name]

    def get_soltab_names(self):
        return list(self.soltabs)

    def make_soltab(self, soltype, soltab_name=None, axes_names=None,
                    axes_vals=None, vals=None, weights=None, **_):
        """utils/h5parm.py:509-640 (in memory; weights kept as given)."""
        st = Soltab(soltab_name, soltype, axes_names, axes_vals,
                    np.asarray(vals), np.asarray(weights), solset=self)
        self.soltabs[soltab_name] = st
        return st


class H5parm:
    """Read-only solution file: ``H5parm(path).get_solset("sol000")``."""

    def __init__(self, path, readonly=True):
        self.path = path
        self.solsets = {}
        ext = os.path.splitext(path)[1].lower()
        if ext == ".npz":
            self._load_npz(path)
        else:
            self._load_h5(path)

    def close(self):
        pass

    def save(self, path, weight_dtype=np.float16):
        """Write every solset -- including soltabs made by
        ``stationscreen.run`` -- to a new H5parm file (see write_h5parm)."""
        write_h5parm(path, list(self.solsets.values()), weight_dtype)

    def get_solset(self, name="sol000"):
        if name not in self.solsets:
            raise KeyError(f"solset {name!r} not in {self.path}")
        return self.solsets[name]

    def _load_npz(self, path):
        z = np.load(path, allow_pickle=False)
        solset_name = str(z["solset"]) if "solset" in z else "sol000"
        ss = Solset(solset_name, [str(s) for s in z["ant_names"]], z["ant_pos"],
                    [str(s) for s in z["dir_names"]], z["dir_radec"])
        axes = ["time", "freq", "ant", "dir"]
        vals = [np.asarray(z["times"], np.float64), np.asarray(z["freqs"], np.float64),
                np.array([str(s) for s in z["ant_names"]]),
                np.array([str(s) for s in z["dir_names"]])]
        name = str(z["soltab"]) if "soltab" in z else "phase000"
        ss.soltabs[name] = Soltab(name, "phase", axes, vals,
                                  np.asarray(z["val"], np.float64),
                                  np.asarray(z["weight"], np.float32), solset=ss)
        if "amp_val" in z:
            aname = name.replace("phase", "amplitude")
            aaxes = axes + ["pol"]
            avals = [np.asarray(z["amp_times"], np.float64),
                     np.asarray(z["amp_freqs"], np.float64), vals[2], vals[3],
                     np.array([str(s) for s in z["amp_pol"]])]
            ss.soltabs[aname] = Soltab(aname, "amplitude", aaxes, avals,
                                       np.asarray(z["amp_val"], np.float64),
                                       np.asarray(z["amp_weight"], np.float32),
                                       solset=ss)
        self.solsets[solset_name] = ss

    def _load_h5(self, path):
        """LoSoTo / DP3 layout through the built-in HDF5 reader (hdf5.py)."""
        from . import hdf5

        def text(v):
            v = v.decode() if isinstance(v, bytes) else str(v)
            return v

        with hdf5.File(path) as f:
            for ssn in f.keys():
                g = f[ssn]
                if not isinstance(g, hdf5.Group) or "antenna" not in g:
                    continue
                ants = g["antenna"][()]
                srcs = g["source"][()]
                ss = Solset(ssn, [text(a) for a in ants["name"]],
                            np.asarray(ants["position"]),
                            [text(s) for s in srcs["name"]],
                            np.asarray(srcs["dir"]))
                for stn in g.keys():
                    if stn in ("antenna", "source"):
                        continue
                    st = g[stn]
                    if not isinstance(st, hdf5.Group) or "val" not in st:
                        continue
                    val = st["val"]
                    axes = text(val.attrs["AXES"]).split(",")
                    avals = []
                    for a in axes:
                        v = st[a][()]
                        if v.dtype.kind in "SO":
                            v = np.array([text(x) for x in v])
                        avals.append(v)
                    title = text(st.attrs.get("TITLE", b""))
                    extra = {k: v for k, v in st.attrs.items()
                             if k not in ("TITLE", "CLASS", "VERSION",
                                          "parmdb_type", "h5parm_version")}
                    tab = Soltab(stn, title, axes, avals,
                                 np.asarray(val[()], np.float64),
                                 np.asarray(st["weight"][()], np.float32), ss,
                                 attrs=extra)
                    if "piercepoint" in st:
                        tab.piercepoint = st["piercepoint"][()]
                    ss.soltabs[stn] = tab
                self.solsets[ssn] = ss


def _bytes_array(values):
    a = np.asarray(values)
    return np.char.encode(a.astype(str), "utf8") if a.dtype.kind in "UO" else a


def write_h5parm(path, solsets, weight_dtype=np.float16):
    """Write solsets (``H5parm.solsets`` values) as a new H5parm file in the
    LoSoTo layout PyTables reads (utils/h5parm.py:164-221 make_solset,
    :509-640 make_soltab): per solset the ``antenna`` (name S16, position
    f4[3]) and ``source`` (name S128, dir f4[2]) tables; per soltab a group
    titled with the soltab type, one array per axis, ``val`` (f8) and
    ``weight`` (f16 by default) with the ``AXES`` attribute, the soltab's
    attributes (the screen soltabs' beta, r_0, height, midra, middec) and its
    ``piercepoint`` array when set (stationscreen.py:1147-1157)."""
    from .hdf5 import Writer
    w = Writer()
    for ss in solsets:
        root = "/" + ss.name
        w.group_attrs(root, {"h5parm_version": b"1.0"})
        ants = ss.get_ant()
        at = np.zeros(len(ants), dtype=[("name", "S16"), ("position", "<f4", (3,))])
        at["name"] = _bytes_array(list(ants))
        at["position"] = np.array(list(ants.values()), np.float32).reshape(-1, 3)
        w.dataset(root + "/antenna", at)
        srcs = ss.get_source()
        sr = np.zeros(len(srcs), dtype=[("name", "S128"), ("dir", "<f4", (2,))])
        sr["name"] = _bytes_array(list(srcs))
        sr["dir"] = np.array(list(srcs.values()), np.float32).reshape(-1, 2)
        w.dataset(root + "/source", sr)
        for name, st in ss.soltabs.items():
            g = f"{root}/{name}"
            attrs = {"TITLE": str(st.get_type()).encode(), "parmdb_type": b"",
                     "h5parm_version": b"1.0"}
            for k, v in st.attrs.items():
                attrs[k] = np.float64(v) if np.isscalar(v) and not isinstance(v, (str, bytes)) else v
            w.group_attrs(g, attrs)
            axes = st.get_axes_names()
            for a in axes:
                w.dataset(f"{g}/{a}", _bytes_array(getattr(st, a)))
            ax = ",".join(axes).encode()
            w.dataset(g + "/val", np.asarray(st.val, np.float64), {"AXES": ax})
            w.dataset(g + "/weight", np.asarray(st.weight).astype(weight_dtype),
                      {"AXES": ax})
            if st.piercepoint is not None:
                w.dataset(g + "/piercepoint", np.asarray(st.piercepoint, np.float64))
    w.save(path)


def get_reference_station(soltab, max_ind=None):
    """utils/processing_utils.py:538-574: first station (among the first
    ``max_ind``) with the largest summed weight."""
    names = soltab.get_axes_names()
    n_ant = len(soltab.ant)
    if max_ind is None or max_ind > n_ant:
        max_ind = n_ant
    w = np.sum(soltab.weight, axis=tuple(i for i, a in enumerate(names) if a != "ant"),
               dtype=np.float64)
    return int(np.nonzero(w[:max_ind] == np.max(w[:max_ind]))[0][0])
