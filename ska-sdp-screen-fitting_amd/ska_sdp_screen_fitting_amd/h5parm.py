"""The subset of the H5parm solution-file API the KL path uses.

Mirrors, for the drop-in, the reference's ``utils/h5parm.py`` objects as far
as ``make_aterm_image`` / ``KLScreen.fit`` / ``stationscreen.run`` touch them
(``H5parm.get_solset`` :78-457, ``Solset.get_soltab/get_source/get_ant/
make_soltab`` :460-799, ``Soltab`` axis access :1306-1324).

Storage backends:

* ``.h5`` / ``.h5parm`` through h5py when h5py is importable (read only; the
  LoSoTo layout: ``/<solset>/<soltab>/{val,weight,<axis>}`` with an ``AXES``
  attribute, ``/<solset>/antenna`` and ``/<solset>/source`` tables);
* ``.npz`` produced by ``tools/h5parm_to_npz.py`` (the GPU box has no h5py):
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
        try:
            import h5py
        except ImportError as exc:  # the GPU box has no h5py
            raise ImportError(
                "reading .h5 H5parm files needs h5py; convert with "
                "tools/h5parm_to_npz.py and pass the .npz") from exc
        with h5py.File(path, "r") as f:
            for ssn in f:
                g = f[ssn]
                ants = g["antenna"][:]
                srcs = g["source"][:]
                ss = Solset(ssn, [a["name"].decode() for a in ants],
                            [a["position"] for a in ants],
                            [s["name"].decode() for s in srcs],
                            [s["dir"] for s in srcs])
                for stn in g:
                    if stn in ("antenna", "source"):
                        continue
                    st = g[stn]
                    axes = st["val"].attrs["AXES"].decode().split(",")
                    avals = []
                    for a in axes:
                        v = st[a][:]
                        if v.dtype.kind == "S":
                            v = v.astype(str)
                        avals.append(v)
                    title = st.attrs.get("TITLE", b"").decode()
                    ss.soltabs[stn] = Soltab(stn, title, axes, avals,
                                             st["val"][:], st["weight"][:], ss)
                self.solsets[ssn] = ss


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
