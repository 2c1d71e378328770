"""H5parm reader (ska_sdp_screen_fitting_amd/hdf5.py)
vs h5py 3.3: files written and read back by h5py in the reference's
interpreter (tests/golden/h5/make_h5_cases.py) -- a DP3-style H5parm holding
the reference fixture's arrays (contiguous layouts, compound tables),
PyTables-style chunked + gzip + shuffle + fletcher32 datasets (float16
weights), vlen / fixed string attributes, a 40-member symbol-table group,
and the libver="latest" format."""

import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from ska_sdp_screen_fitting_amd import hdf5
from ska_sdp_screen_fitting_amd.h5parm import H5parm

H5 = os.path.join(GOLDEN, "h5")


@pytest.fixture(scope="module")
def expected():
    return dict(np.load(os.path.join(H5, "expected.npz")))


def _walk(node, prefix=""):
    for k in node.keys():
        child = node[k]
        name = f"{prefix}{k}"
        yield name, child
        if isinstance(child, hdf5.Group):
            yield from _walk(child, name + "/")


@pytest.mark.parametrize("tag", ["cases_v0", "cases_latest"])
def test_reader_matches_h5py(expected, tag):
    seen = 0
    with hdf5.File(os.path.join(H5, tag + ".h5")) as f:
        for name, node in _walk(f.root):
            for k, v in node.attrs.items():
                want = expected[f"{tag}@{name}@{k}"]
                got = np.array(v)
                if want.dtype.kind == "U":
                    got = got.astype("U")
                np.testing.assert_array_equal(got, want, err_msg=f"{name}@{k}")
                seen += 1
            if isinstance(node, hdf5.Dataset):
                got = node[()]
                parts = ([(f"{tag}:{name}#{fld}", got[fld]) for fld in got.dtype.names]
                         if got.dtype.names else [(f"{tag}:{name}", got)])
                for key, arr in parts:
                    want = expected[key]
                    assert arr.shape == want.shape, key
                    assert arr.dtype.newbyteorder("=") == want.dtype.newbyteorder("="), key
                    np.testing.assert_array_equal(arr, want, err_msg=key)
                    seen += 1
    n_exp = sum(1 for k in expected if k.startswith(tag + ":") or k.startswith(tag + "@"))
    assert seen == n_exp


def test_dp3_like_h5parm_matches_fixture():
    g = load_golden("fixture_kl")
    h5 = H5parm(os.path.join(H5, "dp3_like.h5"))
    ss = h5.get_solset("sol000")
    st = ss.get_soltab("phase000")
    np.testing.assert_array_equal(st.val, g["val"])
    np.testing.assert_array_equal(st.weight, g["weight"])
    np.testing.assert_array_equal(st.time, g["times"])
    assert list(st.dir) == [str(d) for d in g["dir_names"]]
    assert list(st.ant) == [str(a) for a in g["ant_names"]]
    np.testing.assert_array_equal(np.array(list(ss.get_source().values())), g["dir_radec"])
    np.testing.assert_array_equal(np.array(list(ss.get_ant().values())), g["ant_pos"])


def test_amplitude_soltab_with_pol_and_f16_weights():
    h5 = H5parm(os.path.join(H5, "cases_v0.h5"))
    st = h5.get_solset("sol000").get_soltab("amplitude000")
    assert st.get_type() == "amplitude"
    assert st.get_axes_names() == ["time", "freq", "ant", "dir", "pol"]
    assert st.val.shape == (6, 4, 5, 3, 2) and st.weight.dtype == np.float32
    assert list(st.pol) == ["XX", "YY"]


def test_not_hdf5(tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"not an hdf5 file" * 10)
    with pytest.raises(hdf5.H5FormatError):
        hdf5.File(str(p))


def _screen_h5parm():
    """fixture_kl solutions plus a screen soltab shaped as stationscreen.run
    makes it (attrs + piercepoint)."""
    g = load_golden("fixture_kl")
    h5 = H5parm(os.path.join(GOLDEN, "fixture_kl.npz"))
    ss = h5.get_solset("sol000")
    st = ss.get_soltab("phase000")
    scr = ss.make_soltab("phasescreen", "phase_screen000",
                         axes_names=st.get_axes_names(),
                         axes_vals=[st.time, st.freq, st.ant, st.dir],
                         vals=g["coef"], weights=g["w_out"])
    scr.attrs.update(beta=5.0 / 3.0, r_0=100, height=0.0,
                     midra=float(g["mid_ra"]), middec=float(g["mid_dec"]))
    scr.piercepoint = g["piercepoints"]
    return g, h5


def test_h5parm_write_read_roundtrip(tmp_path):
    g, h5 = _screen_h5parm()
    path = str(tmp_path / "out.h5")
    h5.save(path)
    back = H5parm(path).get_solset("sol000")
    orig = h5.get_solset("sol000")
    assert sorted(back.get_soltab_names()) == sorted(orig.get_soltab_names())
    for name in orig.get_soltab_names():
        a, b = orig.get_soltab(name), back.get_soltab(name)
        assert b.get_type() == a.get_type()
        assert b.get_axes_names() == a.get_axes_names()
        np.testing.assert_array_equal(b.val, a.val)
        # weights are stored as float16 (utils/h5parm.py make_soltab default)
        np.testing.assert_array_equal(b.weight, np.asarray(a.weight).astype(np.float16))
        for ax in a.get_axes_names():
            np.testing.assert_array_equal(np.asarray(getattr(b, ax)),
                                          np.asarray(getattr(a, ax)))
    scr = back.get_soltab("phase_screen000")
    np.testing.assert_array_equal(scr.piercepoint, g["piercepoints"])
    assert scr.attrs["r_0"] == 100 and scr.attrs["midra"] == float(g["mid_ra"])
    assert back.get_ant().keys() == orig.get_ant().keys()
    for k, v in orig.get_source().items():
        np.testing.assert_array_equal(back.get_source()[k], v)


def test_writer_many_members_and_types(tmp_path):
    w = hdf5.Writer()
    for k in range(100):  # 13 symbol-table leaves
        w.dataset(f"/grp/d{k:03d}", np.full(k % 5 + 1, k, np.int64))
    w.dataset("/grp/f2", np.arange(7, dtype=np.float16))
    w.dataset("/grp/u1", np.arange(3, dtype=np.uint8), {"s": b"x", "v": np.arange(2.0)})
    w.dataset("/scalar", np.float32(3.5))
    w.group_attrs("/", {"top": np.int32(-7)})
    path = str(tmp_path / "w.h5")
    w.save(path)
    with hdf5.File(path) as f:
        assert f.attrs["top"] == -7
        grp = f["grp"]
        assert len(grp.keys()) == 102
        for k in range(100):
            np.testing.assert_array_equal(grp[f"d{k:03d}"][()], np.full(k % 5 + 1, k))
        np.testing.assert_array_equal(f["grp/f2"][()], np.arange(7, dtype=np.float16))
        assert f["grp/u1"].attrs["s"] == b"x"
        np.testing.assert_array_equal(f["grp/u1"].attrs["v"], [0.0, 1.0])
        assert f["scalar"].shape == () and f["scalar"][()] == np.float32(3.5)


REF_H5 = "/root/reference/resources/solutions.h5"


@pytest.mark.skipif(not os.path.exists(REF_H5),
                    reason="the reference tree is only present in the build container")
def test_reference_solutions_h5_reads_as_fixture():
    """The reference's own resources/solutions.h5 (the file its tests feed
    make_aterm_image, written by DP3 / PyTables) read by this build's HDF5
    reader equals the golden fixture the reference itself produced from it
    (make_golden.py read it with h5py)."""
    g = load_golden("fixture_kl")
    ss = H5parm(REF_H5).get_solset("sol000")
    st = ss.get_soltab("phase000")
    assert st.get_axes_names() == ["time", "freq", "ant", "dir"]
    np.testing.assert_array_equal(st.val, g["val"])
    np.testing.assert_array_equal(st.weight, g["weight"])
    np.testing.assert_array_equal(st.time, g["times"])
    np.testing.assert_array_equal(st.freq, g["freqs"])
    assert list(st.dir) == [str(d) for d in g["dir_names"]]
    assert list(st.ant) == [str(a) for a in g["ant_names"]]
    src, ant = ss.get_source(), ss.get_ant()
    np.testing.assert_array_equal(np.array([src[str(d)] for d in g["dir_names"]]),
                                  g["dir_radec"])
    np.testing.assert_array_equal(np.array([ant[str(a)] for a in g["ant_names"]]),
                                  g["ant_pos"])
