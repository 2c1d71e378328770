"""Host-side logic of the product package (CPU): geometry, orders, time
chunking, FITS writer, solution-file loader."""

import json
import os

import numpy as np
import pytest

from conftest import FIELD, GOLDEN, load_golden
from ska_sdp_screen_fitting_amd import fits as sffits
from ska_sdp_screen_fitting_amd import geometry
from ska_sdp_screen_fitting_amd.h5parm import H5parm, get_reference_station
from ska_sdp_screen_fitting_amd.screen import _angle_deg, time_chunks
from ska_sdp_screen_fitting_amd.stationscreen import station_orders


def test_product_geometry_vs_reference(golden):
    pp, mra, mdec = geometry.piercepoints(golden["dir_radec"])
    assert mra == golden["mid_ra"] and mdec == golden["mid_dec"]
    np.testing.assert_allclose(pp, golden["piercepoints"], rtol=0, atol=1e-9)
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"], 0.2,
                                mra, mdec)
    np.testing.assert_allclose(x, golden["x17"], atol=1e-9)
    np.testing.assert_allclose(y, golden["y17"], atol=1e-9)


@pytest.mark.parametrize("n", [17, 128, 256, 512])
def test_grid_size_rule(n):
    cell = {17: 0.2, 128: 0.02602, 256: 0.01301, 512: 0.006505}[n]
    assert geometry.grid_size(FIELD["width"], cell) == n
    g = load_golden("fixture_kl")
    x, y = geometry.grid_coords(FIELD["rad"], FIELD["dec"], FIELD["width"], cell,
                                float(g["mid_ra"]), float(g["mid_dec"]))
    np.testing.assert_allclose(x, g[f"coords{n}_x"], atol=1e-9)


def test_station_orders_vs_reference(golden):
    ref = int(golden["ref_ant"])
    st = station_orders(golden["ant_pos"], ref, int(golden["order"]))
    # the reference's initial orders survive where nothing was adapted;
    # at least the ref-skipped / unadapted stations carry them
    o = golden["orders"]
    for a in range(len(st)):
        if a == ref:
            continue
        vals = set(np.unique(o[:, :, a]).tolist()) - {0}
        if len(vals) == 1 and golden["name"] == "fixture_kl":
            assert vals == {st[a]}
    assert all(5 <= v <= int(golden["order"]) for v in st)


def test_reference_station(golden):
    h = H5parm(os.path.join(GOLDEN, "fixture_kl.npz"))
    st = h.get_solset("sol000").get_soltab("phase000")
    assert get_reference_station(st, 10) == 0
    assert st.get_axes_names() == ["time", "freq", "ant", "dir"]
    assert len(st.dir) == 7 and len(st.ant) == 62


def test_time_chunks_gaps_and_memory():
    t = np.arange(20) * 8.0
    assert time_chunks(t, 0.001, available_gb=100) == [20]
    t2 = np.concatenate([t, 200 + np.arange(5) * 8.0])
    assert time_chunks(t2, 0.001, available_gb=100) == [20, 25]
    # memory: at most 6 per chunk -> halving (screen.py:305-317)
    assert time_chunks(t, 1.0, available_gb=6) == [5, 10, 15, 20]


def test_angle_parsing():
    assert _angle_deg(12.5) == 12.5
    assert _angle_deg("8h37m42s") == pytest.approx((8 + 37 / 60 + 42 / 3600) * 15)
    assert _angle_deg("-65d13m47s") == pytest.approx(-(65 + 13 / 60 + 47 / 3600))


def test_fits_header_matches_reference(tmp_path):
    g = load_golden("fixture_kl")
    want = json.load(open(os.path.join(GOLDEN, "fixture_headers.json")))
    for n, cell in ((17, 0.2), (128, 0.02602)):
        cards = sffits.aterm_header(126.23, 64.5, n, n, cell, g["freqs"],
                                    g["times"][0:20], 62)
        assert [k for k, _ in cards] == [k for k, _ in want[str(n)]]
        for (k, v), (k2, v2) in zip(cards, want[str(n)]):
            if isinstance(v2, float):
                # the value as written in the card text (16 significant digits)
                assert float(sffits.card(k, v)[10:30]) == v2, k
            elif k in ("SIMPLE", "EXTEND"):
                assert v is True
            else:
                assert v == v2, k
        shape = (2, 3, 4, 4, n, n)
        data = np.random.default_rng(0).normal(size=shape).astype(np.float32)
        path = str(tmp_path / f"c{n}.fits")
        w = sffits.CubeWriter(path, cards[:3] + [("NAXIS1", n), ("NAXIS2", n),
                                                  ("NAXIS3", 4), ("NAXIS4", 4),
                                                  ("NAXIS5", 3), ("NAXIS6", 2)]
                              + cards[10:], shape)
        w.write(data[:1])
        w.write(data[1:])
        w.close()
        assert os.path.getsize(path) % 2880 == 0
        hdr, back = sffits.read_cube(path)
        np.testing.assert_array_equal(back, data)
        assert hdr["CTYPE1"] == "RA---SIN" and hdr["CDELT1"] == -cell


def test_fits_card_format():
    assert sffits.card("CRVAL1", 126.23) == "CRVAL1  =               126.23".ljust(80)
    assert sffits.card("CTYPE1", "RA---SIN") == "CTYPE1  = 'RA---SIN'".ljust(80)
    assert sffits.card("SIMPLE", True) == "SIMPLE  =                    T".ljust(80)
    assert sffits.card("CUNIT3", "") == "CUNIT3  = '        '".ljust(80)


def test_wg_jacobi_pair_shares_cover_every_pair_once():
    """wg_jacobi<NW> (sf_wave.h) splits each round's column pairs into
    consecutive shares, one per wave: for every subset size (1..63
    directions) and wave count, every pair belongs to exactly one wave, so
    each column of a round is written once (the same rotations as the
    one-wave solve)."""
    for nw in (1, 2, 3, 4):
        for n in range(1, 64):
            m = n + (n & 1)
            npairs = m // 2
            share = (npairs + nw - 1) // nw
            owned = []
            for w in range(nw):
                kb = min(w * share, npairs)
                ke = min(kb + share, npairs)
                owned.extend(range(kb, ke))
            assert sorted(owned) == list(range(npairs)), (nw, n)


def test_private_context_pool(monkeypatch):
    """_lib.private_context (round 6): a context is held by one block at a
    time, reused once released, and at most _IDLE_MAX idle contexts per
    device are kept (the rest closed) -- checked with a stand-in Context,
    no GPU."""
    import threading
    from ska_sdp_screen_fitting_amd import _lib

    made, closed = [], []

    class Fake:
        def __init__(self, device):
            self.device = device
            made.append(self)

        def close(self):
            closed.append(self)

    monkeypatch.setattr(_lib, "Context", Fake)
    monkeypatch.setattr(_lib, "_idle", {})
    with _lib.private_context(3) as a:
        with _lib.private_context(3) as b:
            assert a is not b                      # held exclusively
    with _lib.private_context(3) as c:
        assert c in (a, b)                         # reused, not created
    assert len(made) == 2
    # many concurrent holders: at most _IDLE_MAX stay idle afterwards
    n = _lib._IDLE_MAX + 3
    barrier = threading.Barrier(n)
    held = []

    def hold():
        with _lib.private_context(5) as ctx:
            held.append(ctx)
            barrier.wait()

    ths = [threading.Thread(target=hold) for _ in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert len({id(x) for x in held}) == n
    assert len(_lib._idle[5]) == _lib._IDLE_MAX and len(closed) == 3
