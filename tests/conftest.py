import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "ska-sdp-screen-fitting_amd"))
sys.path.insert(0, REPO)

GOLDEN_SETS = ("fixture_kl", "synth20", "synth12tiny", "synth50")
FIELD = dict(rad=126.23, dec=64.50, width=3.3300000000000054)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


@pytest.fixture(params=GOLDEN_SETS)
def golden(request):
    g = load_golden(request.param)
    g["name"] = request.param
    return g
