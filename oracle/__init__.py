"""CPU oracle for the KL screen path -- TEST INFRASTRUCTURE ONLY.

This package is a plain numpy (float64) restatement of the reference
algorithm (ska-sdp-screen-fitting v0.1.0, ``/root/reference``).  It is the
*checker*: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product package
(``ska-sdp-screen-fitting_amd/ska_sdp_screen_fitting_amd``) never imports or
calls anything here; its compute path is the HIP library and fails loudly
when that library is missing.

Parity status: PINNED.  The restatement is checked against golden vectors
produced by running the reference itself (``tests/golden/make_golden.py``,
committed outputs ``tests/golden/*.npz``), see ``tests/test_oracle_golden.py``.
"""

from .geometry import (  # noqa: F401
    getxy, grid_coords, piercepoints, sin_world2pix, tan_pix2world,
    tan_world2pix)
from .kl import (  # noqa: F401
    calculate_svd, circ_chi2, cpix_matrix, eval_phase_screens, eval_planes,
    fit_screen, fit_slot, flag_outliers_slot, nancircstd, normalize_phase,
    reference_station, run_phase, station_orders)
