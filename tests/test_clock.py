"""CPU: the in-kernel clock reduction (eg_clock_median, include/eg_hip.h) that bench.py reports as
roofline.clock_ghz.  Round 2 summed raw ticks over every workgroup record, so one wrapped or garbage
record published 2e8 GHz; the median of per-workgroup ratios with unset, wrapped and out-of-range
records dropped cannot be moved by a few bad records."""
import ctypes

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__
    __graft_entry__.build_hip()
    from electionguard.core import native
    return native.load()


def median(lib, recs):
    a = np.ascontiguousarray(np.asarray(recs, dtype=np.uint64).reshape(-1, 2))
    ghz, used, dropped = ctypes.c_double(), ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.eg_clock_median(a.ctypes.data_as(ctypes.c_void_p), len(a), ctypes.byref(ghz), ctypes.byref(used),
                               ctypes.byref(dropped)) == 0
    return ghz.value, used.value, dropped.value


def test_median_of_good_records(lib):
    # 100 MHz real-time ticks: 0.1 ms of wall time = 10,000 ticks; 2.2 GHz -> 220,000 shader ticks
    rng = np.random.default_rng(3)
    wall = rng.integers(10_000, 5_000_000, size=501)
    ghz = rng.normal(2.2, 0.01, size=501)
    recs = np.stack([(wall * ghz * 10).astype(np.uint64), wall.astype(np.uint64)], axis=1)
    g, used, dropped = median(lib, recs)
    assert (used, dropped) == (501, 0)
    assert g == pytest.approx(float(np.median((recs[:, 0] / recs[:, 1]) * 0.1)), rel=1e-12)


def test_wrapped_and_garbage_records_are_dropped(lib):
    good = [[22_000_000 + i, 1_000_000] for i in range(9)]              # 10 ms at 2.2 GHz
    wrapped = [[2**64 - 12345, 1_000_000]]                              # negative delta: wrapped
    unset = [[0, 0], [0, 1_000_000], [5_000, 0]]
    garbage = [[22_000_000 * 10**8, 1_000_000], [1, 1_000_000]]         # 2.2e8 GHz, 1e-7 GHz
    short = [[2_200, 500]]                                              # 5 us: too coarse to use
    g, used, dropped = median(lib, good + wrapped + unset + garbage + short)
    assert used == 9 and dropped == 7
    assert g == pytest.approx(22_000_004 / 1_000_000 * 0.1, rel=1e-12)
    # round 2's sum-of-ticks reduction over the same records reads ~1e7 GHz
    recs = np.array(good + wrapped + garbage, dtype=np.float64)
    assert recs[:, 0].sum() / recs[:, 1].sum() * 0.1 > 1e6


def test_no_usable_record_reads_zero(lib):
    assert median(lib, [[0, 0], [2**63, 5]])[:3] == (0.0, 0, 2)
    assert median(lib, np.zeros((0, 2)))[:3] == (0.0, 0, 0)
