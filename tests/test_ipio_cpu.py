"""CPU: the interest-point list files (.ip.txt) written and read by the library's
host-side entry points (no GPU involved), against the oracle restatement of
InterestPointList.saveInterestPoints / loadInterestPoints and Double.toString."""
import math
import os

import numpy as np
import pytest

from oracle import ip_ref
from spim_registration_amd import _lib
from spim_registration_amd.dog import InterestPoint, InterestPointList, java_double_to_string

KNOWN = [  # java.lang.Double.toString (spec examples and boundaries)
    (1.0, "1.0"), (12.0, "12.0"), (100.0, "100.0"), (0.001, "0.001"), (0.0015, "0.0015"), (1e-4, "1.0E-4"),
    (9999999.0, "9999999.0"), (1e7, "1.0E7"), (1.5e7, "1.5E7"), (123.456, "123.456"), (-2.5, "-2.5"),
    (0.1 + 0.2, "0.30000000000000004"), (1e23, "1.0E23"), (0.0, "0.0"), (-0.0, "-0.0"),
    (float("nan"), "NaN"), (float("inf"), "Infinity"), (5e-324, "4.9E-324"),
    (1.7976931348623157e308, "1.7976931348623157E308"), (float(np.float32(12.3456)), "12.345600128173828"),
]


def test_java_double_to_string_known_answers(lib):
    for v, s in KNOWN:
        assert ip_ref.java_double_to_string(v) == s, (v, s)
        assert java_double_to_string(v) == s, (v, s)


def test_java_double_to_string_matches_oracle_random(lib):
    rng = np.random.default_rng(5)
    vals = np.concatenate([rng.random(2000) * 2048, rng.normal(0, 1, 500), 10.0 ** rng.uniform(-8, 12, 500),
                           rng.integers(0, 2048, 300).astype(np.float64),
                           rng.random(300).astype(np.float32).astype(np.float64) * 1000])
    for v in vals:
        assert java_double_to_string(v) == ip_ref.java_double_to_string(v), v
        assert float(java_double_to_string(v).replace("E", "e")) == v


def test_save_and_load_interest_points(lib, tmp_path):
    rng = np.random.default_rng(6)
    pos = rng.random((257, 3)) * 700
    pos[:40] = np.floor(pos[:40])                         # localization 0: integer positions
    pts = [InterestPoint(i, tuple(p)) for i, p in enumerate(pos)]
    ipl = InterestPointList(tmp_path, "interestpoints/tpId_0_viewSetupId_3.beads")
    assert not ipl.save_interest_points()                  # no list yet (:68-71)
    ipl.set_interest_points(pts)
    assert ipl.save_interest_points()
    path = tmp_path / "interestpoints" / "tpId_0_viewSetupId_3.beads.ip.txt"
    assert path.read_text() == ip_ref.ip_txt(pos)          # byte for byte
    back = InterestPointList(tmp_path, "interestpoints/tpId_0_viewSetupId_3.beads")
    assert back.load_interest_points()
    got = back.get_interest_points()
    assert [p.id for p in got] == list(range(len(pos)))
    np.testing.assert_array_equal(np.array([p.location for p in got]), pos)


def test_load_skips_preamble_and_keeps_ids(lib, tmp_path):
    (tmp_path / "x.ip.txt").write_text("# note\nid\tx\ty\tz\n7\t1.0\t2.5\t3.0E-4\n9\t4.0\t5.0\t6.0\n")
    ipl = InterestPointList(str(tmp_path), "x")
    assert ipl.load_interest_points()
    assert [(p.id, p.location) for p in ipl.get_interest_points()] == [(7, (1.0, 2.5, 3e-4)), (9, (4.0, 5.0, 6.0))]
    # a missing file is the reference's caught IOException: false, no exception (:209-214)
    assert InterestPointList(str(tmp_path), "missing").load_interest_points() is False


def test_load_trims_fields_like_java(lib, tmp_path):
    """p[i].trim() before parseInt / parseDouble (InterestPointList.java:194-199): blanks
    around every tab-separated field are accepted; a non-number still raises."""
    (tmp_path / "w.ip.txt").write_text("id\tx\ty\tz\n 3 \t 1.5 \t2.0 \t 4.25 \r\n4\t0.5\t0.25\t1.0E1\n")
    ipl = InterestPointList(str(tmp_path), "w")
    assert ipl.load_interest_points()
    assert [(p.id, p.location) for p in ipl.get_interest_points()] == [(3, (1.5, 2.0, 4.25)), (4, (0.5, 0.25, 10.0))]
    (tmp_path / "bad.ip.txt").write_text("id\tx\ty\tz\n3\tabc\t2.0\t4.0\n")
    with pytest.raises(_lib.SpimDeconError):
        InterestPointList(str(tmp_path), "bad").load_interest_points()


def test_convolution_cpu_has_no_cpu_path(lib):
    img = np.ones((4, 4, 4), np.float32)
    k = np.ones(3, np.float32)
    st = lib.convolutionCPU(_lib.fptr(img), _lib.fptr(k), _lib.fptr(k), _lib.fptr(k), 1, 1, 1, 4, 4, 4, 0, 0.0)
    assert st == -2 and "no CPU path" in _lib.last_error()
    assert (img == 1).all()
