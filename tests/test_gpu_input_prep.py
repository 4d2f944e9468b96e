"""GPU parity of the deconvolution input preparation against the oracle."""
import math

import numpy as np
import pytest

from oracle import input_ref as ir
from oracle import fusion_ref as fr
from spim_registration_amd.input_prep import WeightType, fuse_weighted_average, prepare_inputs

pytestmark = pytest.mark.gpu


def rot(axis, deg):
    c, s = math.cos(math.radians(deg)), math.sin(math.radians(deg))
    if axis == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def views(V=3, shape=(18, 20, 22), seed=5):
    rng = np.random.default_rng(seed)
    srcs, models = [], []
    for v in range(V):
        srcs.append((rng.random(shape) * 100 + 1).astype(np.float32))
        a = rot("y", 360.0 / V * v + 7) @ rot("z", 5 * v) @ np.diag([1.0, 1.0, 1.6])
        m = np.zeros((3, 4))
        m[:, :3] = a
        m[:, 3] = [2.3 + v, -1.7, 3.1 * v]
        models.append(m)
    return srcs, models


def assert_mismatches_on_ties(got, want, models, bb_min, bb_dims, ds=1.0, half=False, rtol=1e-5):
    """Every voxel where the GPU and the oracle differ by more than rtol must sit on a
    decision boundary of the float32 source position t = inverse(model)(s) of some
    view: a coordinate within 4 ulp of an integer (the floor of n-linear
    interpolation and the inside test t >= 0, t < size) or, with nearest-neighbour
    interpolation (``half``), of a half-integer (floor(t + 0.5)).  Those are the
    voxels where a 1-ulp difference in the double->float position flips a discrete
    choice; anywhere else the results agree within rtol."""
    bad = np.abs(got - want) > rtol * np.maximum(1, np.abs(want))
    if not bad.any():
        return 0
    idx = np.nonzero(bad)
    near = np.zeros(len(idx[0]), bool)
    for m in models:
        t = ir.image_positions(m, bb_min, bb_dims, ds)[idx]           # [n, 3] float32
        t64 = t.astype(np.float64)
        ulp = np.spacing(np.abs(t)).astype(np.float64)
        for off in ((0.0, 0.5) if half else (0.0,)):
            d = np.abs(t64 + off - np.round(t64 + off))
            near |= (d <= 4 * ulp + 1e-12).any(axis=1)
    assert near.all(), (int((~near).sum()), [tuple(int(i[k]) for i in idx) for k in np.nonzero(~near)[0][:5]])
    assert bad.mean() < 1e-3
    return int(bad.sum())


@pytest.mark.parametrize("wt", list(WeightType))
@pytest.mark.parametrize("osem_index,osem", [(0, 1.0), (0, 2.5), (1, 1.0), (2, 1.0)])
def test_prepare_inputs_matches_oracle(gpu, wt, osem_index, osem):
    srcs, models = views()
    bb_min, bb_dims = (-12, -10, -8), (40, 34, 30)
    imgs, ws, info = prepare_inputs(srcs, models, bb_min, bb_dims, (-2, -2, -1), (6, 6, 4), wt,
                                    osem_index, osem)
    ei, ew, eo = ir.prepare_inputs(srcs, models, bb_min, bb_dims, (-2, -2, -1), (6, 6, 4), int(wt),
                                   osem_index, osem)
    for v in range(len(srcs)):
        assert_mismatches_on_ties(imgs[v], ei[v], [models[v]], bb_min, bb_dims)
        np.testing.assert_allclose(ws[v], ew[v], rtol=1e-5, atol=1e-6)
        assert (imgs[v] > 0).any() and (imgs[v] == 0).any()  # bounding box larger than a view
    if wt != WeightType.NO_WEIGHTS:
        assert info["osem"] == pytest.approx(eo)


def test_identity_model_reproduces_source(gpu):
    """An identity model over the source's own extent is a copy (>= minValue)."""
    srcs, _ = views(V=1)
    ident = np.hstack([np.eye(3), np.zeros((3, 1))])
    s = srcs[0]
    imgs, ws, _ = prepare_inputs([s], [ident], (0, 0, 0), (s.shape[2], s.shape[1], s.shape[0]),
                                 weight_type=WeightType.NO_WEIGHTS)
    np.testing.assert_array_equal(imgs[0], np.maximum(np.float32(1e-4), s))
    assert (ws[0] == 1).all()


@pytest.mark.parametrize("interp,blend,ds", [(1, True, 1.0), (0, True, 1.0), (1, False, 1.0), (1, True, 2.0),
                                             (0, False, 1.5)])
def test_weighted_average_fusion_matches_oracle(gpu, interp, blend, ds):
    """SURVEY 8f #3 (BASELINE configs[0] plumbing): weighted-average fusion."""
    srcs, models = views(V=2)
    bb_min, bb_dims = (-10, -9, -8), (36, 30, 26)
    borders, ranges = [(0, 0, 0), (1, 1, 0)], [(5, 5, 3), (4, 6, 3)]
    got = fuse_weighted_average(srcs, models, bb_min, bb_dims, ds, interp, blend, borders, ranges)
    want = fr.fuse_weighted_average(srcs, models, bb_min, bb_dims, ds, interp, blend, borders, ranges)
    assert_mismatches_on_ties(got, want, models, bb_min, bb_dims, ds, half=(interp == 0))
    assert (want > 0).any() and (want == 0).any()
