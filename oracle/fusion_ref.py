"""Oracle: CPU restatement of the weighted-average fusion.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Paths relative to
``/root/reference/src/main/java/spim/process/fusion/weightedavg/``.

Per fused voxel s (cursor position * downsampling + bb.min, float), for every
view whose inverse-transformed position t lies inside its stack: the value
interpolated over extendMirrorSingle (nearest neighbour or n-linear) and, with
blending, the cosine weight at t.  Result sum(w * v) / sum(w) in double
(ProcessParalellPortionWeight.java:86-127), or the plain mean over the
covering views without weights (ProcessParalellPortion.java:86-120); 0 where
no view covers the voxel.  PARITY UNPINNED for the imglib2 pieces listed in
``oracle/input_ref.py`` and for NearestNeighborInterpolator (restated:
index = floor(t + 0.5)).
"""
from __future__ import annotations

import numpy as np

from . import input_ref as ir


def nearest(img: np.ndarray, pos: np.ndarray) -> np.ndarray:
    nz, ny, nx = img.shape
    i = np.floor(pos.astype(np.float64) + 0.5).astype(np.int64)
    return img[ir._mirror(i[..., 2], nz), ir._mirror(i[..., 1], ny), ir._mirror(i[..., 0], nx)]


def fuse_weighted_average(srcs, models, bb_min, bb_dims, downsampling=1.0, interpolation=1,
                          use_blending=True, borders=None, ranges=None) -> np.ndarray:
    """Returns the fused float32 [nz, ny, nx] volume."""
    shape = (int(bb_dims[2]), int(bb_dims[1]), int(bb_dims[0]))
    acc = np.zeros(shape)
    wsum = np.zeros(shape)
    cnt = np.zeros(shape, np.int64)
    for v, (src, m) in enumerate(zip(srcs, models)):
        src = np.asarray(src, np.float32)
        sz, sy, sx = src.shape
        t = ir.image_positions(m, bb_min, bb_dims, downsampling)
        inside = ((t[..., 0] >= 0) & (t[..., 1] >= 0) & (t[..., 2] >= 0)
                  & (t[..., 0] < sx) & (t[..., 1] < sy) & (t[..., 2] < sz))
        val = (ir.nlinear(src, t) if interpolation == 1 else nearest(src, t)).astype(np.float64)
        if use_blending:
            w = ir.blending_weight(t, (sx, sy, sz), borders[v], ranges[v]).astype(np.float64)
            acc = np.where(inside, acc + val * w, acc)
            wsum = np.where(inside, wsum + w, wsum)
        else:
            acc = np.where(inside, acc + val, acc)
            cnt = cnt + inside
    if use_blending:
        with np.errstate(invalid="ignore", divide="ignore"):
            return np.where(wsum > 0, acc / wsum, 0.0).astype(np.float32)
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.where(cnt > 0, acc / cnt, 0.0).astype(np.float32)
