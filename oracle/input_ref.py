"""Oracle: CPU restatement of the deconvolution input preparation.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Paths relative to
``/root/reference/src/main/java/``; DECON = spim/process/fusion/deconvolution/.

Per view (DECON/ProcessForDeconvolution.java:159-268): the source stack is
resampled into the fused bounding box through the inverse of its affine model,
and a cosine-blending weight is computed at the same source position; the
weights are then normalised across views (DECON/WeightNormalizer.java) and
adjusted for the OSEM speed-up (ProcessForDeconvolution.java:351-384).

PARITY UNPINNED for three imglib2 internals that are not in the container:
the inverse of an ``AffineTransform3D`` (restated: cofactor inverse of the 3x3
part in double), ``AffineTransform3D.applyInverse(float[], float[])``
(restated: subtract the translation, multiply by the inverse 3x3, in double,
round to float) and ``NLinearInterpolator3D`` on ``FloatType`` (restated:
floor, double weights, float accumulation over the corners in the order
000, 100, 110, 010, 011, 111, 101, 001).  The blending function, the virtual
weight transform, ``intersects``, the sum image and the normalisation rules
are restated from the reference's own code, cited per function.
"""
from __future__ import annotations

import math

import numpy as np

from .mvdecon_ref import MIN_VALUE, divide_into_portions

NO_WEIGHTS, PRECOMPUTED_WEIGHTS, VIRTUAL_WEIGHTS = 0, 1, 2   # WeightType subset on the deconvolution path


def blending_lookup() -> np.ndarray:
    """spim/process/fusion/weights/BlendingRealRandomAccess.java:25-33: the table is
    filled at the accumulated double d (d += 0.001), index round(d * 1000)."""
    lut = np.zeros(1001)
    d = 0.0
    while d <= 1.0001:
        lut[int(math.floor(d * 1000.0 + 0.5))] = (math.cos((1 - d) * math.pi) + 1) / 2
        d = d + 0.001
    return lut


LUT = blending_lookup()


def blending_weight(loc: np.ndarray, dims, border, blending) -> np.ndarray:
    """BlendingRealRandomAccess.computeWeight (:78-104) on float32 locations
    loc[..., 3] (source x, y, z); interval min 0, dimMinus1 = dims - 1."""
    loc = np.asarray(loc, np.float32)
    w = np.ones(loc.shape[:-1], np.float32)
    zero = np.zeros(loc.shape[:-1], bool)
    for d in range(3):
        l = loc[..., d]                                         # location - min (min = 0)
        bd = np.float32(border[d])
        a = (l - bd).astype(np.float32)
        b = ((np.float32(dims[d] - 1) - l) - bd).astype(np.float32)
        dist = np.maximum(np.float32(0), np.minimum(a, b)).astype(np.float32)
        zero |= dist == 0
        rel = (dist / np.float32(blending[d])).astype(np.float32)
        m = rel < 1
        idx = np.floor(rel.astype(np.float64) * 1000.0 + 0.5).astype(np.int64)
        idx = np.clip(idx, 0, 1000)
        w = np.where(m, (w.astype(np.float64) * LUT[idx]).astype(np.float32), w)
    return np.where(zero, np.float32(0), w).astype(np.float32)


def invert_affine(model: np.ndarray):
    """Full inverse (3x4, row-major) and the inverse 3x3 of a 3x4 affine model
    (PARITY UNPINNED: imglib2 AffineTransform3D inverse arithmetic)."""
    m = np.asarray(model, np.float64).reshape(3, 4)
    a = m[:, :3]
    det = (a[0, 0] * (a[1, 1] * a[2, 2] - a[1, 2] * a[2, 1])
           - a[0, 1] * (a[1, 0] * a[2, 2] - a[1, 2] * a[2, 0])
           + a[0, 2] * (a[1, 0] * a[2, 1] - a[1, 1] * a[2, 0]))
    inv = np.empty((3, 3))
    inv[0, 0] = (a[1, 1] * a[2, 2] - a[1, 2] * a[2, 1]) / det
    inv[0, 1] = (a[0, 2] * a[2, 1] - a[0, 1] * a[2, 2]) / det
    inv[0, 2] = (a[0, 1] * a[1, 2] - a[0, 2] * a[1, 1]) / det
    inv[1, 0] = (a[1, 2] * a[2, 0] - a[1, 0] * a[2, 2]) / det
    inv[1, 1] = (a[0, 0] * a[2, 2] - a[0, 2] * a[2, 0]) / det
    inv[1, 2] = (a[0, 2] * a[1, 0] - a[0, 0] * a[1, 2]) / det
    inv[2, 0] = (a[1, 0] * a[2, 1] - a[1, 1] * a[2, 0]) / det
    inv[2, 1] = (a[0, 1] * a[2, 0] - a[0, 0] * a[2, 1]) / det
    inv[2, 2] = (a[0, 0] * a[1, 1] - a[0, 1] * a[1, 0]) / det
    t = m[:, 3]
    full = np.empty((3, 4))
    full[:, :3] = inv
    for r in range(3):   # -inv . t, summed in order
        full[r, 3] = -(inv[r, 0] * t[0] + inv[r, 1] * t[1] + inv[r, 2] * t[2])
    return full, inv, t


def _grid(bb_min, bb_dims):
    nx, ny, nz = (int(v) for v in bb_dims)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    return x + int(bb_min[0]), y + int(bb_min[1]), z + int(bb_min[2])


def image_positions(model, bb_min, bb_dims, downsampling: float = 1.0) -> np.ndarray:
    """DECON/TransformInput.java:74-95: s = (float) cursor position + offset,
    t = transform.applyInverse(s) (restated: inv3 . (s - translation) in double,
    rounded to float).  With ``downsampling`` != 1 (weighted-average fusion,
    weightedavg/ProcessParalellPortion.java:86-95) s = pos * ds + bb.min in float.
    Returns float32 [nz, ny, nx, 3]."""
    _, inv, tr = invert_affine(model)
    nx, ny, nz = (int(v) for v in bb_dims)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    s = []
    for g, b in zip((x, y, z), bb_min):
        f = g.astype(np.float32)
        if downsampling != 1.0:
            f = (f * np.float32(downsampling)).astype(np.float32)
        s.append((f + np.float32(b)).astype(np.float32).astype(np.float64))
    d = [s[i] - tr[i] for i in range(3)]
    out = np.empty(x.shape + (3,), np.float32)
    for r in range(3):
        out[..., r] = (inv[r, 0] * d[0] + inv[r, 1] * d[1] + inv[r, 2] * d[2]).astype(np.float32)
    return out


def weight_positions(model, bb_min, bb_dims) -> np.ndarray:
    """spim/process/fusion/weights/TransformedInterpolatedRealRandomAccess.java:96-118:
    t = (double)(position + offset), s = t . inverse (row-packed, with the
    translation column) in double, rounded to float."""
    full, _, _ = invert_affine(model)
    gx, gy, gz = _grid(bb_min, bb_dims)
    t = [g.astype(np.float64) for g in (gx, gy, gz)]
    out = np.empty(gx.shape + (3,), np.float32)
    for r in range(3):
        out[..., r] = (t[0] * full[r, 0] + t[1] * full[r, 1] + t[2] * full[r, 2] + full[r, 3]).astype(np.float32)
    return out


def _mirror(i, n):
    """extendMirrorSingle (numpy 'reflect') of integer index arrays."""
    if n == 1:
        return np.zeros_like(i)
    p = 2 * (n - 1)
    j = np.mod(i, p)
    return np.where(j >= n, p - j, j)


def nlinear(img: np.ndarray, pos: np.ndarray, boundary: str = "mirror") -> np.ndarray:
    """NLinearInterpolator3D on FloatType (PARITY UNPINNED, see the module
    docstring) over extendMirrorSingle ("mirror"), extendPeriodic ("periodic")
    or extendZero ("zero").  img [nz, ny, nx], pos [..., 3] (x, y, z), float32
    or float64 positions."""
    img = np.asarray(img, np.float32)
    nz, ny, nx = img.shape
    p = pos.astype(np.float64)
    f = np.floor(p).astype(np.int64)
    w = p - f
    wi = 1.0 - w
    x0, y0, z0 = f[..., 0], f[..., 1], f[..., 2]

    def at(dx, dy, dz):
        x, y, z = x0 + dx, y0 + dy, z0 + dz
        if boundary == "mirror":
            return img[_mirror(z, nz), _mirror(y, ny), _mirror(x, nx)]
        if boundary == "periodic":
            return img[np.mod(z, nz), np.mod(y, ny), np.mod(x, nx)]
        inside = (x >= 0) & (x < nx) & (y >= 0) & (y < ny) & (z >= 0) & (z < nz)
        v = img[np.clip(z, 0, nz - 1), np.clip(y, 0, ny - 1), np.clip(x, 0, nx - 1)]
        return np.where(inside, v, np.float32(0))

    wt = {(0, 0, 0): wi[..., 0] * wi[..., 1] * wi[..., 2], (1, 0, 0): w[..., 0] * wi[..., 1] * wi[..., 2],
          (0, 1, 0): wi[..., 0] * w[..., 1] * wi[..., 2], (1, 1, 0): w[..., 0] * w[..., 1] * wi[..., 2],
          (0, 0, 1): wi[..., 0] * wi[..., 1] * w[..., 2], (1, 0, 1): w[..., 0] * wi[..., 1] * w[..., 2],
          (0, 1, 1): wi[..., 0] * w[..., 1] * w[..., 2], (1, 1, 1): w[..., 0] * w[..., 1] * w[..., 2]}
    order = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 1, 1), (1, 1, 1), (1, 0, 1), (0, 0, 1)]
    acc = None
    for c in order:
        term = (at(*c).astype(np.float64) * wt[c]).astype(np.float32)   # FloatType.mul(double)
        acc = term if acc is None else (acc + term).astype(np.float32)  # FloatType.add
    return acc


def transform_view(src: np.ndarray, model, bb_min, bb_dims, border, blending, weight_type: int):
    """One view of ProcessForDeconvolution.fuseStacksAndGetPSFs (:159-268):
    (img, raw weight), float32 [nz, ny, nx] in the bounding box."""
    sz, sy, sx = src.shape
    t = image_positions(model, bb_min, bb_dims)
    inside = ((t[..., 0] >= 0) & (t[..., 1] >= 0) & (t[..., 2] >= 0)
              & (t[..., 0] < sx) & (t[..., 1] < sy) & (t[..., 2] < sz))   # FusionHelper.java:54-60
    val = nlinear(src, t)
    img = np.where(inside, np.maximum(np.float32(MIN_VALUE), val), np.float32(0)).astype(np.float32)
    if weight_type == PRECOMPUTED_WEIGHTS:       # TransformInputAndWeights.java:118-120 (same t)
        w = blending_weight(t, (sx, sy, sz), border, blending)
    elif weight_type == VIRTUAL_WEIGHTS:         # TransformedInterpolatedRealRandomAccess
        w = blending_weight(weight_positions(model, bb_min, bb_dims), (sx, sy, sz), border, blending)
    else:
        w = np.ones_like(img)
    return img, w


def normalize_weights(ws, weight_type: int, ij_threads: int = 8):
    """DECON/WeightNormalizer.java:52-205.  Returns (weights, min_overlap, avg_overlap):
    PRECOMPUTED: w_v = (float)(w_v / sum_v w) (ApplyDirectly, always);
    VIRTUAL: the sum image S = sumW > 1 ? (float) sumW : 1 is returned as the
    second element of each weight's pair for ``virtual_weight``; NO_WEIGHTS: as is.
    Overlap statistics per portion (divideIntoPortions(size, 2T)): min of the
    per-voxel count of views with w > 0, average of the per-portion averages."""
    ws = [np.asarray(w, np.float32) for w in ws]
    if weight_type == NO_WEIGHTS:
        return ws, None, None, None
    flat = np.stack([w.reshape(-1) for w in ws])          # [V, N]
    sumw = np.zeros(flat.shape[1])
    for v in range(flat.shape[0]):                         # double sum in view order
        sumw = sumw + flat[v].astype(np.float64)
    count = (flat > 0).sum(axis=0)
    mins, avgs = [], []
    for start, loop in divide_into_portions(flat.shape[1], 2 * ij_threads):
        c = count[start:start + loop]
        mins.append(int(c.min()) if loop else len(ws))
        avgs.append(float(c.sum()) / float(loop) if loop else float("nan"))
    min_ov = min([len(ws)] + [int(round(m)) for m in mins])
    avg_ov = float(np.sum(avgs) / len(avgs))
    if weight_type == PRECOMPUTED_WEIGHTS:
        out = [(flat[v].astype(np.float64) / sumw).astype(np.float32).reshape(ws[0].shape) for v in range(len(ws))]
        return out, None, min_ov, avg_ov
    S = np.where(sumw > 1, sumw.astype(np.float32), np.float32(1)).astype(np.float32).reshape(ws[0].shape)
    return ws, S, min_ov, avg_ov


def osem_speedup(osem_index: int, given: float, min_ov, avg_ov) -> float:
    """ProcessForDeconvolution.java:318-336: 0 = the given value, 1 = minimal,
    2 = average number of overlapping views (each at least 1)."""
    if osem_index == 1:
        return float(max(1, min_ov))
    if osem_index == 2:
        return float(max(1.0, avg_ov))
    return float(given)


def final_weights(ws, S, weight_type: int, osem: float):
    """adjustForOSEM (:351-384) and NormalizingRandomAccess.get (:36-45)."""
    if weight_type == VIRTUAL_WEIGHTS:
        return [np.minimum(1.0, (w.astype(np.float64) / S.astype(np.float64)) * osem).astype(np.float32)
                for w in ws]
    if weight_type == PRECOMPUTED_WEIGHTS and osem != 1.0:
        return [np.minimum(np.float32(1), (w * np.float32(osem)).astype(np.float32)).astype(np.float32)
                for w in ws]
    return [np.asarray(w, np.float32) for w in ws]


def prepare_inputs(srcs, models, bb_min, bb_dims, border, blending, weight_type=VIRTUAL_WEIGHTS,
                   osem_index=0, osem=1.0, ij_threads=8):
    """The whole input preparation: ([img_v], [weight_v], osem used)."""
    imgs, raw = [], []
    for src, m in zip(srcs, models):
        i, w = transform_view(src, m, bb_min, bb_dims, border, blending, weight_type)
        imgs.append(i)
        raw.append(w)
    ws, S, mn, av = normalize_weights(raw, weight_type, ij_threads)
    if weight_type == NO_WEIGHTS:
        return imgs, ws, 1.0
    o = osem_speedup(osem_index, osem, mn, av)
    return imgs, final_weights(ws, S, weight_type, o), o
