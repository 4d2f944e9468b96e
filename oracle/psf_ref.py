"""CPU restatement of PSF extraction / transformation.

TEST INFRASTRUCTURE ONLY: imported by tests/ (the checker), never by the
product path.  PARITY UNPINNED: the reference (Java) cannot be built here and
holds no PSF fixtures; the imglib2 pieces it calls (AffineTransform3D inverse /
apply / estimateBounds, NLinearInterpolator3D, extendPeriodic / extendZero)
are restated as in oracle/input_ref.py.

Follows spim/process/fusion/deconvolution/ExtractPSF.java (paths under
/root/reference/src/main/java/):
  extract_psf_local        extractPSFLocal   :383-422
  normalize                normalize         :281-299
  transformed_size         transformPSF      :309-346 (size + offset)
  transform                transform         :424-460
  extract_next_img         extractNextImg    :260-279
  average_transformed_psf  computeAverageTransformedPSF :164-208
  max_projection           computeMaxProjection :110-162
"""
import numpy as np

from oracle.input_ref import invert_affine, nlinear


def apply(model, p):
    """AffineTransform3D.apply: row r = m[r,0]*x + m[r,1]*y + m[r,2]*z + m[r,3]."""
    m = np.asarray(model, np.float64).reshape(3, 4)
    p = np.asarray(p, np.float64)
    return np.stack([p[..., 0] * m[r, 0] + p[..., 1] * m[r, 1] + p[..., 2] * m[r, 2] + m[r, 3]
                     for r in range(3)], axis=-1)


def extract_psf_local(img: np.ndarray, locations, size) -> np.ndarray:
    """:383-422 -- float sum, in location order, of the n-linear samples of the
    periodic-extended image at (i - size/2 + location).  size (x, y, z)."""
    sx, sy, sz = (int(v) for v in size)
    z, y, x = np.meshgrid(np.arange(sz), np.arange(sy), np.arange(sx), indexing="ij")
    rel = np.stack([x - sx // 2, y - sy // 2, z - sz // 2], axis=-1).astype(np.float64)
    psf = np.zeros((sz, sy, sx), np.float32)
    for loc in locations:
        pos = rel + np.asarray(loc, np.float64)
        psf = (psf + nlinear(img, pos, "periodic")).astype(np.float32)
    return psf


def extract_psf_local_batched(img: np.ndarray, locations, size, chunk: int = 512) -> np.ndarray:
    """extract_psf_local vectorised over chunks of beads, same result bit for bit: the
    samples of a chunk are computed at once (nlinear is elementwise) and summed in
    location order by np.add.accumulate (a strictly left-to-right float32 scan, unlike
    np.sum's pairwise reduction).  For the many-bead PSFs of the C4 views."""
    sx, sy, sz = (int(v) for v in size)
    z, y, x = np.meshgrid(np.arange(sz), np.arange(sy), np.arange(sx), indexing="ij")
    rel = np.stack([x - sx // 2, y - sy // 2, z - sz // 2], axis=-1).astype(np.float64)
    locs = np.asarray(locations, np.float64).reshape(-1, 3)
    psf = np.zeros((sz, sy, sx), np.float32)
    for c0 in range(0, len(locs), chunk):
        pos = rel[None] + locs[c0:c0 + chunk, None, None, None, :]
        samples = nlinear(img, pos, "periodic")                       # [n, sz, sy, sx] float32
        psf = np.add.accumulate(np.concatenate([psf[None], samples]), axis=0, dtype=np.float32)[-1]
    return psf


def normalize(psf: np.ndarray) -> np.ndarray:
    """:281-299 -- (v - min) / (max - min) in double, stored as float."""
    v = psf.astype(np.float64)
    finite = v[~np.isnan(v)]                      # NaN never wins `v < min` / `v > max`
    mn = finite.min() if finite.size else np.finfo(np.float64).max
    mx = finite.max() if finite.size else -np.finfo(np.float64).max
    with np.errstate(invalid="ignore", divide="ignore"):
        return ((v - mn) / (mx - mn)).astype(np.float32)


def transformed_size(size, model):
    """:309-346 -- odd output size (the transformed bounding box of [0, dim-1],
    truncated + 1, made odd) and the offset that keeps the centre voxel the
    centre: offset = model(dim / 2) - newSize / 2 (integer halves)."""
    size = [int(v) for v in size]
    corners = np.array([[cx, cy, cz] for cz in (0, size[2] - 1) for cy in (0, size[1] - 1)
                        for cx in (0, size[0] - 1)], np.float64)
    t = apply(model, corners)
    lo, hi = t.min(axis=0), t.max(axis=0)
    new = []
    for d in range(3):
        n = int(hi[d] - lo[d]) + 1
        new.append(n + 1 if n % 2 == 0 else n)
    c = apply(model, np.array([s // 2 for s in size], np.float64))
    off = [float(c[d] - (new[d] // 2)) for d in range(3)]
    return new, off


def transform(psf: np.ndarray, model, new_size, offset) -> np.ndarray:
    """:424-460 -- out[i] = nlinear over extendZero at inverse(model)(i + offset)."""
    full, _, _ = invert_affine(model)
    nx, ny, nz = (int(v) for v in new_size)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    p = np.stack([x + offset[0], y + offset[1], z + offset[2]], axis=-1).astype(np.float64)
    return nlinear(psf, apply(full, p), "zero")


def transform_psf(psf: np.ndarray, model):
    new, off = transformed_size((psf.shape[2], psf.shape[1], psf.shape[0]), model)
    return transform(psf, model, new, off)


def extract_next_img(img, model, locations, size):
    """:260-279 -- (normalised original-calibration PSF, transformed PSF)."""
    orig = normalize(extract_psf_local(img, locations, size))
    return orig, transform_psf(orig, model)


def average_transformed_psf(psfs):
    """:164-208 -- sum of the PSFs, each point-mirrored about its centre into a
    max-size image (loc -> psfCenter - loc + avgCenter; outside dropped)."""
    mx = [max(p.shape[2 - d] for p in psfs) for d in range(3)]
    avg = np.zeros((mx[2], mx[1], mx[0]), np.float32)
    ac = [m // 2 for m in mx]
    for p in psfs:
        nz, ny, nx = p.shape
        pc = [nx // 2, ny // 2, nz // 2]
        z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
        tx, ty, tz = pc[0] - x + ac[0], pc[1] - y + ac[1], pc[2] - z + ac[2]
        ok = (tx >= 0) & (tx < mx[0]) & (ty >= 0) & (ty < mx[1]) & (tz >= 0) & (tz < mx[2])
        add = np.zeros_like(avg)
        add[tz[ok], ty[ok], tx[ok]] = p[ok]          # the mapping is one-to-one
        hit = np.zeros(avg.shape, bool)
        hit[tz[ok], ty[ok], tx[ok]] = True
        avg = np.where(hit, (avg + add).astype(np.float32), avg)
    return avg


def max_projection(img: np.ndarray, min_dim: int = -1):
    """:110-162 -- max along min_dim (x=0, y=1, z=2; < 0: the first smallest
    dimension); the remaining dims keep their order."""
    dims = [img.shape[2], img.shape[1], img.shape[0]]
    if min_dim < 0:
        min_dim = 0
        for d in range(3):
            if dims[d] < dims[min_dim]:
                min_dim = d
    axis = 2 - min_dim
    return img.max(axis=axis).astype(np.float32), min_dim
