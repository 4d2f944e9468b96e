"""Oracle: CPU restatement of the multiview Bayesian/RL deconvolution hot path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  PARITY UNPINNED: the
Java reference cannot run here; every function cites the reference lines it
restates.  Paths are relative to ``/root/reference/src/main/java/``:

  DECON = spim/process/fusion/deconvolution/
  CUDA  = spim/process/cuda/
  FFTM  = fftMethods/

Conventions: volumes are numpy float32 arrays indexed ``[z, y, x]`` (x fastest,
i.e. ImgLib2 ``ArrayImg`` flat order).  Kernels are odd-sized.  Reductions are
float64 (``RealSum``).  Convolutions are evaluated in float64 and rounded to
float32 once (the reference uses a float FFT; the difference is ~1e-7 rel).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import IntEnum

import numpy as np
import scipy.fft
import scipy.signal

MIN_VALUE = np.float32(0.0001)  # DECON/MVDeconvolution.java:49


class PSFTYPE(IntEnum):
    """DECON/MVDeconFFT.java:28 (ordinal order preserved)."""
    OPTIMIZATION_II = 0
    OPTIMIZATION_I = 1
    EFFICIENT_BAYESIAN = 2
    INDEPENDENT = 3


# --------------------------------------------------------------------------
# portions / sums / normalisation
# --------------------------------------------------------------------------

def divide_into_portions(size: int, num_portions: int):
    """spim/process/fusion/FusionHelper.java:236-258.

    Returns [(start, loop_size)]: chunk = size // n, the last portion also gets
    the remainder."""
    chunk = size // num_portions
    mod = size % num_portions
    out = []
    for pid in range(num_portions):
        start = pid * chunk
        loop = chunk + mod if pid == num_portions - 1 else chunk
        out.append((start, loop))
    return out


def sum_img(img: np.ndarray, ij_threads: int) -> float:
    """DECON/AdjustInput.java:41-100 including the double-count quirk.

    Per-portion RealSum over ``2*T`` flat portions, then ``sums[0]`` is added
    once more (``:93-97``).  ``sums[id]`` is indexed by task start order
    (``:62``); the first-started task is pinned to portion 0."""
    flat = np.asarray(img, dtype=np.float32).ravel().astype(np.float64)
    portions = divide_into_portions(flat.size, 2 * ij_threads)
    sums = [math.fsum(flat[s:s + n]) for s, n in portions]
    return math.fsum([sums[0]] + sums)


def norm_img(img: np.ndarray, ij_threads: int) -> np.ndarray:
    """DECON/AdjustInput.java:29-35: t = (float)((double)t / sum)."""
    s = sum_img(img, ij_threads)
    return (np.asarray(img, np.float32).astype(np.float64) / s).astype(np.float32)


def mirror_axis(img: np.ndarray, axis: int) -> np.ndarray:
    """DECON/Mirror.java:31-108 (single-threaded visiting order).

    Every pixel with ``pos <= size/2`` is swapped with ``size-1-pos``.  For odd
    sizes this is an exact reversal.  For even sizes the middle pair is swapped
    twice and therefore stays in place (a latent race in the reference with
    several threads; restated here with the sequential order)."""
    out = np.flip(img, axis=axis).copy()
    s = img.shape[axis]
    if s % 2 == 0 and s >= 2:
        m = s // 2
        idx = [slice(None)] * img.ndim
        for p in (m - 1, m):
            idx[axis] = p
            out[tuple(idx)] = img[tuple(idx)]
    return out


def inverted_kernel(k: np.ndarray) -> np.ndarray:
    """DECON/MVDeconFFT.java:315-323: mirror every dimension (ImgLib2 dim 0 = x)."""
    out = np.asarray(k, np.float32)
    for ax in (2, 1, 0):  # d = 0 (x), 1 (y), 2 (z)
        out = mirror_axis(out, ax)
    return out


def exponential_kernel(k: np.ndarray, num_views: int) -> np.ndarray:
    """DECON/MVDeconFFT.java:305-313,325-333: float power by repeated multiply."""
    k = np.asarray(k, np.float32)
    r = k.copy()
    for _ in range(1, num_views):
        r = (r * k).astype(np.float32)
    return r


# --------------------------------------------------------------------------
# convolutions
# --------------------------------------------------------------------------

def _check_odd(k):
    if any(s % 2 == 0 for s in k.shape):
        raise ValueError(f"kernel dims must be odd, got {k.shape}")


def conv_same_zero(a: np.ndarray, k: np.ndarray) -> np.ndarray:
    """FFTConvolution(extendZero(a), a, extendZero(k), k, out) as used for the
    compound kernels (DECON/MVDeconFFT.java:201-227,264-274); semantics per
    FFTM/FFTConvolution.java:470-551: true convolution, kernel centre at
    ``dim/2``, output interval = input interval."""
    _check_odd(k)
    r = scipy.signal.fftconvolve(np.asarray(a, np.float64), np.asarray(k, np.float64), mode="same")
    return r.astype(np.float32)


def extend(a: np.ndarray, half, ext: str) -> np.ndarray:
    """ImgLib2 out-of-bounds views used on the path:
    ``'mirror'`` = Views.extendMirrorSingle (edge not repeated; numpy 'reflect'),
    ``'one'`` = Views.extendValue(1) (DECON/MVDeconFFTThreads.java:23,42,57,82),
    ``'zero'`` = Views.extendZero."""
    pads = [(h, h) for h in half]
    if ext == "mirror":
        return np.pad(a, pads, mode="reflect")
    if ext == "one":
        return np.pad(a, pads, mode="constant", constant_values=1.0)
    if ext == "zero":
        return np.pad(a, pads, mode="constant", constant_values=0.0)
    raise ValueError(ext)


def convolve(a: np.ndarray, k: np.ndarray, ext: str, precision: str = "f64", workers=None) -> np.ndarray:
    """convolve1 (ext='mirror') / convolve2 (ext='one') of
    DECON/MVDeconFFT.java:363-447,454-535.

    out[x] = sum_j E(a)[x + c - j] * K[j], c = K//2 per axis, i.e. the interior
    of FFTM/FFTConvolution.java:470-551 (padded interval centred, kernel centre
    moved to the origin, R2C * K -> C2R unpad).  Any FFT size >= n+K-1 gives the
    same linear convolution, and blocks are 'precise', so this is also the
    result of the blocked CPU/GPU paths (CUDA/BlockGeneratorFixedSizePrecise.java:25-101).
    ``precision='f32'`` runs the FFTs in single precision (CPU-baseline timing)."""
    _check_odd(k)
    half = [s // 2 for s in k.shape]
    ap = extend(np.asarray(a, np.float32), half, ext)
    if precision == "f64":
        r = scipy.signal.fftconvolve(ap.astype(np.float64), np.asarray(k, np.float64), mode="valid")
        return r.astype(np.float32)
    # single-precision FFT path (pocketfft float32), multithreaded
    shape = [ap.shape[d] + k.shape[d] - 1 for d in range(3)]
    fshape = [scipy.fft.next_fast_len(s, real=True) for s in shape]
    with scipy.fft.set_workers(workers or 1):
        fa = scipy.fft.rfftn(ap, fshape)
        fk = scipy.fft.rfftn(np.asarray(k, np.float32), fshape)
        fa *= fk
        r = scipy.fft.irfftn(fa, fshape)
    sl = tuple(slice(k.shape[d] - 1, ap.shape[d]) for d in range(3))
    return np.ascontiguousarray(r[sl], dtype=np.float32)


def circular_convolve_block(block: np.ndarray, kernel: np.ndarray) -> np.ndarray:
    """Semantics of the legacy native export ``convolution3DfftCUDAInPlace``
    (CUDA/CUDAFourierConvolution.java:10; caller DECON/MVDeconFFTThreads.java:52-94):
    the block is circularly convolved with the kernel whose centre ``kdim/2``
    is moved to the origin (zero-padded to the block size).  The block already
    carries the K-1 halo, so only its interior is pasted back."""
    _check_odd(kernel)
    b = np.asarray(block, np.float64)
    kp = np.zeros(b.shape, np.float64)
    kz, ky, kx = kernel.shape
    zz = (np.arange(kz) - kz // 2) % b.shape[0]
    yy = (np.arange(ky) - ky // 2) % b.shape[1]
    xx = (np.arange(kx) - kx // 2) % b.shape[2]
    np.add.at(kp, np.ix_(zz, yy, xx), np.asarray(kernel, np.float64))
    r = np.fft.irfftn(np.fft.rfftn(b) * np.fft.rfftn(kp), b.shape, axes=(0, 1, 2))
    return r.astype(np.float32)


# --------------------------------------------------------------------------
# kernel preparation (MVDeconFFT.init, in MVDeconInput list order)
# --------------------------------------------------------------------------

def prepare_kernels(kernels, psftype: PSFTYPE, ij_threads: int):
    """DECON/MVDeconInput.java:41-47 -> DECON/MVDeconFFT.java:162-303.

    Views are initialised in list order and each ``init`` first normalises its
    own kernel1 in place (``:165``), so view v's compound kernel sees the
    *normalised* kernel1 of views w < v and the *raw* kernel1 of views w > v
    (restated literally).  Returns (K1 list, K2 list)."""
    psftype = PSFTYPE(psftype)
    k1 = [np.asarray(k, np.float32).copy() for k in kernels]
    for k in k1:
        _check_odd(k)
    V = len(k1)
    k2 = [None] * V
    for v in range(V):
        k1[v] = norm_img(k1[v], ij_threads)
        if V == 1 or psftype == PSFTYPE.INDEPENDENT:           # :176-180
            k2[v] = inverted_kernel(k1[v])
        elif psftype == PSFTYPE.EFFICIENT_BAYESIAN:            # :181-244
            tmp = inverted_kernel(k1[v])
            for w in range(V):
                if w == v:
                    continue
                out = conv_same_zero(inverted_kernel(k1[v]), k1[w])
                out = conv_same_zero(out, inverted_kernel(k1[w]))
                tmp = (out * tmp).astype(np.float32)
            k2[v] = norm_img(tmp, ij_threads)
        elif psftype == PSFTYPE.OPTIMIZATION_I:                # :245-291
            tmp = k1[v].copy()
            for w in range(V):
                if w == v:
                    continue
                out = conv_same_zero(k1[v], inverted_kernel(k1[w]))
                tmp = (out * tmp).astype(np.float32)
            tmp = norm_img(tmp, ij_threads)
            k2[v] = inverted_kernel(tmp)
        else:                                                  # OPTIMIZATION_II :292-302
            e = exponential_kernel(k1[v], V)
            e = norm_img(e, ij_threads)
            k2[v] = inverted_kernel(e)
    return k1, k2


# --------------------------------------------------------------------------
# pointwise passes
# --------------------------------------------------------------------------

def tikhonov(value, lam):
    """DECON/MVDeconvolution.java:705 (float64)."""
    value = np.asarray(value, np.float64)
    return (np.sqrt(1.0 + 2.0 * lam * value) - 1.0) / lam


def compute_quotient(blurred: np.ndarray, img: np.ndarray) -> np.ndarray:
    """DECON/MVDeconvolution.java:473-525: img > 0 ? img / blurred : 1 (float)."""
    blurred = np.asarray(blurred, np.float32)
    img = np.asarray(img, np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(img > 0, img / blurred, np.float32(1.0))
    return q.astype(np.float32)


def compute_next_value(psi, integral, weight, lam):
    """DECON/MVDeconvolution.java:671-703 vectorised, float32 op order kept."""
    psi = np.asarray(psi, np.float32)
    integral = np.asarray(integral, np.float32)
    weight = np.asarray(weight, np.float32)
    with np.errstate(all="ignore"):
        value = (psi * integral).astype(np.float32)
        if lam > 0:
            adj = tikhonov(value, lam).astype(np.float32)
        else:
            adj = value
        adj = np.where(value > 0, adj, MIN_VALUE).astype(np.float32)
        nxt = np.where(np.isnan(adj), MIN_VALUE, np.maximum(MIN_VALUE, adj)).astype(np.float32)
        diff = (nxt - psi).astype(np.float32)
        out = (psi + (diff * weight).astype(np.float32)).astype(np.float32)
    return out


def compute_final_values(psi, integral, weight, lam):
    """DECON/MVDeconvolution.java:582-659: returns (new psi, sumChange, maxChange)."""
    new = compute_next_value(psi, integral, weight, lam)
    with np.errstate(invalid="ignore"):
        change = np.abs((new - psi).astype(np.float32)).astype(np.float64)
    sum_change = float(change.sum())
    max_change = float(max(-1.0, change.max())) if change.size else -1.0
    return new, sum_change, max_change


def first_iteration(imgs):
    """DECON/FirstIteration.java:101-133 + DECON/MVDeconvolution.java:192-235.

    Returns (count image as float32, avg) where avg = sum_x mean(x) / #{count>0}
    with mean(x) = sum_{v: img_v>0} img_v / count (double)."""
    stack = np.stack([np.asarray(i, np.float32) for i in imgs]).astype(np.float64)
    pos = stack > 0
    count = pos.sum(axis=0)
    ssum = np.where(pos, stack, 0.0).sum(axis=0)
    with np.errstate(invalid="ignore", divide="ignore"):
        mean = np.where(count > 0, ssum / np.maximum(count, 1), 0.0)
    n = int((count > 0).sum())
    avg = math.fsum(mean[count > 0].ravel()) / n if n > 0 else float("nan")
    return count.astype(np.float32), avg


# --------------------------------------------------------------------------
# driver
# --------------------------------------------------------------------------

@dataclass
class DeconResult:
    psi: np.ndarray
    stats: list = field(default_factory=list)   # [iteration][view] = (sumChange, maxChange)
    avg: float = float("nan")


def run_iteration(psi, imgs, weights, k1s, k2s, lam, precision="f64", workers=None):
    """DECON/MVDeconvolution.java:333-444: sequential per-view update of psi."""
    stats = []
    for v in range(len(imgs)):
        tmp1 = convolve(psi, k1s[v], "mirror", precision, workers)       # convolve1
        tmp1 = compute_quotient(tmp1, imgs[v])                            # computeQuotient
        tmp2 = convolve(tmp1, k2s[v], "one", precision, workers)         # convolve2
        psi, s, m = compute_final_values(psi, tmp2, weights[v], lam)     # computeFinalValues
        stats.append((s, m))
    return psi, stats


def init_psi_from_image(initial: np.ndarray, check_numbers: bool = True) -> np.ndarray:
    """DECON/MVDeconvolution.java:237-320 (checkNumbers: v <= 0 -> minValue)."""
    psi = np.asarray(initial, np.float32).copy()
    if check_numbers:
        psi[psi <= 0] = MIN_VALUE
    return psi


def mv_deconvolution(imgs, weights, kernels, psftype, num_iterations, lam,
                     ij_threads=8, initial_psi=None, prepared=None,
                     precision="f64", workers=None) -> DeconResult:
    """DECON/MVDeconvolution.java:73-190.

    ``prepared`` = (K1s, K2s) skips the kernel preparation (already-initialised
    views)."""
    imgs = [np.asarray(i, np.float32) for i in imgs]
    weights = [np.asarray(w, np.float32) for w in weights]
    if prepared is None:
        k1s, k2s = prepare_kernels(kernels, psftype, ij_threads)      # views.init :93
    else:
        k1s, k2s = prepared
    count, avg = first_iteration(imgs)
    if initial_psi is not None:
        psi = init_psi_from_image(initial_psi)
    else:
        if math.isnan(avg):                                           # :117-121
            avg = 0.5
        psi = np.full(imgs[0].shape, np.float32(avg), np.float32)    # :125-126
    res = DeconResult(psi=psi, avg=avg)
    for _ in range(num_iterations):
        psi, st = run_iteration(psi, imgs, weights, k1s, k2s, lam, precision, workers)
        res.stats.append(st)
    psi = np.where(count == 0, np.float32(0.0), psi).astype(np.float32)  # :180-187
    res.psi = psi
    return res


# --------------------------------------------------------------------------
# block tiling (legacy JNA path)
# --------------------------------------------------------------------------

@dataclass
class Block:
    """CUDA/Block.java:67-100 (all vectors in ImgLib2 order: x, y, z)."""
    block_size: tuple
    offset: tuple
    effective_size: tuple
    effective_offset: tuple
    effective_local_offset: tuple


def divide_into_blocks(img_size, kernel_size, block_size):
    """CUDA/BlockGeneratorFixedSizePrecise.java:25-101 (vectors x,y,z; blocks
    enumerated x-fastest by LocalizingZeroMinIntervalIterator)."""
    n = len(img_size)
    eff = [block_size[d] - kernel_size[d] + 1 for d in range(n)]
    if any(e <= 0 for e in eff):
        return None
    loc = [kernel_size[d] // 2 for d in range(n)]
    nb = [img_size[d] // eff[d] + (1 if img_size[d] % eff[d] else 0) for d in range(n)]
    blocks = []
    for idx in np.ndindex(*reversed(nb)):
        cur = list(reversed(idx))
        eo = [cur[d] * eff[d] for d in range(n)]
        off = [eo[d] - kernel_size[d] // 2 for d in range(n)]
        es = [min(eff[d], img_size[d] - eo[d]) for d in range(n)]
        blocks.append(Block(tuple(block_size), tuple(off), tuple(es), tuple(eo), tuple(loc)))
    return blocks


def copy_block(src: np.ndarray, blk: Block, ext: str) -> np.ndarray:
    """CUDA/Block.java:114-153,233-271: block[i] = E(src)[offset + i]."""
    bx, by, bz = blk.block_size
    ox, oy, oz = blk.offset
    nz, ny, nx = src.shape
    zi = _ext_index(np.arange(oz, oz + bz), nz, ext)
    yi = _ext_index(np.arange(oy, oy + by), ny, ext)
    xi = _ext_index(np.arange(ox, ox + bx), nx, ext)
    out = src[np.ix_(np.clip(zi, 0, nz - 1), np.clip(yi, 0, ny - 1), np.clip(xi, 0, nx - 1))].astype(np.float32)
    if ext != "mirror":
        inside = (zi >= 0)[:, None, None] & (yi >= 0)[None, :, None] & (xi >= 0)[None, None, :]
        out = np.where(inside, out, np.float32(1.0 if ext == "one" else 0.0)).astype(np.float32)
    return out


def _ext_index(i, n, ext):
    i = np.asarray(i)
    if ext == "mirror":
        if n == 1:
            return np.zeros_like(i)
        p = 2 * (n - 1)
        j = np.mod(i, p)
        return np.where(j >= n, p - j, j)
    return np.where((i >= 0) & (i < n), i, -1)


def paste_block(target: np.ndarray, block: np.ndarray, blk: Block) -> None:
    """CUDA/Block.java:155-195,313-359: only the effective region is written."""
    ex, ey, ez = blk.effective_size
    eox, eoy, eoz = blk.effective_offset
    lx, ly, lz = blk.effective_local_offset
    target[eoz:eoz + ez, eoy:eoy + ey, eox:eox + ex] = block[lz:lz + ez, ly:ly + ey, lx:lx + ex]


def blocked_convolve(img: np.ndarray, kernel: np.ndarray, block_size, ext: str) -> np.ndarray:
    """DECON/MVDeconFFT.java:415-423 + MVDeconFFTThreads.convolve{1,2}BlockCUDA:
    copy (extended) -> in-place circular FFT conv -> paste."""
    nz, ny, nx = img.shape
    kz, ky, kx = kernel.shape
    blocks = divide_into_blocks((nx, ny, nz), (kx, ky, kz), block_size)
    out = np.zeros_like(img, dtype=np.float32)
    for b in blocks:
        blk = copy_block(img, b, ext)
        blk = circular_convolve_block(blk, kernel)
        paste_block(out, blk, b)
    return out
