"""Oracle: CPU restatement of the Difference-of-Gaussian bead-detection pass.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  PARITY UNPINNED: the
imglib1 Gaussian (``Util.createGaussianKernel1DDouble``,
``GaussianConvolutionReal``, ``ImageCalculatorInPlace``) and the external
SeparableConvolutionCUDALib are not in the container; their published
algorithms are restated below.  Paths relative to
``/root/reference/src/main/java/``; IPD = spim/process/interestpointdetection/.

The sub-pixel quadratic fit (imglib1 ``SubpixelLocalization``, external) is
restated after the reference's own fit in LaPlaceFunctions.java (same author,
same finite differences); its tolerance rule is an assumption (see
``quadratic_localization``).

The restated variant is the GPU "accurate" path: blocks copied with
``extendMirrorSingle`` (IPD/DifferenceOfGaussianCUDA.java:153-154,170), float
kernels zero-padded to the supported size
(spim/process/cuda/CUDASeparableConvolutionFunctions.java:199-245), separable
passes x -> y -> z in float32.
"""
from __future__ import annotations

import math

import numpy as np

SUPPORTED_KERNEL_SIZES = (7, 15, 31, 63, 127)  # CUDASeparableConvolutionFunctions.java:14


def f32(x):
    return np.float32(x)


def compute_k(steps_per_octave: int) -> np.float32:
    """mpicbg/spim/registration/bead/laplace/LaPlaceFunctions.java:572-575:
    (float)Math.pow(2f, 1f/steps)."""
    return f32(math.pow(2.0, float(f32(1.0) / f32(steps_per_octave))))


def compute_k_weight(k: np.float32) -> np.float32:
    """LaPlaceFunctions.java:577-580: 1.0f / (k - 1.0f)."""
    return f32(f32(1.0) / f32(f32(k) - f32(1.0)))


def compute_sigma(steps: int, k: np.float32, initial_sigma: float):
    """LaPlaceFunctions.java:542-556 (float products)."""
    s = [f32(initial_sigma)]
    for _ in range(steps):
        s.append(f32(s[-1] * f32(k)))
    return s


def get_diff_sigma(sigma_a, sigma_b) -> np.float32:
    """LaPlaceFunctions.java:558-561: (float)Math.sqrt(b*b - a*a) (float ops, double sqrt)."""
    a = f32(sigma_a)
    b = f32(sigma_b)
    d = f32(f32(b * b) - f32(a * a))
    return f32(math.sqrt(float(d)))


def compute_sigma_diff(sigma, image_sigma):
    """LaPlaceFunctions.java:563-570."""
    return [get_diff_sigma(image_sigma, s) for s in sigma]


def dog_sigmas(sigma: float, image_sigma=(0.5, 0.5, 0.5)):
    """IPD/ProcessDOG.java:88-105 with the caller's min(imageSigma, sigma)
    (spim/fiji/plugin/interestpointdetection/DifferenceOfGaussian.java:121-123).
    Returns (sigma1[3], sigma2[3], k, K_MIN1_INV) for axes x, y, z."""
    k = compute_k(4)
    kinv = compute_k_weight(k)
    steps = compute_sigma(3, k, sigma)
    s1, s2 = [], []
    for d in range(3):
        isg = min(float(f32(image_sigma[d])), float(f32(sigma)))
        diff = compute_sigma_diff(steps, isg)
        s1.append(float(diff[0]))
        s2.append(float(diff[1]))
    return s1, s2, k, kinv


def gaussian_kernel_1d(sigma: float, normalize: bool = True) -> np.ndarray:
    """imglib1 ``mpicbg.imglib.util.Util.createGaussianKernel1DDouble`` (external;
    published algorithm): size = max(3, 2*(int)(3*sigma + 0.5) + 1),
    g[c +- x] = exp(-(x*x) / (2*sigma*sigma)), normalised to sum 1 (double)."""
    if sigma <= 0:
        g = np.zeros(3)
        g[1] = 1.0
    else:
        size = max(3, 2 * int(3 * sigma + 0.5) + 1)
        two_sq = 2 * sigma * sigma
        g = np.zeros(size)
        c = size // 2
        for x in range(c, -1, -1):
            val = math.exp(-(x * x) / two_sq)
            g[c - x] = val
            g[c + x] = val
    if normalize:
        s = 0.0
        for v in g:
            s += v
        g = g / s
    return g


def padded_float_kernel(kernel: np.ndarray, size: int) -> np.ndarray:
    """CUDASeparableConvolutionFunctions.getFloatKernelPadded (:235-245)."""
    k = np.zeros(size, np.float32)
    s = (size - len(kernel)) // 2
    k[s:s + len(kernel)] = np.asarray(kernel, np.float64).astype(np.float32)
    return k


def cuda_kernels(sigmas):
    """CUDASeparableConvolutionFunctions.getCUDAKernels (:199-233): pick the
    smallest supported size >= the longest kernel, pad every kernel to it."""
    ks = [gaussian_kernel_1d(s, True) for s in sigmas]
    longest = max(len(k) for k in ks)
    size = min([s for s in SUPPORTED_KERNEL_SIZES if longest <= s], default=None)
    if size is None:
        return None
    return [padded_float_kernel(k, size) for k in ks]


def _mirror_index(i, n):
    if n == 1:
        return np.zeros_like(i)
    p = 2 * (n - 1)
    j = np.mod(i, p)
    return np.where(j >= n, p - j, j)


def convolve_axis(img: np.ndarray, kernel: np.ndarray, axis: int, mode: str = "mirror",
                  value: float = 0.0) -> np.ndarray:
    """One separable pass, out[i] = sum_j in[i + j - r] * k[j] (centred odd kernel,
    correlation form -- Gaussian kernels are symmetric), accumulated in float32
    in tap order.  ``mode``: 'mirror' (extendMirrorSingle), 'zero', 'value',
    'border' (extend last pixel) = the native OOB modes 0/1/2 plus mirror."""
    img = np.asarray(img, np.float32)
    kernel = np.asarray(kernel, np.float32)
    r = len(kernel) // 2
    n = img.shape[axis]
    acc = np.zeros_like(img, dtype=np.float32)
    base = np.arange(n)
    for j in range(len(kernel)):
        if kernel[j] == 0:
            # zero taps add exactly 0 (skip keeps float32 order identical)
            continue
        idx = base + j - r
        if mode == "mirror":
            src = np.take(img, _mirror_index(idx, n), axis=axis)
        elif mode == "border":
            src = np.take(img, np.clip(idx, 0, n - 1), axis=axis)
        else:
            fill = 0.0 if mode == "zero" else value
            src = np.take(img, np.clip(idx, 0, n - 1), axis=axis)
            shape = [1] * img.ndim
            shape[axis] = n
            inside = ((idx >= 0) & (idx < n)).reshape(shape)
            src = np.where(inside, src, np.float32(fill))
        acc = (acc + (src * kernel[j]).astype(np.float32)).astype(np.float32)
    return acc


def gauss3d(img: np.ndarray, kernels_xyz, mode="mirror", value=0.0) -> np.ndarray:
    """Separable 3D convolution, passes x -> y -> z (array axes 2, 1, 0)."""
    out = convolve_axis(img, kernels_xyz[0], 2, mode, value)
    out = convolve_axis(out, kernels_xyz[1], 1, mode, value)
    out = convolve_axis(out, kernels_xyz[2], 0, mode, value)
    return out


def normalize_image(img: np.ndarray, mn: float, mx: float) -> np.ndarray:
    """spim/process/fusion/FusionHelper.java:176-234: (t - min) / (max - min) in float.
    A NaN / infinite / zero range leaves the image unchanged (``:180-186`` returns
    false and ProcessDOG.java:84 ignores it)."""
    mn = f32(mn)
    diff = f32(f32(mx) - mn)
    if math.isnan(diff) or math.isinf(diff) or diff == 0:
        return np.asarray(img, np.float32).copy()
    return ((np.asarray(img, np.float32) - mn) / diff).astype(np.float32)


def dog_image(img_norm: np.ndarray, sigma: float, image_sigma=(0.5, 0.5, 0.5)) -> np.ndarray:
    """IPD/DifferenceOfGaussianNewPeakFinder.java:54-136: gauss(s2) - gauss(s1),
    times K_MIN1_INV (imglib1 normalized subtraction, float)."""
    s1, s2, k, kinv = dog_sigmas(sigma, image_sigma)
    g1 = gauss3d(img_norm, cuda_kernels(s1))
    g2 = gauss3d(img_norm, cuda_kernels(s2))
    return ((g2 - g1).astype(np.float32) * kinv).astype(np.float32)


def find_peaks(dog: np.ndarray, min_value: float, ij_threads: int = 8):
    """mpicbg/spim/segmentation/InteractiveIntegral.java:360-468.

    Skips the 1-voxel border; |v| >= min_value; 26-neighbour test with
    inclusive comparisons; "all neighbours >= centre" => MAX (bright bead),
    "all <= centre" => MIN.  Returned order = the reference's: per-thread
    lists by ``x % T`` concatenated, each in flat (x-fastest) order.
    Returns list of (x, y, z, intensity=|v|, is_min, is_max)."""
    d = np.asarray(dog, np.float32)
    nz, ny, nx = d.shape
    if nz < 3 or ny < 3 or nx < 3:
        return []
    c = d[1:-1, 1:-1, 1:-1]
    ge = np.ones_like(c, dtype=bool)
    le = np.ones_like(c, dtype=bool)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if dz == dy == dx == 0:
                    continue
                nb = d[1 + dz:nz - 1 + dz, 1 + dy:ny - 1 + dy, 1 + dx:nx - 1 + dx]
                ge &= nb >= c
                le &= nb <= c
    cand = np.abs(c) >= np.float32(min_value)
    is_max = cand & ge
    is_min = cand & le & ~ge
    zz, yy, xx = np.nonzero(is_max | is_min)
    peaks = []
    for z, y, x in zip(zz, yy, xx):
        v = c[z, y, x]
        peaks.append((int(x + 1), int(y + 1), int(z + 1), float(abs(v)),
                      bool(is_min[z, y, x]), bool(is_max[z, y, x])))
    T = ij_threads
    flat = [p[2] * ny * nx + p[1] * nx + p[0] for p in peaks]
    order = sorted(range(len(peaks)), key=lambda i: (peaks[i][0] % T, flat[i]))
    return [peaks[i] for i in order]


MAX_NUM_MOVES = 10        # IPD/Localization.java:57 (spl.setMaxNumMoves(10))
MAXIMA_TOLERANCE = 0.01   # imglib1 SubpixelLocalization default, allowMaximaTolerance = true (:56)


def _hessian_and_gradient(d: np.ndarray, x: int, y: int, z: int):
    """Finite differences of the quadratic fit, in the reference's arithmetic
    (mpicbg/spim/registration/bead/laplace/LaPlaceFunctions.java:288-466):
    diagonal = float(v(+1) - 2 v(0)) + v(-1) in double; cross terms
    ((a - b) / 2 - (c - d) / 2) / 2 in float; gradient (v(+1) - v(-1)) / 2 in double."""
    v = lambda dx, dy, dz: d[z + dz, y + dy, x + dx]   # float32 scalars
    two = np.float32(2)
    temp = two * v(0, 0, 0)
    H = np.zeros(9)
    H[0] = float(v(1, 0, 0) - temp) + float(v(-1, 0, 0))
    H[4] = float(v(0, 1, 0) - temp) + float(v(0, -1, 0))
    H[8] = float(v(0, 0, 1) - temp) + float(v(0, 0, -1))

    def cross(a, b, c, e):
        return float(((a - b) / two - (c - e) / two) / two)
    H[5] = H[7] = cross(v(0, 1, 1), v(0, -1, 1), v(0, 1, -1), v(0, -1, -1))
    H[2] = H[6] = cross(v(1, 0, 1), v(-1, 0, 1), v(1, 0, -1), v(-1, 0, -1))
    H[1] = H[3] = cross(v(1, 1, 0), v(-1, 1, 0), v(1, -1, 0), v(-1, -1, 0))
    g = np.array([(float(v(1, 0, 0)) - float(v(-1, 0, 0))) / 2.0,
                  (float(v(0, 1, 0)) - float(v(0, -1, 0))) / 2.0,
                  (float(v(0, 0, 1)) - float(v(0, 0, -1))) / 2.0])
    return H, g


def _invert3(a):
    """LaPlaceFunctions.java:243-286 (det, adjugate / det); None when det == 0."""
    det = (a[0] * a[4] * a[8] + a[3] * a[7] * a[2] + a[6] * a[1] * a[5]
           - a[2] * a[4] * a[6] - a[5] * a[7] * a[0] - a[8] * a[1] * a[3])
    if det == 0:
        return None
    return np.array([(a[4] * a[8] - a[5] * a[7]) / det, (a[2] * a[7] - a[1] * a[8]) / det,
                     (a[1] * a[5] - a[2] * a[4]) / det, (a[5] * a[6] - a[3] * a[8]) / det,
                     (a[0] * a[8] - a[2] * a[6]) / det, (a[2] * a[3] - a[0] * a[5]) / det,
                     (a[3] * a[7] - a[4] * a[6]) / det, (a[1] * a[6] - a[0] * a[7]) / det,
                     (a[0] * a[4] - a[1] * a[3]) / det])


def quadratic_localization(dog: np.ndarray, peaks, max_moves: int = MAX_NUM_MOVES,
                           tolerance: float = MAXIMA_TOLERANCE):
    """Sub-pixel quadratic fit of each peak (IPD/Localization.java:47-88 via
    imglib1 ``SubpixelLocalization``; the iteration restated after the
    reference's own fit, LaPlaceFunctions.java:30-170).

    Per peak: Hessian H and gradient g at the current voxel, offset
    X = -H^-1 g; every axis with |X_d| > 0.5 + moves * tolerance moves one voxel
    towards sign(X_d); repeat up to ``max_moves`` moves.  A move onto the image
    border, a singular H or no stable solution leave the peak as detected
    (integer position, value = |v|).  Otherwise position = voxel + (float) X,
    value = (float) v(voxel) + (float) (X . g / 2).
    Returns [(x, y, z, value)] as float32 (value is signed)."""
    d = np.asarray(dog, np.float32)
    nz, ny, nx = d.shape
    dims = (nx, ny, nz)
    out = []
    for pk in peaks:
        x0, y0, z0, inten = pk[0], pk[1], pk[2], pk[3]
        p = [int(x0), int(y0), int(z0)]
        res = (np.float32(x0), np.float32(y0), np.float32(z0), np.float32(inten))
        moves = 0
        stable = False
        valid = True
        X = g = None
        while True:
            moves += 1
            H, g = _hessian_and_gradient(d, *p)
            A = _invert3(H)
            if A is None:
                valid = False
                break
            X = -np.array([A[0] * g[0] + A[1] * g[1] + A[2] * g[2],
                           A[3] * g[0] + A[4] * g[1] + A[5] * g[2],
                           A[6] * g[0] + A[7] * g[1] + A[8] * g[2]])
            stable = True
            thr = 0.5 + moves * tolerance
            for a in range(3):
                if abs(X[a]) > thr:
                    p[a] += 1 if X[a] > 0 else -1
                    stable = False
            if not stable and any(p[a] <= 0 or p[a] >= dims[a] - 1 for a in range(3)):
                valid = False
                break
            if stable or moves > max_moves:
                break
        if valid and stable:
            fit = (X[0] * g[0] + X[1] * g[1] + X[2] * g[2]) / 2.0
            val = np.float32(d[p[2], p[1], p[0]]) + np.float32(fit)
            res = (np.float32(p[0]) + np.float32(X[0]), np.float32(p[1]) + np.float32(X[1]),
                   np.float32(p[2]) + np.float32(X[2]), np.float32(val))
        out.append(res)
    return out


def process_dog(img: np.ndarray, sigma: float = 1.8, threshold: float = 0.008,
                localization: int = 0, image_sigma=(0.5, 0.5, 0.5),
                find_min: bool = False, find_max: bool = True,
                min_intensity=float("nan"), max_intensity=float("nan"),
                ij_threads: int = 8):
    """IPD/ProcessDOG.java:40-178 with localization 0 (IPD/Localization.java:19-45)
    or 1 (quadratic fit, :47-88).  Returns (points [(x, y, z, intensity)], dog
    image); localization 1 keeps the points with |fitted value| > threshold and
    reports the fitted value."""
    min_peak = f32(threshold) if localization == 0 else f32(f32(threshold) / f32(10.0))
    if (math.isnan(min_intensity) or math.isnan(max_intensity) or math.isinf(min_intensity)
            or math.isinf(max_intensity) or min_intensity == max_intensity):
        mn, mx = float(np.min(img)), float(np.max(img))
    else:
        mn, mx = float(f32(min_intensity)), float(f32(max_intensity))
    norm = normalize_image(img, mn, mx)
    dog = dog_image(norm, sigma, image_sigma)
    peaks = find_peaks(dog, float(min_peak), ij_threads)
    out = [(p[0], p[1], p[2], p[3]) for p in peaks if (p[5] and find_max) or (p[4] and find_min)]
    if localization == 1:
        fitted = quadratic_localization(dog, out)
        out = [(float(x), float(y), float(z), float(v)) for x, y, z, v in fitted
               if abs(v) > np.float32(threshold)]
    return out, dog
