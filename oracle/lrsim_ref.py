"""Oracle: the legacy simultaneous-update multiview Lucy-Richardson rule.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Restates
``mpicbg/spim/postprocessing/deconvolution/LucyRichardsonMultiViewDeconvolution.java``
(paths under ``/root/reference/src/main/java/``; ``LRMV`` below):

  lucyRichardsonMultiView  LRMV:24-358   kernel norm, psi init, the iteration
  normAllImages            LRMV:360-457  average intensity where >= 2 views overlap
  normImage / sumImage     LRMV:460-490  kernel / exact (BigDecimal) sum
  LucyRichardsonFFT        LucyRichardsonFFT.java:7-38 (image, weight, kernel)

This is the opt-in "compound correction" mode of SURVEY.md section 8e: every
view's correction is computed from the same psi, so the views shard across ranks
and the per-voxel combination (a sum, or a product of powers) is one all-reduce.
It is NOT ``MVDeconvolution``'s sequential rule, and the reference never runs it
(``fiji/plugin/Multi_View_Deconvolution.java:226-231`` comments the call out).

PARITY UNPINNED, twice over: no fixture exists (as for the whole oracle), and the
convolution is imglib1's ``mpicbg.imglib.algorithm.fft.FourierConvolution``
(absent from /root/reference), whose out-of-bounds extension is not restated.
Both convolutions here use ``mvdecon_ref.convolve(..., 'mirror')``
(extendMirrorSingle, the extension of the maintained path); only voxels within
the kernel's reach of a border can depend on that choice.
"""
from __future__ import annotations

import math

import numpy as np

from .mvdecon_ref import convolve

MIN_VALUE = 0.0001   # LRMV:30 (a double here, unlike MVDeconvolution's float)


def norm_image(k: np.ndarray) -> np.ndarray:
    """LRMV:460-490: t = (float)((double)t / sum), sum = the exact sum of the
    values (BigDecimal) rounded once to double (math.fsum is correctly rounded)."""
    k = np.asarray(k, np.float32)
    s = math.fsum(k.astype(np.float64).ravel().tolist())
    return (k.astype(np.float64) / s).astype(np.float32)


def norm_all_images(imgs, weights) -> float:
    """LRMV:360-457: per voxel the views with weight != 0 are summed (double) and
    counted; voxels where more than one view counts add to the sum and the count.
    Returns sum / count, or 1 when no voxel qualifies.  ``weights`` are required:
    the reference indexes ``cursorsWeight.get(i)`` (:401), which throws when the
    views carry none."""
    if any(w is None for w in weights):
        raise ValueError("normAllImages needs a weight image for every view (LRMV:401)")
    s = np.zeros(np.shape(imgs[0]), np.float64)
    c = np.zeros(np.shape(imgs[0]), np.int64)
    for img, w in zip(imgs, weights):
        m = np.asarray(w, np.float32) != 0
        s = s + np.where(m, np.asarray(img, np.float32).astype(np.float64), 0.0)
        c = c + m
    sel = c > 1
    count = int(c[sel].sum())
    if count == 0:
        return 1.0
    return math.fsum(s[sel].ravel().tolist()) / count


def combine(psi, contribs, weights, multiplicative: bool):
    """LRMV:201-270: value starts at nextPsi (= 1) or 0; per view with weight > 0:
    value *= pow(c, w) (multiplicative) or value += c * w (float product, double
    sum); num += w.  num > 0: psi * pow(value, 1/num), resp. psi * 1 * value / num
    (double, left to right); else minValue.  Returned rounded to float."""
    value = np.full(psi.shape, 1.0 if multiplicative else 0.0, np.float64)
    num = np.zeros(psi.shape, np.float64)
    for c, w in zip(contribs, weights):
        c = np.asarray(c, np.float32)
        w = np.asarray(w, np.float32)
        m = w > 0
        if multiplicative:
            with np.errstate(all="ignore"):
                value = np.where(m, value * np.power(c.astype(np.float64), w.astype(np.float64)), value)
        else:
            value = np.where(m, value + (c * w).astype(np.float32).astype(np.float64), value)
        num = num + np.where(m, w.astype(np.float64), 0.0)
    p = np.asarray(psi, np.float32).astype(np.float64)
    with np.errstate(all="ignore"):
        if multiplicative:
            out = p * np.power(value, 1.0 / np.where(num > 0, num, 1.0))
        else:
            out = p * 1.0 * value / np.where(num > 0, num, 1.0)
    out = np.where(num > 0, out, MIN_VALUE)
    return out.astype(np.float32)


def tikhonov(f: np.ndarray, lam: float) -> np.ndarray:
    """LRMV:290-301: (float)((sqrt(1 + 2 lambda f) - 1) / lambda), double."""
    with np.errstate(all="ignore"):
        return ((np.sqrt(1.0 + 2.0 * lam * np.asarray(f, np.float32).astype(np.float64)) - 1.0) / lam
                ).astype(np.float32)


def finish(psi, nxt):
    """LRMV:306-330: NaN -> (float)minValue, else (float)max(minValue, v); returns
    (new psi, sum |change| (double), max |change|)."""
    nxt = np.asarray(nxt, np.float32)
    new = np.where(np.isnan(nxt), np.float32(MIN_VALUE),
                   np.maximum(MIN_VALUE, nxt.astype(np.float64)).astype(np.float32)).astype(np.float32)
    ch = np.abs((np.asarray(psi, np.float32) - new).astype(np.float32))
    return new, math.fsum(ch.astype(np.float64).ravel().tolist()), float(ch.max()) if ch.size else -1.0


def view_contribution(psi, img, kernel):
    """LRMV:127-173: blurred = conv(psi, K); q = img / blurred (float); the view's
    contribution = conv(q, K) -- the same kernel both times (FourierConvolution)."""
    blurred = convolve(psi, kernel, "mirror")
    with np.errstate(all="ignore"):
        q = (np.asarray(img, np.float32) / blurred).astype(np.float32)
    return convolve(q, kernel, "mirror")


def lucy_richardson_multi_view(imgs, weights, kernels, max_iterations: int, multiplicative: bool,
                               lam: float, views_of=None):
    """LRMV:24-358.  Returns (psi, avg, stats) with stats = [(sumChange, maxChange)]
    per iteration.  ``views_of`` (tests): a list of view-index lists, one per rank;
    the per-rank partial combinations are then merged the way the all-reduce does
    (sum of the additive partials, product of the multiplicative ones)."""
    ks = [norm_image(k) for k in kernels]
    avg = norm_all_images(imgs, weights)
    psi = np.full(np.shape(imgs[0]), np.float32(avg), np.float32)
    stats = []
    for _ in range(max(1, max_iterations)):   # do { ... } while (i < maxIterations)
        contribs = [view_contribution(psi, imgs[v], ks[v]) for v in range(len(imgs))]
        if views_of is None:
            nxt = combine(psi, contribs, weights, multiplicative)
        else:
            nxt = combine_ranks(psi, contribs, weights, multiplicative, views_of)
        if lam > 0:
            nxt = tikhonov(nxt, lam)
        psi, s, m = finish(psi, nxt)
        stats.append((s, m))
    return psi, avg, stats


def partial_value(contribs, weights, views, multiplicative: bool):
    """One rank's share of LRMV:215-237 over its views: (value partial, num partial)
    in double, starting from the identity of the merge (1 for the product, 0 for
    the sum)."""
    shape = np.shape(contribs[0])
    value = np.full(shape, 1.0 if multiplicative else 0.0, np.float64)
    num = np.zeros(shape, np.float64)
    for v in views:
        c = np.asarray(contribs[v], np.float32)
        w = np.asarray(weights[v], np.float32)
        m = w > 0
        if multiplicative:
            with np.errstate(all="ignore"):
                value = np.where(m, value * np.power(c.astype(np.float64), w.astype(np.float64)), value)
        else:
            value = np.where(m, value + (c * w).astype(np.float32).astype(np.float64), value)
        num = num + np.where(m, w.astype(np.float64), 0.0)
    return value, num


def apply_value(psi, value, num, multiplicative: bool):
    """LRMV:256-269 from the merged value and num."""
    p = np.asarray(psi, np.float32).astype(np.float64)
    with np.errstate(all="ignore"):
        if multiplicative:
            out = p * np.power(value, 1.0 / np.where(num > 0, num, 1.0))
        else:
            out = p * 1.0 * value / np.where(num > 0, num, 1.0)
    return np.where(num > 0, out, MIN_VALUE).astype(np.float32)


def combine_ranks(psi, contribs, weights, multiplicative: bool, views_of):
    parts = [partial_value(contribs, weights, vs, multiplicative) for vs in views_of]
    value = parts[0][0].copy()
    num = parts[0][1].copy()
    for v, n in parts[1:]:
        value = value * v if multiplicative else value + v
        num = num + n
    return apply_value(psi, value, num, multiplicative)
