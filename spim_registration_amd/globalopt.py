"""Global optimisation of view models from point correspondences (host side).

Restates the registration's last step, ``GlobalOpt.compute``
(/root/reference/src/main/java/spim/process/interestpointregistration/GlobalOpt.java:44-135):
one tile per view (or per timepoint, ``considerTimePointsAsUnit``, :252-290), each
pairwise match's inliers added to both tiles (:292-305), the registration type's
tiles fixed (:220-250), then ``TileConfiguration.preAlign()`` and
``optimize(10, 10000, 200)`` (:66-78).  ``Tile``/``TileConfiguration`` and the
model fits live in mpicbg (a third-party dependency absent from /root/reference);
their published algorithms are restated here:

  * Tile.fitModel: the tile's model is fitted to its matches, local point ->
    the partner point as the partner tile's current model maps it; Tile.apply
    then updates this tile's transformed points.  The tiles are visited in order
    and each applies at once (Gauss-Seidel).
  * Tile.updateCost: distance = the unweighted mean over the tile's matches of
    |model(p) - partner_model(q)|; TileConfiguration.error = mean over tiles.
  * optimize(maxAllowedError, maxIterations, maxPlateauWidth): iterate; after
    maxPlateauWidth iterations stop once error <= maxAllowedError and the
    error's slope over d = w, w/2, ..., 1 iterations is <= 1e-4 everywhere.
  * preAlign: starting from the fixed tiles (or the first tile), a list iterator
    walks the aligned tiles; each unaligned tile connected to the current one is
    fitted to its matches with that tile only and visited next (ListIterator.add +
    previous); the tiles never reached are returned.
  * a NotEnoughDataPoints / IllDefinedDataPoints from preAlign or optimize is
    caught and printed, and the models are returned as they stand (GlobalOpt.java:92-100).
  * TranslationModel3D (weighted mean offset), RigidModel3D (Horn's closed-form
    unit quaternion, weighted), AffineModel3D (weighted least squares about the
    weighted centroids); 1 / 3 / 4 matches minimum.

Parity unpinned: mpicbg is not in the reference tree and the reference has no
fixtures for this stage; the tests check exact recovery of known models.

This is CPU work in the reference too (SURVEY 8f keeps registration on the host).
A tile's fit runs on per-partner moments (3x3 algebra per pair), so an iteration
costs one distance evaluation per match: 8 views with 20,000 beads each (28
pairs, 560k matches) take 7-8 s for the 202 iterations the plateau test needs
(this container, one thread).  Points are
(x, y, z) in the frame the views' current models map them to; the returned tile
models are the corrections to pre-concatenate onto those models (the fixed tiles
keep the identity).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

MIN_MATCHES = {"translation": 1, "rigid": 3, "affine": 4}


class NotEnoughDataPoints(ValueError):
    """mpicbg NotEnoughDataPointsException."""


class IllDefinedDataPoints(ValueError):
    """mpicbg IllDefinedDataPointsException (a singular affine system)."""


def _identity():
    return np.hstack([np.eye(3), np.zeros((3, 1))])


def apply(m, pts):
    return pts @ m[:, :3].T + m[:, 3]


def fit(kind: str, p, q, w):
    """The 3x4 model of ``kind`` that maps p onto q, least squares weighted by w."""
    p, q, w = np.asarray(p, np.float64), np.asarray(q, np.float64), np.asarray(w, np.float64)
    return _fit_moments(kind, len(p), *_moments(p, q, w))


def _moments(p, q, w):
    """(sum w, sum w p, sum w q, sum w p p^T, sum w p q^T): all a fit needs."""
    wp = p * w[:, None]
    return w.sum(), wp.sum(axis=0), w @ q, wp.T @ p, wp.T @ q


def _fit_moments(kind, n, ws, sp, sq, spp, spq):
    if n < MIN_MATCHES[kind]:
        raise NotEnoughDataPoints(f"{n} matches, {kind} needs {MIN_MATCHES[kind]}")
    pc, qc = sp / ws, sq / ws
    m = _identity()
    if kind == "translation":
        m[:, 3] = qc - pc
        return m
    s = spq - ws * np.outer(pc, qc)                    # sum w (p - pc)(q - qc)^T
    if kind == "rigid":
        sxx, sxy, sxz, syx, syy, syz, szx, szy, szz = s.ravel()
        nm = np.array([[sxx + syy + szz, syz - szy, szx - sxz, sxy - syx],
                       [syz - szy, sxx - syy - szz, sxy + syx, szx + sxz],
                       [szx - sxz, sxy + syx, -sxx + syy - szz, syz + szy],
                       [sxy - syx, szx + sxz, syz + szy, -sxx - syy + szz]])
        _, vec = np.linalg.eigh(nm)
        q0, qx, qy, qz = vec[:, -1]                    # the largest eigenvalue's unit quaternion
        r = np.array([[q0 * q0 + qx * qx - qy * qy - qz * qz, 2 * (qx * qy - q0 * qz), 2 * (qx * qz + q0 * qy)],
                      [2 * (qy * qx + q0 * qz), q0 * q0 - qx * qx + qy * qy - qz * qz, 2 * (qy * qz - q0 * qx)],
                      [2 * (qz * qx - q0 * qy), 2 * (qz * qy + q0 * qx), q0 * q0 - qx * qx - qy * qy + qz * qz]])
    else:
        a = spp - ws * np.outer(pc, pc)                # sum w (p - pc)(p - pc)^T
        if abs(np.linalg.det(a)) < 1e-12 * max(1.0, np.abs(a).max()) ** 3:
            raise IllDefinedDataPoints("singular point configuration for an affine fit")
        r = np.linalg.solve(a, s).T
    m[:, :3] = r
    m[:, 3] = qc - r @ pc
    return m


@dataclass
class PairwiseMatch:
    """The inliers of one view pair (PairwiseMatch.getInliers): pa[i] in view a
    corresponds to pb[i] in view b."""
    a: int
    b: int
    pa: np.ndarray
    pb: np.ndarray
    weights: np.ndarray | None = None


@dataclass
class GlobalOptResult:
    models: list          # per view: 3x4 correction (the tile's model)
    error: float          # TileConfiguration.getError (mean tile distance)
    min_error: float
    max_error: float
    iterations: int
    unaligned: list       # views whose tile preAlign could not reach
    tiles: list           # per view: tile index (views of one timepoint share one)
    failure: str | None = None   # the caught NotEnoughDataPoints / IllDefinedDataPoints message


class _Tiles:
    """The tiles' models and matches.  A match's partner point moves only with
    the partner's (affine) model, so a tile's fit needs per partner only the
    moments of its local points against the partner's local points; the
    distances are evaluated per pair (both tiles of a pair share them)."""

    def __init__(self, ntiles, kind):
        self.kind = kind
        self.models = [_identity() for _ in range(ntiles)]
        self.pairs = []                          # (ta, tb, pa, pb)
        self.sides = [[] for _ in range(ntiles)]  # per tile: (partner, n, moments of own vs partner points)

    def add(self, ta, tb, pa, pb, w):
        self.pairs.append((ta, tb, pa, pb))
        self.sides[ta].append((tb, len(pa), _moments(pa, pb, w)))
        self.sides[tb].append((ta, len(pa), _moments(pb, pa, w)))

    def fit(self, t, only=None):
        n, ws, sp, sq, spp, spq = 0, 0.0, np.zeros(3), np.zeros(3), np.zeros((3, 3)), np.zeros((3, 3))
        for partner, k, (w0, p1, q1, pp, pq) in self.sides[t]:
            if only is not None and partner not in only:
                continue
            a, tr = self.models[partner][:, :3], self.models[partner][:, 3]
            n += k
            ws += w0
            sp = sp + p1
            sq = sq + a @ q1 + w0 * tr
            spp = spp + pp
            spq = spq + pq @ a.T + np.outer(p1, tr)
        self.models[t] = _fit_moments(self.kind, n, ws, sp, sq, spp, spq)

    def partners(self, t):
        return [partner for partner, *_ in self.sides[t]]

    def distances(self, ntiles):
        """Per tile Tile.getDistance: the mean over its matches of |model(p) - partner_model(q)|."""
        tot, cnt = np.zeros(ntiles), np.zeros(ntiles)
        for ta, tb, pa, pb in self.pairs:
            d = np.linalg.norm(apply(self.models[ta], pa) - apply(self.models[tb], pb), axis=1).sum()
            tot[ta] += d
            tot[tb] += d
            cnt[ta] += len(pa)
            cnt[tb] += len(pa)
        return tot, cnt


def compute(n_views: int, pairs, model: str = "affine", fixed=(0,), timepoint_of=None,
            max_allowed_error: float = 10.0, max_iterations: int = 10000,
            max_plateau_width: int = 200) -> GlobalOptResult | None:
    """GlobalOpt.compute over ``n_views`` views and their ``pairs`` (PairwiseMatch).

    ``fixed``: the views whose tile is fixed (GlobalOptimizationType.isFixedTile);
    ``timepoint_of``: per view its timepoint id to make one tile per timepoint
    (considerTimePointsAsUnit), None for one tile per view.  Returns None when no
    tile is connected (the reference prints "no connected tiles" and returns null)."""
    if model not in MIN_MATCHES:
        raise ValueError(f"model must be one of {sorted(MIN_MATCHES)}")
    if timepoint_of is None:
        tile_of = list(range(n_views))
    else:
        ids = {}
        tile_of = [ids.setdefault(t, len(ids)) for t in timepoint_of]
    ntiles = max(tile_of) + 1 if n_views else 0
    tiles = _Tiles(ntiles, model)
    connected = set()
    for pm in pairs:
        pa = np.asarray(pm.pa, np.float64).reshape(-1, 3)
        pb = np.asarray(pm.pb, np.float64).reshape(-1, 3)
        if len(pa) != len(pb):
            raise ValueError("a pairwise match needs as many points in a as in b")
        if len(pa) == 0:
            continue
        w = np.ones(len(pa)) if pm.weights is None else np.asarray(pm.weights, np.float64)
        ta, tb = tile_of[pm.a], tile_of[pm.b]
        tiles.add(ta, tb, pa, pb, w)
        connected |= {ta, tb}
    order = sorted(connected)                        # TileConfiguration.addTile: connected tiles
    if not order:
        return None
    fixed_tiles = {tile_of[v] for v in fixed} & connected

    # preAlign then optimize(10, 10000, 200); a NotEnoughDataPoints / IllDefinedDataPoints
    # from either is caught, printed and the tiles' models returned as they stand
    # (GlobalOpt.java:64-100)
    aligned, failure, i = [], None, 0
    try:
        _pre_align(tiles, order, fixed_tiles, aligned)
        i = _optimize(tiles, order, fixed_tiles, ntiles, max_allowed_error, max_iterations, max_plateau_width)
    except (NotEnoughDataPoints, IllDefinedDataPoints) as e:
        failure = f"Global optimization failed: {type(e).__name__}: {e}"
        print(failure)
    unaligned_tiles = [t for t in order if t not in aligned]
    tot, cnt = tiles.distances(ntiles)
    d = tot[order] / cnt[order]
    return GlobalOptResult(models=[tiles.models[tile_of[v]] for v in range(n_views)],
                           error=float(np.mean(d)), min_error=float(np.min(d)), max_error=float(np.max(d)),
                           iterations=i, unaligned=[v for v in range(n_views) if tile_of[v] in unaligned_tiles],
                           tiles=tile_of, failure=failure)


def _pre_align(tiles, order, fixed_tiles, aligned):
    """TileConfiguration.preAlign: walk a list of aligned tiles (the fixed ones, or the
    first tile) with a list iterator; every unaligned tile connected to the current one is
    fitted to its matches with that tile only, inserted at the iterator's cursor and
    stepped back over (ListIterator.add + previous), so it is visited next.  Fills
    ``aligned`` (so a fit that raises leaves the tiles aligned so far); the rest are the
    ones preAlign reports as unaligned."""
    aligned[:] = [t for t in order if t in fixed_tiles] or [order[0]]
    unaligned = [t for t in order if t not in aligned]
    cur = 0
    while cur < len(aligned):
        a = aligned[cur]
        cur += 1                                     # ita.next()
        partners = set(tiles.partners(a))
        for u in list(unaligned):
            if u in partners:
                tiles.fit(u, only={a})
                aligned.insert(cur, u)               # ita.add(u); ita.previous()
                unaligned.remove(u)


def _optimize(tiles, order, fixed_tiles, ntiles, max_allowed_error, max_iterations, max_plateau_width):
    """TileConfiguration.optimize(maxAllowedError, maxIterations, maxPlateauWidth): the
    number of iterations run."""
    history = []
    i = 0
    proceed = i < max_iterations
    while proceed:
        for t in order:
            if t not in fixed_tiles:
                tiles.fit(t)
        tot, cnt = tiles.distances(ntiles)
        err = float(np.mean(tot[order] / cnt[order]))
        history.append(err)
        if i > max_plateau_width:
            proceed = err > max_allowed_error
            k = max_plateau_width
            while not proceed and k >= 1:
                proceed |= abs((history[-1] - history[-1 - k]) / k) > 1e-4
                k //= 2
        i += 1
        proceed &= i < max_iterations
    return i


def correspondences(points, models, radius: float = 2.0):
    """Pairwise matches from detections and approximate view models: per view
    pair, the mutual nearest neighbours within ``radius`` world pixels (an
    ICP-style stand-in for the descriptor matching that produces the
    reference's inliers, which stays out of scope).  Returns PairwiseMatch
    lists over world coordinates under ``models``."""
    from scipy.spatial import cKDTree
    world = [apply(np.asarray(m, np.float64).reshape(3, 4), np.asarray(p, np.float64).reshape(-1, 3))
             for p, m in zip(points, models)]
    trees = [cKDTree(w) if len(w) else None for w in world]
    out = []
    for a in range(len(world)):
        for b in range(a + 1, len(world)):
            if trees[a] is None or trees[b] is None:
                continue
            dab, jab = trees[b].query(world[a], distance_upper_bound=radius)
            dba, jba = trees[a].query(world[b], distance_upper_bound=radius)
            ia = np.nonzero(np.isfinite(dab))[0]
            ia = ia[jba[jab[ia]] == ia]               # mutual nearest neighbours
            if len(ia):
                out.append(PairwiseMatch(a, b, world[a][ia], world[b][jab[ia]]))
    return out


def concatenate(correction, model):
    """correction o model, both 3x4 (the refined view model)."""
    c, m = np.asarray(correction, np.float64), np.asarray(model, np.float64).reshape(3, 4)
    out = np.empty((3, 4))
    out[:, :3] = c[:, :3] @ m[:, :3]
    out[:, 3] = c[:, :3] @ m[:, 3] + c[:, 3]
    return out
