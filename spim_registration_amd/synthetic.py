"""Synthetic multiview bead stacks (SURVEY.md section 8d "Synthetic inputs").

There is no network and no dataset: every test and benchmark input is
generated here from a seed.  ``numpy`` variants serve the parity tests (small
volumes); ``make_views_torch`` builds the large benchmark volumes on the GPU.

  truth  = 0.2 * sum of 8 smooth Gaussian blobs (sigma = min(dim)/8) + beads
           (Poisson count with mean N/16^3, amplitude U(0.5, 1), trilinear splat)
  PSF_v  = anisotropic Gaussian sigma (1.2, 1.2, 3.5) px (x, y, z), axial axis
           rotated by v*180/V degrees about y, on an odd grid, sum 1 (float64)
  img_v  = Poisson(1000 * (truth (*) PSF_v) + 5) / 1000, float32, >= 1e-4
  w_v    = cosine blend along the view's axial direction, normalised across
           views with the VIRTUAL rule w_v / max(sum_w, 1)
"""
from __future__ import annotations

import math

import numpy as np
import scipy.signal

SEED0 = 20140611


def rng_for(config_id: int):
    return np.random.default_rng(SEED0 + int(config_id))


def psf(view: int, num_views: int, size=(25, 25, 25), sigma=(1.2, 1.2, 3.5)) -> np.ndarray:
    """[z, y, x] PSF of view ``view`` (odd ``size`` = (kx, ky, kz))."""
    kx, ky, kz = size
    th = math.radians(view * 180.0 / max(num_views, 1))
    z, y, x = np.meshgrid(np.arange(kz) - kz // 2, np.arange(ky) - ky // 2, np.arange(kx) - kx // 2,
                          indexing="ij")
    # rotate coordinates about y by -theta (axial axis z -> rotated)
    xr = math.cos(th) * x - math.sin(th) * z
    zr = math.sin(th) * x + math.cos(th) * z
    sx, sy, sz = sigma
    g = np.exp(-0.5 * ((xr / sx) ** 2 + (y / sy) ** 2 + (zr / sz) ** 2))
    g /= g.sum()
    return g.astype(np.float32)


def truth_volume(shape, rng, bead_density=1.0 / 16 ** 3) -> np.ndarray:
    """[z, y, x] ground truth."""
    nz, ny, nx = shape
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij", sparse=True)
    s = min(shape) / 8.0
    t = np.zeros(shape, np.float64)
    for _ in range(8):
        cz, cy, cx = rng.uniform(0, nz), rng.uniform(0, ny), rng.uniform(0, nx)
        t += np.exp(-0.5 * (((z - cz) ** 2 + (y - cy) ** 2 + (x - cx) ** 2) / s ** 2))
    t *= 0.2
    nb = rng.poisson(np.prod(shape) * bead_density)
    pos = rng.uniform([0, 0, 0], [nz - 1, ny - 1, nx - 1], size=(nb, 3))
    amp = rng.uniform(0.5, 1.0, size=nb)
    i0 = np.floor(pos).astype(np.int64)
    f = pos - i0
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                wgt = ((f[:, 0] if dz else 1 - f[:, 0]) * (f[:, 1] if dy else 1 - f[:, 1]) *
                       (f[:, 2] if dx else 1 - f[:, 2]))
                iz = np.minimum(i0[:, 0] + dz, nz - 1)
                iy = np.minimum(i0[:, 1] + dy, ny - 1)
                ix = np.minimum(i0[:, 2] + dx, nx - 1)
                np.add.at(t, (iz, iy, ix), amp * wgt)
    return t


def blend_weight(shape, view: int, num_views: int) -> np.ndarray:
    """cosine blend (1 in the centre, 0 at the ends) along the view's axial direction."""
    nz, ny, nx = shape
    th = math.radians(view * 180.0 / max(num_views, 1))
    z, y, x = np.meshgrid(np.linspace(-1, 1, nz), np.linspace(-1, 1, ny), np.linspace(-1, 1, nx),
                          indexing="ij", sparse=True)
    t = np.abs(math.sin(th) * x + math.cos(th) * z) / max(abs(math.sin(th)) + abs(math.cos(th)), 1e-9)
    r = np.clip((t - 0.5) / 0.5, 0.0, 1.0)
    w = 0.5 + 0.5 * np.cos(math.pi * r)
    return np.broadcast_to(w, shape).astype(np.float64)


def make_views(shape, num_views: int, config_id: int = 0, ksize=(25, 25, 25),
               weights: str = "blend", partial: bool = False, bead_density=1.0 / 16 ** 3,
               photons: float = 1000.0):
    """Returns (imgs, weights, psfs, truth); shape = (nz, ny, nx).

    ``weights``: 'blend' (VIRTUAL-normalised cosine blending) or 'ones'.
    ``partial``: view 0 has no data (img = 0, w = 0) in its last third along z."""
    rng = rng_for(config_id)
    truth = truth_volume(shape, rng, bead_density)
    imgs, ws, psfs = [], [], []
    for v in range(num_views):
        k = psf(v, num_views, ksize)
        psfs.append(k)
        blurred = scipy.signal.fftconvolve(np.pad(truth, [(s // 2, s // 2) for s in k.shape], mode="reflect"),
                                           k.astype(np.float64), mode="valid")
        lam = np.maximum(photons * blurred + 5.0, 0.0)
        img = (rng.poisson(lam) / photons).astype(np.float32)
        img = np.maximum(img, np.float32(1e-4))
        imgs.append(img)
        ws.append(blend_weight(shape, v, num_views) if weights == "blend" else np.ones(shape))
    if partial:
        z3 = shape[0] - shape[0] // 3
        imgs[0][z3:] = 0.0
        ws[0][z3:] = 0.0
    if weights == "blend":
        s = np.sum(ws, axis=0)
        ws = [(w / np.maximum(s, 1.0)) for w in ws]
    ws = [np.ascontiguousarray(w, np.float32) for w in ws]
    return imgs, ws, psfs, truth.astype(np.float32)


def make_views_torch(shape, num_views: int, config_id: int = 1, ksize=(25, 25, 25), device="cuda",
                     photons: float = 1000.0):
    """Large benchmark inputs generated on the GPU with torch (test-data plumbing,
    not product compute).  Returns (list of img tensors, list of weight tensors,
    list of numpy PSFs) on ``device``; same recipe as ``make_views`` (beads
    splatted to the nearest voxel for speed)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(SEED0 + int(config_id))
    nz, ny, nx = shape
    dev = torch.device(device)
    z = torch.arange(nz, device=dev, dtype=torch.float32).view(-1, 1, 1)
    y = torch.arange(ny, device=dev, dtype=torch.float32).view(1, -1, 1)
    x = torch.arange(nx, device=dev, dtype=torch.float32).view(1, 1, -1)
    s = min(shape) / 8.0
    truth = torch.zeros(shape, device=dev, dtype=torch.float32)
    for _ in range(8):
        c = torch.rand(3, generator=g, device=dev) * torch.tensor([nz, ny, nx], device=dev)
        truth += torch.exp(-0.5 * ((z - c[0]) ** 2 + (y - c[1]) ** 2 + (x - c[2]) ** 2) / s ** 2)
    truth *= 0.2
    nb = int(np.prod(shape) / 16 ** 3)
    idx = (torch.rand(nb, generator=g, device=dev) * (nz * ny * nx)).long().clamp_(0, nz * ny * nx - 1)
    amp = 0.5 + 0.5 * torch.rand(nb, generator=g, device=dev)
    truth.view(-1).index_add_(0, idx, amp)
    psfs = [psf(v, num_views, ksize) for v in range(num_views)]
    pads = [k // 2 for k in (ksize[2], ksize[1], ksize[0])]
    fshape = [shape[d] + 2 * pads[d] for d in range(3)]
    tp = torch.nn.functional.pad(truth[None, None], (pads[2], pads[2], pads[1], pads[1], pads[0], pads[0]),
                                 mode="reflect")[0, 0]
    ft = torch.fft.rfftn(tp)
    imgs, ws = [], []
    wsum = torch.zeros(shape, device=dev)
    for v in range(num_views):
        kp = torch.zeros(fshape, device=dev)
        k = torch.from_numpy(psfs[v]).to(dev)
        kz, ky, kx = k.shape
        kp[:kz, :ky, :kx] = k
        kp = torch.roll(kp, shifts=(-(kz // 2), -(ky // 2), -(kx // 2)), dims=(0, 1, 2))
        blurred = torch.fft.irfftn(ft * torch.fft.rfftn(kp), s=fshape)
        blurred = blurred[pads[0]:pads[0] + nz, pads[1]:pads[1] + ny, pads[2]:pads[2] + nx]
        lam = (photons * blurred + 5.0).clamp_(min=0.0)
        img = (torch.poisson(lam, generator=g) / photons).clamp_(min=1e-4).float().contiguous()
        imgs.append(img)
        w = torch.from_numpy(blend_weight((nz, 1, nx), v, num_views).astype(np.float32)).to(dev)
        w = w.expand(nz, ny, nx).contiguous()
        ws.append(w)
        wsum += w
        del blurred, lam, kp
    ws = [(w / wsum.clamp(min=1.0)).contiguous() for w in ws]
    del ft, tp, truth
    return imgs, ws, psfs


def rotation_about_y(angle_deg: float, center_world, center_local):
    """3x4 view -> world affine: a rotation about the y axis through the world
    centre, mapping the local stack centre onto it (SPIM angles)."""
    a = math.radians(angle_deg)
    R = np.array([[math.cos(a), 0.0, math.sin(a)], [0.0, 1.0, 0.0], [-math.sin(a), 0.0, math.cos(a)]])
    m = np.zeros((3, 4))
    m[:, :3] = R
    m[:, 3] = np.asarray(center_world, np.float64) - R @ np.asarray(center_local, np.float64)
    return m


def make_timepoint_torch(world_xyz, view_xyz, num_views: int, timepoint: int = 0, config_id: int = 4,
                         psf_sigma=(1.2, 1.2, 3.0), photons: float = 1000.0, bead_density=1.0 / 20 ** 3,
                         drift=(1.5, 0.5, 1.0), device="cuda", log=None):
    """One timepoint of a multiview acquisition (BASELINE configs[3]) generated on
    the GPU: a world volume of beads (3x3x3 footprint, drifting by ``drift`` pixels
    per timepoint) and smooth blobs; view v is that volume seen through a rotation
    about y by v * 360 / V degrees (trilinear resampling), blurred with an
    axis-aligned Gaussian PSF in its own frame (sigma x, y, z), with Poisson noise.
    Returns (views: list of [z, y, x] torch tensors, models: list of 3x4 view ->
    world affines)."""
    import torch
    import torch.nn.functional as F

    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED0 + 1000 * int(config_id))      # the same beads at every timepoint ...
    wx, wy, wz = (int(v) for v in world_xyz)
    z = torch.arange(wz, device=dev, dtype=torch.float32).view(-1, 1, 1)
    y = torch.arange(wy, device=dev, dtype=torch.float32).view(1, -1, 1)
    x = torch.arange(wx, device=dev, dtype=torch.float32).view(1, 1, -1)
    truth = torch.zeros((wz, wy, wx), device=dev)
    s = min(wx, wy, wz) / 8.0
    for _ in range(6):
        c = torch.rand(3, generator=g, device=dev) * torch.tensor([wz, wy, wx], device=dev, dtype=torch.float32)
        truth += 0.2 * torch.exp(-0.5 * ((z - c[0]) ** 2 + (y - c[1]) ** 2 + (x - c[2]) ** 2) / s ** 2)
    nb = max(1, int(wx * wy * wz * bead_density))
    pos = torch.rand((nb, 3), generator=g, device=dev) * torch.tensor([wz - 8, wy - 8, wx - 8], device=dev,
                                                                       dtype=torch.float32) + 4
    pos = pos + torch.tensor([drift[2], drift[1], drift[0]], device=dev) * timepoint   # ... drifting
    ip = pos.round().long()
    ok = ((ip >= 1) & (ip < torch.tensor([wz - 1, wy - 1, wx - 1], device=dev))).all(dim=1)
    ip = ip[ok]
    amp = 0.5 + 0.5 * torch.rand(len(ip), generator=g, device=dev)
    # overlapping footprints add up through atomics in an arbitrary order: accumulate the
    # float32 terms in float64, where these few sums are exact, so the volume is the
    # same bits on every run (tests compare a timepoint across processes)
    beads = torch.zeros(truth.numel(), device=dev, dtype=torch.float64)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                f = 0.55 ** (abs(dx) + abs(dy) + abs(dz))
                idx = ((ip[:, 0] + dz) * wy + ip[:, 1] + dy) * wx + ip[:, 2] + dx
                beads.index_add_(0, idx, (amp * f).double())
    truth += beads.view_as(truth).float()
    del beads
    vx, vy, vz = (int(v) for v in view_xyz)
    cw = ((wx - 1) / 2.0, (wy - 1) / 2.0, (wz - 1) / 2.0)
    cl = ((vx - 1) / 2.0, (vy - 1) / 2.0, (vz - 1) / 2.0)
    sx, sy, sz = psf_sigma

    views, models = [], []
    gv = torch.Generator(device=dev)
    gv.manual_seed(SEED0 + 1000 * int(config_id) + 17 * int(timepoint) + 1)
    for v in range(num_views):
        if log:
            log(f"  view {v}")
        m = rotation_about_y(v * 360.0 / num_views, cw, cl)
        models.append(m)
        M = torch.tensor(m, device=dev, dtype=torch.float32)
        out = torch.empty((vz, vy, vx), device=dev)
        zs = max(1, (1 << 26) // (vx * vy))          # resample in z chunks (bounded grid memory)
        for z0 in range(0, vz, zs):
            z1 = min(vz, z0 + zs)
            lz = torch.arange(z0, z1, device=dev, dtype=torch.float32).view(-1, 1, 1)
            ly = torch.arange(vy, device=dev, dtype=torch.float32).view(1, -1, 1)
            lx = torch.arange(vx, device=dev, dtype=torch.float32).view(1, 1, -1)
            px = M[0, 0] * lx + M[0, 1] * ly + M[0, 2] * lz + M[0, 3]
            py = M[1, 0] * lx + M[1, 1] * ly + M[1, 2] * lz + M[1, 3]
            pz = M[2, 0] * lx + M[2, 1] * ly + M[2, 2] * lz + M[2, 3]
            grid = torch.stack([2 * px / (wx - 1) - 1, 2 * py / (wy - 1) - 1, 2 * pz / (wz - 1) - 1], dim=-1)
            out[z0:z1] = F.grid_sample(truth[None, None], grid[None], mode="bilinear", padding_mode="zeros",
                                       align_corners=True)[0, 0]
            del px, py, pz, grid
        # Gaussian blur in the view's own frame: one FFT multiply by the separable
        # transfer function (circular boundary -- synthetic data)
        fz = torch.fft.fftfreq(vz, device=dev).view(-1, 1, 1)
        fy = torch.fft.fftfreq(vy, device=dev).view(1, -1, 1)
        fx = torch.fft.rfftfreq(vx, device=dev).view(1, 1, -1)
        tf = torch.exp(-2.0 * math.pi ** 2 * ((fx * sx) ** 2 + (fy * sy) ** 2 + (fz * sz) ** 2))
        out = torch.fft.irfftn(torch.fft.rfftn(out) * tf, s=(vz, vy, vx)).float()
        del tf
        lam = (photons * out + 5.0).clamp_(min=0.0)
        img = (torch.poisson(lam, generator=gv) / photons).float().contiguous()
        views.append(img)
        del out, lam
    del truth
    return views, models
