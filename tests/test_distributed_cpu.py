"""CPU, world_size 2 over gloo: the z-slab decomposition used by the multi-GPU
path is exact.

Each rank owns the slab ``mvd_slab_range`` (the C-ABI the GPU path uses)
assigns it, exchanges ``c_z`` halo planes with its neighbour before each
convolution exactly as libspimdecon's exchange does (psi before convolve1,
the quotient before convolve2; mirror / constant-1 extension only at the
global boundary), and all-reduces {sumChange (sum), maxChange (max)}.  The
compute per slab is the oracle's; the gathered psi must equal the
whole-volume oracle result, and the RCCL id broadcast helper must deliver
rank 0's bytes to every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import mvdecon_ref as ref
from spim_registration_amd import synthetic
from spim_registration_amd.distributed import broadcast_comm_id, halo_planes_needed, slab_range

SHAPE = (30, 12, 14)      # z, y, x
KS = (5, 5, 7)            # kx, ky, kz  -> cz = 3
ITERS = 2
LAM = 0.006


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _exchange(block, z0, z1, nz, cz, rank, world):
    """block: local slab [z1-z0, y, x]; returns the slab with cz halo planes
    from the neighbours (None where the global boundary is)."""
    lower = upper = None
    reqs = []
    if rank > 0:
        lower = torch.empty((cz,) + block.shape[1:], dtype=torch.float32)
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(block[:cz])), rank - 1))
        reqs.append(dist.irecv(lower, rank - 1))
    if rank < world - 1:
        upper = torch.empty((cz,) + block.shape[1:], dtype=torch.float32)
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(block[-cz:])), rank + 1))
        reqs.append(dist.irecv(upper, rank + 1))
    for r in reqs:
        r.wait()
    return (lower.numpy() if lower is not None else None), (upper.numpy() if upper is not None else None)


def _slab_conv(block, lower, upper, k, ext, cz):
    """conv over the slab: neighbour planes where present, `ext` at the global ends."""
    mode = {"mirror": "reflect", "one": "constant"}[ext]
    kw = {"constant_values": 1.0} if ext == "one" else {}
    pad_z_lo = lower if lower is not None else None
    pad_z_hi = upper if upper is not None else None
    ext_full = np.pad(block, [(cz, cz), (0, 0), (0, 0)], mode=mode, **kw)
    if pad_z_lo is not None:
        ext_full[:cz] = pad_z_lo
    if pad_z_hi is not None:
        ext_full[-cz:] = pad_z_hi
    # x/y extension + valid convolution in z, x, y
    out = ref.convolve(ext_full, k, ext)          # pads z again (ignored below)
    return out[cz:-cz]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        imgs, ws, psfs, _ = synthetic.make_views(SHAPE, 2, config_id=21, ksize=KS,
                                                 bead_density=1.0 / 5 ** 3)
        k1s, k2s = ref.prepare_kernels(psfs, ref.PSFTYPE.OPTIMIZATION_I, 8)
        nz = SHAPE[0]
        cz = KS[2] // 2
        z0, z1 = slab_range(nz, world, rank)
        lo, up = halo_planes_needed(z0, z1, nz, cz)
        assert (lo[1] - lo[0]) in (0, cz) and (up[1] - up[0]) in (0, cz)
        # initial psi: global first-iteration average (all-reduced sums)
        cnt, _ = ref.first_iteration([i[z0:z1] for i in imgs])
        st = np.stack([i[z0:z1].astype(np.float64) for i in imgs])
        pos = st > 0
        c = pos.sum(0)
        mean = np.where(c > 0, np.where(pos, st, 0).sum(0) / np.maximum(c, 1), 0)
        acc = torch.tensor([mean[c > 0].sum(), float((c > 0).sum())], dtype=torch.float64)
        dist.all_reduce(acc)
        avg = float(acc[0] / acc[1])
        psi = np.full((z1 - z0,) + SHAPE[1:], np.float32(avg), np.float32)
        stats = []
        for _ in range(ITERS):
            for v in range(2):
                l, u = _exchange(psi, z0, z1, nz, cz, rank, world)
                blurred = _slab_conv(psi, l, u, k1s[v], "mirror", cz)
                qt = ref.compute_quotient(blurred, imgs[v][z0:z1])
                l, u = _exchange(qt, z0, z1, nz, cz, rank, world)
                integ = _slab_conv(qt, l, u, k2s[v], "one", cz)
                psi, s, m = ref.compute_final_values(psi, integ, ws[v][z0:z1], LAM)
                t = torch.tensor([s], dtype=torch.float64)
                mm = torch.tensor([m], dtype=torch.float64)
                dist.all_reduce(t)
                dist.all_reduce(mm, op=dist.ReduceOp.MAX)
                stats.append((float(t), float(mm)))
        psi = np.where(cnt == 0, np.float32(0), psi).astype(np.float32)
        gathered = [None] * world
        dist.all_gather_object(gathered, (z0, psi))
        cid = broadcast_comm_id(dist, rank, make_id=lambda: bytes(range(128)))
        if rank == 0:
            full = np.concatenate([g[1] for g in sorted(gathered, key=lambda g: g[0])])
            res = ref.mv_deconvolution(imgs, ws, psfs, ref.PSFTYPE.OPTIMIZATION_I, ITERS, LAM)
            err = float(np.linalg.norm(full - res.psi) / np.linalg.norm(res.psi))
            serr = float(np.max(np.abs(np.array(stats) - np.array(res.stats).reshape(-1, 2)) /
                                np.abs(np.array(res.stats).reshape(-1, 2))))
            q.put(("ok", err, serr, cid == bytes(range(128))))
        else:
            q.put(("rank", rank, cid == bytes(range(128))))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", repr(e)))
    finally:
        dist.destroy_process_group()


def test_slab_decomposition_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [o for o in out if o[0] == "err"]
    assert not errs, errs
    ok = [o for o in out if o[0] == "ok"][0]
    assert ok[1] < 1e-6, ok          # slab decomposition == whole volume
    assert ok[2] < 1e-6, ok          # all-reduced per-view statistics
    assert all(o[-1] for o in out)   # RCCL id broadcast delivered rank 0's bytes


# ---------------------------------------------------------------------------- halo plan
# The RCCL send / recv offsets, the device-group peer pulls and the local slab copies
# all come from one helper (mvd_halo_plan / session.cpp halo_plan).  Here the plan is
# replayed as RCCL would execute it -- rank r sends [send_hi] to r + 1, which receives
# it at [recv_lo]; rank r sends [send_lo] to r - 1, which receives it at [recv_hi] --
# over the internal geometry of the 8-rank decompositions of BASELINE configs[2] (C3,
# 1024 y-rows -> 8 y-slabs of 128 + 2*12 halo rows: Mz = 152 != nz) and configs[4] (C5,
# 2048 y-rows -> 256 + 24 = 280), plus a ragged split; every rank's halo planes must
# then hold exactly its neighbours' global planes.  (The gloo test above validates the
# decomposition arithmetic with its own numpy exchange; this one pins the addresses.)

from spim_registration_amd.distributed import halo_plan  # noqa: E402


def _hp_geometry(plane_rows, Mx):
    """floats per padded plane of the engine spectrum: 2 * Hp * My, Hp = 16-padded Mx/2+1."""
    Hp = -(-(Mx // 2 + 1) // 16) * 16
    return 2 * Hp * plane_rows


@pytest.mark.parametrize("name,nglob,nranks,cz,My,Mx", [
    ("C3", 1024, 8, 12, 536, 1050),     # internal (x, z, y): planes = y rows, My = padded z
    ("C5", 2048, 8, 12, 1050, 2100),
    ("ragged", 1000, 3, 15, 96, 128),
])
def test_halo_plan_replayed_as_rccl(name, nglob, nranks, cz, My, Mx):
    plane_real = _hp_geometry(My, Mx)
    P = 3                                    # small plane for the replay; offsets scale by plane
    ranks = []
    for r in range(nranks):
        z0, z1 = slab_range(nglob, nranks, r)
        nz = z1 - z0
        Mz = nz + 2 * cz                     # the direct z pass pads exactly
        h = halo_plan(nz, Mz, cz, P)
        hr = halo_plan(nz, Mz, cz, plane_real)
        # offsets are plane multiples of the same plan at the real plane size
        for k in h:
            assert hr[k] == h[k] // P * plane_real, (k, h, hr)
        assert h["send_lo"] == 0 and h["recv_hi"] == nz * P and h["recv_lo"] == (Mz - cz) * P
        assert h["send_hi"] == (nz - cz) * P and h["count"] == cz * P
        buf = np.full(Mz * P, -1.0)
        buf[:nz * P] = np.repeat(np.arange(z0, z1, dtype=np.float64), P)   # interior = global plane ids
        ranks.append(dict(z0=z0, z1=z1, nz=nz, Mz=Mz, h=h, buf=buf))
    sent = [r["buf"].copy() for r in ranks]  # sends read the pre-exchange buffers
    for r, st in enumerate(ranks):
        h = st["h"]
        if r > 0:        # from the lower neighbour: its send_hi -> my recv_lo
            lo = ranks[r - 1]
            assert lo["h"]["count"] == h["count"]
            st["buf"][h["recv_lo"]:h["recv_lo"] + h["count"]] = \
                sent[r - 1][lo["h"]["send_hi"]:lo["h"]["send_hi"] + lo["h"]["count"]]
        if r < nranks - 1:   # from the upper neighbour: its send_lo -> my recv_hi
            hi = ranks[r + 1]
            st["buf"][h["recv_hi"]:h["recv_hi"] + h["count"]] = \
                sent[r + 1][hi["h"]["send_lo"]:hi["h"]["send_lo"] + hi["h"]["count"]]
    for r, st in enumerate(ranks):
        planes = st["buf"].reshape(st["Mz"], P)[:, 0]
        nz, Mz = st["nz"], st["Mz"]
        np.testing.assert_array_equal(planes[:nz], np.arange(st["z0"], st["z1"]))   # interior untouched
        if r < nranks - 1:
            np.testing.assert_array_equal(planes[nz:nz + cz], np.arange(st["z1"], st["z1"] + cz))
        if r > 0:
            np.testing.assert_array_equal(planes[Mz - cz:], np.arange(st["z0"] - cz, st["z0"]))
    # first, middle and last rank: which transfers exist
    assert ranks[0]["z0"] == 0 and ranks[-1]["z1"] == nglob


def test_halo_plan_rejects_bad_geometry():
    from spim_registration_amd import _lib
    with pytest.raises(_lib.SpimDeconError):
        halo_plan(10, 20, 6, 4)      # Mz < nz + 2 cz


# ------------------------------------------------------- rank consistency before exchanging
# bench.py all-gathers every rank's exchange plan (distributed.rank_plan) over the gloo
# control group after mvd_init and refuses to start when they disagree, so ranks can never
# post mismatched ncclSend / ncclRecv and wait forever.  The plans here are what rank_plan
# returns for C3's 8-rank y-slab decomposition (1024 rows -> 128 + 2 * 12 per rank).

from spim_registration_amd.distributed import check_rank_plans, verify_rank_plans  # noqa: E402


def _c3_plan(rank, world=8, nglob=1024, cz=12, Mx=1050, My=540, nviews=6, zmode=3):
    z0, z1 = slab_range(nglob, world, rank)
    nz = z1 - z0
    Mz = nz + 2 * cz
    plane = 2 * (-(-(Mx // 2 + 1) // 16) * 16) * My
    sl = {"fft_dims": [Mx, My, Mz], "extent": [1024, 512, nz], "kernel_planes": 2 * cz + 1,
          "zpass_mode": zmode, "halo": halo_plan(nz, Mz, cz, plane)}
    return {"rank": rank, "world": world, "nranks": world, "nviews": nviews, "storage_fp16": 0,
            "fft_backend": 0, "slab_axis": 1, "nz_global": nglob, "z_offset": z0, "extent": nz,
            "zpass_modes": [zmode], "slabs": [sl]}


def test_rank_plans_agree_and_disagree():
    plans = [_c3_plan(r) for r in range(8)]
    assert check_rank_plans(plans) == []
    bad = [dict(p) for p in plans]
    bad[3] = _c3_plan(3, nviews=5)
    assert any(e.startswith("nviews") for e in check_rank_plans(bad))
    bad = [_c3_plan(r, zmode=3 if r != 5 else 1) for r in range(8)]
    assert any(e.startswith("zpass_modes") for e in check_rank_plans(bad))
    bad = [_c3_plan(r) for r in range(8)]
    bad[4]["z_offset"] += 1                              # a gap between ranks 3 and 4
    assert any("rank 3 owns" in e for e in check_rank_plans(bad))
    bad = [_c3_plan(r, cz=12 if r != 6 else 10) for r in range(8)]   # other halo widths
    assert any("halo transfer" in e for e in check_rank_plans(bad))
    bad = [_c3_plan(r, My=540 if r < 7 else 576) for r in range(8)]
    assert any("x-y spectrum planes" in e for e in check_rank_plans(bad))
    assert check_rank_plans(plans[:7])                   # the last rank is missing


def _plan_worker(rank, world, port, q, disagree):
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    t0 = time.perf_counter()
    try:
        plan = _c3_plan(rank, world=world, nglob=256, nviews=6 if (rank == 0 or not disagree) else 4)
        verify_rank_plans(dist, plan)
        q.put(("ok", rank, time.perf_counter() - t0))
    except RuntimeError as e:
        q.put(("refused", rank, time.perf_counter() - t0, str(e)))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("disagree", [False, True])
def test_rank_plans_gloo_world2_fail_fast(disagree):
    """world 2 over gloo: agreeing ranks both start; ranks with other view counts are both
    refused, within seconds (no exchange is ever posted)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, 2, port, q, disagree)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in procs], key=lambda o: o[1])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    kinds = {o[0] for o in out}
    assert kinds == ({"refused"} if disagree else {"ok"}), out
    assert all(o[2] < 30 for o in out), out
    if disagree:
        assert all("nviews: rank 1 has 4, rank 0 has 6" in o[3] for o in out), out
