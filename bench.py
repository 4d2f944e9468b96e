#!/usr/bin/env python3
"""Benchmark: Mvoxels/s per RL iteration of the multiview deconvolution path.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric: "6-view 512^3 deconv"; configs[1] geometry and
RL settings): 6-view 512^3 synthetic PSF-blurred bead volume, 25^3 PSFs,
multiview RL (PSFTYPE INDEPENDENT, lambda 0) -- one *step* = one full RL
iteration (all views, sequential per-view updates) over the volume, inputs
resident in HBM.  With N GPUs each GPU holds a 512^3 z-slab of a
512x512x(512N) volume (weak scaling); the slabs exchange 12-plane halos before
every convolution.  value = all GPUs' voxels * steps / max time / 1e6.

Two ways to drive N GPUs, both one slab per GPU:
  * no launcher (RANK unset): one process, ``Session(devices=range(N))`` -- the
    reference's ``int[] deviceList`` driven from one JVM (MVDeconFFT.java:424-446);
    one host thread per GPU, halo planes pulled peer to peer over xGMI.  Fewer
    than N visible GPUs is an error (rc != 0), never a silent 1-GPU run.
  * torchrun (RANK set): one process per GPU, halos over RCCL send/recv.

Also reported: ``roofline`` of the dominant engine pass (largest total time;
algorithmic bytes per launch in DESIGN.md "Kernels") timed with HIP events on
the session's stream, ``roofline_iteration`` (whole iteration against the
engine's compulsory traffic), ``default_mode`` (the reference default
OPTIMIZATION_I lambda 0.006 on the same views, with its own roofline and
kernel breakdown), ``strong`` (BASELINE configs[2]: 6-view 1024x1024x512,
EFFICIENT_BAYESIAN 0.006, split into N y-slabs -- the strong-scaling line) and
``cpu_baseline`` = the oracle's float32 scipy.fft restatement of the same
iteration on a bounded sample (rank 0, N=1 only; 1 warm-up + 2 timed
iterations, BASELINE.md protocol).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mvoxels/sec per RL iter, 6-view 512³ deconv; 1/2/4/8-GPU scaling"  # BASELINE.json
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--views", type=int, default=6)
    ap.add_argument("--size", type=int, default=512, help="per-GPU cube edge")
    ap.add_argument("--shape", type=int, nargs=3, metavar=("X", "Y", "Z"),
                    help="per-GPU slab x y z (overrides --size; z-slabs stack over GPUs)")
    ap.add_argument("--ksize", type=int, default=25)
    ap.add_argument("--psftype", default="INDEPENDENT")
    ap.add_argument("--lam", type=float, default=0.0)
    ap.add_argument("--fp16", action="store_true", help="fp16 img/weight storage")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-size", type=int, default=384,
                    help="edge of the CPU-baseline sample cube (same views, PSFs and mode)")
    ap.add_argument("--cpu-iters", type=int, default=2, help="timed CPU-baseline iterations (after 1 warm-up)")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event roofline pass")
    ap.add_argument("--backend", default="engine", choices=["engine", "rocfft"])
    ap.add_argument("--pad-policy", default="auto", choices=["auto", "fast", "smooth"])
    ap.add_argument("--local-slabs", type=int, default=1, help="slabs per GPU (virtual shards)")
    ap.add_argument("--strong", action="store_true",
                    help="headline = strong scaling: the global volume --shape (default 1024 1024 512, "
                         "EFFICIENT_BAYESIAN lambda 0.006 = BASELINE configs[2]) split into N slabs along "
                         "the longer of y and z, one per GPU")
    ap.add_argument("--no-strong-line", action="store_true",
                    help="skip the extra strong-scaling C3 measurement (the 'strong' key)")
    ap.add_argument("--strong-steps", type=int, default=4)
    ap.add_argument("--no-legacy-line", action="store_true",
                    help="skip the opt-in legacy simultaneous-update line (lrsim_*: one view per GPU, "
                         "the compound-correction all-reduce over the ranks)")
    ap.add_argument("--allow-fallback", action="store_true",
                    help="measure even when a slab runs outside the fast engine passes (else rc != 0)")
    ap.add_argument("--no-default-mode", action="store_true",
                    help="skip the second measurement in the reference default mode (OPTIMIZATION_I, 0.006)")
    ap.add_argument("--slab-axis", default="auto", choices=["auto", "z", "y"],
                    help="split / internal slab axis of the headline session (y: rows kept as (x, z, y), "
                         "the layout of a y-slab rank; one GPU only unless --strong)")
    ap.add_argument("--c5-rank", action="store_true",
                    help="BASELINE configs[4] per rank: the 2048x256x1024 y-slab one of 8 ranks holds "
                         "(padded 2100x1050x280 internally), fp16 img/weight storage, OPTIMIZATION_I 0.006")
    ap.add_argument("--c3-rank", action="store_true",
                    help="BASELINE configs[2] per rank: the 1024x128x512 y-slab one of 8 ranks holds "
                         "(padded 1050x540x152 internally), EFFICIENT_BAYESIAN 0.006")
    a = ap.parse_args(argv)
    if a.c3_rank:
        a.shape = [1024, 128, 512]
        a.slab_axis = "y"
        a.psftype, a.lam = "EFFICIENT_BAYESIAN", 0.006
        a.no_strong_line = a.no_default_mode = True
    if a.c5_rank:
        a.shape = [2048, 256, 1024]
        a.fp16, a.slab_axis = True, "y"
        a.psftype, a.lam = "OPTIMIZATION_I", 0.006
        a.no_strong_line = a.no_default_mode = True
        if a.cpu_size == 384:
            a.cpu_size = 256
    if a.strong and a.shape is None:
        a.shape = [1024, 1024, 512]
        if a.psftype == "INDEPENDENT" and a.lam == 0.0:
            a.psftype, a.lam = "EFFICIENT_BAYESIAN", 0.006
    return a


def plan_gpus(args, env, visible):
    """How the N GPUs are driven: ('ranks', world) under a launcher (RANK set; WORLD_SIZE
    must equal --gpus) or ('devices', N) in one process.  Raises SystemExit (rc != 0)
    rather than measuring fewer GPUs than asked for."""
    n = int(args.gpus)
    if n < 1:
        raise SystemExit("--gpus must be >= 1")
    if "RANK" in env:
        world = int(env.get("WORLD_SIZE", "1"))
        if world != n:
            raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}")
        return "ranks", world
    if visible < n:
        raise SystemExit(f"--gpus {n} asked for, but only {visible} GPU(s) visible: refusing to measure fewer")
    return "devices", n


# engine kernel class -> kernel-name prefixes in the PMC table (tools/pmc_summary.py --json)
PMC_KERNELS = {"z_convolve": ("k_zdmc<", "k_col2f<2,", "k_colpass<2,"), "y_pass": ("k_col2f<1,", "k_colpass<1,"),
               "x_update": ("k_xtile<2,", "k_xrows<2,", "k_xpass<2,"),
               "x_quotient": ("k_xtile<1,", "k_xrows<1,", "k_xpass<1,")}


def pmc_traffic(cls, M, fp16, backend):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes
    (profiles/pmc_traffic.json, same FFT dims and storage), or (None, None)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if backend != "engine" or not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    if list(d.get("fft_dims", [])) != list(M) or bool(d.get("fp16", False)) != bool(fp16):
        return None, None
    hits = []   # the class's kernels (the y class: forward and inverse, launched equally often)
    for name, ent in d["kernels"].items():
        if name.startswith(PMC_KERNELS.get(cls, ())):
            targs = [a.strip() for a in name.split("<", 1)[1].rstrip(">").split(",")]
            if cls == "z_convolve" and name.startswith("k_col2f") and targs[3] not in ("2", "4", "5"):
                continue   # the fused z pass: k_col2f MODE 2/4/5 (5 = compact kernels)
            hits.append((name, int(ent.get("hbm_bytes_per_launch_median", ent["hbm_bytes_per_launch"]))))
    if not hits:
        return None, None
    if cls == "z_convolve":
        hits = hits[:1]
    return (int(sum(b for _, b in hits) / len(hits)),
            "profiles/pmc_traffic.json: " + " / ".join(n for n, _ in hits) + (" (mean of the median launches)" if len(hits) > 1 else " (median launch)"))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args):
    """The oracle (numpy + scipy.fft float32, multithreaded) on a bounded sample of the
    SAME workload (V views, same PSFs and RL mode, a --cpu-size cube): 1 warm-up
    iteration, then --cpu-iters timed iterations (BASELINE.md protocol), per-iteration
    Mvox/s.  Threads: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the MI355X
    pool; os.cpu_count() elsewhere) -- reported as `cores` next to the host's logical
    CPU count and model."""
    from oracle import mvdecon_ref as ref
    from spim_registration_amd import synthetic

    n = args.cpu_size
    host_cpus = os.cpu_count() or 1
    cores = int(os.environ.get("OMP_NUM_THREADS", host_cpus))
    imgs, ws, psfs, _ = synthetic.make_views((n, n, n), args.views, config_id=1,
                                             ksize=(args.ksize,) * 3, weights="blend")
    k1s, k2s = ref.prepare_kernels(psfs, ref.PSFTYPE[args.psftype], 8)
    _, avg = ref.first_iteration(imgs)
    psi = np.full(imgs[0].shape, np.float32(avg), np.float32)
    psi, _ = ref.run_iteration(psi, imgs, ws, k1s, k2s, args.lam, "f32", cores)   # warm-up
    iters = max(1, args.cpu_iters)
    t0 = time.perf_counter()
    for _ in range(iters):
        psi, _ = ref.run_iteration(psi, imgs, ws, k1s, k2s, args.lam, "f32", cores)
    dt = (time.perf_counter() - t0) / iters
    return {"value": round(n ** 3 / dt / 1e6, 3), "unit": "Mvoxels/s per RL iteration",
            "cores": cores, "host_cpus": host_cpus, "cpu_model": cpu_model(), "kind": "port",
            "seconds_per_iteration": round(dt, 2),
            "sample": f"{args.views}-view {n}^3 (bounded sample of the benchmarked workload), {args.ksize}^3 PSF, "
                      f"{args.psftype} lambda={args.lam}; 1 warm-up + {iters} timed iterations "
                      f"(numpy + scipy.fft float32, workers={cores}); stand-in for the Java/ImgLib2 CPU path"}


def engine_classes(geom, wb):
    """(name, bytes per voxel, voxels, bytes per half-spectrum bin) of every timing class,
    and the iteration model.  geom: N (slab voxels), S (half-spectrum bins), nz_int (the
    slab's planes along its internal outermost axis, the one the z pass runs along),
    Mz (its padded length), kplanes (z-planes per stored kernel spectrum)."""
    N, S, nzi, Mz, kp = geom["N"], geom["S"], geom["nz_int"], geom["Mz"], geom["kplanes"]
    kz = 8.0 * kp / Mz
    # z pass: reads all Mz planes, writes only the nz interior planes (the x passes read
    # nothing else back); the inverse y pass transforms those nz planes only, so a y
    # launch moves 16 S (forward) or 16 S nz/Mz (inverse), as many of each
    zw = 8.0 * nzi / Mz
    zb = 8.0 + zw + kz
    yb = 8.0 * (1.0 + nzi / Mz)
    classes = [("x_update", 8 + wb, N, 16), ("x_quotient", wb, N, 16), ("y_pass", 0, 0, yb),
               ("z_convolve", 0, 0, zb), ("x_forward_psi", 4, N, 8), ("halo_exchange", 0, 0, 0),
               ("stats_reduce", 0, 0, 0), ("exchange_window", 0, 0, 0)]
    b_view = (12 + 2 * wb) * N + (32.0 + 4 * yb + 2 * zb) * S
    model = (f"V*((12+2w)N + (32+4y+2z)S) B/iter, S = (Mx/2+1)*My*Mz, w = img/weight bytes, "
             f"y = mean y-pass bytes per bin = {yb:.3f}, "
             f"z = z-pass bytes per bin = {zb:.3f} (8 read + {zw:.3f} write + {kz:.3f} kernel)")
    return classes, b_view, model


def timing_pass(sess, lam, views, slabs_per_group, geom, wb, fp16, backend, ms_per_step):
    """Two timed iterations with HIP events on the session stream around every kernel
    class: per-class launches / average / GB/s, the roofline of the dominant class and
    the whole-iteration roofline."""
    sess.enable_timing(True)
    sess.run(2, lam)
    tm = sess.timing()
    sess.enable_timing(False)
    M = geom["M"]
    if backend == "engine":
        classes, b_view, model = engine_classes(geom, wb)
    else:
        Mlog = M[0] * M[1] * M[2]
        classes = [("update_pad", 8 + wb, geom["N"], 0), ("quotient_pad", wb, geom["N"], 0), ("r2c", 0, 0, 0),
                   ("spec_mul", 0, 0, 0), ("c2r", 0, 0, 0), ("halo_exchange", 0, 0, 0),
                   ("stats_reduce", 0, 0, 0)]
        b_view = (12 + 2 * wb) * geom["N"] + 56.0 * Mlog
        model = "V*((12+2w)N + 56M) B/iter (rocFFT passes counted as 56M)"
    S = geom["S"]
    kernel_ms = {}
    best = None
    for i, (nm, bvox, nv, bspec) in enumerate(classes):
        cnt = int(tm[8 + i])
        if not cnt:
            continue
        if nm == "y_pass" and backend == "engine":
            # with a halo exchange the forward y pass runs as plane ranges around the
            # exchange wait (3 launches): count whole-volume passes, 4 per view and slab
            cnt = min(cnt, 4 * views * 2 * max(1, slabs_per_group))
        if nm in ("x_update", "x_quotient") and backend == "engine":
            # overlapped exchanges split an x pass into the boundary pairs and the rest
            # (2 launches): count whole-slab passes, 1 per view and slab
            cnt = min(cnt, views * 2 * max(1, slabs_per_group))
        avg = tm[i] / cnt
        ent = {"total_ms": round(tm[i], 4), "launches": cnt, "avg_ms": round(avg, 5)}
        byts = bvox * nv + bspec * S
        if byts:
            ent["algorithmic_bytes"] = int(byts)
            ent["GBps"] = round(byts / (avg * 1e-3) / 1e9, 1)
            if best is None or tm[i] > best[1]:
                best = (nm, tm[i], byts, avg)
        kernel_ms[nm] = ent
    # SURVEY 8d's pointwise target: (20 + 2w) B per voxel and view (quotient: blurred, img,
    # write; update: psi, integral, weight, write) over the two x-tile launches of a view
    pointwise = None
    if backend == "engine" and "x_quotient" in kernel_ms and "x_update" in kernel_ms:
        tq, tu = kernel_ms["x_quotient"]["avg_ms"], kernel_ms["x_update"]["avg_ms"]
        pb = (20 + 2 * wb) * geom["N"]
        pointwise = {"bytes_per_view": int(pb), "t_quotient_ms": tq, "t_update_ms": tu,
                     "achieved": round(pb / ((tq + tu) * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(pb / ((tq + tu) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "model": f"({20 + 2 * wb}*N) / (t_quotient + t_update), N = slab voxels"}
    roofline = None
    if best is not None:
        nm, _, byts, avg = best
        achieved = byts / (avg * 1e-3) / 1e9
        traffic, tsrc = pmc_traffic(nm, M, fp16, backend)
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "kernel": nm, "algorithmic_bytes_per_launch": int(byts),
                    "avg_launch_ms": round(avg, 5)}
        if tsrc:
            roofline["traffic_source"] = tsrc
    # every slab of the session moves b_view bytes per view (geom is slab 0's)
    b_iter = views * b_view * geom["nslabs"]
    t_iter = ms_per_step * 1e-3
    it_roof = {"achieved": round(b_iter / t_iter / 1e9, 1), "peak": HBM_PEAK_GBS * geom["ngpus"],
               "unit": "GB/s", "frac": round(b_iter / t_iter / 1e9 / (HBM_PEAK_GBS * geom["ngpus"]), 4),
               "model": model, "M": list(M)}
    return roofline, kernel_ms, it_roof, pointwise


def slab_geom(sess, nslabs, ngpus):
    """Slab 0's geometry in the session's INTERNAL order (a y-split session keeps its
    rows as (x, z, y-slab): fft_dims and the z pass run along the slab axis)."""
    M = sess.fft_dims(0)
    ext = sess.slab_extent(0)              # internal (x, y, z) voxels of slab 0
    return {"M": M, "N": ext[0] * ext[1] * ext[2], "S": (M[0] // 2 + 1) * M[1] * M[2],
            "nz_int": ext[2], "Mz": M[2], "kplanes": sess.kernel_planes(0), "nslabs": nslabs, "ngpus": ngpus}


def legacy_line(args, rank, world, local, dist, broadcast_comm_id, barrier, max_over_ranks, edge=512, iters=3):
    """LucyRichardsonMultiViewDeconvolution (:24-358) through lrsim_*: V = world views of
    edge^3 (view v on rank v % world, generated from its own seed on the rank that owns it),
    25^3 PSFs, additive rule, lambda 0.006; Mvoxels/s of the volume per iteration, max over
    ranks, after one warm-up iteration."""
    import ctypes as C

    import numpy as np
    import torch

    from spim_registration_amd import _lib, synthetic
    lib = _lib.load()
    V = max(1, world)
    os.environ.setdefault("SPIMDECON_RCCL_TIMEOUT", "120")   # (read when the session is created)
    comm_id = broadcast_comm_id(dist, rank) if world > 1 else None
    d = (C.c_int64 * 3)(edge, edge, edge)
    h = C.c_void_p()
    cid = None if comm_id is None else C.create_string_buffer(bytes(comm_id), 128)
    _lib.check(lib.lrsim_create(d, local, world, rank, cid, C.byref(h)))
    keep = []
    try:
        kd = np.array([25, 25, 25], np.int32)
        for v in range(V):
            k = synthetic.psf(v, V, (25, 25, 25))
            keep.append(k)
            if v % world == rank:
                g = torch.Generator(device=f"cuda:{local}").manual_seed(1000 + v)
                img = torch.rand((edge,) * 3, device=f"cuda:{local}", generator=g) + 0.1
                w = torch.rand((edge,) * 3, device=f"cuda:{local}", generator=g)
                torch.cuda.synchronize()
                _lib.check(lib.lrsim_add_view(h, img.data_ptr(), w.data_ptr(), k.ctypes.data,
                                              kd.ctypes.data_as(_lib._pi)))
                del img, w
            else:
                _lib.check(lib.lrsim_add_view(h, None, None, None, kd.ctypes.data_as(_lib._pi)))
        _lib.check(lib.lrsim_init(h, None))
        _lib.check(lib.lrsim_run(h, 1, 0, 0.006, None))
        barrier()
        t0 = time.perf_counter()
        _lib.check(lib.lrsim_run(h, iters, 0, 0.006, None))
        t = time.perf_counter() - t0
        barrier()
        t = max_over_ranks(t)
    finally:
        lib.lrsim_destroy(h)
    return {"workload": f"{V}-view {edge}^3 (one view per GPU), 25^3 PSF, additive rule, lambda=0.006: "
                        "LucyRichardsonMultiViewDeconvolution via lrsim_* (opt-in; not the headline rule)",
            "value": round(edge ** 3 * iters / t / 1e6, 1), "unit": "Mvoxels/s per iteration",
            "ms_per_step": round(t / iters * 1e3, 3), "views": V, "ranks": world,
            "allreduce": ("ncclAllReduce (sum) of 8 B per voxel per iteration" if world > 1 else
                          "none (one rank)")}


def main(argv=None):
    args = parse(argv)
    import torch
    import torch.distributed as dist

    mode, N = plan_gpus(args, os.environ, torch.cuda.device_count())
    from spim_registration_amd import synthetic
    from spim_registration_amd.decon import PSFTYPE, Session
    from spim_registration_amd.distributed import (broadcast_comm_id, env_rank, rank_plan, slab_range,
                                                   verify_rank_plans)

    if mode == "ranks":
        rank, world, local = env_rank()
        devices = [local]
    else:
        rank, world, local = 0, 1, 0
        devices = list(range(N))
    torch.cuda.set_device(local)
    if world > 1:
        # control plane only; a rank that never arrives fails the others within 10 minutes
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(t):
        if world > 1:
            tt = torch.tensor([t], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt)
        return t

    def build_case(shape_xyz, strong):
        """Views of this process (the whole global volume in device-group mode, this
        rank's slab under a launcher) and the session arguments."""
        nx, ny, nz = shape_xyz
        axis = "z"
        ny_g = ny
        if strong:   # the global volume is fixed; split along the longer of y and z
            nz_g = nz
            # (1024x1024x512: 128 + 24 halo rows per GPU, not 64 + 24 planes; local slabs
            # emulate the same decomposition on one GPU)
            if ny > nz and (N > 1 or args.local_slabs > 1):
                axis = "y"
            if mode == "ranks":
                o0, o1 = slab_range(ny_g if axis == "y" else nz_g, world, rank)
                if axis == "y":
                    ny = o1 - o0
                else:
                    nz = o1 - o0
            else:
                o0 = 0
        else:        # weak scaling: every GPU adds an nz-plane slab
            nz_g = nz * N
            o0 = rank * nz
            if mode == "devices":
                nz = nz_g
            if args.slab_axis != "auto":
                if N > 1 and args.slab_axis != "z":
                    raise SystemExit("--slab-axis y stacks nothing: one GPU, or --strong")
                axis = args.slab_axis
        imgs, ws, psfs = synthetic.make_views_torch((nz, ny, nx), args.views,
                                                    config_id=(2 if strong else 1) + rank,
                                                    ksize=(args.ksize,) * 3, device=f"cuda:{local}")
        torch.cuda.synchronize()
        kw = dict(slab_axis=axis, storage_fp16=args.fp16, local_slabs=args.local_slabs,
                  fft_backend=args.backend, fft_pad_policy=args.pad_policy)
        if mode == "ranks":
            kw.update(device=local, nranks=world, rank=rank, nz_global=ny_g if axis == "y" else nz_g,
                      z_offset=o0)
        else:
            kw.update(devices=devices)
        return (nx, ny, nz), (nx, ny_g, nz_g), axis, imgs, ws, psfs, kw

    def make_session(dims, kw, imgs, ws, psfs, psftype):
        # a fresh RCCL id per communicator (an id bootstraps one communicator only)
        comm_id = broadcast_comm_id(dist, rank) if world > 1 else None
        s = Session(dims, comm_id=comm_id, **kw)
        for i, w, k in zip(imgs, ws, psfs):
            s.add_view_device(i.data_ptr(), w.data_ptr(), k)
        s.init(PSFTYPE[psftype])
        if world > 1:   # every rank's exchange plan, before the first exchange (no mismatched RCCL waits)
            verify_rank_plans(dist, rank_plan(s, rank, world))
        s.init_psi()
        return s

    def timed(s, lam, steps, warmup):
        """W warm-up iterations (untimed), then K iterations between barriers and
        device syncs (every GPU of the session: Session.run returns after all of its
        device groups finished); the max over ranks."""
        if warmup:
            s.run(warmup, lam)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.run(steps, lam)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        barrier()
        return max_over_ranks(t)

    def placement(s):
        """devices, slabs and the engine pass each slab ran (fast: x pass 2, z pass 3);
        a run outside the fast passes is refused unless --allow-fallback."""
        ns = s.num_slabs()
        out = {"num_devices": s.num_devices(), "slabs": ns,
               "slab_devices": [s.slab_device(i) for i in range(ns)]}
        if args.backend == "engine":
            out["xpass_modes"] = sorted({s.xpass_mode(i) for i in range(ns)})
            out["zpass_modes"] = sorted({s.zpass_mode(i) for i in range(ns)})
            fast = out["xpass_modes"] == [2] and out["zpass_modes"] == [3]
            if not fast and not args.allow_fallback:
                raise SystemExit(f"engine fallback (x pass {out['xpass_modes']}, z pass {out['zpass_modes']}): "
                                 "refusing to report it; --allow-fallback to measure anyway")
        return out

    wb = 2 if args.fp16 else 4

    def measure(s, dims_g, lam, steps, warmup, want_timing):
        t = timed(s, lam, steps, warmup)
        out = {"value": round(dims_g[0] * dims_g[1] * dims_g[2] * steps / t / 1e6, 2),
               "ms_per_step": round(t / max(steps, 1) * 1e3, 3)}
        if want_timing and not args.no_timing:
            geom = slab_geom(s, s.num_slabs(), s.num_devices())
            out["roofline"], out["kernel_ms"], out["roofline_iteration"], out["pointwise"] = timing_pass(
                s, lam, args.views, geom["nslabs"] // geom["ngpus"], geom, wb, args.fp16, args.backend,
                out["ms_per_step"])
        return out

    # ---- headline (weak, or --strong) and the reference-default mode on the same views
    shape = args.shape if args.shape else (args.size,) * 3
    dims, dims_g, axis, imgs, ws, psfs, kw = build_case(shape, args.strong)
    default_mode = None
    if not args.no_default_mode and not (args.psftype == "OPTIMIZATION_I" and args.lam == 0.006):
        with make_session(dims, kw, imgs, ws, psfs, "OPTIMIZATION_I") as s2:
            default_mode = {"psftype": "OPTIMIZATION_I", "lambda": 0.006,
                            **measure(s2, dims_g, 0.006, args.steps, args.warmup, True)}
        torch.cuda.empty_cache()
    sess = make_session(dims, kw, imgs, ws, psfs, args.psftype)
    del imgs, ws
    torch.cuda.empty_cache()
    head = measure(sess, dims_g, args.lam, args.steps, args.warmup, True)
    place = placement(sess)
    M = sess.fft_dims(0)
    sess.close()
    torch.cuda.empty_cache()

    # ---- the strong-scaling line (BASELINE configs[2]) beside the weak headline
    strong = None
    if not args.strong and not args.no_strong_line and not args.fp16 and args.backend == "engine":
        sdims, sdims_g, saxis, simgs, sws, spsfs, skw = build_case((1024, 1024, 512), True)
        with make_session(sdims, skw, simgs, sws, spsfs, "EFFICIENT_BAYESIAN") as s3:
            del simgs, sws
            torch.cuda.empty_cache()
            strong = {"workload": f"{args.views}-view 1024x1024x512 global (BASELINE configs[2]), split into "
                                  f"{s3.num_slabs()} {saxis}-slab(s), {args.ksize}^3 PSF, EFFICIENT_BAYESIAN "
                                  f"lambda=0.006",
                      "scaling": "strong", "steps": args.strong_steps, "warmup": 1,
                      **measure(s3, sdims_g, 0.006, args.strong_steps, 1, False), **placement(s3),
                      "fft_dims_xyz_slab0_internal": list(s3.fft_dims(0))}
        torch.cuda.empty_cache()

    # ---- the opt-in legacy simultaneous update (lrsim_*): one 512^3 view per GPU, the views
    # sharded over the ranks and one all-reduce of a double per voxel per iteration -- on the
    # 8-GPU node the first data-path RCCL all-reduce; reported beside the headline, never as it
    legacy = None
    if not args.no_legacy_line and (mode == "ranks" or N == 1):
        try:
            legacy = legacy_line(args, rank, world, local, dist, broadcast_comm_id, barrier, max_over_ranks)
        except Exception as e:   # (a failure here must not cost the headline line)
            legacy = {"error": repr(e)[:400]}
        torch.cuda.empty_cache()

    cpu = None
    if rank == 0 and N == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        nx, ny_g, nz_g = dims_g
        how = "device groups in one process, xGMI peer halo pulls" if mode == "devices" else "RCCL halo send/recv"
        line = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "Mvoxels/s per RL iteration",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32" + ("(fp16 img/w storage)" if args.fp16 else ""),
            "data": "synthetic (seeded bead stacks generated on the GPU, SURVEY 8d)",
            "config": {"workload": ((f"{args.views}-view {nx}x{ny_g}x{nz_g} global, split into "
                                     f"{place['slabs']} {axis}-slab(s)"
                                     if args.strong else
                                     (f"{args.views}-view {shape[0]}^3" if len(set(shape)) == 1
                                      else f"{args.views}-view {shape[0]}x{shape[1]}x{shape[2]}")
                                     + f" per GPU (global {nx}x{ny_g}x{nz_g})")
                                    + (" (one rank's y-slab of BASELINE configs[4], 2048x2048x1024 over 8 ranks)"
                                       if args.c5_rank else "")
                                    + (" (one rank's y-slab of BASELINE configs[2], 1024x1024x512 over 8 ranks)"
                                       if args.c3_rank else "")
                                    + f", {args.ksize}^3 PSF, RL {args.psftype} lambda={args.lam}"),
                       "views": args.views, "volume_xyz": [nx, ny_g, nz_g], "psf": [args.ksize] * 3,
                       "fft_dims_xyz": list(M), "local_slabs": args.local_slabs,
                       "parallelism": f"{axis}-slab x{place['slabs']} over {N} GPU(s) ({how})",
                       "launch": mode, **place},
            "default_mode": default_mode,
            "roofline": head.get("roofline"),
            "roofline_iteration": head.get("roofline_iteration"),
            "pointwise": head.get("pointwise"),
            "kernel_ms": head.get("kernel_ms"),
            "strong": strong,
            "legacy_simultaneous": legacy,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
