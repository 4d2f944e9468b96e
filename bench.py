#!/usr/bin/env python3
"""Benchmark: Mvoxels/s per RL iteration of the multiview deconvolution path.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric: "6-view 512^3 deconv"; configs[1] geometry and
RL settings): 6-view 512^3 synthetic PSF-blurred bead volume, 25^3 PSFs,
multiview RL (PSFTYPE INDEPENDENT, lambda 0) -- one *step*
= one full RL iteration (all views, sequential per-view updates) over the
volume, inputs resident in HBM.  With N ranks each GPU holds a 512^3 z-slab of
a 512x512x(512N) volume (weak scaling); the slabs exchange 12-plane halos over
RCCL before every convolution.  value = all ranks' voxels * steps / max-rank
time / 1e6.

Also reported: ``roofline`` of the dominant engine pass (largest total time;
algorithmic bytes per launch in DESIGN.md "Kernels") timed with HIP events on
the session's stream, ``roofline_iteration`` (whole iteration against the
engine's compulsory traffic), and ``cpu_baseline`` = the oracle's float32 scipy.fft
restatement of the same iteration on a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mvoxels/sec per RL iter, 6-view 512\u00b3 deconv; 1/2/4/8-GPU scaling"  # BASELINE.json
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--views", type=int, default=6)
    ap.add_argument("--size", type=int, default=512, help="per-GPU cube edge")
    ap.add_argument("--shape", type=int, nargs=3, metavar=("X", "Y", "Z"),
                    help="per-GPU slab x y z (overrides --size; z-slabs stack over ranks)")
    ap.add_argument("--ksize", type=int, default=25)
    ap.add_argument("--psftype", default="INDEPENDENT")
    ap.add_argument("--lam", type=float, default=0.0)
    ap.add_argument("--fp16", action="store_true", help="fp16 img/weight storage")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-size", type=int, default=256, help="edge of the CPU-baseline sample")
    ap.add_argument("--no-timing", action="store_true", help="skip the HIP-event roofline pass")
    ap.add_argument("--backend", default="engine", choices=["engine", "rocfft"])
    ap.add_argument("--pad-policy", default="auto", choices=["auto", "fast", "smooth"])
    ap.add_argument("--local-slabs", type=int, default=1, help="z-slabs per process (virtual shards)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the global volume --shape (default 1024 1024 512, EFFICIENT_BAYESIAN "
                         "lambda 0.006 = BASELINE configs[2]) is split into N slabs along the longer of y and z, one per rank")
    ap.add_argument("--no-default-mode", action="store_true",
                    help="skip the second measurement in the reference default mode (OPTIMIZATION_I, 0.006)")
    a = ap.parse_args()
    if a.strong and a.shape is None:
        a.shape = [1024, 1024, 512]
        if a.psftype == "INDEPENDENT" and a.lam == 0.0:
            a.psftype, a.lam = "EFFICIENT_BAYESIAN", 0.006
    return a


# engine kernel class -> kernel-name prefixes in the PMC table (tools/pmc_summary.py --json)
PMC_KERNELS = {"z_convolve": ("k_zdmc<", "k_zdma<", "k_zdirect<", "k_col2f<2,", "k_colpass<2,"), "y_pass": ("k_col2f<1,", "k_colpass<1,"),
               "x_update": ("k_xtile<2,", "k_xrows<2,", "k_xpass<2,"),
               "x_quotient": ("k_xtile<1,", "k_xrows<1,", "k_xpass<1,")}


def pmc_traffic(cls, M, args):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes
    (profiles/pmc_traffic.json, same FFT dims and storage), or (None, None)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if args.backend != "engine" or not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    if list(d.get("fft_dims", [])) != list(M) or bool(d.get("fp16", False)) != bool(args.fp16):
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


def cpu_baseline(args, shape_xyz):
    """The oracle (numpy + scipy.fft float32, multithreaded) on the SAME workload as
    the GPU line (V views of the benchmarked volume, same PSFs): one RL iteration,
    timed from an initialised psi.  Threads: the box's CPU share (OMP_NUM_THREADS,
    16 per GPU on the MI355X pool; os.cpu_count() elsewhere) -- reported as `cores`
    next to the host's logical CPU count and model."""
    from oracle import mvdecon_ref as ref
    from spim_registration_amd import synthetic

    nx, ny, nz = shape_xyz
    if args.cpu_size != 256:          # explicit smaller sample (cube of --cpu-size)
        nx = ny = nz = args.cpu_size
    host_cpus = os.cpu_count() or 1
    cores = int(os.environ.get("OMP_NUM_THREADS", host_cpus))
    imgs, ws, psfs, _ = synthetic.make_views((nz, ny, nx), args.views, config_id=1,
                                             ksize=(args.ksize,) * 3, weights="blend")
    k1s, k2s = ref.prepare_kernels(psfs, ref.PSFTYPE[args.psftype], 8)
    _, avg = ref.first_iteration(imgs)
    psi = np.full(imgs[0].shape, np.float32(avg), np.float32)
    t0 = time.perf_counter()
    psi, _ = ref.run_iteration(psi, imgs, ws, k1s, k2s, args.lam, "f32", cores)
    dt = time.perf_counter() - t0
    return {"value": round(nx * ny * nz / dt / 1e6, 3), "unit": "Mvoxels/s per RL iteration",
            "cores": cores, "host_cpus": host_cpus, "cpu_model": cpu_model(), "kind": "port",
            "seconds": round(dt, 2),
            "sample": f"{args.views}-view {nx}x{ny}x{nz} (the benchmarked volume), {args.ksize}^3 PSF, "
                      f"{args.psftype} lambda={args.lam}, 1 timed iteration (numpy + scipy.fft float32, "
                      f"workers={cores}); stand-in for the Java/ImgLib2 CPU path"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from spim_registration_amd import synthetic
    from spim_registration_amd.decon import PSFTYPE, Session
    from spim_registration_amd.distributed import broadcast_comm_id, env_rank

    rank, world, local = env_rank()
    if world != args.gpus and "RANK" in os.environ:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)   # control plane only

    nx, ny, nz = args.shape if args.shape else (args.size,) * 3
    V = args.views
    axis = "z"
    ny_g = ny
    if args.strong:      # the global volume is fixed; rank r owns slab r of N along the longer of y, z
        from spim_registration_amd.distributed import slab_range
        nz_g = nz
        if ny > nz and (world > 1 or args.local_slabs > 1):   # (1024x1024x512: 128 + 24 halo rows per rank, not 64 + 24 planes)
            axis = "y"
            o0, o1 = slab_range(ny_g, world, rank)
            ny = o1 - o0
        else:
            o0, o1 = slab_range(nz_g, world, rank)
            nz = o1 - o0
    else:                # weak scaling: every rank adds an nz-plane slab
        nz_g = nz * world
        o0 = rank * nz
    imgs, ws, psfs = synthetic.make_views_torch((nz, ny, nx), V, config_id=1 + rank,
                                                ksize=(args.ksize,) * 3, device=f"cuda:{local}")
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    def make_session(psftype):
        # a fresh RCCL id per communicator (an id bootstraps one communicator only)
        comm_id = broadcast_comm_id(dist, rank) if world > 1 else None
        s = Session((nx, ny, nz), device=local, nranks=world, rank=rank, comm_id=comm_id,
                    nz_global=ny_g if axis == "y" else nz_g, z_offset=o0, slab_axis=axis,
                    storage_fp16=args.fp16, local_slabs=args.local_slabs,
                    fft_backend=args.backend, fft_pad_policy=args.pad_policy)
        for i, w, k in zip(imgs, ws, psfs):
            s.add_view_device(i.data_ptr(), w.data_ptr(), k)
        s.init(PSFTYPE[psftype])
        s.init_psi()
        return s

    def timed(s, lam):
        """W warm-up iterations (untimed), then K iterations between barriers and
        device syncs; the max over ranks."""
        if args.warmup:
            s.run(args.warmup, lam)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.run(args.steps, lam)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        barrier()
        if world > 1:
            tt = torch.tensor([t], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt)
        return t

    # the reference's default mode (EfficientBayesianBased.java:83,89), measured on the same
    # views after the primary line's mode unless that already is the default
    default_mode = None
    if not args.no_default_mode and not (args.psftype == "OPTIMIZATION_I" and args.lam == 0.006):
        with make_session("OPTIMIZATION_I") as s2:
            t2 = timed(s2, 0.006)
        default_mode = {"psftype": "OPTIMIZATION_I", "lambda": 0.006,
                        "value": round(nx * ny_g * nz_g * args.steps / t2 / 1e6, 2),
                        "ms_per_step": round(t2 / max(args.steps, 1) * 1e3, 3)}
        torch.cuda.empty_cache()
    sess = make_session(args.psftype)
    del imgs, ws
    torch.cuda.empty_cache()
    M = sess.fft_dims(0)
    dt = timed(sess, args.lam)
    ms_per_step = dt / max(args.steps, 1) * 1e3
    n_vox_total = nx * ny_g * nz_g
    value = n_vox_total * args.steps / dt / 1e6

    # roofline pass: HIP events on the session stream around every kernel class
    roofline = None
    kernel_ms = None
    it_roof = None
    if not args.no_timing:
        sess.enable_timing(True)
        sess.run(2, args.lam)
        tm = sess.timing()
        sess.enable_timing(False)
        N = nx * ny * nz
        Mlog = M[0] * M[1] * M[2]
        S = (M[0] // 2 + 1) * M[1] * M[2]   # half-spectrum elements (algorithmic, unpadded)
        wb = 2 if args.fp16 else 4          # bytes per img / weight voxel
        if args.backend == "engine":
            # algorithmic HBM bytes per launch of each fused pass (DESIGN.md "kernels"); the
            # z pass reads its kernel's stored z-planes: 2cz+1 of Mz when compact
            kz = 8.0 * sess.kernel_planes(0) / M[2]
            # z pass: reads all Mz planes, writes only the nz interior planes (the x passes
            # read nothing else back); the inverse y pass transforms those nz planes only,
            # so a y launch moves 16 S (forward) or 16 S nz/Mz (inverse), as many of each
            zw = 8.0 * nz / M[2]
            zb = 8.0 + zw + kz
            yb = 8.0 * (1.0 + nz / M[2])
            classes = [("x_update", 8 + wb, N, 16), ("x_quotient", wb, N, 16), ("y_pass", 0, 0, yb),
                       ("z_convolve", 0, 0, zb), ("x_forward_psi", 4, N, 8), ("halo_exchange", 0, 0, 0),
                       ("stats_reduce", 0, 0, 0), ("yzy_banded", 0, 0, 16 + kz)]
            b_iter = V * ((12 + 2 * wb) * N + (32.0 + 4 * yb + 2 * zb) * S)
            model = (f"V*((12+2w)N + (32+4y+2z)S) B/iter, S = (Mx/2+1)*My*Mz, w = img/weight bytes, "
                     f"y = mean y-pass bytes per bin = {yb:.3f}, "
                     f"z = z-pass bytes per bin = {zb:.3f} (8 read + {zw:.3f} write + {kz:.3f} kernel)")
        else:
            classes = [("update_pad", 8 + wb, N, 0), ("quotient_pad", wb, N, 0), ("r2c", 0, 0, 0),
                       ("spec_mul", 0, 0, 0), ("c2r", 0, 0, 0), ("halo_exchange", 0, 0, 0),
                       ("stats_reduce", 0, 0, 0)]
            b_iter = V * ((12 + 2 * wb) * N + 56.0 * Mlog)
            model = "V*((12+2w)N + 56M) B/iter (rocFFT passes counted as 56M)"
        kernel_ms = {}
        best = None
        for i, (nm, bvox, nv, bspec) in enumerate(classes):
            cnt = int(tm[8 + i])
            if not cnt:
                continue
            if nm == "y_pass" and args.backend == "engine":
                # with a halo exchange the forward y pass runs as plane ranges around the
                # exchange wait (3 launches): count whole-volume passes, 4 per view and slab
                cnt = min(cnt, 4 * V * 2 * max(1, args.local_slabs))
            avg = tm[i] / cnt
            ent = {"total_ms": round(tm[i], 4), "launches": cnt, "avg_ms": round(avg, 5)}
            byts = bvox * nv + bspec * S
            if byts:
                ent["algorithmic_bytes"] = int(byts)
                ent["GBps"] = round(byts / (avg * 1e-3) / 1e9, 1)
                if best is None or tm[i] > best[1]:
                    best = (nm, tm[i], byts, avg)
            kernel_ms[nm] = ent
        if best is not None:
            nm, _, byts, avg = best
            achieved = byts / (avg * 1e-3) / 1e9
            traffic, tsrc = pmc_traffic(nm, M, args)
            roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "kernel": nm, "algorithmic_bytes_per_launch": int(byts),
                        "avg_launch_ms": round(avg, 5)}
            if tsrc:
                roofline["traffic_source"] = tsrc
        t_iter = ms_per_step * 1e-3
        it_roof = {"achieved": round(b_iter / t_iter / 1e9, 1), "peak": HBM_PEAK_GBS,
                   "unit": "GB/s", "frac": round(b_iter / t_iter / 1e9 / HBM_PEAK_GBS, 4),
                   "model": model, "M": list(M)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, (nx, ny_g, nz_g))

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mvoxels/s per RL iteration",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32" + ("(fp16 img/w storage)" if args.fp16 else ""),
            "data": "synthetic (seeded bead stacks generated on the GPU, SURVEY 8d)",
            "config": {"workload": ((f"{V}-view {nx}x{ny_g}x{nz_g} global, split into {world} {axis}-slabs"
                                    if args.strong else
                                    (f"{V}-view {nx}^3" if nx == ny == nz else f"{V}-view {nx}x{ny}x{nz}")
                                    + f" per GPU (global {nx}x{ny_g}x{nz_g})")
                                   + f", {args.ksize}^3 PSF, RL {args.psftype} lambda={args.lam}"),
                       "views": V, "volume_xyz": [nx, ny_g, nz_g], "psf": [args.ksize] * 3,
                       "fft_dims_xyz": list(M), "local_slabs": args.local_slabs,
                       "parallelism": f"{axis}-slab x{world} (RCCL halo)"},
            "default_mode": default_mode,
            "roofline": roofline,
            "roofline_iteration": it_roof,
            "kernel_ms": kernel_ms,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    sess.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
