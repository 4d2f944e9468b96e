"""Two-rank RCCL probe of the z-slab session on ONE GPU box (run under gpurun).

    python tools/rccl_probe.py [--devices 0 0]

Spawns two worker processes (ranks 0 and 1 of a 2-rank RCCL communicator,
torch.distributed/gloo only for the id hand-off), each owning one z-slab of a
small volume, plus a third worker that runs the same RL on the whole volume
with one session.  Compares the gathered psi and the per-view statistics.
The parent never touches the GPU (it only spawns and compares), so no process
that initialised HIP forks or execs.  When RCCL refuses two ranks on one device
the probe reports that and exits 0: the real-RCCL path is then covered only by
the driver's multi-GPU bench.  Not a pytest test for that reason.
"""
from __future__ import annotations

import argparse
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPE = (48, 40, 36)      # z, y, x
KS = (7, 7, 9)            # kx, ky, kz -> cz = 4
ITERS = 3
LAM = 0.006


def _inputs():
    from spim_registration_amd import synthetic
    imgs, ws, psfs, _ = synthetic.make_views(SHAPE, 2, config_id=31, ksize=KS, bead_density=1.0 / 6 ** 3)
    return imgs, ws, psfs


def _run(dims_xyz, imgs, ws, psfs, **kw):
    from spim_registration_amd.decon import PSFTYPE, Session
    with Session(dims_xyz, **kw) as s:
        for i, w, k in zip(imgs, ws, psfs):
            s.add_view(np.ascontiguousarray(i), np.ascontiguousarray(w), k)
        s.init(PSFTYPE.OPTIMIZATION_I)
        s.init_psi()
        st = s.run(ITERS, LAM)
        s.apply_mask()
        return s.get_psi(), np.asarray(st)


def _rank_worker(rank, world, port, dev, q):
    try:
        import torch.distributed as dist
        from spim_registration_amd.distributed import broadcast_comm_id, slab_range
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cid = broadcast_comm_id(dist, rank)
        imgs, ws, psfs = _inputs()
        nz = SHAPE[0]
        z0, z1 = slab_range(nz, world, rank)
        sl = [i[z0:z1] for i in imgs], [w[z0:z1] for w in ws]
        psi, st = _run((SHAPE[2], SHAPE[1], z1 - z0), sl[0], sl[1], psfs, device=dev, nranks=world,
                       rank=rank, comm_id=cid, nz_global=nz, z_offset=z0)
        q.put(("rank", rank, z0, psi, st))
        dist.destroy_process_group()
    except Exception as e:  # reported to the parent
        q.put(("err", rank, repr(e)))


def _whole_worker(dev, q):
    try:
        imgs, ws, psfs = _inputs()
        psi, st = _run((SHAPE[2], SHAPE[1], SHAPE[0]), imgs, ws, psfs, device=dev)
        q.put(("whole", psi, st))
    except Exception as e:
        q.put(("err", "whole", repr(e)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", type=int, nargs=2, default=[0, 0])
    a = ap.parse_args()
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, a.devices[r], q), daemon=True) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    errs = [o for o in out if o[0] == "err"]
    if errs:
        msg = " ".join(str(e) for e in errs)
        if "uplicate" in msg or "invalid usage" in msg.lower():
            print(f"RCCL refused two ranks on one device: {msg}")
            return 0
        print(f"FAIL: {msg}")
        return 1
    w = ctx.Process(target=_whole_worker, args=(a.devices[0], q), daemon=True)
    w.start()
    whole = q.get(timeout=180)
    w.join(timeout=60)
    if whole[0] == "err":
        print(f"FAIL whole-volume run: {whole}")
        return 1
    parts = sorted([o for o in out if o[0] == "rank"], key=lambda o: o[2])
    psi = np.concatenate([o[3] for o in parts])
    err = float(np.linalg.norm(psi - whole[1]) / np.linalg.norm(whole[1]))
    serr = float(np.max(np.abs(parts[0][4] - whole[2]) / np.maximum(np.abs(whole[2]), 1e-30)))
    same_stats = bool(np.allclose(parts[0][4], parts[1][4]))
    print(f"2-rank RCCL z-slabs vs one session: psi rel-L2 {err:.3e}, stats max rel {serr:.3e}, "
          f"ranks agree on stats {same_stats}")
    return 0 if err < 1e-5 and serr < 1e-3 and same_stats else 1


if __name__ == "__main__":
    sys.exit(main())
