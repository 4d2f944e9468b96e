"""One process per GPU: rank bootstrap, z-slab ownership and the RCCL id hand-off.

The volume is split into z-slabs (``mvd_slab_range``, balanced) -- views do
not shard because the RL update is sequential over views
(MVDeconvolution.java:353-441).  Each rank owns one slab (optionally split
further into local virtual slabs); the halo exchange of ``c_z`` padded planes
per convolution and the {sumChange, maxChange} all-reduce run inside
libspimdecon.so over RCCL (xGMI).  torch.distributed is only the control
plane here: it broadcasts the 128-byte RCCL unique id and takes the
max-over-ranks wall time in bench.py.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _lib


def env_rank():
    """(rank, world_size, local_rank) from the torchrun environment (1 process = 1 GPU)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def slab_range(nz: int, parts: int, idx: int):
    """Global [z0, z1) of part ``idx`` (C-ABI ``mvd_slab_range``)."""
    lib = _lib.load()
    z0, z1 = C.c_int64(), C.c_int64()
    _lib.check(lib.mvd_slab_range(int(nz), int(parts), int(idx), C.byref(z0), C.byref(z1)))
    return z0.value, z1.value


def halo_planes_needed(z0: int, z1: int, nz: int, cz: int):
    """Which neighbour planes a slab [z0, z1) receives: (lower [a,b), upper [a,b));
    empty ranges at the global boundary (mirror / constant extension there)."""
    lower = (max(z0 - cz, 0), z0) if z0 > 0 else (z0, z0)
    upper = (z1, min(z1 + cz, nz)) if z1 < nz else (z1, z1)
    return lower, upper


def halo_plan(nz: int, Mz: int, cz: int, plane_elems: int):
    """Float offsets of one slab's halo transfers (C-ABI ``mvd_halo_plan``, the helper
    behind libspimdecon's local copies, device-group pulls and RCCL send / recv):
    dict send_lo, recv_lo, send_hi, recv_hi, count."""
    lib = _lib.load()
    out = (C.c_int64 * 5)()
    _lib.check(lib.mvd_halo_plan(int(nz), int(Mz), int(cz), int(plane_elems), out))
    return dict(zip(("send_lo", "recv_lo", "send_hi", "recv_hi", "count"), list(out)))


def unique_id_bytes() -> bytes:
    """128-byte RCCL unique id created on this process (rank 0)."""
    lib = _lib.load()
    buf = C.create_string_buffer(128)
    _lib.check(lib.mvd_comm_unique_id(buf))
    return buf.raw


def broadcast_comm_id(dist, rank: int, make_id=unique_id_bytes) -> bytes:
    """Rank 0 creates the RCCL id, every rank receives it (torch.distributed
    object broadcast; works on the gloo and nccl backends)."""
    obj = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


# ---- rank-consistency check before the first exchange -------------------------------
# Ranks whose halo sends and receives do not match (another slab geometry, another z-pass
# mode, other views) would post mismatched ncclSend / ncclRecv and wait for each other
# forever.  bench.py all-gathers every rank's plan over the gloo control group after
# mvd_init and refuses to start when they disagree; the library repeats the geometry part
# of the check over RCCL (Session::verify_ranks) for callers without a control group.

def rank_plan(session, rank: int, world: int) -> dict:
    """What this rank will exchange: geometry of its first and last slab, the halo plan
    of each, the z-pass modes, views and storage (JSON-able)."""
    p = session.params
    ns = session.num_slabs()
    slabs = []
    for s in sorted({0, ns - 1}):
        Mx, My, Mz = session.fft_dims(s)
        nx, ny, nz = session.slab_extent(s)
        kp = session.kernel_planes(s)
        hp = -(-(Mx // 2 + 1) // 16) * 16              # engine x-spectrum row (complex, padded)
        plane = 2 * hp * My
        cz = (kp - 1) // 2 if kp < Mz else (Mz - nz) // 2
        slabs.append({"fft_dims": [Mx, My, Mz], "extent": [nx, ny, nz], "kernel_planes": kp,
                      "zpass_mode": session.zpass_mode(s), "halo": halo_plan(nz, Mz, cz, plane) if nz >= cz else None})
    ext = sum(session.slab_extent(s)[2] for s in range(ns))
    return {"rank": int(rank), "world": int(world), "nranks": int(p.nranks), "nviews": int(session.nviews),
            "storage_fp16": int(p.storage_fp16), "fft_backend": int(p.fft_backend), "slab_axis": int(p.slab_axis),
            "nz_global": int(p.nz_global), "z_offset": int(p.z_offset), "extent": int(ext),
            "zpass_modes": sorted({session.zpass_mode(s) for s in range(ns)}), "slabs": slabs}


def check_rank_plans(plans) -> list:
    """Disagreements between the ranks' plans (empty = consistent).  Pure function of
    the gathered plans, so every rank reaches the same verdict."""
    errs = []
    if not plans:
        return ["no plans"]
    world = len(plans)
    same = ("world", "nranks", "nviews", "storage_fp16", "fft_backend", "slab_axis", "nz_global", "zpass_modes")
    for r, q in enumerate(plans):
        if q.get("rank") != r:
            errs.append(f"plan {r} comes from rank {q.get('rank')}")
        for k in same:
            if q.get(k) != plans[0].get(k):
                errs.append(f"{k}: rank {r} has {q.get(k)}, rank 0 has {plans[0].get(k)}")
        if q.get("world") != world:
            errs.append(f"rank {r} believes world = {q.get('world')}, {world} plans gathered")
    if errs:
        return errs
    if plans[0]["z_offset"] != 0:
        errs.append(f"rank 0 starts at {plans[0]['z_offset']}, not 0")
    if plans[-1]["z_offset"] + plans[-1]["extent"] != plans[-1]["nz_global"]:
        errs.append(f"the last rank ends at {plans[-1]['z_offset'] + plans[-1]['extent']}, "
                    f"not nz_global = {plans[-1]['nz_global']}")
    for r in range(world - 1):
        lo, hi = plans[r], plans[r + 1]
        if lo["z_offset"] + lo["extent"] != hi["z_offset"]:
            errs.append(f"rank {r} owns [{lo['z_offset']}, {lo['z_offset'] + lo['extent']}) but rank {r + 1} "
                        f"starts at {hi['z_offset']}")
        a, b = lo["slabs"][-1], hi["slabs"][0]            # the two slabs that exchange
        if a["fft_dims"][:2] != b["fft_dims"][:2]:
            errs.append(f"ranks {r}/{r + 1}: x-y spectrum planes {a['fft_dims'][:2]} vs {b['fft_dims'][:2]}")
        if a["kernel_planes"] != b["kernel_planes"] and min(a["kernel_planes"], b["kernel_planes"]) < min(
                a["fft_dims"][2], b["fft_dims"][2]):
            errs.append(f"ranks {r}/{r + 1}: kernel planes {a['kernel_planes']} vs {b['kernel_planes']}")
        ha, hb = a["halo"], b["halo"]
        if ha is None or hb is None or ha["count"] != hb["count"]:
            errs.append(f"ranks {r}/{r + 1}: halo transfer of {ha and ha['count']} vs {hb and hb['count']} floats")
    return errs


def verify_rank_plans(dist, plan: dict) -> list:
    """All-gathers ``plan`` over the (gloo) control group and raises RuntimeError on every
    rank when the plans disagree; returns the gathered plans."""
    world = dist.get_world_size()
    plans = [None] * world
    dist.all_gather_object(plans, plan)
    errs = check_rank_plans(plans)
    if errs:
        raise RuntimeError("ranks disagree on the halo exchange, refusing to start: " + "; ".join(errs[:6]))
    return plans
