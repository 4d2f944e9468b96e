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
