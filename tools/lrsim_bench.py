"""Throughput of the legacy simultaneous-update mode (lrsim_*, include/spimdecon.h section 10)
on one GPU: V views of an nx x ny x nz volume (synthetic, resident in HBM), Gaussian PSFs
of 25^3; prints one JSON line with Mvoxels/s per iteration.

    python tools/lrsim_bench.py --shape 512 512 512 --views 4 --iters 3 [--mult]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spim_registration_amd import _lib, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=3, default=[512, 512, 512], help="nx ny nz")
    ap.add_argument("--views", type=int, default=4)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--mult", action="store_true")
    ap.add_argument("--lam", type=float, default=0.006)
    a = ap.parse_args()
    lib = _lib.load()
    import torch
    nx, ny, nz = a.shape
    g = torch.Generator(device="cuda").manual_seed(7)
    imgs = [torch.rand((nz, ny, nx), device="cuda", generator=g) + 0.1 for _ in range(a.views)]
    ws = [torch.rand((nz, ny, nx), device="cuda", generator=g) for _ in range(a.views)]
    ks = [synthetic.psf(v, a.views, (25, 25, 25)) for v in range(a.views)]
    torch.cuda.synchronize()
    d = (C.c_int64 * 3)(nx, ny, nz)
    h = C.c_void_p()
    _lib.check(lib.lrsim_create(d, 0, 1, 0, None, C.byref(h)))
    try:
        kd = np.array([25, 25, 25], np.int32)
        for v in range(a.views):
            _lib.check(lib.lrsim_add_view(h, imgs[v].data_ptr(), ws[v].data_ptr(), ks[v].ctypes.data,
                                          kd.ctypes.data_as(_lib._pi)))
        t0 = time.perf_counter()
        avg = C.c_double()
        _lib.check(lib.lrsim_init(h, C.byref(avg)))
        t_init = time.perf_counter() - t0
        _lib.check(lib.lrsim_run(h, 1, int(a.mult), a.lam, None))   # warm-up (plans, first touch)
        st = np.zeros(2 * a.iters)
        t0 = time.perf_counter()
        _lib.check(lib.lrsim_run(h, a.iters, int(a.mult), a.lam, st.ctypes.data_as(_lib._pd)))
        dt = (time.perf_counter() - t0) / a.iters
        m = (C.c_int64 * 3)()
        _lib.check(lib.lrsim_fft_dims(h, m))
        n = nx * ny * nz
        print(json.dumps({"metric": "Mvoxels/sec per iteration (legacy simultaneous update)",
                          "value": round(n / dt / 1e6, 1), "ms_per_iter": round(dt * 1e3, 3),
                          "views": a.views, "shape": [nx, ny, nz], "fft": list(m), "mult": a.mult,
                          "init_ms": round(t_init * 1e3, 1), "avg": avg.value,
                          "last_stats": [float(st[-2]), float(st[-1])]}))
    finally:
        lib.lrsim_destroy(h)


if __name__ == "__main__":
    main()
