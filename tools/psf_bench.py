"""PSF extraction stage of the C4 pipeline in isolation: 8 device-resident 768^3 views,
~1,500 bead locations each, 19x19x25 PSFs transformed by a rotation about y
(spim_extract_psfs).  Prints per-call wall times and, with --profile-host, where the host
time of one call goes (Python-side preparation vs the library call).

    python tools/psf_bench.py [--size 768] [--views 8] [--beads 1500] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=768)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--beads", type=int, default=1500)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from spim_registration_amd import psf as psf_mod
    n, V = a.size, a.views
    g = torch.Generator(device="cuda").manual_seed(7)
    views = [torch.rand((n, n, n), device="cuda", generator=g) for _ in range(V)]
    rng = np.random.default_rng(3)
    beads = [rng.uniform(20, n - 20, size=(a.beads, 3)) for _ in range(V)]
    models = []
    for v in range(V):
        th = 2 * math.pi * v / V
        c, s = math.cos(th), math.sin(th)
        models.append(np.array([[c, 0, s, 0], [0, 1, 0, 0], [-s, 0, c, 0]], np.float64))
    out = []
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        psf_mod.extract_psfs(views, beads, (19, 19, 25), models)
        torch.cuda.synchronize()
        out.append(round((time.perf_counter() - t0) * 1e3, 2))
    print(json.dumps({"workload": f"{V} views {n}^3, {a.beads} beads each, 19x19x25 PSFs",
                      "ms_per_call": out}))


if __name__ == "__main__":
    main()
