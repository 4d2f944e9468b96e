"""DoG bead detection throughput (SURVEY 8 config C4 detection step): one view of
768^3 synthetic beads through spim_dog_interest_points (ProcessDOG.compute with
the reference defaults: sigma 1.8, threshold 0.008, quadratic localisation).

    python tools/dog_bench.py [--size 768] [--reps 3]

The reference hands ImgLib2 (host) arrays to the native library, so the first
number includes the host->device upload of the view; the same C-ABI call also
takes a device pointer, and the second number is a view already resident in HBM
(a torch tensor).  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def beads(n: int, count: int, seed: int = 20140611) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = np.full((n, n, n), 0.02, np.float32)
    pos = rng.integers(3, n - 3, size=(count, 3))
    amp = rng.uniform(0.5, 1.0, size=count).astype(np.float32)
    # 3x3x3 blobs so every bead survives the DoG as one extremum
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                w = np.float32(np.exp(-0.9 * (dx * dx + dy * dy + dz * dz)))
                np.add.at(img, (pos[:, 0] + dz, pos[:, 1] + dy, pos[:, 2] + dx), amp * w)
    return img


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=768)
    ap.add_argument("--beads", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--device-only", action="store_true", help="skip the host-view calls")
    a = ap.parse_args()
    import torch  # before the library loads: one shared HIP runtime (_lib.load)
    import ctypes as C
    from spim_registration_amd import _lib, dog
    img = beads(a.size, a.beads)
    dog.compute(img[:64, :64, :64].copy(), localization=1)  # warm-up (module load, kernels)
    ts, td = [], []
    pts = dog.compute(img, localization=1) if a.device_only else []
    for _ in range(0 if a.device_only else a.reps):
        t0 = time.perf_counter()
        pts = dog.compute(img, localization=1)
        ts.append(time.perf_counter() - t0)
    for _ in range(0 if a.device_only else a.reps):
        t0 = time.perf_counter()
        dog.compute(img, localization=1, return_dog=True)
        td.append(time.perf_counter() - t0)
    # device-resident view: the same entry point with a device pointer
    lib = _lib.load()
    dimg = torch.from_numpy(img).to("cuda:0")
    p = _lib.DogParams()
    lib.spim_dog_params_default(C.byref(p))
    p.localization = 1
    dims = (C.c_int64 * 3)(img.shape[2], img.shape[1], img.shape[0])
    cap = max(1024, len(pts) * 2)
    out = (_lib.InterestPointC * cap)()
    nout = C.c_int64(0)
    tdev = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check(lib.spim_dog_interest_points(C.cast(C.c_void_p(dimg.data_ptr()), C.POINTER(C.c_float)),
                                                dims, C.byref(p), None, out, cap, C.byref(nout)))
        tdev.append(time.perf_counter() - t0)
    if not os.environ.get("SPIMDECON_BENCH_NOCHECK"):   # (experiment builds with wrong values)
        assert int(nout.value) == len(pts), (int(nout.value), len(pts))
    n = img.size
    med = lambda v: float(np.median(v)) if v else float("nan")
    t, t2, t3 = med(ts), med(td), med(tdev)
    print(json.dumps({
        "workload": f"DoG bead detection, one {a.size}^3 view, {a.beads} synthetic beads, sigma 1.8, "
                    "threshold 0.008, quadratic localisation (ProcessDOG defaults)",
        "interest_points": len(pts),
        "ms": round(t * 1e3, 2), "Mvoxels_per_s": round(n / t / 1e6, 1),
        "ms_with_dog_image": round(t2 * 1e3, 2),
        "ms_device_resident": round(t3 * 1e3, 2), "Mvoxels_per_s_device_resident": round(n / t3 / 1e6, 1),
        "note": "ms: host view in (PCIe upload included); ms_device_resident: the view already in HBM",
    }), flush=True)


if __name__ == "__main__":
    main()
