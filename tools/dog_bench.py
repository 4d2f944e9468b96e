"""DoG bead detection throughput (SURVEY 8 config C4 detection step): one view of
768^3 synthetic beads through spim_dog_interest_points (ProcessDOG.compute with
the reference defaults: sigma 1.8, threshold 0.008, quadratic localisation).

    python tools/dog_bench.py [--size 768] [--reps 3]

The C-ABI takes host buffers (the reference hands ImgLib2 arrays to the native
library), so the time includes the host->device upload of the view and the
download of the peaks; a second number is the same call with the DoG image
also downloaded.  Prints one JSON line.
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
    a = ap.parse_args()
    from spim_registration_amd import dog
    img = beads(a.size, a.beads)
    dog.compute(img[:64, :64, :64].copy(), localization=1)  # warm-up (module load, kernels)
    ts, td = [], []
    pts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        pts = dog.compute(img, localization=1)
        ts.append(time.perf_counter() - t0)
    for _ in range(a.reps):
        t0 = time.perf_counter()
        dog.compute(img, localization=1, return_dog=True)
        td.append(time.perf_counter() - t0)
    n = img.size
    t, t2 = float(np.median(ts)), float(np.median(td))
    print(json.dumps({
        "workload": f"DoG bead detection, one {a.size}^3 view, {a.beads} synthetic beads, sigma 1.8, "
                    "threshold 0.008, quadratic localisation (ProcessDOG defaults)",
        "interest_points": len(pts),
        "ms": round(t * 1e3, 2), "Mvoxels_per_s": round(n / t / 1e6, 1),
        "ms_with_dog_image": round(t2 * 1e3, 2),
        "note": "host buffers in and out (C-ABI contract): includes PCIe upload of the view",
    }), flush=True)


if __name__ == "__main__":
    main()
