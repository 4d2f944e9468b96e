"""BASELINE configs[3]: 8-view 768^3 time series (4 timepoints), DoG bead detection
+ (given) registration + input preparation / PSF extraction + RL deconvolution,
all device resident (spim_registration_amd.pipeline).  Prints one JSON line with
the per-stage times of every timepoint.

    python tools/c4_pipeline.py [--size 768] [--views 8] [--timepoints 4] [--iterations 10]
                                [--only T] [--digest]

--only T runs timepoint T alone (a fresh process: nothing cached from earlier
timepoints); --digest adds the SHA-256 of psi and of the RL statistics per timepoint
(tests/test_gpu_scale.py compares a back-to-back run with a fresh-process one).

The synthetic acquisition (spim_registration_amd.synthetic.make_timepoint_torch) is
generated on the GPU before each timepoint and is not timed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=768)
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--timepoints", type=int, default=4)
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--psf", type=int, nargs=3, default=[19, 19, 25], help="extracted PSF size x y z")
    ap.add_argument("--only", type=int, default=None, help="run this timepoint alone")
    ap.add_argument("--digest", action="store_true", help="SHA-256 of psi and stats per timepoint")
    a = ap.parse_args()
    import torch
    from spim_registration_amd import pipeline, synthetic
    pipe = pipeline.Pipeline(psf_size=a.psf, iterations=a.iterations)

    n = a.size
    out = {"workload": f"{a.views}-view {n}^3 x {a.timepoints} timepoints: DoG (sigma 1.8, threshold 0.008, "
                       f"quadratic) -> correspondences from the given models -> input preparation + PSF "
                       f"extraction ({a.psf[0]}x{a.psf[1]}x{a.psf[2]}) -> RL OPTIMIZATION_I lambda 0.006, "
                       f"{a.iterations} iterations",
           "data": "synthetic (beads + blobs, views rotated about y by 360/V degrees, Poisson noise; GPU)",
           "timepoints": []}
    total = 0.0

    def log(msg):
        print(msg, file=sys.stderr, flush=True)

    for t in range(a.timepoints) if a.only is None else [a.only]:
        tg = time.perf_counter()
        views, models = synthetic.make_timepoint_torch((n, n, n), (n, n, n), a.views, timepoint=t, device="cuda:0",
                                                       log=log)
        torch.cuda.synchronize()
        log(f"timepoint {t}: synthetic views generated in {time.perf_counter() - tg:.1f} s")
        t0 = time.perf_counter()
        res = pipe.process(views, models, (0, 0, 0), (n, n, n), log=log, digest=a.digest)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        total += dt
        ent = {"t": t, "s": round(dt, 3), "stage_ms": res.ms,
               "detections": [int(len(p)) for p in res.points],
               "corresponding": [int(len(c)) for c in res.corresponding],
               "psf_dims_zyx": [list(p.shape) for p in res.psfs],
               "rl_Mvox_per_s_per_iter": round(n ** 3 * a.iterations / (res.ms["rl_iterations"] * 1e-3) / 1e6, 1),
               "psi_mean": float(res.psi.mean()), "engine": res.engine}
        if a.digest:
            ent.update(pipeline.result_digest(res))
        out["timepoints"].append(ent)
        print(json.dumps(ent), file=sys.stderr, flush=True)
        del views, res
        torch.cuda.empty_cache()
    out["total_s"] = round(total, 3)
    out["s_per_timepoint"] = round(total / max(a.timepoints, 1), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
