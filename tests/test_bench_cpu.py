"""bench.py's GPU planning (CPU only): --gpus N either runs N device groups in one
process or N launcher ranks, and never silently measures fewer GPUs."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_plan_devices_without_launcher():
    a = bench.parse(["--gpus", "4"])
    assert bench.plan_gpus(a, {}, 8) == ("devices", 4)
    assert bench.plan_gpus(bench.parse([]), {}, 1) == ("devices", 1)


def test_plan_refuses_too_few_gpus():
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.plan_gpus(bench.parse(["--gpus", "2"]), {}, 1)


def test_plan_ranks_under_launcher():
    env = {"RANK": "1", "WORLD_SIZE": "4", "LOCAL_RANK": "1"}
    assert bench.plan_gpus(bench.parse(["--gpus", "4"]), env, 8) == ("ranks", 4)
    with pytest.raises(SystemExit, match="WORLD_SIZE"):
        bench.plan_gpus(bench.parse(["--gpus", "8"]), env, 8)


def test_bench_gpus2_exits_nonzero_without_gpus():
    """The driver-shaped command on a box with fewer GPUs: rc != 0, clear message."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "refusing to measure fewer" in (r.stdout + r.stderr)


def test_engine_iteration_model_bytes():
    """The roofline model uses the slab's internal extents (y-split: the slab's y rows
    are the z pass's axis), not the caller's nz."""
    geom = {"N": 1024 * 128 * 512, "S": (1050 // 2 + 1) * 536 * 152, "nz_int": 128, "Mz": 152, "kplanes": 25,
            "M": (1050, 536, 152)}
    classes, b_view, model = bench.engine_classes(geom, 4)
    y = dict((c[0], c) for c in classes)["y_pass"][3]
    assert y == pytest.approx(8.0 * (1 + 128 / 152))
    z = dict((c[0], c) for c in classes)["z_convolve"][3]
    assert z == pytest.approx(8.0 + 8.0 * 128 / 152 + 8.0 * 25 / 152)


def test_c5_rank_preset():
    """--c5-rank: one rank's y-slab of BASELINE configs[4] (2048 x 256 x 1024, fp16
    img / weights, OPTIMIZATION_I 0.006) as the headline, no extra lines."""
    a = bench.parse(["--c5-rank"])
    assert a.shape == [2048, 256, 1024] and a.fp16 and a.slab_axis == "y"
    assert (a.psftype, a.lam) == ("OPTIMIZATION_I", 0.006)
    assert a.no_strong_line and a.no_default_mode


def test_engine_classes_pointwise_bytes():
    """The iteration model counts (12 + 2w) N + (32 + 4y + 2z) S bytes per view; the
    exchange-window class carries no bytes (it is a time, not a pass)."""
    geom = {"N": 1000, "S": 600, "nz_int": 10, "Mz": 12, "kplanes": 5}
    classes, b_view, _ = bench.engine_classes(geom, 2)
    names = [c[0] for c in classes]
    assert names[7] == "exchange_window" and classes[7][1:] == (0, 0, 0)
    yb = 8.0 * (1 + 10 / 12)
    zb = 8.0 + 8.0 * 10 / 12 + 8.0 * 5 / 12
    assert abs(b_view - ((12 + 4) * 1000 + (32 + 4 * yb + 2 * zb) * 600)) < 1e-6
