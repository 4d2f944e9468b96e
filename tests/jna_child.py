"""The JNA deployment configuration, run as a fresh child process (test infrastructure).

A Java consumer of libspimdecon.so (the JNA interfaces of
``spim/process/cuda/CUDAFourierConvolution.java:9-10``,
``CUDASeparableConvolution.java:13-21`` and the ``mvd_*`` / ``spim_dog_*`` session
API; loaded the way ``spim/process/cuda/NativeLibraryTools.java:86-124`` loads a
native library) has no torch: the library binds the ROCm stack it is linked
against, /opt/rocm.  This script is that process: numpy + ctypes only, the
in-tree library loaded with ``SPIMDECON_HIP_RUNTIME=system``, and

- /proc/self/maps must show libamdhip64 / librocfft from /opt/rocm and nothing
  from torch's bundled ROCm;
- ``convolution3DfftCUDAInPlace`` + the legacy blocked convolutions against
  golden ``conv.npz``;
- ``convolve_15`` (and 63) against ``oracle/dog_ref.gauss3d`` (bit-exact);
- the ``mvd_*`` session on host buffers against every ``rl_*.npz``;
- ``spim_dog_compute`` against ``dog.npz`` (bit-exact image and peaks).

Prints one JSON line and exits 0 when everything matched, 1 otherwise.
``tests/test_gpu_jna_runtime.py`` starts it with ``subprocess``.
"""
from __future__ import annotations

import glob
import json
import os
import sys

os.environ["SPIMDECON_HIP_RUNTIME"] = "system"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")

import numpy as np  # noqa: E402

from oracle import dog_ref  # noqa: E402  (numpy-only checker)
from spim_registration_amd import _lib, dog, legacy  # noqa: E402
from spim_registration_amd.decon import PSFTYPE, Session  # noqa: E402


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def mapped_libs():
    """{soname stem: set of real paths} of the HIP / rocFFT / RCCL libraries mapped here."""
    out = {}
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) < 6:
                continue
            path = parts[5]
            for stem in ("libamdhip64.so", "librocfft.so", "librccl.so", "libhsa-runtime64.so"):
                if os.path.basename(path).startswith(stem):
                    out.setdefault(stem, set()).add(os.path.realpath(path))
    return out


def main() -> int:
    res = {"checks": {}, "failures": []}

    def check(name, ok, detail):
        res["checks"][name] = detail
        if not ok:
            res["failures"].append(name)

    lib = _lib.load()
    check("devices", _lib.num_devices() >= 1, _lib.num_devices())

    g = np.load(os.path.join(GOLD, "conv.npz"))
    cuda = legacy.CUDAFourierConvolution()
    blk = g["block"].copy()
    cuda.convolution3DfftCUDAInPlace(blk.reshape(-1), list(blk.shape), g["k"], list(g["k"].shape), 0)
    e = rel_l2(blk, g["circular"])
    check("convolution3DfftCUDAInPlace", e < 1e-6, e)
    for ext in ("mirror", "one"):
        out = legacy.convolve_blocks_cuda(g["a"], g["k"], (16, 14, 12), ext, cuda, 0)
        e = rel_l2(out, g[ext])
        check(f"blocked_{ext}", e < 1e-6, e)

    sep = legacy.CUDASeparableConvolution()
    rng = np.random.default_rng(3)
    img = rng.random((13, 17, 19)).astype(np.float32)
    for sigmas in ([1.7, 2.0, 1.2], [6.0, 3.0, 9.5]):      # convolve_15, convolve_63
        for oob, mode in ((legacy.OutOfBounds.VALUE, "value"), (legacy.OutOfBounds.MIRROR_SINGLE, "mirror")):
            im = img.copy().reshape(-1)
            ok = legacy.gauss(im, [19, 17, 13], sigmas, oob, 0.25, sep, 0)
            exp = dog_ref.gauss3d(img, legacy.get_cuda_kernels(sigmas), mode, 0.25)
            same = bool(ok) and np.array_equal(im.reshape(img.shape), exp)
            n = len(legacy.get_cuda_kernels(sigmas)[0])
            check(f"convolve_{n}_{mode}", same, same)

    for path in sorted(glob.glob(os.path.join(GOLD, "rl_*.npz"))):
        g = np.load(path)
        imgs, ws, psfs = g["imgs"], g["weights"], g["psfs"]
        nz, ny, nx = imgs.shape[1:]
        with Session((nx, ny, nz), ij_threads=int(g["ij_threads"])) as s:
            for i, w, k in zip(imgs, ws, psfs):
                s.add_view(i, w, k)
            s.init(PSFTYPE(int(g["psftype"])))
            ek = 0.0                      # kernels: 1e-6 (K1) and 1e-5 (K2) as test_gpu_golden.py
            for v in range(len(psfs)):
                k1, k2 = s.get_kernels(v, psfs[v].shape)
                ek = max(ek, rel_l2(k1, g["k1"][v]), rel_l2(k2, g["k2"][v]) / 10)
            avg = s.init_psi()
            st = s.run(int(g["iters"]), float(g["lam"]))
            s.apply_mask()
            psi = s.get_psi()
        name = os.path.basename(path)[:-4]
        e = rel_l2(psi, g["psi"])
        ea = abs(avg - float(g["avg"])) / abs(float(g["avg"]))
        es = float(np.max(np.abs(st[:, :, 0] - g["stats"][:, :, 0]) / np.abs(g["stats"][:, :, 0])))
        check(name, e < 1e-4 and ek < 1e-6 and ea <= 1e-12 and es < 1e-3,
              {"psi_rel_l2": e, "kernels": ek, "avg": ea, "stats_rtol": es})

    g = np.load(os.path.join(GOLD, "dog.npz"))
    pts, d = dog.compute(g["img"], 1.8, 0.008, return_dog=True, keep_intensity=True)
    same = np.array_equal(d, g["dog"]) and np.array_equal(dog.peaks_array(pts), g["peaks"])
    check("spim_dog_compute", same, {"bit_exact": bool(same), "peaks": len(pts)})

    maps = mapped_libs()
    res["maps"] = {k: sorted(v) for k, v in maps.items()}
    rocm = os.path.realpath("/opt/rocm")
    for stem in ("libamdhip64.so", "librocfft.so"):
        paths = maps.get(stem, set())
        check(f"maps_{stem}", len(paths) == 1 and all(p.startswith(rocm + "/") for p in paths), sorted(paths))
    torch_libs = sorted(p for v in maps.values() for p in v if "torch" in p)
    check("no_torch_runtime", not torch_libs and "torch" not in sys.modules, torch_libs)
    res["version"] = lib.spimdecon_version().decode()
    print(json.dumps(res, sort_keys=True), flush=True)
    return 1 if res["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
