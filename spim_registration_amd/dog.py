"""Host-side mirror of the DoG bead-detection pass (ProcessDOG.compute).

spim/process/interestpointdetection/ProcessDOG.java:40-178 and
Localization.noLocalization (Localization.java:19-45); the whole pass
(min/max, normalisation, both Gaussians, subtraction, 26-neighbour peak
test, compaction) runs on the GPU in ``spim_dog_compute``.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, fptr


@dataclass
class InterestPoint:
    """spim.fiji.spimdata.interestpoints.InterestPoint(Value)."""
    id: int
    location: tuple
    intensity: float | None = None


def compute(img: np.ndarray, sigma: float = 1.8, threshold: float = 0.008, localization: int = 0,
            image_sigma=(0.5, 0.5, 0.5), find_min: bool = False, find_max: bool = True,
            min_intensity: float = float("nan"), max_intensity: float = float("nan"),
            keep_intensity: bool = False, device: int = 0, ij_threads: int = 8,
            return_dog: bool = False, max_peaks: int | None = None):
    """ProcessDOG.compute: returns the list of InterestPoint (and the DoG image
    when ``return_dog``).  ``img`` is a [z, y, x] float32 volume (not modified)."""
    lib = _lib.load()
    img = np.ascontiguousarray(img, np.float32)
    if img.ndim != 3:
        raise ValueError("img must be 3D [z, y, x]")
    p = _lib.DogParams()
    lib.spim_dog_params_default(C.byref(p))
    p.sigma = float(sigma)
    p.threshold = float(threshold)
    p.localization = int(localization)
    for d in range(3):
        p.image_sigma[d] = float(image_sigma[d])
    p.find_min = int(bool(find_min))
    p.find_max = int(bool(find_max))
    p.min_intensity = float(min_intensity)
    p.max_intensity = float(max_intensity)
    p.ij_threads = int(ij_threads)
    p.device = int(device)
    dims = (C.c_int64 * 3)(img.shape[2], img.shape[1], img.shape[0])
    dog = np.empty_like(img) if return_dog else None
    cap = int(max_peaks) if max_peaks is not None else max(1024, img.size // 64)
    peaks = (_lib.Peak * cap)()
    n = C.c_int64(0)
    check(lib.spim_dog_compute(fptr(img), dims, C.byref(p), fptr(dog) if dog is not None else None,
                               peaks, cap, C.byref(n)))
    total = int(n.value)
    if total > cap:   # rerun with the exact capacity
        peaks = (_lib.Peak * total)()
        check(lib.spim_dog_compute(fptr(img), dims, C.byref(p), fptr(dog) if dog is not None else None,
                                   peaks, total, C.byref(n)))
    out = []
    for i in range(min(total, len(peaks))):
        pk = peaks[i]
        loc = (float(pk.x), float(pk.y), float(pk.z))
        out.append(InterestPoint(i, loc, float(pk.intensity) if keep_intensity else None))
    return (out, dog) if return_dog else out


def peaks_array(points) -> np.ndarray:
    """[(x, y, z)] int array of interest-point locations."""
    return np.array([[int(c) for c in p.location] for p in points], np.int64).reshape(-1, 3)
