"""Host-side mirror of the DoG bead-detection pass (ProcessDOG.compute).

spim/process/interestpointdetection/ProcessDOG.java:40-178 and Localization
(Localization.java:19-88: none, or the quadratic sub-pixel fit); the whole
pass (min/max, normalisation, both Gaussians, subtraction, 26-neighbour peak
test, compaction, fit) runs on the GPU in ``spim_dog_interest_points``.
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
            keep_intensity: bool = False, device: int | None = None, ij_threads: int = 8,
            return_dog: bool = False, max_peaks: int | None = None):
    """ProcessDOG.compute: returns the list of InterestPoint (and the DoG image
    when ``return_dog``).  ``img`` is a [z, y, x] float32 volume (not modified):
    a numpy array, or a torch tensor on the GPU -- a view already resident in HBM
    is read in place (the returned DoG image is then a torch tensor too).
    ``device``: the GPU that runs the pass; default the tensor's own GPU (device 0 for
    a host array)."""
    lib = _lib.load()
    on_dev = hasattr(img, "is_cuda") and img.is_cuda
    if device is None:
        device = img.device.index if on_dev else 0
    if on_dev:
        img = img.contiguous().float()
        if img.dim() != 3:
            raise ValueError("img must be 3D [z, y, x]")
        return _compute_device(lib, img, sigma, threshold, localization, image_sigma, find_min, find_max,
                               min_intensity, max_intensity, keep_intensity, device, ij_threads, return_dog,
                               max_peaks)
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
    pts = (_lib.InterestPointC * cap)()
    n = C.c_int64(0)
    dptr = fptr(dog) if dog is not None else None
    check(lib.spim_dog_interest_points(fptr(img), dims, C.byref(p), dptr, pts, cap, C.byref(n)))
    total = int(n.value)
    if total > cap:   # rerun with the exact capacity
        pts = (_lib.InterestPointC * total)()
        check(lib.spim_dog_interest_points(fptr(img), dims, C.byref(p), dptr, pts, total, C.byref(n)))
    out = []
    for i in range(min(total, len(pts))):
        ip = pts[i]
        out.append(InterestPoint(i, (ip.pos[0], ip.pos[1], ip.pos[2]),
                                 float(ip.intensity) if keep_intensity else None))
    return (out, dog) if return_dog else out


def _params(lib, sigma, threshold, localization, image_sigma, find_min, find_max, min_intensity, max_intensity,
            device, ij_threads):
    p = _lib.DogParams()
    lib.spim_dog_params_default(C.byref(p))
    p.sigma, p.threshold, p.localization = float(sigma), float(threshold), int(localization)
    for d in range(3):
        p.image_sigma[d] = float(image_sigma[d])
    p.find_min, p.find_max = int(bool(find_min)), int(bool(find_max))
    p.min_intensity, p.max_intensity = float(min_intensity), float(max_intensity)
    p.ij_threads, p.device = int(ij_threads), int(device)
    return p


# InterestPointC as a numpy record (pos: 3 doubles, intensity float, is_max int32)
IP_DTYPE = np.dtype([("pos", "<f8", (3,)), ("intensity", "<f4"), ("is_max", "<i4")])


def _points_device(lib, img, p, dog):
    """spim_dog_interest_points on a GPU tensor: a numpy IP_DTYPE record array."""
    import torch
    torch.cuda.synchronize(img.device)   # the library runs on its own stream
    dims = (C.c_int64 * 3)(img.shape[2], img.shape[1], img.shape[0])
    fp = C.POINTER(C.c_float)
    iptr = C.cast(C.c_void_p(img.data_ptr()), fp)
    dptr = C.cast(C.c_void_p(dog.data_ptr()), fp) if dog is not None else None
    cap = max(1 << 16, img.numel() // 512)   # room for a dense bead field: no second pass
    n = C.c_int64(0)
    while True:
        buf = np.empty(cap, IP_DTYPE)
        check(lib.spim_dog_interest_points(iptr, dims, C.byref(p), dptr,
                                           buf.ctypes.data_as(C.POINTER(_lib.InterestPointC)), cap, C.byref(n)))
        if int(n.value) <= cap:
            return buf[:int(n.value)]
        cap = int(n.value)


def _compute_device(lib, img, sigma, threshold, localization, image_sigma, find_min, find_max, min_intensity,
                    max_intensity, keep_intensity, device, ij_threads, return_dog, max_peaks):
    import torch
    p = _params(lib, sigma, threshold, localization, image_sigma, find_min, find_max, min_intensity,
                max_intensity, device, ij_threads)
    dog = torch.empty_like(img) if return_dog else None
    rec = _points_device(lib, img, p, dog)
    if max_peaks is not None:
        rec = rec[:int(max_peaks)]
    out = [InterestPoint(i, tuple(r["pos"].tolist()), float(r["intensity"]) if keep_intensity else None)
           for i, r in enumerate(rec)]
    return (out, dog) if return_dog else out


def interest_points_array(img, sigma: float = 1.8, threshold: float = 0.008, localization: int = 0,
                          image_sigma=(0.5, 0.5, 0.5), find_min: bool = False, find_max: bool = True,
                          min_intensity: float = float("nan"), max_intensity: float = float("nan"),
                          device: int | None = None, ij_threads: int = 8):
    """ProcessDOG.compute on a GPU tensor, as arrays: (positions (n, 3) x, y, z;
    intensities (n,)) in the reference's order -- no per-point Python objects.
    ``device`` defaults to the tensor's own GPU."""
    lib = _lib.load()
    if device is None:
        device = img.device.index
    img = img.contiguous().float()
    p = _params(lib, sigma, threshold, localization, image_sigma, find_min, find_max, min_intensity,
                max_intensity, device, ij_threads)
    rec = _points_device(lib, img, p, None)
    return np.ascontiguousarray(rec["pos"]), np.ascontiguousarray(rec["intensity"])


def simple_peaks(img: np.ndarray, sigma: float = 1.8, threshold: float = 0.008, localization: int = 0,
                 image_sigma=(0.5, 0.5, 0.5), find_min: bool = False, find_max: bool = True,
                 min_intensity: float = float("nan"), max_intensity: float = float("nan"),
                 device: int = 0, ij_threads: int = 8):
    """DifferenceOfGaussianNewPeakFinder.getSimplePeaks: [(x, y, z, |v|, is_min, is_max)]
    (threshold / 10 when ``localization`` is 1)."""
    lib = _lib.load()
    img = np.ascontiguousarray(img, np.float32)
    p = _lib.DogParams()
    lib.spim_dog_params_default(C.byref(p))
    p.sigma, p.threshold, p.localization = float(sigma), float(threshold), int(localization)
    for d in range(3):
        p.image_sigma[d] = float(image_sigma[d])
    p.find_min, p.find_max = int(bool(find_min)), int(bool(find_max))
    p.min_intensity, p.max_intensity = float(min_intensity), float(max_intensity)
    p.ij_threads, p.device = int(ij_threads), int(device)
    dims = (C.c_int64 * 3)(img.shape[2], img.shape[1], img.shape[0])
    n = C.c_int64(0)
    check(lib.spim_dog_compute(fptr(img), dims, C.byref(p), None, None, 0, C.byref(n)))
    pk = (_lib.Peak * max(int(n.value), 1))()
    check(lib.spim_dog_compute(fptr(img), dims, C.byref(p), None, pk, int(n.value), C.byref(n)))
    return [(q.x, q.y, q.z, q.intensity, bool(q.is_min), bool(q.is_max)) for q in pk[:int(n.value)]]


def peaks_array(points) -> np.ndarray:
    """[(x, y, z)] int array of interest-point locations."""
    return np.array([[int(c) for c in p.location] for p in points], np.int64).reshape(-1, 3)


class InterestPointList:
    """spim/fiji/spimdata/interestpoints/InterestPointList.java:19-220 (interest points
    only; correspondences belong to registration, out of scope).  ``base_dir`` + ``file``
    name the list as in the XML; the text file is ``<base_dir>/<file>.ip.txt``, written
    and read by the library (``spim_save_interest_points`` / ``spim_load_interest_points``)."""

    def __init__(self, base_dir, file):
        self.base_dir = str(base_dir) if base_dir is not None else ""
        self.file = str(file)
        self.interest_points: list[InterestPoint] | None = None
        self.parameters = ""

    def get_interest_points_ext(self):
        return ".ip.txt"

    def set_interest_points(self, pts):
        self.interest_points = list(pts)

    def get_interest_points(self):
        return self.interest_points

    def save_interest_points(self) -> bool:
        """saveInterestPoints (:66-100); False without a list, like the reference."""
        if self.interest_points is None:
            return False
        n = len(self.interest_points)
        arr = (_lib.InterestPointC * max(n, 1))()
        ids = (C.c_int32 * max(n, 1))()
        for i, p in enumerate(self.interest_points):
            for d in range(3):
                arr[i].pos[d] = float(p.location[d])
            ids[i] = int(p.id)
        check(_lib.load().spim_save_interest_points(self.base_dir.encode(), self.file.encode(), arr, ids, n))
        return True

    def load_interest_points(self) -> bool:
        """loadInterestPoints (:178-220): False when the file cannot be read (the
        reference catches the IOException); a malformed line raises (Java's
        NumberFormatException is not caught there either)."""
        # the reference starts a fresh list before opening the file (:184): a failed
        # load leaves it empty, never the previous points (a malformed line raises, as
        # the reference's NumberFormatException does; its partial list is not kept here)
        self.interest_points = []
        lib = _lib.load()
        n = C.c_int64(0)
        st = lib.spim_load_interest_points(self.base_dir.encode(), self.file.encode(), None, None, 0, C.byref(n))
        if st == _lib.ERR_IO:
            return False
        check(st)
        cap = max(int(n.value), 1)
        arr = (_lib.InterestPointC * cap)()
        ids = (C.c_int32 * cap)()
        check(lib.spim_load_interest_points(self.base_dir.encode(), self.file.encode(), arr, ids, cap,
                                            C.byref(n)))
        self.interest_points = [InterestPoint(int(ids[i]), (arr[i].pos[0], arr[i].pos[1], arr[i].pos[2]))
                                for i in range(int(n.value))]
        return True


def set_java_version(jdk: int) -> None:
    """Double.toString form used by the .ip.txt writer: 8 (default, Fiji's Java 8
    FloatingDecimal) or 19 (JDK 19+ shortest round trip)."""
    check(_lib.load().spim_set_java_version(int(jdk)))


def java_double_to_string(d: float) -> str:
    """Double.toString as written into .ip.txt files (library formatter)."""
    buf = C.create_string_buffer(64)
    check(_lib.load().spim_java_double_to_string(float(d), buf, 64))
    return buf.value.decode()
