"""Host-side mirror of the reference's deconvolution API (drop-in surface).

Mirrors ``spim.process.fusion.deconvolution`` (paths under
/root/reference/src/main/java/spim/process/fusion/deconvolution/):

  PSFTYPE            MVDeconFFT.java:28
  MVDeconFFT         MVDeconFFT.java:58-151    (one view: image, weight, kernel1)
  MVDeconInput       MVDeconInput.java:10-59   (ordered list of views)
  MVDeconvolution    MVDeconvolution.java:73-190 (runs the whole deconvolution in
                                                  its constructor, getPsi())

All arithmetic runs in libspimdecon.so on the GPU (session API of
include/spimdecon.h).  Volumes are numpy float32 arrays indexed [z, y, x]
(x fastest, ImgLib2 ArrayImg order); kernels likewise.
"""
from __future__ import annotations

import atexit
import ctypes as C
import weakref
from enum import IntEnum

import numpy as np

from . import _lib
from ._lib import check, fptr

MIN_VALUE = np.float32(0.0001)


class PSFTYPE(IntEnum):
    """MVDeconFFT.PSFTYPE (MVDeconFFT.java:28), ordinals preserved."""
    OPTIMIZATION_II = 0
    OPTIMIZATION_I = 1
    EFFICIENT_BAYESIAN = 2
    INDEPENDENT = 3


def _as_volume(a, name):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 3:
        raise ValueError(f"{name} must be a 3D [z, y, x] array, got shape {a.shape}")
    return a


def _kdims(k):
    kz, ky, kx = k.shape
    if kx % 2 == 0 or ky % 2 == 0 or kz % 2 == 0:
        raise ValueError(f"kernel dims must be odd (EfficientBayesianBased.java:792-799), got {k.shape}")
    return np.array([kx, ky, kz], np.int32)


class MVDeconFFT:
    """One view of the deconvolution (MVDeconFFT.java:58-151).

    ``device_list``: HIP device ids (the reference's -1 = CPU is rejected: there
    is no CPU path).  ``use_blocks`` / ``block_size`` / ``save_memory`` are
    accepted for API parity; the GPU-resident session keeps the whole volume in
    HBM (blocks are 'precise', so the result does not depend on them)."""

    def __init__(self, image, weight, kernel, block_factory=None, device_list=(0,),
                 use_blocks=False, block_size=None, save_memory=False):
        self.image = _as_volume(image, "image")
        self.weight = _as_volume(weight, "weight")
        if self.weight.shape != self.image.shape:
            raise ValueError("image and weight dims differ")
        self.kernel1 = _as_volume(kernel, "kernel")
        _kdims(self.kernel1)
        self.kernel2 = None
        self.device_list = list(device_list)
        if not self.device_list or any(d < 0 for d in self.device_list):
            raise ValueError("device_list must hold GPU ids >= 0 (no CPU path in this framework)")
        self.use_blocks = use_blocks
        self.block_size = block_size
        self.save_memory = save_memory
        self.num_views = 0

    def set_num_views(self, n):
        self.num_views = n

    def get_image(self):
        return self.image

    def get_weight(self):
        return self.weight

    def get_kernel1(self):
        return self.kernel1

    def get_kernel2(self):
        return self.kernel2


class MVDeconInput:
    """MVDeconInput.java:10-59."""
    min_value = MIN_VALUE

    def __init__(self, img_factory=None):
        self.views: list[MVDeconFFT] = []
        self.img_factory = img_factory

    def add(self, view: MVDeconFFT):
        self.views.append(view)
        for v in self.views:
            v.set_num_views(len(self.views))

    def get_views(self):
        return self.views

    def get_num_views(self):
        return len(self.views)

    def init(self, iteration_type: PSFTYPE, ij_threads: int = 8):
        """MVDeconInput.init -> MVDeconFFT.init for every view, in list order,
        computed on the GPU by ``mvd_prepare_kernels``."""
        prepare_kernels(self.views, iteration_type, ij_threads)
        return self


def prepare_kernels(views, iteration_type, ij_threads=8, device=None):
    """Fills view.kernel1 (normalised) and view.kernel2 via the C-ABI."""
    lib = _lib.load()
    V = len(views)
    k1_in = [np.ascontiguousarray(v.kernel1, np.float32) for v in views]
    k1_out = [np.empty_like(k) for k in k1_in]
    k2_out = [np.empty_like(k) for k in k1_in]
    kd = np.concatenate([_kdims(k) for k in k1_in]).astype(np.int32)
    PF = C.POINTER(C.c_float)
    arr_in = (PF * V)(*[fptr(k) for k in k1_in])
    arr_o1 = (PF * V)(*[fptr(k) for k in k1_out])
    arr_o2 = (PF * V)(*[fptr(k) for k in k2_out])
    dev = views[0].device_list[0] if device is None else device
    check(lib.mvd_prepare_kernels(V, arr_in, _lib.iptr(kd), int(iteration_type), int(ij_threads),
                                  arr_o1, arr_o2, int(dev)))
    for v, a, b in zip(views, k1_out, k2_out):
        v.kernel1, v.kernel2 = a, b
    return k1_out, k2_out


# Sessions still open at interpreter exit are destroyed by an atexit handler, while the
# library, the HIP runtime and rocFFT are all still intact -- not by __del__ during module
# teardown, whose order relative to the other libraries' own teardown is arbitrary.
_open_sessions: "weakref.WeakSet[Session]" = weakref.WeakSet()


@atexit.register
def _close_open_sessions() -> None:
    for s in list(_open_sessions):
        s.close()


class Session:
    """Thin RAII wrapper of an ``mvd_session`` (GPU-resident RL state)."""

    def __init__(self, dims_xyz, device=0, local_slabs=1, nranks=1, rank=0, comm_id=None,
                 nz_global=None, z_offset=0, storage_fp16=False, ij_threads=8, halo=None,
                 fft_backend="engine", fft_pad_policy="auto", devices=None, slab_axis="auto"):
        """``devices``: several GPUs of this process (``mvd_create_devices``; the
        reference's ``deviceList``, MVDeconFFT.java:58-64) -- the volume is split into
        len(devices) * local_slabs slabs and one ``run`` drives all of them.
        ``slab_axis``: "z", "y" or "auto" (the longer of y and z; z for several ranks)."""
        self.lib = _lib.load()
        p = _lib.MvdParams()
        self.lib.mvd_params_default(C.byref(p))
        for d in range(3):
            p.dims[d] = int(dims_xyz[d])
        p.nz_global = int(nz_global) if nz_global is not None else 0   # 0: this volume (slab axis)
        p.z_offset = int(z_offset)
        p.device = int(device)
        p.local_slabs = int(local_slabs)
        p.nranks = int(nranks)
        p.rank = int(rank)
        self._comm_id = comm_id  # keep alive during create
        p.comm_id = comm_id
        p.storage_fp16 = int(bool(storage_fp16))
        p.ij_threads = int(ij_threads)
        p.fft_backend = {"engine": 0, "rocfft": 1}[fft_backend]
        p.fft_pad_policy = {"auto": 0, "fast": 1, "smooth": 2}[fft_pad_policy]
        p.slab_axis = {"z": 0, "y": 1, "auto": -1}[slab_axis]
        if halo is not None:
            for d in range(3):
                p.halo[d] = int(halo[d])
        h = C.c_void_p()
        if devices is not None and len(devices) > 1:
            devs = np.ascontiguousarray(devices, np.int32)
            check(self.lib.mvd_create_devices(_lib.iptr(devs), len(devs), C.byref(p), C.byref(h)))
        else:
            if devices:
                p.device = int(devices[0])
            check(self.lib.mvd_create(C.byref(p), C.byref(h)))
        self.h = h
        _open_sessions.add(self)
        self.params = p
        self.nviews = 0
        self.shape = (int(dims_xyz[2]), int(dims_xyz[1]), int(dims_xyz[0]))

    def close(self):
        if getattr(self, "h", None):
            self.lib.mvd_destroy(self.h)
            self.h = None
            _open_sessions.discard(self)

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def add_view(self, img, weight, kernel1):
        img = _as_volume(img, "img")
        weight = _as_volume(weight, "weight")
        if img.shape != self.shape or weight.shape != self.shape:
            raise ValueError(f"view dims {img.shape} != session dims {self.shape}")
        k = _as_volume(kernel1, "kernel1")
        check(self.lib.mvd_add_view(self.h, fptr(img), fptr(weight), fptr(k), _lib.iptr(_kdims(k))))
        self.nviews += 1

    def add_view_device(self, d_img_ptr, d_weight_ptr, kernel1):
        k = _as_volume(kernel1, "kernel1")
        check(self.lib.mvd_add_view_device(self.h, C.c_void_p(d_img_ptr), C.c_void_p(d_weight_ptr),
                                           fptr(k), _lib.iptr(_kdims(k))))
        self.nviews += 1

    def init(self, psftype):
        check(self.lib.mvd_init(self.h, int(psftype)))

    def set_kernels(self, view, k1, k2):
        k1 = np.ascontiguousarray(k1, np.float32)
        k2 = np.ascontiguousarray(k2, np.float32)
        check(self.lib.mvd_set_kernels(self.h, int(view), fptr(k1), fptr(k2)))

    def get_kernels(self, view, kshape):
        k1 = np.empty(kshape, np.float32)
        k2 = np.empty(kshape, np.float32)
        check(self.lib.mvd_get_kernels(self.h, int(view), fptr(k1), fptr(k2)))
        return k1, k2

    def init_psi(self, psi=None):
        avg = C.c_double(0.0)
        if psi is None:
            check(self.lib.mvd_init_psi(self.h, None, C.byref(avg)))
        else:
            psi = _as_volume(psi, "psi")
            check(self.lib.mvd_init_psi(self.h, fptr(psi), C.byref(avg)))
        return avg.value

    def run(self, iters, lam):
        stats = np.zeros((max(iters, 1), max(self.nviews, 1), 2), np.float64)
        check(self.lib.mvd_run(self.h, int(iters), float(lam),
                               stats.ctypes.data_as(C.POINTER(C.c_double))))
        return stats[:iters]

    def apply_mask(self):
        check(self.lib.mvd_apply_mask(self.h))

    def get_psi(self):
        out = np.empty(self.shape, np.float32)
        check(self.lib.mvd_get_psi(self.h, fptr(out)))
        return out

    def fft_dims(self, slab=0):
        out = (C.c_int64 * 3)()
        check(self.lib.mvd_fft_dims(self.h, int(slab), out))
        return tuple(out)

    def kernel_planes(self, slab=0):
        """z-planes per stored kernel spectrum (2*cz+1 compact, else Mz)."""
        out = C.c_int()
        check(self.lib.mvd_kernel_planes(self.h, int(slab), C.byref(out)))
        return out.value

    def zpass_mode(self, slab=0):
        """0 fused FFT z pass (full kernels), 1 fused FFT (compact), 3 direct z convolution (z chunks)."""
        out = C.c_int()
        check(self.lib.mvd_zpass_mode(self.h, int(slab), C.byref(out)))
        return out.value

    def xpass_mode(self, slab=0):
        """x pass of the last update launch: 2 two-factor tiles, 1 per-wave rows, 0 Stockham."""
        out = C.c_int()
        check(self.lib.mvd_xpass_mode(self.h, int(slab), C.byref(out)))
        return out.value

    def num_devices(self):
        out = C.c_int()
        check(self.lib.mvd_num_devices(self.h, C.byref(out)))
        return out.value

    def slab_device(self, slab):
        out = C.c_int()
        check(self.lib.mvd_slab_device(self.h, int(slab), C.byref(out)))
        return out.value

    def num_slabs(self):
        """slabs of the session (devices x local slabs, after the automatic split of
        slabs whose buffers exceed the fast passes' 32-bit offsets)."""
        out = C.c_int()
        check(self.lib.mvd_num_slabs(self.h, C.byref(out)))
        return out.value

    def exchange_stats(self):
        """(bytes, copies) of halo planes moved between slabs since creation."""
        b, c = C.c_int64(), C.c_int64()
        check(self.lib.mvd_exchange_stats(self.h, C.byref(b), C.byref(c)))
        return b.value, c.value

    def slab_extent(self, slab=0):
        """voxels (nx, ny, nz) of a slab in the session's internal order (y-split
        sessions: (x, z, y-slab))."""
        out = (C.c_int64 * 3)()
        check(self.lib.mvd_slab_extent(self.h, int(slab), out))
        return tuple(out)

    def enable_timing(self, on=True):
        check(self.lib.mvd_enable_timing(self.h, int(on)))

    def timing(self):
        out = (C.c_double * 16)()
        check(self.lib.mvd_timing(self.h, out))
        return list(out)

    def stream(self):
        return self.lib.mvd_stream(self.h)


class MVDeconvolution:
    """MVDeconvolution.java:73-190: initialises the views, fuses the first
    iteration (or loads ``initial_image``), runs ``num_iterations`` RL iterations
    and masks voxels no view covers.  ``osem_speedup``/``osem_speedup_index`` are
    accepted and unused, as in the reference (``:78-79``)."""

    min_value = MIN_VALUE

    def __init__(self, views: MVDeconInput, iteration_type: PSFTYPE, num_iterations: int,
                 lam: float, osem_speedup: float = 1.0, osem_speedup_index: int = 0,
                 name: str = "deconvolved", *, ij_threads: int = 8, initial_image=None,
                 local_slabs: int = 1, storage_fp16: bool = False, run: bool = True):
        self.views = views
        self.name = name
        self.num_iterations = int(num_iterations)
        self.lam = float(lam)
        data = views.get_views()
        if not data:
            raise ValueError("no views")
        shape = data[0].get_image().shape
        # MVDeconFFT.java:91-100: every view carries the same device list; all of its GPUs
        # share the volume (z-slabs, halo exchange inside the library)
        devs = list(data[0].device_list)
        self.session = Session((shape[2], shape[1], shape[0]), devices=devs, local_slabs=local_slabs,
                               storage_fp16=storage_fp16, ij_threads=ij_threads)
        for v in data:
            self.session.add_view(v.get_image(), v.get_weight(), v.kernel1)
        self.session.init(iteration_type)                                   # views.init :93
        for i, v in enumerate(data):
            v.kernel1, v.kernel2 = self.session.get_kernels(i, v.kernel1.shape)
        self.avg = self.session.init_psi(initial_image)                     # :95-127
        self.stats = np.zeros((0, len(data), 2))
        self.i = 0
        if run:
            self.run_iterations(self.num_iterations)
            self.session.apply_mask()                                       # :180-187

    def run_iterations(self, n):
        st = self.session.run(n, self.lam)
        self.stats = np.concatenate([self.stats, st]) if self.stats.size else st
        self.i += n

    def run_iteration(self):
        """MVDeconvolution.runIteration (:328-331)."""
        self.run_iterations(1)

    def get_psi(self):
        return self.session.get_psi()

    def get_current_iteration(self):
        return self.i

    def get_data(self):
        return self.views

    def get_name(self):
        return self.name
