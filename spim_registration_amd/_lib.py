"""ctypes binding of libspimdecon.so (C-ABI declared in include/spimdecon.h).

The binding mirrors what the reference's JNA interfaces would bind
(``spim/process/cuda/CUDAFourierConvolution.java``, ``CUDAStandardFunctions.java``,
``CUDASeparableConvolution.java``): Java ``boolean`` -> ``int32``, ``long`` ->
``int64``, arrays -> pointers.  Loading never falls back to anything: if the
in-tree library is missing the import of the compute API fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

# SPIMDECON_LIB: an experiment build of the same sources (tools/build_variant.sh) for A/B runs
LIB_PATH = Path(os.environ.get("SPIMDECON_LIB") or Path(__file__).resolve().parent / "libspimdecon.so")

_i32, _i64, _f32, _f64 = C.c_int32, C.c_int64, C.c_float, C.c_double
_pf = C.POINTER(C.c_float)
_pi = C.POINTER(C.c_int)
_pi64 = C.POINTER(C.c_int64)
_pd = C.POINTER(C.c_double)


class MvdParams(C.Structure):
    _fields_ = [
        ("dims", C.c_int64 * 3),
        ("nz_global", C.c_int64),
        ("z_offset", C.c_int64),
        ("device", C.c_int),
        ("local_slabs", C.c_int),
        ("nranks", C.c_int),
        ("rank", C.c_int),
        ("comm_id", C.c_char_p),
        ("storage_fp16", C.c_int),
        ("fft_pad_policy", C.c_int),
        ("halo", C.c_int * 3),
        ("ij_threads", C.c_int),
        ("fft_backend", C.c_int),
        ("slab_axis", C.c_int),
        ("reserved", C.c_int * 6),
    ]


class DogParams(C.Structure):
    _fields_ = [
        ("sigma", C.c_float),
        ("threshold", C.c_float),
        ("localization", C.c_int),
        ("image_sigma", C.c_double * 3),
        ("find_min", C.c_int32),
        ("find_max", C.c_int32),
        ("min_intensity", C.c_double),
        ("max_intensity", C.c_double),
        ("ij_threads", C.c_int),
        ("device", C.c_int),
    ]


class Peak(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("z", C.c_int32),
                ("intensity", C.c_float), ("is_min", C.c_int32), ("is_max", C.c_int32)]


class ViewSource(C.Structure):
    _fields_ = [("img", C.POINTER(C.c_float)), ("dims", C.c_int64 * 3), ("model", C.c_double * 12)]


class InputParams(C.Structure):
    _fields_ = [("bb_min", C.c_int64 * 3), ("bb_dims", C.c_int64 * 3),
                ("blending_border", C.c_float * 3), ("blending_range", C.c_float * 3),
                ("weight_type", C.c_int), ("osem_index", C.c_int), ("osem_speedup", C.c_double),
                ("ij_threads", C.c_int), ("device", C.c_int), ("src_on_device", C.c_int),
                ("out_on_device", C.c_int), ("reserved", C.c_int * 8)]


class FusionParams(C.Structure):
    _fields_ = [("bb_min", C.c_int64 * 3), ("bb_dims", C.c_int64 * 3), ("downsampling", C.c_float),
                ("interpolation", C.c_int), ("use_blending", C.c_int), ("device", C.c_int),
                ("src_on_device", C.c_int), ("out_on_device", C.c_int), ("reserved", C.c_int * 8)]


class InterestPointC(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("intensity", C.c_float), ("is_max", C.c_int32)]


# name -> (restype, argtypes); exactly the declarations of include/spimdecon.h
SIGNATURES = {
    "spimdecon_last_error": (C.c_char_p, []),
    "spimdecon_version": (C.c_char_p, []),
    "convolution3DfftCUDAInPlace": (C.c_int, [_pf, _pi, _pf, _pi, C.c_int]),
    "convolution3DfftCUDA": (_pf, [_pf, _pi, _pf, _pi, C.c_int]),
    "spimdecon_free": (None, [C.c_void_p]),
    "getNumDevicesCUDA": (C.c_int, []),
    "getNameDeviceCUDA": (None, [C.c_int, C.c_char_p]),
    "getMemDeviceCUDA": (_i64, [C.c_int]),
    "getFreeMemDeviceCUDA": (_i64, [C.c_int]),
    "getCUDAcomputeCapabilityMajorVersion": (C.c_int, [C.c_int]),
    "getCUDAcomputeCapabilityMinorVersion": (C.c_int, [C.c_int]),
    "spimdecon_next_value": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_double, C.c_void_p]),
    "mvd_prepare_kernels": (C.c_int, [C.c_int, C.POINTER(_pf), _pi, C.c_int, C.c_int,
                                      C.POINTER(_pf), C.POINTER(_pf), C.c_int]),
    "mvd_params_default": (None, [C.POINTER(MvdParams)]),
    "mvd_comm_unique_id": (C.c_int, [C.c_char_p]),
    "mvd_slab_range": (C.c_int, [_i64, C.c_int, C.c_int, _pi64, _pi64]),
    "mvd_halo_plan": (C.c_int, [_i64, _i64, C.c_int, _i64, _pi64]),
    "mvd_create": (C.c_int, [C.POINTER(MvdParams), C.POINTER(C.c_void_p)]),
    "mvd_create_devices": (C.c_int, [_pi, C.c_int, C.POINTER(MvdParams), C.POINTER(C.c_void_p)]),
    "mvd_destroy": (None, [C.c_void_p]),
    "mvd_num_devices": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "mvd_slab_device": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "mvd_num_slabs": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "mvd_slab_extent": (C.c_int, [C.c_void_p, C.c_int, _pi64]),
    "mvd_exchange_stats": (C.c_int, [C.c_void_p, _pi64, _pi64]),
    "mvd_add_view": (C.c_int, [C.c_void_p, _pf, _pf, _pf, _pi]),
    "mvd_add_view_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, _pf, _pi]),
    "mvd_init": (C.c_int, [C.c_void_p, C.c_int]),
    "mvd_set_kernels": (C.c_int, [C.c_void_p, C.c_int, _pf, _pf]),
    "mvd_get_kernels": (C.c_int, [C.c_void_p, C.c_int, _pf, _pf]),
    "mvd_init_psi": (C.c_int, [C.c_void_p, _pf, _pd]),
    "mvd_run": (C.c_int, [C.c_void_p, C.c_int, C.c_double, _pd]),
    "mvd_apply_mask": (C.c_int, [C.c_void_p]),
    "mvd_get_psi": (C.c_int, [C.c_void_p, _pf]),
    "mvd_psi_device": (C.c_void_p, [C.c_void_p, C.c_int]),
    "mvd_fft_dims": (C.c_int, [C.c_void_p, C.c_int, _pi64]),
    "mvd_kernel_planes": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "mvd_zpass_mode": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "mvd_xpass_mode": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "mvd_stream": (C.c_void_p, [C.c_void_p]),
    "mvd_enable_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "mvd_timing": (C.c_int, [C.c_void_p, _pd]),
    "convolve_7": (_i32, [_pf, _pf, _pf, _pf, C.c_int, C.c_int, C.c_int, _i32, _i32, _i32,
                          C.c_int, C.c_float, C.c_int]),
    "spim_dog_params_default": (None, [C.POINTER(DogParams)]),
    "spim_dog_compute": (C.c_int, [_pf, _pi64, C.POINTER(DogParams), _pf, C.POINTER(Peak),
                                   _i64, _pi64]),
    "spim_dog_interest_points": (C.c_int, [_pf, _pi64, C.POINTER(DogParams), _pf,
                                           C.POINTER(InterestPointC), _i64, _pi64]),
    "spim_dog_release_workspace": (C.c_int, [C.c_int]),
    "spim_psf_release_workspace": (C.c_int, [C.c_int]),
    "spim_save_interest_points": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(InterestPointC),
                                            C.POINTER(C.c_int32), C.c_int64]),
    "spim_load_interest_points": (C.c_int, [C.c_char_p, C.c_char_p, C.POINTER(InterestPointC),
                                            C.POINTER(C.c_int32), C.c_int64, _pi64]),
    "spim_java_double_to_string": (C.c_int, [C.c_double, C.c_char_p, C.c_int]),
    "spim_set_java_version": (C.c_int, [C.c_int]),
    "convolutionCPU": (C.c_int, [_pf, _pf, _pf, _pf, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_float]),
    "spim_input_params_default": (None, [C.POINTER(InputParams)]),
    "spim_fusion_params_default": (None, [C.POINTER(FusionParams)]),
    "spim_psf_transformed_size": (C.c_int, [_pi64, _pd, _pi64, _pd]),
    "spim_transform_psf": (C.c_int, [_pf, _pi64, _pd, _pf, C.c_int]),
    "spim_extract_psf": (C.c_int, [C.c_void_p, _pi64, C.c_int, _pd, C.c_int64, _pi64, _pd, _pf, _pf, C.c_int]),
    "spim_extract_psfs": (C.c_int, [C.c_int, C.POINTER(C.c_void_p), _pi64, C.c_int, C.POINTER(C.c_void_p), _pi64,
                                    _pi64, _pd, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int]),
    "spim_average_transformed_psf": (C.c_int, [C.c_int, C.POINTER(_pf), _pi64, _pf, _pi64, C.c_int]),
    "spim_max_projection": (C.c_int, [_pf, _pi64, C.c_int, _pf, _pi64, C.POINTER(C.c_int), C.c_int]),
    "spim_fuse_weighted_average": (C.c_int, [C.c_int, C.POINTER(ViewSource), C.POINTER(FusionParams),
                                             _pf, _pf, _pf]),
    "lrsim_create": (C.c_int, [_pi64, C.c_int, C.c_int, C.c_int, C.c_char_p, C.POINTER(C.c_void_p)]),
    "lrsim_create_devices": (C.c_int, [_pi64, _pi, C.c_int, C.POINTER(C.c_void_p)]),
    "lrsim_destroy": (None, [C.c_void_p]),
    "lrsim_view_device": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "lrsim_add_view": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, _pi]),
    "lrsim_owns_view": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_int)]),
    "lrsim_init": (C.c_int, [C.c_void_p, _pd]),
    "lrsim_run": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, _pd]),
    "lrsim_get_psi": (C.c_int, [C.c_void_p, C.c_void_p]),
    "lrsim_fft_dims": (C.c_int, [C.c_void_p, _pi64]),
    "spim_prepare_inputs": (C.c_int, [C.c_int, C.POINTER(ViewSource), C.POINTER(InputParams),
                                      C.POINTER(_pf), C.POINTER(_pf), C.POINTER(C.c_double),
                                      C.POINTER(C.c_int), C.POINTER(C.c_double)]),
}
for _n in (15, 31, 63, 127):
    SIGNATURES[f"convolve_{_n}"] = SIGNATURES["convolve_7"]

_lib = None


class SpimDeconError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"libspimdecon status {status}: {msg}")
        self.status = status


def load():
    """Loads the in-tree library (raises if it has not been built).

    torch wheels bundle their own libamdhip64.so.7; the loader keeps whichever
    copy of that soname comes first.  A process that uses torch on the GPU
    together with this library must load torch's copy first so both share one
    HIP runtime: the reverse order hands torch the /opt/rocm runtime, and the
    process aborts at exit ("double free or corruption") after a torch GPU
    call.  load() therefore imports torch (when installed) before the library.

    SPIMDECON_HIP_RUNTIME=system skips that import: the library then binds the
    ROCm stack it was linked against (/opt/rocm, the rpath), which is what a
    JNA consumer without torch loads (tests/jna_child.py).
    Such a process must not use torch on the GPU."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(
            f"{LIB_PATH} not found: build it with `python -m spim_registration_amd.build` "
            "(there is no CPU fallback)")
    if os.environ.get("SPIMDECON_HIP_RUNTIME", "") != "system":
        try:
            import torch  # noqa: F401  (binds the HIP runtime soname to torch's copy)
        except ImportError:
            pass
    lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    return load().spimdecon_last_error().decode(errors="replace")


ERR_IO = -8   # SPIMDECON_ERR_IO: a file that cannot be opened


def check(status: int):
    if status != 0:
        raise SpimDeconError(status, last_error())


def fptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous, (a.dtype, a.flags)
    return a.ctypes.data_as(_pf)


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_pi)


def num_devices() -> int:
    return int(load().getNumDevicesCUDA())
