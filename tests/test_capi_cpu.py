"""CPU: the C-ABI library builds, loads and exports every symbol
include/spimdecon.h declares; host-only entry points work; every compute entry
point fails loudly (no CPU fallback) when no GPU is visible."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from spim_registration_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "spimdecon.h")


def declared_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-zA-Z_0-9]+\s*\**\s*\**([a-zA-Z_][a-zA-Z_0-9]*)\s*\(",
                       txt, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "defined")))


def test_header_symbols_exported(lib):
    names = declared_functions()
    assert len(names) >= 35
    for n in names:
        assert hasattr(lib, n), f"{n} declared in spimdecon.h but not exported"
    # and the ctypes binding covers exactly the header
    assert sorted(_lib.SIGNATURES) == names


def test_version(lib):
    v = lib.spimdecon_version().decode()
    assert "gfx950" in v and "rocfft" in v


def test_struct_layouts(lib):
    assert C.sizeof(_lib.Peak) == 24
    p = _lib.MvdParams()
    lib.mvd_params_default(C.byref(p))
    assert p.local_slabs == 1 and p.nranks == 1 and p.ij_threads == 8 and p.comm_id is None
    d = _lib.DogParams()
    lib.spim_dog_params_default(C.byref(d))
    assert abs(d.sigma - 1.8) < 1e-6 and abs(d.threshold - 0.008) < 1e-9
    assert d.find_max == 1 and d.find_min == 0 and np.isnan(d.min_intensity)


@pytest.mark.parametrize("nz,parts", [(512, 8), (100, 3), (7, 7), (1000, 6)])
def test_slab_range_partition(lib, nz, parts):
    z0, z1 = C.c_int64(), C.c_int64()
    prev = 0
    sizes = []
    for i in range(parts):
        _lib.check(lib.mvd_slab_range(nz, parts, i, C.byref(z0), C.byref(z1)))
        assert z0.value == prev
        sizes.append(z1.value - z0.value)
        prev = z1.value
    assert prev == nz and max(sizes) - min(sizes) <= 1


def test_bad_arguments_report_errors(lib):
    z0, z1 = C.c_int64(), C.c_int64()
    st = lib.mvd_slab_range(10, 3, 5, C.byref(z0), C.byref(z1))
    assert st == -1 and "slab_range" in _lib.last_error()


@pytest.mark.skipif(_lib.LIB_PATH.exists() and os.path.exists("/dev/kfd"), reason="GPU visible")
def test_compute_fails_loudly_without_gpu(lib):
    assert lib.getNumDevicesCUDA() == 0
    im = np.ones(27, np.float32)
    k = np.ones(1, np.float32)
    dims = np.array([3, 3, 3], np.int32)
    kd = np.array([1, 1, 1], np.int32)
    st = lib.convolution3DfftCUDAInPlace(_lib.fptr(im), _lib.iptr(dims), _lib.fptr(k), _lib.iptr(kd), 0)
    assert st == -2 and "no HIP device" in _lib.last_error()
    from spim_registration_amd.decon import Session
    with pytest.raises(_lib.SpimDeconError):
        Session((8, 8, 8))
