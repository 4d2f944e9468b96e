"""Host-side mirror of the reference's JNA-facing classes (legacy native ABI).

Paths under /root/reference/src/main/java/spim/process/cuda/:

  CUDAFourierConvolution            CUDAFourierConvolution.java:4-10
  CUDAStandardFunctions             CUDAStandardFunctions.java:15-23
  CUDASeparableConvolution          CUDASeparableConvolution.java:9-21
  CUDASeparableConvolutionFunctions CUDASeparableConvolutionFunctions.java:127-245
  BlockGeneratorFixedSizePrecise    BlockGeneratorFixedSizePrecise.java:25-101
  Block (copy/paste)                Block.java:67-359

plus the per-block driver of spim/process/fusion/deconvolution/MVDeconFFTThreads.java:52-94.
These are the call sites a Java maintainer keeps when swapping in
libspimdecon.so as the JNA library; all arithmetic runs on the
GPU inside the library.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from enum import IntEnum

import numpy as np

from . import _lib
from ._lib import check, fptr


class CUDAStandardFunctions:
    """CUDAStandardFunctions.java:15-23 (device enumeration)."""

    def __init__(self):
        self.lib = _lib.load()

    def getNumDevicesCUDA(self) -> int:
        return int(self.lib.getNumDevicesCUDA())

    def getNameDeviceCUDA(self, dev: int) -> str:
        buf = C.create_string_buffer(256)
        self.lib.getNameDeviceCUDA(int(dev), buf)
        return buf.value.decode(errors="replace")

    def getMemDeviceCUDA(self, dev: int) -> int:
        return int(self.lib.getMemDeviceCUDA(int(dev)))

    def getFreeMemDeviceCUDA(self, dev: int) -> int:
        return int(self.lib.getFreeMemDeviceCUDA(int(dev)))

    def getCUDAcomputeCapabilityMajorVersion(self, dev: int) -> int:
        return int(self.lib.getCUDAcomputeCapabilityMajorVersion(int(dev)))

    def getCUDAcomputeCapabilityMinorVersion(self, dev: int) -> int:
        return int(self.lib.getCUDAcomputeCapabilityMinorVersion(int(dev)))


class CUDAFourierConvolution(CUDAStandardFunctions):
    """CUDAFourierConvolution.java:9-10."""

    def convolution3DfftCUDAInPlace(self, im: np.ndarray, imDim, kernel: np.ndarray, kernelDim,
                                    devCUDA: int) -> None:
        """``im`` (float32, x-fastest) is overwritten; dims are {z, y, x}."""
        assert im.dtype == np.float32 and im.flags.c_contiguous
        imd = np.ascontiguousarray(imDim, np.int32)
        kd = np.ascontiguousarray(kernelDim, np.int32)
        k = np.ascontiguousarray(kernel, np.float32)
        check(self.lib.convolution3DfftCUDAInPlace(fptr(im), _lib.iptr(imd), fptr(k), _lib.iptr(kd),
                                                   int(devCUDA)))

    def convolution3DfftCUDA(self, im, imDim, kernel, kernelDim, devCUDA) -> np.ndarray:
        im = np.ascontiguousarray(im, np.float32)
        imd = np.ascontiguousarray(imDim, np.int32)
        kd = np.ascontiguousarray(kernelDim, np.int32)
        k = np.ascontiguousarray(kernel, np.float32)
        p = self.lib.convolution3DfftCUDA(fptr(im), _lib.iptr(imd), fptr(k), _lib.iptr(kd), int(devCUDA))
        if not p:
            raise _lib.SpimDeconError(-1, _lib.last_error())
        n = int(np.prod(imd))
        out = np.ctypeslib.as_array(p, shape=(n,)).copy()
        self.lib.spimdecon_free(p)
        return out


class OutOfBounds(IntEnum):
    """CUDASeparableConvolutionFunctions.OutOfBounds (ordinal = native code);
    MIRROR_SINGLE is this library's extension (code 3)."""
    ZERO = 0
    VALUE = 1
    EXTEND_BORDER_PIXELS = 2
    MIRROR_SINGLE = 3


SUPPORTED_KERNEL_SIZES = (7, 15, 31, 63, 127)  # CUDASeparableConvolutionFunctions.java:14


class CUDASeparableConvolution(CUDAStandardFunctions):
    """CUDASeparableConvolution.java:13-17 (returns the native boolean)."""

    def _conv(self, n, image, kx, ky, kz, w, h, d, cx, cy, cz, oob, oobv, dev) -> bool:
        f = getattr(self.lib, f"convolve_{n}")

        def kp(k):
            if k is None:
                return None
            k = np.ascontiguousarray(k, np.float32)
            assert k.size == n
            return k

        kx, ky, kz = kp(kx), kp(ky), kp(kz)
        keep = (kx, ky, kz)  # noqa: F841 (keep buffers alive during the call)
        r = f(fptr(image), fptr(kx) if kx is not None else None, fptr(ky) if ky is not None else None,
              fptr(kz) if kz is not None else None, int(w), int(h), int(d), int(bool(cx)),
              int(bool(cy)), int(bool(cz)), int(oob), float(oobv), int(dev))
        return bool(r)

    def convolve_7(self, *a):
        return self._conv(7, *a)

    def convolve_15(self, *a):
        return self._conv(15, *a)

    def convolve_31(self, *a):
        return self._conv(31, *a)

    def convolve_63(self, *a):
        return self._conv(63, *a)

    def convolve_127(self, *a):
        return self._conv(127, *a)


def create_gaussian_kernel_1d(sigma: float, normalize: bool = True) -> np.ndarray:
    """imglib1 Util.createGaussianKernel1DDouble (external; published algorithm),
    used by CUDASeparableConvolutionFunctions.getCUDAKernels (:208)."""
    if sigma <= 0:
        g = np.zeros(3)
        g[1] = 1.0
    else:
        size = max(3, 2 * int(3 * sigma + 0.5) + 1)
        two_sq = 2 * sigma * sigma
        g = np.zeros(size)
        c = size // 2
        for x in range(c, -1, -1):
            val = math.exp(-(x * x) / two_sq)
            g[c - x] = val
            g[c + x] = val
    if normalize:
        g = g / sum(g)
    return g


def get_cuda_kernels(sigma, supported=SUPPORTED_KERNEL_SIZES):
    """CUDASeparableConvolutionFunctions.getCUDAKernels (:199-233)."""
    kernels = [create_gaussian_kernel_1d(s, True) for s in sigma]
    longest = max(len(k) for k in kernels)
    size = min([s for s in supported if longest <= s], default=None)
    if size is None:
        return None
    out = []
    for k in kernels:
        p = np.zeros(size, np.float32)
        s = (size - len(k)) // 2
        p[s:s + len(k)] = k.astype(np.float32)
        out.append(p)
    return out


def gauss(img: np.ndarray, dim, sigma, oobs: OutOfBounds, oobs_value: float,
          cuda: CUDASeparableConvolution, device: int) -> bool:
    """CUDASeparableConvolutionFunctions.gauss (:127-197): in-place Gaussian of a
    flat x-fastest image of ``dim`` (x, y[, z])."""
    n = len(dim)
    sig = [sigma] * n if np.isscalar(sigma) else list(sigma)
    if n == 0 or n > 3 or len(sig) != n:
        return False
    ks = get_cuda_kernels(sig)
    if ks is None:
        return False
    size = len(ks[0])
    w = dim[0]
    h = dim[1] if n > 1 else 1
    d = dim[2] if n > 2 else 1
    kx = ks[0]
    ky = ks[1] if n > 1 else None
    kz = ks[2] if n > 2 else None
    return cuda._conv(size, img, kx, ky, kz, w, h, d, kx is not None, ky is not None, kz is not None,
                      int(oobs), oobs_value, device)


# --------------------------------------------------------------------------- blocks

@dataclass
class Block:
    """CUDA/Block.java:67-100; vectors in ImgLib2 order (x, y, z)."""
    block_size: tuple
    offset: tuple
    effective_size: tuple
    effective_offset: tuple
    effective_local_offset: tuple

    def copy_block(self, source: np.ndarray, ext: str) -> np.ndarray:
        """Block.copyBlock (:114-153) from the extended source ('mirror' =
        extendMirrorSingle, 'one' = extendValue(1), 'zero')."""
        bx, by, bz = self.block_size
        ox, oy, oz = self.offset
        nz, ny, nx = source.shape
        zi, zin = _ext(np.arange(oz, oz + bz), nz, ext)
        yi, yin = _ext(np.arange(oy, oy + by), ny, ext)
        xi, xin = _ext(np.arange(ox, ox + bx), nx, ext)
        out = source[np.ix_(zi, yi, xi)].astype(np.float32)
        if ext != "mirror":
            inside = zin[:, None, None] & yin[None, :, None] & xin[None, None, :]
            out = np.where(inside, out, np.float32(1.0 if ext == "one" else 0.0)).astype(np.float32)
        return np.ascontiguousarray(out)

    def paste_block(self, target: np.ndarray, block: np.ndarray) -> None:
        """Block.pasteBlock (:155-195): only the effective region."""
        ex, ey, ez = self.effective_size
        eox, eoy, eoz = self.effective_offset
        lx, ly, lz = self.effective_local_offset
        target[eoz:eoz + ez, eoy:eoy + ey, eox:eox + ex] = block[lz:lz + ez, ly:ly + ey, lx:lx + ex]


def _ext(i, n, ext):
    inside = (i >= 0) & (i < n)
    if ext == "mirror":
        if n == 1:
            return np.zeros_like(i), np.ones_like(inside)
        p = 2 * (n - 1)
        j = np.mod(i, p)
        return np.where(j >= n, p - j, j), np.ones_like(inside)
    return np.clip(i, 0, n - 1), inside


class BlockGeneratorFixedSizePrecise:
    """BlockGeneratorFixedSizePrecise.java:25-101."""

    def __init__(self, block_size):
        self.block_size = tuple(int(b) for b in block_size)

    def divide_into_blocks(self, img_size, kernel_size):
        n = len(img_size)
        eff = [self.block_size[d] - kernel_size[d] + 1 for d in range(n)]
        if any(e <= 0 for e in eff):
            return None
        loc = tuple(kernel_size[d] // 2 for d in range(n))
        nb = [img_size[d] // eff[d] + (1 if img_size[d] % eff[d] else 0) for d in range(n)]
        blocks = []
        for idx in np.ndindex(*reversed(nb)):   # LocalizingZeroMinIntervalIterator: dim 0 fastest
            cur = list(reversed(idx))
            eo = [cur[d] * eff[d] for d in range(n)]
            off = tuple(eo[d] - kernel_size[d] // 2 for d in range(n))
            es = tuple(min(eff[d], img_size[d] - eo[d]) for d in range(n))
            blocks.append(Block(self.block_size, off, es, tuple(eo), loc))
        return blocks


def cuda_coordinates(c):
    """MVDeconFFTThreads.getCUDACoordinates (:136-144): reverse the dims."""
    return list(reversed(list(c)))


def convolve_blocks_cuda(image: np.ndarray, kernel: np.ndarray, block_size, ext: str,
                         cuda: CUDAFourierConvolution, device: int) -> np.ndarray:
    """MVDeconFFT.convolve{1,2} GPU branch (MVDeconFFT.java:415-423,503-510) with
    MVDeconFFTThreads.convolve{1,2}BlockCUDA (:52-94): copy (extended) ->
    convolution3DfftCUDAInPlace -> paste.  ext 'mirror' = convolve1, 'one' = convolve2."""
    image = np.ascontiguousarray(image, np.float32)
    kernel = np.ascontiguousarray(kernel, np.float32)
    nz, ny, nx = image.shape
    kz, ky, kx = kernel.shape
    gen = BlockGeneratorFixedSizePrecise(block_size)
    blocks = gen.divide_into_blocks((nx, ny, nz), (kx, ky, kz))
    if blocks is None:
        raise ValueError("block smaller than kernel")
    result = np.empty_like(image)
    for b in blocks:
        blk = b.copy_block(image, ext)
        cuda.convolution3DfftCUDAInPlace(blk, cuda_coordinates(blk.shape[::-1]), kernel,
                                         cuda_coordinates(kernel.shape[::-1]), device)
        b.paste_block(result, blk)
    return result
