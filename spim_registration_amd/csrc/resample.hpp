// resample.hpp -- shared pieces of the affine resampling kernels (input_prep.hip,
// psf.hip): the imglib2 AffineTransform3D inverse and NLinearInterpolator3D on
// FloatType over the out-of-bounds strategies the reference uses
// (extendMirrorSingle, extendPeriodic, extendZero), restated after
// oracle/input_ref.py (parity unpinned: imglib2 is not in the reference tree).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "common.hpp"

namespace spimdecon {

struct AffineInv {
    double inv[9];   // inverse of the 3x3 part, row-major
    double tr[3];    // translation of the model
    double full[12]; // full inverse, row-major 3x4
};

enum Ext { kExtMirror = 0, kExtPeriodic = 1, kExtZero = 2 };

__device__ __forceinline__ int mirror1(int i, int n) {
    if (n == 1) return 0;
    const int p = 2 * (n - 1);
    int j = i % p;
    if (j < 0) j += p;
    return j >= n ? p - j : j;
}

template <int EXT>
__device__ __forceinline__ float ext_at(const float* src, int sx, int sy, int sz, int x, int y, int z) {
    if constexpr (EXT == kExtMirror) {
        x = mirror1(x, sx);
        y = mirror1(y, sy);
        z = mirror1(z, sz);
    } else if constexpr (EXT == kExtPeriodic) {
        x %= sx;
        y %= sy;
        z %= sz;
        x += x < 0 ? sx : 0;
        y += y < 0 ? sy : 0;
        z += z < 0 ? sz : 0;
    } else {
        if (x < 0 || y < 0 || z < 0 || x >= sx || y >= sy || z >= sz) return 0.0f;
    }
    return src[(int64_t(z) * sy + y) * sx + x];
}

// NLinearInterpolator3D: weights in double, FloatType.mul(double) / add per corner,
// corner order 000, 100, 110, 010, 011, 111, 101, 001
template <int EXT>
__device__ float nlinear_at(const float* src, int sx, int sy, int sz, double p0, double p1, double p2) {
    const double f0 = floor(p0), f1 = floor(p1), f2 = floor(p2);
    const int xa = int(f0), ya = int(f1), za = int(f2);
    const int xb = xa + 1, yb = ya + 1, zb = za + 1;
    const double w0 = p0 - f0, w1 = p1 - f1, w2 = p2 - f2;
    const double i0 = 1.0 - w0, i1 = 1.0 - w1, i2 = 1.0 - w2;
    if (xa >= 0 && ya >= 0 && za >= 0 && xb < sx && yb < sy && zb < sz) {
        // every corner inside: one base index, no per-corner extension arithmetic
        const float* b = src + (int64_t(za) * sy + ya) * sx + xa;
        const int64_t py = sx, pz = int64_t(sx) * sy;
        float acc = float(double(b[0]) * (i0 * i1 * i2));
        acc = acc + float(double(b[1]) * (w0 * i1 * i2));
        acc = acc + float(double(b[py + 1]) * (w0 * w1 * i2));
        acc = acc + float(double(b[py]) * (i0 * w1 * i2));
        acc = acc + float(double(b[pz + py]) * (i0 * w1 * w2));
        acc = acc + float(double(b[pz + py + 1]) * (w0 * w1 * w2));
        acc = acc + float(double(b[pz + 1]) * (w0 * i1 * w2));
        acc = acc + float(double(b[pz]) * (i0 * i1 * w2));
        return acc;
    }
    auto at = [&](int x, int y, int z) { return double(ext_at<EXT>(src, sx, sy, sz, x, y, z)); };
    float acc = float(at(xa, ya, za) * (i0 * i1 * i2));
    acc = acc + float(at(xb, ya, za) * (w0 * i1 * i2));
    acc = acc + float(at(xb, yb, za) * (w0 * w1 * i2));
    acc = acc + float(at(xa, yb, za) * (i0 * w1 * i2));
    acc = acc + float(at(xa, yb, zb) * (i0 * w1 * w2));
    acc = acc + float(at(xb, yb, zb) * (w0 * w1 * w2));
    acc = acc + float(at(xb, ya, zb) * (w0 * i1 * w2));
    acc = acc + float(at(xa, ya, zb) * (i0 * i1 * w2));
    return acc;
}

// (x, y, z) of a flat x-fastest index: 32-bit divisions when the volume allows
// (a 64-bit division is a ~100-instruction software routine on the GPU)
// Output traversal in (x, z) tiles of kTileX x kTileZ voxels, one y row each, y fastest
// over the blocks: the voxels of a block then sample a compact source region (a rotated
// view's x runs cross the source's z planes diagonally: a 256-voxel x run touched ~180
// 2.4-MB planes, a 32 x 8 tile ~30) while each block still writes whole 128-B row
// segments.  Per-voxel arithmetic is unchanged (bit-identical output).
constexpr int kTileX = 32, kTileZ = 8;
inline int64_t tiled_blocks(int64_t nx, int64_t ny, int64_t nz) {
    return ny * ((nx + kTileX - 1) / kTileX) * ((nz + kTileZ - 1) / kTileZ);
}
__device__ __forceinline__ bool tiled_xyz(int64_t nx, int64_t ny, int64_t nz, int64_t& x, int64_t& y, int64_t& z) {
    const int64_t b = blockIdx.x;
    const int64_t ntx = (nx + kTileX - 1) / kTileX;
    y = b % ny;
    const int64_t r = b / ny;
    x = (r % ntx) * kTileX + threadIdx.x % kTileX;
    z = (r / ntx) * kTileZ + threadIdx.x / kTileX;
    return x < nx && z < nz;
}

__device__ __forceinline__ void flat_xyz(int64_t i, int64_t nx, int64_t ny, int64_t n, int64_t& x, int64_t& y,
                                         int64_t& z) {
    if (n < (int64_t(1) << 32)) {
        const uint32_t ii = uint32_t(i), ux = uint32_t(nx), uy = uint32_t(ny);
        const uint32_t q = ii / ux;
        x = ii - q * ux;
        z = q / uy;
        y = q - uint32_t(z) * uy;
    } else {
        x = i % nx;
        y = (i / nx) % ny;
        z = i / (nx * ny);
    }
}

inline AffineInv invert_model(const double* m) {
    const double a00 = m[0], a01 = m[1], a02 = m[2], a10 = m[4], a11 = m[5], a12 = m[6];
    const double a20 = m[8], a21 = m[9], a22 = m[10];
    const double det = a00 * (a11 * a22 - a12 * a21) - a01 * (a10 * a22 - a12 * a20) +
                       a02 * (a10 * a21 - a11 * a20);
    SD_CHECK(det != 0.0 && std::isfinite(det), SPIMDECON_ERR_ARG, "affine model is not invertible");
    AffineInv r{};
    r.inv[0] = (a11 * a22 - a12 * a21) / det;
    r.inv[1] = (a02 * a21 - a01 * a22) / det;
    r.inv[2] = (a01 * a12 - a02 * a11) / det;
    r.inv[3] = (a12 * a20 - a10 * a22) / det;
    r.inv[4] = (a00 * a22 - a02 * a20) / det;
    r.inv[5] = (a02 * a10 - a00 * a12) / det;
    r.inv[6] = (a10 * a21 - a11 * a20) / det;
    r.inv[7] = (a01 * a20 - a00 * a21) / det;
    r.inv[8] = (a00 * a11 - a01 * a10) / det;
    r.tr[0] = m[3];
    r.tr[1] = m[7];
    r.tr[2] = m[11];
    for (int row = 0; row < 3; ++row) {
        for (int c = 0; c < 3; ++c) r.full[4 * row + c] = r.inv[3 * row + c];
        r.full[4 * row + 3] =
            -(r.inv[3 * row] * r.tr[0] + r.inv[3 * row + 1] * r.tr[1] + r.inv[3 * row + 2] * r.tr[2]);
    }
    return r;
}


}  // namespace spimdecon
