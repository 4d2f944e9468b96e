// fftconv.hip -- fused spectral-convolution engine (see fftconv.hpp).
//
// Semantics restated (paths under /root/reference/src/main/java/):
//   convolve1 / convolve2   spim/process/fusion/deconvolution/MVDeconFFT.java:363-535
//                           (true convolution, kernel centre at dim/2, extendMirrorSingle
//                            for psi, extendValue(1) for the quotient)
//   computeQuotient         spim/process/fusion/deconvolution/MVDeconvolution.java:473-525
//   computeFinalValues      spim/process/fusion/deconvolution/MVDeconvolution.java:582-705
#include "fftconv.hpp"

#include <climits>
#include "rl_math.hpp"

#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <cstdio>
#include <cstring>

namespace spimdecon {

namespace {

// ------------------------------------------------------------------ small helpers

// The FFT arithmetic below may contract into FMAs (the build is -ffp-contract=off
// so that the RL pointwise steps keep the reference's float op order; those use
// explicit __f*_rn intrinsics).  The spectra are not bit-matched to any
// reference anyway, and FMA is the more accurate of the two.
// Written on 2-wide float vectors so that every complex op is one packed VALU op
// (v_pk_mul/add/fma_f32 with operand swizzles and negations folded in): a complex
// multiply is a v_pk_mul + a v_pk_fma instead of scalar ops and register moves.
typedef float sd_v2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ sd_v2 v2_(float2 a) { return sd_v2{a.x, a.y}; }
__device__ __forceinline__ float2 f2_(sd_v2 a) { return make_float2(a.x, a.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    const sd_v2 A = v2_(a), B = v2_(b);
    const sd_v2 t = A.xx * B;                                              // (ax bx, ax by)
    return f2_(__builtin_elementwise_fma(A.yy, sd_v2{-B.y, B.x}, t));      // (- ay by, + ay bx)
}
// contract(fast): a scale feeding an add (radix-3/5/7 butterflies) may fuse into one
// v_pk_fma (the build is -ffp-contract=off for the RL pointwise steps)
__device__ __forceinline__ float2 cadd(float2 a, float2 b) {
#pragma clang fp contract(fast)
    return f2_(v2_(a) + v2_(b));
}
__device__ __forceinline__ float2 csub(float2 a, float2 b) {
#pragma clang fp contract(fast)
    return f2_(v2_(a) - v2_(b));
}
__device__ __forceinline__ float2 cscale(float2 a, float s) {
#pragma clang fp contract(fast)
    return f2_(v2_(a) * sd_v2{s, s});
}
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) {
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}
// a + mul_mi<INV>(d) and a - mul_mi<INV>(d) as ONE v_pk_fma (d swizzled, times
// (+-1, -+1), plus a): exact like the add, but without the xor + mov the separate
// swap-and-negate cost
template <bool INV>
__device__ __forceinline__ float2 cadd_mi(float2 a, float2 d) {
    const sd_v2 D = v2_(d);
    return f2_(__builtin_elementwise_fma(D.yx, INV ? sd_v2{-1.0f, 1.0f} : sd_v2{1.0f, -1.0f}, v2_(a)));
}
template <bool INV>
__device__ __forceinline__ float2 csub_mi(float2 a, float2 d) {
    const sd_v2 D = v2_(d);
    return f2_(__builtin_elementwise_fma(D.yx, INV ? sd_v2{1.0f, -1.0f} : sd_v2{-1.0f, 1.0f}, v2_(a)));
}

template <int S>
__device__ __forceinline__ float ldv(const void* p, int64_t i) {
    if constexpr (S == 0) return static_cast<const float*>(p)[i];
    else return __half2float(static_cast<const __half*>(p)[i]);
}

// ------------------------------------------------------------------ radix-R DFTs

template <int R, bool INV>
__device__ __forceinline__ void dft(float2* a) {
    if constexpr (R == 2) {
        const float2 t = a[0];
        a[0] = cadd(t, a[1]);
        a[1] = csub(t, a[1]);
    } else if constexpr (R == 3) {
        const float2 s = cadd(a[1], a[2]);
        const float2 m = csub(a[0], cscale(s, 0.5f));
        const float2 d = cscale(csub(a[1], a[2]), 0.86602540378443864676f);
        a[0] = cadd(a[0], s);
        a[1] = cadd_mi<INV>(m, d);  // m - i*d forward
        a[2] = csub_mi<INV>(m, d);
    } else if constexpr (R == 4) {
        const float2 s0 = cadd(a[0], a[2]), d0 = csub(a[0], a[2]);
        const float2 s1 = cadd(a[1], a[3]), d1 = csub(a[1], a[3]);
        a[0] = cadd(s0, s1);
        a[2] = csub(s0, s1);
        a[1] = cadd_mi<INV>(d0, d1);
        a[3] = csub_mi<INV>(d0, d1);
    } else if constexpr (R == 5) {
        constexpr float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
        constexpr float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
        const float2 b1 = cadd(a[1], a[4]), b2 = cadd(a[2], a[3]);
        const float2 d1 = csub(a[1], a[4]), d2 = csub(a[2], a[3]);
        const float2 m1 = cadd(a[0], cadd(cscale(b1, c1), cscale(b2, c2)));
        const float2 m2 = cadd(a[0], cadd(cscale(b1, c2), cscale(b2, c1)));
        const float2 n1 = cadd(cscale(d1, s1), cscale(d2, s2));
        const float2 n2 = csub(cscale(d1, s2), cscale(d2, s1));
        a[0] = cadd(a[0], cadd(b1, b2));
        a[1] = cadd_mi<INV>(m1, n1);
        a[4] = csub_mi<INV>(m1, n1);
        a[2] = cadd_mi<INV>(m2, n2);
        a[3] = csub_mi<INV>(m2, n2);
    } else {
        static_assert(R == 7, "radix 2, 3, 4, 5, 7 only");
        constexpr float c1 = 0.62348980185873353053f, c2 = -0.22252093395631440429f,
                        c3 = -0.90096886790241912624f;
        constexpr float s1 = 0.78183148246802980871f, s2 = 0.97492791218182360702f,
                        s3 = 0.43388373911755812048f;
        const float2 b1 = cadd(a[1], a[6]), b2 = cadd(a[2], a[5]), b3 = cadd(a[3], a[4]);
        const float2 d1 = csub(a[1], a[6]), d2 = csub(a[2], a[5]), d3 = csub(a[3], a[4]);
        const float2 r1 = cadd(a[0], cadd(cscale(b1, c1), cadd(cscale(b2, c2), cscale(b3, c3))));
        const float2 r2 = cadd(a[0], cadd(cscale(b1, c2), cadd(cscale(b2, c3), cscale(b3, c1))));
        const float2 r3 = cadd(a[0], cadd(cscale(b1, c3), cadd(cscale(b2, c1), cscale(b3, c2))));
        const float2 i1 = cadd(cscale(d1, s1), cadd(cscale(d2, s2), cscale(d3, s3)));
        const float2 i2 = csub(cscale(d1, s2), cadd(cscale(d2, s3), cscale(d3, s1)));
        const float2 i3 = cadd(csub(cscale(d1, s3), cscale(d2, s1)), cscale(d3, s2));
        a[0] = cadd(a[0], cadd(b1, cadd(b2, b3)));
        a[1] = cadd_mi<INV>(r1, i1);
        a[6] = csub_mi<INV>(r1, i1);
        a[2] = cadd_mi<INV>(r2, i2);
        a[5] = csub_mi<INV>(r2, i2);
        a[3] = cadd_mi<INV>(r3, i3);
        a[4] = csub_mi<INV>(r3, i3);
    }
}

// One ping-pong Stockham stage: `ncols` interleaved transforms, element n of
// column c at buf[n * ES + c * CS].  Thread (c, g) walks butterflies
// j = g, g + TPC, ... of column c; one butterfly (R values) in registers at a time.
template <int R, bool INV>
__device__ __forceinline__ void stage_pp(const float2* __restrict__ src, float2* __restrict__ dst,
                                         const float2* __restrict__ tw, int L, int Ns, int c, int g,
                                         int TPC, int ES, int CS) {
    const int nb = L / R;
    const int step = L / (Ns * R);
    for (int j = g; j < nb; j += TPC) {
        const int k = j % Ns;
        float2 v[R];
#pragma unroll
        for (int t = 0; t < R; ++t) v[t] = src[(j + t * nb) * ES + c * CS];
        if (Ns > 1) {
#pragma unroll
            for (int t = 1; t < R; ++t) {
                float2 w = tw[t * k * step];
                if (INV) w.y = -w.y;
                v[t] = cmul(v[t], w);
            }
        }
        dft<R, INV>(v);
        const int base = (j - k) * R + k;
#pragma unroll
        for (int t = 0; t < R; ++t) dst[(base + t * Ns) * ES + c * CS] = v[t];
    }
}

// LDS hand-off between the lanes of one wave (a wave's LDS operations execute
// in order; this only stops the compiler from moving them across).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Full 1D FFT ping-ponging between a and b; returns the buffer holding the result.
// Every stage ends with a block barrier (callers must call it uniformly), or a
// wave-local one when WAVE (the transform is private to one wave).
template <bool INV, bool WAVE = false>
__device__ __forceinline__ float2* fft_pp(float2* a, float2* b, const float2* tw, const Fft1D& f, int c, int g,
                          int TPC, int ES, int CS, bool active) {
    int Ns = 1;
    float2* src = a;
    float2* dst = b;
    for (int s = 0; s < f.ns; ++s) {
        const int R = f.radix(s);
        if (active) {
            switch (R) {
                case 2: stage_pp<2, INV>(src, dst, tw, f.L, Ns, c, g, TPC, ES, CS); break;
                case 3: stage_pp<3, INV>(src, dst, tw, f.L, Ns, c, g, TPC, ES, CS); break;
                case 4: stage_pp<4, INV>(src, dst, tw, f.L, Ns, c, g, TPC, ES, CS); break;
                case 5: stage_pp<5, INV>(src, dst, tw, f.L, Ns, c, g, TPC, ES, CS); break;
                default: stage_pp<7, INV>(src, dst, tw, f.L, Ns, c, g, TPC, ES, CS); break;
            }
        }
        if constexpr (WAVE) wave_sync();
        else __syncthreads();
        Ns *= R;
        float2* t = src;
        src = dst;
        dst = t;
    }
    return src;
}

// ------------------------------------------------------------------ X pass (rows)

enum XMode { XM_PSI = 0, XM_QUOT = 1, XM_UPDATE = 2, XM_KERNEL = 3 };

struct XArgs {
    SlabGeom g;
    int64_t Hx, Hp;
    Fft1D fx;
    const int* row_mirror;
    const int* row_one;
    const float2* Cin;
    float2* Cout;
    const float* psi_in;
    float* psi_out;
    const void* img;
    const void* w;
    double lambda;
    double* partials;
    const float* kern;
    int kx, ky, kz;
    float kscale;
    uint32_t spec_bytes;  // k_xrows buffer ranges (< 2 GiB each)
    uint32_t nvox;
    // packed row pairs processed by this launch: [pb0, pb0 + pn0) then [pb1, pb1 + pn1)
    int pb0, pn0, pb1, pn1;
};

// linear index of a launch -> packed row pair (-1 past the ranges)
__device__ __forceinline__ int x_pair(const XArgs& a, int i) {
    return i < a.pn0 ? a.pb0 + i : (i - a.pn0 < a.pn1 ? a.pb1 + (i - a.pn0) : -1);
}

constexpr int kXThreads = 256;             // four waves; one packed row pair per wave
constexpr int kXPairs = kXThreads / 64;

// per-wave LDS: A[Mx + 2] | B[Mx + 2]; block: tw[Mx]
__host__ __device__ inline int x_wave_elems(int Mx) { return 2 * (Mx + 2); }

template <int MODE, int S>
__global__ __launch_bounds__(kXThreads) void k_xpass(XArgs a) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const SlabGeom& g = a.g;
    const int Mx = int(g.Mx);
    const int Hx = int(a.Hx);
    const int Hp = int(a.Hp);
    const int nx = int(g.nx);
    const int cx = g.cx;
    float2* tw = smem;
    const int wv = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    float2* A = smem + Mx + wv * x_wave_elems(Mx);
    float2* B = A + Mx + 2;
    for (int i = threadIdx.x; i < Mx; i += kXThreads) tw[i] = a.fx.tw[i];
    const int nrows = int(g.My * g.Mz);
    const int nlin = a.pn0 + a.pn1;
    double ssum = 0.0;
    float smax = -1.0f;
    __syncthreads();
    for (int pg = blockIdx.x; pg * kXPairs < nlin; pg += gridDim.x) {
        const int pair = x_pair(a, pg * kXPairs + wv);
        const bool active = pair >= 0;
        const int r0 = 2 * pair, r1 = 2 * pair + 1;
        const bool valid0 = active && r0 < nrows, valid1 = active && r1 < nrows;
        const int sm0 = valid0 ? a.row_mirror[r0] : -1, sm1 = valid1 ? a.row_mirror[r1] : -1;
        const int so0 = valid0 ? a.row_one[r0] : -1, so1 = valid1 ? a.row_one[r1] : -1;
        float2* Z = A;  // buffer holding the real-space row pair (x = row 0, y = row 1)
        // ---------------- inverse half: previous convolution result
        if constexpr (MODE == XM_QUOT || MODE == XM_UPDATE) {
            int p0 = -1, p1 = -1;  // padded rows holding the needed convolution results
            if constexpr (MODE == XM_QUOT) {
                p0 = so0 >= 0 ? r0 : -1;
                p1 = so1 >= 0 ? r1 : -1;
            } else {
                p0 = sm0 >= 0 ? (sm0 / int(g.ny)) * int(g.My) + sm0 % int(g.ny) : -1;
                p1 = sm1 >= 0 ? (sm1 / int(g.ny)) * int(g.My) + sm1 % int(g.ny) : -1;
            }
            const float2* row0 = a.Cin + int64_t(p0) * Hp;
            const float2* row1 = a.Cin + int64_t(p1) * Hp;
            for (int k = lane; k < Hx; k += 64) {
                B[k] = p0 >= 0 ? row0[k] : make_float2(0.f, 0.f);
                B[Hx + k] = p1 >= 0 ? row1[k] : make_float2(0.f, 0.f);
            }
            __syncthreads();
            for (int k = lane; k < Mx; k += 64) {
                float2 xa, xb;
                if (k <= Mx / 2) {
                    xa = B[k];
                    xb = B[Hx + k];
                    if (k == 0 || k == Mx / 2) {
                        xa.y = 0.f;
                        xb.y = 0.f;
                    }
                } else {
                    xa = B[Mx - k];
                    xb = B[Hx + Mx - k];
                    xa.y = -xa.y;
                    xb.y = -xb.y;
                }
                A[k] = make_float2(xa.x - xb.y, xa.y + xb.x);
            }
            __syncthreads();
            Z = fft_pp<true>(A, B, tw, a.fx, 0, lane, 64, 1, 0, active);
        }
        float2* O = (Z == A) ? B : A;  // the other buffer
        // ---------------- pointwise: real rows -> Z (in place)
        if constexpr (MODE == XM_PSI) {
            const float* p0 = a.psi_in + int64_t(sm0 < 0 ? 0 : sm0) * nx;
            const float* p1 = a.psi_in + int64_t(sm1 < 0 ? 0 : sm1) * nx;
            for (int qx = lane; qx < Mx; qx += 64) {
                const int sx = qx < nx + cx ? qx : qx - Mx;
                const int lx = int(mirror_idx(sx, nx));
                Z[qx] = make_float2(sm0 >= 0 ? p0[lx] : 0.f, sm1 >= 0 ? p1[lx] : 0.f);
            }
        } else if constexpr (MODE == XM_KERNEL) {
            for (int qx = lane; qx < Mx; qx += 64) {
                float v[2] = {0.f, 0.f};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int r = h == 0 ? r0 : r1;
                    if (!(h == 0 ? valid0 : valid1)) continue;
                    const int qz = r / int(g.My), qy = r % int(g.My);
                    const int jz = (qz + a.kz / 2) % int(g.Mz), jy = (qy + a.ky / 2) % int(g.My);
                    const int jx = (qx + a.kx / 2) % Mx;
                    if (jz < a.kz && jy < a.ky && jx < a.kx)
                        v[h] = a.kern[(int64_t(jz) * a.ky + jy) * a.kx + jx] * a.kscale;
                }
                Z[qx] = make_float2(v[0], v[1]);
            }
        } else if constexpr (MODE == XM_QUOT) {
            const bool live0 = valid0 && sm0 != -1, live1 = valid1 && sm1 != -1;
            for (int qx = lane; qx < Mx; qx += 64) {
                const float2 bz = Z[qx];
                float q0 = live0 ? 1.0f : 0.0f, q1 = live1 ? 1.0f : 0.0f;  // constant-1 extension
                if (qx < nx) {
                    if (so0 >= 0) {
                        const float iv = ldv<S>(a.img, int64_t(so0) * nx + qx);
                        if (iv > 0.0f) q0 = __fdiv_rn(iv, bz.x);
                    }
                    if (so1 >= 0) {
                        const float iv = ldv<S>(a.img, int64_t(so1) * nx + qx);
                        if (iv > 0.0f) q1 = __fdiv_rn(iv, bz.y);
                    }
                }
                Z[qx] = make_float2(q0, q1);
            }
        } else {  // XM_UPDATE
            for (int qx = lane; qx < nx; qx += 64) {
                const float2 iz = Z[qx];
                float o0 = 0.f, o1 = 0.f;
                if (sm0 >= 0) {
                    const int64_t vi = int64_t(sm0) * nx + qx;
                    const float last = a.psi_in[vi];
                    o0 = next_value(last, iz.x, ldv<S>(a.w, vi), a.lambda);
                    if (so0 >= 0) {  // interior row: the one writer of psi_out
                        a.psi_out[vi] = o0;
                        const float ch = fabsf(__fsub_rn(o0, last));
                        ssum += (double)ch;
                        smax = fmaxf(smax, ch);
                    }
                }
                if (sm1 >= 0) {
                    const int64_t vi = int64_t(sm1) * nx + qx;
                    const float last = a.psi_in[vi];
                    o1 = next_value(last, iz.y, ldv<S>(a.w, vi), a.lambda);
                    if (so1 >= 0) {
                        a.psi_out[vi] = o1;
                        const float ch = fabsf(__fsub_rn(o1, last));
                        ssum += (double)ch;
                        smax = fmaxf(smax, ch);
                    }
                }
                Z[qx] = make_float2(o0, o1);
            }
            __syncthreads();
            for (int qx = nx + lane; qx < Mx; qx += 64) {
                const int sx = qx < nx + cx ? qx : qx - Mx;
                Z[qx] = Z[mirror_idx(sx, nx)];
            }
        }
        __syncthreads();
        if (MODE == XM_UPDATE && a.Cout == nullptr) continue;
        // ---------------- forward half
        float2* F = fft_pp<false>(Z, O, tw, a.fx, 0, lane, 64, 1, 0, active);
        const bool w0 = valid0 && sm0 != -1, w1 = valid1 && sm1 != -1;
        float2* out0 = a.Cout + int64_t(r0) * Hp;
        float2* out1 = a.Cout + int64_t(r1) * Hp;
        for (int k = lane; k < Hp; k += 64) {
            float2 xa = make_float2(0.f, 0.f), xb = make_float2(0.f, 0.f);
            if (k < Hx) {
                const float2 zk = F[k];
                const float2 zm = F[k == 0 ? 0 : Mx - k];
                xa = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
                xb = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
            }
            if (w0) out0[k] = xa;
            if (w1) out1[k] = xb;
        }
        __syncthreads();
    }
    if constexpr (MODE == XM_UPDATE) {
        __shared__ double sh_sum[kXThreads / 64];
        __shared__ float sh_max[kXThreads / 64];
        for (int off = 32; off > 0; off >>= 1) {
            ssum += __shfl_xor(ssum, off, 64);
            smax = fmaxf(smax, __shfl_xor(smax, off, 64));
        }
        if (lane == 0) {
            sh_sum[wv] = ssum;
            sh_max[wv] = smax;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < kXThreads / 64; ++i) {
                ssum += sh_sum[i];
                smax = fmaxf(smax, sh_max[i]);
            }
            a.partials[2 * blockIdx.x] = ssum;
            a.partials[2 * blockIdx.x + 1] = (double)smax;
        }
    }
}

// ------------------------------------------------------------------ column passes

constexpr int kCThreads = 1024;

// dynamic LDS: A[L*TX] | B[L*TX] | tw[L]
// AXIS 1 = y (stride Hp), 2 = z (stride My*Hp).  ZMODE: 0 = one FFT (fwd/inv by INV),
// 1 = fwd * K * inv.
#include "fftconv_col.inc"
#include "fft_reg.inc"
#include "fftconv_2f.inc"
#include "fftconv_x.inc"
#include "fftconv_xt.inc"
#include "fftconv_zd.inc"

// ------------------------------------------------------------------ host side

Fft1D make_fft(int L, bool allow_2f, DBuf<float2>& tw, hipStream_t s) {
    Fft1D f;
    f.L = L;
    int m = L;
    auto push = [&](int r) {
        SD_CHECK(f.ns < kFftMaxStages, SPIMDECON_ERR_ARG, "too many FFT stages");
        f.radix_packed |= uint64_t(r) << (4 * f.ns);
        f.ns++;
        m /= r;
    };
    while (m % 4 == 0) push(4);
    while (m % 2 == 0) push(2);
    while (m % 3 == 0) push(3);
    while (m % 5 == 0) push(5);
    while (m % 7 == 0) push(7);
    SD_CHECK(m == 1, SPIMDECON_ERR_ARG, "FFT length " + std::to_string(L) + " is not 2,3,5,7-smooth");
#define SD_2F_LOOKUP(A, B) \
    if (L == (A) * (B)) { f.n1 = (A); f.n2 = (B); }
    if (allow_2f) { SD_2F_SIZES(SD_2F_LOOKUP) }
#undef SD_2F_LOOKUP
    std::vector<float2> h(L);
    for (int i = 0; i < L; ++i) {
        const double ang = -2.0 * M_PI * double(i) / double(L);
        h[i] = make_float2(float(std::cos(ang)), float(std::sin(ang)));
    }
    tw.alloc(L);
    SD_HIP(hipMemcpyAsync(tw.p, h.data(), L * sizeof(float2), hipMemcpyHostToDevice, s));
    SD_HIP(hipStreamSynchronize(s));
    f.tw = tw.p;
    return f;
}

size_t x_lds(const SpectralPlan& p) {
    return size_t(p.g.Mx + kXPairs * x_wave_elems(int(p.g.Mx))) * sizeof(float2);
}

// x-pass grid, shared by k_xpass and k_xrows (also the number of stats
// partials an update pass writes)
unsigned x_grid(const XArgs& a) {
    const int64_t b = ceil_div(int64_t(a.pn0) + a.pn1, kXPairs);
    return unsigned(std::max<int64_t>(1, std::min<int64_t>(b, 256 * 8)));
}

XArgs base_args(const SpectralPlan& p) {
    XArgs a{};
    SD_CHECK(p.g.My * p.g.Mz < (int64_t(1) << 30), SPIMDECON_ERR_ARG, "too many rows");
    a.pb0 = 0;
    a.pn0 = int((p.g.My * p.g.Mz + 1) / 2);
    a.pb1 = 0;
    a.pn1 = 0;
    a.g = p.g;
    a.Hx = p.Hx;
    a.Hp = p.Hp;
    a.fx = p.fx;
    a.row_mirror = p.row_mirror.p;
    a.row_one = p.row_one.p;
    return a;
}

// two-factor x tiles: lengths >= 256 of the fast-path table
#define SD_X2F_SIZES(M) M(16, 16) M(16, 24) M(16, 32) M(20, 27) M(24, 24) M(20, 32) M(25, 32) M(30, 35) M(42, 50)

bool aligned_to(const void* q, size_t n) { return q == nullptr || reinterpret_cast<uintptr_t>(q) % n == 0; }

// buffer ranges for k_xrows / k_xtile; false when a buffer exceeds the 31-bit range
bool x_buffer_args(const XArgs& a, Store st, const SpectralPlan& p, XArgs& b) {
    const size_t va = st == Store::F32 ? 16 : 8;
    const uint64_t spec_bytes = uint64_t(p.spectrum_elems()) * sizeof(float2);
    const uint64_t nvox = uint64_t(p.g.nx) * p.g.ny * p.g.nz;
    if (p.g.nx % 4 != 0 || !aligned_to(a.img, va) || !aligned_to(a.w, va) || !aligned_to(a.psi_in, 16) ||
        !aligned_to(a.psi_out, 16) || spec_bytes >= kOOB || nvox * 4 >= kOOB)
        return false;
    b = a;
    b.spec_bytes = uint32_t(spec_bytes);
    b.nvox = uint32_t(nvox);
    return true;
}

// k_xtile for two-factor lengths; returns the grid, 0 when it does not apply.
// xt_np row pairs per tile, one tile per block: fresh blocks keep loading while the resident
// ones transform (quotient 0.40 vs 0.43 ms with 16 pairs and 0.45 with 4, update 0.52 vs
// 0.58 / 0.54 ms at 540; at L = 1050 quotient 0.90 vs 1.05 ms with 16 pairs; grid-stride
// blocks in lock step measured slower)
template <int MODE>
unsigned launch_xtile(const XArgs& a, Store st, const SpectralPlan& p, hipStream_t s) {
    XArgs b;
    if (!p.fx.n1 || !x_buffer_args(a, st, p, b)) return 0;
    const int L = int(p.g.Mx);
    const int NP = xt_np(MODE, L);
    const size_t lds = xt_lds(L, NP, xt_twg(L, NP));
    if (lds > 160 * 1024) return 0;
    const unsigned grid = unsigned(std::max<int64_t>(1, ceil_div(int64_t(a.pn0) + a.pn1, int64_t(NP))));
    const int sv = st == Store::F32 ? 0 : 1;
    bool done = false;
    const bool tik = MODE == XM_UPDATE && a.lambda > 0.0;
#define SD_XT(SV, A, B, TK)                                                                                \
    if (!done && sv == SV && L == (A) * (B) && tik == TK) {                                               \
        constexpr int TRv = SD_2F_TR(A, B);                                                               \
        constexpr int NPv = xt_np(MODE, (A) * (B));                                                       \
        auto kfn = &k_xtile<MODE, SV, A, B, TK, NPv, TRv>;                                                \
        SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                   int(lds)));                                                            \
        hipLaunchKernelGGL(kfn, dim3(grid), dim3(NPv * TRv), lds, s, b);                                  \
        done = true;                                                                                      \
    }
#define SD_XT_S(A, B) \
    SD_XT(0, A, B, false) SD_XT(1, A, B, false) if constexpr (MODE == XM_UPDATE) { SD_XT(0, A, B, true) SD_XT(1, A, B, true) }
    SD_X2F_SIZES(SD_XT_S)
#undef SD_XT_S
#undef SD_XT
    if (!done) return 0;
    SD_HIP(hipGetLastError());
#if SD_XT_STAMPS
    {
        unsigned long long h[3][8];
        SD_HIP(hipStreamSynchronize(s));
        SD_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_xt_stamp), sizeof(h)));
        const unsigned long long n = std::max(1ull, h[MODE][7]);
        std::fprintf(stderr, "[xt_stamp] L=%d mode=%d fp16=%d tiles=%llu cycles/tile: load %llu inv %llu rl %llu fwd %llu store %llu prologue %llu\n",
                     L, MODE, sv, h[MODE][7], h[MODE][0] / n, h[MODE][1] / n, h[MODE][2] / n, h[MODE][3] / n,
                     h[MODE][4] / n, h[MODE][5] / n);
        std::memset(h, 0, sizeof(h));
        SD_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_xt_stamp), h, sizeof(h)));
    }
#endif
    return grid;
}

// k_xrows when the rows allow 16-B voxel access; returns the grid, 0 = use k_xpass
template <int MODE>
unsigned launch_xrows(const XArgs& a, Store st, const SpectralPlan& p, hipStream_t s) {
    const int nx = int(p.g.nx);
    const int U = int(ceil_div(p.Hp / 2, 64));
    const int UV = int(ceil_div(nx / 4, 64));
    XArgs b;
    if (U > 4 || (UV != U && UV != U - 1) || !x_buffer_args(a, st, p, b)) return 0;
    const int Mx = int(p.g.Mx);
    const size_t lds = size_t(Mx + kXPairs * xrows_wave_elems(Mx, false)) * sizeof(float2);
    SD_CHECK(lds <= 160 * 1024, SPIMDECON_ERR_ARG, "x pass LDS too large");
    SD_CHECK(p.g.My * p.g.Mz < (int64_t(1) << 30), SPIMDECON_ERR_ARG, "too many rows");
    const unsigned grid = x_grid(a);
    const int sv = st == Store::F32 ? 0 : 1;
    bool done = false;
#define SD_XR(SV, UU, VV)                                                                               \
    if (!done && sv == SV && U == UU && UV == VV) {                                                     \
        SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_xrows<MODE, SV, UU, VV, 0, 0>),    \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));              \
        hipLaunchKernelGGL((k_xrows<MODE, SV, UU, VV, 0, 0>), dim3(grid), dim3(kXThreads), lds, s, b); \
        done = true;                                                                                    \
    }
#define SD_XR_S(SV) SD_XR(SV, 1, 1) SD_XR(SV, 2, 1) SD_XR(SV, 2, 2) SD_XR(SV, 3, 2) \
                    SD_XR(SV, 3, 3) SD_XR(SV, 4, 3) SD_XR(SV, 4, 4)
    SD_XR_S(0) SD_XR_S(1)
#undef SD_XR_S
#undef SD_XR
    SD_CHECK(done, SPIMDECON_ERR_ARG, "no x-row kernel for this configuration");
    SD_HIP(hipGetLastError());
    return grid;
}

// launches the x pass; returns its grid (= number of stats partials of an update pass)
template <int MODE>
unsigned launch_x(const XArgs& a, Store st, const SpectralPlan& p, hipStream_t s) {
    if constexpr (MODE == XM_QUOT || MODE == XM_UPDATE || MODE == XM_PSI) {
        if (const unsigned gt = launch_xtile<MODE>(a, st, p, s)) {
            if (MODE == XM_UPDATE) p.xmode_update = 2;
            return gt;
        }
    }
    if constexpr (MODE == XM_QUOT || MODE == XM_UPDATE) {
        if (const unsigned gr = launch_xrows<MODE>(a, st, p, s)) {
            if (MODE == XM_UPDATE) p.xmode_update = 1;
            return gr;
        }
    }
    if (MODE == XM_UPDATE) p.xmode_update = 0;
    const size_t lds = x_lds(p);
    SD_CHECK(lds <= 160 * 1024, SPIMDECON_ERR_ARG, "x pass LDS too large");
    SD_CHECK(p.g.My * p.g.Mz < (int64_t(1) << 30), SPIMDECON_ERR_ARG, "too many rows");
    const unsigned grid = x_grid(a);
    if (st == Store::F32) {
        SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_xpass<MODE, 0>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
        hipLaunchKernelGGL((k_xpass<MODE, 0>), dim3(grid), dim3(kXThreads), lds, s, a);
    } else {
        SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_xpass<MODE, 1>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
        hipLaunchKernelGGL((k_xpass<MODE, 1>), dim3(grid), dim3(kXThreads), lds, s, a);
    }
    SD_HIP(hipGetLastError());
    return grid;
}

int col_tx(int L) {
    for (int tx : {16, 8, 4})
        if (size_t(2 * L * tx + L) * sizeof(float2) <= 160 * 1024) return tx;
    fail(SPIMDECON_ERR_ARG, "column FFT length " + std::to_string(L) + " exceeds the LDS tile");
}

// blocks per resident slot of the column passes (grid-stride tiles; 16 ~ one or two
// tiles per block measured best: z 0.364 -> 0.327 ms vs 4)
constexpr int kColGridRounds = 16;

// two-factor column pass; false when the buffer-offset path does not apply.
// MODE 5: K is the compact kernel (2*kc+1 z-planes, engine_kernel_compact).
template <int AXIS, int MODE>
bool launch_col2f(const SpectralPlan& p, const Fft1D& f, float2* C, const float2* K, hipStream_t s,
                  int tx0 = 0, int ntxb = -1, int kc = 0, int nout = -1, int zsplit = INT_MAX, int zskip = 0) {
    // nout: z planes the pass must produce (AXIS 1: planes transformed; AXIS 2 fused
    // modes: planes stored) -- the RL loop only reads the nz interior planes back
    if (nout < 0) nout = int(p.g.Mz);
    const int L = f.L;
    // 16-column tiles (128-B row segments) when they fit the LDS (160 KB); else 8 columns
    // (8-column tiles measured slower for the fused z pass, 0.69 vs 0.60 ms, but beat
    // the Stockham passes: L = 640 / 800 / 1024 at 32 threads, 2100 at 64)
    const int tr = (f.n1 > 32 || f.n2 > 32) ? 64 : 32;  // SD_2F_TR
    // 16-column tiles up to 160 KB (one block per CU) rather than 8-column tiles at two
    // blocks per CU: 128-B segments won at 800 (C4 RL 815 -> 745 ms per timepoint)
    const size_t budget = size_t(160) * 1024;
    auto tile_lds = [&](int tx) { return size_t(L * tx + L + (MODE == 5 ? f.n2 * tx : 0)) * sizeof(float2); };
    // (1050, 64 threads per column: 8-column tiles at two blocks per CU measured slower,
    // y pass 0.892 -> 1.098 ms, profiles/r05_ypass_tx8_ab.txt)
    const int TX = tile_lds(k2fTX) <= budget ? k2fTX : 8;
    const int kplanes = MODE == 5 ? 2 * kc + 1 : 0;
    const size_t lds = tile_lds(TX);
    const uint64_t bytes = uint64_t(p.spectrum_elems()) * sizeof(float2);
    const uint64_t kbytes = MODE == 5 ? uint64_t(kplanes) * p.Hp * p.g.My * sizeof(float2)
                                      : (MODE >= 2 ? bytes : 0);
    // the fused z modes hold two length-N2 vectors per thread: TR = 64 (N2 > 32) would
    // spill, so long lengths run them on the Stockham column pass
    if (MODE >= 2 && tr == 64) return false;
    if (lds > budget || (AXIS == 2 && bytes >= (uint64_t(1) << 31))) return false;
    if (MODE == 5 && (AXIS != 2 || kplanes > f.n2)) return false;
    // AXIS 1 resources span one z plane from the tile's first column
    const uint32_t rbytes = AXIS == 1 ? uint32_t(uint64_t(p.g.My * p.Hp) * sizeof(float2)) : uint32_t(bytes);
    if (ntxb < 0) ntxb = int(p.Hp / TX);
    SD_CHECK(tx0 >= 0 && ntxb > 0 && tx0 + ntxb <= p.Hp / TX, SPIMDECON_ERR_ARG, "bad column band");
    const int64_t ntiles = int64_t(ntxb) * (AXIS == 1 ? nout : p.g.My);
    const int64_t per_cu = std::max<int64_t>(1, (160 * 1024) / int64_t(lds));
    const unsigned grid = unsigned(std::min<int64_t>(ntiles, 256 * per_cu * kColGridRounds));
    const int n1 = f.n1, n2 = f.n2;
    // y passes at one block per CU (16-column tiles past 80 KB, 32 threads per column):
    // the next tile's phase-A inputs prefetched in registers (k_col2f PF); the plan's
    // ypf knob (SPIMDECON_YPF=0 at plan creation) keeps the plain kernel
    const bool pf = p.knobs.ypf && AXIS == 1 && MODE < 2 && tr == 32 && TX == 16 && lds > size_t(80 * 1024);
    bool done = false;
#define SD_2F_L(A, B, T, PFV)                                                                                   \
            constexpr int TRv = SD_2F_TR(A, B);                                                                 \
            SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_col2f<AXIS, A, B, MODE, T, TRv, PFV>), \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));                  \
            hipLaunchKernelGGL((k_col2f<AXIS, A, B, MODE, T, TRv, PFV>), dim3(grid), dim3(T * TRv), lds, s,     \
                               p.g, p.Hp, f.tw, C, K, rbytes, tx0, ntxb, kc, uint32_t(kbytes), nout, zsplit,  \
                               zskip);                                                                       \
            done = true;
#define SD_2F_C1(A, B, T)                                                                                  \
    if constexpr (MODE < 2 || SD_2F_TR(A, B) == 32) {                                                      \
        if (!done && n1 == (A) && n2 == (B) && TX == (T)) {                                                \
            if constexpr (AXIS == 1 && MODE < 2 && (T) == 16 && SD_2F_TR(A, B) == 32 && (A) * (B) >= 512) { \
                if (pf) { SD_2F_L(A, B, T, true) }                                                         \
            }                                                                                              \
            if (!done) { SD_2F_L(A, B, T, false) }                                                         \
        }                                                                                                  \
    }
#define SD_2F_C(A, B) \
    SD_2F_C1(A, B, 16) if constexpr ((A) * (B) > 600) { SD_2F_C1(A, B, 8) }
    SD_2F_SIZES(SD_2F_C)
#undef SD_2F_C
#undef SD_2F_C1
#undef SD_2F_L
    SD_CHECK(done, SPIMDECON_ERR_ARG, "no two-factor column kernel for this length");
    SD_HIP(hipGetLastError());
    return true;
}

template <int AXIS, bool INV, int ZMODE>
void launch_col(const SpectralPlan& p, const Fft1D& f, float2* C, const float2* K, hipStream_t s,
                int nout = -1) {
    if constexpr (ZMODE == 1) {   // the kernel spectrum tile in LDS, else in phase-B registers
        if (f.n1 && launch_col2f<AXIS, 4>(p, f, C, K, s, 0, -1, 0, nout)) return;
    }
    if (f.n1 && launch_col2f<AXIS, ZMODE == 1 ? 2 : (INV ? 1 : 0)>(p, f, C, K, s, 0, -1, 0, nout)) return;
    const int tx = col_tx(f.L);
    SD_CHECK(f.L * tx / 2 <= kColMaxU * kCThreads, SPIMDECON_ERR_ARG, "column tile exceeds prefetch registers");
    const size_t lds = size_t(2 * f.L * tx + f.L) * sizeof(float2);
    const int64_t ntiles = (p.Hp / tx) * (AXIS == 1 ? p.g.Mz : p.g.My);
    const unsigned grid = unsigned(std::min<int64_t>(ntiles, 256 * (tx == 16 ? 1 : 2)));
#define CL(TXV)                                                                                    \
    case TXV:                                                                                      \
        SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_colpass<AXIS, TXV, INV, ZMODE>), \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));         \
        hipLaunchKernelGGL((k_colpass<AXIS, TXV, INV, ZMODE>), dim3(grid), dim3(kCThreads), lds, s, \
                           p.g, p.Hp, f, C, K);                                                    \
        break;
    switch (tx) {
        CL(16) CL(8) CL(4)
        default: fail(SPIMDECON_ERR_ARG, "bad TX");
    }
#undef CL
    SD_HIP(hipGetLastError());
}

}  // namespace

int64_t engine_fast_size(int64_t need, bool even, int policy) {
    need = std::max<int64_t>(need, 1);
    int64_t smooth = 0;
    for (int64_t m = need;; ++m) {
        if (even && (m & 1)) continue;
        int64_t r = m;
        for (int64_t q : {2, 3, 5, 7})
            while (r % q == 0) r /= q;
        if (r == 1) {
            smooth = m;
            break;
        }
    }
    int64_t fast = 0;
#define SD_2F_PICK(A, B) \
    if ((A) * (B) >= need && (fast == 0 || (A) * (B) < fast)) fast = (A) * (B);
    SD_2F_SIZES(SD_2F_PICK)
#undef SD_2F_PICK
    if (policy == 2 || fast == 0) {
        SD_CHECK(policy != 1, SPIMDECON_ERR_ARG, "length " + std::to_string(need) + " beyond the fast-path table");
        return smooth;
    }
    if (policy == 1) return fast;
    return fast * 4 <= smooth * 5 ? fast : smooth;
}

bool engine_slab_fits(int64_t nx, int64_t ny, int64_t nzs, const int halo[3], int policy) {
    const int64_t Mx = engine_fast_size(nx + 2 * halo[0], true, policy);
    const int64_t My = engine_fast_size(ny + 2 * halo[1], false, policy);
    const int64_t Mz = engine_fast_size(nzs + 2 * halo[2], false, policy);   // >= the exact nz + 2 cz
    const int64_t Hp = ceil_div(Mx / 2 + 1, int64_t(16)) * 16;
    return uint64_t(nx) * uint64_t(ny) * uint64_t(nzs) * 4u < kOOB &&
           uint64_t(Hp) * uint64_t(My) * uint64_t(Mz) * sizeof(float2) < kOOB;
}

// direct z convolution (fftconv_zd.inc) unless SPIMDECON_ZDIRECT=0 (read at plan creation)
// selects the fused FFT z pass (k_col2f MODE 5)
static bool zdirect_env() {
    const char* e = std::getenv("SPIMDECON_ZDIRECT");
    return !(e && e[0] == '0');
}

EngineKnobs EngineKnobs::from_env() {
    auto off = [](const char* name) {
        const char* e = std::getenv(name);
        return e && e[0] == '0';
    };
    EngineKnobs k;
    k.ypf = !off("SPIMDECON_YPF");
    k.zkd = !off("SPIMDECON_ZKD");
    k.zdirect = zdirect_env();
    return k;
}

void SpectralPlan::create(const SlabGeom& geom, bool allow_2f, bool z_fft, const EngineKnobs& kn) {
    g = geom;
    knobs = kn;
    SD_CHECK(g.Mx % 2 == 0, SPIMDECON_ERR_ARG, "Mx must be even");
    Hx = g.Mx / 2 + 1;
    Hp = ceil_div(Hx, 16) * 16;  // column tiles of 16 (or 8/4) complex stay 128-B aligned
    hipStream_t s = nullptr;
    fx = make_fft(int(g.Mx), allow_2f, twx, s);
    fy = make_fft(int(g.My), allow_2f, twy, s);
    if (z_fft) {
        fz = make_fft(int(g.Mz), allow_2f, twz, s);
    } else {
        fz = Fft1D{};
        fz.L = int(g.Mz);
    }
    const int64_t nrows = g.My * g.Mz;
    std::vector<int> rm(nrows), ro(nrows);
    auto mir = [](int64_t sidx, int64_t n) -> int64_t {
        if (n == 1) return 0;
        const int64_t p = 2 * (n - 1);
        int64_t j = sidx % p;
        if (j < 0) j += p;
        return j >= n ? p - j : j;
    };
    for (int64_t qz = 0; qz < g.Mz; ++qz) {
        const int64_t sz = qz < g.nz + g.cz ? qz : qz - g.Mz;
        const int64_t gz = g.z0 + sz;
        const bool gin = gz >= 0 && gz < g.nzg;
        const bool skip = gin && (sz < 0 || sz >= g.nz);
        const int64_t lz = mir(gz, g.nzg) - g.z0;
        for (int64_t qy = 0; qy < g.My; ++qy) {
            const int64_t r = qz * g.My + qy;
            if (skip) {
                rm[r] = ro[r] = -1;
                continue;
            }
            SD_CHECK(lz >= 0 && lz < g.nz, SPIMDECON_ERR_ARG, "slab too thin for its mirror halo");
            const int64_t sy = qy < g.ny + g.cy ? qy : qy - g.My;
            const int64_t ly = mir(sy, g.ny);
            rm[r] = int(lz * g.ny + ly);
            const bool interior = (sz >= 0 && sz < g.nz) && (sy >= 0 && sy < g.ny);
            ro[r] = interior ? int(sz * g.ny + sy) : -2;
        }
    }
    row_mirror.alloc(nrows);
    row_one.alloc(nrows);
    SD_HIP(hipMemcpy(row_mirror.p, rm.data(), nrows * sizeof(int), hipMemcpyHostToDevice));
    SD_HIP(hipMemcpy(row_one.p, ro.data(), nrows * sizeof(int), hipMemcpyHostToDevice));
}

void engine_forward_psi(const SpectralPlan& p, const float* psi, float2* C, hipStream_t s) {
    XArgs a = base_args(p);
    a.psi_in = psi;
    a.Cout = C;
    launch_x<XM_PSI>(a, Store::F32, p, s);
}

void engine_kernel_spectrum(const SpectralPlan& p, const float* d_kernel, int kx, int ky, int kz,
                            float scale, float2* Kspec, hipStream_t s) {
    XArgs a = base_args(p);
    // every padded row is a data row for the kernel (no mirror / skip semantics)
    a.Cout = Kspec;
    a.kern = d_kernel;
    a.kx = kx;
    a.ky = ky;
    a.kz = kz;
    a.kscale = scale;
    // temporarily use a map that marks all rows valid: row_mirror >= 0 is all we test
    DBuf<int> all(size_t(p.g.My * p.g.Mz));
    SD_HIP(hipMemsetAsync(all.p, 0, all.bytes(), s));
    a.row_mirror = all.p;
    a.row_one = all.p;
    launch_x<XM_KERNEL>(a, Store::F32, p, s);
    launch_col<1, false, 0>(p, p.fy, Kspec, nullptr, s);
    launch_col<2, false, 0>(p, p.fz, Kspec, nullptr, s);
    SD_HIP(hipStreamSynchronize(s));
}

bool engine_kernel_compact_ok(const SpectralPlan& p) {
    const int kc = p.g.cz;
    return p.fz.n1 && p.fz.n1 <= 32 && p.fz.n2 <= 32 && 2 * kc + 1 <= p.fz.n2 &&  // MODE 5 is TR = 32 only
           size_t(p.fz.L * 8 + p.fz.L + p.fz.n2 * 8) * sizeof(float2) <= 80 * 1024 &&   // 8- or 16-column tiles
           uint64_t(p.spectrum_elems()) * sizeof(float2) < (uint64_t(1) << 31);
}

int64_t engine_kernel_compact_elems(const SpectralPlan& p) { return int64_t(2 * p.g.cz + 1) * p.g.My * p.Hp; }

void engine_kernel_compact(const SpectralPlan& p, const float* d_kernel, int kx, int ky, int kz, float scale,
                           float2* work, float2* Kc, hipStream_t s) {
    // x and y transforms of the placed kernel (work = full spectrum buffer), then the
    // z-planes qz in [-kc, kc] (wrapped) -> Kc[qz + kc]: all the z pass needs, since
    // the placed kernel is zero outside them (|qz| <= kz/2 <= cz)
    SD_CHECK(engine_kernel_compact_ok(p) || engine_zdirect_ok(p), SPIMDECON_ERR_ARG,
             "compact kernel path not available");
    SD_CHECK(kz / 2 <= p.g.cz, SPIMDECON_ERR_ARG, "kernel z half size exceeds the halo");
    // Only those 2kc+1 planes are transformed: the kernel placed with z period
    // 2kc+1 (>= kz) instead of Mz has the same planes in the same circular order, and
    // the x and y transforms act per plane (the full Mz-plane passes were ~96 % zero
    // rows: 2.6 ms per kernel at 800^3).
    const int kc = p.g.cz;
    const int mzc = 2 * kc + 1;
    XArgs a = base_args(p);
    a.g.Mz = mzc;
    a.pn0 = int((p.g.My * mzc + 1) / 2);
    a.Cout = work;
    a.kern = d_kernel;
    a.kx = kx;
    a.ky = ky;
    a.kz = kz;
    a.kscale = scale;
    DBuf<int> all(size_t(p.g.My * mzc));
    SD_HIP(hipMemsetAsync(all.p, 0, all.bytes(), s));
    a.row_mirror = all.p;
    a.row_one = all.p;
    launch_x<XM_KERNEL>(a, Store::F32, p, s);
    launch_col<1, false, 0>(p, p.fy, work, nullptr, s, mzc);
    const size_t plane = size_t(p.g.My * p.Hp) * sizeof(float2);
    SD_HIP(hipMemcpyAsync(Kc + size_t(kc) * p.g.My * p.Hp, work, size_t(kc + 1) * plane,
                          hipMemcpyDeviceToDevice, s));
    if (kc > 0)
        SD_HIP(hipMemcpyAsync(Kc, work + size_t(mzc - kc) * p.g.My * p.Hp, size_t(kc) * plane,
                              hipMemcpyDeviceToDevice, s));
    SD_HIP(hipStreamSynchronize(s));
}

// taps bound KC: 4, 8, 12 or 16 (33-plane kernels).  Measured at 540^3 against the fused
// FFT z pass (0.30-0.31 ms): kc 4 0.258, kc 6 0.272, kc 8 0.274 ms; the chunked LDS-DMA
// pass runs kc 12 (25 taps) at 0.27-0.28 ms.  Larger kernels keep the FFT z pass.
static int zdirect_kc_bound(int kc) {
    for (int b : {4, 8, 12, 16})
        if (kc <= b) return b;
    return 0;
}

// k_zdmc: z chunks carried inside a block, 32-column tiles (256-B plane segments); OPT
// outputs per thread from the instantiated set with the fewest idle output slots
// (nch * TR * OPT - nz), chunks of H = ceil(nz / nch).  Measured and removed (DESIGN §4.1;
// profiles/r03_zpattern_microbench.txt, r04_zpass_configs_ab.txt, r04_zpass_two_blocks_ab.txt):
// whole-column tiles (k_zdma / k_zdirect: 0.285-0.29 vs 0.277 ms at 540, C4 870 -> 815 ms per
// timepoint for the chunks), 16- and 64-column tiles, three buffers (0.318 vs 0.273 ms), two
// blocks per CU (C4 1.11 -> 1.41-1.54 ms), 1024-thread blocks (1.07 -> 1.51 ms), stagger groups.
struct ZChunk { int opt = 0, H = 0; };
static ZChunk zdmc_plan(int64_t nz, int KC) {
    ZChunk best;
    if (KC == 0 || nz < 1) return best;
    int64_t bw = -1;
    for (int opt : {KC == 16 ? 15 : 16, 12, 8}) {
        const int64_t cap = int64_t(kZdThreads / 32) * opt;
        const int64_t nch = ceil_div(nz, cap);
        const int64_t waste = nch * cap - nz;
        if (bw < 0 || waste < bw) {
            best = {opt, int(ceil_div(nz, nch))};
            bw = waste;
        }
    }
    return best;
}

bool engine_zdirect_dims_ok(int64_t Mx, int64_t My, int64_t Mz, int cz, bool zdirect_knob) {
    const int KC = zdirect_kc_bound(cz);
    const int64_t Hp = ceil_div(Mx / 2 + 1, int64_t(16)) * 16;
    // Mz >= KC: a chunk's window slots (plane zc - KC + s mod Mz) wrap at most once
    return zdirect_knob && KC > 0 && Mz >= 2 * cz + 1 && Mz >= KC &&
           uint64_t(Hp) * uint64_t(My) * uint64_t(Mz) * sizeof(float2) <= kOOB;
}

bool engine_zdirect_ok(const SpectralPlan& p) {
    return p.Hp % 16 == 0 && engine_zdirect_dims_ok(p.g.Mx, p.g.My, p.g.Mz, p.g.cz, p.knobs.zdirect);
}

int engine_zpass_mode(const SpectralPlan& p, bool compact) {
    if (!compact) return 0;
    return engine_zdirect_ok(p) ? 3 : 1;
}

void engine_zpass_compact(const SpectralPlan& p, float2* C, const float2* Kc, hipStream_t s) {
    if (!engine_zdirect_ok(p)) {
        const bool ok = launch_col2f<2, 5>(p, p.fz, C, Kc, s, 0, -1, p.g.cz, int(p.g.nz));
        SD_CHECK(ok, SPIMDECON_ERR_ARG, "compact-kernel z pass not available");
        return;
    }
    const int64_t nflat = p.g.My * p.Hp;   // a multiple of 16
    const int KC = zdirect_kc_bound(p.g.cz);
    const ZChunk zc = zdmc_plan(p.g.nz, KC);
    const int64_t ntiles = ceil_div(nflat, int64_t(32));
    const uint32_t bytes = uint32_t(uint64_t(nflat) * p.g.Mz * sizeof(float2));
    const float kscale = float(p.g.Mz);
    // kernels of 2 KC - 1 planes in the KC layout (C4's 31-plane PSFs: KC 16; 23-plane ones:
    // KC 12) skip the two zero outer taps at compile time (C4: z pass 1.076 -> 1.046 ms,
    // profiles/r04_zpass_tap_trim_ab.txt); the plan's zkd knob (SPIMDECON_ZKD=0) keeps the
    // runtime-masked kernels
    const int kd = p.knobs.zkd && (KC == 12 || KC == 16) && KC - p.g.cz == 1 ? 1 : 0;   // (instantiated there)
    bool done = false;
#define SD_ZC(KCV, OPTV, KDV)                                                                                 \
    if (!done && KC == (KCV) && zc.opt == (OPTV) && kd == (KDV)) {                                            \
        constexpr size_t lds = size_t(zdc_lds(KCV, OPTV, 32));                                                \
        SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_zdmc<KCV, OPTV, KDV>),                    \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));                    \
        /* persistent blocks: as many per CU as are resident together (LDS and VGPRs), once */             \
        static const int per_cu = [] {                                                                        \
            int n = 1;                                                                                        \
            SD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(                                              \
                &n, reinterpret_cast<const void*>(&k_zdmc<KCV, OPTV, KDV>), kZdThreads, lds));                \
            return std::max(1, n);                                                                            \
        }();                                                                                                  \
        const unsigned grid = unsigned(std::min<int64_t>(ntiles, 256 * per_cu));                              \
        hipLaunchKernelGGL((k_zdmc<KCV, OPTV, KDV>), dim3(grid), dim3(kZdThreads), lds, s, p.g, nflat, C, Kc,  \
                           p.g.cz, zc.H, bytes, kscale);                                                      \
        done = true;                                                                                          \
    }
#define SD_ZC3(KCV) SD_ZC(KCV, 16, 0) SD_ZC(KCV, 12, 0) SD_ZC(KCV, 8, 0)
    SD_ZC3(4) SD_ZC3(8) SD_ZC3(12)
    SD_ZC(12, 16, 1) SD_ZC(12, 12, 1) SD_ZC(12, 8, 1)
    SD_ZC(16, 15, 0) SD_ZC(16, 12, 0) SD_ZC(16, 8, 0) SD_ZC(16, 15, 1) SD_ZC(16, 12, 1) SD_ZC(16, 8, 1)
#undef SD_ZC3
#undef SD_ZC
    SD_CHECK(done, SPIMDECON_ERR_ARG, "no z-chunked LDS-DMA z kernel for this kernel size");
    SD_HIP(hipGetLastError());
}

void engine_ypass(const SpectralPlan& p, float2* C, bool inv, hipStream_t s) {
    // the inverse feeds the x passes, which read the nz interior planes only
    if (inv) launch_col<1, true, 0>(p, p.fy, C, nullptr, s, int(p.g.nz));
    else launch_col<1, false, 0>(p, p.fy, C, nullptr, s);
}

bool engine_ypass_planes2(const SpectralPlan& p, float2* C, int z0, int z1, int z2, int z3, hipStream_t s) {
    if (!p.fy.n1 || z0 < 0 || z1 < z0 || z2 < z1 || z3 < z2 || z3 > int(p.g.Mz)) return false;
    if (z3 - z2 + z1 - z0 <= 0) return true;
    // planes [z0, z1) and [z2, z3) in one launch: tile rows past z1 - z0 skip z2 - z1 planes
    return launch_col2f<1, 0>(p, p.fy, C + size_t(z0) * size_t(p.g.My) * size_t(p.Hp), nullptr, s, 0, -1, 0,
                              (z1 - z0) + (z3 - z2), z1 - z0, z2 - z1);
}

bool engine_ypass_planes(const SpectralPlan& p, float2* C, int z0, int z1, hipStream_t s) {
    if (!p.fy.n1 || z0 < 0 || z1 > int(p.g.Mz)) return false;  // Stockham passes: whole volume only
    if (z1 <= z0) return true;
    // the y transforms of one z plane touch that plane only: a plane range is the same
    // pass over a shifted base
    return launch_col2f<1, 0>(p, p.fy, C + size_t(z0) * size_t(p.g.My) * size_t(p.Hp), nullptr, s, 0, -1, 0,
                              z1 - z0);
}

void engine_zpass(const SpectralPlan& p, float2* C, const float2* K, hipStream_t s) {
    // fused forward * K * inverse (0.57 ms at 540^3) beat forward z + (C*K) inverse z
    // as two launches (0.61 ms)
    if (K) launch_col<2, false, 1>(p, p.fz, C, K, s, int(p.g.nz));
    else launch_col<2, false, 0>(p, p.fz, C, nullptr, s);
}

PairRanges all_pairs(const SpectralPlan& p) {
    PairRanges r;
    r.n0 = int((p.g.My * p.g.Mz + 1) / 2);
    return r;
}

void engine_quotient(const SpectralPlan& p, Store st, const float2* Cin, const void* img,
                     float2* Cout, const PairRanges& pr, hipStream_t s) {
    XArgs a = base_args(p);
    a.pb0 = pr.b0;
    a.pn0 = pr.n0;
    a.pb1 = pr.b1;
    a.pn1 = pr.n1;
    a.Cin = Cin;
    a.Cout = Cout;
    a.img = img;
    launch_x<XM_QUOT>(a, st, p, s);
}

int64_t engine_update(const SpectralPlan& p, Store st, const float2* Cin, const float* psi_in,
                      const void* w, double lambda, float* psi_out, float2* Cout, double* partials,
                      const PairRanges& pr, hipStream_t s) {
    XArgs a = base_args(p);
    a.pb0 = pr.b0;
    a.pn0 = pr.n0;
    a.pb1 = pr.b1;
    a.pn1 = pr.n1;
    a.Cin = Cin;
    a.Cout = Cout;
    a.psi_in = psi_in;
    a.psi_out = psi_out;
    a.w = w;
    a.lambda = lambda;
    a.partials = partials;
    return launch_x<XM_UPDATE>(a, st, p, s);
}

}  // namespace spimdecon
