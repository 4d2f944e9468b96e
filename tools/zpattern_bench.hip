// zpattern_bench.hip -- HBM rate of the z pass's access pattern, without its compute.
// A spectrum of P planes x E complex elements (540^3 engine: P = 536, E = 540 * 272);
// a tile = SEG consecutive elements, all planes (the z pass reads and rewrites every
// plane's SEG * 8-byte segment of its tile).  Every block walks its tiles; its waves
// read 1-KiB pieces (1024 / (SEG * 8) planes per piece, or part of a plane for
// SEG > 128), DEPTH pieces in flight per wave, and write each back (+1).  The layout
// variant "brick" stores planes in groups of ZB: [P / ZB][E][ZB], so a tile's ZB
// planes are one contiguous ZB * SEG * 8-byte run (what a z-brick layout would give).
// usage: zpattern_bench [P E [quick]]  (prints one line per variant; default P = 536, E = 540 * 272;
//        quick: only the plane-strided 256- / 512-B variants and the contiguous references)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

// piece j of tile t: plane-major pieces.  Plane layout: element (p, e) at p * E + e
// (planar) or (p / ZB) * E * ZB + e * ZB + p % ZB (brick, SEG elements per plane run
// become SEG * ZB contiguous elements per plane group).
template <int DEPTH>
__global__ __launch_bounds__(512) void k_pattern(float4* buf, long E, int P, int seg, int zb, int stagger,
                                                 float4* dst = nullptr) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const long ntiles = E / seg;
    const int bytes_tile_plane = seg * 8;                  // bytes of one plane's segment
    const long tile_bytes = long(bytes_tile_plane) * P;    // bytes of a tile
    const int npieces = int(tile_bytes / 1024);
    const int lseg = __builtin_ctz(bytes_tile_plane);
    const int lzb = zb > 1 ? __builtin_ctz(zb) : 0;
    for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int stag = stagger ? int((uint32_t(blockIdx.x) * 2654435761u) % uint32_t(npieces)) : 0;
        for (int j0 = wave * DEPTH; j0 < npieces; j0 += 8 * DEPTH) {
            float4 v[DEPTH];
            long off[DEPTH];
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
                int j = j0 + d;
                off[d] = -1;
                if (j < npieces) {
                    j += stag;
                    if (j >= npieces) j -= npieces;
                    // byte b of the tile: 16 * (64 j + lane); segment sizes are powers of two
                    const int b = (j * 64 + lane) * 16;
                    if (zb <= 1) {
                        const int p = b >> lseg, eb = b & (bytes_tile_plane - 1);
                        off[d] = (long(p) * E * 8 + tile * bytes_tile_plane + eb) >> 4;
                    } else {
                        const int g = b >> (lseg + lzb), eb = b & ((bytes_tile_plane << lzb) - 1);
                        off[d] = (long(g) * E * 8 * zb + (tile * bytes_tile_plane << lzb) + eb) >> 4;
                    }
                    v[d] = buf[off[d]];
                }
            }
#pragma unroll
            for (int d = 0; d < DEPTH; ++d)
                if (off[d] >= 0) {
                    float4 w = v[d];
                    w.x += 1.0f;
                    (dst ? dst : buf)[off[d]] = w;   // dst: out of place (read buf, write dst)
                }
        }
    }
}

// Contiguous references.  Round 3's k_stream kept ONE dependent float4 load -> store
// per thread in flight (4.7-4.9 TB/s); these keep DEPTH independent float4 loads per
// thread in flight before their stores (a block's DEPTH * 512 * 16 B = one chunk).
// k_rmw: in place (the z pass's shape); k_copy: read src, write dst (the guide's copy).
template <int DEPTH>
__global__ __launch_bounds__(256) void k_rmw(float4* buf, long n) {
    const long chunk = long(DEPTH) * 256;
    for (long base = long(blockIdx.x) * chunk; base < n; base += long(gridDim.x) * chunk) {
        float4 v[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const long i = base + d * 256 + threadIdx.x;
            if (i < n) v[d] = buf[i];
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const long i = base + d * 256 + threadIdx.x;
            if (i < n) {
                v[d].x += 1.0f;
                buf[i] = v[d];
            }
        }
    }
}

template <int DEPTH>
__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ src, float4* __restrict__ dst, long n) {
    const long chunk = long(DEPTH) * 256;
    for (long base = long(blockIdx.x) * chunk; base < n; base += long(gridDim.x) * chunk) {
        float4 v[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const long i = base + d * 256 + threadIdx.x;
            if (i < n) v[d] = src[i];
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const long i = base + d * 256 + threadIdx.x;
            if (i < n) dst[i] = v[d];
        }
    }
}

// Round-5 references (the round-4 copy topped out at 5.54 TB/s against the
// guide's ~6.3): one-shot blocks (no grid stride), 32-bit float4 indices, no per-element
// test (n_eff is a whole number of chunks), DEPTH independent 16-B loads per thread in
// flight, 256-thread blocks -- enough resident waves per SIMD to cover HBM latency.
template <int DEPTH>
__global__ __launch_bounds__(256) void k_copy2(const float4* __restrict__ src, float4* __restrict__ dst) {
    const uint32_t base = blockIdx.x * uint32_t(DEPTH * 256) + threadIdx.x;
    float4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) v[d] = src[base + d * 256];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) dst[base + d * 256] = v[d];
}
template <int DEPTH>
__global__ __launch_bounds__(256) void k_rmw2(float4* buf) {
    const uint32_t base = blockIdx.x * uint32_t(DEPTH * 256) + threadIdx.x;
    float4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) v[d] = buf[base + d * 256];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        v[d].x += 1.0f;
        buf[base + d * 256] = v[d];
    }
}
// the z pass's plane-strided shape with the same hygiene: one block per tile of SEG
// elements x P planes, 1-KiB pieces (wave-uniform tail test only), 32-bit offsets
template <int DEPTH, int SEG>
__global__ __launch_bounds__(512) void k_pattern2(float4* buf, uint32_t E, int P) {
    constexpr int bytes_tile_plane = SEG * 8;
    constexpr int lseg = __builtin_ctz(bytes_tile_plane);
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x;
    const int npieces = (bytes_tile_plane * P) >> 10;
    const int stag = int((tile * 2654435761u) % uint32_t(npieces));
    for (int j0 = wave * DEPTH; j0 < npieces; j0 += 8 * DEPTH) {
        float4 v[DEPTH];
        uint32_t off[DEPTH];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            int j = j0 + d < npieces ? j0 + d : j0;   // (wave-uniform)
            j += stag;
            if (j >= npieces) j -= npieces;
            const int b = (j * 64 + lane) * 16;
            off[d] = (uint32_t(b >> lseg) * E * 8u + tile * uint32_t(bytes_tile_plane) + uint32_t(b & (bytes_tile_plane - 1))) >> 4;
            v[d] = buf[off[d]];
        }
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            if (j0 + d < npieces) {
                v[d].x += 1.0f;
                buf[off[d]] = v[d];
            }
        }
    }
}

int main(int argc, char** argv) {
    const int P = argc > 2 ? std::atoi(argv[1]) : 536;
    const long E = argc > 2 ? std::atol(argv[2]) : 540L * 272;   // multiple of every SEG below
    const bool quick = argc > 3;
    if (E % 64 != 0) {
        std::fprintf(stderr, "E must be a multiple of 64\n");
        return 1;
    }
    std::printf("P %d planes, E %ld elements per plane (%.2f MB planes)\n", P, E, E * 8.0 / 1e6);
    const size_t bytes = size_t(P) * E * 8;
    float4* buf;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct V { int seg, zb, stag, grid, depth; };
    std::vector<V> vs;
    if (quick) {
        for (int seg : {32, 64}) vs.push_back({seg, 1, 1, 1024, 4});
    } else {
        for (int seg : {16, 32, 64})
            for (int stag : {1, 0})
                for (int grid : {256, 1024})
                    vs.push_back({seg, 1, stag, grid, 4});
        for (int seg : {16, 32})
            for (int zb : {4, 8})
                for (int grid : {256, 1024})
                    vs.push_back({seg, zb, 1, grid, 4});
        vs.push_back({32, 1, 1, 256, 8});
        vs.push_back({32, 1, 1, 256, 2});
    }
    std::printf("seg_bytes zbrick stagger grid depth ms TB/s(read+write)\n");
    for (const V& v : vs) {
        auto launch = [&] {
            if (v.depth == 8) hipLaunchKernelGGL(k_pattern<8>, dim3(v.grid), dim3(512), 0, 0, buf, E, P, v.seg, v.zb, v.stag);
            else if (v.depth == 2) hipLaunchKernelGGL(k_pattern<2>, dim3(v.grid), dim3(512), 0, 0, buf, E, P, v.seg, v.zb, v.stag);
            else hipLaunchKernelGGL(k_pattern<4>, dim3(v.grid), dim3(512), 0, 0, buf, E, P, v.seg, v.zb, v.stag);
        };
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        std::printf("%d %d %d %d %d %.4f %.3f\n", v.seg * 8, v.zb, v.stag, v.grid, v.depth, ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
        std::fflush(stdout);
    }
    // plane-strided pattern at higher occupancy (grid 2048-4096 blocks of 8 waves)
    for (int seg : {32, 64})
        for (int grid : {2048, 4096}) {
            if (quick) break;
            auto launch = [&] { hipLaunchKernelGGL(k_pattern<8>, dim3(grid), dim3(512), 0, 0, buf, E, P, seg, 1, 1); };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < 10; ++r) launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ms /= 10;
            std::printf("%d 1 1 %d 8 %.4f %.3f\n", seg * 8, grid, ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
            std::fflush(stdout);
        }
    // contiguous references: in place (read + write the same bytes) and copy (src -> dst)
    float4* dst;
    CK(hipMalloc(&dst, bytes));
    CK(hipMemset(dst, 0, bytes));
    // the plane-strided pattern out of place (read buf, write dst: a z pass into the other buffer)
    std::printf("out-of-place pattern: seg_bytes grid depth ms TB/s(read+write)\n");
    for (int seg : {32, 64})
        for (int grid : {1024, 2048}) {
            auto launch = [&] { hipLaunchKernelGGL(k_pattern<4>, dim3(grid), dim3(512), 0, 0, buf, E, P, seg, 1, 1, dst); };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < 10; ++r) launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ms /= 10;
            std::printf("oop %d %d 4 %.4f %.3f\n", seg * 8, grid, ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
            std::fflush(stdout);
        }
    const long n = long(bytes / 16);
    std::printf("kind depth grid(256-thread blocks) ms TB/s(read+write)\n");
    for (int kind = 0; kind < 2; ++kind)
        for (int depth : {1, 4, 8})
            for (int grid : {2048, 8192, 32768}) {
                if (quick && (depth != 4 || grid != 32768)) continue;
                auto launch = [&] {
                    if (kind == 0) {
                        if (depth == 1) hipLaunchKernelGGL(k_rmw<1>, dim3(grid), dim3(256), 0, 0, buf, n);
                        else if (depth == 4) hipLaunchKernelGGL(k_rmw<4>, dim3(grid), dim3(256), 0, 0, buf, n);
                        else hipLaunchKernelGGL(k_rmw<8>, dim3(grid), dim3(256), 0, 0, buf, n);
                    } else {
                        if (depth == 1) hipLaunchKernelGGL(k_copy<1>, dim3(grid), dim3(256), 0, 0, buf, dst, n);
                        else if (depth == 4) hipLaunchKernelGGL(k_copy<4>, dim3(grid), dim3(256), 0, 0, buf, dst, n);
                        else hipLaunchKernelGGL(k_copy<8>, dim3(grid), dim3(256), 0, 0, buf, dst, n);
                    }
                };
                launch();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a));
                for (int r = 0; r < 10; ++r) launch();
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                ms /= 10;
                std::printf("%s %d %d %.4f %.3f\n", kind == 0 ? "rmw" : "copy", depth, grid, ms,
                            2.0 * bytes / (ms * 1e-3) / 1e12);
                std::fflush(stdout);
            }
    // round-5 references
    std::printf("round-5 references: kind depth blocks ms TB/s(read+write)\n");
    auto timeit = [&](auto&& launch, double moved) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < 10; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= 10;
        return std::make_pair(ms, moved / (ms * 1e-3) / 1e12);
    };
    for (int depth : {2, 4, 8}) {
        const uint32_t chunk = uint32_t(depth) * 256;
        const uint32_t blocks = uint32_t(n / chunk);
        const double moved = 2.0 * double(blocks) * chunk * 16;
        for (int kind = 0; kind < 2; ++kind) {
            auto r = timeit([&] {
                if (kind == 0) {
                    if (depth == 2) hipLaunchKernelGGL(k_copy2<2>, dim3(blocks), dim3(256), 0, 0, buf, dst);
                    else if (depth == 4) hipLaunchKernelGGL(k_copy2<4>, dim3(blocks), dim3(256), 0, 0, buf, dst);
                    else hipLaunchKernelGGL(k_copy2<8>, dim3(blocks), dim3(256), 0, 0, buf, dst);
                } else {
                    if (depth == 2) hipLaunchKernelGGL(k_rmw2<2>, dim3(blocks), dim3(256), 0, 0, buf);
                    else if (depth == 4) hipLaunchKernelGGL(k_rmw2<4>, dim3(blocks), dim3(256), 0, 0, buf);
                    else hipLaunchKernelGGL(k_rmw2<8>, dim3(blocks), dim3(256), 0, 0, buf);
                }
            }, moved);
            std::printf("%s2 %d %u %.4f %.3f\n", kind == 0 ? "copy" : "rmw", depth, blocks, r.first, r.second);
            std::fflush(stdout);
        }
    }
    std::printf("round-5 plane-strided pattern: seg_bytes depth tiles ms TB/s(read+write)\n");
    for (int seg : {16, 32, 64}) {
        const uint32_t tiles = uint32_t(E / seg);
        for (int depth : {4, 8}) {
            auto r = timeit([&] {
#define PAT(D, S) if (depth == D && seg == S) hipLaunchKernelGGL((k_pattern2<D, S>), dim3(tiles), dim3(512), 0, 0, buf, uint32_t(E), P);
                PAT(4, 16) PAT(8, 16) PAT(4, 32) PAT(8, 32) PAT(4, 64) PAT(8, 64)
#undef PAT
            }, 2.0 * double(bytes));
            std::printf("pat2 %d %d %u %.4f %.3f\n", seg * 8, depth, tiles, r.first, r.second);
            std::fflush(stdout);
        }
    }
    CK(hipFree(dst));
    CK(hipFree(buf));
    return 0;
}
