// bwdprobe — where does the split run pay over the bare transpose?  On one box,
// back to back: the float4 copy, tools/widebw.hip's bare F=8/R=64 pattern (one
// LDS round trip, no arithmetic), and tools/splitbw.hip's XI run (the engine's
// structure) with parts removed:
//   bit 0  no bucket arithmetic (phase 1 / phase 2 skipped)
//   bit 1  no exchange table (the second LDS round trip and its barrier)
//   bit 2  (bwd) slab stores in widebw's order: wave w, store e -> slab 16 e + w
//   bit 3  rows of the tile in widebw's order: wave w's i-th 1-KiB row access is
//          row 16 i + w (a workgroup instruction covers 16 contiguous KiB), not 4 w + i
// Results are not checked (the removed parts make them wrong); only time.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/bwdprobe.hip -o build/bwdprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <chrono>

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr long kTotal = 1L << 32;
constexpr int N = 256, R = 64;
constexpr long L = kTotal / N;
constexpr int ROWB = N * 4 + 16;
constexpr int ROW = N + 4;

// a wave-uniform pointer in SGPRs: every access is then base + (32-bit lane offset)
template <typename P>
__device__ __forceinline__ P *uni(P *p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return (P *)(((unsigned long long)hi << 32) | lo);
}
// base + byte offset as a global-address-space pointer (global_load/store with
// an SGPR base and a 32-bit VGPR offset, not flat accesses)
template <typename P>
__device__ __forceinline__ __attribute__((address_space(1))) P *at(P *base, unsigned byte_off) {
    return (__attribute__((address_space(1))) P *)((char *)base + byte_off);
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int PJ, int PQ>
__device__ __forceinline__ void step(float (&t)[16], const float *gp, int qu) {
    const v4f g0 = *(const v4f *)(gp + (PQ ? 0 : 4 * qu)), g1 = PQ ? *(const v4f *)(gp + 4) : g0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        if (e & PJ) continue;
        const v4f g = PQ && (e & PQ) ? g1 : g0;
        const v2f m0 = {t[e], t[e]}, m1 = {t[e | PJ], t[e | PJ]};
        const v2f gx0 = {g[0], g[2]}, gx1 = {g[1], g[3]};
        const v2f a = gx0 * m0 + gx1 * m1;
        t[e] = a[0];
        t[e | PJ] = a[1];
    }
}
__device__ __forceinline__ void phase1(float (&t)[16], const float *g, int w) {
    step<8, 4>(t, g + 0, 0);
    step<4, 2>(t, g + 8, 0);
    step<2, 1>(t, g + 16, 0);
    step<1, 0>(t, g + 24, (w >> 3) & 1);
}
__device__ __forceinline__ void phase2(float (&t)[16], const float *g) {
    step<8, 4>(t, g + 32, 0);
    step<4, 2>(t, g + 40, 0);
    step<2, 1>(t, g + 48, 0);
    step<1, 0>(t, g + 56, 0);
}

template <int MODE>
__global__ __launch_bounds__(1024) void fwd(const float *__restrict__ in, float *__restrict__ out, long tiles,
                                             const float *__restrict__ gsrc) {
    constexpr bool AR = !(MODE & 1), XI = !(MODE & 2), ROWS = MODE & 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);
    unsigned char *img = lds + 256;
    float *xch = reinterpret_cast<float *>(lds + 256 + 64 * ROWB);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    const float *tb = in + (long)w * L + lane;
    auto load = [&](long tile, float (&v)[16]) {
        const float *p = tb + tile * R;
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = p[(long)e * 16 * L];
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    float ra[16], rb[16];
    load(tile, ra);
    load(tile + gridDim.x < tiles ? tile + gridDim.x : tile, rb);
    float lmax = 0.f;
    while (true) {
        float t[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) { t[e] = ra[e]; ra[e] = rb[e]; }
        const long nt = tile + 2 * gridDim.x < tiles ? tile + 2 * gridDim.x : tiles - 1;
        load(nt, rb);
        if (AR) phase1(t, gt, w);
        if (XI) {
#pragma unroll
            for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = t[e];
            lds_barrier();
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] = xch[(e * 16 + w) * 64 + lane];
        }
        if (AR) phase2(t, gt);
#pragma unroll
        for (int e = 0; e < 16; ++e) lmax = fmaxf(lmax, t[e]);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *(v4f *)(img + lane * ROWB + 64 * w + 16 * c) = v4f{t[4 * c], t[4 * c + 1], t[4 * c + 2], t[4 * c + 3]};
        lds_barrier();
        float *ob = out + tile * (long)R * N;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int rw = ROWS ? 16 * it + w : 4 * w + it, q = rw * 64 + lane;
            const v4f v = *(const v4f *)(img + rw * ROWB + 16 * lane);
            __builtin_nontemporal_store(v, (v4f *)(ob + 4L * q));
        }
        if (!XI) lds_barrier();                              // image reuse (XI: the exchange barrier covers it)
        if (tile + gridDim.x >= tiles) break;
        tile += gridDim.x;
    }
    if (lmax < 0.f) out[0] = lmax;
}

template <int MODE>
__global__ __launch_bounds__(1024) void bwd(const float *__restrict__ in, float *__restrict__ out, long tiles,
                                             const float *__restrict__ gsrc) {
    constexpr bool AR = !(MODE & 1), XI = !(MODE & 2), SWAP = MODE & 4, ROWS = MODE & 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);
    unsigned char *img = lds + 256;
    float *xch = reinterpret_cast<float *>(lds + 256 + 64 * ROWB);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    auto load = [&](long tile, v4f (&v)[4]) {
        const float *p = in + tile * (long)R * N + 4 * lane;
#pragma unroll
        for (int it = 0; it < 4; ++it) v[it] = *(const v4f *)(p + (ROWS ? 16 * it + w : 4 * w + it) * N);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    v4f ra[4];
    load(tile, ra);
    int fixed = 0;
#pragma unroll
    for (int p = 4; p < 8; ++p) fixed |= ((w >> (7 - p)) & 1) << p;
    float lmax = 0.f;
    while (true) {
        v4f cur[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) cur[it] = ra[it];
        const long nt = tile + gridDim.x < tiles ? tile + gridDim.x : tiles - 1;
        load(nt, ra);
#pragma unroll
        for (int it = 0; it < 4; ++it) *(v4f *)(img + (ROWS ? 16 * it + w : 4 * w + it) * ROWB + 16 * lane) = cur[it];
        lds_barrier();
        float u[16], t[16];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const v4f v = *(const v4f *)(img + lane * ROWB + 4 * fixed + 16 * c);
            u[4 * c] = v[0]; u[4 * c + 1] = v[1]; u[4 * c + 2] = v[2]; u[4 * c + 3] = v[3];
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = u[((e >> 3) & 1) | (((e >> 2) & 1) << 1) | (((e >> 1) & 1) << 2) | ((e & 1) << 3)];
        if (AR) phase1(t, gt, w);
        if (XI) {
#pragma unroll
            for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = t[e];
            lds_barrier();
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] = xch[(e * 16 + w) * 64 + lane];
        } else {
            lds_barrier();                                   // image reuse by the next tile
        }
        if (AR) phase2(t, gt);
#pragma unroll
        for (int e = 0; e < 16; ++e) lmax = fmaxf(lmax, t[e]);
        float *ob = out + tile * (long)R + lane + (SWAP ? (long)w * L : (long)w * 16 * L);
#pragma unroll
        for (int e = 0; e < 16; ++e) __builtin_nontemporal_store(t[e], ob + (long)e * (SWAP ? 16 : 1) * L);
        if (tile + gridDim.x >= tiles) break;
        tile += gridDim.x;
    }
    if (lmax < 0.f) out[0] = lmax;
}

// rows in place, ONE image per workgroup (66.5 KiB): two workgroups fit a CU
// (OCC = 2: 8 waves per SIMD, 64 VGPRs, grid 2 x CUs), each one's
// barriers and arithmetic hidden behind the other's memory traffic.  Three
// barriers per tile (the image is reused without a parity copy).
template <int OCC>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4 * OCC))) void fwd2(const float *__restrict__ in, float *__restrict__ out, long tiles,
                                                   const float *__restrict__ gsrc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);
    unsigned char *img = lds + 256;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    auto load = [&](long tile, float (&v)[16]) {
        const float *p = uni(in + (long)w * L + tile * R);
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = *at(uni(p + (long)e * 16 * L), 4 * lane);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    float ra[16];
    load(tile, ra);
    float lmax = 0.f;
    while (true) {
        float t[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = ra[e];
        const long nt = tile + gridDim.x < tiles ? tile + gridDim.x : tiles - 1;
        load(nt, ra);
        phase1(t, gt, w);
#pragma unroll
        for (int e = 0; e < 16; ++e) *(float *)(img + lane * ROWB + 4 * (e * 16 + w)) = t[e];
        lds_barrier();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const v4f v = *(const v4f *)(img + lane * ROWB + 64 * w + 16 * c);
            t[4 * c] = v[0]; t[4 * c + 1] = v[1]; t[4 * c + 2] = v[2]; t[4 * c + 3] = v[3];
        }
        phase2(t, gt);
#pragma unroll
        for (int e = 0; e < 16; ++e) lmax = fmaxf(lmax, t[e]);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *(v4f *)(img + lane * ROWB + 64 * w + 16 * c) = v4f{t[4 * c], t[4 * c + 1], t[4 * c + 2], t[4 * c + 3]};
        lds_barrier();
        float *ob = uni(out + tile * (long)R * N + (long)w * N);
        v4f sv[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) sv[it] = *(const v4f *)(img + (16 * it + w) * ROWB + 16 * lane);
        lds_barrier();                                       // image free for the next tile
#pragma unroll
        for (int it = 0; it < 4; ++it) __builtin_nontemporal_store(sv[it], at((v4f *)(ob + 16 * it * N), 16 * lane));
        if (tile + gridDim.x >= tiles) break;
        tile += gridDim.x;
    }
    if (lmax < 0.f) out[0] = lmax;
}

template <int OCC>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4 * OCC))) void bwd2(const float *__restrict__ in, float *__restrict__ out, long tiles,
                                                   const float *__restrict__ gsrc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);
    unsigned char *img = lds + 256;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    auto load = [&](long tile, v4f (&v)[4]) {
        const float *p = uni(in + tile * (long)R * N + (long)w * N);
#pragma unroll
        for (int it = 0; it < 4; ++it) v[it] = *at((const v4f *)(p + 16 * it * N), 16 * lane);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    v4f ra[4];
    load(tile, ra);
    int fixed = 0, lo = 0;
#pragma unroll
    for (int p = 4; p < 8; ++p) fixed |= ((w >> (7 - p)) & 1) << p;
#pragma unroll
    for (int p = 0; p < 4; ++p) lo |= ((w >> (3 - p)) & 1) << p;
    float lmax = 0.f;
    while (true) {
        v4f cur[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) cur[it] = ra[it];
        const long nt = tile + gridDim.x < tiles ? tile + gridDim.x : tiles - 1;
        load(nt, ra);
#pragma unroll
        for (int it = 0; it < 4; ++it) *(v4f *)(img + (16 * it + w) * ROWB + 16 * lane) = cur[it];
        lds_barrier();
        float u[16], t[16];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const v4f v = *(const v4f *)(img + lane * ROWB + 4 * fixed + 16 * c);
            u[4 * c] = v[0]; u[4 * c + 1] = v[1]; u[4 * c + 2] = v[2]; u[4 * c + 3] = v[3];
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = u[((e >> 3) & 1) | (((e >> 2) & 1) << 1) | (((e >> 1) & 1) << 2) | ((e & 1) << 3)];
        phase1(t, gt, w);
#pragma unroll
        for (int e = 0; e < 16; ++e)
            u[((e >> 3) & 1) | (((e >> 2) & 1) << 1) | (((e >> 1) & 1) << 2) | ((e & 1) << 3)] = t[e];
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *(v4f *)(img + lane * ROWB + 4 * fixed + 16 * c) = v4f{u[4 * c], u[4 * c + 1], u[4 * c + 2], u[4 * c + 3]};
        lds_barrier();
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int hi = (((e >> 3) & 1) << 4) | (((e >> 2) & 1) << 5) | (((e >> 1) & 1) << 6) | ((e & 1) << 7);
            t[e] = *(const float *)(img + lane * ROWB + 4 * (hi | lo));
        }
        lds_barrier();                                       // image free for the next tile
        phase2(t, gt);
#pragma unroll
        for (int e = 0; e < 16; ++e) lmax = fmaxf(lmax, t[e]);
        float *ob = uni(out + tile * (long)R + (long)w * L);
#pragma unroll
        for (int e = 0; e < 16; ++e) __builtin_nontemporal_store(t[e], at(uni(ob + (long)e * 16 * L), 4 * lane));
        if (tile + gridDim.x >= tiles) break;
        tile += gridDim.x;
    }
    if (lmax < 0.f) out[0] = lmax;
}

// bwd<12> with a padded slab stride (slab s at s * sstride floats) and/or a
// rotation of each slab's contents by s * rot floats (mod L): do the 256
// scattered write streams stop colliding?
__global__ __launch_bounds__(1024) void bwdp(const float *__restrict__ in, float *__restrict__ out, long tiles,
                                             const float *__restrict__ gsrc, long sstride, long rot) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);
    unsigned char *img = lds + 256;
    float *xch = reinterpret_cast<float *>(lds + 256 + 64 * ROWB);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    auto load = [&](long tile, v4f (&v)[4]) {
        const float *p = in + tile * (long)R * N + 4 * lane;
#pragma unroll
        for (int it = 0; it < 4; ++it) v[it] = *(const v4f *)(p + (16 * it + w) * N);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    v4f ra[4];
    load(tile, ra);
    int fixed = 0;
#pragma unroll
    for (int p = 4; p < 8; ++p) fixed |= ((w >> (7 - p)) & 1) << p;
    float lmax = 0.f;
    while (true) {
        v4f cur[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) cur[it] = ra[it];
        const long nt = tile + gridDim.x < tiles ? tile + gridDim.x : tiles - 1;
        load(nt, ra);
#pragma unroll
        for (int it = 0; it < 4; ++it) *(v4f *)(img + (16 * it + w) * ROWB + 16 * lane) = cur[it];
        lds_barrier();
        float u[16], t[16];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const v4f v = *(const v4f *)(img + lane * ROWB + 4 * fixed + 16 * c);
            u[4 * c] = v[0]; u[4 * c + 1] = v[1]; u[4 * c + 2] = v[2]; u[4 * c + 3] = v[3];
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = u[((e >> 3) & 1) | (((e >> 2) & 1) << 1) | (((e >> 1) & 1) << 2) | ((e & 1) << 3)];
        phase1(t, gt, w);
#pragma unroll
        for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = t[e];
        lds_barrier();
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = xch[(e * 16 + w) * 64 + lane];
        phase2(t, gt);
#pragma unroll
        for (int e = 0; e < 16; ++e) lmax = fmaxf(lmax, t[e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const long sl = w + 16 * e;
            __builtin_nontemporal_store(t[e], out + sl * sstride + ((tile * R + lane + sl * rot) & (L - 1)));
        }
        if (tile + gridDim.x >= tiles) break;
        tile += gridDim.x;
    }
    if (lmax < 0.f) out[0] = lmax;
}

// tools/widebw.hip's bare pattern at F = 8, R = 64
__global__ __launch_bounds__(1024) void wfwd(const float *__restrict__ in, float *__restrict__ out, long tiles) {
    constexpr int PER = 16;
    extern __shared__ __attribute__((aligned(16))) float wl[];
    const int t = threadIdx.x;
    float cur[PER], nxt[PER];
    const float *tb = in + (long)(t / R) * L + (t % R);
    auto load = [&](long tile, float (&v)[PER]) {
        const float *p = tb + tile * R;
#pragma unroll
        for (int i = 0; i < PER; ++i) v[i] = __builtin_nontemporal_load(p + (long)i * 16 * L);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    load(tile, cur);
    while (true) {
        const long nt = tile + gridDim.x < tiles ? tile + gridDim.x : tile;
        load(nt, nxt);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = i * 1024 + t, x = q / R, r = q % R;
            wl[r * ROW + x] = cur[i];
        }
        __syncthreads();
        float *ob = out + tile * (long)R * N;
#pragma unroll
        for (int j = 0; j < PER / 4; ++j) {
            const int q = (j * 1024 + t) * 4, r = q / N, n = q % N;
            __builtin_nontemporal_store(*(const v4f *)(wl + r * ROW + n), (v4f *)(ob + q));
        }
        if (nt == tile) break;
        tile = nt;
#pragma unroll
        for (int i = 0; i < PER; ++i) cur[i] = nxt[i];
    }
}

__global__ __launch_bounds__(1024) void wbwd(const float *__restrict__ in, float *__restrict__ out, long tiles) {
    constexpr int PER = 16;
    extern __shared__ __attribute__((aligned(16))) float wl[];
    const int t = threadIdx.x;
    v4f cur[PER / 4], nxt[PER / 4];
    auto load = [&](long tile, v4f (&v)[PER / 4]) {
        const float *ib = in + tile * (long)R * N;
#pragma unroll
        for (int j = 0; j < PER / 4; ++j) v[j] = *(const v4f *)(ib + (j * 1024 + t) * 4);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    load(tile, cur);
    while (true) {
        const long nt = tile + gridDim.x < tiles ? tile + gridDim.x : tile;
        load(nt, nxt);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER / 4; ++j) {
            const int q = (j * 1024 + t) * 4, r = q / N, n = q % N;
            *(v4f *)(wl + r * ROW + n) = cur[j];
        }
        __syncthreads();
        float *p = out + (long)(t / R) * L + (t % R) + tile * R;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = i * 1024 + t, x = q / R, r = q % R;
            __builtin_nontemporal_store(wl[r * ROW + x], p + (long)i * 16 * L);
        }
        if (nt == tile) break;
        tile = nt;
#pragma unroll
        for (int j = 0; j < PER / 4; ++j) cur[j] = nxt[j];
    }
}

__global__ __launch_bounds__(256) void copyf(const v4f *__restrict__ a, v4f *__restrict__ b) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    __builtin_nontemporal_store(a[i], b + i);
}

__global__ void fill(float *p, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        p[i] = 0.5f + 0.25f * ((i * 2654435761u) % 1024) / 1024.f;
}

int main(int argc, char **argv) {
    const int reps = argc > 5 ? 2 : 5;
    float *a, *b, *g;
    // "offsets": a and b inside one allocation, b at 16 GiB + delta after a, for
    // a range of deltas (does the in/out placement move the runs?)
    const bool offsets = argc > 1 && argv[1][0] == 'o';
    // "regions": one arena of argv[2] GB (the engine's), a and b walked over
    // consecutive 16-GiB regions of it (is some of the arena slower?)
    const bool regions = argc > 1 && argv[1][0] == 'r';
    char *big = nullptr;
    size_t arena = 0;
    if (regions) {
        // argv[3]: 0 hipMalloc, 1 hipExtMallocWithFlags(contiguous), 2 VMM: physical
        // chunks of argv[4] MiB (default 2048) mapped into one reserved range
        arena = (size_t)((argc > 2 ? atof(argv[2]) : 250.0) * 1e9);
        const int how = argc > 3 ? atoi(argv[3]) : 0;
        const auto t0 = std::chrono::steady_clock::now();
        if (how == 0) {
            CK(hipMalloc((void **)&big, arena));
        } else if (how == 1) {
            CK(hipExtMallocWithFlags((void **)&big, arena, hipDeviceMallocContiguous));
        } else {
            const size_t chunk = (size_t)(argc > 4 ? atol(argv[4]) : 2048) << 20;
            arena = arena / chunk * chunk;
            hipMemAllocationProp prop = {};
            prop.type = hipMemAllocationTypePinned;
            prop.location.type = hipMemLocationTypeDevice;
            prop.location.id = 0;
            void *va = nullptr;
            CK(hipMemAddressReserve(&va, arena, 0, nullptr, 0));
            for (size_t off = 0; off < arena; off += chunk) {
                hipMemGenericAllocationHandle_t h;
                CK(hipMemCreate(&h, chunk, &prop, 0));
                CK(hipMemMap((char *)va + off, chunk, 0, h, 0));
            }
            hipMemAccessDesc acc = {};
            acc.location.type = hipMemLocationTypeDevice;
            acc.location.id = 0;
            acc.flags = hipMemAccessFlagsProtReadWrite;
            CK(hipMemSetAccess(va, arena, &acc, 1));
            big = (char *)va;
        }
        printf("{\"alloc\": %d, \"GB\": %.1f, \"ms\": %.1f}\n", how, arena / 1e9,
               std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        a = (float *)big;
        b = (float *)(big + kTotal * 4);
    } else if (offsets) {
        CK(hipMalloc((void **)&big, (size_t)kTotal * 4 * 2 + (256L << 20)));
        a = (float *)big;
        b = (float *)(big + kTotal * 4);
    } else {
        CK(hipMalloc(&a, kTotal * 4)); CK(hipMalloc(&b, kTotal * 4));
    }
    CK(hipMalloc(&g, 64 * 4));
    fill<<<4096, 256>>>(a, kTotal);
    fill<<<4096, 256>>>(b, kTotal);
    fill<<<1, 256>>>(g, 64);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const long tiles = L / R;
    auto run = [&](const char *name, auto launch) {
        launch(); CK(hipGetLastError()); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, 2.0 * kTotal * 4 / (ms * 1e6));
        fflush(stdout);
    };
    const size_t shm = 256 + 64 * ROWB + 64 * N * 4, wshm = (size_t)R * ROW * 4;
    auto go = [&](const char *name, auto k) {
        CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        run(name, [&] { hipLaunchKernelGGL(k, dim3(cus), dim3(1024), shm, 0, a, b, tiles, g); });
    };
    const size_t shm2 = 256 + 64 * ROWB;
    auto go1 = [&](const char *name, auto k, int occ) {
        CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        run(name, [&] { hipLaunchKernelGGL(k, dim3(occ * cus), dim3(1024), shm2, 0, a, b, tiles, g); });
    };
    auto gw = [&](const char *name, auto k) {
        CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        run(name, [&] { hipLaunchKernelGGL(k, dim3(cus), dim3(1024), wshm, 0, a, b, tiles); });
    };
    if (regions && argc > 6) {
        // padding / rotation sweep of the backward writes at the output
        // placements base + k GiB, k in argv[6] (comma list); input at 200 GiB
        char *fixedp = big + (200L << 30);
        fill<<<4096, 256>>>((float *)fixedp, kTotal);
        CK(hipFuncSetAttribute((const void *)bwdp, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        const long pads[] = {0, 64, 1024, 16384, 262144, 1048576};
        const long rots[] = {64, 1024, 16384, 262144};
        for (char *q = argv[6]; *q;) {
            const int k = (int)strtol(q, &q, 10);
            if (*q == ',') ++q;
            char *mv = big + ((size_t)k << 30);
            a = (float *)fixedp; b = (float *)mv;
            for (long pd : pads) {
                char lab[64]; snprintf(lab, sizeof lab, "k%d_pad%ld", k, pd);
                run(lab, [&] { hipLaunchKernelGGL(bwdp, dim3(cus), dim3(1024), shm, 0, a, b, tiles, g, L + pd, 0L); });
            }
            for (long rt : rots) {
                char lab[64]; snprintf(lab, sizeof lab, "k%d_rot%ld", k, rt);
                run(lab, [&] { hipLaunchKernelGGL(bwdp, dim3(cus), dim3(1024), shm, 0, a, b, tiles, g, L, rt); });
            }
        }
        return 0;
    }
    if (regions && argc > 5) {
        // fine sweep: the scattered side (forward input, backward output) at
        // base + k GiB for k = 0 .. argv[5]-1; the row side at base + 200 GiB
        const int nk = atoi(argv[5]);
        char *fixedp = big + (200L << 30);
        fill<<<4096, 256>>>((float *)fixedp, kTotal);
        for (int k = 0; k < nk; ++k) {
            char *mv = big + ((size_t)k << 30);
            fill<<<4096, 256>>>((float *)mv, kTotal);
            CK(hipDeviceSynchronize());
            printf("{\"gib\": %d}\n", k);
            a = (float *)mv; b = (float *)fixedp;
            go("fwd_rows", fwd<8>);
            a = (float *)fixedp; b = (float *)mv;
            go("bwd_swap_rows", bwd<12>);
        }
        return 0;
    }
    if (regions) {
        const int nreg = (int)(arena / (kTotal * 4));
        for (int k = 0; k + 1 < nreg; ++k) {
            a = (float *)(big + (size_t)k * kTotal * 4);
            b = (float *)(big + (size_t)(k + 1) * kTotal * 4);
            fill<<<4096, 256>>>(a, kTotal);
            CK(hipDeviceSynchronize());
            printf("{\"region\": %d}\n", k);
            go("fwd_rows", fwd<8>);
            go("bwd_swap_rows", bwd<12>);
        }
        return 0;
    }
    if (offsets) {
        const long deltas[] = {0, 64L << 10, 256L << 10, 1L << 20, 2L << 20, 4L << 20, 8L << 20, 16L << 20, 32L << 20,
                               48L << 20, 96L << 20, 160L << 20, 0};
        for (long dl : deltas) {
            b = (float *)(big + kTotal * 4 + dl);
            fill<<<4096, 256>>>(b, kTotal);
            CK(hipDeviceSynchronize());
            printf("{\"delta_bytes\": %ld}\n", dl);
            go("fwd_rows", fwd<8>);
            go("bwd_swap_rows", bwd<12>);
            // the other direction: b -> a
            std::swap(a, b);
            go("fwd_rows_ba", fwd<8>);
            go("bwd_swap_rows_ba", bwd<12>);
            std::swap(a, b);
        }
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        run("copy", [&] { copyf<<<kTotal / 1024, 256>>>((const v4f *)a, (v4f *)b); });
        gw("wide_fwd", wfwd);
        go("fwd_full", fwd<0>);
        go("fwd_noar", fwd<1>);
        go("fwd_noxi", fwd<2>);
        go("fwd_bare", fwd<3>);
        go("fwd_rows", fwd<8>);
        go("fwd_bare_rows", fwd<11>);
        gw("wide_bwd", wbwd);
        go("bwd_full", bwd<0>);
        go("bwd_noar", bwd<1>);
        go("bwd_noxi", bwd<2>);
        go("bwd_bare", bwd<3>);
        go("bwd_swap", bwd<4>);
        go("bwd_bare_swap", bwd<7>);
        go("bwd_swap_rows", bwd<12>);
        go("bwd_bare_swap_rows", bwd<15>);
        go1("fwd2_occ1", fwd2<1>, 1);
        go1("fwd2_occ2", fwd2<2>, 2);
        go1("bwd2_occ1", bwd2<1>, 1);
        go1("bwd2_occ2", bwd2<2>, 2);
    }
    return 0;
}
