// splitbw — the 8-bucket split run (chainsplit.cuh) with its real arithmetic,
// in two LDS structures, to find what the engine pays over the bare pattern
// of tools/widebw.hip (fwd 5.83 / bwd 5.43 ms per 2^32-entry message, no
// arithmetic, one LDS round trip):
//   XI  the engine's: phase 1 in registers, exchange table (16 x 4-B writes and
//       reads), phase 2, row image (4 x 16-B writes and reads), stores
//   RI  rows in place: phase-1 results go straight to the row image (16 x 4-B
//       writes), phase 2 reads its 16 contiguous row entries (4 x 16-B), writes
//       them back in place, stores read the image (28 LDS instructions per lane
//       per tile instead of 40, one 66-KiB region instead of two)
// Backward is the transpose (rows in, slab stores out).  G_j is a constant
// 2x2x2 table per bucket (dependency on the next slot) read packed from LDS
// as in the engine; products and sums in the engine's order.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/splitbw.hip -o build/splitbw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr long kTotal = 1L << 32;
constexpr int F = 8, N = 256, R = 64, W = 16;
constexpr long L = kTotal / N;                 // slab length
constexpr int ROWB = N * 4 + 16;               // image row stride (bytes)

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// one bucket on 16 local entries: slot J at local bit PJ; G(q, n, x) packed at
// gp[4 q + 2 n + x]; q = digit of slot J + 1 (local bit PQ, or uniform qu)
template <int PJ, int PQ>
__device__ __forceinline__ void step(float (&t)[16], const float *gp, int qu) {
    const v4f g0 = *(const v4f *)gp, g1 = *(const v4f *)(gp + 4);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        if (e & PJ) continue;
        const int q = PQ ? ((e & PQ) ? 1 : 0) : qu;
        const v4f g = q ? g1 : g0;
        const v2f m0 = {t[e], t[e]}, m1 = {t[e | PJ], t[e | PJ]};
        const v2f gx0 = {g[0], g[2]}, gx1 = {g[1], g[3]};
        const v2f a = gx0 * m0 + gx1 * m1;
        t[e] = a[0];
        t[e | PJ] = a[1];
    }
}

// phase 1: slots 0-3 local (slot p at bit 8 >> p), slot 4 = wave bit 3
__device__ __forceinline__ void phase1(float (&t)[16], const float *g, int w) {
    step<8, 4>(t, g + 0, 0);
    step<4, 2>(t, g + 8, 0);
    step<2, 1>(t, g + 16, 0);
    step<1, 0>(t, g + 24, (w >> 3) & 1);
}
// phase 2: slots 4-7 local (slot p at bit 8 >> (p - 4)); slot 8 does not exist
__device__ __forceinline__ void phase2(float (&t)[16], const float *g) {
    step<8, 4>(t, g + 32, 0);
    step<4, 2>(t, g + 40, 0);
    step<2, 1>(t, g + 48, 0);
    step<1, 0>(t, g + 56, 0);
}

template <bool RI, int DEPTH>
__global__ __launch_bounds__(1024) void fwd(const float *__restrict__ in, float *__restrict__ out, long tiles,
                                             const float *__restrict__ gsrc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);                      // 64 floats of G
    unsigned char *img0 = lds + 256;                                 // RI: two images (tile parity)
    float *xch = reinterpret_cast<float *>(lds + 256 + 64 * ROWB);    // XI only
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    const float *tb = in + (long)w * L + lane;                       // slab (e << 4 | w)
    auto load = [&](long tile, float (&v)[16]) {
        const float *p = tb + tile * R;
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = p[(long)e * 16 * L];
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    float ra[16], rb[16];
    load(tile, ra);
    if (DEPTH == 2) load(tile + gridDim.x < tiles ? tile + gridDim.x : tile, rb);
    float lmax = 0.f;
    int par = 0;
    while (true) {
        unsigned char *img = img0 + (RI ? par * 64 * ROWB : 0);
        par ^= 1;
        float t[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = ra[e];
        if (DEPTH == 2) {
#pragma unroll
            for (int e = 0; e < 16; ++e) ra[e] = rb[e];
        }
        const long nt = tile + DEPTH * gridDim.x < tiles ? tile + DEPTH * gridDim.x : tiles - 1;
        load(nt, DEPTH == 2 ? rb : ra);
        phase1(t, gt, w);
        if (RI) {
#pragma unroll
            for (int e = 0; e < 16; ++e) *(float *)(img + lane * ROWB + 4 * (e * 16 + w)) = t[e];
            lds_barrier();
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const v4f v = *(const v4f *)(img + lane * ROWB + 64 * w + 16 * c);
                t[4 * c] = v[0]; t[4 * c + 1] = v[1]; t[4 * c + 2] = v[2]; t[4 * c + 3] = v[3];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = t[e];
            lds_barrier();
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] = xch[(e * 16 + w) * 64 + lane];
        }
        phase2(t, gt);
#pragma unroll
        for (int e = 0; e < 16; ++e) lmax = fmaxf(lmax, t[e]);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *(v4f *)(img + lane * ROWB + 64 * w + 16 * c) = v4f{t[4 * c], t[4 * c + 1], t[4 * c + 2], t[4 * c + 3]};
        lds_barrier();
        float *ob = out + tile * (long)R * N;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int q = w * 256 + it * 64 + lane, rw = q / 64, ch = q % 64;
            const v4f v = *(const v4f *)(img + rw * ROWB + 16 * ch);
            __builtin_nontemporal_store(v, (v4f *)(ob + 4L * q));
        }
        if (tile + gridDim.x >= tiles) break;
        tile += gridDim.x;
    }
    if (lmax < 0.f) out[0] = lmax;                       // keep lmax live
}

template <bool RI, int DEPTH>
__global__ __launch_bounds__(1024) void bwd(const float *__restrict__ in, float *__restrict__ out, long tiles,
                                             const float *__restrict__ gsrc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);
    unsigned char *img0 = lds + 256;
    float *xch = reinterpret_cast<float *>(lds + 256 + 64 * ROWB);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    // rows of the tile: wave w loads rows 4w..4w+3, 16 B per lane per row
    auto load = [&](long tile, v4f (&v)[4]) {
        const float *p = in + tile * (long)R * N + (long)w * 4 * N + 4 * lane;
#pragma unroll
        for (int it = 0; it < 4; ++it) v[it] = *(const v4f *)(p + it * N);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    v4f ra[4], rb[4];
    load(tile, ra);
    if (DEPTH == 2) load(tile + gridDim.x < tiles ? tile + gridDim.x : tile, rb);
    // slot p of the row position is bit p (slot 0 fastest); the wave's digits
    // of slots 4-7 (phase 1): bit (7 - p) of w, placed at bits 4..7
    int fixed = 0;
#pragma unroll
    for (int p = 4; p < 8; ++p) fixed |= ((w >> (7 - p)) & 1) << p;
    float lmax = 0.f;
    int par = 0;
    while (true) {
        unsigned char *img = img0 + (RI ? par * 64 * ROWB : 0);
        par ^= 1;
        v4f cur[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) cur[it] = ra[it];
        if (DEPTH == 2) {
#pragma unroll
            for (int it = 0; it < 4; ++it) ra[it] = rb[it];
        }
        const long nt = tile + DEPTH * gridDim.x < tiles ? tile + DEPTH * gridDim.x : tiles - 1;
        load(nt, DEPTH == 2 ? rb : ra);
#pragma unroll
        for (int it = 0; it < 4; ++it) *(v4f *)(img + (4 * w + it) * ROWB + 16 * lane) = cur[it];
        lds_barrier();
        float u[16], t[16];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const v4f v = *(const v4f *)(img + lane * ROWB + 4 * fixed + 16 * c);
            u[4 * c] = v[0]; u[4 * c + 1] = v[1]; u[4 * c + 2] = v[2]; u[4 * c + 3] = v[3];
        }
        // local e: slot 0 = bit 3 ... slot 3 = bit 0 (row position bit p = slot p)
#pragma unroll
        for (int e = 0; e < 16; ++e) t[e] = u[((e >> 3) & 1) | (((e >> 2) & 1) << 1) | (((e >> 1) & 1) << 2) | ((e & 1) << 3)];
        phase1(t, gt, w);
        if (RI) {
            // back in place (position bits 0-3 = slots 0-3), then each lane takes
            // slots 4-7 for the wave's fixed n_0..n_3 = w (bit 3 - p of w at bit p)
#pragma unroll
            for (int e = 0; e < 16; ++e)
                u[((e >> 3) & 1) | (((e >> 2) & 1) << 1) | (((e >> 1) & 1) << 2) | ((e & 1) << 3)] = t[e];
#pragma unroll
            for (int c = 0; c < 4; ++c)
                *(v4f *)(img + lane * ROWB + 4 * fixed + 16 * c) = v4f{u[4 * c], u[4 * c + 1], u[4 * c + 2], u[4 * c + 3]};
            lds_barrier();
            int lo = 0;
#pragma unroll
            for (int p = 0; p < 4; ++p) lo |= ((w >> (3 - p)) & 1) << p;
            // local e: slot 4 = bit 3 ... slot 7 = bit 0 -> position bits 4..7
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int hi = (((e >> 3) & 1) << 4) | (((e >> 2) & 1) << 5) | (((e >> 1) & 1) << 6) | ((e & 1) << 7);
                t[e] = *(const float *)(img + lane * ROWB + 4 * (hi | lo));
            }
        } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = t[e];
            lds_barrier();
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] = xch[(e * 16 + w) * 64 + lane];
        }
        phase2(t, gt);
#pragma unroll
        for (int e = 0; e < 16; ++e) lmax = fmaxf(lmax, t[e]);
        // slab stores: n_0..n_3 = w, n_4..n_7 = e (n_0 most significant)
        float *ob = out + tile * (long)R + lane + (long)w * 16 * L;
#pragma unroll
        for (int e = 0; e < 16; ++e) __builtin_nontemporal_store(t[e], ob + (long)e * L);
        if (tile + gridDim.x >= tiles) break;
        tile += gridDim.x;
    }
    if (lmax < 0.f) out[0] = lmax;
}

__global__ __launch_bounds__(256) void copyf(const v4f *__restrict__ a, v4f *__restrict__ b) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    __builtin_nontemporal_store(a[i], b + i);
}

__global__ void fill(float *p, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = 0.5f + 0.25f * ((i * 2654435761u) % 1024) / 1024.f;
}

int main(int argc, char **argv) {
    const int reps = 5;
    float *a, *b, *g;
    // argv[1] = GB: both messages inside one allocation of that size, at its
    // two ends (the engine's 257-GB arena), instead of two 17-GB allocations
    const double arena_gb = argc > 1 ? atof(argv[1]) : 0;
    if (arena_gb > 0) {
        char *big = nullptr;
        const size_t bytes = (size_t)(arena_gb * 1e9);
        CK(hipMalloc((void **)&big, bytes));
        a = (float *)big;
        b = (float *)(big + ((bytes - kTotal * 4) & ~(size_t)((1 << 21) - 1)));
        printf("{\"arena_GB\": %.1f}\n", arena_gb);
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
    auto go = [&](const char *name, auto k, bool xi) {
        const size_t shm = 256 + 64 * ROWB + (xi ? 64 * N * 4 : 64 * ROWB);
        CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        run(name, [&] { hipLaunchKernelGGL(k, dim3(cus), dim3(1024), shm, 0, a, b, tiles, g); });
    };
    for (int rep = 0; rep < (arena_gb > 0 ? 1 : 2); ++rep) {
        run("copy", [&] { copyf<<<kTotal / 1024, 256>>>((const v4f *)a, (v4f *)b); });
        go("fwd_XI_d2", fwd<false, 2>, true);
        go("fwd_XI_d1", fwd<false, 1>, true);
        if (arena_gb == 0) {
            go("fwd_RI_d2", fwd<true, 2>, false);
            go("fwd_RI_d1", fwd<true, 1>, false);
        }
        go("bwd_XI_d1", bwd<false, 1>, true);
        go("bwd_XI_d2", bwd<false, 2>, true);
        if (arena_gb == 0) {
            go("bwd_RI_d1", bwd<true, 1>, false);
            go("bwd_RI_d2", bwd<true, 2>, false);
        }
    }
    return 0;
}
