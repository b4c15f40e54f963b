// bwdprobe — where does the split run pay over the bare transpose?  On one box,
// back to back: the float4 copy, tools/widebw.hip's bare F=8/R=64 pattern (one
// LDS round trip, no arithmetic), and tools/splitbw.hip's XI run (the engine's
// structure) with parts removed:
//   bit 0  no bucket arithmetic (phase 1 / phase 2 skipped)
//   bit 1  no exchange table (the second LDS round trip and its barrier)
//   bit 2  (bwd) slab stores in widebw's order: wave w, store e -> slab 16 e + w
// Results are not checked (the removed parts make them wrong); only time.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/bwdprobe.hip -o build/bwdprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr long kTotal = 1L << 32;
constexpr int N = 256, R = 64;
constexpr long L = kTotal / N;
constexpr int ROWB = N * 4 + 16;
constexpr int ROW = N + 4;

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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
    constexpr bool AR = !(MODE & 1), XI = !(MODE & 2);
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
            const int q = w * 256 + it * 64 + lane, rw = q / 64, ch = q % 64;
            const v4f v = *(const v4f *)(img + rw * ROWB + 16 * ch);
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
    constexpr bool AR = !(MODE & 1), XI = !(MODE & 2), SWAP = MODE & 4;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float *gt = reinterpret_cast<float *>(lds);
    unsigned char *img = lds + 256;
    float *xch = reinterpret_cast<float *>(lds + 256 + 64 * ROWB);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) gt[threadIdx.x] = gsrc[threadIdx.x];
    __syncthreads();
    auto load = [&](long tile, v4f (&v)[4]) {
        const float *p = in + tile * (long)R * N + (long)w * 4 * N + 4 * lane;
#pragma unroll
        for (int it = 0; it < 4; ++it) v[it] = *(const v4f *)(p + it * N);
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
        for (int it = 0; it < 4; ++it) *(v4f *)(img + (4 * w + it) * ROWB + 16 * lane) = cur[it];
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

int main() {
    const int reps = 5;
    float *a, *b, *g;
    CK(hipMalloc(&a, kTotal * 4)); CK(hipMalloc(&b, kTotal * 4)); CK(hipMalloc(&g, 64 * 4));
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
    auto gw = [&](const char *name, auto k) {
        CK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        run(name, [&] { hipLaunchKernelGGL(k, dim3(cus), dim3(1024), wshm, 0, a, b, tiles); });
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("copy", [&] { copyf<<<kTotal / 1024, 256>>>((const v4f *)a, (v4f *)b); });
        gw("wide_fwd", wfwd);
        go("fwd_full", fwd<0>);
        go("fwd_noar", fwd<1>);
        go("fwd_noxi", fwd<2>);
        go("fwd_bare", fwd<3>);
        gw("wide_bwd", wbwd);
        go("bwd_full", bwd<0>);
        go("bwd_noar", bwd<1>);
        go("bwd_noxi", bwd<2>);
        go("bwd_bare", bwd<3>);
        go("bwd_swap", bwd<4>);
        go("bwd_bare_swap", bwd<7>);
    }
    return 0;
}
