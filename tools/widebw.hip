// widebw — could a fused sweep run cover more than 8 buckets?  The bare access
// pattern of a run of F buckets over a 2^32-entry binary fp32 message, tiles of
// R rest entries (one workgroup of 1024 threads per tile, persistent grid, the
// next tile's loads in flight while the current one goes through LDS):
//   fwd<F,R>  reads 2^F slab pieces of R contiguous floats (slab stride 2^32 / 2^F),
//             transposes through LDS, writes R contiguous rows of 2^F floats
//   bwd<F,R>  the transpose: reads R rows, writes 2^F slab pieces
// The tile state is 2^F * R floats (64 KiB at F=8, R=64 -- the engine today;
// 128 KiB at F=9/R=64, F=10/R=32, F=11/R=16).  No bucket arithmetic: this is
// the ceiling of the layout, to compare with tools/slabpad.hip / chainbw.hip.
// Build: hipcc -O3 --offload-arch=gfx950 tools/widebw.hip -o build/widebw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr long kTotal = 1L << 32;

template <int F, int R>
__global__ __launch_bounds__(1024) void fwd(const float *__restrict__ in, float *__restrict__ out, long tiles) {
    constexpr int NS = 1 << F, T = NS * R, PER = T / 1024, ROW = NS + 4;
    constexpr long L = kTotal / NS;                       // slab length
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int t = threadIdx.x;
    float cur[PER], nxt[PER];
    // thread t: rest entry t % R of slab t / R + i * (1024 / R): one base
    // pointer, the rest are uniform strides (no per-load address registers)
    const float *tb = in + (long)(t / R) * L + (t % R);
    auto load = [&](long tile, float (&v)[PER]) {
        const float *p = tb + tile * R;
#pragma unroll
        for (int i = 0; i < PER; ++i) v[i] = __builtin_nontemporal_load(p + (long)i * (1024 / R) * L);
    };
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    load(tile, cur);
    while (true) {
        const long nt = tile + gridDim.x < tiles ? tile + gridDim.x : tile;
        load(nt, nxt);
        __syncthreads();                                  // the previous tile's LDS reads are done
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = i * 1024 + t, x = q / R, r = q % R;
            lds[r * ROW + x] = cur[i];
        }
        __syncthreads();
        float *ob = out + tile * (long)T;
#pragma unroll
        for (int j = 0; j < PER / 4; ++j) {
            const int q = (j * 1024 + t) * 4, r = q / NS, n = q % NS;
            const v4f v = *(const v4f *)(lds + r * ROW + n);
            __builtin_nontemporal_store(v, (v4f *)(ob + q));
        }
        if (nt == tile) break;
        tile = nt;
#pragma unroll
        for (int i = 0; i < PER; ++i) cur[i] = nxt[i];
    }
}

template <int F, int R>
__global__ __launch_bounds__(1024) void bwd(const float *__restrict__ in, float *__restrict__ out, long tiles) {
    constexpr int NS = 1 << F, T = NS * R, PER = T / 1024, ROW = NS + 4;
    constexpr long L = kTotal / NS;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int t = threadIdx.x;
    v4f cur[PER / 4], nxt[PER / 4];
    auto load = [&](long tile, v4f (&v)[PER / 4]) {
        const float *ib = in + tile * (long)T;
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
            const int q = (j * 1024 + t) * 4, r = q / NS, n = q % NS;
            *(v4f *)(lds + r * ROW + n) = cur[j];
        }
        __syncthreads();
        float *p = out + (long)(t / R) * L + (t % R) + tile * R;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int q = i * 1024 + t, x = q / R, r = q % R;
            __builtin_nontemporal_store(lds[r * ROW + x], p + (long)i * (1024 / R) * L);
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

int main() {
    const int reps = 4;
    float *a, *b;
    CK(hipMalloc(&a, kTotal * 4)); CK(hipMalloc(&b, kTotal * 4));
    CK(hipMemset(a, 0, kTotal * 4)); CK(hipMemset(b, 0, kTotal * 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, int F, int R, auto launch) {
        launch(); CK(hipGetLastError()); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"F\": %d, \"R\": %d, \"ms\": %.4f, \"GBps\": %.1f, \"ms_per_bucket\": %.4f}\n", name, F,
               R, ms, 2.0 * kTotal * 4 / (ms * 1e6), F ? ms / F : 0.0);
        fflush(stdout);
    };
    auto both = [&](auto fk, auto bk, int F, int R) {
        const long tiles = kTotal / ((1L << F) * R);
        const size_t shm = (size_t)R * ((1 << F) + 4) * 4;
        CK(hipFuncSetAttribute((const void *)fk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        CK(hipFuncSetAttribute((const void *)bk, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        const long grid = tiles < cus ? tiles : cus;
        run("fwd", F, R, [&] { hipLaunchKernelGGL(fk, dim3(grid), dim3(1024), shm, 0, a, b, tiles); });
        run("bwd", F, R, [&] { hipLaunchKernelGGL(bk, dim3(grid), dim3(1024), shm, 0, a, b, tiles); });
    };
    run("copy", 0, 0, [&] { copyf<<<kTotal / 1024, 256>>>((const v4f *)a, (v4f *)b); });
    both(fwd<8, 64>, bwd<8, 64>, 8, 64);
    both(fwd<8, 128>, bwd<8, 128>, 8, 128);
    both(fwd<9, 64>, bwd<9, 64>, 9, 64);
    both(fwd<10, 32>, bwd<10, 32>, 10, 32);
    both(fwd<10, 16>, bwd<10, 16>, 10, 16);
    both(fwd<11, 16>, bwd<11, 16>, 11, 16);
    both(fwd<12, 8>, bwd<12, 8>, 12, 8);
    run("copy", 0, 0, [&] { copyf<<<kTotal / 1024, 256>>>((const v4f *)a, (v4f *)b); });
    return 0;
}
