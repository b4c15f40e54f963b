// splitbw64 -- the global access pattern of an fp64 forward split run of 7
// buckets (chainsplit.cuh, F = 7: 8 waves per 64-row tile, 16 slab loads of
// 8 B per lane, the tile's 64 rows of 1 KiB stored as 16-B chunks, chunk
// it * 512 + 64 w + lane), with no arithmetic and no LDS: what the pattern
// alone costs per 2^32-entry message, with one or two workgroups per CU and
// loads one tile ahead.  Also the fp32 F = 8 pattern (16 waves) for scale.
// Build: hipcc -O3 --offload-arch=gfx950 tools/splitbw64.hip -o build/splitbw64
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr long kTotal = 1L << 32;

template <typename T, int F>
__global__ __launch_bounds__(64 * (1 << (F - 4))) void fwd(const T *__restrict__ in, T *__restrict__ out, long tiles) {
    constexpr int N = 1 << F, W = 1 << (F - 4), VE = 16 / sizeof(T), IT = sizeof(T);
    constexpr long L = kTotal / N;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const T *tb = in + (long)w * L + lane;
    T cur[16], nxt[16];
    long tile = blockIdx.x;
    if (tile >= tiles) return;
    auto load = [&](long t, T (&v)[16]) {
        const T *p = tb + t * 64;
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = p[(long)e * W * L];
    };
    auto store = [&](long t, const T (&v)[16]) {
        T *o = out + t * 64 * N;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            typedef T vt __attribute__((ext_vector_type(VE)));
            vt x;
#pragma unroll
            for (int k = 0; k < VE; ++k) x[k] = v[VE * it + k];
            __builtin_nontemporal_store(x, (vt *)(o + (long)VE * (it * 64 * W + 64 * w + lane)));
        }
    };
    load(tile, cur);
    while (true) {
        const long tn = tile + gridDim.x;
        load(tn < tiles ? tn : tiles - 1, nxt);
        store(tile, cur);
        tile = tn;
        if (tile >= tiles) break;
        const long t2 = tile + gridDim.x;
        load(t2 < tiles ? t2 : tiles - 1, cur);
        store(tile, nxt);
        tile = t2;
        if (tile >= tiles) break;
    }
}

template <typename T, int F>
void run(const char *name, void *in, void *out, int cus, int per_cu) {
    constexpr int N = 1 << F, W = 1 << (F - 4);
    const long tiles = kTotal / N / 64;
    const int grid = cus * per_cu;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL((fwd<T, F>), dim3(grid), dim3(64 * W), 0, 0, (const T *)in, (T *)out, tiles);
    CK(hipEventRecord(a));
    const int reps = 5;
    for (int rep = 0; rep < reps; ++rep) hipLaunchKernelGGL((fwd<T, F>), dim3(grid), dim3(64 * W), 0, 0, (const T *)in, (T *)out, tiles);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double bytes = 2.0 * kTotal * sizeof(T);
    printf("%s: %d workgroups per CU (%d waves): %.3f ms per message, %.2f TB/s\n", name, per_cu, per_cu * W, ms, bytes / ms / 1e9);
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    void *in, *out;
    CK(hipMalloc(&in, kTotal * 8));
    CK(hipMalloc(&out, kTotal * 8));
    CK(hipMemset(in, 0, kTotal * 8));
    run<double, 7>("fp64 F=7", in, out, cus, 1);
    run<double, 7>("fp64 F=7", in, out, cus, 2);
    run<double, 7>("fp64 F=7", in, out, cus, 4);
    run<float, 8>("fp32 F=8", in, out, cus, 1);
    run<float, 8>("fp32 F=8", in, out, cus, 2);
    return 0;
}
