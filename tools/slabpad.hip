// slabpad — does the power-of-two slab spacing of a 2^32-entry message cost
// bandwidth in the 8-bucket split runs (chainsplit.cuh)?
// A forward run reads 256 slabs of L = 2^24 floats (one per assignment of its
// summed variables), 64 MiB apart in the dense canonical layout, and writes
// 1-KiB rows; a backward run is the transpose.  Here the slabs sit S = L + pad
// floats apart; pad = 0 is the engine's layout.  Same tile shape as the engine
// (16 waves per 64 rest entries, LDS exchange, 1-KiB rows through an image).
// Build: hipcc -O3 --offload-arch=gfx950 tools/slabpad.hip -o build/slabpad
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ void mix16(float (&t)[16]) {
#pragma unroll
    for (int b = 1; b < 16; b <<= 1)
#pragma unroll
        for (int a = 0; a < 16; ++a)
            if (!(a & b)) {
                const float x = t[a], y = t[a | b];
                t[a] = x * 0.75f + y * 0.25f;
                t[a | b] = x * 0.25f + y * 0.75f;
            }
}

// forward: slab c*16+w of the input (stride S floats), rows of 256 out
__global__ __launch_bounds__(1024) void fwd(const float *__restrict__ in, float *__restrict__ out, long S) {
    constexpr int ROWB = 1024 + 16;
    __shared__ __attribute__((aligned(16))) unsigned char lds[64 * ROWB];
    float *xch = reinterpret_cast<float *>(lds);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long r0 = blockIdx.x * 64L;
    float t[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) t[c] = in[(long)(16 * c + w) * S + r0 + lane];
    mix16(t);
#pragma unroll
    for (int c = 0; c < 16; ++c) xch[(w * 16 + c) * 64 + lane] = t[c];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 16; ++c) t[c] = xch[(c * 16 + w) * 64 + lane];
    mix16(t);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c)
        *(v4f *)(lds + lane * ROWB + w * 64 + 16 * c) = v4f{t[4 * c], t[4 * c + 1], t[4 * c + 2], t[4 * c + 3]};
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int row = 4 * w + it;
        v4f v = *(const v4f *)(lds + row * ROWB + 16 * lane);
        __builtin_nontemporal_store(v, (v4f *)(out + (r0 + row) * 256 + 4 * lane));
    }
}

// backward: rows of 256 in, 256 output slabs (stride S floats)
__global__ __launch_bounds__(1024) void bwd(const float *__restrict__ in, float *__restrict__ out, long S) {
    constexpr int ROWB = 1024 + 16;
    __shared__ __attribute__((aligned(16))) unsigned char lds[64 * ROWB];
    float *xch = reinterpret_cast<float *>(lds);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long r0 = blockIdx.x * 64L;
    v4f ld[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) ld[it] = *(const v4f *)(in + (r0 + 4 * w + it) * 256 + 4 * lane);
#pragma unroll
    for (int it = 0; it < 4; ++it) *(v4f *)(lds + (4 * w + it) * ROWB + 16 * lane) = ld[it];
    __syncthreads();
    float t[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        v4f v = *(const v4f *)(lds + lane * ROWB + w * 64 + 16 * c);
        t[4 * c] = v[0]; t[4 * c + 1] = v[1]; t[4 * c + 2] = v[2]; t[4 * c + 3] = v[3];
    }
    mix16(t);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 16; ++c) xch[(w * 16 + c) * 64 + lane] = t[c];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 16; ++c) t[c] = xch[(c * 16 + w) * 64 + lane];
    mix16(t);
#pragma unroll
    for (int c = 0; c < 16; ++c) __builtin_nontemporal_store(t[c], out + (long)(16 * w + c) * S + r0 + lane);
}

__global__ __launch_bounds__(256) void copyf(const v4f *__restrict__ a, v4f *__restrict__ b) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    __builtin_nontemporal_store(a[i], b + i);
}

int main(int argc, char **argv) {
    const long L = argc > 1 ? atol(argv[1]) : (1L << 24);     // rest entries (slab length)
    const long total = 256 * L;
    const long maxpad = 1L << 16;
    const int reps = 5;
    float *a, *b;
    CK(hipMalloc(&a, (256 * (L + maxpad)) * 4)); CK(hipMalloc(&b, (256 * (L + maxpad)) * 4));
    CK(hipMemset(a, 0, (256 * (L + maxpad)) * 4)); CK(hipMemset(b, 0, (256 * (L + maxpad)) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, long pad, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"pad_floats\": %ld, \"ms\": %.4f, \"GBps\": %.1f}\n", name, pad, ms,
               2.0 * total * 4 / (ms * 1e6));
        fflush(stdout);
    };
    run("copy", 0, [&] { copyf<<<total / 1024, 256>>>((const v4f *)a, (v4f *)b); });
    const long pads[] = {0, 16, 64, 256, 1024, 4096, 4096 + 64, 16384 + 1024, 65536 - 64};
    for (long pad : pads) {
        const long S = L + pad;
        run("fwd", pad, [&] { fwd<<<L / 64, 1024>>>(a, b, S); });
        run("bwd", pad, [&] { bwd<<<L / 64, 1024>>>(a, b, S); });
    }
    run("copy", 0, [&] { copyf<<<total / 1024, 256>>>((const v4f *)a, (v4f *)b); });
    return 0;
}
