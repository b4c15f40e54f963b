// layoutbw — would a rotated message layout speed up the 8-bucket split runs
// (chainsplit.cuh)?  The dense canonical layout puts a forward run's 8 summed
// variables slowest: 256 slabs 64 MiB apart, one 256-B piece of each per tile.
// The rotated layout (newest group fastest, the next-summed group right above
// it: (N_{k-2}, N_{k-3}, X_k = N_{k-4}, B_k = N_{k-1})) puts the 256 slabs of a
// tile 1 KiB apart inside one 256-KiB block; the output rows (1 KiB each) land
// 256 KiB apart, consecutive tiles on adjacent rows.  Same tile work as the
// engine (16 waves per 64 rest entries, LDS exchange, rows through an image).
//   fwd/bwd      dense layout (the engine today)
//   fwdR/bwdR    rotated layout (bwdR is fwdR's transpose)
// Build: hipcc -O3 --offload-arch=gfx950 tools/layoutbw.hip -o build/layoutbw
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


// rotated forward: tile t = (a = t >> 2, 64-block of b = t & 3); input
// in[a * 65536 + x * 256 + b], output row (b * 65536 + a), 256 entries
__global__ __launch_bounds__(1024) void fwdR(const float *__restrict__ in, float *__restrict__ out) {
    constexpr int ROWB = 1024 + 16;
    __shared__ __attribute__((aligned(16))) unsigned char lds[64 * ROWB];
    float *xch = reinterpret_cast<float *>(lds);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long a = blockIdx.x >> 2, b0 = (blockIdx.x & 3) * 64L;
    const float *ib = in + a * 65536 + b0 + lane;
    float t[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) t[c] = ib[(long)(16 * c + w) * 256];
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
        __builtin_nontemporal_store(v, (v4f *)(out + ((b0 + row) * 65536 + a) * 256 + 4 * lane));
    }
}

// rotated backward (transpose of fwdR): input rows (b * 65536 + a), output
// out[a * 65536 + x * 256 + b]
__global__ __launch_bounds__(1024) void bwdR(const float *__restrict__ in, float *__restrict__ out) {
    constexpr int ROWB = 1024 + 16;
    __shared__ __attribute__((aligned(16))) unsigned char lds[64 * ROWB];
    float *xch = reinterpret_cast<float *>(lds);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long a = blockIdx.x >> 2, b0 = (blockIdx.x & 3) * 64L;
    v4f ld[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) ld[it] = *(const v4f *)(in + ((b0 + 4 * w + it) * 65536 + a) * 256 + 4 * lane);
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
    float *ob = out + a * 65536 + b0 + lane;
#pragma unroll
    for (int c = 0; c < 16; ++c) __builtin_nontemporal_store(t[c], ob + (long)(16 * w + c) * 256);
}

__global__ __launch_bounds__(256) void copyf(const v4f *__restrict__ a, v4f *__restrict__ b) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    __builtin_nontemporal_store(a[i], b + i);
}

int main() {
    const long L = 1L << 24;                               // rest entries
    const long total = 256 * L;                            // 2^32 floats per message
    const int reps = 5;
    float *a, *b;
    CK(hipMalloc(&a, total * 4)); CK(hipMalloc(&b, total * 4));
    CK(hipMemset(a, 0, total * 4)); CK(hipMemset(b, 0, total * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, 2.0 * total * 4 / (ms * 1e6));
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("copy", [&] { copyf<<<total / 1024, 256>>>((const v4f *)a, (v4f *)b); });
        run("fwd", [&] { fwd<<<L / 64, 1024>>>(a, b, L); });
        run("fwdR", [&] { fwdR<<<L / 64, 1024>>>(a, b); });
        run("bwd", [&] { bwd<<<L / 64, 1024>>>(a, b, L); });
        run("bwdR", [&] { bwdR<<<L / 64, 1024>>>(a, b); });
    }
    return 0;
}
