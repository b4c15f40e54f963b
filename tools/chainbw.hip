// chainbw — what bounds the fused sweep runs (chain.cuh) at ~5 TB/s?
// The forward run reads NS = K^F slabs (one per assignment of the run's summed
// variables, each contiguous along the rest index r) and writes one row of NS
// entries per r; the backward run is its transpose.  Same bytes as a copy, but
// NS read (or write) streams instead of one.  Variants:
//   fwd<NS, FLAT>   lane = one r: NS scalar slab loads, a mixing pass standing in
//                   for the F buckets, the row stored through a per-wave LDS image
//                   (128-B parts); FLAT: one workgroup per 256 r, else grid-stride
//                   over 3 workgroups per CU (the engine's chain launch)
//   bwd<NS, FLAT>   lane = one r: NS contiguous values (16-B loads), NS scalar
//                   slab stores
//   copy            flat float4 copy of the same bytes (the ceiling)
// Build: hipcc -O3 --offload-arch=gfx950 tools/chainbw.hip -o build/chainbw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int NS>
__device__ __forceinline__ void mix(float (&t)[NS]) {
#pragma unroll
    for (int b = 1; b < NS; b <<= 1)
#pragma unroll
        for (int a = 0; a < NS; ++a)
            if (!(a & b)) {
                const float x = t[a], y = t[a | b];
                t[a] = x * 0.75f + y * 0.25f;
                t[a | b] = x * 0.25f + y * 0.75f;
            }
}

template <int NS, bool FLAT>
__global__ __launch_bounds__(256) void fwd(const float *__restrict__ in, float *__restrict__ out, long L) {
    constexpr int PART = NS * 4 < 128 ? NS : 32;             // entries per 128-B row part
    constexpr int ROWP = PART * 4 + 16;
    __shared__ __attribute__((aligned(16))) unsigned char img[4][64 * ROWP];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned char *im = img[w];
    const long step = FLAT ? L : (long)gridDim.x * 256;
    for (long r0 = blockIdx.x * 256L; r0 < L; r0 += step) {
        const long r = r0 + threadIdx.x;
        float t[NS];
#pragma unroll
        for (int a = 0; a < NS; ++a) t[a] = in[(long)a * L + r];
        mix<NS>(t);
        const long wr0 = r0 + (threadIdx.x & ~63);
#pragma unroll
        for (int p = 0; p < NS / PART; ++p) {
            __syncthreads();
#pragma unroll
            for (int c = 0; c < PART / 4; ++c)
                *(v4f *)(im + lane * ROWP + 16 * c) = v4f{t[p * PART + 4 * c], t[p * PART + 4 * c + 1],
                                                          t[p * PART + 4 * c + 2], t[p * PART + 4 * c + 3]};
            __syncthreads();
            constexpr int CPR = PART / 4;                      // 16-B chunks per row part
#pragma unroll
            for (int it = 0; it < CPR; ++it) {
                const int q = it * 64 + lane, sl = q / CPR, wi = q % CPR;
                v4f v = *(const v4f *)(im + sl * ROWP + 16 * wi);
                __builtin_nontemporal_store(v, (v4f *)(out + (wr0 + sl) * NS + p * PART + 4 * wi));
            }
        }
    }
}

template <int NS, bool FLAT>
__global__ __launch_bounds__(256) void bwd(const float *__restrict__ in, float *__restrict__ out, long L) {
    const long step = FLAT ? L : (long)gridDim.x * 256;
    for (long r0 = blockIdx.x * 256L; r0 < L; r0 += step) {
        const long r = r0 + threadIdx.x;
        float t[NS];
#pragma unroll
        for (int c = 0; c < NS / 4; ++c) {
            v4f v = *(const v4f *)(in + r * NS + 4 * c);
            t[4 * c] = v[0]; t[4 * c + 1] = v[1]; t[4 * c + 2] = v[2]; t[4 * c + 3] = v[3];
        }
        mix<NS>(t);
#pragma unroll
        for (int a = 0; a < NS; ++a) __builtin_nontemporal_store(t[a], out + (long)a * L + r);
    }
}

// forward run of 64 slabs by one workgroup of 4 waves per 64 rest entries:
// wave w holds the 16 slabs whose two last slot digits are w (16 loads per
// lane, 256 B per slab per wave-instruction), runs buckets 0-3 in registers,
// exchanges through LDS, then produces the 16 outputs per row whose last two
// new-variable digits are w (buckets 4-5); rows leave through an LDS image.
template <int TBW>
__global__ __launch_bounds__(256) void fwd64split(const float *__restrict__ in, float *__restrict__ out, long L) {
    constexpr int ROWB = 256 + 16;                               // row image stride (bytes)
    __shared__ __attribute__((aligned(16))) unsigned char lds[64 * ROWB];
    float *xch = reinterpret_cast<float *>(lds);                 // [w][c][lane]: 4 * 16 * 64 floats = 16 KiB
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long r0 = blockIdx.x * 64L;
    float t[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) t[c] = in[(long)(4 * c + w) * L + r0 + lane];
    // buckets 0-3: slot j is bit (3 - j) of c
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        constexpr int dummy = 0; (void)dummy;
        const int b = 8 >> j;
#pragma unroll
        for (int c = 0; c < 16; ++c)
            if (!(c & b)) {
                const float x = t[c], y = t[c | b];
                t[c] = x * 0.75f + y * 0.25f;
                t[c | b] = x * 0.25f + y * 0.75f;
            }
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) xch[(w * 16 + c) * 64 + lane] = t[c];
    __syncthreads();
    const int n4 = w >> 1, n5 = w & 1;
    float o[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const float t00 = xch[(0 * 16 + c) * 64 + lane], t01 = xch[(1 * 16 + c) * 64 + lane];
        const float t10 = xch[(2 * 16 + c) * 64 + lane], t11 = xch[(3 * 16 + c) * 64 + lane];
        const float g0 = n4 ? 0.25f : 0.75f, g1 = n4 ? 0.75f : 0.25f;     // bucket 4 over x4
        const float u0 = t00 * g0 + t10 * g1, u1 = t01 * g0 + t11 * g1;
        o[c] = n5 ? u0 * 0.25f + u1 * 0.75f : u0 * 0.75f + u1 * 0.25f;   // bucket 5 over x5
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 16; ++c) *reinterpret_cast<float *>(lds + lane * ROWB + (4 * c + w) * 4) = o[c];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 4; ++it) {                             // wave w stores rows 16w .. 16w+15
        const int q = it * 64 + lane, row = w * 16 + q / 16, ch = q % 16;
        v4f v = *(const v4f *)(lds + row * ROWB + 16 * ch);
        __builtin_nontemporal_store(v, (v4f *)(out + (r0 + row) * 64 + 4 * ch));
    }
}

// runs of 8 buckets (256 slabs) by one workgroup of 16 waves per 64 rest
// entries.  Forward: wave w loads the 16 slabs whose slots 4-7 are w (256 B per
// slab per wave-instruction), buckets 0-3 in registers, exchange through LDS,
// wave w then holds new digits 0-3 = w and runs buckets 4-7; its 16 outputs
// per row are contiguous (64 B), rows leave through an LDS image (1 KiB rows).
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

__global__ __launch_bounds__(1024) void fwd256split16(const float *__restrict__ in, float *__restrict__ out, long L) {
    constexpr int ROWB = 1024 + 16;
    __shared__ __attribute__((aligned(16))) unsigned char lds[64 * ROWB];
    float *xch = reinterpret_cast<float *>(lds);                 // [w][c][lane]: 64 KiB
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long r0 = blockIdx.x * 64L;
    float t[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) t[c] = in[(long)(16 * c + w) * L + r0 + lane];
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
    for (int it = 0; it < 4; ++it) {                             // wave w stores rows 4w .. 4w+3
        const int row = 4 * w + it;
        v4f v = *(const v4f *)(lds + row * ROWB + 16 * lane);
        __builtin_nontemporal_store(v, (v4f *)(out + (r0 + row) * 256 + 4 * lane));
    }
}

// backward run of 8 buckets: the input tile (64 rows of 256 contiguous values)
// comes in by coalesced 16-B loads through LDS; wave w takes slots 4-7 = w of
// every row (buckets 0-3), exchange, then new digits 0-3 = w (buckets 4-7) and
// stores 16 output slabs per lane (256 B per slab per wave-instruction)
__global__ __launch_bounds__(1024) void bwd256split16(const float *__restrict__ in, float *__restrict__ out, long L) {
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
    for (int c = 0; c < 16; ++c) __builtin_nontemporal_store(t[c], out + (long)(16 * w + c) * L + r0 + lane);
}

__global__ __launch_bounds__(256) void copyf(const v4f *__restrict__ a, v4f *__restrict__ b) {
    const long i = blockIdx.x * 256L + threadIdx.x;
    __builtin_nontemporal_store(a[i], b + i);
}

template <int NS>
__global__ __launch_bounds__(64) void fwd_w(const float *__restrict__ in, float *__restrict__ out, long L) {
    __shared__ __attribute__((aligned(16))) unsigned char img[64 * (128 + 16)];
    const int lane = threadIdx.x;
    const long r0 = blockIdx.x * 64L, r = r0 + lane;
    float t[NS];
#pragma unroll
    for (int a = 0; a < NS; ++a) t[a] = in[(long)a * L + r];
    mix<NS>(t);
#pragma unroll
    for (int p = 0; p < NS / 32; ++p) {
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int c = 0; c < 8; ++c)
            *(v4f *)(img + lane * 144 + 16 * c) = v4f{t[p * 32 + 4 * c], t[p * 32 + 4 * c + 1], t[p * 32 + 4 * c + 2], t[p * 32 + 4 * c + 3]};
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int q = it * 64 + lane, sl = q / 8, wi = q % 8;
            v4f v = *(const v4f *)(img + sl * 144 + 16 * wi);
            __builtin_nontemporal_store(v, (v4f *)(out + (r0 + sl) * NS + p * 32 + 4 * wi));
        }
    }
}
static void fwd64_tb64(float *a, float *b, long total) { fwd_w<64><<<total / 64 / 64, 64>>>(a, b, total / 64); }

int main(int argc, char **argv) {
    const long total = argc > 1 ? atol(argv[1]) : (1L << 30);     // floats per buffer
    const int reps = 5;
    float *a, *b;
    CK(hipMalloc(&a, total * 4)); CK(hipMalloc(&b, total * 4));
    CK(hipMemset(a, 0, total * 4)); CK(hipMemset(b, 0, total * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int dev; hipDeviceProp_t pr; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&pr, dev));
    const int cus = pr.multiProcessorCount;
    auto run = [&](const char *name, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, 2.0 * total * 4 / (ms * 1e6));
        fflush(stdout);
    };
    run("copy", [&] { copyf<<<total / 1024, 256>>>((const v4f *)a, (v4f *)b); });
#define FW(NS) \
    run("fwd ns=" #NS " gs3", [&] { fwd<NS, false><<<cus * 3, 256>>>(a, b, total / NS); }); \
    run("fwd ns=" #NS " flat", [&] { fwd<NS, true><<<total / NS / 256, 256>>>(a, b, total / NS); }); \
    run("bwd ns=" #NS " gs3", [&] { bwd<NS, false><<<cus * 3, 256>>>(a, b, total / NS); }); \
    run("bwd ns=" #NS " flat", [&] { bwd<NS, true><<<total / NS / 256, 256>>>(a, b, total / NS); });
    FW(4) FW(16) FW(64)
    run("fwd ns=64 flat tb=64", [&] { fwd64_tb64(a, b, total); });
    run("fwd ns=64 split4", [&] { fwd64split<256><<<total / 64 / 64, 256>>>(a, b, total / 64); });
    run("fwd ns=256 split16", [&] { fwd256split16<<<total / 256 / 64, 1024>>>(a, b, total / 256); });
    run("bwd ns=256 split16", [&] { bwd256split16<<<total / 256 / 64, 1024>>>(a, b, total / 256); });
    run("copy", [&] { copyf<<<total / 1024, 256>>>((const v4f *)a, (v4f *)b); });
    return 0;
}
