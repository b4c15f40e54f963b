// membw5 — one tile per workgroup ("flat" grid) vs grid-stride, on the copy and
// on the bench bucket's own shape  out[s*4 + y] = sum_x m[x*S + s] * f[x*4 + y]
// (k = 4, fp32: 4 read streams of S floats, one write stream of 4S floats).
// membw4 measured a flat float4 copy (one 4-KiB chunk per 256-thread
// workgroup) at 6.3 TB/s against 5.5-5.7 for every grid-stride shape.
//   copy<U,TB>        flat copy, U float4 per thread
//   tile44<TB,XCD>    4 s x 4 y per lane (float4 slab loads, 64-B rows out via LDS)
//   tile41<TB>        1 s x 4 y per lane (scalar slab loads, one float4 store)
//   tile42<TB>        2 s x 4 y per lane (float2 slab loads, two float4 stores)
//   XCD = 1: block b -> chunk (b % 8) * (nb / 8) + b / 8 (each XCD its own range)
// Build: hipcc -O3 --offload-arch=gfx950 tools/membw5.hip -o build/membw5
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ long chunk_of(int xcd, long nb) {
    const long b = blockIdx.x;
    if (!xcd) return b;
    const long per = nb / 8;
    return (b % 8) * per + b / 8;
}

template <int U, int TB, bool NS, int XCD>
__global__ __launch_bounds__(TB) void copyf(const v4f *__restrict__ a, v4f *__restrict__ b) {
    const long c = chunk_of(XCD, gridDim.x) * TB * U;
    v4f r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = a[c + u * TB + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        v4f *q = b + c + u * TB + threadIdx.x;
        if (NS) __builtin_nontemporal_store(r[u], q); else *q = r[u];
    }
}

template <int TB, int XCD, bool NS>
__global__ __launch_bounds__(TB) void tile44(const float *__restrict__ m, const float *__restrict__ f,
                                             float *__restrict__ out, long S) {
    __shared__ __attribute__((aligned(16))) float img[TB / 64][64 * 20];
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = f[i];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *im = img[w];
    const long t0 = chunk_of(XCD, gridDim.x) * TB;            // first tile (4 s values) of the block
    const long t = t0 + threadIdx.x;
    float x[4][4];
#pragma unroll
    for (int xx = 0; xx < 4; ++xx) {
        v4f v = *(const v4f *)(m + xx * S + 4 * t);
#pragma unroll
        for (int j = 0; j < 4; ++j) x[xx][j] = v[j];
    }
    float r[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            float acc = 0.f;
#pragma unroll
            for (int xx = 0; xx < 4; ++xx) acc += x[xx][j] * ff[xx * 4 + y];
            r[j * 4 + y] = acc;
        }
#pragma unroll
    for (int c = 0; c < 4; ++c) *(v4f *)(im + lane * 20 + 4 * c) = v4f{r[4 * c], r[4 * c + 1], r[4 * c + 2], r[4 * c + 3]};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const long wt0 = t0 + (threadIdx.x & ~63);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int q = it * 64 + lane, sl = q >> 2, wi = q & 3;
        v4f v = *(const v4f *)(im + sl * 20 + 4 * wi);
        v4f *o = (v4f *)(out + wt0 * 16 + (long)q * 4);
        if (NS) __builtin_nontemporal_store(v, o); else *o = v;
    }
}

template <int TB, int XCD>
__global__ __launch_bounds__(TB) void tile41(const float *__restrict__ m, const float *__restrict__ f,
                                             float *__restrict__ out, long S) {
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = f[i];
    const long s = chunk_of(XCD, gridDim.x) * TB + threadIdx.x;
    float x[4];
#pragma unroll
    for (int xx = 0; xx < 4; ++xx) x[xx] = m[xx * S + s];
    v4f r;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
        float acc = 0.f;
#pragma unroll
        for (int xx = 0; xx < 4; ++xx) acc += x[xx] * ff[xx * 4 + y];
        r[y] = acc;
    }
    __builtin_nontemporal_store(r, (v4f *)(out + s * 4));
}

template <int TB, int XCD>
__global__ __launch_bounds__(TB) void tile42(const float *__restrict__ m, const float *__restrict__ f,
                                             float *__restrict__ out, long S) {
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = f[i];
    const long t = chunk_of(XCD, gridDim.x) * TB + threadIdx.x;   // s = 2t, 2t+1
    float x[4][2];
#pragma unroll
    for (int xx = 0; xx < 4; ++xx) {
        v2f v = *(const v2f *)(m + xx * S + 2 * t);
        x[xx][0] = v[0]; x[xx][1] = v[1];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        v4f r;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            float acc = 0.f;
#pragma unroll
            for (int xx = 0; xx < 4; ++xx) acc += x[xx][j] * ff[xx * 4 + y];
            r[y] = acc;
        }
        __builtin_nontemporal_store(r, (v4f *)(out + (2 * t + j) * 4));
    }
}

int main(int argc, char **argv) {
    const long S = argc > 1 ? atol(argv[1]) : (1L << 28);   // entries per x slab (bench: 4^14 * 4 = 2^28)
    const int reps = 10;
    float *a, *b, *f;
    CK(hipMalloc(&a, 4 * S * 4)); CK(hipMalloc(&b, 4 * S * 4)); CK(hipMalloc(&f, 64));
    CK(hipMemset(a, 0, 4 * S * 4)); CK(hipMemset(b, 0, 4 * S * 4)); CK(hipMemset(f, 0, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, long g, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"grid\": %ld, \"ms\": %.4f, \"GBps\": %.1f}\n", name, g, ms, 2.0 * 4 * S * 4 / (ms * 1e6));
        fflush(stdout);
    };
    const long n4 = S;                       // float4s per buffer
    const v4f *a4 = (const v4f *)a; v4f *b4 = (v4f *)b;
#define CP(U, TB, NS, X) run("copy U=" #U " tb=" #TB " ns=" #NS " xcd=" #X, n4 / (TB * U), \
        [&] { copyf<U, TB, NS, X><<<n4 / (TB * U), TB>>>(a4, b4); })
    CP(1, 256, false, 0); CP(1, 256, true, 0); CP(1, 256, false, 1);
    CP(1, 64, false, 0); CP(1, 128, false, 0); CP(1, 512, false, 0); CP(1, 1024, false, 0);
    CP(2, 256, false, 0); CP(2, 128, false, 0); CP(4, 64, false, 0);
#define T44(TB, X, NS) run("tile44 tb=" #TB " xcd=" #X " ns=" #NS, S / 4 / TB, [&] { tile44<TB, X, NS><<<S / 4 / TB, TB>>>(a, f, b, S); })
    T44(256, 0, true); T44(256, 0, false); T44(256, 1, true); T44(128, 0, true); T44(64, 0, true); T44(64, 0, false);
#define T41(TB, X) run("tile41 tb=" #TB " xcd=" #X, S / TB, [&] { tile41<TB, X><<<S / TB, TB>>>(a, f, b, S); })
    T41(256, 0); T41(256, 1); T41(512, 0); T41(1024, 0); T41(128, 0);
#define T42(TB, X) run("tile42 tb=" #TB " xcd=" #X, S / 2 / TB, [&] { tile42<TB, X><<<S / 2 / TB, TB>>>(a, f, b, S); })
    T42(256, 0); T42(256, 1); T42(128, 0); T42(512, 0);
    CP(1, 256, false, 0);
    return 0;
}
