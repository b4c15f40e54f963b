// membw2 — where does the bench bucket's HBM rate go?  (k = 4, fp32)
//   copy        : float4 grid-stride copy (read + write ceiling)
//   read1/read4 : read-only sums over 1 stream / 4 slabs at distance S (no stores)
//   slab<pad>   : out[s*4+y] = sum_x m[x*(S+pad) + s] * f[x*4+y]; lane: 4 s x 4 y tile,
//                 float4 loads per x, 64-B rows transposed through a per-wave LDS image
//   inter       : same arithmetic with x fastest in m (m[s*4+x]): 4 float4 loads per lane
// Build: hipcc -O3 --offload-arch=gfx950 tools/membw2.hip -o build/membw2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void copy_f4(const v4f *__restrict__ a, v4f *__restrict__ b, long n4) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}

template <int NS>
__global__ __launch_bounds__(256) void readn(const v4f *__restrict__ a, long slab4, long n4, float *sink) {
    v4f acc = {0, 0, 0, 0};
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
#pragma unroll
        for (int x = 0; x < NS; ++x) acc += a[x * slab4 + i];
    }
    if (acc[0] == 12345.f) sink[0] = acc[1];
}

// 4 s x 4 y tile per lane; rows of 64 B go out through a per-wave LDS image
template <bool INTER, bool NT>
__global__ __launch_bounds__(256) void tile44(const float *__restrict__ m, const float *__restrict__ f,
                                              float *__restrict__ out, long S, long slab, long ntiles) {
    __shared__ __attribute__((aligned(16))) float img[4][64 * 20];
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = f[i];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *im = img[w];
    for (long t0 = blockIdx.x * 256L; t0 < ntiles; t0 += (long)gridDim.x * 256) {
        const long t = t0 + threadIdx.x;
        float x[4][4];                                   // [x][s]
        if (t < ntiles) {
            if (INTER) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {           // s = 4t + j: m[s*4 + x]
                    v4f v = *(const v4f *)(m + (4 * t + j) * 4);
#pragma unroll
                    for (int xx = 0; xx < 4; ++xx) x[xx][j] = v[xx];
                }
            } else {
#pragma unroll
                for (int xx = 0; xx < 4; ++xx) {
                    const v4f *p = (const v4f *)(m + xx * slab + 4 * t);
                    v4f v = NT ? __builtin_nontemporal_load(p) : *p;
#pragma unroll
                    for (int j = 0; j < 4; ++j) x[xx][j] = v[j];
                }
            }
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
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < 4; ++c) *(v4f *)(im + lane * 20 + 4 * c) = v4f{r[4 * c], r[4 * c + 1], r[4 * c + 2], r[4 * c + 3]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const long wt0 = t0 + (threadIdx.x & ~63);
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int q = it * 64 + lane, sl = q >> 2, wi = q & 3;
            if (wt0 + sl < ntiles) {
                v4f v = *(const v4f *)(im + sl * 20 + 4 * wi);
                v4f *o = (v4f *)(out + (wt0 * 16) + (long)q * 4);
                if (NT) __builtin_nontemporal_store(v, o); else *o = v;
            }
        }
    }
    (void)S;
}

// skewed slab loads: at step i a lane loads slab x for its iteration i + LEAD[x]
// (LEAD = 3,2,1,0: concurrent loads of one lane sit on different rows of the
// slabs) or, with SKEW = false, every slab one iteration ahead (plain prefetch)
template <bool SKEW>
__global__ __launch_bounds__(256) void tile44_pf(const float *__restrict__ m, const float *__restrict__ f,
                                                 float *__restrict__ out, long slab, long ntiles) {
    __shared__ __attribute__((aligned(16))) float img[4][64 * 20];
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = f[i];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *im = img[w];
    const long step = (long)gridDim.x * 256;
    const long first = blockIdx.x * 256L + threadIdx.x;
    auto ld = [&](int xx, long it) -> v4f {
        long t = first + it * step;
        if (t >= ntiles) t = first < ntiles ? first : 0;     // harmless re-read past the end
        return *(const v4f *)(m + xx * slab + 4 * t);
    };
    constexpr int L0 = SKEW ? 3 : 1, L1 = SKEW ? 2 : 1, L2 = SKEW ? 1 : 1, L3 = SKEW ? 0 : 1;
    v4f b0[4], b1[4], b2[4], b3[4];                      // b_x[d]: slab x of iteration i + d
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        if (d < L0) b0[d] = ld(0, d);
        if (d < L1) b1[d] = ld(1, d);
        if (d < L2) b2[d] = ld(2, d);
        if (d < L3) b3[d] = ld(3, d);
    }
    const long wbase = blockIdx.x * 256L + (threadIdx.x & ~63);
    for (long i = 0; wbase + i * step < ntiles; ++i) {
        b0[L0] = ld(0, i + L0); b1[L1] = ld(1, i + L1); b2[L2] = ld(2, i + L2); b3[L3] = ld(3, i + L3);
        float x[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) { x[0][j] = b0[0][j]; x[1][j] = b1[0][j]; x[2][j] = b2[0][j]; x[3][j] = b3[0][j]; }
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            if (d < L0) b0[d] = b0[d + 1];
            if (d < L1) b1[d] = b1[d + 1];
            if (d < L2) b2[d] = b2[d + 1];
            if (d < L3) b3[d] = b3[d + 1];
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
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < 4; ++c) *(v4f *)(im + lane * 20 + 4 * c) = v4f{r[4 * c], r[4 * c + 1], r[4 * c + 2], r[4 * c + 3]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const long wt0 = wbase + i * step;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int q = it * 64 + lane, sl = q >> 2, wi = q & 3;
            if (wt0 + sl < ntiles) {
                v4f v = *(const v4f *)(im + sl * 20 + 4 * wi);
                __builtin_nontemporal_store(v, (v4f *)(out + (wt0 * 16) + (long)q * 4));
            }
        }
    }
}

int main(int argc, char **argv) {
    const long S = argc > 1 ? atol(argv[1]) : (1L << 28);    // entries per x slab (bench: 4^14 * 4 = 2^30 / 4)
    const int reps = 10;
    const long pad_max = 1 << 16;
    float *a, *b, *f, *sink;
    CK(hipMalloc(&a, (4 * (S + pad_max)) * 4)); CK(hipMalloc(&b, 4 * S * 4)); CK(hipMalloc(&f, 64)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 0, (4 * (S + pad_max)) * 4)); CK(hipMemset(b, 0, 4 * S * 4));
    std::vector<float> hf(16, 0.25f);
    CK(hipMemcpy(f, hf.data(), 64, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int dev; hipDeviceProp_t pr; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&pr, dev));
    const int cus = pr.multiProcessorCount;
    auto run = [&](const char *name, double bytes, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e6));
        fflush(stdout);
    };
    const long n = 4 * S;          // floats read and written
    char nm[96];
    for (int g : {cus * 2, cus * 3, cus * 4}) {
        snprintf(nm, sizeof nm, "pf g=%d", g);
        run(nm, 2.0 * n * 4, [&] { tile44_pf<false><<<g, 256>>>(a, f, b, S, S / 4); });
        snprintf(nm, sizeof nm, "skew g=%d", g);
        run(nm, 2.0 * n * 4, [&] { tile44_pf<true><<<g, 256>>>(a, f, b, S, S / 4); });
        snprintf(nm, sizeof nm, "inter nt-store g=%d", g);
        run(nm, 2.0 * n * 4, [&] { tile44<true, true><<<g, 256>>>(a, f, b, S, S, S / 4); });
    }
    for (int g : {cus * 4, cus * 8}) {
        snprintf(nm, sizeof nm, "copy g=%d", g);
        run(nm, 2.0 * n * 4, [&] { copy_f4<<<g, 256>>>((const v4f *)a, (v4f *)b, n / 4); });
        snprintf(nm, sizeof nm, "read1 g=%d", g);
        run(nm, 1.0 * n * 4, [&] { readn<1><<<g, 256>>>((const v4f *)a, 0, n / 4, sink); });
        snprintf(nm, sizeof nm, "read4 g=%d", g);
        run(nm, 1.0 * n * 4, [&] { readn<4><<<g, 256>>>((const v4f *)a, S / 4, S / 4, sink); });
        snprintf(nm, sizeof nm, "read4 pad4k g=%d", g);
        run(nm, 1.0 * n * 4, [&] { readn<4><<<g, 256>>>((const v4f *)a, (S + 1024 + 16) / 4, S / 4, sink); });
        for (long pad : {0L, 64L, 1040L, 4096L + 320L, 65536L - 192L}) {
            snprintf(nm, sizeof nm, "slab pad=%ld g=%d", pad, g);
            run(nm, 2.0 * n * 4, [&] { tile44<false, false><<<g, 256>>>(a, f, b, S, S + pad, S / 4); });
        }
        snprintf(nm, sizeof nm, "slab nt g=%d", g);
        run(nm, 2.0 * n * 4, [&] { tile44<false, true><<<g, 256>>>(a, f, b, S, S, S / 4); });
        snprintf(nm, sizeof nm, "inter g=%d", g);
        run(nm, 2.0 * n * 4, [&] { tile44<true, false><<<g, 256>>>(a, f, b, S, S, S / 4); });
        snprintf(nm, sizeof nm, "inter nt-store g=%d", g);
        run(nm, 2.0 * n * 4, [&] { tile44<true, true><<<g, 256>>>(a, f, b, S, S, S / 4); });
    }
    return 0;
}
