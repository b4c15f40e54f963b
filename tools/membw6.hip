// membw6 — why does a flat grid beat grid-stride on the copy (6.3 vs 5.6 TB/s)
// but not in the engine's stream kernel?  Hypotheses tested:
//   pf      grid-stride with the next chunk's loads issued before this chunk's
//           stores (vmcnt is in order: a load wait also waits for every older
//           store, so a plain grid-stride loop serialises on its own stores)
//   pre     flat tile with an engine-like preamble: descriptor fields read from
//           global memory (dependent chain) and the small table staged through
//           LDS with two barriers before the big loads
//   ntl     flat tile41 with nontemporal big loads (the single-op path's NTL)
// Build: hipcc -O3 --offload-arch=gfx950 tools/membw6.hip -o build/membw6
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// grid-stride copy, U float4 per thread per chunk; PF: loads of chunk c+1 before stores of chunk c
template <int U, bool PF>
__global__ __launch_bounds__(256) void copy_gs(const v4f *__restrict__ a, v4f *__restrict__ b, long n4) {
    const long chunk = 256L * U, step = (long)gridDim.x * chunk;
    long c = blockIdx.x * chunk;
    if (c >= n4) return;
    v4f r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = a[c + u * 256 + threadIdx.x];
    for (; c < n4; c += step) {
        v4f nx[U];
        const long cn = c + step;
        if (PF && cn < n4) {
#pragma unroll
            for (int u = 0; u < U; ++u) nx[u] = a[cn + u * 256 + threadIdx.x];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], b + c + u * 256 + threadIdx.x);
        if (cn < n4) {
            if (!PF) {
#pragma unroll
                for (int u = 0; u < U; ++u) nx[u] = a[cn + u * 256 + threadIdx.x];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = nx[u];
        }
    }
}

struct Desc { const float *m; const float *f; float *out; long S; long n_tiles; };

// tile41 (1 s x 4 y per lane), grid-stride, next tile's 4 slab loads before this tile's store
template <bool PF>
__global__ __launch_bounds__(256) void t41_gs(const float *__restrict__ m, const float *__restrict__ f,
                                              float *__restrict__ out, long S) {
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = f[i];
    const long step = (long)gridDim.x * 256;
    long s = blockIdx.x * 256L + threadIdx.x;
    float x[4];
#pragma unroll
    for (int xx = 0; xx < 4; ++xx) x[xx] = m[xx * S + s];
    for (; s < S; s += step) {
        float nx[4];
        const long sn = s + step < S ? s + step : s;
        if (PF) {
#pragma unroll
            for (int xx = 0; xx < 4; ++xx) nx[xx] = m[xx * S + sn];
        }
        v4f r;
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            float acc = 0.f;
#pragma unroll
            for (int xx = 0; xx < 4; ++xx) acc += x[xx] * ff[xx * 4 + y];
            r[y] = acc;
        }
        __builtin_nontemporal_store(r, (v4f *)(out + s * 4));
        if (!PF) {
#pragma unroll
            for (int xx = 0; xx < 4; ++xx) nx[xx] = m[xx * S + sn];
        }
#pragma unroll
        for (int xx = 0; xx < 4; ++xx) x[xx] = nx[xx];
    }
}

// flat tile41 with an engine-like preamble (descriptor in global memory, f staged in LDS)
template <bool PRE, bool NTL>
__global__ __launch_bounds__(256) void t41_flat(const Desc *__restrict__ dp, const float *__restrict__ m0,
                                                const float *__restrict__ f0, float *__restrict__ out0, long S0) {
    __shared__ float fl[16];
    const float *m = m0, *f = f0;
    float *out = out0;
    long S = S0;
    if (PRE) {
        const Desc d = *dp;
        m = d.m; f = d.f; out = d.out; S = d.S;
        if (threadIdx.x < 16) fl[threadIdx.x] = f[threadIdx.x];
        __syncthreads();
    }
    const long s = blockIdx.x * 256L + threadIdx.x;
    float x[4];
#pragma unroll
    for (int xx = 0; xx < 4; ++xx) x[xx] = NTL ? __builtin_nontemporal_load(m + xx * S + s) : m[xx * S + s];
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = PRE ? fl[i] : f[i];
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

int main(int argc, char **argv) {
    const long S = argc > 1 ? atol(argv[1]) : (1L << 28);
    const int reps = 10;
    float *a, *b, *f;
    Desc *dd;
    CK(hipMalloc(&a, 4 * S * 4)); CK(hipMalloc(&b, 4 * S * 4)); CK(hipMalloc(&f, 64)); CK(hipMalloc(&dd, sizeof(Desc)));
    CK(hipMemset(a, 0, 4 * S * 4)); CK(hipMemset(b, 0, 4 * S * 4)); CK(hipMemset(f, 0, 64));
    Desc hd{a, f, b, S, S};
    CK(hipMemcpy(dd, &hd, sizeof hd, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int dev; hipDeviceProp_t pr; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&pr, dev));
    const int cus = pr.multiProcessorCount;
    auto run = [&](const char *name, long g, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"grid\": %ld, \"ms\": %.4f, \"GBps\": %.1f}\n", name, g, ms, 2.0 * 4 * S * 4 / (ms * 1e6));
        fflush(stdout);
    };
    const v4f *a4 = (const v4f *)a; v4f *b4 = (v4f *)b;
    for (int mult : {2, 4, 8, 16}) {
        const int g = cus * mult;
        run("copy_gs U=1", g, [&] { copy_gs<1, false><<<g, 256>>>(a4, b4, S); });
        run("copy_gs U=1 pf", g, [&] { copy_gs<1, true><<<g, 256>>>(a4, b4, S); });
        run("copy_gs U=2 pf", g, [&] { copy_gs<2, true><<<g, 256>>>(a4, b4, S); });
        run("t41_gs", g, [&] { t41_gs<false><<<g, 256>>>(a, f, b, S); });
        run("t41_gs pf", g, [&] { t41_gs<true><<<g, 256>>>(a, f, b, S); });
    }
    const long nb = S / 256;
    run("t41_flat", nb, [&] { t41_flat<false, false><<<nb, 256>>>(dd, a, f, b, S); });
    run("t41_flat ntl", nb, [&] { t41_flat<false, true><<<nb, 256>>>(dd, a, f, b, S); });
    run("t41_flat pre", nb, [&] { t41_flat<true, false><<<nb, 256>>>(dd, a, f, b, S); });
    run("t41_flat pre ntl", nb, [&] { t41_flat<true, true><<<nb, 256>>>(dd, a, f, b, S); });
    return 0;
}
