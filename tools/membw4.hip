// membw4 — what read+write rate can a stream of float4 copies reach on this box?
// The bench bucket reads 4.29 GB and writes 4.29 GB per launch; this sweeps the
// copy shape (loads in flight per thread, grid size, workgroup size, cache
// policy) to find the achievable ceiling for that 1:1 read/write mix.
//   gs<U,NL,NS>   grid-stride: each iteration a thread issues U float4 loads
//                 (1 KiB per wave-instruction, U blocks of 256 float4 apart),
//                 then U stores; NL / NS = nontemporal loads / stores
//   flat<U>       one chunk of 256*U float4 per workgroup, grid = n / chunk
//   rd<U> / wr<U> read-only / write-only with the same shape
// Build: hipcc -O3 --offload-arch=gfx950 tools/membw4.hip -o build/membw4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int U, bool NL, bool NS, int TB>
__global__ __launch_bounds__(TB) void gs(const v4f *__restrict__ a, v4f *__restrict__ b, long n4) {
    const long chunk = (long)TB * U;
    for (long c = blockIdx.x * chunk; c < n4; c += (long)gridDim.x * chunk) {
        v4f r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const v4f *p = a + c + u * TB + threadIdx.x;
            r[u] = NL ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v4f *q = b + c + u * TB + threadIdx.x;
            if (NS) __builtin_nontemporal_store(r[u], q); else *q = r[u];
        }
    }
}

template <int U, bool NS>
__global__ __launch_bounds__(256) void flat(const v4f *__restrict__ a, v4f *__restrict__ b) {
    const long c = blockIdx.x * 256L * U;
    v4f r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = a[c + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        v4f *q = b + c + u * 256 + threadIdx.x;
        if (NS) __builtin_nontemporal_store(r[u], q); else *q = r[u];
    }
}

template <int U>
__global__ __launch_bounds__(256) void rd(const v4f *__restrict__ a, long n4, float *sink) {
    v4f acc = {0, 0, 0, 0};
    for (long c = blockIdx.x * 256L * U; c < n4; c += (long)gridDim.x * 256 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc += a[c + u * 256 + threadIdx.x];
    }
    if (acc[0] == 12345.f) sink[0] = acc[1];
}

template <int U, bool NS>
__global__ __launch_bounds__(256) void wr(v4f *__restrict__ b, long n4) {
    const v4f v = {1, 2, 3, 4};
    for (long c = blockIdx.x * 256L * U; c < n4; c += (long)gridDim.x * 256 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v4f *q = b + c + u * 256 + threadIdx.x;
            if (NS) __builtin_nontemporal_store(v, q); else *q = v;
        }
    }
}

int main(int argc, char **argv) {
    const long bytes = argc > 1 ? atol(argv[1]) : (1L << 32);   // per buffer (bench: 4.29 GB each way)
    const int reps = 10;
    const long n4 = bytes / 16;
    v4f *a, *b; float *sink;
    CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, bytes)); CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int dev; hipDeviceProp_t pr; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&pr, dev));
    const int cus = pr.multiProcessorCount;
    auto run = [&](const char *name, int g, double moved, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", name, g, ms, moved / (ms * 1e6));
        fflush(stdout);
    };
    const double cp = 2.0 * bytes;
#define GS(U, NL, NS, TB, G) run("gs U=" #U " nl=" #NL " ns=" #NS " tb=" #TB, G, cp, [&] { gs<U, NL, NS, TB><<<G, TB>>>(a, b, n4); })
    for (int m : {2, 4, 8, 16}) {
        const int g = cus * m;
        GS(1, false, false, 256, g);
        GS(2, false, false, 256, g);
        GS(4, false, false, 256, g);
        GS(8, false, false, 256, g);
        GS(4, false, true, 256, g);
        GS(4, true, true, 256, g);
        GS(4, true, false, 256, g);
        GS(2, false, true, 512, g / 2);
        GS(4, false, true, 512, g / 2);
        GS(2, false, true, 1024, g / 4);
    }
    run("flat U=1", (int)(n4 / 256), cp, [&] { flat<1, false><<<n4 / 256, 256>>>(a, b); });
    run("flat U=4", (int)(n4 / 1024), cp, [&] { flat<4, false><<<n4 / 1024, 256>>>(a, b); });
    run("flat U=4 ns", (int)(n4 / 1024), cp, [&] { flat<4, true><<<n4 / 1024, 256>>>(a, b); });
    run("flat U=8 ns", (int)(n4 / 2048), cp, [&] { flat<8, true><<<n4 / 2048, 256>>>(a, b); });
    for (int m : {4, 8, 16}) {
        const int g = cus * m;
        run("rd U=4", g, (double)bytes, [&] { rd<4><<<g, 256>>>(a, n4, sink); });
        run("rd U=8", g, (double)bytes, [&] { rd<8><<<g, 256>>>(a, n4, sink); });
        run("wr U=4", g, (double)bytes, [&] { wr<4, false><<<g, 256>>>(b, n4); });
        run("wr U=4 ns", g, (double)bytes, [&] { wr<4, true><<<g, 256>>>(b, n4); });
    }
    return 0;
}
