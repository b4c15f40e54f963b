// membw — HBM ceilings for the bench bucket's access pattern on MI355X.
//   copy    : float4 grid-stride copy of N floats (the achievable read+write rate)
//   copy_nt : the same with nontemporal loads/stores
//   b4_dw   : out[j*4+y] = sum_x m[x*N/4 + j] * f[x*4+y]  — lane j: 4 dword loads, one float4 store
//   b4_dw2  : b4_dw with two j per lane (loads of both issued first)
//   b4_dw_nt: b4_dw with nontemporal loads/stores
// Build: hipcc -O3 --offload-arch=gfx950 tools/membw.hip -o build/membw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void copy_f4(const float4 *__restrict__ a, float4 *__restrict__ b, long n4) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void copy_f4_nt(const float4 *__restrict__ a, float4 *__restrict__ b, long n4) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load((const v4f *)a + i), (v4f *)b + i);
}

template <int J, bool NT>
__global__ __launch_bounds__(256) void b4(const float *__restrict__ m, const float *__restrict__ f,
                                          float4 *__restrict__ out, long nj) {
    float ff[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ff[i] = f[i];
    const long stride = (long)gridDim.x * blockDim.x * J;
    for (long j0 = blockIdx.x * (long)blockDim.x * J + threadIdx.x; j0 < nj; j0 += stride) {
        float x[J][4];
#pragma unroll
        for (int u = 0; u < J; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                long j = j0 + u * (long)blockDim.x;
                const float *p = m + v * nj + (j < nj ? j : 0);
                x[u][v] = NT ? __builtin_nontemporal_load(p) : *p;
            }
#pragma unroll
        for (int u = 0; u < J; ++u) {
            long j = j0 + u * (long)blockDim.x;
            float r[4];
#pragma unroll
            for (int y = 0; y < 4; ++y) {
                float acc = 0.f;
#pragma unroll
                for (int v = 0; v < 4; ++v) acc += x[u][v] * ff[v * 4 + y];
                r[y] = acc;
            }
            if (j < nj) {
                v4f o = {r[0], r[1], r[2], r[3]};
                if (NT) __builtin_nontemporal_store(o, (v4f *)out + j); else ((v4f *)out)[j] = o;
            }
        }
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : (1L << 30);     // floats per buffer
    const int reps = 10;
    float *a, *b, *f;
    CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&f, 64));
    CK(hipMemset(a, 0, n * 4)); CK(hipMemset(b, 0, n * 4));
    std::vector<float> hf(16, 0.25f);
    CK(hipMemcpy(f, hf.data(), 64, hipMemcpyHostToDevice));
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
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, 2.0 * n * 4 / (ms * 1e6));
    };
    for (int g : {cus * 4, cus * 8, cus * 16, cus * 32}) {
        char nm[64];
        snprintf(nm, sizeof nm, "copy g=%d", g);
        run(nm, [&] { copy_f4<<<g, 256>>>((const float4 *)a, (float4 *)b, n / 4); });
        snprintf(nm, sizeof nm, "copy_nt g=%d", g);
        run(nm, [&] { copy_f4_nt<<<g, 256>>>((const float4 *)a, (float4 *)b, n / 4); });
        snprintf(nm, sizeof nm, "b4_dw g=%d", g);
        run(nm, [&] { b4<1, false><<<g, 256>>>(a, f, (float4 *)b, n / 4); });
        snprintf(nm, sizeof nm, "b4_dw2 g=%d", g);
        run(nm, [&] { b4<2, false><<<g, 256>>>(a, f, (float4 *)b, n / 4); });
        snprintf(nm, sizeof nm, "b4_dw4 g=%d", g);
        run(nm, [&] { b4<4, false><<<g, 256>>>(a, f, (float4 *)b, n / 4); });
        snprintf(nm, sizeof nm, "b4_dw2_nt g=%d", g);
        run(nm, [&] { b4<2, true><<<g, 256>>>(a, f, (float4 *)b, n / 4); });
    }
    return 0;
}
