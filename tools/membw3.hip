// membw3 — the fused sweep kernels' access patterns (16 slabs, fp32) and the
// effect of padding the slab distance off a power of two.
//   s2s  : read 16 slabs, write 16 slabs (same offsets)      float4 per lane
//   c2s  : read 64 contiguous floats per lane, write 16 slabs  (backward form)
//   s2c  : read 16 slabs, write 64 contiguous floats per lane through LDS (forward form, V = 4)
//   s2c1 : read 16 slabs (dword), write 16 contiguous floats per lane through LDS (forward form, V = 1)
// Build: hipcc -O3 --offload-arch=gfx950 tools/membw3.hip -o build/membw3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// MODE 0 s2s, 1 c2s, 2 s2c (V=4), 3 s2c1 (V=1)
template <int MODE>
__global__ __launch_bounds__(256) void k16(const float *__restrict__ in, float *__restrict__ out, long S, long slab,
                                           long nthreads) {
    __shared__ __attribute__((aligned(16))) float img[4][64 * 68];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int V = MODE == 3 ? 1 : 4;
    for (long t0 = blockIdx.x * 256L; t0 < nthreads; t0 += (long)gridDim.x * 256) {
        const long t = t0 + threadIdx.x;
        float v[16][V];
        if (t < nthreads) {
            if (MODE == 1) {
#pragma unroll
                for (int c = 0; c < 16; ++c) {
                    v4f x = *(const v4f *)(in + t * 64 + 4 * c);
                    v[c][0] = x[0]; v[c][1] = x[1]; v[c][2] = x[2]; v[c][3] = x[3];
                }
            } else if (MODE == 3) {
#pragma unroll
                for (int a = 0; a < 16; ++a) v[a][0] = in[a * slab + t];
            } else {
#pragma unroll
                for (int a = 0; a < 16; ++a) {
                    v4f x = *(const v4f *)(in + a * slab + 4 * t);
                    v[a][0] = x[0]; v[a][1] = x[1]; v[a][2] = x[2]; v[a][3] = x[3];
                }
            }
#pragma unroll
            for (int a = 0; a < 16; ++a)
#pragma unroll
                for (int u = 0; u < V; ++u) v[a][u] = v[a][u] * 1.0001f + 0.5f;
        }
        if (MODE == 0 || MODE == 1) {
            if (t < nthreads) {
#pragma unroll
                for (int a = 0; a < 16; ++a)
                    __builtin_nontemporal_store(v4f{v[a][0], v[a][1], v[a][2], v[a][3]}, (v4f *)(out + a * slab + 4 * t));
            }
        } else {
            // rows of 16*V floats per lane -> contiguous wave region via LDS
            constexpr int RW = 16 * V, RP = RW + 4;
            float *im = img[w];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int u = 0; u < V; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    *(v4f *)(im + lane * RP + u * 16 + 4 * c) = v4f{v[4 * c][u], v[4 * c + 1][u], v[4 * c + 2][u], v[4 * c + 3][u]};
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const long wt0 = t0 + (threadIdx.x & ~63);
            constexpr int CPR = RW / 4;
#pragma unroll
            for (int it = 0; it < CPR; ++it) {
                const int q = it * 64 + lane, sl = q / CPR, wi = q % CPR;
                if (wt0 + sl < nthreads)
                    __builtin_nontemporal_store(*(const v4f *)(im + sl * RP + 4 * wi), (v4f *)(out + wt0 * RW + (long)q * 4));
            }
        }
    }
    (void)S;
}

int main(int argc, char **argv) {
    const long S = argc > 1 ? atol(argv[1]) : (1L << 28);    // floats per slab (16 slabs)
    const long padmax = 1 << 16;
    const int reps = 5;
    float *a, *b;
    CK(hipMalloc(&a, 16 * (S + padmax) * 4)); CK(hipMalloc(&b, 16 * (S + padmax) * 4));
    CK(hipMemset(a, 0, 16 * (S + padmax) * 4)); CK(hipMemset(b, 0, 16 * (S + padmax) * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int dev; hipDeviceProp_t pr; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&pr, dev));
    const int cus = pr.multiProcessorCount;
    const double bytes = 2.0 * 16 * S * 4;
    auto run = [&](const char *name, auto launch) {
        launch(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
        printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e6));
        fflush(stdout);
    };
    char nm[96];
    for (int g : {cus * 2, cus * 3}) {
        for (long pad : {0L, 1040L, 4096L + 320L}) {
            const long sl = S + pad;
            snprintf(nm, sizeof nm, "s2s pad=%ld g=%d", pad, g);
            run(nm, [&] { k16<0><<<g, 256>>>(a, b, S, sl, S / 4); });
            snprintf(nm, sizeof nm, "c2s pad=%ld g=%d", pad, g);
            run(nm, [&] { k16<1><<<g, 256>>>(a, b, S, sl, S / 4); });
            snprintf(nm, sizeof nm, "s2c pad=%ld g=%d", pad, g);
            run(nm, [&] { k16<2><<<g, 256>>>(a, b, S, sl, S / 4); });
            snprintf(nm, sizeof nm, "s2c1 pad=%ld g=%d", pad, g);
            run(nm, [&] { k16<3><<<g, 256>>>(a, b, S, sl, S); });
        }
    }
    return 0;
}
