// Message exchange steps of sliced bucket-tree runs (plan.hpp BucketSpec::xchg,
// DESIGN §6): the device side of one re-slicing of a message between the ranks.
//
// A message sliced over R = 2^b ranks is stored by each rank as its block
// (the slice variables fixed to the rank's bits) with its own power-of-two
// scale (TableMeta::exp2, maxbits).  Before the blocks travel, every rank's
// largest true exponent E_r = exp2 + exponent(max) and its exp2 are
// all-gathered (sync: 16 B per rank, x[2r] = E_r, x[2r + 1] = exp2_r); the
// pack step then writes the rank's block at the common exponent C = max_r E_r
// (stored * 2^(exp2 - C), exact power-of-two scaling; values 2^-4096 below the
// largest flush to zero as fp32/fp64 would) in the order the collective sends
// it -- destination blocks slowest -- so the received message holds one scale.
// Where the destination blocks already are the slowest and the received
// message is transposed anyway (the backward lane), the pack is skipped: the
// raw block travels and the unpack scales each source block b by
// 2^(exp2_b - C) as it transposes (mode 2) -- the same ldexp on the same
// values, one data pass instead of two.
// Pack / unpack are the only data passes: a straight copy, or an R-way
// transpose when the slice variables are the fastest of the layout (each
// thread moves the R values of one inner entry: one contiguous R-vector on the
// transposed side, R coalesced streams on the other).  HBM-bound; 2 x 4 B per
// entry for fp32.
#include <hip/hip_runtime.h>

#include "kernels.cuh"

namespace bnpp {

namespace {

constexpr int64_t kNoExp = -((int64_t)1 << 40);    // an all-zero block: below every other rank

template <typename T>
__global__ void xchg_sync_kernel(const TableMeta *__restrict__ meta, int in_t, int x_t, int R) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const TableMeta m = meta[in_t];
        int64_t *x = static_cast<int64_t *>(meta[x_t].ptr);
        x[2 * R] = m.maxbits == 0 ? kNoExp : m.exp2 + (int64_t)FBits<T>::exponent(m.maxbits);
        x[2 * R + 1] = m.exp2;
    }
}

// the common exponent C = max_r E_r of the gathered (E_r, exp2_r) pairs
__device__ __forceinline__ int64_t common_exp(const int64_t *x, int R) {
    int64_t c = x[0];
    for (int r = 1; r < R; ++r) c = x[2 * r] > c ? x[2 * r] : c;
    return c;
}
__device__ __forceinline__ int clamp_shift(int64_t d) { return (int)(d < -4096 ? -4096 : d > 4096 ? 4096 : d); }

// mode 0: out = in * 2^sh (same order, 16-B vectors); mode 1: out[b * inner + j] =
// in[j * R + b] * 2^sh -- a thread reads its entry's R values as one vector
// (RC: R at compile time, 0 = runtime R), the lanes' writes to each block coalesce
template <typename T, int RC>
__global__ __launch_bounds__(256) void xchg_pack_kernel(TableMeta *__restrict__ meta, int in_t, int x_t, int out_t, int R,
                                                        int mode, int64_t n) {
    const int64_t c = common_exp(static_cast<const int64_t *>(meta[x_t].ptr), R);
    const TableMeta mi = meta[in_t];
    const int sh = clamp_shift(mi.exp2 - c);
    const T *__restrict__ in = static_cast<const T *>(mi.ptr);
    T *__restrict__ out = static_cast<T *>(meta[out_t].ptr);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (mode == 0) {
        constexpr int V = 16 / sizeof(T);
        const int64_t nv = n / V;
        for (int64_t i = t0; i < nv; i += stride) {
            vec_t<T, V> v = reinterpret_cast<const vec_t<T, V> *>(in)[i];
#pragma unroll
            for (int k = 0; k < V; ++k) v[k] = ldexp_t(v[k], sh);
            reinterpret_cast<vec_t<T, V> *>(out)[i] = v;
        }
        for (int64_t i = nv * V + t0; i < n; i += stride) out[i] = ldexp_t(in[i], sh);
    } else if constexpr (RC > 0) {
        const int64_t inner = n / RC;
        if (inner % 4 == 0) {
            // four consecutive entries per thread: four R-vector loads, then
            // one 4-entry vector store per block (a wave's store is 1 KiB
            // contiguous fp32 instead of 256 B: 1.30 ms per 2^29-entry fp32
            // block before, 3.3 TB/s)
            for (int64_t q = t0; q < inner / 4; q += stride) {
                const int64_t j = q * 4;
                vec_t<T, RC> v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = reinterpret_cast<const vec_t<T, RC> *>(in)[j + u];
#pragma unroll
                for (int b = 0; b < RC; ++b) {
                    vec_t<T, 4> w;
#pragma unroll
                    for (int u = 0; u < 4; ++u) w[u] = ldexp_t(v[u][b], sh);
                    *reinterpret_cast<vec_t<T, 4> *>(out + b * inner + j) = w;
                }
            }
        } else {
            for (int64_t j = t0; j < inner; j += stride) {
                const vec_t<T, RC> v = reinterpret_cast<const vec_t<T, RC> *>(in)[j];
#pragma unroll
                for (int b = 0; b < RC; ++b) out[b * inner + j] = ldexp_t(v[b], sh);
            }
        }
    } else {
        const int64_t inner = n / R;
        for (int64_t j = t0; j < inner; j += stride)
            for (int b = 0; b < R; ++b) out[b * inner + j] = ldexp_t(in[j * R + b], sh);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        meta[out_t].exp2 = c;
        meta[out_t].maxbits = FBits<T>::bits(T(0.75));   // every rank's block now lies below 2^0
    }
}

// out[j * R + b] = in[b * inner + j]: R coalesced reads, one vector store.
// x_t >= 0 (mode 2): in holds every rank's raw block (no pack scaled them) and
// source block b is scaled by 2^(exp2_b - C) on the way, as b's pack would
// have; x_t < 0: in is already at one scale
template <typename T, int RC>
__global__ __launch_bounds__(256) void xchg_unpack_kernel(TableMeta *__restrict__ meta, int in_t, int x_t, int out_t,
                                                          int R, int64_t n) {
    const TableMeta mi = meta[in_t];
    const T *__restrict__ in = static_cast<const T *>(mi.ptr);
    T *__restrict__ out = static_cast<T *>(meta[out_t].ptr);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t *x = x_t >= 0 ? static_cast<const int64_t *>(meta[x_t].ptr) : nullptr;
    const int64_t c = x ? common_exp(x, R) : 0;
    auto shift = [&](int b) { return x ? clamp_shift(x[2 * b + 1] - c) : 0; };
    if constexpr (RC > 0) {
        int sh[RC];
#pragma unroll
        for (int b = 0; b < RC; ++b) sh[b] = shift(b);
        const int64_t inner = n / RC;
        if (inner % 4 == 0) {
            // four consecutive entries per thread: one 4-entry vector load per
            // block, four R-vector stores (1.32 ms per 2^29-entry fp32 block before)
            for (int64_t q = t0; q < inner / 4; q += stride) {
                const int64_t j = q * 4;
                vec_t<T, 4> w[RC];
#pragma unroll
                for (int b = 0; b < RC; ++b) w[b] = *reinterpret_cast<const vec_t<T, 4> *>(in + b * inner + j);
                if (x) {
#pragma unroll
                    for (int b = 0; b < RC; ++b)
#pragma unroll
                        for (int u = 0; u < 4; ++u) w[b][u] = ldexp_t(w[b][u], sh[b]);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    vec_t<T, RC> v;
#pragma unroll
                    for (int b = 0; b < RC; ++b) v[b] = w[b][u];
                    reinterpret_cast<vec_t<T, RC> *>(out)[j + u] = v;
                }
            }
        } else {
            for (int64_t j = t0; j < inner; j += stride) {
                vec_t<T, RC> v;
#pragma unroll
                for (int b = 0; b < RC; ++b) v[b] = x ? ldexp_t(in[b * inner + j], sh[b]) : in[b * inner + j];
                reinterpret_cast<vec_t<T, RC> *>(out)[j] = v;
            }
        }
    } else {
        const int64_t inner = n / R;
        for (int64_t j = t0; j < inner; j += stride)
            for (int b = 0; b < R; ++b) out[j * R + b] = x ? ldexp_t(in[b * inner + j], shift(b)) : in[b * inner + j];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        meta[out_t].exp2 = x ? c : mi.exp2;
        // (as the pack: every rank's block now lies below 2^0)
        meta[out_t].maxbits = x ? FBits<T>::bits(T(0.75)) : mi.maxbits;
    }
}

__global__ void xchg_meta_kernel(TableMeta *__restrict__ meta, int in_t, int out_t) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        meta[out_t].exp2 = meta[in_t].exp2;
        meta[out_t].maxbits = meta[in_t].maxbits;
    }
}

// one wave sleeping on the device clock for `ticks`: the stream it is on
// waits that long while other streams' kernels run (the loopback collective's
// stand-in for a transfer's duration)
__global__ void delay_kernel(uint64_t ticks) {
    if (threadIdx.x == 0) {
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    }
}

unsigned grid_for(int64_t work) {
    const int64_t g = (work + 255) / 256;
    return (unsigned)(g < 1 ? 1 : g > 16384 ? 16384 : g);
}

}  // namespace

hipError_t launch_xchg_sync(bool f32, TableMeta *meta, int in_t, int x_t, int R, hipStream_t s) {
    if (f32) hipLaunchKernelGGL(xchg_sync_kernel<float>, dim3(1), dim3(64), 0, s, meta, in_t, x_t, R);
    else hipLaunchKernelGGL(xchg_sync_kernel<double>, dim3(1), dim3(64), 0, s, meta, in_t, x_t, R);
    return hipGetLastError();
}

// R = 2, 4, 8 with the entry's R values one vector (8 / 16 / 32 B for fp32)
#define BNPP_XCHG_R(X) \
    switch (R) {       \
        case 2: X(2); break; \
        case 4: X(4); break; \
        case 8: X(8); break; \
        default: X(0); break; \
    }

hipError_t launch_xchg_pack(bool f32, TableMeta *meta, int in_t, int x_t, int out_t, int R, int mode, int64_t n,
                            hipStream_t s) {
    const unsigned g = grid_for(mode == 0 ? n / 4 : n / R / 4);
#define BNPP_PACK(RC)                                                                                            \
    if (f32) hipLaunchKernelGGL((xchg_pack_kernel<float, RC>), dim3(g), dim3(256), 0, s, meta, in_t, x_t, out_t, R, \
                                mode, n);                                                                        \
    else hipLaunchKernelGGL((xchg_pack_kernel<double, RC>), dim3(g), dim3(256), 0, s, meta, in_t, x_t, out_t, R,  \
                            mode, n);
    BNPP_XCHG_R(BNPP_PACK)
#undef BNPP_PACK
    return hipGetLastError();
}

hipError_t launch_xchg_unpack(bool f32, TableMeta *meta, int in_t, int x_t, int out_t, int R, int64_t n,
                              hipStream_t s) {
    const unsigned g = grid_for(n / R / 4);
#define BNPP_UNPACK(RC)                                                                                          \
    if (f32) hipLaunchKernelGGL((xchg_unpack_kernel<float, RC>), dim3(g), dim3(256), 0, s, meta, in_t, x_t, out_t, R, \
                                n);                                                                              \
    else hipLaunchKernelGGL((xchg_unpack_kernel<double, RC>), dim3(g), dim3(256), 0, s, meta, in_t, x_t, out_t, R, n);
    BNPP_XCHG_R(BNPP_UNPACK)
#undef BNPP_UNPACK
    return hipGetLastError();
}

hipError_t launch_xchg_meta(TableMeta *meta, int in_t, int out_t, hipStream_t s) {
    hipLaunchKernelGGL(xchg_meta_kernel, dim3(1), dim3(64), 0, s, meta, in_t, out_t);
    return hipGetLastError();
}

}  // namespace bnpp

namespace bnpp {
hipError_t launch_delay(double ns, hipStream_t s) {
    static int khz = 0;
    if (khz <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
            khz <= 0)
            khz = 100000;                                  // 100 MHz, the gfx9 constant clock
    }
    const uint64_t ticks = (uint64_t)(ns * 1e-6 * khz);
    hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, ticks);
    return hipGetLastError();
}
}  // namespace bnpp
