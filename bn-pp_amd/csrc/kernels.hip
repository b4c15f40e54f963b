// Fused bucket-elimination kernels for gfx950 (CDNA4).
//
// One launch executes a *level*: a set of independent buckets (model.cpp:409-439
// iterations whose inputs are ready).  Each bucket is cut into virtual blocks of
// kBlock vectors; workgroups walk the virtual blocks grid-stride, so tiny
// buckets cost one workgroup and a 2^33-entry bucket spreads over the whole chip.
//
// Per output vector (vec consecutive entries of the fastest output dim) a thread
//   - decodes its mixed-radix digits once (magic-number divmod; domain.cpp:162-190
//     restated as  pos_i = base_i + sum_d digit_d * stride_{i,d}),
//   - runs the reference's arithmetic in the reference's order:
//        acc = 0;  for v < k:  p = 1;  p *= in_0;  p *= in_1; ... ;  acc += p
//     (factor.cpp:131-143 chain, then factor.cpp:199-205 sum) — compiled with
//     -ffp-contract=off, so fp64 results are bit-identical to Factor::product +
//     Factor::sum_out for the same chain order,
//   - rescales by an exact power of two (the inputs' max exponents) so messages
//     never overflow; the exponent is carried in TableMeta::exp2,
//   - writes the output with a vec-wide store and folds its max into a
//     per-workgroup max that is published with one atomicMax per bucket.
// Inputs whose stride on the fastest output dim is 1 are read with vec-wide
// loads, stride-0 inputs are broadcast, anything else is gathered.
#include <hip/hip_runtime.h>

#include "bnpp_device.h"
#include "runtime.hpp"

namespace bnpp {

template <typename T> struct FBits;
template <> struct FBits<float> {
    using U = unsigned int;
    static __device__ __forceinline__ U bits(float x) { return __float_as_uint(x); }
    static __device__ __forceinline__ int exponent(uint64_t b) {   // max = m * 2^e, m in [0.5, 1)
        unsigned e = (unsigned)(b >> 23) & 0xffu;
        return b == 0 ? 0 : (int)e - 126;
    }
};
template <> struct FBits<double> {
    using U = unsigned long long;
    static __device__ __forceinline__ U bits(double x) { return (U)__double_as_longlong(x); }
    static __device__ __forceinline__ int exponent(uint64_t b) {
        unsigned e = (unsigned)(b >> 52) & 0x7ffu;
        return b == 0 ? 0 : (int)e - 1022;
    }
};

template <typename T, int N> struct VecT;
template <> struct VecT<float, 1> { using type = float; };
template <> struct VecT<float, 2> { using type = float2; };
template <> struct VecT<float, 4> { using type = float4; };
template <> struct VecT<double, 1> { using type = double; };
template <> struct VecT<double, 2> { using type = double2; };

template <typename T, int VEC>
__device__ __forceinline__ void load_vec(const T *p, T (&x)[VEC]) {
    if constexpr (VEC == 1) {
        x[0] = p[0];
    } else {
        using V = typename VecT<T, VEC>::type;
        V v = *reinterpret_cast<const V *>(p);
        if constexpr (VEC == 2) { x[0] = v.x; x[1] = v.y; }
        if constexpr (VEC == 4) { x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w; }
    }
}
template <typename T, int VEC>
__device__ __forceinline__ void store_vec(T *p, const T (&x)[VEC]) {
    if constexpr (VEC == 1) {
        p[0] = x[0];
    } else {
        using V = typename VecT<T, VEC>::type;
        V v;
        if constexpr (VEC == 2) { v.x = x[0]; v.y = x[1]; }
        if constexpr (VEC == 4) { v.x = x[0]; v.y = x[1]; v.z = x[2]; v.w = x[3]; }
        *reinterpret_cast<V *>(p) = v;
    }
}

__device__ __forceinline__ double ldexp_t(double x, int e) { return __builtin_amdgcn_ldexp(x, e); }
__device__ __forceinline__ float ldexp_t(float x, int e) { return __builtin_amdgcn_ldexpf(x, e); }

// n / d and n % d for one output dim (Granlund–Montgomery magic for 32-bit n).
__device__ __forceinline__ void divmod_dim(uint64_t n, int64_t w0, int64_t w1, uint64_t &q, uint64_t &r) {
    uint32_t card = (uint32_t)((uint64_t)w0 & 0xffffffffu);
    uint32_t shift = (uint32_t)(((uint64_t)w0 >> 32) & 0xffu);
    bool pow2 = ((uint64_t)w0 >> 40) & 1u;
    if (pow2) {
        q = n >> shift;
        r = n & (uint64_t)(card - 1u);
    } else if ((n >> 32) == 0) {
        uint32_t n32 = (uint32_t)n;
        uint32_t t = __umulhi((uint32_t)w1, n32);
        uint32_t q32 = (t + ((n32 - t) >> 1)) >> (shift - 1u);
        q = q32;
        r = n32 - q32 * card;
    } else {
        q = n / card;
        r = n - q * card;
    }
}

struct LoadedBucket {
    int64_t base[kMaxIn];
    int64_t es[kMaxIn];
    int64_t sf[kMaxIn];      // stride on the fastest output dim
    const void *ptr[kMaxIn];
    void *out;
    const int64_t *dims;
    int64_t n_vec;
    int n_in, n_dims, k, vec, flags, neg_e;
};

template <typename T, int NIN, int VEC>
__device__ __forceinline__ T eval_vec(const LoadedBucket &b, int64_t vid) {
    int64_t pos[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) pos[i] = b.base[i];
    uint64_t rem = (uint64_t)vid * VEC;
    const int64_t *dp = b.dims;
    for (int j = 0; j < b.n_dims; ++j) {
        uint64_t q, r;
        divmod_dim(rem, dp[0], dp[1], q, r);
#pragma unroll
        for (int i = 0; i < NIN; ++i) pos[i] += (int64_t)r * dp[2 + i];
        rem = q;
        dp += 2 + NIN;
    }

    T acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = T(0);
    for (int v = 0; v < b.k; ++v) {
        T p[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) p[j] = T(1);
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
            const T *src = static_cast<const T *>(b.ptr[i]) + pos[i] + (int64_t)v * b.es[i];
            if (b.sf[i] == 0) {
                T x = src[0];
#pragma unroll
                for (int j = 0; j < VEC; ++j) p[j] = p[j] * x;
            } else if (VEC > 1 && b.sf[i] == 1) {
                T x[VEC];
                load_vec<T, VEC>(src, x);
#pragma unroll
                for (int j = 0; j < VEC; ++j) p[j] = p[j] * x[j];
            } else {
#pragma unroll
                for (int j = 0; j < VEC; ++j) p[j] = p[j] * src[(int64_t)j * b.sf[i]];
            }
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] = acc[j] + p[j];
    }
    T m = T(0);
    if (b.flags & kScale) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] = ldexp_t(acc[j], b.neg_e);
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) m = acc[j] > m ? acc[j] : m;
    store_vec<T, VEC>(static_cast<T *>(b.out) + vid * VEC, acc);
    return m;
}

template <typename T, int NIN>
__device__ __forceinline__ T eval_nin(const LoadedBucket &b, int64_t vid) {
    if (b.vec == 1) return eval_vec<T, NIN, 1>(b, vid);
    if constexpr (sizeof(T) == 4) {
        if (b.vec == 4) return eval_vec<T, NIN, 4>(b, vid);
    }
    return eval_vec<T, NIN, 2>(b, vid);
}

template <typename T>
__device__ __forceinline__ T eval_any(const LoadedBucket &b, int64_t vid) {
    switch (b.n_in) {
        case 1: return eval_nin<T, 1>(b, vid);
        case 2: return eval_nin<T, 2>(b, vid);
        case 3: return eval_nin<T, 3>(b, vid);
        case 4: return eval_nin<T, 4>(b, vid);
        case 5: return eval_nin<T, 5>(b, vid);
        case 6: return eval_nin<T, 6>(b, vid);
        case 7: return eval_nin<T, 7>(b, vid);
        default: return eval_nin<T, 8>(b, vid);
    }
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

// Publish the workgroup's max of bucket `bi` (uniform control flow).
template <typename T>
__device__ __forceinline__ void flush_max(T lmax, TableMeta *meta, int out_table, int flags, T *red) {
    T w = wave_max(lmax);
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = w;
    __syncthreads();
    if (threadIdx.x == 0 && (flags & kTrackMax)) {
        T m = red[0];
        for (int i = 1; i < kBlock / 64; ++i) m = red[i] > m ? red[i] : m;
        if (m > T(0)) atomicMax(reinterpret_cast<typename FBits<T>::U *>(&meta[out_table].maxbits), FBits<T>::bits(m));
    }
    __syncthreads();
}

__device__ __forceinline__ int find_bucket(const BucketDesc *descs, int n_desc, int64_t vb) {
    int lo = 0, hi = n_desc - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (descs[mid].vblk_begin <= vb) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void bucket_level_kernel(const BucketDesc *__restrict__ descs, int n_desc,
                                                              const int64_t *__restrict__ pool,
                                                              TableMeta *__restrict__ meta, int64_t total_vblocks) {
    __shared__ T red[kBlock / 64];
    LoadedBucket b;
    int cur = -1;
    int64_t cur_begin = 0;
    T lmax = T(0);
    for (int64_t vb = blockIdx.x; vb < total_vblocks; vb += gridDim.x) {
        int bi = n_desc == 1 ? 0 : find_bucket(descs, n_desc, vb);
        if (bi != cur) {
            if (cur >= 0) flush_max<T>(lmax, meta, descs[cur].out_table, descs[cur].flags, red);
            cur = bi;
            lmax = T(0);
            const BucketDesc &d = descs[bi];
            cur_begin = d.vblk_begin;
            b.n_in = d.n_in; b.n_dims = d.n_dims; b.k = d.k; b.vec = d.vec; b.flags = d.flags;
            b.n_vec = d.n_vec;
            b.dims = pool + d.dim_off;
            b.out = meta[d.out_table].ptr;
            int64_t e_sum = 0, x_sum = 0;
            for (int i = 0; i < kMaxIn; ++i) {
                if (i < d.n_in) {
                    const TableMeta &mi = meta[d.in_table[i]];
                    b.ptr[i] = mi.ptr;
                    b.base[i] = d.in_base[i];
                    b.es[i] = d.elim_stride[i];
                    b.sf[i] = d.n_dims > 0 ? b.dims[2 + i] : 0;
                    int e = FBits<T>::exponent(mi.maxbits);
                    e_sum += e;
                    x_sum += mi.exp2 + e;
                } else {
                    b.ptr[i] = nullptr; b.base[i] = 0; b.es[i] = 0; b.sf[i] = 0;
                }
            }
            if (!(d.flags & kScale)) { e_sum = 0; x_sum = 0; for (int i = 0; i < d.n_in; ++i) x_sum += meta[d.in_table[i]].exp2; }
            b.neg_e = (int)(-e_sum);
            // the first virtual block of the bucket publishes the output's scale exponent
            if (vb == cur_begin && threadIdx.x == 0) meta[d.out_table].exp2 = x_sum;
        }
        int64_t vid = (vb - cur_begin) * kBlock + threadIdx.x;
        if (vid < b.n_vec) {
            T m = eval_any<T>(b, vid);
            lmax = m > lmax ? m : lmax;
        }
    }
    if (cur >= 0) flush_max<T>(lmax, meta, descs[cur].out_table, descs[cur].flags, red);
}

// One bucket whose descriptor travels in the kernel-argument segment: used by
// the single-op API (Factor::product / sum_out / conditioning), no rescaling.
template <typename T>
__global__ __launch_bounds__(kBlock) void bucket_single_kernel(const SingleArgs args) {
    // read the argument block in place (constant address space, scalar loads)
    // instead of letting the compiler copy it to scratch
#if defined(__HIP_DEVICE_COMPILE__)
    (void)args;
    const SingleArgs &a = *(const __attribute__((address_space(4))) SingleArgs *)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const SingleArgs &a = args;
#endif
    const BucketDesc &d = a.d;
    LoadedBucket b;
    b.n_in = d.n_in; b.n_dims = d.n_dims; b.k = d.k; b.vec = d.vec; b.flags = 0; b.neg_e = 0;
    b.n_vec = d.n_vec;
    b.dims = a.pool;
    b.out = a.meta[d.n_in].ptr;
    for (int i = 0; i < kMaxIn; ++i) {
        bool on = i < d.n_in;
        b.ptr[i] = on ? a.meta[i].ptr : nullptr;
        b.base[i] = on ? d.in_base[i] : 0;
        b.es[i] = on ? d.elim_stride[i] : 0;
        b.sf[i] = on && d.n_dims > 0 ? a.pool[2 + i] : 0;
    }
    for (int64_t vid = (int64_t)blockIdx.x * kBlock + threadIdx.x; vid < b.n_vec; vid += (int64_t)gridDim.x * kBlock)
        (void)eval_any<T>(b, vid);
}

// ---------------------------------------------------------------- launchers
template <typename T>
static hipError_t launch_level_t(const BucketDesc *descs, int n_desc, const int64_t *pool, TableMeta *meta,
                                 int64_t total_vblocks, int max_grid, hipStream_t stream) {
    if (n_desc <= 0 || total_vblocks <= 0) return hipSuccess;
    int64_t grid = total_vblocks < max_grid ? total_vblocks : max_grid;
    hipLaunchKernelGGL(bucket_level_kernel<T>, dim3((unsigned)grid), dim3(kBlock), 0, stream, descs, n_desc, pool,
                       meta, total_vblocks);
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_single_t(const SingleArgs &a, int max_grid, hipStream_t stream) {
    int64_t blocks = (a.d.n_vec + kBlock - 1) / kBlock;
    if (blocks <= 0) return hipSuccess;
    int64_t grid = blocks < max_grid ? blocks : max_grid;
    hipLaunchKernelGGL(bucket_single_kernel<T>, dim3((unsigned)grid), dim3(kBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_single(int is_f32, const SingleArgs &a, int max_grid, hipStream_t stream) {
    return is_f32 ? launch_single_t<float>(a, max_grid, stream) : launch_single_t<double>(a, max_grid, stream);
}

hipError_t launch_level(int is_f32, const BucketDesc *descs, int n_desc, const int64_t *pool, TableMeta *meta,
                        int64_t total_vblocks, int max_grid, hipStream_t stream) {
    return is_f32 ? launch_level_t<float>(descs, n_desc, pool, meta, total_vblocks, max_grid, stream)
                  : launch_level_t<double>(descs, n_desc, pool, meta, total_vblocks, max_grid, stream);
}

}  // namespace bnpp
