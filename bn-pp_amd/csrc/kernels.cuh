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
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

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

// N contiguous elements through 16-byte (or narrower) vector accesses; NT
// marks the access nontemporal (streamed bytes that no later wave re-reads).
template <typename T, int W>
using vec_t = T __attribute__((ext_vector_type(W)));

// G: the pointer is into device memory (a table).  Table pointers come out of
// TableMeta as generic pointers, and accesses through them would compile to
// flat_* instructions, which also count against lgkmcnt (so every LDS wait
// would stall on the HBM loads in flight); the cast at the access makes them
// global_* instructions.
template <typename T>
using gbl_t = __attribute__((address_space(1))) T;

template <int W, bool NT, bool G = false, typename T>
__device__ __forceinline__ vec_t<T, W> vload(const T *p) {
    if constexpr (G) {
        const gbl_t<vec_t<T, W>> *q = (const gbl_t<vec_t<T, W>> *)p;
        if constexpr (NT) return __builtin_nontemporal_load(q);
        else return *q;
    } else {
        const vec_t<T, W> *q = reinterpret_cast<const vec_t<T, W> *>(p);
        if constexpr (NT) return __builtin_nontemporal_load(q);
        else return *q;
    }
}
template <int W, bool NT, bool G = false, typename T>
__device__ __forceinline__ void vstore(T *p, vec_t<T, W> v) {
    if constexpr (G) {
        gbl_t<vec_t<T, W>> *q = (gbl_t<vec_t<T, W>> *)p;
        if constexpr (NT) __builtin_nontemporal_store(v, q);
        else *q = v;
    } else {
        vec_t<T, W> *q = reinterpret_cast<vec_t<T, W> *>(p);
        if constexpr (NT) __builtin_nontemporal_store(v, q);
        else *q = v;
    }
}
// one element of a table in device memory
template <typename T>
__device__ __forceinline__ T gload(const T *p) { return *(const gbl_t<T> *)p; }

template <typename T, int N, bool NT = false, bool G = false>
__device__ __forceinline__ void load_n(const T *p, T *x) {
    constexpr int W = (sizeof(T) == 4 && N % 4 == 0) ? 4 : (N % 2 == 0 ? 2 : 1);
    if constexpr (W == 1) {
#pragma unroll
        for (int c = 0; c < N; ++c) {
            if constexpr (G) {
                const gbl_t<T> *q = (const gbl_t<T> *)(p + c);
                x[c] = NT ? __builtin_nontemporal_load(q) : *q;
            } else {
                x[c] = NT ? __builtin_nontemporal_load(p + c) : p[c];
            }
        }
    } else {
#pragma unroll
        for (int c = 0; c < N / W; ++c) {
            vec_t<T, W> v = vload<W, NT, G>(p + W * c);
#pragma unroll
            for (int e = 0; e < W; ++e) x[W * c + e] = v[e];
        }
    }
}
template <typename T, int N, bool NT = false, bool G = false>
__device__ __forceinline__ void store_n(T *p, const T *x) {
    constexpr int W = (sizeof(T) == 4 && N % 4 == 0) ? 4 : (N % 2 == 0 ? 2 : 1);
    if constexpr (W == 1) {
#pragma unroll
        for (int c = 0; c < N; ++c) {
            if constexpr (G) {
                gbl_t<T> *q = (gbl_t<T> *)(p + c);
                if constexpr (NT) __builtin_nontemporal_store(x[c], q);
                else *q = x[c];
            } else {
                if constexpr (NT) __builtin_nontemporal_store(x[c], p + c);
                else p[c] = x[c];
            }
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < N / W; ++c) {
        vec_t<T, W> v;
#pragma unroll
        for (int e = 0; e < W; ++e) v[e] = x[W * c + e];
        vstore<W, NT, G>(p + W * c, v);
    }
}

#ifndef BNPP_NT_LOAD
#define BNPP_NT_LOAD 0
#endif
#ifndef BNPP_NT_STORE
#define BNPP_NT_STORE 1      // measured: bench bucket -4 %, 32x32 PR -2 % (nt loads: chain +10 %, off)
#endif
constexpr bool kNtLoad = BNPP_NT_LOAD != 0;
constexpr bool kNtStore = BNPP_NT_STORE != 0;

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

// NMAX: the input slots a kernel reads (the generic kernels' NIN class): the
// per-input fields are uniform and belong in scalar registers, and sized for
// eight inputs they overflowed them into vector registers (a 4-input 7x1
// fp64 tile: 207 VGPRs)
template <int NMAX>
struct LoadedBucketT {
    int64_t base[NMAX];
    int64_t es[NMAX];
    int64_t s0[NMAX];        // stride on the fastest output dim
    int64_t s1[NMAX];        // stride on the second output dim
    const void *ptr[NMAX];
    void *out;
    const int64_t *dims;     // dims pool rows, fastest first
    int64_t n_tiles;
    int64_t card0, card1;
    int64_t t0h, t0m, t1h, t1m;
    int n_in, n_dims, k, v1, v2, flags, neg_e;
};
using LoadedBucket = LoadedBucketT<kMaxIn>;

// Element `off` of a table.  O32: a 32-bit offset added to the table's
// uniform base (global_load ... vOff, s[base] -- one address VGPR per load
// instead of two, and no 64-bit address arithmetic); used when every input
// of the launch is under 4 GiB.
template <bool O32>
using toff_t = typename std::conditional<O32, uint32_t, int64_t>::type;
template <bool O32, typename T>
__device__ __forceinline__ const T *tptr(const T *base, toff_t<O32> off) {
    if constexpr (O32) return (const T *)((const char *)base + (uint32_t)(off * (uint32_t)sizeof(T)));
    else return base + off;
}

// One input's V1 x V2 tile (strides s0 / s1 along output dims 0 / 1).  The
// values stay where their loads put them -- a broadcast input fills x[0] (or
// x[j2 * V1] per row, or one row x[0 .. V1)) -- and expand_tile spreads them
// once every input's loads are in flight.  Expanding here (x[j] = y) would
// make the copy wait for its load, and vmcnt counts in issue order: every
// input's loads would finish before the next input's were issued.
template <typename T, int V1, int V2, bool O32>
__device__ __forceinline__ void load_tile(const T *base, toff_t<O32> off, int64_t s0_, int64_t s1_,
                                          T (&x)[V1 * V2]) {
    const toff_t<O32> s0 = (toff_t<O32>)s0_, s1 = (toff_t<O32>)s1_;
    const bool row1 = V2 == 1 || s1 == 0;                 // the same along dim 1
    if (s0 == 0) {
        if (row1) {
            x[0] = gload(tptr<O32>(base, off));
        } else {
#pragma unroll
            for (int j2 = 0; j2 < V2; ++j2) x[j2 * V1] = gload(tptr<O32>(base, off + j2 * s1));
        }
    } else if (V1 > 1 && s0 == 1) {                       // contiguous along the fastest dim
        if (row1) {
            load_n<T, V1, false, true>(tptr<O32>(base, off), x);
        } else {
#pragma unroll
            for (int j2 = 0; j2 < V2; ++j2) load_n<T, V1, false, true>(tptr<O32>(base, off + j2 * s1), x + j2 * V1);
        }
    } else {                                              // general gather
#pragma unroll
        for (int j2 = 0; j2 < V2; ++j2)
#pragma unroll
            for (int j1 = 0; j1 < V1; ++j1)
                if (j2 == 0 || !row1) x[j2 * V1 + j1] = gload(tptr<O32>(base, off + j1 * s0 + j2 * s1));
    }
}

// spread what load_tile left compact over the whole tile
template <typename T, int V1, int V2>
__device__ __forceinline__ void expand_tile(T (&x)[V1 * V2], int64_t s0, int64_t s1) {
    const bool row1 = V2 == 1 || s1 == 0;
    if (s0 == 0 && row1) {
#pragma unroll
        for (int j = 1; j < V1 * V2; ++j) x[j] = x[0];
    } else if (s0 == 0) {
#pragma unroll
        for (int j2 = 0; j2 < V2; ++j2)
#pragma unroll
            for (int j1 = 1; j1 < V1; ++j1) x[j2 * V1 + j1] = x[j2 * V1];
    } else if (row1) {
#pragma unroll
        for (int j2 = 1; j2 < V2; ++j2)
#pragma unroll
            for (int j1 = 0; j1 < V1; ++j1) x[j2 * V1 + j1] = x[j1];
    }
}

// Evaluate one V1 x V2 output tile: decode its mixed-radix position once, then
// run the reference's product chain and sum in the reference's order.
template <typename T, int NIN, int V1, int V2, bool O32>
__device__ __forceinline__ T compute_tile(const LoadedBucketT<NIN> &b, int64_t tid, T (&acc)[V1 * V2]) {
    constexpr int TS = V1 * V2;
    using O = toff_t<O32>;
    O pos[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) pos[i] = (O)b.base[i];
    int64_t obase = 0;
    if (b.n_dims > 0) {
        uint64_t q, r;
        divmod_dim((uint64_t)tid, b.t0h, b.t0m, q, r);
        int64_t i0 = (int64_t)r * V1;
#pragma unroll
        for (int i = 0; i < NIN; ++i) pos[i] += (O)i0 * (O)b.s0[i];
        obase = i0;
        if (b.n_dims > 1) {
            uint64_t q1, r1;
            divmod_dim(q, b.t1h, b.t1m, q1, r1);
            int64_t i1 = (int64_t)r1 * V2;
#pragma unroll
            for (int i = 0; i < NIN; ++i) pos[i] += (O)i1 * (O)b.s1[i];
            obase = ((int64_t)q1 * b.card1 + i1) * b.card0 + i0;
            uint64_t rem = q1;
            const int row = 2 + b.n_in;                  // dims-pool row length
            // the pool is read-only while kernels run and its address is
            // uniform: read it through the scalar cache (constant address
            // space) instead of a vector load and a wait per dim
            const __attribute__((address_space(4))) int64_t *dp =
                (const __attribute__((address_space(4))) int64_t *)(b.dims + 2 * row);
            for (int j = 2; j < b.n_dims; ++j) {
                uint64_t qq, rr;
                divmod_dim(rem, dp[0], dp[1], qq, rr);
#pragma unroll
                for (int i = 0; i < NIN; ++i)
                    if (i < b.n_in) pos[i] += (O)rr * (O)dp[2 + i];
                rem = qq;
                dp += row;
            }
        }
    }

#pragma unroll
    for (int j = 0; j < TS; ++j) acc[j] = T(0);
    // Every input's loads for VB consecutive summed values are issued before
    // the first product uses one: loading and multiplying input by input
    // leaves one load in flight per thread, and a gather-heavy bucket (Munin1's
    // largest: 3 inputs x 7 values per output) then pays a memory round trip
    // per input and summed value in series.  Unused input slots (i >= n_in)
    // read entry 0 of the output table (their pointer, set with the others),
    // so the loads are issued without a branch per slot.  The arithmetic that follows is unchanged: p = 1;
    // p *= in_0; ...; acc += p per summed value in order (factor.cpp:131-143,
    // 199-205).
    constexpr int VB = TS * NIN >= 16 ? 1 : 16 / (TS * NIN);
    for (int v0 = 0; v0 < b.k; v0 += VB) {
        T x[VB][NIN][TS];
#pragma unroll
        for (int vv = 0; vv < VB; ++vv) {
            const O v = (O)(v0 + vv);
#pragma unroll
            for (int i = 0; i < NIN; ++i)
                if (VB == 1 || v0 + vv < b.k)              // uniform
                    load_tile<T, V1, V2, O32>(static_cast<const T *>(b.ptr[i]), pos[i] + v * (O)b.es[i], b.s0[i],
                                              b.s1[i], x[vv][i]);
        }
#pragma unroll
        for (int vv = 0; vv < VB; ++vv)
#pragma unroll
            for (int i = 0; i < NIN; ++i)
                if (v0 + vv < b.k && i < b.n_in) expand_tile<T, V1, V2>(x[vv][i], b.s0[i], b.s1[i]);
#pragma unroll
        for (int vv = 0; vv < VB; ++vv) {
            if (v0 + vv < b.k) {                           // uniform
                T p[TS];
#pragma unroll
                for (int j = 0; j < TS; ++j) p[j] = T(1);
#pragma unroll
                for (int i = 0; i < NIN; ++i) {
                    if (i >= b.n_in) continue;             // uniform
                    if (i == 1 && (b.flags & kDivide)) {  // (*this)[pos1] / f[pos2], factor.cpp:166
#pragma unroll
                        for (int j = 0; j < TS; ++j) p[j] = p[j] / x[vv][i][j];
                    } else {
#pragma unroll
                        for (int j = 0; j < TS; ++j) p[j] = p[j] * x[vv][i][j];
                    }
                }
#pragma unroll
                for (int j = 0; j < TS; ++j) acc[j] = acc[j] + p[j];
            }
        }
    }
    if (b.flags & kScale) {
#pragma unroll
        for (int j = 0; j < TS; ++j) acc[j] = ldexp_t(acc[j], b.neg_e);
    }
    (void)obase;                                          // == tid * TS (tiles are enumerated in output order)
    T m = T(0);
#pragma unroll
    for (int j = 0; j < TS; ++j) m = acc[j] > m ? acc[j] : m;
    return m;
}

// LDS image of one wave's output tiles: 64 rows of TS entries, padded by 16 B
constexpr int kLdsRowPad = 16;
constexpr int kLdsWaveBytes = 64 * (64 + kLdsRowPad);      // largest tile: 64 B per lane

// Store the wave's tiles (lane l holds tile `wave_tid0 + l`, which covers
// output entries [tid*TS, tid*TS + TS)).  Tiles of one 16-B access are stored
// directly (already coalesced); wider tiles go through the wave's LDS image so
// every global store instruction writes 64 consecutive 16-B chunks.
#ifndef BNPP_WAVE_SYNC
#define BNPP_WAVE_SYNC 0
#endif
#ifndef BNPP_DIRECT_STORE
#define BNPP_DIRECT_STORE 0
#endif
// the LDS image is private to one wave: ordering its writes and reads needs
// only the wave itself (LDS executes a wave's instructions in order), not the
// workgroup barrier
__device__ __forceinline__ void image_sync() {
    if constexpr (BNPP_WAVE_SYNC != 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

template <typename T, int TS>
__device__ __forceinline__ void store_tiles(T *out, int64_t wave_tid0, int64_t n_tiles, const T (&acc)[TS],
                                            unsigned char *lds) {
    const int lane = threadIdx.x & 63;
    const int64_t tid = wave_tid0 + lane;
    constexpr int row_bytes = TS * (int)sizeof(T);
    if constexpr (row_bytes <= 8 || row_bytes == 16 || BNPP_DIRECT_STORE != 0) {
        if (tid < n_tiles) store_n<T, TS, kNtStore, true>(out + tid * TS, acc);
    } else if constexpr (row_bytes % 16 != 0) {
        // rows that are no whole number of 16-B chunks (a whole fastest dim
        // of card 3, 5, 6 or 7 per thread): the wave's tiles are one run of
        // 64 * TS consecutive entries, staged unpadded and stored as 16-B
        // chunks (the run starts 16-B aligned: 64 * TS entries per wave)
        constexpr int EPC = 16 / (int)sizeof(T);
        constexpr int chunks = 64 * row_bytes / 16;
        image_sync();
        store_n<T, TS>(reinterpret_cast<T *>(lds + lane * row_bytes), acc);
        image_sync();
        const int64_t left = (n_tiles - wave_tid0) * TS;       // entries of this wave's tiles that exist
        const int64_t valid = left < 64 * TS ? left : 64 * TS;
        T *wout = out + wave_tid0 * TS;
#pragma unroll
        for (int it = 0; it < (chunks + 63) / 64; ++it) {
            const int q = it * 64 + lane;
            if (q < chunks) {
                const int64_t e0 = (int64_t)q * EPC;
                T x[EPC];
                load_n<T, EPC>(reinterpret_cast<const T *>(lds + q * 16), x);
                if (e0 + EPC <= valid) {
                    store_n<T, EPC, kNtStore, true>(wout + e0, x);
                } else {
#pragma unroll
                    for (int e = 0; e < EPC; ++e)
                        if (e0 + e < valid) store_n<T, 1, kNtStore, true>(wout + e0 + e, x + e);
                }
            }
        }
    } else {
        constexpr int rowp = row_bytes + kLdsRowPad;
        constexpr int cpr = row_bytes / 16;                   // 16-B chunks per row
        constexpr int EPC = 16 / (int)sizeof(T);              // entries per chunk
        image_sync();                                         // previous reads of this image are done
        store_n<T, TS>(reinterpret_cast<T *>(lds + lane * rowp), acc);
        image_sync();
        const int64_t valid = n_tiles - wave_tid0;            // tiles of this wave that exist
#pragma unroll
        for (int it = 0; it < cpr; ++it) {
            const int q = it * 64 + lane;                     // chunk index within the wave's region
            const int src_lane = q / cpr, within = q % cpr;
            if (src_lane < valid) {
                T x[EPC];
                load_n<T, EPC>(reinterpret_cast<const T *>(lds + src_lane * rowp + within * 16), x);
                store_n<T, EPC, kNtStore, true>(out + wave_tid0 * TS + (int64_t)q * EPC, x);
            }
        }
    }
}

// uniform read-only data (descriptors, the dims pool, table pointers) read
// through the scalar cache: the compiler cannot prove on its own that the
// kernel's stores leave them alone, and reads them with vector loads into
// vector registers
template <typename T>
using cst_t = const __attribute__((address_space(4))) T;
template <typename T>
__device__ __forceinline__ cst_t<T> *as_const(const T *p) { return (cst_t<T> *)p; }

// fill the per-bucket register state from a descriptor + table pointers
template <int NMAX, typename D>
__device__ __forceinline__ void load_common(LoadedBucketT<NMAX> &b, const D &d, const int64_t *dims_) {
    cst_t<int64_t> *dims = as_const(dims_);
    b.n_in = d.n_in; b.n_dims = d.n_dims; b.k = d.k; b.v1 = d.v1; b.v2 = d.v2;
    b.n_tiles = d.n_tiles;
    b.dims = dims_;
    b.t0h = d.tdiv0[0]; b.t0m = d.tdiv0[1]; b.t1h = d.tdiv1[0]; b.t1m = d.tdiv1[1];
    b.card0 = d.n_dims > 0 ? (int64_t)((uint64_t)dims[0] & 0xffffffffu) : 1;
    b.card1 = d.n_dims > 1 ? (int64_t)((uint64_t)dims[2 + d.n_in] & 0xffffffffu) : 1;
    for (int i = 0; i < NMAX; ++i) {
        bool on = i < d.n_in;
        b.base[i] = on ? d.in_base[i] : 0;
        b.es[i] = on ? d.elim_stride[i] : 0;
        b.s0[i] = on && d.n_dims > 0 ? dims[2 + i] : 0;
        b.s1[i] = on && d.n_dims > 1 ? dims[2 + d.n_in + 2 + i] : 0;
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
        // skip the atomic when the table's max already covers this block: with
        // one workgroup per block, hundreds of thousands of same-address
        // atomics would serialise (~12 ns each); a stale read only costs a
        // needless atomic
        using U = typename FBits<T>::U;
        U *mb = reinterpret_cast<U *>(&meta[out_table].maxbits);
        const U mine = FBits<T>::bits(m);
        if (m > T(0) && __hip_atomic_load(mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mine) atomicMax(mb, mine);
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

template <typename T, int NIN, int V1, int V2, bool O32>
__global__ __launch_bounds__(kBlock) void bucket_level_kernel(const BucketDesc *__restrict__ descs, int n_desc,
                                                              const int64_t *__restrict__ pool,
                                                              TableMeta *__restrict__ meta, int64_t total_vblocks) {
    __shared__ T red[kBlock / 64];
    __shared__ __attribute__((aligned(16))) unsigned char lds[(kBlock / 64) * kLdsWaveBytes];
    LoadedBucketT<NIN> b;
    int cur = -1;
    int64_t cur_begin = 0;
    T lmax = T(0);
    for (int64_t vb = blockIdx.x; vb < total_vblocks; vb += gridDim.x) {
        int bi = n_desc == 1 ? 0 : find_bucket(descs, n_desc, vb);
        if (bi != cur) {
            if (cur >= 0) flush_max<T>(lmax, meta, descs[cur].out_table, descs[cur].flags, red);
            cur = bi;
            lmax = T(0);
            cst_t<BucketDesc> &d = *as_const(descs + bi);
            cur_begin = d.vblk_begin;
            load_common(b, d, pool + d.dim_off);
            b.flags = d.flags;
            b.out = meta[d.out_table].ptr;
            int64_t e_sum = 0, x_sum = 0;
            for (int i = 0; i < NIN; ++i) {
                if (i < d.n_in) {
                    // the input tables' metadata is final (written by earlier
                    // launches); only the output's changes in this one
                    cst_t<TableMeta> &mi = *as_const(meta + d.in_table[i]);
                    b.ptr[i] = mi.ptr;
                    int e = FBits<T>::exponent(mi.maxbits);
                    if (d.flags & kScale) {
                        e_sum += e;
                        x_sum += mi.exp2 + e;
                    } else {
                        x_sum += mi.exp2;
                    }
                } else {
                    b.ptr[i] = b.out;                      // unused slot: compute_tile reads entry 0 (a
                                                           // valid address even for a bucket of no inputs)
                }
            }
            b.neg_e = (int)(-e_sum);
            // the first virtual block of the bucket publishes the output's scale exponent
            if (vb == cur_begin && threadIdx.x == 0) meta[d.out_table].exp2 = x_sum;
        }
        const int64_t tid0 = (vb - cur_begin) * kBlock;
        const int64_t tid = tid0 + threadIdx.x;
        T acc[V1 * V2];
        if (tid < b.n_tiles) {
            T m = compute_tile<T, NIN, V1, V2, O32>(b, tid, acc);
            lmax = m > lmax ? m : lmax;
        }
        store_tiles<T, V1 * V2>(static_cast<T *>(b.out), tid0 + (threadIdx.x & ~63), b.n_tiles, acc,
                                lds + (threadIdx.x >> 6) * kLdsWaveBytes);
    }
    if (cur >= 0) flush_max<T>(lmax, meta, descs[cur].out_table, descs[cur].flags, red);
}

// One bucket whose descriptor travels in the kernel-argument segment: used by
// the single-op API (Factor::product / sum_out / conditioning), no rescaling.
template <typename T, int NIN, int V1, int V2, bool O32>
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
    LoadedBucketT<NIN> b;
    load_common(b, d, a.pool);
    b.flags = d.flags & kDivide;
    b.neg_e = 0;
    b.out = a.meta[d.n_in].ptr;
    for (int i = 0; i < NIN; ++i) b.ptr[i] = i < d.n_in ? a.meta[i].ptr : b.out;   // unused: entry 0 of the output
    __shared__ __attribute__((aligned(16))) unsigned char lds[(kBlock / 64) * kLdsWaveBytes];
    for (int64_t tid0 = (int64_t)blockIdx.x * kBlock; tid0 < b.n_tiles; tid0 += (int64_t)gridDim.x * kBlock) {
        const int64_t tid = tid0 + threadIdx.x;
        T acc[V1 * V2];
        if (tid < b.n_tiles) (void)compute_tile<T, NIN, V1, V2, O32>(b, tid, acc);
        store_tiles<T, V1 * V2>(static_cast<T *>(b.out), tid0 + (threadIdx.x & ~63), b.n_tiles, acc,
                                lds + (threadIdx.x >> 6) * kLdsWaveBytes);
    }
}

// ------------------------------------------------------------ stream form
// One big input streamed from HBM (its loads for 4 consecutive values of the
// summed variable are issued before any is used; their class is a template
// parameter, so no register shuffling sits between issue and use) and every
// small input (factor tables, <= kStreamSmallMax entries) read from a copy in
// LDS made once per workgroup and bucket.  Product order is still the
// reference's chain order.
template <typename T, int V1, int V2, int BC>
struct BigTile {
    static constexpr int TS = V1 * V2;
    static constexpr int N = BC == kBigRow ? V1 : BC == kBigCol ? V2 : (BC == kBigOne || BC >= kBigInter2) ? 1 : TS;
    template <bool NTL>
    static __device__ __forceinline__ void issue(const T *src, int64_t s0, int64_t s1, T (&buf)[N]) {
        if constexpr (BC == kBigOne) {
            buf[0] = gload(src);
        } else if constexpr (BC == kBigRow) {
            load_n<T, V1, NTL, true>(src, buf);
        } else if constexpr (BC == kBigCol) {
            load_n<T, V2, NTL, true>(src, buf);
        } else if constexpr (BC == kBigFull) {
            load_n<T, TS, NTL, true>(src, buf);
        } else {
#pragma unroll
            for (int j2 = 0; j2 < V2; ++j2)
#pragma unroll
                for (int j1 = 0; j1 < V1; ++j1) buf[j2 * V1 + j1] = gload(src + (int64_t)j1 * s0 + (int64_t)j2 * s1);
        }
    }
    static __device__ __forceinline__ void apply(const T (&buf)[N], T (&p)[TS]) {
#pragma unroll
        for (int j = 0; j < TS; ++j) {
            if constexpr (BC == kBigOne) p[j] = p[j] * buf[0];
            else if constexpr (BC == kBigRow) p[j] = p[j] * buf[j % V1];
            else if constexpr (BC == kBigCol) p[j] = p[j] * buf[j / V1];
            else p[j] = p[j] * buf[j];
        }
    }
};

constexpr int kStreamMaxIn = 4;     // stream form: inputs of the default class (planner-enforced)
// a stream bucket of 5-8 inputs (one big, the rest small) launches its own
// instantiation, NI = 8 (stream_key(..., n_in)): the conditioned 32x32 PR's
// 5-input bucket over an 8-GiB message ran 46 ms on the generic 8-input kernel
// with 64-bit offsets

struct StreamState {
    int big;
    int32_t lds_off[kMaxIn];
    int32_t span[kMaxIn];
};

// NTL: nontemporal loads of the big input -- the single-op calls (cold, user
// tables: measured -2 % on the bench bucket); level kernels keep kNtLoad (a
// VE chain re-reads the message the previous bucket just wrote)
template <typename T, int V1, int V2, int BC, bool NTL, int NI = kStreamMaxIn>
__device__ __forceinline__ T compute_stream_tile(const LoadedBucket &b, const StreamState &st, const T *small,
                                                 int64_t tid, T (&acc)[V1 * V2], int64_t &out_off) {
    constexpr bool kRows = (BC == kBigInter2 || BC == kBigInter4) && V2 > 1;   // output rows at a stride
    constexpr int TS = V1 * V2;
    using BT = BigTile<T, V1, V2, BC>;
    int64_t pos[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) pos[i] = b.base[i];
    out_off = 0;
    if (b.n_dims > 0) {
        const int row = 2 + b.n_in;
        // dims pool through the scalar cache (read-only while the launch
        // runs): vector loads here would make each tile wait, in vmcnt
        // order, for the previous tile's stores
        cst_t<int64_t> *os = as_const(b.dims) + (int64_t)b.n_dims * row;   // kOutStrided: output stride per dim
        uint64_t q, r;
        divmod_dim((uint64_t)tid, b.t0h, b.t0m, q, r);
        int64_t i0 = (int64_t)r * V1;
#pragma unroll
        for (int i = 0; i < NI; ++i) pos[i] += i0 * b.s0[i];
        if constexpr (kRows) out_off = i0 * os[0];
        if (b.n_dims > 1) {
            uint64_t q1, r1;
            divmod_dim(q, b.t1h, b.t1m, q1, r1);
            int64_t i1 = (int64_t)r1 * V2;
#pragma unroll
            for (int i = 0; i < NI; ++i) pos[i] += i1 * b.s1[i];
            if constexpr (kRows) out_off += i1 * os[1];
            uint64_t rem = q1;
            cst_t<int64_t> *dp = as_const(b.dims) + 2 * row;
            for (int j = 2; j < b.n_dims; ++j) {
                uint64_t qq, rr;
                divmod_dim(rem, dp[0], dp[1], qq, rr);
#pragma unroll
                for (int i = 0; i < NI; ++i)
                    if (i < b.n_in) pos[i] += (int64_t)rr * dp[2 + i];
                if constexpr (kRows) out_off += (int64_t)rr * os[j];
                rem = qq;
                dp += row;
            }
        }
    }
    // LDS-relative positions of the small inputs; the big input's address and
    // strides picked with static indices (a runtime index would go to scratch)
    int32_t rel[NI];
    const T *bsrc = nullptr;
    int64_t bes = 0, bs0 = 0, bs1 = 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        rel[i] = st.lds_off[i] + (int32_t)(pos[i] - b.base[i]);
        if (i == st.big) {
            bsrc = static_cast<const T *>(b.ptr[i]) + pos[i];
            bes = b.es[i];
            bs0 = b.s0[i];
            bs1 = b.s1[i];
        }
    }

    // every small input (from LDS) into the product, in chain order around the
    // big one (interleaved path; the streamed path below keeps it inline)
    auto smalls = [&](int v, T (&p)[TS], auto &&big_apply) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (i >= b.n_in) break;                         // uniform
            if (i == st.big) {
                big_apply(p);
            } else {
                // small input from LDS, read once per distinct entry of the tile
                const T *t = small + rel[i] + v * (int32_t)b.es[i];
                const int32_t s0 = (int32_t)b.s0[i], s1 = (int32_t)b.s1[i];
                if (s0 == 0 && s1 == 0) {
                    const T y = t[0];
#pragma unroll
                    for (int j = 0; j < TS; ++j) p[j] = p[j] * y;
                } else if (s1 == 0) {
                    T y[V1];
#pragma unroll
                    for (int j1 = 0; j1 < V1; ++j1) y[j1] = t[j1 * s0];
#pragma unroll
                    for (int j = 0; j < TS; ++j) p[j] = p[j] * y[j % V1];
                } else if (s0 == 0) {
                    T y[V2];
#pragma unroll
                    for (int j2 = 0; j2 < V2; ++j2) y[j2] = t[j2 * s1];
#pragma unroll
                    for (int j = 0; j < TS; ++j) p[j] = p[j] * y[j / V1];
                } else {
#pragma unroll
                    for (int j2 = 0; j2 < V2; ++j2)
#pragma unroll
                        for (int j1 = 0; j1 < V1; ++j1) p[j2 * V1 + j1] = p[j2 * V1 + j1] * t[j1 * s0 + j2 * s1];
                }
            }
        }
    };
#pragma unroll
    for (int j = 0; j < TS; ++j) acc[j] = T(0);
    if constexpr (BC == kBigInter2 || BC == kBigInter4) {
        // the summed variable is the big input's fastest dim and the tile's
        // dim 0 follows it: the tile's big entries for every v are V1*K
        // contiguous values, fetched by one vector load (V2 == 1)
        constexpr int K = BC == kBigInter2 ? 2 : 4;
        T all[V1 * K];
        load_n<T, V1 * K, NTL, true>(bsrc, all);
#pragma unroll
        for (int v = 0; v < K; ++v) {
            T p[TS];
#pragma unroll
            for (int j = 0; j < TS; ++j) p[j] = T(1);
            smalls(v, p, [&](T (&q)[TS]) {                 // same big values for every row j / V1
#pragma unroll
                for (int j = 0; j < TS; ++j) q[j] = q[j] * all[(j % V1) * K + v];
            });
#pragma unroll
            for (int j = 0; j < TS; ++j) acc[j] = acc[j] + p[j];
        }
    } else {
#ifndef BNPP_STREAM_U
// measured: 16 -> forward 2x8 Col 4.78 -> 5.49 TB/s; 32 -> the 32x32 sweep's
// k = 2 2x8 full tiles (two 64-B loads in flight instead of one) 13.1 -> 9.7 ms
// per 2^32-entry output, MAR stream time 186 -> 172 ms per two calls
// (profiles/r04_stream_u_ab.txt; 64 spills back to 13.1 ms)
#define BNPP_STREAM_U 32
#endif
        // values of the summed variable whose big loads are issued together;
        // BNPP_STREAM_U > 0 caps the registers they take at that many entries
        constexpr int U = BNPP_STREAM_U == 0 ? 4
                          : (BNPP_STREAM_U / BT::N < 1 ? 1 : BNPP_STREAM_U / BT::N > 4 ? 4 : BNPP_STREAM_U / BT::N);
        for (int v0 = 0; v0 < b.k; v0 += U) {
            T bb[U][BT::N];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (v0 + u < b.k) BT::template issue<NTL>(bsrc + (int64_t)(v0 + u) * bes, bs0, bs1, bb[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int v = v0 + u;
                if (v >= b.k) break;                                // uniform
                T p[TS];
#pragma unroll
                for (int j = 0; j < TS; ++j) p[j] = T(1);
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    if (i >= b.n_in) break;                         // uniform
                    if (i == st.big) {
                        BT::apply(bb[u], p);
                    } else {
                        // small input from LDS, read once per distinct entry of the tile
                        const T *t = small + rel[i] + v * (int32_t)b.es[i];
                        const int32_t s0 = (int32_t)b.s0[i], s1 = (int32_t)b.s1[i];
                        if (s0 == 0 && s1 == 0) {
                            const T y = t[0];
#pragma unroll
                            for (int j = 0; j < TS; ++j) p[j] = p[j] * y;
                        } else if (s1 == 0) {
                            T y[V1];
#pragma unroll
                            for (int j1 = 0; j1 < V1; ++j1) y[j1] = t[j1 * s0];
#pragma unroll
                            for (int j = 0; j < TS; ++j) p[j] = p[j] * y[j % V1];
                        } else if (s0 == 0) {
                            T y[V2];
#pragma unroll
                            for (int j2 = 0; j2 < V2; ++j2) y[j2] = t[j2 * s1];
#pragma unroll
                            for (int j = 0; j < TS; ++j) p[j] = p[j] * y[j / V1];
                        } else {
#pragma unroll
                            for (int j2 = 0; j2 < V2; ++j2)
#pragma unroll
                                for (int j1 = 0; j1 < V1; ++j1)
                                    p[j2 * V1 + j1] = p[j2 * V1 + j1] * t[j1 * s0 + j2 * s1];
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < TS; ++j) acc[j] = acc[j] + p[j];
            }
        }
    }
    if (b.flags & kScale) {
#pragma unroll
        for (int j = 0; j < TS; ++j) acc[j] = ldexp_t(acc[j], b.neg_e);
    }
    T m = T(0);
#pragma unroll
    for (int j = 0; j < TS; ++j) m = acc[j] > m ? acc[j] : m;
    return m;
}

// store one stream tile: V2 rows of V1 entries at the output stride of dim 1
// (interleaved tiles over a broadcast dim), else the contiguous-tile path
template <typename T, int V1, int V2, int BC>
__device__ __forceinline__ void stream_store(const LoadedBucket &b, int64_t tid0, int64_t tid, int64_t out_off,
                                             const T (&acc)[V1 * V2], unsigned char *stage) {
    if constexpr ((BC == kBigInter2 || BC == kBigInter4) && V2 > 1) {
        if (tid < b.n_tiles) {
            const int64_t os1 = as_const(b.dims)[(int64_t)b.n_dims * (2 + b.n_in) + 1];
            T *o = static_cast<T *>(b.out) + out_off;
#pragma unroll
            for (int j2 = 0; j2 < V2; ++j2) store_n<T, V1, kNtStore, true>(o + j2 * os1, acc + j2 * V1);
        }
    } else {
        store_tiles<T, V1 * V2>(static_cast<T *>(b.out), tid0 + (threadIdx.x & ~63), b.n_tiles, acc,
                                stage + (threadIdx.x >> 6) * kLdsWaveBytes);
    }
}

// copy every small input of the bucket into LDS (uniform control flow)
template <typename T, int NI = kStreamMaxIn>
__device__ __forceinline__ void stage_small(const LoadedBucket &b, const StreamState &st, T *small) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NI; ++i) {                      // static indices: no scratch
        if (i >= b.n_in) break;
        if (i == st.big) continue;
        const T *src = static_cast<const T *>(b.ptr[i]) + b.base[i];
        for (int e = threadIdx.x; e < st.span[i]; e += kBlock) small[st.lds_off[i] + e] = gload(src + e);
    }
    __syncthreads();
}

__device__ __forceinline__ void load_stream_state(StreamState &st, const BucketDesc &d) {
    st.big = d.big;
    for (int i = 0; i < kMaxIn; ++i) {
        st.lds_off[i] = d.in_lds_off[i];
        st.span[i] = d.in_span[i];
    }
}

constexpr int kRedBytes = 64;       // block max reduction scratch at the head of dynamic LDS

#ifndef BNPP_STREAM_MINWAVES
#define BNPP_STREAM_MINWAVES 1
#endif
template <typename T, int V1, int V2, int BC, int NI>
__global__ __launch_bounds__(kBlock, BNPP_STREAM_MINWAVES) void stream_level_kernel(const BucketDesc *__restrict__ descs, int n_desc,
                                                              const int64_t *__restrict__ pool,
                                                              TableMeta *__restrict__ meta, int64_t total_vblocks) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    T *red = reinterpret_cast<T *>(dyn);
    unsigned char *stage = dyn + kRedBytes;
    T *small = reinterpret_cast<T *>(dyn + kRedBytes + (kBlock / 64) * kLdsWaveBytes);
    LoadedBucket b;
    StreamState st;
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
            load_common(b, d, pool + d.dim_off);
            load_stream_state(st, d);
            b.flags = d.flags;
            b.out = meta[d.out_table].ptr;
            int64_t e_sum = 0, x_sum = 0;
            for (int i = 0; i < kMaxIn; ++i) {
                if (i < d.n_in) {
                    const TableMeta &mi = meta[d.in_table[i]];
                    b.ptr[i] = mi.ptr;
                    int e = FBits<T>::exponent(mi.maxbits);
                    if (d.flags & kScale) {
                        e_sum += e;
                        x_sum += mi.exp2 + e;
                    } else {
                        x_sum += mi.exp2;
                    }
                } else {
                    b.ptr[i] = nullptr;
                }
            }
            b.neg_e = (int)(-e_sum);
            if (vb == cur_begin && threadIdx.x == 0) meta[d.out_table].exp2 = x_sum;
            stage_small<T, NI>(b, st, small);
        }
        const int64_t tid0 = (vb - cur_begin) * kBlock;
        const int64_t tid = tid0 + threadIdx.x;
        T acc[V1 * V2];
        int64_t oo = 0;
        if (tid < b.n_tiles) {
            T m = compute_stream_tile<T, V1, V2, BC, kNtLoad, NI>(b, st, small, tid, acc, oo);
            lmax = m > lmax ? m : lmax;
        }
        stream_store<T, V1, V2, BC>(b, tid0, tid, oo, acc, stage);
    }
    if (cur >= 0) flush_max<T>(lmax, meta, descs[cur].out_table, descs[cur].flags, red);
}

template <typename T, int V1, int V2, int BC, int NI>
__global__ __launch_bounds__(kBlock, BNPP_STREAM_MINWAVES) void stream_single_kernel(const SingleArgs args) {
#if defined(__HIP_DEVICE_COMPILE__)
    (void)args;
    const SingleArgs &a = *(const __attribute__((address_space(4))) SingleArgs *)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const SingleArgs &a = args;
#endif
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    unsigned char *stage = dyn + kRedBytes;
    T *small = reinterpret_cast<T *>(dyn + kRedBytes + (kBlock / 64) * kLdsWaveBytes);
    const BucketDesc &d = a.d;
    LoadedBucket b;
    StreamState st;
    load_common(b, d, a.pool);
    load_stream_state(st, d);
    b.flags = 0;
    b.neg_e = 0;
    b.out = a.meta[d.n_in].ptr;
    for (int i = 0; i < kMaxIn; ++i) b.ptr[i] = i < d.n_in ? a.meta[i].ptr : nullptr;
    stage_small<T, NI>(b, st, small);
    const int64_t gstride = (int64_t)gridDim.x * kBlock;
    int64_t tid0 = (int64_t)blockIdx.x * kBlock;
    for (; tid0 < b.n_tiles; tid0 += gstride) {
        const int64_t tid = tid0 + threadIdx.x;
        T acc[V1 * V2];
        int64_t oo = 0;
        if (tid < b.n_tiles) (void)compute_stream_tile<T, V1, V2, BC, true, NI>(b, st, small, tid, acc, oo);
        stream_store<T, V1, V2, BC>(b, tid0, tid, oo, acc, stage);
    }
}

// ---------------------------------------------------------------- launchers

template <typename T, int NIN, int V1, int V2, bool O32>
static hipError_t go_level(const LevelArgs &a, int max_grid, hipStream_t stream) {
    int64_t grid = a.vblocks < max_grid ? a.vblocks : max_grid;
    hipLaunchKernelGGL((bucket_level_kernel<T, NIN, V1, V2, O32>), dim3((unsigned)grid), dim3(kBlock), 0, stream, a.descs,
                       a.n_desc, a.pool, a.meta, a.vblocks);
    return hipGetLastError();
}

template <typename T, int NIN, int V1, int V2, bool O32>
static hipError_t go_single(const SingleArgs &a, int max_grid, hipStream_t stream) {
    int64_t blocks = (a.d.n_tiles + kBlock - 1) / kBlock;
    int64_t grid = blocks < max_grid ? blocks : max_grid;
    hipLaunchKernelGGL((bucket_single_kernel<T, NIN, V1, V2, O32>), dim3((unsigned)grid), dim3(kBlock), 0, stream, a);
    return hipGetLastError();
}

template <typename T, int V1, int V2, int BC, int NI = kStreamMaxIn>
static hipError_t go_stream_level(const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream) {
    int64_t grid = a.vblocks < max_grid ? a.vblocks : max_grid;
    size_t shm = kRedBytes + (kBlock / 64) * kLdsWaveBytes + (size_t)small_elems * sizeof(T);
    hipLaunchKernelGGL((stream_level_kernel<T, V1, V2, BC, NI>), dim3((unsigned)grid), dim3(kBlock), shm, stream, a.descs,
                       a.n_desc, a.pool, a.meta, a.vblocks);
    return hipGetLastError();
}

template <typename T, int V1, int V2, int BC, int NI = kStreamMaxIn>
static hipError_t go_stream_single(const SingleArgs &a, int max_grid, hipStream_t stream) {
    int64_t blocks = (a.d.n_tiles + kBlock - 1) / kBlock;
    int64_t grid = blocks < max_grid ? blocks : max_grid;
    size_t shm = kRedBytes + (kBlock / 64) * kLdsWaveBytes + (size_t)a.d.small_elems * sizeof(T);
    hipLaunchKernelGGL((stream_single_kernel<T, V1, V2, BC, NI>), dim3((unsigned)grid), dim3(kBlock), shm, stream, a);
    return hipGetLastError();
}

#define BNPP_STREAM_BC(X, T, V1, V2) X(T, V1, V2, 1) X(T, V1, V2, 2) X(T, V1, V2, 3) X(T, V1, V2, 4) X(T, V1, V2, 5)
#define BNPP_STREAM_INTER(X, T) X(T, 2, 1, 6) X(T, 4, 1, 6) X(T, 8, 1, 6) X(T, 2, 1, 7) X(T, 4, 1, 7) X(T, 8, 1, 7) \
    X(T, 4, 2, 6) X(T, 8, 2, 6) X(T, 4, 4, 6) X(T, 4, 2, 7) X(T, 8, 2, 7) X(T, 4, 4, 7) X(T, 2, 2, 6) X(T, 2, 2, 7) \
    X(T, 2, 4, 6) X(T, 2, 4, 7)
#define BNPP_STREAM_F32(X, T) BNPP_STREAM_INTER(X, T) BNPP_STREAM_BC(X, T, 1, 1) BNPP_STREAM_BC(X, T, 2, 1) BNPP_STREAM_BC(X, T, 4, 1) \
    BNPP_STREAM_BC(X, T, 2, 2) BNPP_STREAM_BC(X, T, 2, 4) BNPP_STREAM_BC(X, T, 4, 2) BNPP_STREAM_BC(X, T, 4, 4) \
    BNPP_STREAM_BC(X, T, 2, 8)
#define BNPP_STREAM_F64(X, T) BNPP_STREAM_INTER(X, T) BNPP_STREAM_BC(X, T, 1, 1) BNPP_STREAM_BC(X, T, 2, 1) BNPP_STREAM_BC(X, T, 4, 1) \
    BNPP_STREAM_BC(X, T, 2, 2) BNPP_STREAM_BC(X, T, 2, 4) BNPP_STREAM_BC(X, T, 4, 2)
#define BNPP_CASE_SLEVEL(T, V1, V2, BC) \
    case 4096 + BC * 256 + V1 * 16 + V2: return go_stream_level<T, V1, V2, BC>(a, small_elems, max_grid, stream);
#define BNPP_CASE_SSINGLE(T, V1, V2, BC) \
    case 4096 + BC * 256 + V1 * 16 + V2: return go_stream_single<T, V1, V2, BC>(a, max_grid, stream);
// 5-8 inputs (kStream8In): the direct big classes over the plain tiles, no interleaved forms
#define BNPP_STREAM8_BC(X, T, V1, V2) X(T, V1, V2, 1) X(T, V1, V2, 2) X(T, V1, V2, 3) X(T, V1, V2, 4) X(T, V1, V2, 5)
#define BNPP_STREAM8_F32(X, T) BNPP_STREAM8_BC(X, T, 1, 1) BNPP_STREAM8_BC(X, T, 2, 1) BNPP_STREAM8_BC(X, T, 4, 1) \
    BNPP_STREAM8_BC(X, T, 2, 2) BNPP_STREAM8_BC(X, T, 2, 4) BNPP_STREAM8_BC(X, T, 4, 2) BNPP_STREAM8_BC(X, T, 4, 4)
#define BNPP_STREAM8_F64(X, T) BNPP_STREAM8_BC(X, T, 1, 1) BNPP_STREAM8_BC(X, T, 2, 1) BNPP_STREAM8_BC(X, T, 4, 1) \
    BNPP_STREAM8_BC(X, T, 2, 2) BNPP_STREAM8_BC(X, T, 2, 4) BNPP_STREAM8_BC(X, T, 4, 2)
#define BNPP_CASE_SLEVEL8(T, V1, V2, BC) \
    case 4096 + kStream8In + BC * 256 + V1 * 16 + V2: return go_stream_level<T, V1, V2, BC, 8>(a, small_elems, max_grid, stream);
#define BNPP_CASE_SSINGLE8(T, V1, V2, BC) \
    case 4096 + kStream8In + BC * 256 + V1 * 16 + V2: return go_stream_single<T, V1, V2, BC, 8>(a, max_grid, stream);

// (3, 1) (5, 1) (6, 1) (7, 1): a whole fastest dim of that card per thread
#define BNPP_TILES_ODD(X, T, NIN) X(T, NIN, 3, 1) X(T, NIN, 5, 1) X(T, NIN, 6, 1) X(T, NIN, 7, 1)
// tiles along one output dim (k_generic_*.hip) and along two (k_generic2_*.hip,
// compiled without SimplifyCFG's store sinking: Makefile)
#define BNPP_TILES_1D(X, T, NIN) X(T, NIN, 1, 1) X(T, NIN, 2, 1) X(T, NIN, 4, 1) BNPP_TILES_ODD(X, T, NIN)
#define BNPP_TILES_F32_2D(X, T, NIN) X(T, NIN, 2, 2) X(T, NIN, 2, 4) X(T, NIN, 4, 2) X(T, NIN, 4, 4) X(T, NIN, 2, 8)
#define BNPP_TILES_F64_2D(X, T, NIN) X(T, NIN, 2, 2) X(T, NIN, 2, 4) X(T, NIN, 4, 2)
#define BNPP_ALL(X, TILES, T) TILES(X, T, 1) TILES(X, T, 2) TILES(X, T, 4) TILES(X, T, 8)

#define BNPP_CASE_LEVEL(T, NIN, V1, V2) \
    case NIN * 64 + V1 * 8 + V2: return go_level<T, NIN, V1, V2, false>(a, max_grid, stream); \
    case kGenericO32 + NIN * 64 + V1 * 8 + V2: return go_level<T, NIN, V1, V2, true>(a, max_grid, stream);
#define BNPP_CASE_SINGLE(T, NIN, V1, V2) \
    case NIN * 64 + V1 * 8 + V2: return go_single<T, NIN, V1, V2, false>(a, max_grid, stream); \
    case kGenericO32 + NIN * 64 + V1 * 8 + V2: return go_single<T, NIN, V1, V2, true>(a, max_grid, stream);


}  // namespace bnpp
