// Chain (sweep) kernels: F consecutive buckets of an elimination chain fused
// into one pass over the message (bnpp_device.h, ChainForm).
//
// In a sweep (the column-sweep order on a grid, the forward and backward
// passes of the bucket tree) bucket q's only large input is bucket q-1's
// message, and it swaps one variable of the message for one new variable:
//     msg_q(rest, n_q) = sum_{x_q} G_q(x_q, n_q, ...) * msg_{q-1}(x_q, rest)
// (model.cpp:414-418 with G_q = Factor(1.0) *= the bucket's factor tables).
// Run one bucket per launch and every message crosses HBM twice (written,
// read back).  Here one thread owns K^F entries of the run's input (the
// assignments of its F summed variables for one entry of the rest), runs the
// F buckets on them in registers -- each in the reference's arithmetic order,
// p = G_q * msg, acc = 0; acc += p for x_q = 0..K-1 (factor.cpp:131-143,
// 199-205) -- and writes the run's output once: HBM traffic per bucket / F.
// The intermediate messages are exactly the unfused ones up to a power-of-two
// scale (folded into the G tables, chain_fold), so fp64 stays bit-identical.
#pragma once
#include <type_traits>
#include <utility>

#include "kernels.cuh"

namespace bnpp {

__host__ __device__ constexpr int ipow(int k, int f) { return f == 0 ? 1 : k * ipow(k, f - 1); }

// compile-time loop: f(std::integral_constant<int, I>) for I in [0, N) -- the
// register table must only ever be indexed by constants (else it goes to scratch)
template <int I, int N, typename Fn>
__device__ __forceinline__ void static_for_impl(Fn &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for_impl<I + 1, N>(f);
    }
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn &&f) { static_for_impl<0, N>(f); }

template <int K, int F>
struct ChainShape {
    static constexpr int N = ipow(K, F);
    // digit of slot p in register index a (slot 0 most significant)
    static __device__ __forceinline__ constexpr int digit(int a, int p) { return (a / ipow(K, F - 1 - p)) % K; }
    static __device__ __forceinline__ constexpr int place(int p) { return ipow(K, F - 1 - p); }
    // memory position of register index a in a block whose slot 0 is fastest
    static __device__ __forceinline__ constexpr int rev(int a) {
        int r = 0;
        for (int p = 0; p < F; ++p) r += digit(a, p) * ipow(K, p);
        return r;
    }
};

__device__ __forceinline__ int64_t readfirstlane64(int64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x & 0xffffffffu));
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <int F>
struct ChainState {
    const void *big;
    void *out;
    const int64_t *dims;
    int64_t n_tiles, in_base;
    int64_t t0h, t0m;
    int64_t is[F], os[F];
    int32_t gs[F][F], gsn[F], glds[F];
    int n_dims, gmask, flags, neg_e;
};

template <typename T, int K, int F, int FORM>
__device__ __forceinline__ void chain_load_state(ChainState<F> &c, const BucketDesc &d, const int64_t *pool,
                                                 TableMeta *meta) {
    c.dims = pool;
    c.n_dims = d.n_dims;
    c.n_tiles = d.n_tiles;
    c.t0h = d.tdiv0[0];
    c.t0m = d.tdiv0[1];
    c.gmask = (d.chain >> 8) & 0xff;
    c.flags = d.flags;
    c.in_base = d.in_base[0];
    const int row = 4 + F;
    const int64_t *sl = pool + (int64_t)d.n_dims * row;
#pragma unroll
    for (int p = 0; p < F; ++p) {
        c.is[p] = sl[2 * p];
        c.os[p] = sl[2 * p + 1];
    }
    const int64_t *st = sl + 2 * F;
    int gi = 1;
#pragma unroll
    for (int j = 0; j < F; ++j) {
#pragma unroll
        for (int p = 0; p < F; ++p) c.gs[j][p] = (int32_t)st[j * (F + 1) + p];
        c.gsn[j] = (int32_t)st[j * (F + 1) + F];
        const bool on = (c.gmask >> j) & 1;
        c.glds[j] = on ? d.in_lds_off[gi] : 0;
        gi += on ? 1 : 0;
    }
    c.big = meta[d.in_table[0]].ptr;
    c.out = meta[d.out_table].ptr;
    c.neg_e = 0;                                           // chain_stage: the share not folded into G
}

template <typename T>
__device__ __forceinline__ int64_t chain_exp2(const BucketDesc &d, TableMeta *meta) {
    int64_t x_sum = 0;
    for (int i = 0; i < kMaxDescIn; ++i) {
        if (i >= d.n_in) break;
        const TableMeta &mi = meta[d.in_table[i]];
        x_sum += mi.exp2 + ((d.flags & kScale) ? FBits<T>::exponent(mi.maxbits) : 0);
    }
    return x_sum;
}

// A run's power-of-two rescale, folded into its G tables as they are staged
// in LDS.  Input i >= 1 (a G table) is staged as G * 2^s[i] with s[i] = -(its
// max exponent); the first one also takes -(the incoming message's, input 0).
// Every bucket's output then differs from the unfused bucket's (rescaled by
// its inputs' max exponents, kernels.cuh) by one power of two common to all
// its entries, so intermediate values stay where one bucket per launch keeps
// them (normal floats, however peaked the potentials) and the results are
// bit-identical to it: a power-of-two scale commutes with IEEE rounding.  A
// share beyond +-cap (maxima far outside the normal range) carries into the
// next table; the return value is what is left after the last one, for the
// output (applied by the one-thread runs, kept in exp2 by the split runs).
template <typename T>
__device__ __forceinline__ int chain_fold(const BucketDesc &d, const TableMeta *meta, int (&s)[kMaxDescIn]) {
    constexpr int cap = sizeof(T) == 4 ? 120 : 1000;
    int carry = 0;
#pragma unroll
    for (int i = 0; i < kMaxDescIn; ++i) {
        s[i] = 0;
        if (i >= d.n_in || !(d.flags & kScale)) continue;
        carry -= FBits<T>::exponent(meta[d.in_table[i]].maxbits);
        if (i == 0) continue;
        s[i] = carry > cap ? cap : carry < -cap ? -cap : carry;
        carry -= s[i];
    }
    return carry;
}

// copy the G tables of the run into LDS, scaled by chain_fold's shares
// (uniform control flow); returns the share left for the output
template <typename T>
__device__ __forceinline__ int chain_stage(const BucketDesc &d, TableMeta *meta, T *small) {
    int s[kMaxDescIn];
    const int left = chain_fold<T>(d, meta, s);
    __syncthreads();
#pragma unroll
    for (int i = 1; i < kMaxDescIn; ++i) {
        if (i < d.n_in) {                                  // uniform (a guard, not a break: the loop unrolls)
            const T *src = static_cast<const T *>(meta[d.in_table[i]].ptr) + d.in_base[i];
            const int off = d.in_lds_off[i], span = d.in_span[i];
            const T sc = ldexp_t(T(1), s[i]);
            for (int e = threadIdx.x; e < span; e += kBlock) small[off + e] = gload(src + e) * sc;
        }
    }
    __syncthreads();
    return left;
}

// Bucket J of a run on the register table t (MODE 0: no factor tables,
// 1: G_J, the same for the thread's V rest entries).  Every G value the bucket
// needs is fetched from LDS before any is used (one wait); then each output
// entry is  acc = 0; acc += G * m  over x_J = 0..K-1.  DEP (ChainDep) says
// which other slot G_J may vary with, so only K^3 values are fetched (any:
// one per (other slots, x, n)).
// SUM: the bucket only sums x_J out (no new variable): slots < J were summed
// before and hold digit 0; only digit 0 of slot J is written.
template <typename T, int K, int F, int V, int J, int MODE, int DEP, bool SUM = false>
__device__ __forceinline__ void chain_step(T (&t)[ipow(K, F)][V], const T *small, int32_t gb,
                                           const int32_t (&gs)[F], int32_t gsn) {
    using S = ChainShape<K, F>;
    constexpr int N = S::N;
    constexpr int PJ = S::place(J);
    constexpr int NA = N / K;                       // assignments of the other slots
    constexpr int NK = SUM ? 1 : K;                 // values of the new variable
    constexpr int Q = DEP == kDepNext ? J + 1 : DEP == kDepPrev ? J - 1 : -1;   // neighbour slot
    constexpr bool HASQ = Q >= 0 && Q < F;
    constexpr int NG = MODE == 0 ? 1 : DEP == kDepAny ? NA : (HASQ ? K : 1);
    T g[NG][NK][K];
    if constexpr (MODE != 0) {
        static_for<NG>([&](auto ic) {
            constexpr int gi = decltype(ic)::value;
            int32_t go = gb;
            if constexpr (DEP == kDepAny) {
                constexpr int a = (gi / PJ) * PJ * K + gi % PJ;          // slot J digit 0
#pragma unroll
                for (int p = 0; p < F; ++p)
                    if (p != J) go += S::digit(a, p) * gs[p];
            } else if constexpr (HASQ) {
                go += gi * gs[Q];
            }
#pragma unroll
            for (int n = 0; n < NK; ++n)
#pragma unroll
                for (int x = 0; x < K; ++x) g[gi][n][x] = small[go + x * gs[J] + n * gsn];
        });
    }
    static_for<NA>([&](auto ic) {
        constexpr int ai = decltype(ic)::value;
        constexpr int a = (ai / PJ) * PJ * K + ai % PJ;
        if constexpr (SUM && (a / (PJ * K)) != 0) return;    // a slot summed earlier is not 0: dead entry
        constexpr int gi = MODE == 0 ? 0 : DEP == kDepAny ? ai : (HASQ ? S::digit(a, HASQ ? Q : 0) : 0);
        T nw[NK][V];
#pragma unroll
        for (int n = 0; n < NK; ++n) {
#pragma unroll
            for (int v = 0; v < V; ++v) nw[n][v] = T(0);
#pragma unroll
            for (int x = 0; x < K; ++x) {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const T m = t[a + x * PJ][v];
                    T p = m;
                    if constexpr (MODE == 1) p = g[gi][n][x] * m;
                    nw[n][v] = nw[n][v] + p;
                }
            }
        }
#pragma unroll
        for (int n = 0; n < NK; ++n)
#pragma unroll
            for (int v = 0; v < V; ++v) t[a + n * PJ][v] = nw[n][v];
    });
}

__host__ __device__ constexpr bool chain_fwd(int form) { return form == kChainFwd || form == kChainFwdV; }
// rest entries per thread
template <typename T, int K, int F, int FORM>
constexpr int chain_v() {
    return FORM == kChainFwd ? 1
           : FORM == kChainFwdV ? chain_fwd_v(ipow(K, F), (int)sizeof(T))
           : FORM == kChainSum ? 16 / (int)sizeof(T) : chain_bwd_v(ipow(K, F), (int)sizeof(T));
}
// bytes of one forward output row, and of the part of it staged at a time
template <typename T, int K, int F, int FORM>
constexpr int chain_row_bytes() { return chain_v<T, K, F, FORM>() * ipow(K, F) * (int)sizeof(T); }
template <typename T, int K, int F, int FORM>
constexpr int chain_part_bytes() { return chain_row_bytes<T, K, F, FORM>() < 128 ? chain_row_bytes<T, K, F, FORM>() : 128; }
// per-wave LDS image of the forward forms: 64 row parts (+16 B pad)
template <typename T, int K, int F, int FORM>
constexpr int chain_img_wave() { return 64 * (chain_part_bytes<T, K, F, FORM>() + kLdsRowPad); }

// Store one wave's rows of TS entries (row tid at out + tid * TS) through the
// wave's LDS image, TH entries (<= 128 B) of every row at a time: each store
// instruction then writes whole 128-B segments.  TS == TH is store_tiles.
template <typename T, int TS, int TH>
__device__ __forceinline__ void store_rows_parts(T *out, int64_t wave_tid0, int64_t n_tiles, const T (&row)[TS],
                                                 unsigned char *lds) {
    if constexpr (TS == TH) {
        store_tiles<T, TS>(out, wave_tid0, n_tiles, row, lds);
    } else {
        static_assert(TS % TH == 0 && TH * (int)sizeof(T) % 16 == 0, "row parts of whole 16-B chunks");
        const int lane = threadIdx.x & 63;
        constexpr int rowp = TH * (int)sizeof(T) + kLdsRowPad;
        constexpr int cpr = TH * (int)sizeof(T) / 16;
        constexpr int EPC = 16 / (int)sizeof(T);
        const int64_t valid = n_tiles - wave_tid0;
        static_for<TS / TH>([&](auto pc) {
            constexpr int p = decltype(pc)::value;
            T part[TH];
#pragma unroll
            for (int i = 0; i < TH; ++i) part[i] = row[p * TH + i];
            image_sync();
            store_n<T, TH>(reinterpret_cast<T *>(lds + lane * rowp), part);
            image_sync();
#pragma unroll
            for (int it = 0; it < cpr; ++it) {
                const int q = it * 64 + lane;
                const int src_lane = q / cpr, within = q % cpr;
                if (src_lane < valid) {
                    T x[EPC];
                    load_n<T, EPC>(reinterpret_cast<const T *>(lds + src_lane * rowp + within * 16), x);
                    store_n<T, EPC, kNtStore, true>(out + (wave_tid0 + src_lane) * TS + p * TH + within * EPC, x);
                }
            }
        });
    }
}

// waves per SIMD the register allocation must leave room for (0: compiler's
// choice).  Measured on the 32x32 sweep: the forward 32-entry run at 3 waves
// 7.26 -> 6.57 ms per 2^32 message (4 waves spills); the same bound on the
// 64-entry runs takes the 32x32 PR 1.23 -> 1.19 s and MAR 3.95 -> 3.81 s (2
// waves: 3.92 s, 4 waves spills: 5.03 s); the backward runs are best left to
// the compiler (bounds of 2 or 3 waves: same or slower, tools/ab_mar.sh).
template <typename T, int K, int F, int FORM>
constexpr int chain_min_waves() {
    return FORM == kChainFwd && sizeof(T) == 4 && ipow(K, F) >= 32 ? 3 : 1;
}

template <typename T, int K, int F, int FORM, int DEP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(chain_min_waves<T, K, F, FORM>())))
void chain_level_kernel(const BucketDesc *__restrict__ descs, int n_desc,
                                                             const int64_t *__restrict__ pool,
                                                             TableMeta *__restrict__ meta, int64_t total_vblocks) {
    using S = ChainShape<K, F>;
    constexpr int N = S::N;
    constexpr bool SUM = FORM == kChainSum;
    constexpr bool FWD = chain_fwd(FORM);
    constexpr int V = chain_v<T, K, F, FORM>();
    static_assert(!FWD || V * N * (int)sizeof(T) <= 256, "forward rows go through the wave's LDS image");
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    T *red = reinterpret_cast<T *>(dyn);
    unsigned char *stage = dyn + kRedBytes;
    constexpr int kImg = FWD ? (kBlock / 64) * chain_img_wave<T, K, F, FORM>() : 0;
    T *small = reinterpret_cast<T *>(dyn + kRedBytes + kImg);

    ChainState<F> c;
    int cur = -1;
    int64_t cur_begin = 0;
    T lmax = T(0);
    for (int64_t vb = blockIdx.x; vb < total_vblocks; vb += gridDim.x) {
        const int bi = n_desc == 1 ? 0 : find_bucket(descs, n_desc, vb);
        if (bi != cur) {
            if (cur >= 0) flush_max<T>(lmax, meta, descs[cur].out_table, descs[cur].flags, red);
            cur = bi;
            lmax = T(0);
            const BucketDesc &d = descs[bi];
            cur_begin = d.vblk_begin;
            chain_load_state<T, K, F, FORM>(c, d, pool + d.dim_off, meta);
            if (vb == cur_begin && threadIdx.x == 0) meta[d.out_table].exp2 = chain_exp2<T>(d, meta);
            c.neg_e = chain_stage<T>(d, meta, small);      // the rescale is in the G tables but this share
        }
        const int64_t tid0 = (vb - cur_begin) * kBlock;
        const int64_t tid = tid0 + threadIdx.x;
        T t[N][V];
        if (tid < c.n_tiles) {
            // rest position of this thread: in / out offsets, G offsets in LDS
            const int row = 4 + F;
            cst_t<int64_t> *dp = as_const(c.dims);     // scalar cache: read-only while the launch runs
            int64_t in_off = c.in_base, out_off = 0;
            int32_t gb[F], gv[F];
            uint64_t q, r;
            divmod_dim((uint64_t)tid, c.t0h, c.t0m, q, r);
            const int64_t i0 = (int64_t)r * V;
            in_off += i0 * dp[2];
            out_off += i0 * dp[3];
            const int64_t in_v = dp[2];
#pragma unroll
            for (int j = 0; j < F; ++j) {
                gv[j] = (int32_t)dp[4 + j];
                gb[j] = c.glds[j] + (int32_t)i0 * gv[j];
            }
            uint64_t rem = q;
            dp += row;
            for (int dd = 1; dd < c.n_dims; ++dd) {
                uint64_t qq, rr;
                divmod_dim(rem, dp[0], dp[1], qq, rr);
                in_off += (int64_t)rr * dp[2];
                out_off += (int64_t)rr * dp[3];
#pragma unroll
                for (int j = 0; j < F; ++j) gb[j] += (int32_t)rr * (int32_t)dp[4 + j];
                rem = qq;
                dp += row;
            }
            const T *big = static_cast<const T *>(c.big);
            if constexpr (SUM) {
                // one slab per slot assignment, V contiguous rest entries each
                const int64_t w0 = readfirstlane64(in_off);
                const uint32_t lob = (uint32_t)((in_off - w0) * (int64_t)sizeof(T));
                const char *wb = reinterpret_cast<const char *>(big + w0);
#pragma unroll
                for (int a = 0; a < N; ++a) {
                    int64_t o = 0;
#pragma unroll
                    for (int p = 0; p < F; ++p) o += (int64_t)S::digit(a, p) * c.is[p];
                    load_n<T, V, kNtLoad, true>(reinterpret_cast<const T *>(wb + o * (int64_t)sizeof(T) + lob), t[a]);
                }
            } else if constexpr (FWD) {
                // one slab per slot assignment: V-wide loads, coalesced over the wave
                // slab base uniform (SGPRs), lane offset 32-bit (planner: kChainLo32)
                const int64_t w0 = readfirstlane64(in_off);
                const uint32_t lob = (uint32_t)((in_off - w0) * (int64_t)sizeof(T));
                const char *wb = reinterpret_cast<const char *>(big + w0);
#pragma unroll
                for (int a = 0; a < N; ++a) {
                    int64_t o = 0;
#pragma unroll
                    for (int p = 0; p < F; ++p) o += (int64_t)S::digit(a, p) * c.is[p];
                    if constexpr (V == 1)
                        t[a][0] = gload(reinterpret_cast<const T *>(wb + o * (int64_t)sizeof(T) + lob));
                    else
                        load_n<T, V, kNtLoad, true>(reinterpret_cast<const T *>(wb + o * (int64_t)sizeof(T) + lob), t[a]);
                }
            } else {
                // K^F contiguous entries (slot 0 fastest) per rest entry
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    T buf[N];
                    load_n<T, N, kNtLoad, true>(big + in_off + v * in_v, buf);
#pragma unroll
                    for (int a = 0; a < N; ++a) t[a][v] = buf[S::rev(a)];
                }
            }
            // the F buckets of the run, in order
            static_for<F>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                if (!((c.gmask >> j) & 1))                     // uniform
                    chain_step<T, K, F, V, j, 0, DEP, SUM>(t, small, gb[j], c.gs[j], c.gsn[j]);
                else                       // V > 1: G_j constant along the V entries (planner-checked)
                    chain_step<T, K, F, V, j, 1, DEP, SUM>(t, small, gb[j], c.gs[j], c.gsn[j]);
            });
            constexpr int NOUT = SUM ? 1 : N;                   // live entries (summing run: t[0])
            if (c.neg_e != 0) {                                 // uniform; 0 unless maxima leave the fold's range
#pragma unroll
                for (int a = 0; a < NOUT; ++a)
#pragma unroll
                    for (int v = 0; v < V; ++v) t[a][v] = ldexp_t(t[a][v], c.neg_e);
            }
#pragma unroll
            for (int a = 0; a < NOUT; ++a)
#pragma unroll
                for (int v = 0; v < V; ++v) lmax = t[a][v] > lmax ? t[a][v] : lmax;
            if constexpr (SUM) store_n<T, V, kNtStore, true>(static_cast<T *>(c.out) + out_off, t[0]);
            if constexpr (FORM == kChainBwd) {
                T *out = static_cast<T *>(c.out);
                const int64_t w0 = readfirstlane64(out_off);       // planner: kChainLo32
                const uint32_t lob = (uint32_t)((out_off - w0) * (int64_t)sizeof(T));
                char *wb = reinterpret_cast<char *>(out + w0);
#pragma unroll
                for (int a = 0; a < N; ++a) {
                    int64_t o = 0;
#pragma unroll
                    for (int p = 0; p < F; ++p) o += (int64_t)S::digit(a, p) * c.os[p];
                    store_n<T, V, kNtStore, true>(reinterpret_cast<T *>(wb + o * (int64_t)sizeof(T) + lob), t[a]);
                }
            }
        }
        if constexpr (FWD) {
            // the thread's V * K^F outputs are the contiguous row tid (planner-checked)
            T row[V * N];
#pragma unroll
            for (int v = 0; v < V; ++v)
#pragma unroll
                for (int a = 0; a < N; ++a) row[v * N + a] = t[a][v];
            store_rows_parts<T, V * N, chain_part_bytes<T, K, F, FORM>() / (int)sizeof(T)>(
                static_cast<T *>(c.out), tid0 + (threadIdx.x & ~63), c.n_tiles, row,
                stage + (threadIdx.x >> 6) * chain_img_wave<T, K, F, FORM>());
        }
    }
    if (cur >= 0) flush_max<T>(lmax, meta, descs[cur].out_table, descs[cur].flags, red);
}

template <typename T, int K, int F, int FORM, int DEP>
static hipError_t go_chain_level(const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream) {
    const int64_t grid = a.vblocks < max_grid ? a.vblocks : max_grid;
    const size_t img = chain_fwd(FORM) ? (size_t)(kBlock / 64) * chain_img_wave<T, K, F, FORM>() : 0;
    const size_t shm = kRedBytes + img + (size_t)small_elems * sizeof(T);
    hipLaunchKernelGGL((chain_level_kernel<T, K, F, FORM, DEP>), dim3((unsigned)grid), dim3(kBlock), shm, stream,
                       a.descs, a.n_desc, a.pool, a.meta, a.vblocks);
    return hipGetLastError();
}

#define BNPP_CASE_CHAIN(T, K, F, FORM, DEP) \
    case 8192 + DEP * 2048 + FORM * 256 + K * 16 + F: return go_chain_level<T, K, F, FORM, DEP>(a, small_elems, max_grid, stream);
#define BNPP_CASE_CHAIN_OK(T, K, F, FORM, DEP) case 8192 + DEP * 2048 + FORM * 256 + K * 16 + F: return true;
// instantiated shapes: forward rows <= 256 B (V-wide forward for runs of
// 4..16 entries), backward tables <= 64 entries
// (V = 1 there); dep "any" only for tables <= 16 entries
#define BNPP_CHAIN_ND(X, T, K, F, FORM) X(T, K, F, FORM, 0) X(T, K, F, FORM, 1)
#define BNPP_CHAIN_F32(X, T) \
    BNPP_CHAIN_ND(X, T, 2, 2, 1) BNPP_CHAIN_ND(X, T, 2, 3, 1) BNPP_CHAIN_ND(X, T, 2, 4, 1) BNPP_CHAIN_ND(X, T, 2, 5, 1) \
    BNPP_CHAIN_ND(X, T, 2, 6, 1) BNPP_CHAIN_ND(X, T, 4, 2, 1) X(T, 2, 2, 1, 2) X(T, 2, 3, 1, 2) X(T, 2, 4, 1, 2) X(T, 4, 2, 1, 2) \
    BNPP_CHAIN_ND(X, T, 2, 2, 2) BNPP_CHAIN_ND(X, T, 2, 3, 2) BNPP_CHAIN_ND(X, T, 2, 4, 2) BNPP_CHAIN_ND(X, T, 2, 5, 2) \
    BNPP_CHAIN_ND(X, T, 2, 6, 2) BNPP_CHAIN_ND(X, T, 4, 2, 2) BNPP_CHAIN_ND(X, T, 4, 3, 2) \
    X(T, 2, 2, 2, 2) X(T, 2, 3, 2, 2) X(T, 2, 4, 2, 2) X(T, 4, 2, 2, 2) BNPP_CHAIN_SUM(X, T) \
    BNPP_CHAIN_ND(X, T, 2, 2, 4) BNPP_CHAIN_ND(X, T, 2, 3, 4) BNPP_CHAIN_ND(X, T, 2, 4, 4) BNPP_CHAIN_ND(X, T, 4, 2, 4) \
    X(T, 2, 2, 4, 2) X(T, 2, 3, 4, 2)
#define BNPP_CHAIN_SUM(X, T) X(T, 2, 2, 3, 0) X(T, 2, 3, 3, 0) X(T, 2, 4, 3, 0) X(T, 4, 2, 3, 0) \
    X(T, 2, 2, 3, 2) X(T, 2, 3, 3, 2) X(T, 2, 4, 3, 2) X(T, 4, 2, 3, 2)
#define BNPP_CHAIN_F64(X, T) \
    BNPP_CHAIN_ND(X, T, 2, 2, 1) BNPP_CHAIN_ND(X, T, 2, 3, 1) BNPP_CHAIN_ND(X, T, 2, 4, 1) \
    X(T, 2, 2, 1, 2) X(T, 2, 3, 1, 2) \
    BNPP_CHAIN_ND(X, T, 2, 2, 2) BNPP_CHAIN_ND(X, T, 2, 3, 2) BNPP_CHAIN_ND(X, T, 2, 4, 2) BNPP_CHAIN_ND(X, T, 2, 5, 2) \
    X(T, 2, 2, 2, 2) X(T, 2, 3, 2, 2) BNPP_CHAIN_SUM(X, T) \
    BNPP_CHAIN_ND(X, T, 2, 2, 4) BNPP_CHAIN_ND(X, T, 2, 3, 4) X(T, 2, 2, 4, 2) X(T, 2, 3, 4, 2)

}  // namespace bnpp
