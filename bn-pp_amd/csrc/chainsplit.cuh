// Split chain runs (gfx950): F consecutive sweep buckets of a binary (K = 2)
// message fused in one pass, the 2^F-entry table of one rest entry spread
// over W = 2^(F-4) waves of one workgroup (16 entries per lane): F = 5..8
// (an fp64 run of 8 has a 128-KiB exchange table and a 129-KiB row image:
// they share their LDS, split_alias, and such runs form no fused belief).
//
// Same arithmetic as chain.cuh (one thread per rest entry, all 2^F entries in
// its registers), which caps a run at 6 buckets (64 registers of table, 3 waves
// per SIMD).  Here a workgroup owns 64 consecutive rest entries (one per lane):
//   phase 1  wave w holds the 16 assignments of slots 0-3 whose slots 4..F-1
//            are w, and runs buckets 0-3 in registers;
//   exchange the 64 x 2^F table goes through LDS (one barrier);
//   phase 2  wave w holds new digits 0-3 in its group and slots 4..F-1, and
//            runs buckets 4..F-1 in registers.
// Every bucket is the reference's arithmetic in the reference's order (p = G *
// m; acc = 0; acc += p over x = 0, 1: factor.cpp:131-143, 199-205), so the
// result is the unfused one's up to the power-of-two scale applied at the end.
// A G value depends on at most one other slot (ChainDep next / prev); a slot
// outside the wave's register group has a wave-uniform digit.
//
// Forward form (summed variables the input's slowest): 16 slab loads per lane
// (256 B per slab per wave-instruction); the wave's 16 outputs of a row are
// contiguous, rows (2^F entries) leave through an LDS image as 4 KiB per wave.
// Backward form (summed variables the input's fastest): the 64 input rows come
// in by 16-B loads through the LDS image; 16 slab stores per lane.
// G tables are staged packed in LDS (8 entries [q][n][x] per base offset, one
// 16-B read per bucket half).  Persistent grid (16 waves per CU) with the next
// two (forward) or one (backward) tiles' loads in flight while a tile is
// computed (tools/chainbw.hip: the 8-bucket split access pattern moves 5.4-5.5
// TB/s against 5.1-5.3 for 6-bucket runs one thread per rest entry).
//
// Dense runs (DENSE, forms kChainFwdSD / kChainBwdSD): the rest is at most two
// dims, dim 0 a power of two contiguous on the streamed side, G_j constant
// along it, and the slot strides one dense block (forward: x = slots as a
// binary number times S; backward: the output slabs likewise).  That is every
// run of a grid's column sweep.  There a tile's addresses are a uniform base
// plus compile-time multiples of S plus the lane: no mixed-radix decode, no
// per-slab 64-bit address arithmetic (tools/splitbw.hip: the same run with
// constant addressing takes 5.99 / 5.81 ms per 2^32-entry message against the
// general form's 6.90 / 6.58 ms).
#pragma once
#include "chain.cuh"

// The split forms need the 160-KiB dynamic-LDS opt-in of gfx950 (CDNA4); the
// planner emits them unconditionally, so any other target must not build.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "chainsplit.cuh: split chain runs need gfx950 (160 KiB LDS per workgroup)"
#endif

#include <algorithm>
#include <mutex>

namespace bnpp {

constexpr int kSplitRows = kSplitRowsHost;   // rest entries per workgroup (one per lane)
constexpr int kMaxDevices = 64;
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
static_assert(kRedBytes == 64, "split_g_budget_bytes assumes 64 B of reduction scratch");
template <typename T, int W>
__device__ __forceinline__ vec_t<T, W> pack_vec(const T *x) {
    vec_t<T, W> v;
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] = x[k];
    return v;
}
// max of two non-negative, non-NaN values: one v_max (a compare and select
// otherwise, for NaN semantics that cannot arise here)
template <typename T>
__device__ __forceinline__ T max_nn(T a, T b) {
    if constexpr (sizeof(T) == 4) return __builtin_fmaxf(a, b);
    else return __builtin_fmax(a, b);
}
// entry `lane` of a run starting at the uniform address `base`, as a scalar
// base plus a 32-bit vector byte offset (the saddr form of global_load /
// global_store): the base is pinned to scalar registers (readfirstlane of its
// halves) and the offset is made opaque in the accessing block (instruction
// selection works block by block; a loop-invariant offset hoisted out of the
// loop arrives as a 64-bit value and every access gets a 64-bit vector
// address add)
__device__ __forceinline__ uint32_t lane_bytes(int lane, int eb) {
    uint32_t o;
    asm volatile("v_mov_b32 %0, %1" : "=v"(o) : "v"((uint32_t)lane * (uint32_t)eb));
    return o;
}
template <typename T>
__device__ __forceinline__ T *lane_at(T *base, uint32_t lane_off) {
    const uint64_t v = (uint64_t)base;
    const uint64_t u = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return (T *)((char *)u + lane_off);
}
template <typename T>
__device__ __forceinline__ T pow2_t(int e) {
    if constexpr (sizeof(T) == 4) return __builtin_amdgcn_ldexpf(1.0f, e);
    else return __builtin_amdgcn_ldexp(1.0, e);
}

__host__ __device__ constexpr int split_waves(int f) { return 1 << (f - 4); }
// LDS: the exchange table and the row image side by side (so a tile needs two
// barriers, not four), then the packed G tables (split_xch_bytes /
// split_img_bytes / kSplitPack, bnpp_device.h)

// One bucket J (slot J, 0-3 in phase 1, 4..F-1 in phase 2) on the lane's 16
// entries.  The local index e holds the local slots' digits; digit(e, p) gives
// any slot's digit for entry e (local ones from e, the others wave-uniform).
template <typename T, int F, int PH, int J, int DEP, typename Digit>
__device__ __forceinline__ void split_step(T (&t)[16], const T *gp, Digit &&digit) {
    // place of slot J in the local index
    constexpr int PJ = PH == 1 ? (8 >> J) : (1 << (F - 1 - J));
    constexpr int Q = DEP == kDepNext ? J + 1 : J - 1;
    constexpr bool HASQ = Q >= 0 && Q < F;
    // the bucket's G values, fetched once from the packed table: [q][n][x]
    // (q: digit of slot Q), one 16-B read per q
    constexpr int NQ = HASQ ? 2 : 1;
    T g[NQ][2][2];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const vec_t<T, 4> v = *reinterpret_cast<const vec_t<T, 4> *>(gp + 4 * q);
        g[q][0][0] = v[0];
        g[q][0][1] = v[1];
        g[q][1][0] = v[2];
        g[q][1][1] = v[3];
    }
    auto gv = [&](int q, int n, int x) { return NQ == 2 && q ? g[NQ - 1][n][x] : g[0][n][x]; };
    // acc = 0; acc += G(0, n) m0; acc += G(1, n) m1 for n = 0, 1.  0 + p == p
    // exactly for the non-negative p of a potential table (no -0 can arise),
    // so the leading add is dropped.
    if constexpr (sizeof(T) == 4) {
        // packed pairs: entries e and e | 1 are one register pair throughout
        // (no moves to pair them up per bucket).  The bucket whose slot sits
        // at bit 0 has both its inputs in one pair; every other bucket takes
        // two pairs, {e, e|1} (x = 0) and {e|PJ, e|PJ|1} (x = 1), to two.
        // Each entry's products and sum are the scalar ones, in that order.
        if constexpr (PJ == 1) {
#pragma unroll
            for (int e = 0; e < 16; e += 2) {
                const int q = HASQ ? digit(e, HASQ ? Q : 0) : 0;
                const v2f a = {t[e], t[e | 1]};
                const v2f m0 = __builtin_shufflevector(a, a, 0, 0), m1 = __builtin_shufflevector(a, a, 1, 1);
                const v2f gx0 = {gv(q, 0, 0), gv(q, 1, 0)}, gx1 = {gv(q, 0, 1), gv(q, 1, 1)};
                const v2f p0 = gx0 * m0, p1 = gx1 * m1;
                const v2f r = p0 + p1;
                t[e] = r[0];
                t[e | 1] = r[1];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 16; e += 2) {
                if (e & PJ) continue;
                const int qa = HASQ ? digit(e, HASQ ? Q : 0) : 0, qb = HASQ ? digit(e | 1, HASQ ? Q : 0) : 0;
                const v2f a = {t[e], t[e | 1]}, c = {t[e | PJ], t[e | PJ | 1]};
                const v2f g00 = {gv(qa, 0, 0), gv(qb, 0, 0)}, g10 = {gv(qa, 0, 1), gv(qb, 0, 1)};
                const v2f g01 = {gv(qa, 1, 0), gv(qb, 1, 0)}, g11 = {gv(qa, 1, 1), gv(qb, 1, 1)};
                const v2f pa0 = g00 * a, pa1 = g10 * c, pc0 = g01 * a, pc1 = g11 * c;
                const v2f ra = pa0 + pa1, rc = pc0 + pc1;
                t[e] = ra[0];
                t[e | 1] = ra[1];
                t[e | PJ] = rc[0];
                t[e | PJ | 1] = rc[1];
            }
        }
    } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            if (e & PJ) continue;
            const int q = HASQ ? digit(e, HASQ ? Q : 0) : 0;    // constant for local slots
            const T m0 = t[e], m1 = t[e | PJ];
            const T p00 = gv(q, 0, 0) * m0, p01 = gv(q, 1, 0) * m0, p10 = gv(q, 0, 1) * m1, p11 = gv(q, 1, 1) * m1;
            t[e] = p00 + p10;
            t[e | PJ] = p01 + p11;
        }
    }
}

// What a split run needs of its descriptor, kept small (uniform registers):
// the slab offsets of the wave's 16 phase-1 entries (forward), the output
// strides of its 16 phase-2 entries (backward), and per bucket the strides of
// G_j along x_j, along the dependency slot and along n_j.
template <typename T, int F, int DEP>
struct SplitState {
    const T *big;
    T *out;
    const int64_t *dims;
    int64_t n_tiles, in_base, t0h, t0m;
    // the power-of-two rescale is folded into the G tables as they are staged
    // (chain_fold: G_j' = G_j * 2^s_j, every bucket's output scaled as the
    // unfused bucket's); there is no per-tile rescale: 16 v_ldexp per lane per
    // tile, or even the untaken branch to them, cost 0.2 ms of a 6.45-ms
    // forward run (profiles/r03_split_fold_ab.jsonl).  left: the share past
    // the fold's range (never, unless maxima leave the normal range), kept in
    // the output's exp2
    int n_dims, gmask, flags, left;
    int64_t is4[4], isw;          // input stride of slots 0-3; slots 4.. of this wave
    int64_t osl[4], osw;          // output stride of the 4 phase-2 local slots; the wave's other slots
    int32_t glds[F], gsj[F], gsq[F], gsn[F];
    // dense runs: tiles per dim-0 row (log2), dim-1 strides (in, out, G_j), slab stride
    int d_shift;
    int64_t d_in1, d_out1, d_slab;
    int32_t d_g1[F];
    // kChainBel (dense backward runs): the forward message and the belief table
    const T *lam;
    T *bel;
};

template <typename T, int F, int DEP, bool DENSE, int FORM>
__device__ __forceinline__ void split_load_state(SplitState<T, F, DEP> &c, cst_t<BucketDesc> &d, const int64_t *pool_,
                                                 TableMeta *meta_, int w) {
    // descriptor, dims pool and table pointers through the scalar cache (they
    // are read-only while the run executes): the state is uniform, and read
    // with vector loads it would sit in vector registers, making every tile's
    // address arithmetic 64-bit vector work
    cst_t<int64_t> *pool = as_const(pool_);
    cst_t<TableMeta> *meta = as_const(meta_);
    constexpr int HB = 8 - F;
    c.dims = pool_;
    c.n_dims = d.n_dims;
    c.n_tiles = d.n_tiles;
    c.t0h = d.tdiv0[0];
    c.t0m = d.tdiv0[1];
    c.gmask = (d.chain >> 8) & 0xff;
    c.flags = d.flags;
    c.in_base = d.in_base[0];
    cst_t<int64_t> *sl = pool + (int64_t)d.n_dims * (4 + F);
    c.isw = 0;
    c.osw = 0;
#pragma unroll
    for (int p = 0; p < F; ++p) {
        const int64_t is = sl[2 * p], os = sl[2 * p + 1];
        if (p < 4) c.is4[p] = is;
        else c.isw += (int64_t)((w >> (F - 1 - p)) & 1) * is;
        // phase 2: local bits of e are slots 4-HB .. F-1 (MSB first); slots
        // below 4-HB carry the wave's digits (cgrp = w << HB | h, slot p = bit 3-p)
        if (p >= 4 - HB) c.osl[p - (4 - HB)] = os;
        else c.osw += (int64_t)((((w << HB) >> (3 - p)) & 1)) * os;
    }
    if constexpr (DENSE) {
        c.d_shift = __builtin_ctz((uint32_t)((uint64_t)pool[0] & 0xffffffffu)) - 6;     // card0 / 64 tiles per row
        cst_t<int64_t> *r1 = pool + (4 + F);
        const bool two = d.n_dims == 2;
        c.d_in1 = two ? r1[2] : 0;
        c.d_out1 = two ? r1[3] : 0;
#pragma unroll
        for (int j = 0; j < F; ++j) c.d_g1[j] = two ? (int32_t)r1[4 + j] : 0;
        c.d_slab = FORM == kChainFwd ? sl[2 * (F - 1)] : sl[1];          // is[F-1] / os[0]
    }
    cst_t<int64_t> *st = sl + 2 * F;
    int gi = 1;
#pragma unroll
    for (int j = 0; j < F; ++j) {
        const int q = DEP == kDepNext ? j + 1 : j - 1;
        c.gsj[j] = (int32_t)st[j * (F + 1) + j];
        c.gsq[j] = q >= 0 && q < F ? (int32_t)st[j * (F + 1) + q] : 0;
        c.gsn[j] = (int32_t)st[j * (F + 1) + F];
        const bool on = (c.gmask >> j) & 1;
        c.glds[j] = on ? d.in_lds_off[gi] : 0;
        gi += on ? 1 : 0;
    }
    c.big = static_cast<const T *>(meta[d.in_table[0]].ptr);
    c.out = static_cast<T *>(meta[d.out_table].ptr);
    c.left = 0;
    c.lam = nullptr;
    c.bel = nullptr;
    if constexpr (DENSE && FORM == kChainBwd) {
        if (d.flags & kChainBel) {
            c.lam = static_cast<const T *>(meta[d.in_table[d.n_in]].ptr) + d.in_base[d.n_in];
            c.bel = static_cast<T *>(meta[d.aux_out].ptr);
        }
    }
}

// workgroup barrier for the LDS exchange only: waits for this wave's LDS
// operations, not for its global loads and stores (__syncthreads would wait
// vmcnt(0) and drain the next tile's prefetched loads)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Persistent workgroups walk the level's tiles (64 rest entries each) grid-
// stride; the next tile's message loads are issued before the current tile is
// computed, so HBM stays busy through the exchange barriers and the stores.
// MODE 2: the launch holds several runs (descriptors); otherwise exactly one,
// and the kernel is the one-run loop only -- without the multi-run path's
// per-bucket restaging live in the same body, the uniform state fits the
// scalar registers (with it: ~80 SGPRs spilled to VGPR lanes, re-read per
// tile).  One-run backward launches come in two kernels, MODE 1 forming a
// fused belief (kChainBel) and MODE 0 not, so the plain runs' register
// allocation does not carry the belief's (fp64: 242 against ~130 VGPRs).
// BNPP_F64_SPLIT_WAVES (variant builds): hold the fp64 dense one-run kernels
// without a belief to that many waves per SIMD (4: 128 VGPRs, the persistent
// grid's 16 waves per CU, at the price of a few spilled registers; left
// alone they take 128-164 VGPRs, 3 waves)
//
// fp64 one-run kernels without a belief (MODE 0) alias the row image with the
// exchange table (split_alias): 65 KiB of LDS per workgroup instead of 129,
// so two 8-wave workgroups share a CU, at two more barriers per tile (the
// image's reads and the exchange's must finish before the other is written);
// the next tile's loads wait in registers instead of the exchange slots, and
// the registers are held to 128 (four waves per SIMD).
#ifndef BNPP_F64_ALIAS
#define BNPP_F64_ALIAS 1
#endif
// BNPP_F64_BEL_ALIAS=1 (variant builds): fp64 runs forming a fused belief on
// the aliased layout too (two 8-wave workgroups per CU at 128 VGPRs, 76 B
// spilled): 29.0 -> 31.9 ms per run of 7, fp64 32x32 MAR 8.21 -> 8.31 s,
// results bit-identical (profiles/r05_f64_belief_alias_ab.txt); off
#ifndef BNPP_F64_BEL_ALIAS
#define BNPP_F64_BEL_ALIAS 0
#endif
// BNPP_BEL_SUM_LATE=0 (variant builds): the round-5 placement of a one-run
// launch's belief sum, at the end of its own tile (1: one tile late, bel_sum)
#ifndef BNPP_BEL_SUM_LATE
#define BNPP_BEL_SUM_LATE 1
#endif
// (fp64 runs of 8 need it in every kernel they have: one-run and multi-run;
// they form no fused belief, so there is no MODE 1 kernel of them)
template <typename T, int MODE, int F>
__host__ __device__ constexpr bool split_alias() {
    return sizeof(T) == 8 && (((BNPP_F64_ALIAS != 0 || F == 8) && MODE == 0) || (F == 8 && MODE == 2) ||
                              ((BNPP_F64_BEL_ALIAS != 0 || F == 8) && MODE == 1));
}
template <int F, int EB, bool ALIAS>
__host__ __device__ constexpr int split_tile_lds() {
    return ALIAS ? (split_xch_bytes(F, EB) > split_img_bytes(F, EB) ? split_xch_bytes(F, EB) : split_img_bytes(F, EB))
                 : split_xch_bytes(F, EB) + split_img_bytes(F, EB);
}
template <typename T, int F, int FORM, int DEP, bool DENSE, int MODE>
__global__ __launch_bounds__(64 * (1 << (F - 4)))
__attribute__((amdgpu_waves_per_eu(split_alias<T, MODE, F>() ? 4 : 1)))
void chain_split_kernel(const BucketDesc *__restrict__ descs, int n_desc, const int64_t *__restrict__ pool,
                        TableMeta *__restrict__ meta, int64_t total_vblocks) {
    constexpr int EB = sizeof(T);
    constexpr int VE = 16 / EB;                            // entries per 16-B chunk
    constexpr int IT = EB;                                 // 16-B chunks per lane per tile (16 entries)
    constexpr int W = split_waves(F);
    constexpr int N = 1 << F;
    constexpr int ROWB = N * EB + 16;                      // image row stride (bytes)
    constexpr int HB = 8 - F;                              // phase 2: bits of h (n-digits 0-3 local)
    constexpr int SB = F - 4;                              // phase 2: bits of the slot combo (slots 4..F-1)
    constexpr int CPR = N * EB / 16;                       // 16-B chunks per row

    // fp64: the row image and exchange table leave room for one workgroup
    // (8 waves at F = 7) per CU, so forward runs keep two tiles' loads in
    // flight instead of one (2 waves per SIMD: the registers are there):
    // 17.08 -> 16.34 ms per 2^32-entry message; the backward runs got slower
    // that way (17.12 -> 17.57 ms) and keep one, and so did fp32 forward runs
    // at 16 waves per CU (5.99 -> 6.23 ms; profiles/r05_f64_ahead2.txt)
    constexpr bool ALIAS = split_alias<T, MODE, F>();
    constexpr bool AHEAD2 = EB == 8 && !ALIAS;
    static_assert(EB == 4 || F <= 7 || ALIAS, "fp64 split runs of 8: the aliased LDS layout only");
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    // the per-wave maxima at a flush: the reduction scratch, or (16 fp64
    // waves) the start of the tile region, free there -- flush() waits for
    // every wave first, and what follows it (setup) waits before LDS is reused
    T *red = reinterpret_cast<T *>(W * EB <= kRedBytes ? dyn : dyn + kRedBytes);
    T *xch = reinterpret_cast<T *>(dyn + kRedBytes);
    unsigned char *img = dyn + kRedBytes + (ALIAS ? 0 : split_xch_bytes(F, EB));
    T *small = reinterpret_cast<T *>(dyn + kRedBytes + split_tile_lds<F, EB, ALIAS>());
    // the wave id as a uniform (scalar) value: derived from threadIdx the
    // compiler takes it as varying per lane, and everything computed from it
    // (slab bases, digits) would occupy vector registers and instructions
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // digit of slot p (4 <= p < F) in phase 1: bit (F-1-p) of w
    auto wdig = [&](int p) { return (w >> (F - 1 - p)) & 1; };
    // the tile's 64 rows are 64 * N * EB contiguous bytes; row traffic
    // (backward loads, forward stores) goes in IT = EB instructions per lane,
    // instruction `it` of the whole workgroup covering W contiguous KiB: 16-B
    // chunk it * 64 W + 64 w + lane (row 16 it + w at F = 8 fp32), not IT
    // consecutive rows per wave (forward 6.06 -> 5.97 ms, backward 5.81 ->
    // 5.69-5.73 ms in tools/bwdprobe.hip, profiles/r04_bwdprobe.jsonl)
    auto chunk = [&](int it) { return it * 64 * W + 64 * w + lane; };

    int cur = -1;
    int64_t cur_begin = 0, cur_end = 0;
    SplitState<T, F, DEP> c;
    T lmax = T(0);
    T bmax = T(0);                                         // kChainBel: the belief's running max (wave 0)

    // bucket of virtual block vb: state, published exponent, G tables in LDS
    auto setup = [&](int64_t vb) {
        const int bi = n_desc == 1 ? 0 : find_bucket(descs, n_desc, vb);
        const BucketDesc &d = descs[bi];
        cur = bi;
        cur_begin = d.vblk_begin;
        cur_end = bi + 1 < n_desc ? descs[bi + 1].vblk_begin : total_vblocks;
        split_load_state<T, F, DEP, DENSE, FORM>(c, *as_const(descs + bi), pool + d.dim_off, meta, w);
        int fs[kMaxDescIn];
        c.left = chain_fold<T>(d, meta, fs);
        // exp2 of the output: the inputs' exp2 and max exponents, plus the
        // share of the rescale not folded (chain_fold)
        if (vb == cur_begin && threadIdx.x == 0) {
            const int64_t e_out = chain_exp2<T>(d, meta) + c.left;
            meta[d.out_table].exp2 = e_out;
            // the belief is stored unscaled: true value = stored * 2^(exp2(lam) + exp2(out))
            if (c.bel) meta[d.aux_out].exp2 = meta[d.in_table[d.n_in]].exp2 + e_out;
        }
        lds_barrier();                                     // the previous bucket's tables are no longer read
        // G_j packed: entry (o, q, n, x) at 8 o + 4 q + 2 n + x holds G_j[o + q
        // gsq + n gsn + x gsj] * 2^fs (gmask is all ones: G_j is input j + 1)
#pragma unroll
        for (int j = 0; j < F; ++j) {
            const T *src = static_cast<const T *>(meta[d.in_table[j + 1]].ptr) + d.in_base[j + 1];
            const int span = d.in_span[j + 1];
            T *dst = small + d.in_lds_off[j + 1];
            const T sc = pow2_t<T>(fs[j + 1]);
            for (int e = threadIdx.x; e < span * kSplitPack; e += 64 * W) {
                const int si = (e >> 3) + ((e >> 2) & 1) * c.gsq[j] + ((e >> 1) & 1) * c.gsn[j] + (e & 1) * c.gsj[j];
                const T g = si < span ? gload(src + si) : T(0);
                dst[e] = g * sc;
            }
        }
        lds_barrier();
    };
    // rest entry of this lane in tile vb: input / output offsets, G offsets
    // (base offsets into the native G tables; packed entries at kSplitPack x).
    // A tile's 64 entries are consecutive along rest dim 0 (planner: its card
    // is a multiple of 64), so the mixed-radix decode is done once per tile on
    // uniform values and each lane adds lane * (stride on dim 0).
    // dense runs: the tile's uniform bases (tin, tout) and G offsets in closed form
    int64_t tin = 0, tout = 0;
    auto decode = [&](int64_t vb, int64_t &in_off, int64_t &out_off, int32_t (&gb)[F]) {
        if constexpr (DENSE) {
            const int64_t rel = vb - cur_begin;
            const int64_t d0 = (rel & ((int64_t(1) << c.d_shift) - 1)) * kSplitRows, d1 = rel >> c.d_shift;
            if constexpr (FORM == kChainFwd) {
                tin = c.in_base + d0 + d1 * c.d_in1;
                tout = d0 * N + d1 * c.d_out1;
                in_off = tin + lane;
                out_off = tout + (int64_t)lane * N;
            } else {
                tin = c.in_base + d0 * N + d1 * c.d_in1;
                tout = d0 + d1 * c.d_out1;
                in_off = tin + (int64_t)lane * N;
                out_off = tout + lane;
            }
            // only the run's boundary bucket (the last forward, the first
            // backward) may have a G table varying along rest dim 1 (planner)
            constexpr int JR = FORM == kChainFwd ? F - 1 : 0;
#pragma unroll
            for (int j = 0; j < F; ++j) gb[j] = j == JR ? (int32_t)d1 * c.d_g1[j] : 0;
            return;
        }
        const int64_t tid0 = (vb - cur_begin) * kSplitRows;
        const int row = 4 + F;
        cst_t<int64_t> *dp = as_const(c.dims);          // scalar cache: read-only while the launch runs
        uint64_t q, r;
        divmod_dim((uint64_t)tid0, c.t0h, c.t0m, q, r);
        int64_t ui = c.in_base + (int64_t)r * dp[2], uo = (int64_t)r * dp[3];
        int32_t ug[F];
#pragma unroll
        for (int j = 0; j < F; ++j) ug[j] = (int32_t)r * (int32_t)dp[4 + j];
        const int64_t si = dp[2], so = dp[3];
        int32_t sg[F];
#pragma unroll
        for (int j = 0; j < F; ++j) sg[j] = (int32_t)dp[4 + j];
        uint64_t rem = q;
        dp += row;
        for (int dd = 1; dd < c.n_dims; ++dd) {
            uint64_t qq, rr;
            divmod_dim(rem, dp[0], dp[1], qq, rr);
            ui += (int64_t)rr * dp[2];
            uo += (int64_t)rr * dp[3];
#pragma unroll
            for (int j = 0; j < F; ++j) ug[j] += (int32_t)rr * (int32_t)dp[4 + j];
            rem = qq;
            dp += row;
        }
        in_off = ui + (int64_t)lane * si;
        out_off = uo + (int64_t)lane * so;
#pragma unroll
        for (int j = 0; j < F; ++j) gb[j] = ug[j] + lane * sg[j];
    };
    // the tile's message loads (16 values per lane)
    auto issue = [&](int64_t in_off, T (&rg)[16]) {
        if constexpr (DENSE && FORM == kChainFwd) {
            // slab x = (slots 0-3 = e) << (F - 4) | (slots 4.. = w), at x * S:
            // uniform slab bases plus the lane's 32-bit byte offset
            const T *wb = c.big + tin + (int64_t)w * c.d_slab;
            const int64_t step = c.d_slab << (F - 4);
            const uint32_t lo = lane_bytes(lane, EB);
#pragma unroll
            for (int e = 0; e < 16; ++e) rg[e] = gload(lane_at(wb + e * step, lo));
        } else if constexpr (DENSE) {
            // 64 input rows of N contiguous values at tin + row * N
            // (the rows are contiguous: chunk q at VE q; uniform part + lane)
            const T *big = c.big + tin;
            const uint32_t lo = lane_bytes(lane, 16);
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const vec_t<T, VE> v = vload<VE, kNtLoad, true>(lane_at(big + VE * (it * 64 * W + 64 * w), lo));
#pragma unroll
                for (int k = 0; k < VE; ++k) rg[VE * it + k] = v[k];
            }
        } else if constexpr (FORM == kChainFwd) {
            // slab of assignment (slots 0-3 = e, slots 4.. = w): uniform base + 32-bit lane offset
            const int64_t w0 = readfirstlane64(in_off);
            const uint32_t lob = (uint32_t)((in_off - w0) * EB);
            const T *wb = c.big + w0 + c.isw;              // uniform
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                int64_t o = 0;
#pragma unroll
                for (int p = 0; p < 4; ++p) o += (int64_t)((e >> (3 - p)) & 1) * c.is4[p];
                const T *sp = wb + o;                      // uniform slab base
                rg[e] = gload(reinterpret_cast<const T *>(reinterpret_cast<const char *>(sp) + lob));
            }
        } else {
            // 64 input rows of N contiguous values (slot 0 fastest), 16-B loads
            // (IT per lane)
            const T *big = c.big;
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int q = chunk(it);
                const int rw = q / CPR, ch = q % CPR;
                const int64_t ro = __shfl(in_off, rw, 64);  // row rw's input offset (held by lane rw)
                const vec_t<T, VE> v = vload<VE, kNtLoad, true>(big + ro + VE * ch);
#pragma unroll
                for (int k = 0; k < VE; ++k) rg[VE * it + k] = v[k];
            }
        }
    };
    auto flush = [&]() {
        const T wm = wave_max(lmax);
        lds_barrier();
        if (lane == 0) red[w] = wm;
        lds_barrier();
        if (threadIdx.x == 0 && (c.flags & kTrackMax)) {
            T m = red[0];
            for (int i = 1; i < W; ++i) m = red[i] > m ? red[i] : m;
            using U = typename FBits<T>::U;
            U *mb = reinterpret_cast<U *>(&meta[descs[cur].out_table].maxbits);
            const U mine = FBits<T>::bits(m);
            if (m > T(0) && __hip_atomic_load(mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mine) atomicMax(mb, mine);
        }
        lmax = T(0);
        if constexpr (FORM == kChainBwd && DENSE) {
            if (c.bel && w == 0 && (c.flags & kTrackMax)) {     // only wave 0 forms beliefs
                const T bm = wave_max(bmax);
                using U = typename FBits<T>::U;
                U *mb = reinterpret_cast<U *>(&meta[descs[cur].aux_out].maxbits);
                if (lane == 0 && bm > T(0)) atomicMax(mb, FBits<T>::bits(bm));
            }
        }
        bmax = T(0);
    };

    // one tile: the 16 values per lane in t, this lane's rest entry decoded
    // Barriers per tile: forward  [phase 1, xch write] B [xch read, phase 2, image write] B [image read];
    // backward [image write] B [image read, phase 1, xch write] B [xch read, phase 2].  A wave past one
    // of them knows every wave has finished the previous tile's reads of the region it writes next.
    // slab of entry e (backward dense runs): the wave's digits (wsl) | e's (sl)
    auto slab_w = [&]() {
        int wsl = 0;
#pragma unroll
        for (int p = 0; p < 4 - HB; ++p) wsl |= (((w << HB) >> (3 - p)) & 1) << p;
        return wsl;
    };
    auto slab_e = [&](int e) {
        int sl = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) sl |= ((e >> (3 - b)) & 1) << (4 - HB + b);
        return sl;
    };
    // kChainBel: the forward message at this lane's 16 output positions of the
    // tile whose rest offset is `to` (the same scattered addresses as the
    // stores), loaded before the tile's exchange so they arrive behind it --
    // in one-run launches before the next tile's row prefetch (BM = 1,
    // below).  They are most of a fused run's extra time (10.4 ms per run
    // against 6.3 ms unfused; 10.9 ms when issued after the prefetch, 6.9 ms
    // with the loads removed); loading them a whole tile ahead needed 128
    // VGPRs and was slower -- profiles/r04_belief_fusion_ab.txt
    T lv[16];
    auto load_lam = [&](int64_t to) {
        if constexpr (FORM == kChainBwd && DENSE) {
            const T *lb = c.lam + to + (int64_t)slab_w() * c.d_slab;
            const uint32_t lo = lane_bytes(lane, EB);
#pragma unroll
            for (int e = 0; e < 16; ++e) lv[e] = gload(lane_at(lb + (int64_t)slab_e(e) * c.d_slab, lo));
        }
    };
    // The belief of the tile whose rest offset is `to`, from the lam * pi
    // products its run_tile left in the image: one wave adds each row's 2^F
    // products in slab order -- the unfused bucket's order (p = lam * pi;
    // acc = 0; acc += p for s = 0, 1, ...) -- a 2^F-long dependent chain per
    // row; the barrier after it hands the image back to the next tile.
    auto bel_sum = [&](int64_t to) {
        if constexpr (FORM == kChainBwd && DENSE) {
            if (w == 0) {
                // (reading the chunks 8 ahead through a register ring measured
                // the same: the chain, not the LDS latency, is what it costs)
                T acc = T(0);
#pragma unroll 4
                for (int c4 = 0; c4 < N / VE; ++c4) {
                    const vec_t<T, VE> v = *reinterpret_cast<const vec_t<T, VE> *>(img + lane * ROWB + 16 * c4);
#pragma unroll
                    for (int k = 0; k < VE; ++k) acc = acc + v[k];
                }
                store_n<T, 1, kNtStore, true>(c.bel + to + lane, &acc);
                bmax = acc > bmax ? acc : bmax;
            }
            lds_barrier();                                 // the image is the next tile's again
        }
    };
    // BM (belief mode): 0 = the run forms no belief; 1 = it does and the
    // caller issued the tile's lam loads (one-run launches: before the next
    // tile's row loads, so waiting for lam leaves those in flight) and sums the
    // products later (bel_sum, after it has issued the next tile's loads); 2 =
    // check c.bel at run time, load lam here and sum here (multi-run launches)
    auto run_tile = [&](auto bmc, T (&t)[16], int64_t out_off, const int32_t (&gb)[F]) {
        constexpr int BM = decltype(bmc)::value;
        if constexpr (FORM == kChainBwd && DENSE && BM == 2) {
            if (c.bel) load_lam(tout);
        }
        if constexpr (FORM == kChainBwd) {
            // rows through the image, then this lane's 16 entries (slots 4.. = w)
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int q = chunk(it);
                const int rw = q / CPR, ch = q % CPR;
                *reinterpret_cast<vec_t<T, VE> *>(img + rw * ROWB + 16 * ch) = pack_vec<T, VE>(t + VE * it);
            }
            lds_barrier();
            int fixed = 0;
#pragma unroll
            for (int p = 4; p < F; ++p) fixed += wdig(p) << p;
            // local index e: slot 0 = bit 3 ... slot 3 = bit 0; row position: slot p
            // at 2^p, so the lane's 16 entries are the 16 consecutive positions
            // fixed .. fixed + 15 (e bit-reversed): IT 16-B reads (lane stride
            // ROWB = 65 x 16 B: a quarter-wave covers all 64 banks once) instead
            // of sixteen 4-B reads, which share 16 banks 4-way
            T u[16];
#pragma unroll
            for (int c4 = 0; c4 < IT; ++c4) {
                const vec_t<T, VE> v = *reinterpret_cast<const vec_t<T, VE> *>(img + lane * ROWB + EB * fixed + 16 * c4);
#pragma unroll
                for (int k = 0; k < VE; ++k) u[VE * c4 + k] = v[k];
            }
#pragma unroll
            for (int e = 0; e < 16; ++e)
                t[e] = u[((e >> 3) & 1) | (((e >> 2) & 1) << 1) | (((e >> 1) & 1) << 2) | ((e & 1) << 3)];
        }

        // phase 1: buckets 0-3 (other slots: local bits of e, slots >= 4 from w)
        auto dig1 = [&](int e, int p) { return p < 4 ? (e >> (3 - p)) & 1 : wdig(p); };
        static_for<4>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            split_step<T, F, 1, j, DEP>(t, small + c.glds[j] + gb[j] * kSplitPack, dig1);
        });
        // exchange: entry (n-digits 0-3 = e, slots 4.. = w) -> xch[(w * 16 + e) * 64 + lane]
        if constexpr (ALIAS) lds_barrier();                // every wave's image reads are done
#pragma unroll
        for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = t[e];
        lds_barrier();
        // phase 2: local e = h << SB | sc; n-digits 0-3 = cgrp = w << HB | h; slots 4.. = sc
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int h = e >> SB, sc = e & ((1 << SB) - 1);
            t[e] = xch[(sc * 16 + ((w << HB) | h)) * 64 + lane];
        }
        // (forward: the image write below; backward: the next tile's image write)
        if constexpr (ALIAS) lds_barrier();                // every wave's exchange reads are done
        auto dig2 = [&](int e, int p) {
            if (p >= 4) return (e >> (F - 1 - p)) & 1;
            const int cg = (w << HB) | (e >> SB);
            return (cg >> (3 - p)) & 1;
        };
        static_for<F - 4>([&](auto jc) {
            constexpr int j = 4 + decltype(jc)::value;
            split_step<T, F, 2, j, DEP>(t, small + c.glds[j] + gb[j] * kSplitPack, dig2);
        });
        // (no per-tile rescale: it is folded into the G tables, SplitState)
#pragma unroll
        for (int e = 0; e < 16; ++e)
            lmax = max_nn(lmax, t[e]);                     // entries are >= 0, never NaN

        if constexpr (FORM == kChainFwd) {
            // row position of entry e: w * 16 + e (slot 0 most significant)
#pragma unroll
            for (int c4 = 0; c4 < IT; ++c4)
                *reinterpret_cast<vec_t<T, VE> *>(img + lane * ROWB + EB * (w * 16 + VE * c4)) =
                    pack_vec<T, VE>(t + VE * c4);
            lds_barrier();
            // the 64 rows are one contiguous block of 64 * N entries (planner-checked):
            // 1 KiB per wave-instruction (chunk())
            T *out = c.out + (DENSE ? tout : __shfl(out_off, 0, 64));
            const uint32_t lo = lane_bytes(lane, 16);
            // (tiles are whole: the planner requires rest dim 0 to be a multiple of 64)
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int q = chunk(it);                   // 16-B chunk within the block
                const int rw = q / CPR, ch = q % CPR;
                const vec_t<T, VE> v = *reinterpret_cast<const vec_t<T, VE> *>(img + rw * ROWB + 16 * ch);
                vstore<VE, kNtStore, true>(lane_at(out + VE * (int64_t)(it * 64 * W + 64 * w), lo), v);
            }
        } else {
            // slab stores: entry e has n-digits 0-3 = (w << HB | h), slots 4.. = sc
            if constexpr (DENSE) {
                // output slab of n-digits (slot p at S << p): e's local bits are
                // slots 4-HB .. F-1 (MSB first), the wave's digits the others
                const int wsl = slab_w();
                T *wb = c.out + tout + (int64_t)wsl * c.d_slab;
                const uint32_t lo = lane_bytes(lane, EB);
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    store_n<T, 1, kNtStore, true>(lane_at(wb + (int64_t)slab_e(e) * c.d_slab, lo), &t[e]);
                if (BM == 1 || (BM == 2 && c.bel)) {
                    // belief of rest entry r = lane: lam * pi per slab s into row r
                    // of the image (free: every wave read its rows before the
                    // exchange barrier); summed by bel_sum -- here (BM 2) or by
                    // the caller once the next tile's loads are in flight (BM 1:
                    // the chain then overlaps them instead of idling the other
                    // waves at a barrier with nothing in flight)
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        *reinterpret_cast<T *>(img + lane * ROWB + EB * (wsl | slab_e(e))) = lv[e] * t[e];
                    lds_barrier();
                    if constexpr (BM == 2 || (BM == 1 && !BNPP_BEL_SUM_LATE)) bel_sum(tout);
                }
            } else {
                const int64_t w0 = readfirstlane64(out_off);
                const uint32_t lob = (uint32_t)((out_off - w0) * EB);
                T *wb = c.out + w0 + c.osw;                // uniform
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    int64_t o = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) o += (int64_t)((e >> (3 - b)) & 1) * c.osl[b];
                    T *dst = reinterpret_cast<T *>(reinterpret_cast<char *>(wb + o) + lob);
                    store_n<T, 1, kNtStore, true>(dst, &t[e]);
                }
            }
        }
    };

    int64_t vb = blockIdx.x;
    if (vb >= total_vblocks) return;
    setup(vb);
    T rg[16];
    int64_t in_off, out_off;
    int32_t gb[F];
    if constexpr (MODE != 2 && FORM == kChainBwd) {
        // one bucket, backward form: the next tile's loads are issued
        // (unconditionally: the last tile is re-read rather than branching, so
        // the wait counts stay static) before the current tile is computed (two
        // tiles ahead, as the forward form: 6.37-6.42 against 6.33-6.41 ms per
        // 2^32-entry message, profiles/r04_split_ab.txt)
        //
        // The loop's memory waits are what the compiler derives from its
        // scoreboard, so the loop is shaped for it: (1) the prologue's row
        // loads are waited for before the loop -- pending at the loop header
        // they merged with the back edge into a wait, at the top of every
        // tile, for the previous tile's slab stores and this tile's lam loads;
        // (2) the lam loads are unconditional in a loop of their own -- issued
        // under a branch, the merge at the branch's join took the path without
        // them and drained them at the top of the tile as well
        decode(vb, in_off, out_off, gb);
        issue(in_off, rg);
        __builtin_amdgcn_s_waitcnt(0x0f70);                // vmcnt(0): the first tile's rows
        // (3) a fused belief's sum (bel_sum) runs one tile late: after the
        // next tile's lam and row loads are issued, so the wave adding the
        // products overlaps them (the other waves wait at its barrier with
        // those loads in flight, not with an idle memory queue)
        auto loop = [&](auto belc) {
            constexpr bool BEL = decltype(belc)::value;
            int64_t bel_to = -1;                           // the tile whose products wait in the image
            while (true) {
                T t[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) t[e] = rg[e];
                if constexpr (BEL) {
                    decode(vb, in_off, out_off, gb);
                    load_lam(tout);
                }
                const int64_t vbn = vb + gridDim.x;
                decode(vbn < total_vblocks ? vbn : total_vblocks - 1, in_off, out_off, gb);
                issue(in_off, rg);
                if constexpr (BEL && BNPP_BEL_SUM_LATE) {
                    if (bel_to >= 0) bel_sum(bel_to);      // uniform
                }
                decode(vb, in_off, out_off, gb);
                run_tile(std::integral_constant<int, BEL ? 1 : 0>{}, t, out_off, gb);
                if constexpr (BEL) bel_to = tout;
                vb = vbn;
                if (vb >= total_vblocks) break;
            }
            if constexpr (BEL && BNPP_BEL_SUM_LATE) bel_sum(bel_to);   // the last tile's
        };
        loop(std::integral_constant<bool, DENSE && MODE == 1>{});
    } else if constexpr (MODE != 2) {
        // one bucket, forward form: the next tile's loads go into registers at
        // the top of a tile and, once the tile is done, into this lane's own
        // slots of the exchange table, where the next tile reads them back
        // (its phase 1 then writes its results to those same slots).  The
        // loop carries no register set with loads in flight: with two
        // alternating sets the compiled loop copied the freshly loaded set at
        // the latch, a wait for every load in flight once per two tiles.
        // Safe without another barrier: a lane reads and rewrites only its own
        // slots, and it stages the next tile after the tile's image barrier,
        // which every wave reaches only after its phase-2 reads of the table.
        // Loads are issued unconditionally (the last tile is re-read rather
        // than branching) so the wait counts stay static
        const int64_t last = total_vblocks - 1;
        T p[16];
        auto stage = [&]() {
#pragma unroll
            for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = p[e];
        };
        if constexpr (ALIAS) {
            // fp64 with the image on the exchange table: the next tile's loads
            // wait in registers (two sets in turn, the loop unrolled twice, so
            // no set is copied at the latch)
            T pa[16], pb[16];
            decode(vb, in_off, out_off, gb);
            issue(in_off, pa);
            auto step = [&](T (&cur)[16], T (&nxt)[16]) {
                const int64_t vbn = vb + gridDim.x;
                decode(vbn < last ? vbn : last, in_off, out_off, gb);
                issue(in_off, nxt);
                decode(vb, in_off, out_off, gb);
                run_tile(std::integral_constant<int, 0>{}, cur, out_off, gb);
                vb = vbn;
                return vb < total_vblocks;
            };
            while (step(pa, pb) && step(pb, pa)) {
            }
            flush();
            return;
        }
        if constexpr (AHEAD2) {
            // fp64: the tile after next is loaded while this one is computed
            // (two register sets in turn, a loop unrolled twice); the next
            // one's set is staged into the exchange slots after the tile
            T p2[16];
            auto stage_from = [&](T (&px)[16]) {
#pragma unroll
                for (int e = 0; e < 16; ++e) xch[(w * 16 + e) * 64 + lane] = px[e];
            };
            decode(vb, in_off, out_off, gb);
            issue(in_off, p);
            stage_from(p);
            decode(vb + gridDim.x < last ? vb + gridDim.x : last, in_off, out_off, gb);
            issue(in_off, p2);
            auto step = [&](T (&pn)[16], T (&pf)[16]) {
                T t[16];
#pragma unroll
                for (int e = 0; e < 16; ++e) t[e] = xch[(w * 16 + e) * 64 + lane];
                const int64_t vb2 = vb + 2 * (int64_t)gridDim.x;
                decode(vb2 < last ? vb2 : last, in_off, out_off, gb);
                issue(in_off, pf);
                decode(vb, in_off, out_off, gb);
                run_tile(std::integral_constant<int, 0>{}, t, out_off, gb);
                stage_from(pn);
                vb += gridDim.x;
                return vb < total_vblocks;
            };
            while (step(p2, p) && step(p, p2)) {
            }
            flush();
            return;
        }
        decode(vb, in_off, out_off, gb);
        issue(in_off, p);
        stage();
        while (true) {
            T t[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) t[e] = xch[(w * 16 + e) * 64 + lane];
            const int64_t vbn = vb + gridDim.x;
            decode(vbn < last ? vbn : last, in_off, out_off, gb);
            issue(in_off, p);
            decode(vb, in_off, out_off, gb);
            run_tile(std::integral_constant<int, 0>{}, t, out_off, gb);
            stage();
            vb = vbn;
            if (vb >= total_vblocks) break;
        }
    } else {
        while (true) {
            T t[16];
            decode(vb, in_off, out_off, gb);
            issue(in_off, t);
            run_tile(std::integral_constant<int, 2>{}, t, out_off, gb);
            const int64_t vbn = vb + gridDim.x;
            if (vbn >= total_vblocks) break;
            if (vbn >= cur_end) {                          // the next tile is in another bucket of the level
                flush();
                setup(vbn);
            }
            vb = vbn;
        }
    }
    flush();
}

#ifndef BNPP_SPLIT_WAVES_PER_CU
#define BNPP_SPLIT_WAVES_PER_CU 16     // resident waves per CU the persistent grid is sized for
#endif
template <typename T, int F, int FORM, int DEP, bool DENSE, bool BEL>
static hipError_t go_chain_split(const LevelArgs &a, int small_elems, hipStream_t stream) {
    constexpr int EB = sizeof(T);
    constexpr int MODE1 = BEL ? 1 : 0;                    // one-run kernel of this key
    const bool one = a.n_desc == 1;
    const bool alias = one ? split_alias<T, MODE1, F>() : split_alias<T, 2, F>();
    const size_t tile_lds = alias ? split_tile_lds<F, EB, true>() : split_tile_lds<F, EB, false>();
    const size_t shm = kRedBytes + tile_lds + (size_t)small_elems * EB;
    // per device (a process may drive several): the 160-KiB LDS opt-in of
    // this instantiation and the CU count the persistent grid is sized for
    struct DevState {
        std::mutex mu;
        bool done[kMaxDevices] = {};
        hipError_t attr[kMaxDevices] = {};
        int cus[kMaxDevices] = {};
    };
    static DevState ds;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    int cus;
    {
        std::lock_guard<std::mutex> g(ds.mu);
        if (!ds.done[dev]) {
            ds.attr[dev] = hipFuncSetAttribute((const void *)chain_split_kernel<T, F, FORM, DEP, DENSE, MODE1>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (ds.attr[dev] == hipSuccess)
                ds.attr[dev] = hipFuncSetAttribute((const void *)chain_split_kernel<T, F, FORM, DEP, DENSE, 2>,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (hipDeviceGetAttribute(&ds.cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                ds.cus[dev] <= 0)
                ds.cus[dev] = 256;
            ds.done[dev] = true;
        }
        if (ds.attr[dev] != hipSuccess) return ds.attr[dev];
        cus = ds.cus[dev];
    }
    // workgroups per CU: the wave target, capped by what fits the CU's LDS
    // (an fp64 run of 7 buckets holds 130.5 KiB: one workgroup, 8 waves)
    int per_cu = BNPP_SPLIT_WAVES_PER_CU / split_waves(F) > 0 ? BNPP_SPLIT_WAVES_PER_CU / split_waves(F) : 1;
    per_cu = std::max(1, std::min<int>(per_cu, (int)((size_t)kSplitLdsBytes / shm)));
    const int64_t grid = a.vblocks < (int64_t)cus * per_cu ? a.vblocks : (int64_t)cus * per_cu;
    if (one)
        hipLaunchKernelGGL((chain_split_kernel<T, F, FORM, DEP, DENSE, MODE1>), dim3((unsigned)grid),
                           dim3(64 * split_waves(F)), shm, stream, a.descs, a.n_desc, a.pool, a.meta, a.vblocks);
    else
        hipLaunchKernelGGL((chain_split_kernel<T, F, FORM, DEP, DENSE, 2>), dim3((unsigned)grid),
                           dim3(64 * split_waves(F)), shm, stream, a.descs, a.n_desc, a.pool, a.meta, a.vblocks);
    return hipGetLastError();
}

// forms kChainFwdS / kChainBwdS and their dense variants kChainFwdSD /
// kChainBwdSD (bnpp_device.h), K = 2, dep next / prev; F = 5..8 (fp64 runs of
// 8 without a belief kernel); dense backward runs forming a fused belief have their own key
// (chain_key + kChainBelKey)
#define BNPP_CASE_CHAIN_SPLIT(T, F, FORM, KFORM, DEP, DENSE, BEL) \
    case 8192 + DEP * 2048 + FORM * 256 + 2 * 16 + F + (BEL ? kChainBelKey : 0): \
        return go_chain_split<T, F, KFORM, DEP, DENSE, BEL>(a, small_elems, stream);
#define BNPP_CASE_CHAIN_SPLIT_OK(T, F, FORM, KFORM, DEP, DENSE, BEL) \
    case 8192 + DEP * 2048 + FORM * 256 + 2 * 16 + F + (BEL ? kChainBelKey : 0): return true;
#define BNPP_CHAIN_SPLIT_FD(X, T, F) X(T, F, 5, kChainFwd, 0, false, false) X(T, F, 5, kChainFwd, 1, false, false) \
    X(T, F, 6, kChainBwd, 0, false, false) X(T, F, 6, kChainBwd, 1, false, false) \
    X(T, F, 7, kChainFwd, 0, true, false) X(T, F, 7, kChainFwd, 1, true, false) \
    X(T, F, 8, kChainBwd, 0, true, false) X(T, F, 8, kChainBwd, 1, true, false) \
    X(T, F, 8, kChainBwd, 0, true, true) X(T, F, 8, kChainBwd, 1, true, true)
#define BNPP_CHAIN_SPLIT(X) BNPP_CHAIN_SPLIT_FD(X, float, 5) BNPP_CHAIN_SPLIT_FD(X, float, 6) \
    BNPP_CHAIN_SPLIT_FD(X, float, 7) BNPP_CHAIN_SPLIT_FD(X, float, 8)
// fp64 runs of 8: no fused-belief kernel (the belief's run is at most 7, split_max_bel_f)
#define BNPP_CHAIN_SPLIT_FD_NOBEL(X, T, F) X(T, F, 5, kChainFwd, 0, false, false) X(T, F, 5, kChainFwd, 1, false, false) \
    X(T, F, 6, kChainBwd, 0, false, false) X(T, F, 6, kChainBwd, 1, false, false) \
    X(T, F, 7, kChainFwd, 0, true, false) X(T, F, 7, kChainFwd, 1, true, false) \
    X(T, F, 8, kChainBwd, 0, true, false) X(T, F, 8, kChainBwd, 1, true, false)
#if BNPP_F64_BEL8
#define BNPP_CHAIN_SPLIT_F64(X) BNPP_CHAIN_SPLIT_FD(X, double, 5) BNPP_CHAIN_SPLIT_FD(X, double, 6) \
    BNPP_CHAIN_SPLIT_FD(X, double, 7) BNPP_CHAIN_SPLIT_FD(X, double, 8)
#else
#define BNPP_CHAIN_SPLIT_F64(X) BNPP_CHAIN_SPLIT_FD(X, double, 5) BNPP_CHAIN_SPLIT_FD(X, double, 6) \
    BNPP_CHAIN_SPLIT_FD(X, double, 7) BNPP_CHAIN_SPLIT_FD_NOBEL(X, double, 8)
#endif

}  // namespace bnpp
