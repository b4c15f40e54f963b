// Plain-old-data structures shared by the host planner and the HIP kernels.
//
// A *bucket* is one fused   out = sum_{x} prod_i in_i   over a set of input
// *views* (model.cpp:414-418: Factor(1.0) *= f_1 *= ... *= f_m; .sum_out(x)).
// A pure product (Factor::product, factor.cpp:117-147) is a bucket with k = 1,
// a plain sum-out (factor.cpp:182-212) a bucket with one input, and evidence
// conditioning (factor.cpp:214-242) is folded into a view's base offset.
//
// The mixed-radix index arithmetic of domain.cpp:15-190 is compiled into
// per-dimension (card, stride_i) rows: output dims are stored fastest-first,
// after merging adjacent dims that are contiguous in every input.
#pragma once
#include <stdint.h>

#if !defined(__HIPCC__) && !defined(__host__)
#define __host__
#define __device__
#endif

namespace bnpp {

constexpr int kMaxIn = 8;          // inputs per fused launch; longer chains are split
constexpr int kMaxDescIn = 10;     // descriptor slots: a fused run of 8 buckets has 8 G tables + the message
                                   // (+ the forward message of a fused belief, kChainBel)
constexpr int kSplitRowsHost = 64; // rest entries per workgroup of the split chain forms (chainsplit.cuh)
// split forms: each G_j staged in LDS packed, 8 entries [q][n][x] per base
// offset (one 32-B pair of 16-B reads per bucket); LDS per workgroup: the
// reduction scratch, the exchange table, the row image, then the packed G
constexpr int kSplitPack = 8;
constexpr int kSplitLdsBytes = 160 * 1024;
constexpr int split_xch_bytes(int f, int eb = 4) { return kSplitRowsHost * (1 << f) * eb; }
constexpr int split_img_bytes(int f, int eb = 4) { return kSplitRowsHost * ((1 << f) * eb + 16); }
// fp64 runs of 8 exist only as kernels whose row image shares the exchange
// table's LDS (chainsplit.cuh split_alias): the larger of the two, not the sum
constexpr int split_g_budget_bytes(int f, int eb = 4) {
    return kSplitLdsBytes - 64 -
           (eb == 8 && f == 8 ? (split_xch_bytes(f, eb) > split_img_bytes(f, eb) ? split_xch_bytes(f, eb) : split_img_bytes(f, eb))
                              : split_xch_bytes(f, eb) + split_img_bytes(f, eb));
}
constexpr int split_max_f(int) { return 8; }                    // longest split run (fp32 and fp64)
// longest run forming a fused belief; BNPP_F64_BEL8 (variant builds): fp64
// runs of 8 forming one too (the aliased layout, chainsplit.cuh split_alias)
#ifndef BNPP_F64_BEL8
#define BNPP_F64_BEL8 0
#endif
constexpr int split_max_bel_f(int eb) { return eb == 4 || BNPP_F64_BEL8 ? 8 : 7; }
constexpr int kBlock = 256;        // threads per workgroup (4 waves of 64)

// One per table (source factor or message), resident in device memory.
// true value = stored value * 2^exp2.  maxbits holds the IEEE bits of the
// table's max entry (entries are >= 0, so unsigned order == float order) and
// is raised with atomicMax by the producing kernel.
struct TableMeta {
    void *ptr;
    uint64_t maxbits;
    int64_t exp2;
    int64_t size;
};

enum BucketFlags : int32_t {
    kScale = 1,        // renormalise by the inputs' max exponents (exact power-of-two)
    kTrackMax = 2,     // raise meta[out].maxbits
    kOutStrided = 4,   // dims permuted: output offset from per-dim output strides
                       // (n_dims words after the dims rows in the pool)
    kDivide = 16,      // Factor::divide (factor.cpp:149-180): p = in_0 / in_1 instead of the product
    kChainLo32 = 8,    // chain form: the streamed side (forward input / backward output)
                       // is linear in the thread index, so one wave's accesses are a
                       // uniform base + a 32-bit lane offset (saddr addressing)
    kChainBel = 32,    // dense backward split run that also forms a delivery's belief:
                       // aux_out[r] = sum over the run's slot combination s (ascending)
                       // of lam[r + s S] * out[r + s S] (lam: in_table[n_in], laid out
                       // as the run's output), unscaled (exp2 = exp2(lam) + exp2(out))
};

// Each thread evaluates a V1 x V2 register tile of the output: V1 entries of
// the fastest output dim times V2 entries of the next one (V2 > 1 only when
// V1 covers the whole fastest dim, so a tile is V1*V2 contiguous entries).
struct BucketDesc {
    int64_t out_size;               // entries of the output table
    int64_t n_tiles;                // out_size / (v1 * v2)
    int64_t vblk_begin;             // first virtual block of this bucket within its launch
    int64_t tdiv0[2], tdiv1[2];     // divisors card0/v1 and card1/v2 (dim header, magic)
    int32_t n_in, n_dims, k, v1, v2;// k = card of the summed variable (1: pure product)
    int32_t out_table, flags;
    int32_t in_table[kMaxDescIn];
    int64_t in_base[kMaxDescIn];        // evidence offset of each view
    int64_t elim_stride[kMaxDescIn];    // stride of the summed variable in each view (0: absent)
    int64_t dim_off;                // offset into the dims pool
    // stream form (big >= 0): input `big` is read from HBM with loads of class
    // bcls; every other input is copied whole into LDS once per workgroup
    int32_t big, bcls;
    int32_t small_elems;            // LDS elements for the small inputs
    int32_t in_lds_off[kMaxDescIn];     // element offset of each small input in LDS
    int32_t in_span[kMaxDescIn];        // elements of each small input's reachable range
    // chain form (chain != 0): F consecutive buckets of a sweep fused in
    // registers; chain = F | gmask << 8 | form << 16 | dep << 20 (ChainForm, ChainDep)
    int32_t chain;
    // slab form: lanes sharing one output tile (0/1, or 2 when a tile's row is
    // 32 B: each lane then stores 16 B and a wave's store is one contiguous
    // 1-KiB run instead of 16-B pieces at a 32-B stride)
    int32_t lanes;
    // kChainBel: the belief table the run also writes
    int32_t aux_out;
    // slab form with outer dims (outer_n > 0 combinations of the output dims
    // slower than the slab dim, each a run of whole virtual blocks):
    // outer_div = (dim header, magic) of the blocks per combination; the pool
    // at dim_off + outer_rel holds, per combination, n_in offsets added to the
    // inputs' bases (the big input's net of the combination's output offset)
    int32_t outer_n, outer_rel;
    int64_t outer_div[2];
    // slab level launches: passes of kBlock / lanes tiles per block (0/1, or 2)
    int32_t slab_r;
    // slab form whose tile row (C0 = v1 entries) spans output dims 0 and 1:
    // the card of dim 0 (the small inputs' y offset is (y % slab_y2) * stride0
    // + (y / slab_y2) * stride1); 0 when the row is output dim 0 alone
    int32_t slab_y2;
};
constexpr int kSlabMaxOuter = 64;

// arguments of one level launch (a group of buckets of one kernel variant)
struct LevelArgs {
    const BucketDesc *descs;
    int n_desc;
    const int64_t *pool;
    TableMeta *meta;
    int64_t vblocks;
};

// loads of the big input of a stream bucket, relative to one thread's tile
enum BigClass : int32_t { kBigRow = 1, kBigCol = 2, kBigFull = 3, kBigDirect = 4, kBigOne = 5,
                                kBigInter2 = 6, kBigInter4 = 7,    // summed var fastest in the big input, card 2 / 4
                                kBigSlab = 8 };   // slab form (slab.cuh): v1 = card of output dim 0, v2 = s per lane
constexpr int kStreamSmallMax = 4096;      // entries: inputs at most this big go to LDS
constexpr int kStreamLdsBudget = 32768;    // bytes of LDS for the small inputs

// Kernel variant: one instantiation per (input-count class, v1, v2) so every
// launch gets the register allocation of its own shape (v1*8+v2 is unique over
// the instantiated tiles 1x1 2x1 4x1 2x2 2x4 4x2 4x4 2x8 and the whole-dim
// rows 3x1 5x1 6x1 7x1).
__host__ __device__ inline int nin_class(int n_in) { return n_in <= 1 ? 1 : n_in <= 2 ? 2 : n_in <= 4 ? 4 : 8; }
__host__ __device__ inline int variant_key(int n_in, int v1, int v2) { return nin_class(n_in) * 64 + v1 * 8 + v2; }
// + kGenericO32: the same kernel with 32-bit table offsets, for launches whose
// every input is under 4 GiB (generic_o32)
constexpr int kGenericO32 = 1024;
__host__ __device__ inline bool generic_o32(int64_t max_in_bytes) { return max_in_bytes <= (int64_t)0xffffffff; }
// stream kernels: 4096 + big-class * 256 + v1 * 16 + v2  (v1, v2 <= 8), + kStream8In
// for buckets of 5-8 inputs (their own instantiations: kernels.cuh NI = 8)
constexpr int kStream8In = 2048;
constexpr int kStream8Bcls = 5;            // big classes Row .. One (no interleaved forms) for 5-8 inputs
__host__ __device__ inline int stream_key(int bcls, int v1, int v2, int n_in = 0) {
    return 4096 + (n_in > 4 ? kStream8In : 0) + bcls * 256 + v1 * 16 + v2;
}
// slab kernels (slab.cuh): K summed values, C0 entries of output dim 0, V slow-dim entries per lane
// and R passes of tiles per block (level launches, BucketDesc::slab_r: 1 or 2)
// + kSlab8In for buckets of 5-8 inputs and for rows over two output dims
// (slab_y2; their own instantiations: slab.cuh NI = 8; pass n_in = 8 for those)
constexpr int kSlab8In = 8192;
__host__ __device__ constexpr int slab_key(int k, int c0, int v, int h = 1, int r = 1, int n_in = 0) {
    return 16384 + (n_in > 4 ? kSlab8In : 0) + k * 1024 + (r == 4 ? 512 : r == 2 ? 256 : 0) + c0 * 16 + v + (h == 2 ? 8 : 0);
}

// Chain (sweep) form: F consecutive buckets of an elimination chain in one
// pass.  Input 0 is the message entering the run; bucket j of the run sums
// slot variable x_j out of a K^F register table and puts its new variable n_j
// in the same slot, multiplying by G_j (the product of bucket j's factor
// tables, inputs 1.. in order, present when bit j of gmask is set).
//   kChainFwd: x_j are the input's slowest variables (one slab per slot
//              assignment), n_j the output's fastest block (per-thread row of
//              K^F entries, stored through the wave's LDS image)
//   kChainBwd: x_j are the input's fastest variables (slot 0 fastest: one
//              contiguous K^F block per entry of the rest), the output holds
//              n_j at slab strides; 16 B of the rest's fastest dim per thread
//   kChainSum: every bucket only sums its variable out (no new variable: the
//              last column of a sweep); slots are the input's slabs, V rest
//              entries per thread contiguous in input and output
//   kChainFwdV: kChainFwd with V rest entries per thread (vector slab loads,
//              rows of V * K^F entries); short runs, where one entry per
//              thread leaves the kernel issue-bound
//   kChainFwdS / kChainBwdS: the forward / backward layouts with the 2^F table
//              of one rest entry split over 2^(F-4) waves (chainsplit.cuh;
//              K = 2, fp32, F = 5..8), one workgroup per 64 rest entries
//   kChainFwdSD / kChainBwdSD: the same with dense addressing (rest of <= 2
//              dims, dim 0 a power of two, slots one dense block of strides)
enum ChainForm : int32_t { kChainFwd = 1, kChainBwd = 2, kChainSum = 3, kChainFwdV = 4, kChainFwdS = 5, kChainBwdS = 6,
                           kChainFwdSD = 7, kChainBwdSD = 8 };
__host__ __device__ inline bool chain_split_form(int form) {
    return form == kChainFwdS || form == kChainBwdS || form == kChainFwdSD || form == kChainBwdSD;
}
// Which slots G_j depends on besides its own (x_j, n_j): the next slot (j+1,
// e.g. a forward sweep's vertical factor), the previous one (j-1, backward),
// or any (every G value of a bucket fetched separately; small tables only).
enum ChainDep : int32_t { kDepNext = 0, kDepPrev = 1, kDepAny = 2 };
__host__ __device__ inline int chain_key(int form, int k, int f, int dep) {
    return 8192 + dep * 2048 + form * 256 + k * 16 + f;
}
// a dense backward split run forming a fused belief (kChainBel) launches its
// own kernel: key chain_key(...) + kChainBelKey (k * 16 + f < 128 leaves the bit free)
constexpr int kChainBelKey = 128;
// rest entries per thread of the backward form (the forward form has 1)
__host__ __device__ constexpr int chain_bwd_v(int n, int elem_bytes) {
    return 64 / n < 1 ? 1 : (64 / n > 16 / elem_bytes ? 16 / elem_bytes : 64 / n);
}
// rest entries per thread of kChainFwdV: 16 B loads, rows of at most 128 B
__host__ __device__ constexpr int chain_fwd_v(int n, int elem_bytes) {
    return n * elem_bytes * (16 / elem_bytes) <= 128 ? 16 / elem_bytes
           : n * elem_bytes * (8 / elem_bytes) <= 128 && elem_bytes <= 4 ? 8 / elem_bytes : 1;
}
// chain pool rows: per rest dim (fastest first) 4 + F words
//   w0 header  w1 magic  w2 input stride  w3 output stride  w4.. G_j stride (j < F)
// then per slot p: input stride, output stride (2F words); then per bucket j:
// G_j strides of the variable in every slot at that bucket (slot j: x_j), and
// of n_j (F * (F + 1) words)

// dims pool, per output dim (fastest first): 2 + n_in int64 words
//   w0 = card | (shift << 32) | (pow2 << 40)    w1 = magic    w2.. = stride per input
inline int64_t pack_dim_header(uint32_t card, uint32_t shift, bool pow2) {
    return (int64_t)((uint64_t)card | ((uint64_t)shift << 32) | ((uint64_t)(pow2 ? 1 : 0) << 40));
}

// Loopy BP over the factor graph (bp.hip; graph.cpp:256-403).  Edge e joins
// factor edge_fac[e] and its scope variable edge_var[e]; a factor's edges are
// [f_edge_off[f], f_edge_off[f+1]) in scope order, a variable's are
// v_edges[v_edge_off[v] .. v_edge_off[v+1]) by ascending factor id.  Message e
// occupies [msg_off[e], msg_off[e+1]) of v2f / f2v / raw; item_edge maps a
// message entry back to its edge.  edge_stride[e]: stride of edge_var[e] in
// the factor's table (row-major, last scope variable fastest).
// lane class of a factor->variable sum by its number of terms: class 0 (< 16
// terms) one lane, classes 1 / 2 / 3 (from 16 / 64 / 256 terms) 4 / 16 / 64 lanes
__host__ __device__ constexpr int bp_lane_class(int64_t terms) {
    return terms >= 256 ? 3 : terms >= 64 ? 2 : terms >= 16 ? 1 : 0;
}
constexpr int kBpLdsMsgMax = 4096;          // message entries kept in LDS (v2f + f2v: 64 KiB)
struct BpArgs {
    int32_t n_vars, n_edges, n_msg, max_iter;
    double eps;
    const int32_t *cards;
    const double *tables;
    const int64_t *tab_off;                 // n_factors + 1
    const int32_t *f_edge_off;              // n_factors + 1
    const int32_t *edge_var, *edge_fac;     // n_edges
    const uint32_t *edge_stride;            // n_edges
    const int32_t *msg_off;                 // n_edges + 1
    const int32_t *item_edge;               // n_msg
    // factor->variable message entries grouped by lane class (bp_lane_class):
    // class c holds cls_items[cls_off[c] .. cls_off[c+1])
    int32_t cls_off[5];
    const int32_t *cls_items;
    int32_t msgs_in_lds;                    // v2f / f2v live in LDS (2 * n_msg doubles fit)
    const int32_t *v_edge_off, *v_edges;    // n_vars + 1, n_edges
    const int32_t *marg_off;                // n_vars + 1
    double *v2f, *f2v, *raw, *marg;
    int32_t *iterations;
};

// Multi-workgroup flood (bp.hip, bp_flood_*): the same schedule as BpArgs's
// one-workgroup loop, one launch per phase and iteration, for models whose
// per-iteration work would keep one workgroup busy for long (or whose tables
// pass 2^31 entries).  A factor->variable message entry t is a sum over
// n_f / r terms; it is cut into segments of at most kBpSegTerms terms, held
// in entry order (segments of entry t: [seg_off[t], seg_off[t+1]), term
// ranges ascending), each summed by a group of G lanes into part[segment]; the
// finishing launch adds an entry's parts in order.  err is a ring of
// kBpErrRing per-iteration maxima (fp64 bit patterns: non-negative doubles
// order like their bits); a launch of iteration it returns at once when
// iteration it-1 already met the tolerance.
constexpr int kBpFloodBlock = 256;
constexpr uint64_t kBpSegTerms = 16384;     // 64 lanes x 256 terms
constexpr int kBpErrChunk = 32;             // iterations per host check
constexpr int kBpErrRing = 2 * kBpErrChunk;
struct BpFlood {
    int32_t n_vars, n_edges, n_msg;
    int32_t idx64;                          // 64-bit table indices for every factor (test knob)
    int32_t one_seg;                        // every entry is one segment (segment t = entry t)
    double eps;
    const int32_t *cards;
    const double *tables;
    const int64_t *tab_off;                 // n_factors + 1 (entries)
    const int32_t *f_edge_off;              // n_factors + 1
    const int32_t *edge_var, *edge_fac;     // n_edges
    const uint64_t *edge_stride;            // n_edges
    const int32_t *msg_off;                 // n_edges + 1
    const int32_t *item_edge;               // n_msg
    const int64_t *seg_off;                 // n_msg + 1
    const int32_t *seg_item;                // per segment: its message entry
    const uint64_t *seg_q0;                 // per segment: first term
    // segments by lane class c: cls_seg[cls_pos[c] .. cls_pos[c+1]), blocks
    // [cls_blk[c], cls_blk[c+1]) of the factor->variable launch
    int64_t cls_pos[5];
    int32_t cls_blk[5];
    const int32_t *cls_seg;
    const int32_t *v_edge_off, *v_moff;     // n_vars + 1; per edge of a variable: msg_off of that edge
    const int32_t *marg_off;                // n_vars + 1
    double *v2f, *f2v, *raw, *part, *marg;
    unsigned long long *err;                // kBpErrRing
};

}  // namespace bnpp
