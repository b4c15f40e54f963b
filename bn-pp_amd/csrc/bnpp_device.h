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

namespace bnpp {

constexpr int kMaxIn = 8;          // inputs per fused launch; longer chains are split
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
};

struct BucketDesc {
    int64_t out_size;               // entries of the output table
    int64_t n_vec;                  // out_size / vec
    int64_t vblk_begin;             // first virtual block of this bucket within its launch
    int32_t n_in, n_dims, k, vec;   // k = card of the summed variable (1: pure product)
    int32_t out_table, flags;
    int32_t in_table[kMaxIn];
    int64_t in_base[kMaxIn];        // evidence offset of each view
    int64_t elim_stride[kMaxIn];    // stride of the summed variable in each view (0: absent)
    int64_t dim_off;                // offset into the dims pool
};

// dims pool, per output dim (fastest first): 2 + n_in int64 words
//   w0 = card | (shift << 32) | (pow2 << 40)    w1 = magic    w2.. = stride per input
inline int64_t pack_dim_header(uint32_t card, uint32_t shift, bool pow2) {
    return (int64_t)((uint64_t)card | ((uint64_t)shift << 32) | ((uint64_t)(pow2 ? 1 : 0) << 40));
}

}  // namespace bnpp
