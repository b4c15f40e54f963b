// Host-side planning for the fused bucket kernels (no HIP calls; unit-testable on CPU).
#pragma once
#include <cstdint>
#include <climits>
#include <cstdlib>
#include <functional>
#include <string>
#include <memory>
#include <utility>
#include <vector>

#include "bnpp_device.h"

namespace bnpp {

// Environment switches.  The product reads only the switches the tests use to
// compare kernel forms and plan shapes bit for bit (BNPP_NO_CHAIN, _NO_SPLIT,
// _NO_DENSE, _NO_SLAB, _NO_BEL_FUSE, _TREE_SLOTS, _KEEP_LOG2, ...), the memory
// budget and diagnostics.  Tuning knobs -- launch shapes and layouts measured
// once and settled (tools/) -- are read only by a build with
// -DBNPP_TUNING_KNOBS (tools/build_variant.sh); elsewhere they read as unset.
#ifdef BNPP_TUNING_KNOBS
inline const char *tuning_knob(const char *name) { return std::getenv(name); }
#else
inline const char *tuning_knob(const char *) { return nullptr; }
#endif
// the switches that change a plan (the job cache and the slot memo key on them)
constexpr const char *kPlanKnobs[] = {"BNPP_NO_CHAIN", "BNPP_NO_SPLIT", "BNPP_NO_DENSE", "BNPP_NO_SLAB",
                                      "BNPP_NO_SLAB_OUTER", "BNPP_NO_BEL_FUSE", "BNPP_NO_CHAIN_FWDV",
                                      "BNPP_NO_FREE_REDUCE", "BNPP_NO_REDUCE_MANY", "BNPP_NO_DEDUP",
                                      "BNPP_TREE_SLOTS", "BNPP_KEEP_LOG2", "BNPP_SLOW_LOG2", "BNPP_SPLIT_MIN_F",
                                      "BNPP_CHAIN_RUN_MAX", "BNPP_MEM_BUDGET_GB", "BNPP_NO_O32"};

// Run body(i) for i in [0, n) on up to `threads` host threads (0: hardware
// concurrency, capped at 16 — the per-GPU CPU share of the target machines).
void parallel_for(int64_t n, const std::function<void(int64_t)> &body, int threads = 0);
// parallel_for calls on this thread with threads = 0 use `n` threads while in scope (0: default)
extern thread_local int t_host_threads;
struct ScopedHostThreads {
    int saved;
    explicit ScopedHostThreads(int n) : saved(t_host_threads) { t_host_threads = n; }
    ~ScopedHostThreads() { t_host_threads = saved; }
};

// A table as one bucket input sees it: table id, evidence base offset, and the
// (variable, stride) pairs that remain after conditioning (domain.cpp:74-90).
struct View {
    int table = -1;
    int64_t base = 0;
    std::vector<int> vars;
    std::vector<int64_t> strides;
};

// Row-major strides, last variable fastest (domain.cpp:15-26).
// Sizes, strides and byte counts saturate at kSatMax (2^60): a min-fill order
// on a large grid plans tables of 2^100+ entries that no device could hold;
// they must compare as "too big" against any memory budget, not overflow.
constexpr int64_t kSatMax = (int64_t)1 << 60;
inline int64_t sat_mul(int64_t a, int64_t b) {
    int64_t r;
    return __builtin_mul_overflow(a, b, &r) || r > kSatMax ? kSatMax : r;
}
inline int64_t sat_add(int64_t a, int64_t b) {
    int64_t r;
    return __builtin_add_overflow(a, b, &r) || r > kSatMax ? kSatMax : r;
}
// entries a view can reach from its table's start (base + the last entry's
// offset + 1): what the 32-bit-offset generic kernels are chosen by
inline int64_t view_span(const View &v, const std::vector<int> &cards) {
    int64_t span = sat_add(v.base, 1);
    for (size_t j = 0; j < v.vars.size() && j < v.strides.size(); ++j)
        span = sat_add(span, sat_mul(cards[v.vars[j]] - 1, v.strides[j]));
    return span;
}
// generic-kernel variant of a bucket whose largest input view reaches
// max_in_bytes: the 32-bit-offset kernels only when every offset fits
inline int generic_variant(int n_in, int v1, int v2, int64_t max_in_bytes, bool no_o32 = false) {
    return variant_key(n_in, v1, v2) + (generic_o32(max_in_bytes) && !no_o32 ? kGenericO32 : 0);
}
std::vector<int64_t> natural_strides(const std::vector<int> &vars, const std::vector<int> &cards);
int64_t table_size(const std::vector<int> &vars, const std::vector<int> &cards);
View natural_view(int table, const std::vector<int> &vars, const std::vector<int> &cards);
// Factor::conditioning as a view (factor.cpp:214-242): evidence vars leave the
// scope and move into the base offset.  ev_val[v] < 0 means "no evidence on v".
View conditioned_view(int table, const std::vector<int> &vars, const std::vector<int> &cards,
                      const std::vector<int> &ev_val);

// Scope rules of the reference.
std::vector<int> union_scope(const std::vector<int> &a, const std::vector<int> &b);   // domain.cpp:32-41
std::vector<int> chain_scope(const std::vector<View> &in);                             // Factor(1.0) *= ...
std::vector<int> remove_var(const std::vector<int> &s, int v);                         // domain.cpp:54-59

struct BucketSpec {
    std::vector<View> in;
    int elim_var = -1;              // -1: pure product
    std::vector<int> out_vars;      // output layout (slowest first)
    int out_table = -1;
    int level = 0;
    // chain form (bnpp_device.h, ChainForm): in[0] is the message entering a
    // run of fused buckets, bucket j sums chain_x[j] and brings in chain_n[j];
    // in[1..] are the G tables of the buckets whose bit is set in chain_gmask
    std::vector<int> chain_x, chain_n;
    int chain_gmask = 0;
    // a dense backward split run may also form a delivery's belief (kChainBel):
    // its table here, the forward message it multiplies by the last entry of
    // `in` (after the G tables)
    int bel_table = -1;
    bool divide = false;            // Factor::divide: in[0] / in[1] (generic kernel, no sum)
    // build_schedule: a small bucket of a level with several kernel variants
    // runs in the level's one generic 1x1 launch (launch count, not bandwidth,
    // bounds such levels)
    bool simple = false;
    // message-sliced runs (plan_bucket_tree_chain with n_slices > 1): one step
    // of a message exchange between ranks, run by the executor, not a kernel
    // variant -- kXchgSync: all-gather of each rank's (largest true exponent,
    // exp2) of in[0] into out (2 (n_slices + 1) int64 words); kXchgPack: in[0]
    // scaled to the common exponent (read from in[1]) into out, blocks of the
    // destination ranks slowest (xchg_mode 0: in[0] already is, 1: they are
    // in[0]'s fastest variables -- a transpose); kXchgComm: collective from
    // in[0] to out (xchg_mode 0: all-to-all, 1: all-gather), out's blocks by
    // source rank slowest; kXchgUnpack: out = in[0] with the source blocks
    // moved from slowest to fastest (a transpose; xchg_mode 2: the blocks came
    // unpacked, and each is scaled to the common exponent read from in[1])
    int xchg = 0;
    int xchg_mode = 0;
    int xchg_blocks = 1;
    // stream lane (sliced two-front schedules: 0 forward messages, 1 backward
    // messages and deliveries): lanes run concurrently, ordered by the
    // cross-lane table dependencies only
    int lane = 0;
};
enum XchgKind { kXchgNone = 0, kXchgSync = 1, kXchgPack = 2, kXchgComm = 3, kXchgUnpack = 4 };
// schedule group variant of an exchange step: kXchgKeyBase + kind * 16 + mode
// (above every kernel variant key, bnpp_device.h)
constexpr int kXchgKeyBase = 1 << 24;

// Compile one bucket into a descriptor + dims-pool rows.  max_vec: 4 (fp32) / 2 (fp64).
// Returns false (with msg) on an invalid shape.
bool build_desc(const BucketSpec &b, const std::vector<int> &cards, int max_vec, BucketDesc &d,
                std::vector<int64_t> &pool, std::string *msg, bool slab_outer = true);

// Fused chain runs: is the chain kernel with this key (bnpp_device.h,
// chain_key) instantiated for this element size (k_chain_f32/f64.hip)?
bool chain_supported_f32(int key);
bool chain_supported_f64(int key);
inline bool chain_supported(int elem_bytes, int key) {
    return elem_bytes == 4 ? chain_supported_f32(key) : chain_supported_f64(key);
}

struct MsgTable {
    std::vector<int> vars;
    int64_t size = 1;
};

// Symbolic VE plan (BN::variable_elimination, model.cpp:348-446).
struct VEPlan {
    int n_src = 0;                      // tables [0, n_src) are the (conditioned) sources
    std::vector<MsgTable> msgs;         // table id = n_src + index
    std::vector<BucketSpec> buckets;    // execution order (non-decreasing level)
    int n_levels = 0;
    int result_table = -1;              // -1: result is the constant 1 (no factors)
    std::vector<int> result_vars;
    // multi-result plans (bucket-tree marginals): one table per target, -1 =
    // no table (evidence / variable in no factor); replaces result_table
    std::vector<int> results;
    std::vector<std::vector<int>> results_vars;
    std::vector<char> results_owned;    // per result: computed by this part (empty: all)
    // cards of the model followed by virtual (composite) variables the plan
    // sums in one pass; empty: the model's cards
    std::vector<int> cards_ext;
    int64_t max_table = 0;              // largest message entries
    double entries = 0;                 // sum over buckets of prod(card) over the union scope
    double elems_moved = 0;             // sum over buckets of (|inputs| + |output|): algorithmic traffic
    int width = 0;                      // largest bucket output width
    // message slicing: ranks that share the messages (1: none), this plan's
    // rank, and per result the rank bit that indexes it (-1: the result is a
    // table over its target; else a scalar, the target being a slice
    // variable whose value is that bit of the rank)
    int n_slices = 1, slice_rank = 0;
    std::vector<int> results_slice_bit;
    int n_xchg = 0;                     // message exchanges (all-to-all / all-gather)
    double xchg_elems = 0;              // entries this rank sends to other ranks
};

// canonical: lay messages out with variables sorted by elimination rank
// (earlier-eliminated slower) instead of the reference's chain order; values
// are identical, only the storage permutation differs.  Buckets with more than
// kMaxIn inputs are split into materialised pure-product prefixes exactly like
// the reference's left-to-right chain.
VEPlan plan_ve(const std::vector<int> &cards, const std::vector<View> &sources, const std::vector<int> &order,
               bool canonical, int chain_eb = 0);

// All marginals of `targets` from one two-pass bucket tree over `order`
// (Shafer-Shenoy on the VE bucket tree; replaces the N independent VEs of
// BN::marginals, model.cpp:326-334).  Forward messages are plan_ve's; each
// bucket then sends every child the product of its factors, its own incoming
// message and its other children's messages, summed down to the child's
// separator; each target's marginal (unnormalised) is the smallest belief that
// contains it summed down to the target.  results[i] -> targets[i].
// part / n_parts: marginals of targets i with i % n_parts == part only (the
// forward and backward passes are computed in full by every part).
VEPlan plan_bucket_tree(const std::vector<int> &cards, const std::vector<View> &sources,
                        const std::vector<int> &order, const std::vector<int> &targets, int part = 0,
                        int n_parts = 1);

// The same marginals in bounded memory when the bucket tree is a chain (a
// column-sweep order on a grid): forward messages are recomputed from `slots`
// checkpoints by binomial checkpointing (revolve), buckets run in program order
// (one level each) so the arena holds about slots + 5 messages.  Returns false
// (msg) when the tree is not a chain.  part / n_parts: this part owns the
// marginals of one contiguous segment of the chain; it streams the forward
// messages up to the segment, runs the backward messages (which need no
// forward message) down to it, and checkpoints only inside it.  chain_eb > 0:
// runs of consecutive buckets are fused into chain kernels for that element
// size (bnpp_device.h, ChainForm).
// n_slices = 2^b > 1: message slicing over n_slices ranks (this plan is rank
// slice_rank's).  The chain is cut into windows in which b binary variables
// stay in every separator; inside a window each rank holds the messages (and
// computes the buckets) conditioned on those variables = the bits of its
// rank, 1/n_slices of the work and memory; between windows a message is
// re-sliced by one all-to-all (kXchg* steps), at the chain's ends
// all-gathered or conditioned.  Every rank computes a partial (unnormalised)
// marginal of every target: the marginals are the sum over ranks.  lanes:
// the two-front schedule (forward and backward messages on two concurrent
// lanes, no recomputation; `slots` unused), else binomial checkpointing.
// elem_bytes: the dtype's (the kept-set size of a delivery depends on it).
bool plan_bucket_tree_chain(const std::vector<int> &cards, const std::vector<View> &sources,
                            const std::vector<int> &order, const std::vector<int> &targets, int slots,
                            int part, int n_parts, VEPlan &out, std::string *msg, int chain_eb = 0,
                            int n_slices = 1, int slice_rank = 0, bool lanes = false, int elem_bytes = 4);

// Flattened, level-ordered launch schedule over one or more plans sharing the
// same sources.  Tables: [0, n_src) sources, then every plan's messages.
// vector allocator that default-initialises (no zero fill before the
// parallel copy that fills a schedule's descriptor and pool arrays)
template <typename T>
struct DefaultInit : std::allocator<T> {
    template <typename U>
    struct rebind {
        using other = DefaultInit<U>;
    };
    DefaultInit() = default;
    template <typename U>
    DefaultInit(const DefaultInit<U> &) noexcept {}
    template <typename U>
    void construct(U *p) noexcept {
        ::new ((void *)p) U;
    }
    template <typename U, typename... A>
    void construct(U *p, A &&...a) {
        ::new ((void *)p) U(std::forward<A>(a)...);
    }
};

struct Schedule {
    int n_src = 0;
    int n_tables = 0;
    std::vector<int64_t> table_size;        // entries, per table (sources included)
    std::vector<int64_t> table_offset;      // bytes into the arena (messages only; -1 for sources)
    std::vector<BucketDesc, DefaultInit<BucketDesc>> descs;   // grouped by level, vblk_begin relative to the level
    std::vector<int64_t, DefaultInit<int64_t>> pool;
    struct Group {                          // one launch: buckets of one level and one kernel variant
        int level, variant, begin, end;
        int64_t vblocks;
        int small_elems;                    // stream kernels: LDS elements for small inputs
        int lane;                           // BucketSpec::lane (all buckets of a group share it)
    };
    std::vector<Group> groups;
    int n_levels = 0;
    std::vector<int> plan_result_table;     // per plan (-1: constant 1)
    std::vector<std::vector<int>> plan_result_vars;
    std::vector<char> plan_result_owned;     // per result: 0 = another part computes it
    std::vector<int> plan_result_slice_bit;  // per result: VEPlan::results_slice_bit (-1: none)
    int64_t arena_bytes = 0;
    double entries = 0;
    double elems_moved = 0;
    int width = 0;
    int n_lanes = 1;                        // concurrent stream lanes (Group::lane)
};

// Peak bytes of live messages when the plan runs level by level (arena estimate).
int64_t plan_peak_bytes(const VEPlan &p, int elem_bytes);
// Bytes of the arena build_schedule allocates for this plan alone (the same
// best-fit allocator, so fragmentation included).
int64_t plan_arena_bytes(const VEPlan &p, int elem_bytes);

// arena_cap: the most device memory the schedule's arena may take; several
// plans get arenas of their own (placed in parallel) when their sum fits it,
// else one shared arena
bool build_schedule(const std::vector<const VEPlan *> &plans, const std::vector<int> &cards,
                    const std::vector<int64_t> &src_sizes, int elem_bytes, int max_vec, Schedule &s,
                    std::string *msg, int64_t arena_cap = INT64_MAX);

}  // namespace bnpp
