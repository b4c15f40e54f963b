// extern "C" boundary (include/bnpp.h).  No exception crosses it: every entry
// point catches, records bnpp_last_error() and returns a status code.
#include "../../include/bnpp.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <utility>
#include <thread>
#include <unistd.h>
#include <vector>

#include "model_io.hpp"
#include "order.hpp"
#include "plan.hpp"
#include "runtime.hpp"

using namespace bnpp;

constexpr int kTimingPhases = 9;

struct bnpp_ctx {
    Context c;
    std::mutex cache_mu;            // one one-shot call at a time uses c.arena_cache
    // uploaded sources of recent models, per dtype (a model is read-only after
    // creation, so its pre-scaled tables stay valid): a repeated call skips
    // the host pre-scaling and the copy (1.5 of Mildew's 2.2-ms PR).  Keyed on
    // the model's uid, never reused; most recent last
    struct Src {
        uint64_t uid;
        int dtype;
        std::shared_ptr<DeviceSources> s;
    };
    std::mutex src_mu;
    std::vector<Src> srcs;
    // the last one-shot partition / marginals job (plan, schedule, device
    // program on the cached arena), relaunched as is by an identical call
    // (same model, evidence, order, targets, dtype, part, memory budget and
    // BNPP_* environment): a serving caller's repeated query skips ordering
    // and planning.  Guarded by cache_mu, like the arena it runs in
    bnpp_job *job_cached = nullptr;
    uint64_t job_key = 0;
    int64_t job_budget = 0;             // the memory budget the cached job was planned under
};
// live contexts: bnpp_model_free releases what they cache for the model
std::mutex g_ctxs_mu;
std::vector<bnpp_ctx *> g_ctxs;

struct bnpp_model {
    ModelData d;
    uint64_t uid = next_uid();
    static uint64_t next_uid() {
        static std::atomic<uint64_t> n{1};
        return n++;
    }
};
struct bnpp_job {
    bnpp_ctx *ctx = nullptr;
    int kind = 0;
    uint64_t model_uid = 0;            // the model it was planned for (bnpp_model_free evicts a cached job of it)
    std::shared_ptr<DeviceSources> src;
    Program pg;
    std::vector<int> targets;
    std::vector<int> ev_val;          // per variable, -1 = no evidence
    std::vector<int> cards;
    int n_slices = 1, slice_rank = 0;  // message-sliced bucket tree (bnpp_marginals_tree_sliced)
    double stats[10] = {0};            // bnpp_job_stats [0..8), then n_xchg, exchange bytes sent
};

namespace {

thread_local std::string g_err;
// phase split of this thread's last partition / marginals call (bnpp_last_timing)
thread_local double g_timing[kTimingPhases] = {0};

int set_err(int status, const std::string &msg) {
    g_err = msg;
    return status;
}
int from_ctx(bnpp_ctx *ctx, int rc) {
    if (rc == 0) return BNPP_OK;
    g_err = ctx->c.last_error;
    return rc == -3 ? BNPP_ERR_OOM : rc == -1 ? BNPP_ERR_INVALID : BNPP_ERR_HIP;
}
hipStream_t pick_stream(bnpp_ctx *ctx, void *stream) {
    return stream ? static_cast<hipStream_t>(stream) : ctx->c.stream;
}
double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define BNPP_GUARD_BEGIN try {
#define BNPP_GUARD_END                                                       \
    }                                                                        \
    catch (const std::bad_alloc &) {                                         \
        return set_err(BNPP_ERR_OOM, "host out of memory");                  \
    }                                                                        \
    catch (const std::exception &e) {                                        \
        return set_err(BNPP_ERR_INVALID, e.what());                          \
    }                                                                        \
    catch (...) {                                                            \
        return set_err(BNPP_ERR_INVALID, "unknown error");                   \
    }

// every id in [0, n_cards) with a positive cardinality, no repeats
bool valid_scope(int ndims, const int *vars, const int *cards, int n_cards) {
    if (ndims < 0 || (ndims > 0 && !vars)) return false;
    for (int i = 0; i < ndims; ++i) {
        if (vars[i] < 0 || vars[i] >= n_cards || cards[vars[i]] < 1) return false;
        for (int j = 0; j < i; ++j)
            if (vars[j] == vars[i]) return false;
    }
    return true;
}

int max_vec_for(int dtype) { return dtype == BNPP_F32 ? 4 : 2; }

// Launch one bucket with the descriptor in the kernel-argument segment.
int run_single(bnpp_ctx *ctx, void *stream, int dtype, const std::vector<int> &cards, const BucketSpec &b,
               const std::vector<const void *> &in_ptrs, void *out) {
    if (dtype != BNPP_F32 && dtype != BNPP_F64) return set_err(BNPP_ERR_INVALID, "dtype must be BNPP_F64 or BNPP_F32");
    SingleArgs a;
    std::memset(&a, 0, sizeof a);
    std::vector<int64_t> pool;
    std::string msg;
    if (!build_desc(b, cards, max_vec_for(dtype), a.d, pool, &msg, false)) return set_err(BNPP_ERR_INVALID, msg);
    if (pool.size() > (size_t)kMaxPool)
        return set_err(BNPP_ERR_UNSUPPORTED, "too many non-mergeable output dims for a single-op call");
    std::copy(pool.begin(), pool.end(), a.pool);
    a.d.dim_off = 0;
    for (size_t i = 0; i < in_ptrs.size(); ++i) {
        a.meta[i].ptr = const_cast<void *>(in_ptrs[i]);
        // entries the view can reach (the launcher picks 32-bit offsets by it)
        a.meta[i].size = view_span(b.in[i], cards);
    }
    // BNPP_NO_O32=1 (tests): claim a span that rules out the 32-bit-offset kernels
    if (const char *no32 = std::getenv("BNPP_NO_O32"); no32 && *no32 == '1')
        for (size_t i = 0; i < in_ptrs.size(); ++i) a.meta[i].size = (int64_t)1 << 40;
    a.meta[in_ptrs.size()].ptr = out;
    if (a.d.big >= 0) {
        const int eb = dtype == BNPP_F32 ? 4 : 8;
        a.big_ptr = static_cast<const unsigned char *>(in_ptrs[a.d.big]) + a.d.in_base[a.d.big] * eb;
        a.big_es = a.d.elim_stride[a.d.big];
    }
    hipError_t e = hipSetDevice(ctx->c.device);
    if (e == hipSuccess) e = launch_single(dtype == BNPP_F32, a, ctx->c.max_grid, pick_stream(ctx, stream));
    if (e != hipSuccess) return set_err(BNPP_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return BNPP_OK;
}

// Factor::_partition of a single-op call (seqsum.hip), enqueued after the op
// on the same stream: the terms of the inputs' chain product (or in[0] /
// in[1]) over `dims` -- the reference's output scope order, last fastest --
// with elim_var's values inner, added one at a time in that order.
// checked before the op is launched, so an unsupported out_sum never leaves
// an op that ran behind an error status
int seq_sum_supported(const double *out_sum, size_t n_dims, size_t n_in) {
    if (out_sum && (n_dims > (size_t)kSeqMaxDims || n_in > (size_t)kMaxIn))
        return set_err(BNPP_ERR_UNSUPPORTED, "out_sum: at most 32 output variables");
    return BNPP_OK;
}

int run_seq_sum(bnpp_ctx *ctx, void *stream, int dtype, const std::vector<int> &cards, const std::vector<View> &in,
                const std::vector<const void *> &ptrs, const std::vector<int> &dims, int elim_var, bool divide,
                double *out_sum) {
    if (!out_sum) return BNPP_OK;
    if (int rc = seq_sum_supported(out_sum, dims.size(), in.size())) return rc;
    SeqSumArgs a;
    std::memset(&a, 0, sizeof a);
    const int64_t eb = dtype == BNPP_F32 ? 4 : 8;
    bool has_elim = false;
    for (const View &v : in)
        for (int x : v.vars) has_elim = has_elim || (elim_var >= 0 && x == elim_var);
    a.k = has_elim ? cards[elim_var] : 1;
    a.n_terms = a.k;
    for (int x : dims) a.n_terms = sat_mul(a.n_terms, cards[x]);
    a.n_in = (int)in.size();
    a.n_dims = (int)dims.size();
    a.divide = divide ? 1 : 0;
    a.out = out_sum;
    for (size_t d = 0; d < dims.size(); ++d) a.card[d] = cards[dims[d]];
    for (size_t n = 0; n < in.size(); ++n) {
        a.in[n] = static_cast<const unsigned char *>(ptrs[n]) + in[n].base * eb;
        for (size_t j = 0; j < in[n].vars.size(); ++j) {
            const int x = in[n].vars[j];
            if (has_elim && x == elim_var) a.stride[n][kSeqMaxDims] = in[n].strides[j];
            for (size_t d = 0; d < dims.size(); ++d)
                if (dims[d] == x) a.stride[n][d] = in[n].strides[j];
        }
    }
    hipError_t e = hipSetDevice(ctx->c.device);
    if (e == hipSuccess) e = launch_seq_sum(dtype == BNPP_F32, a, pick_stream(ctx, stream));
    if (e != hipSuccess) return set_err(BNPP_ERR_HIP, std::string("partition sum launch: ") + hipGetErrorString(e));
    return BNPP_OK;
}

// evidence as a per-variable array (-1: none); validates ids and values
bool evidence_array(const ModelData &d, int n_ev, const int *ev_vars, const int *ev_vals, std::vector<int> &ev,
                    std::string &msg) {
    ev.assign(d.cards.size(), -1);
    if (n_ev < 0 || (n_ev > 0 && (!ev_vars || !ev_vals))) {
        msg = "bad evidence arrays";
        return false;
    }
    for (int i = 0; i < n_ev; ++i) {
        int v = ev_vars[i], x = ev_vals[i];
        if (v < 0 || v >= (int)d.cards.size() || x < 0 || x >= d.cards[v]) {
            msg = "evidence out of range";
            return false;
        }
        ev[v] = x;                          // evidence[id] = val (io.cpp:171)
    }
    return true;
}

std::vector<std::vector<int>> conditioned_scopes(const ModelData &d, const std::vector<int> &ev) {
    std::vector<std::vector<int>> sc(d.scopes.size());
    for (size_t f = 0; f < d.scopes.size(); ++f)
        for (int v : d.scopes[f])
            if (ev[v] < 0) sc[f].push_back(v);
    return sc;
}

std::vector<View> source_views(const ModelData &d, const std::vector<int> &ev) {
    std::vector<View> views;
    for (size_t f = 0; f < d.scopes.size(); ++f) views.push_back(conditioned_view((int)f, d.scopes[f], d.cards, ev));
    return views;
}

// Checkpoint-slot counts chosen by the bucket-tree search below, keyed on
// everything the plan's arena size depends on except the budget.  The search evaluates ~6 chain
// plans (≈60 ms on the 32x32 grid); a repeated MAR call on the same model then
// builds one plan.
// An entry holds for every budget in [need_ok, need_fail): the arena need of
// the chosen count and of the smallest count found not to fit.
struct SlotMemo {
    struct Entry {
        uint64_t key;
        int slots;
        int64_t need_ok, need_fail;
    };
    std::mutex mu;
    std::vector<Entry> entries;
};
SlotMemo &slot_memo() {
    static SlotMemo m;
    return m;
}
// the plan-changing switches (kPlanKnobs); a tuning build (BNPP_TUNING_KNOBS)
// keys on the whole BNPP_* environment, its knobs included
template <typename Mix>
void mix_plan_knobs(Mix &&mix) {
#ifdef BNPP_TUNING_KNOBS
    for (char **e = environ; e && *e; ++e)
        if (std::strncmp(*e, "BNPP_", 5) == 0)
            for (const char *c = *e; *c; ++c) mix((unsigned char)*c);
#else
    for (const char *k : kPlanKnobs) {
        const char *v = std::getenv(k);
        mix(0x9e37u);
        for (const char *c = v ? v : ""; *c; ++c) mix((unsigned char)*c);
    }
#endif
}

uint64_t slot_key(const std::vector<int> &cards, const std::vector<std::vector<int>> &scopes, const std::vector<int> &ord,
                  const std::vector<int> &targets, int eb, int chain_eb, int part, int n_parts, int n_slices) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
    auto mixv = [&](const std::vector<int> &v) {
        mix(v.size());
        for (int x : v) mix((uint32_t)x);
    };
    mixv(cards);
    mix(scopes.size());
    for (const auto &sc : scopes) mixv(sc);
    mixv(ord);
    mixv(targets);
    mix((uint64_t)eb);                    // the dtype: arena bytes scale with it
    mix((uint64_t)chain_eb);              // fused runs on/off change the plan
    mix((uint64_t)part);
    mix((uint64_t)n_parts);
    mix((uint64_t)n_slices);              // the slice rank does not change the arena need
    mix_plan_knobs(mix);                  // switches that change the plan and its arena need
    return h;
}

// Build the VE plans for a job: kind 0 = partition, kind 1 = marginals of targets.
int build_plans(const ModelData &d, const std::vector<int> &ev, int kind, int heuristic, const int *order,
                int n_order, const std::vector<int> &targets, std::vector<VEPlan> &plans, int &max_width,
                int64_t budget, int eb, int part = 0, int n_parts = 1, int n_slices = 1, int slice_rank = 0) {
    const int nv = (int)d.cards.size();
    auto scopes = conditioned_scopes(d, ev);
    auto views = source_views(d, ev);
    max_width = 0;
    const char *nc = std::getenv("BNPP_NO_CHAIN");                 // A/B: one launch per bucket
    const int chain_eb = nc && *nc == '1' ? 0 : eb;
    if (heuristic < BNPP_ORDER_GIVEN || heuristic > BNPP_MIN_DEGREE)
        return set_err(BNPP_ERR_INVALID, "unknown heuristic");
    if (kind == 2) {                                     // caller-chosen variables
        std::vector<int> vars(order, order + n_order), ord;
        for (int v : vars)
            if (v < 0 || v >= nv) return set_err(BNPP_ERR_INVALID, "bad variable");
        max_width = elimination_order(nv, d.cards, scopes, vars, (Heuristic)heuristic, ord);
        plans.push_back(plan_ve(d.cards, views, ord, true));
    } else if (kind == 0) {
        std::vector<int> vars, ord;
        if (order) {
            std::vector<char> seen(nv, 0);
            for (int i = 0; i < n_order; ++i) {
                int v = order[i];
                if (v < 0 || v >= nv || seen[v]) return set_err(BNPP_ERR_INVALID, "bad explicit order");
                seen[v] = 1;
                if (ev[v] < 0) vars.push_back(v);
            }
            ord = vars;
            max_width = order_width(nv, scopes, ord);
        } else {
            for (int v = 0; v < nv; ++v)
                if (ev[v] < 0) vars.push_back(v);        // model.cpp:277-282
            max_width = elimination_order(nv, d.cards, scopes, vars, (Heuristic)heuristic, ord);
        }
        plans.push_back(plan_ve(d.cards, views, ord, true, chain_eb));
    } else if (kind == 3) {
        // all marginals from one two-pass bucket tree over the PR ordering
        std::vector<int> vars, ord;
        if (order) {
            std::vector<char> seen(nv, 0);
            for (int i = 0; i < n_order; ++i) {
                int v = order[i];
                if (v < 0 || v >= nv || seen[v]) return set_err(BNPP_ERR_INVALID, "bad explicit order");
                seen[v] = 1;
                if (ev[v] < 0) vars.push_back(v);
            }
            for (int v = 0; v < nv; ++v)
                if (!seen[v] && ev[v] < 0) return set_err(BNPP_ERR_INVALID, "explicit order must cover every non-evidence variable");
            ord = vars;
            max_width = order_width(nv, scopes, ord);
        } else {
            for (int v = 0; v < nv; ++v)
                if (ev[v] < 0) vars.push_back(v);
            max_width = elimination_order(nv, d.cards, scopes, vars, (Heuristic)heuristic, ord);
        }
        const bool tt = std::getenv("BNPP_TIMING") != nullptr;
        double tq = now_ms();
        auto need = [&](const VEPlan &p) { return sat_add(plan_arena_bytes(p, eb), (int64_t)p.buckets.size() * 512); };
        std::string msg;
        const char *force = std::getenv("BNPP_TREE_SLOTS");     // testing / tuning: chain mode, fixed slots
        if (force && std::atoi(force) > 0) {
            VEPlan cp;
            if (!plan_bucket_tree_chain(d.cards, views, ord, targets, std::atoi(force), part, n_parts, cp, &msg, chain_eb,
                                        n_slices, slice_rank, false, eb))
                return set_err(BNPP_ERR_UNSUPPORTED, msg);
            plans.push_back(std::move(cp));
            return BNPP_OK;
        }
        // plans the search leaves behind (the whole tree when it does not fit,
        // unused probes: ~2 ms each to free) are freed off the call's path
        std::vector<VEPlan> dead;
        struct Burial {
            std::vector<VEPlan> &d;
            ~Burial() {
                if (!d.empty()) std::thread([x = std::move(d)]() mutable { x.clear(); }).detach();
            }
        } burial{dead};
        // when the forward messages do not all fit, they are recomputed from
        // checkpoints (chain-shaped trees), with as many checkpoint slots as fit.
        // The slot search needs only the order, so its memo's plan or its first
        // probe round is planned beside the whole tree, which is used if it fits
        int lo = 1, hi = n_slices > 1 ? 256 : 64, best_s = 0;
        VEPlan best;
        const uint64_t key = slot_key(d.cards, scopes, ord, targets, eb, chain_eb, part, n_parts, n_slices);
        int memo_s = 0;
        {
            std::lock_guard<std::mutex> g(slot_memo().mu);
            for (const SlotMemo::Entry &e : slot_memo().entries)
                if (e.key == key && e.need_ok <= budget && budget < e.need_fail) memo_s = e.slots;
        }
        // first probe round: eight consecutive counts ending at the estimate
        // budget / largest message (a checkpoint slot holds one message; the
        // answer sits a few below it), so that one round usually brackets it
        int first_hi = 0;
        if (n_slices == 1 && memo_s == 0) {
            const double est = (double)budget / (order_max_table(nv, d.cards, scopes, ord) * eb);
            if (est >= 1 && est < hi) first_hi = (int)est;
        }
        std::vector<int> pre;                                // planned beside the whole tree
        if (n_slices == 1 && memo_s > 0) {
            pre.push_back(memo_s);
        } else if (first_hi > 0) {
            const int k = std::min(8, first_hi);             // first_hi - k + 1 .. first_hi (>= 1)
            for (int i = 0; i < k; ++i) pre.push_back(first_hi - (k - 1) + i);
            first_hi = 0;
        }
        const int npre = (int)pre.size();
        std::vector<VEPlan> pre_cps(npre);
        std::vector<int64_t> pre_nb(npre, 0);
        std::vector<char> pre_ok(npre, 0);
        std::vector<std::string> pre_msgs(npre);
        VEPlan tree;
        int64_t tree_need = 0;
        parallel_for((int64_t)npre + 1, [&](int64_t i) {
            if (i == 0) {
                tree = plan_bucket_tree(d.cards, views, ord, targets, part, n_parts);
                tree_need = need(tree);
                return;
            }
            pre_ok[i - 1] = plan_bucket_tree_chain(d.cards, views, ord, targets, pre[i - 1], part, n_parts, pre_cps[i - 1],
                                                   &pre_msgs[i - 1], chain_eb, n_slices, slice_rank, false, eb) ? 1 : 0;
            if (pre_ok[i - 1]) pre_nb[i - 1] = need(pre_cps[i - 1]);
        });
        if (tt) std::fprintf(stderr, "[bnpp] bucket tree: whole tree beside %d checkpointed plans %.1f ms\n", npre, now_ms() - tq);
        if (tree_need <= budget && n_parts == 1 && n_slices == 1) {
            plans.push_back(std::move(tree));
            for (VEPlan &c : pre_cps) dead.push_back(std::move(c));
            return BNPP_OK;
        }
        dead.push_back(std::move(tree));
        // sliced runs: the two-front schedule (two concurrent lanes, no
        // recomputation) when its arena fits, else checkpointing on one lane
        if (n_slices > 1 && !(tuning_knob("BNPP_SLICE_LANES") && *tuning_knob("BNPP_SLICE_LANES") == '0')) {
            VEPlan cp;
            if (plan_bucket_tree_chain(d.cards, views, ord, targets, 1, part, n_parts, cp, &msg, chain_eb, n_slices,
                                       slice_rank, true, eb)) {
                if (need(cp) <= budget) {
                    plans.push_back(std::move(cp));
                    return BNPP_OK;
                }
            } else {
                return set_err(BNPP_ERR_UNSUPPORTED, msg);
            }
        }
        if (memo_s > 0) {                                    // the search would land on the same count
            if (n_slices == 1) {
                if (pre_ok[0] && pre_nb[0] <= budget) {
                    best_s = memo_s;
                    best = std::move(pre_cps[0]);
                    lo = hi + 1;
                } else {
                    // the memo's count no longer fits this budget: search below
                    // it, the first round ending at the budget's estimate
                    if (pre_ok[0]) hi = std::min(hi, memo_s - 1);
                    const double est = (double)budget / (order_max_table(nv, d.cards, scopes, ord) * eb);
                    if (est >= 1 && est < hi) first_hi = (int)est;
                }
            } else {
                VEPlan cp;
                if (plan_bucket_tree_chain(d.cards, views, ord, targets, memo_s, part, n_parts, cp, &msg, chain_eb,
                                           n_slices, slice_rank, false, eb) &&
                    need(cp) <= budget) {
                    best_s = memo_s;
                    best = std::move(cp);
                    lo = hi + 1;
                }
            }
        }
        int64_t need_ok = 0, need_fail = INT64_MAX;
        bool exact = true;                                   // every probe planned: the bracket is valid
        // one probe round's results (probes ascending): the need grows with the slot count
        auto absorb = [&](const std::vector<int> &probe, std::vector<VEPlan> &cps, const std::vector<char> &planned,
                          const std::vector<int64_t> &nb, const std::vector<std::string> &msgs) {
            int new_lo = lo, new_hi = hi;
            for (size_t i = 0; i < probe.size(); ++i) {
                if (!planned[i]) {                           // as a bisection that stops at its first failure
                    exact = false;
                    if (msg.empty()) msg = msgs[i];
                    new_hi = std::min(new_hi, probe[i] - 1);
                    break;
                }
                if (nb[i] <= budget) {
                    if (probe[i] > best_s) {
                        if (best_s > 0) dead.push_back(std::move(best));
                        best_s = probe[i];
                        best = std::move(cps[i]);
                    }
                    need_ok = std::max(need_ok, nb[i]);      // valid for budgets >= every fitting probe's need
                    new_lo = std::max(new_lo, probe[i] + 1);
                } else {
                    need_fail = std::min(need_fail, nb[i]);
                    new_hi = std::min(new_hi, probe[i] - 1);
                    break;                                   // larger probes need more still
                }
            }
            lo = new_lo;
            hi = new_hi;
            for (VEPlan &c : cps) dead.push_back(std::move(c));
        };
        if (lo <= hi && memo_s == 0 && npre > 0) absorb(pre, pre_cps, pre_ok, pre_nb, pre_msgs);
        else
            for (VEPlan &c : pre_cps) dead.push_back(std::move(c));
        // further rounds: a k-ary search, up to 8 probes planned in parallel per
        // round (two rounds for 64 counts instead of six bisection steps)
        while (lo <= hi && exact) {
            tq = now_ms();
            const int m = hi - lo + 1;
            int n = std::min(8, m);
            std::vector<int> probe(n);                       // ascending, inside [lo, hi]
            for (int i = 0; i < n; ++i) probe[i] = m <= 8 ? lo + i : lo + (int)((int64_t)m * (i + 1) / (n + 1));
            if (first_hi > 0 && m > 8) {                     // (a memo plan that no longer fit)
                const int k = std::min(n, first_hi);
                probe.resize(k);
                n = k;
                for (int i = 0; i < k; ++i) probe[i] = first_hi - (k - 1) + i;
                first_hi = 0;
            }
            std::vector<VEPlan> cps(n);
            std::vector<int64_t> nb(n, 0);
            std::vector<char> planned(n, 0);
            std::vector<std::string> msgs(n);
            parallel_for((int64_t)n, [&](int64_t i) {
                planned[i] = plan_bucket_tree_chain(d.cards, views, ord, targets, probe[i], part, n_parts, cps[i],
                                                    &msgs[i], chain_eb, n_slices, slice_rank, false, eb) ? 1 : 0;
                if (planned[i]) nb[i] = need(cps[i]);
            });
            absorb(probe, cps, planned, nb, msgs);
            if (tt) std::fprintf(stderr, "[bnpp] bucket tree: %d slot probes %.1f ms\n", n, now_ms() - tq);
        }
        if (best_s > 0) {
            if (best_s != memo_s && exact) {
                std::lock_guard<std::mutex> g(slot_memo().mu);
                auto &en = slot_memo().entries;
                if (en.size() >= 64) en.erase(en.begin());
                en.push_back({key, best_s, need_ok, need_fail});
            }
            if (tt) std::fprintf(stderr, "[bnpp] bucket tree: %d checkpoint slots\n", best_s);
            plans.push_back(std::move(best));
        } else if (n_slices > 1) {
            return set_err(msg.empty() ? BNPP_ERR_OOM : BNPP_ERR_UNSUPPORTED,
                           msg.empty() ? "sliced bucket tree: no checkpoint count fits the memory budget" : msg);
        } else {
            // no checkpoint count fits (or the tree is not a chain): the whole
            // tree, which plan_schedules reports as over the budget
            plans.push_back(std::move(dead.front()));
            dead.erase(dead.begin());
        }
    } else {
        // one independent VE per target (model.cpp:326-334), planned in parallel
        plans.resize(targets.size());
        std::vector<int> widths(targets.size(), 0);
        std::vector<double> to(targets.size()), tp(targets.size());
        const double T0 = now_ms();
        parallel_for((int64_t)targets.size(), [&](int64_t i) {
            const int t = targets[i];
            std::vector<int> vars, ord;
            for (int v = 0; v < nv; ++v)                 // model.cpp:327-332 (evidence vars are no-ops)
                if (v != t && ev[v] < 0) vars.push_back(v);
            double a = now_ms();
            widths[i] = elimination_order(nv, d.cards, scopes, vars, (Heuristic)heuristic, ord);
            double b = now_ms();
            plans[i] = plan_ve(d.cards, views, ord, true);
            to[i] = b - a; tp[i] = now_ms() - b;
        });
        if (std::getenv("BNPP_TIMING")) {
            double so = 0, sp = 0;
            for (size_t i = 0; i < to.size(); ++i) {
                so += to[i];
                sp += tp[i];
            }
            std::fprintf(stderr, "[bnpp] per-target plans: wall %.1f ms, ordering %.1f ms, plan_ve %.1f ms (thread sums)\n",
                         now_ms() - T0, so, sp);
        }
        for (int w : widths) max_width = std::max(max_width, w);
    }
    return BNPP_OK;
}

// Analysis aid (BNPP_ARENA_PROFILE=path, host only): for every 1-GiB chunk of
// the arena, the algorithmic bytes the schedule has moved before its first
// launch touching the chunk -- how early a cold call needs each part of its
// arena mapped.  One line per chunk: "chunk cum_bytes group".
void arena_profile(const Schedule &s, int eb, const char *path) {
    FILE *f = std::fopen(path, "w");
    if (!f) return;
    const int64_t G = (int64_t)1 << 30;
    const int64_t nch = (s.arena_bytes + G - 1) / G;
    std::vector<double> first(nch, -1);
    std::vector<int> first_g(nch, -1);
    double cum = 0;
    for (size_t gi = 0; gi < s.groups.size(); ++gi) {
        const Schedule::Group &g = s.groups[gi];
        double moved = 0;
        for (int k = g.begin; k < g.end; ++k) {
            const BucketDesc &d = s.descs[k];
            int tabs[kMaxDescIn + 2];
            int nt = 0;
            const int n_read = d.n_in + ((d.flags & kChainBel) ? 1 : 0);
            for (int i = 0; i < n_read && i < kMaxDescIn; ++i) tabs[nt++] = d.in_table[i];
            tabs[nt++] = d.out_table;
            if (d.flags & kChainBel) tabs[nt++] = d.aux_out;
            for (int i = 0; i < nt; ++i) {
                const int t = tabs[i];
                if (t < 0) continue;
                moved += (double)s.table_size[t] * eb;
                if (t < (int)s.table_offset.size() && s.table_offset[t] >= 0) {
                    const int64_t a = s.table_offset[t] / G, b = (s.table_offset[t] + s.table_size[t] * eb - 1) / G;
                    for (int64_t c = a; c <= b && c < nch; ++c)
                        if (first[c] < 0) {
                            first[c] = cum;
                            first_g[c] = (int)gi;
                        }
                }
            }
        }
        cum += moved;
    }
    std::fprintf(f, "# arena %lld bytes, %zu groups, %.6g bytes moved\n", (long long)s.arena_bytes, s.groups.size(), cum);
    for (int64_t c = 0; c < nch; ++c) std::fprintf(f, "%lld %.6g %d\n", (long long)c, first[c], first_g[c]);
    std::fclose(f);
}

// Plans -> schedules.  MAR targets are split into batches whose estimated
// arenas fit `budget` bytes; a batch runs as one level-aligned schedule.
int plan_schedules(const ModelData &d, const std::vector<int> &ev, int kind, int heuristic, const int *order,
                   int n_order, const std::vector<int> &targets, int dtype, int64_t budget,
                   std::vector<Schedule> &out, double *stats, int part = 0, int n_parts = 1, int n_slices = 1,
                   int slice_rank = 0) {
    std::vector<VEPlan> plans;
    int width = 0;
    const bool timing = std::getenv("BNPP_TIMING") != nullptr;
    double t0 = now_ms();
    const int eb = dtype == BNPP_F32 ? 4 : 8;
    int rc = build_plans(d, ev, kind, heuristic, order, n_order, targets, plans, width, budget, eb, part, n_parts,
                         n_slices, slice_rank);
    if (rc) return rc;
    if (timing) std::fprintf(stderr, "[bnpp] plans %.1f ms\n", now_ms() - t0);
    std::vector<int64_t> src_sizes;
    for (auto &v : d.values) src_sizes.push_back((int64_t)v.size());
    std::vector<std::vector<const VEPlan *>> batches(1);
    std::vector<int64_t> needs(plans.size());
    parallel_for((int64_t)plans.size(), [&](int64_t i) {
        const VEPlan &p = plans[i];
        needs[i] = sat_add(kind == 3 ? plan_arena_bytes(p, eb) : plan_peak_bytes(p, eb), (int64_t)p.buckets.size() * 512);
    });
    int64_t acc = 0;
    for (size_t i = 0; i < plans.size(); ++i) {
        const VEPlan &p = plans[i];
        const int64_t need = needs[i];
        if (kind == 3 && need > budget) {
            char m[256];
            std::snprintf(m, sizeof m, "bucket-tree marginals need %.2f GB, budget %.2f GB: the tree is not a "
                          "chain or no checkpoint count fits (per-target marginals or a narrower order)", need / 1e9, budget / 1e9);
            return set_err(BNPP_ERR_OOM, m);
        }
        if (!batches.back().empty() && sat_add(acc, need) > budget) {
            batches.emplace_back();
            acc = 0;
        }
        batches.back().push_back(&p);
        acc = sat_add(acc, need);
    }
    out.clear();
    std::string msg;
    double entries = 0, moved = 0, arena = 0, levels = 0, buckets = 0;
    for (auto &bp : batches) {
        Schedule s;
        const double tb = now_ms();
        if (!build_schedule(bp, d.cards, src_sizes, eb, max_vec_for(dtype), s, &msg, budget))
            return set_err(s.arena_bytes >= kSatMax ? BNPP_ERR_OOM : BNPP_ERR_INVALID, msg);
        if (timing) std::fprintf(stderr, "[bnpp] build_schedule call %.1f ms\n", now_ms() - tb);
        entries += s.entries;
        moved += s.elems_moved;
        arena = std::max(arena, (double)s.arena_bytes);
        if (timing) {
            int64_t ideal = 0;
            for (const VEPlan *pp : bp) ideal += plan_peak_bytes(*pp, eb);
            std::fprintf(stderr, "[bnpp] schedule: %zu buckets, %zu launches, ideal live peak %.2f GB, arena %.2f GB\n",
                         s.descs.size(), s.groups.size(), ideal / 1e9, s.arena_bytes / 1e9);
        }
        levels += s.n_levels;
        buckets += (double)s.descs.size();
        if (const char *prof = std::getenv("BNPP_ARENA_PROFILE")) arena_profile(s, eb, prof);
        out.push_back(std::move(s));
    }
    if (timing) std::fprintf(stderr, "[bnpp] schedules %.1f ms total\n", now_ms() - t0);
    stats[0] = entries;
    stats[1] = arena;
    stats[2] = levels;
    stats[3] = buckets;
    stats[4] = width;
    int64_t mx = 0;
    for (auto &p : plans) mx = std::max(mx, p.max_table);
    stats[5] = (double)mx;
    stats[6] = moved * eb;
    stats[7] = (double)out.size();
    double nx = 0, xe = 0;
    for (auto &p : plans) {
        nx += p.n_xchg;
        xe += p.xchg_elems;
    }
    stats[8] = nx;
    stats[9] = xe * eb;
    // the plans hold millions of small vectors (per-target MAR: one plan per
    // target, ~25 ms to free): a background thread frees them while the call
    // goes on to upload and launch (plans of one bucket tree: here)
    const double tf = now_ms();
    if (plans.size() > 1) {
        std::thread([dead = std::move(plans)]() mutable {
            parallel_for((int64_t)dead.size(), [&](int64_t i) { VEPlan d = std::move(dead[i]); });
        }).detach();
    } else {
        plans.clear();
    }
    if (timing) std::fprintf(stderr, "[bnpp] plans freed in %.1f ms\n", now_ms() - tf);
    return BNPP_OK;
}

// use_cache: the caller holds ctx->cache_mu and may reuse the cached arena, so
// its bytes count as free; a call that could not take the lock must not plan
// against memory another call is holding
int64_t memory_budget(bnpp_ctx *ctx, bool use_cache = false) {
    if (const char *e = std::getenv("BNPP_MEM_BUDGET_GB")) return (int64_t)(std::atof(e) * 1e9);
    if (ctx) {
        size_t fr = 0, tot = 0;
        (void)hipSetDevice(ctx->c.device);
        // 92 % of the free memory: an idle MI355X reports ~303 GB free, so
        // the 32x32 bucket tree plans 275-GB arenas -- fp64 five checkpoint
        // slots instead of four (30.2 against 31.9 TB), fp32 thirteen instead
        // of eleven (12.1 against 12.3 TB); 85 % until round 6
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 0)
            return (int64_t)((fr + (use_cache ? ctx->c.arena_cache_bytes : 0)) * 0.92);
    }
    return (int64_t)64e9;
}

// the model's sources on the device in `dtype`, from the context's cache or
// uploaded now (and cached: at most 8 models, 512 MB)
int cached_sources(bnpp_ctx *ctx, const bnpp_model *m, int dtype, std::shared_ptr<DeviceSources> &out) {
    {
        std::lock_guard<std::mutex> g(ctx->src_mu);
        for (size_t i = 0; i < ctx->srcs.size(); ++i)
            if (ctx->srcs[i].uid == m->uid && ctx->srcs[i].dtype == dtype) {
                bnpp_ctx::Src e = ctx->srcs[i];
                ctx->srcs.erase(ctx->srcs.begin() + i);
                ctx->srcs.push_back(e);
                out = e.s;
                return BNPP_OK;
            }
    }
    Context *c = &ctx->c;
    std::shared_ptr<DeviceSources> s(new DeviceSources, [c](DeviceSources *p) {
        free_sources(*c, *p);
        delete p;
    });
    int rc = upload_sources(ctx->c, m->d.values, dtype == BNPP_F32 ? kF32 : kF64, *s);
    if (rc) return from_ctx(ctx, rc);
    out = s;
    std::lock_guard<std::mutex> g(ctx->src_mu);
    ctx->srcs.push_back({m->uid, dtype, s});
    size_t bytes = 0;
    for (const auto &e : ctx->srcs) bytes += e.s->buf_cap;
    while (ctx->srcs.size() > 8 || (ctx->srcs.size() > 1 && bytes > ((size_t)512 << 20))) {
        bytes -= ctx->srcs.front().s->buf_cap;
        ctx->srcs.erase(ctx->srcs.begin());
    }
    return BNPP_OK;
}

void evict_cached_job(bnpp_ctx *ctx);

int create_job(bnpp_ctx *ctx, const bnpp_model *m, int kind, int n_ev, const int *ev_vars, const int *ev_vals,
               int heuristic, const int *order, int n_order, int n_targets, const int *targets, int dtype,
               std::unique_ptr<bnpp_job> &job, int part = 0, int n_parts = 1, bool use_cache = false, int n_slices = 1,
               int slice_rank = 0, int64_t budget = 0) {
    if (!ctx || !m) return set_err(BNPP_ERR_INVALID, "null context or model");
    if (dtype != BNPP_F32 && dtype != BNPP_F64) return set_err(BNPP_ERR_INVALID, "bad dtype");
    const ModelData &d = m->d;
    job.reset(new bnpp_job);
    job->ctx = ctx;
    job->kind = kind;
    job->model_uid = m->uid;
    job->cards = d.cards;
    job->n_slices = n_slices;
    job->slice_rank = slice_rank;
    std::string msg;
    if (!evidence_array(d, n_ev, ev_vars, ev_vals, job->ev_val, msg)) return set_err(BNPP_ERR_INVALID, msg);
    if (kind == 1 || kind == 3) {
        if (targets) {
            for (int i = 0; i < n_targets; ++i) {
                if (targets[i] < 0 || targets[i] >= (int)d.cards.size()) return set_err(BNPP_ERR_INVALID, "bad target");
                job->targets.push_back(targets[i]);
            }
        } else {
            for (int v = 0; v < (int)d.cards.size(); ++v) job->targets.push_back(v);
        }
    }
    std::vector<Schedule> batches;
    if (n_parts < 1 || part < 0 || part >= n_parts) return set_err(BNPP_ERR_INVALID, "bad part / n_parts");
    if (use_cache) evict_cached_job(ctx);          // it runs in the arena this job may replace
    const double tp = now_ms();
    int rc = plan_schedules(d, job->ev_val, kind, heuristic, order, n_order, job->targets, dtype,
                            budget > 0 ? budget : memory_budget(ctx, use_cache), batches, job->stats, part, n_parts,
                            n_slices, slice_rank);
    if (rc) return rc;
    const double t0 = now_ms();
    rc = cached_sources(ctx, m, dtype, job->src);
    if (rc) return rc;
    const double t1 = now_ms();
    rc = make_program(ctx->c, *job->src, std::move(batches), job->pg, use_cache);
    if (rc) return from_ctx(ctx, rc);
    g_timing[0] = t0 - tp;
    g_timing[1] = t1 - t0;
    g_timing[2] = now_ms() - t1;
    g_timing[7] = job->pg.arena_reused ? 1.0 : 0.0;
    g_timing[8] = job->pg.arena_alloc_ms;
    if (std::getenv("BNPP_TIMING"))
        std::fprintf(stderr, "[bnpp] job: upload %.1f ms, program (arena %.2f GB at %p) %.1f ms\n", t1 - t0,
                     job->pg.arena_bytes / 1e9, job->pg.arena, now_ms() - t1);
    return BNPP_OK;
}

void destroy_job(bnpp_job *job) {
    if (!job) return;
    (void)hipSetDevice(job->ctx->c.device);
    // the buffers go back to the context's cache for the next call: nothing
    // may still run on them (a job may have been launched on any stream; a
    // hipFree would wait the same way)
    (void)hipDeviceSynchronize();
    free_program(job->ctx->c, job->pg);
    job->src.reset();                               // the context's source cache may keep it
    delete job;
}

void evict_cached_job(bnpp_ctx *ctx) {
    if (ctx && ctx->job_cached) {
        destroy_job(ctx->job_cached);
        ctx->job_cached = nullptr;
        ctx->job_key = 0;
    }
}

// key of a one-shot call for the job cache (0: do not cache)
uint64_t call_key(const bnpp_model *m, int kind, int n_ev, const int *ev_vars, const int *ev_vals, int heuristic,
                  const int *order, int n_order, int n_targets, const int *targets, int dtype, int part, int n_parts) {
    if (std::getenv("BNPP_NO_JOB_CACHE")) return 0;
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
    mix(m->uid);
    mix((uint64_t)kind);
    // evidence as a per-variable array; invalid evidence is never cached, so the
    // call goes on to create_job and fails there with BNPP_ERR_INVALID
    std::vector<int> ev;
    std::string msg;
    if (!evidence_array(m->d, n_ev, ev_vars, ev_vals, ev, msg)) return 0;
    for (int x : ev) mix((uint32_t)x);
    mix((uint64_t)heuristic);
    mix((uint64_t)n_order);
    for (int i = 0; i < n_order && order; ++i) mix((uint32_t)order[i]);
    mix((uint64_t)(targets ? n_targets : -1));
    for (int i = 0; i < n_targets && targets; ++i) mix((uint32_t)targets[i]);
    mix((uint64_t)dtype);
    mix((uint64_t)part);
    mix((uint64_t)n_parts);
    mix_plan_knobs(mix);
    return h ? h : 1;
}

// results of a launched job: partition -> out[0] = log10 Z (z_out: Z);
// marginals -> sum(card) normalised values
int job_results(bnpp_job *job, hipStream_t stream, double *out, double *z_out, int *owned = nullptr) {
    std::vector<std::vector<double>> vals;
    std::vector<int64_t> exp2;
    int rc = fetch_program(job->ctx->c, job->pg, stream, vals, exp2);
    if (rc) return from_ctx(job->ctx, rc);
    std::vector<const std::vector<int> *> rvars;
    std::vector<char> mine;
    for (auto &ex : job->pg.parts) {
        for (auto &v : ex.sched.plan_result_vars) rvars.push_back(&v);
        for (char c : ex.sched.plan_result_owned) mine.push_back(c);
    }
    if (job->kind == 0) {
        double p = 0;                                   // part.partition(): sequential sum
        for (double v : vals[0]) p += v;
        out[0] = p > 0 ? std::log10(p) + (double)exp2[0] * std::log10(2.0) : -INFINITY;
        if (z_out) *z_out = std::ldexp(p, (int)std::max<int64_t>(std::min<int64_t>(exp2[0], 1 << 20), -(1 << 20)));
        return BNPP_OK;
    }
    size_t o = 0;
    for (size_t i = 0; i < job->targets.size(); ++i) {
        int t = job->targets[i];
        int k = job->cards[t];
        const std::vector<double> &r = vals[i];
        const bool own = i >= mine.size() || mine[i];
        if (owned) owned[i] = own ? 1 : 0;
        if (!own) {                                     // another part computes it
            for (int s = 0; s < k; ++s) out[o + s] = 0.0;
        } else if (job->ev_val[t] >= 0) {               // evidence variable: one-hot
            for (int s = 0; s < k; ++s) out[o + s] = s == job->ev_val[t] ? 1.0 : 0.0;
        } else if ((int)r.size() == k && k > 0 && rvars[i]->size() == 1) {
            double part = 0;                            // Factor::normalize (factor.cpp:244-255)
            for (double v : r) part += v;
            for (int s = 0; s < k; ++s) out[o + s] = r[s] / part;
        } else {                                        // variable in no factor
            for (int s = 0; s < k; ++s) out[o + s] = 1.0 / k;
        }
        o += (size_t)k;
    }
    return BNPP_OK;
}

// results of a launched sliced job: this rank's share of every target's
// unnormalised marginal, as mantissas (out, sum(card)) and a power-of-two
// scale per target (out_exp2; kNoExp when the share is zero).  Evidence
// variables and variables in no factor: rank 0 carries the one-hot / uniform
// table.  A target that is a slice variable where it is delivered has a
// scalar share, at the index its value (the rank's bit) selects.
constexpr int64_t kNoExp = -((int64_t)1 << 40);
int job_results_sliced(bnpp_job *job, hipStream_t stream, double *out, int64_t *out_exp2) {
    std::vector<std::vector<double>> vals;
    std::vector<int64_t> exp2;
    int rc = fetch_program(job->ctx->c, job->pg, stream, vals, exp2);
    if (rc) return from_ctx(job->ctx, rc);
    std::vector<const std::vector<int> *> rvars;
    std::vector<int> sbit;
    for (auto &ex : job->pg.parts) {
        for (auto &v : ex.sched.plan_result_vars) rvars.push_back(&v);
        for (int b : ex.sched.plan_result_slice_bit) sbit.push_back(b);
    }
    const bool lead = job->slice_rank == 0;
    size_t o = 0;
    for (size_t i = 0; i < job->targets.size(); ++i) {
        const int t = job->targets[i], k = job->cards[t];
        const std::vector<double> &r = vals[i];
        const int sb = i < sbit.size() ? sbit[i] : -1;
        int64_t e = exp2[i];
        for (int s = 0; s < k; ++s) out[o + s] = 0.0;
        if (job->ev_val[t] >= 0) {                      // evidence variable: one-hot
            if (lead) out[o + job->ev_val[t]] = 1.0;
            e = 0;
        } else if (sb >= 0 && r.size() == 1) {          // slice variable: the rank's value
            out[o + ((job->slice_rank >> sb) & 1)] = r[0];
        } else if ((int)r.size() == k && k > 0 && rvars[i]->size() == 1) {
            for (int s = 0; s < k; ++s) out[o + s] = r[s];
        } else {                                        // variable in no factor: uniform
            if (lead)
                for (int s = 0; s < k; ++s) out[o + s] = 1.0 / k;
            e = 0;
        }
        bool any = false;
        for (int s = 0; s < k; ++s) any = any || out[o + s] != 0.0;
        out_exp2[i] = any ? e : kNoExp;
        o += (size_t)k;
    }
    return BNPP_OK;
}

// The plan depends on the memory budget (free memory, the cached arena
// counted as free), which moves a little between identical calls as other
// allocations come and go: within 2 % of the budget the cached job was
// planned under it is relaunched (its arena is allocated already, and a
// checkpoint count planned for a slightly different budget gives the same
// results); beyond that the call plans afresh
bool same_budget(int64_t a, int64_t b) {
    const int64_t d = a > b ? a - b : b - a;
    return a > 0 && b > 0 && d * 50 <= (a > b ? a : b);
}

// A one-shot call's job: the context's cached one when the call is identical
// (its planning phases read 0), else a new one (create).  cache_ok: the call
// holds cache_mu (it runs in the cached arena)
template <typename Create>
int oneshot_job(bnpp_ctx *ctx, bool cache_ok, uint64_t key, int64_t budget, Create &&create, bnpp_job *&job) {
    job = nullptr;
    if (cache_ok && key && ctx->job_cached && ctx->job_key == key && same_budget(ctx->job_budget, budget)) {
        job = ctx->job_cached;
        ctx->job_cached = nullptr;
        ctx->job_key = 0;
        for (int i = 0; i < 3; ++i) g_timing[i] = 0;
        g_timing[7] = 1;
        g_timing[8] = 0;
        return BNPP_OK;
    }
    std::unique_ptr<bnpp_job> j;
    const int rc = create(j);
    job = j.release();
    return rc;
}

// after the call: keep a good job for the next identical call, free the rest
void oneshot_done(bnpp_ctx *ctx, bool cache_ok, uint64_t key, int64_t budget, bnpp_job *job, int rc) {
    if (!job) return;
    if (rc == BNPP_OK && cache_ok && key) {
        evict_cached_job(ctx);
        ctx->job_cached = job;
        ctx->job_key = key;
        ctx->job_budget = budget;
    } else {
        destroy_job(job);
    }
}

// launch / run+fetch / free / total of a call whose create_job filled phases 0-2
void record_call_timing(double t0, double t1, double t2, double t3) {
    g_timing[3] = t2 - t1;
    g_timing[4] = t3 - t2;
    g_timing[5] = now_ms() - t3;
    g_timing[6] = now_ms() - t0;
}

}  // namespace

extern "C" {

const char *bnpp_strerror(int status) {
    switch (status) {
        case BNPP_OK: return "ok";
        case BNPP_ERR_INVALID: return "invalid argument or shape";
        case BNPP_ERR_NO_DEVICE: return "no usable GPU device";
        case BNPP_ERR_OOM: return "out of memory";
        case BNPP_ERR_HIP: return "HIP runtime error";
        case BNPP_ERR_IO: return "cannot read or parse file";
        case BNPP_ERR_UNSUPPORTED: return "unsupported shape";
        default: return "unknown status";
    }
}

const char *bnpp_last_error(void) { return g_err.c_str(); }

int bnpp_last_timing(double *out, int n) {
    if (!out || n < 0) return set_err(BNPP_ERR_INVALID, "null output");
    for (int i = 0; i < n && i < kTimingPhases; ++i) out[i] = g_timing[i];
    return BNPP_OK;
}
int bnpp_version(void) { return BNPP_VERSION; }

int bnpp_device_count(int *n) {
    if (!n) return set_err(BNPP_ERR_INVALID, "null output");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = e == hipSuccess ? c : 0;
    return BNPP_OK;
}

int bnpp_ctx_create(int device, bnpp_ctx **out) {
    BNPP_GUARD_BEGIN
    if (!out) return set_err(BNPP_ERR_INVALID, "null output");
    *out = nullptr;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c <= 0) return set_err(BNPP_ERR_NO_DEVICE, "no HIP device visible (the engine has no CPU fallback)");
    if (device < 0 || device >= c) return set_err(BNPP_ERR_NO_DEVICE, "device index out of range");
    if ((e = hipSetDevice(device)) != hipSuccess) return set_err(BNPP_ERR_HIP, hipGetErrorString(e));
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return set_err(BNPP_ERR_HIP, hipGetErrorString(e));
    std::unique_ptr<bnpp_ctx> ctx(new bnpp_ctx);
    ctx->c.device = device;
    int per_cu = 3;          // measured: 3 workgroups per CU beat 4 and 8 on the bench bucket and the 32x32 sweep
    if (const char *g = tuning_knob("BNPP_GRID_PER_CU")) per_cu = std::max(0, std::min(64, std::atoi(g)));
    // 0: flat grid, one virtual block per workgroup (no grid-stride)
    ctx->c.max_grid = per_cu == 0 ? INT32_MAX : prop.multiProcessorCount * per_cu;
    if ((e = hipStreamCreateWithFlags(&ctx->c.stream, hipStreamNonBlocking)) != hipSuccess)
        return set_err(BNPP_ERR_HIP, hipGetErrorString(e));
    {
        std::lock_guard<std::mutex> g(g_ctxs_mu);
        g_ctxs.push_back(ctx.get());
    }
    *out = ctx.release();
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_ctx_destroy(bnpp_ctx *ctx) {
    if (!ctx) return BNPP_OK;
    {
        std::lock_guard<std::mutex> g(g_ctxs_mu);
        g_ctxs.erase(std::remove(g_ctxs.begin(), g_ctxs.end(), ctx), g_ctxs.end());
    }
    (void)hipSetDevice(ctx->c.device);
    {
        // a bnpp_model_free on another thread may hold this lock while it
        // evicts the cached job (it collected the context before the erase
        // above): wait for it, so the job is destroyed once and the lock is
        // released before the context is deleted
        std::lock_guard<std::mutex> lk(ctx->cache_mu);
        evict_cached_job(ctx);
    }
    if (ctx->c.stream) (void)hipStreamDestroy(ctx->c.stream);
    if (ctx->c.lane_stream) (void)hipStreamDestroy(ctx->c.lane_stream);
    ctx->srcs.clear();
    drop_arena_cache(ctx->c);
    drop_buffer_cache(ctx->c);
    delete ctx;
    return BNPP_OK;
}

int bnpp_ctx_trim(bnpp_ctx *ctx) {
    if (!ctx) return set_err(BNPP_ERR_INVALID, "null context");
    std::unique_lock<std::mutex> lk(ctx->cache_mu, std::try_to_lock);
    if (!lk.owns_lock()) return set_err(BNPP_ERR_INVALID, "a call on this context is running");
    (void)hipSetDevice(ctx->c.device);
    (void)hipDeviceSynchronize();
    evict_cached_job(ctx);
    {
        std::lock_guard<std::mutex> g(ctx->src_mu);
        ctx->srcs.clear();
    }
    drop_arena_cache(ctx->c);
    drop_buffer_cache(ctx->c);
    return BNPP_OK;
}

int bnpp_ctx_stream(bnpp_ctx *ctx, void **stream) {
    if (!ctx || !stream) return set_err(BNPP_ERR_INVALID, "null argument");
    *stream = ctx->c.stream;
    return BNPP_OK;
}

int bnpp_malloc(bnpp_ctx *ctx, size_t bytes, void **dptr) {
    if (!ctx || !dptr) return set_err(BNPP_ERR_INVALID, "null argument");
    (void)hipSetDevice(ctx->c.device);
    hipError_t e = hipMalloc(dptr, bytes ? bytes : 1);
    if (e != hipSuccess) return set_err(e == hipErrorOutOfMemory ? BNPP_ERR_OOM : BNPP_ERR_HIP, hipGetErrorString(e));
    return BNPP_OK;
}

int bnpp_free(bnpp_ctx *ctx, void *dptr) {
    if (!ctx) return set_err(BNPP_ERR_INVALID, "null context");
    (void)hipSetDevice(ctx->c.device);
    hipError_t e = hipFree(dptr);
    return e == hipSuccess ? BNPP_OK : set_err(BNPP_ERR_HIP, hipGetErrorString(e));
}

int bnpp_memcpy_h2d(bnpp_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return set_err(BNPP_ERR_INVALID, "null context");
    (void)hipSetDevice(ctx->c.device);
    hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
    return e == hipSuccess ? BNPP_OK : set_err(BNPP_ERR_HIP, hipGetErrorString(e));
}

int bnpp_memcpy_d2h(bnpp_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx) return set_err(BNPP_ERR_INVALID, "null context");
    (void)hipSetDevice(ctx->c.device);
    hipError_t e = hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost);
    return e == hipSuccess ? BNPP_OK : set_err(BNPP_ERR_HIP, hipGetErrorString(e));
}

int bnpp_synchronize(bnpp_ctx *ctx, void *stream) {
    if (!ctx) return set_err(BNPP_ERR_INVALID, "null context");
    (void)hipSetDevice(ctx->c.device);
    hipError_t e = hipStreamSynchronize(pick_stream(ctx, stream));
    return e == hipSuccess ? BNPP_OK : set_err(BNPP_ERR_HIP, hipGetErrorString(e));
}

int bnpp_out_scope(int n_in, const int *in_ndims, const int *const *in_vars, int elim_var, int cap,
                   int *out_ndims, int *out_vars) {
    BNPP_GUARD_BEGIN
    if (n_in < 0 || (n_in > 0 && (!in_ndims || !in_vars)) || !out_ndims) return set_err(BNPP_ERR_INVALID, "bad arguments");
    std::vector<int> u;
    for (int i = 0; i < n_in; ++i) {
        std::vector<int> s(in_vars[i], in_vars[i] + in_ndims[i]);
        u = union_scope(u, s);
    }
    if (elim_var >= 0) u = remove_var(u, elim_var);
    *out_ndims = (int)u.size();
    if ((int)u.size() > cap) return set_err(BNPP_ERR_INVALID, "output scope larger than cap");
    std::copy(u.begin(), u.end(), out_vars);
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_bucket_eliminate(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, int n_in,
                          const void *const *in_tables, const int *in_ndims, const int *const *in_vars, int elim_var,
                          void *out_table, int out_ndims, const int *out_vars, double *out_sum) {
    BNPP_GUARD_BEGIN
    if (!ctx || !cards || n_in < 1 || !in_tables || !in_ndims || !in_vars || !out_table)
        return set_err(BNPP_ERR_INVALID, "null argument");
    if (n_in > kMaxIn) return set_err(BNPP_ERR_UNSUPPORTED, "at most 8 inputs per fused call");
    if (n_cards < 0 || elim_var >= n_cards || (out_ndims > 0 && !out_vars))
        return set_err(BNPP_ERR_INVALID, "variable id outside cards[0, n_cards)");
    for (int i = 0; i < n_in; ++i)
        if (!valid_scope(in_ndims[i], in_vars[i], cards, n_cards)) return set_err(BNPP_ERR_INVALID, "bad input scope");
    if (!valid_scope(out_ndims, out_vars, cards, n_cards)) return set_err(BNPP_ERR_INVALID, "bad output scope");
    std::vector<int> cv(cards, cards + n_cards);
    BucketSpec b;
    std::vector<const void *> ptrs;
    for (int i = 0; i < n_in; ++i) {
        std::vector<int> s(in_vars[i], in_vars[i] + in_ndims[i]);
        b.in.push_back(natural_view(i, s, cv));
        ptrs.push_back(in_tables[i]);
    }
    b.elim_var = elim_var;
    // the output must hold exactly the kept variables (domain.cpp:32-72), in any order
    std::vector<int> u = chain_scope(b.in);
    if (elim_var >= 0) u = remove_var(u, elim_var);
    std::vector<int> ov(out_vars, out_vars + out_ndims), us = u, os = ov;
    std::sort(us.begin(), us.end());
    std::sort(os.begin(), os.end());
    if (us != os) return set_err(BNPP_ERR_INVALID, "output scope must be the union of the inputs minus elim_var");
    b.out_vars = ov;
    b.out_table = n_in;
    if (int rc = seq_sum_supported(out_sum, u.size(), b.in.size())) return rc;
    int rc = run_single(ctx, stream, dtype, cv, b, ptrs, out_table);
    if (rc == BNPP_OK) rc = run_seq_sum(ctx, stream, dtype, cv, b.in, ptrs, u, elim_var, false, out_sum);
    return rc;
    BNPP_GUARD_END
}

int bnpp_product(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *a, int a_ndims,
                 const int *a_vars, const void *b, int b_ndims, const int *b_vars, void *out, int out_ndims,
                 const int *out_vars, double *out_sum) {
    const void *tabs[2] = {a, b};
    const int nd[2] = {a_ndims, b_ndims};
    const int *vs[2] = {a_vars, b_vars};
    return bnpp_bucket_eliminate(ctx, stream, dtype, n_cards, cards, 2, tabs, nd, vs, -1, out, out_ndims, out_vars,
                                 out_sum);
}

int bnpp_divide(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *a, int a_ndims,
                const int *a_vars, const void *b, int b_ndims, const int *b_vars, void *out, int out_ndims,
                const int *out_vars, double *out_sum) {
    BNPP_GUARD_BEGIN
    if (!ctx || !cards || !a || !b || !out || (a_ndims > 0 && !a_vars) || (b_ndims > 0 && !b_vars) ||
        (out_ndims > 0 && !out_vars))
        return set_err(BNPP_ERR_INVALID, "null argument");
    if (!valid_scope(a_ndims, a_vars, cards, n_cards) || !valid_scope(b_ndims, b_vars, cards, n_cards))
        return set_err(BNPP_ERR_INVALID, "bad input scope");
    if (!valid_scope(out_ndims, out_vars, cards, n_cards)) return set_err(BNPP_ERR_INVALID, "bad output scope");
    std::vector<int> cv(cards, cards + n_cards);
    BucketSpec bs;
    bs.in.push_back(natural_view(0, std::vector<int>(a_vars, a_vars + a_ndims), cv));
    bs.in.push_back(natural_view(1, std::vector<int>(b_vars, b_vars + b_ndims), cv));
    std::vector<int> u = chain_scope(bs.in), ov(out_vars, out_vars + out_ndims), us = u, os = ov;
    std::sort(us.begin(), us.end());
    std::sort(os.begin(), os.end());
    if (us != os) return set_err(BNPP_ERR_INVALID, "output scope must be the union of the inputs");
    bs.out_vars = ov;
    bs.out_table = 2;
    bs.divide = true;
    if (int rc = seq_sum_supported(out_sum, u.size(), bs.in.size())) return rc;
    int rc = run_single(ctx, stream, dtype, cv, bs, {a, b}, out);
    if (rc == BNPP_OK) rc = run_seq_sum(ctx, stream, dtype, cv, bs.in, {a, b}, u, -1, true, out_sum);
    return rc;
    BNPP_GUARD_END
}

int bnpp_sum_out(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *in, int ndims,
                 const int *vars, int var, void *out, int out_ndims, const int *out_vars, double *out_sum) {
    const void *tabs[1] = {in};
    return bnpp_bucket_eliminate(ctx, stream, dtype, n_cards, cards, 1, tabs, &ndims, &vars, var, out, out_ndims, out_vars,
                                 out_sum);
}

int bnpp_condition(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *in, int ndims,
                   const int *vars, int n_ev, const int *ev_vars, const int *ev_vals, void *out, double *out_sum) {
    BNPP_GUARD_BEGIN
    if (!ctx || !cards || !in || !out || (ndims > 0 && !vars) || n_ev < 0 || (n_ev > 0 && (!ev_vars || !ev_vals)))
        return set_err(BNPP_ERR_INVALID, "null argument");
    if (!valid_scope(ndims, vars, cards, n_cards)) return set_err(BNPP_ERR_INVALID, "bad scope");
    std::vector<int> cv(cards, cards + n_cards);
    std::vector<int> ev(n_cards, -1);
    std::vector<char> in_scope(n_cards, 0);
    for (int i = 0; i < ndims; ++i) in_scope[vars[i]] = 1;
    for (int i = 0; i < n_ev; ++i) {
        int v = ev_vars[i];
        if (v < 0) return set_err(BNPP_ERR_INVALID, "bad evidence variable");
        // evidence on a variable outside the scope does not touch the factor
        // (Domain(d, ev) looks up scope variables only, domain.cpp:74-90)
        if (v >= n_cards || !in_scope[v]) continue;
        if (ev_vals[i] < 0 || ev_vals[i] >= cv[v]) return set_err(BNPP_ERR_INVALID, "evidence value out of range");
        ev[v] = ev_vals[i];
    }
    std::vector<int> s(vars, vars + ndims);
    BucketSpec b;
    b.in.push_back(conditioned_view(0, s, cv, ev));
    b.out_vars = b.in[0].vars;
    b.out_table = 1;
    if (int rc = seq_sum_supported(out_sum, b.out_vars.size(), b.in.size())) return rc;
    int rc = run_single(ctx, stream, dtype, cv, b, {in}, out);
    if (rc == BNPP_OK) rc = run_seq_sum(ctx, stream, dtype, cv, b.in, {in}, b.out_vars, -1, false, out_sum);
    return rc;
    BNPP_GUARD_END
}

int bnpp_model_load_uai(const char *path, bnpp_model **out) {
    BNPP_GUARD_BEGIN
    if (!path || !out) return set_err(BNPP_ERR_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<bnpp_model> m(new bnpp_model);
    std::string err;
    if (load_uai(path, m->d, &err)) return set_err(BNPP_ERR_IO, err);
    *out = m.release();
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_model_from_arrays(int is_bayes, int n_vars, const int *cards, int n_factors, const int *widths,
                           const int *scopes, const double *values, bnpp_model **out) {
    BNPP_GUARD_BEGIN
    if (!out || n_vars < 0 || n_factors < 0 || (n_vars > 0 && !cards) || (n_factors > 0 && (!widths || !scopes || !values)))
        return set_err(BNPP_ERR_INVALID, "bad arguments");
    *out = nullptr;
    std::unique_ptr<bnpp_model> m(new bnpp_model);
    m->d.is_bayes = is_bayes != 0;
    m->d.cards.assign(cards, cards + n_vars);
    for (int c : m->d.cards)
        if (c < 1) return set_err(BNPP_ERR_INVALID, "cardinality must be >= 1");
    const int *sc = scopes;
    const double *vals = values;
    for (int f = 0; f < n_factors; ++f) {
        if (widths[f] < 0) return set_err(BNPP_ERR_INVALID, "negative width");
        std::vector<int> s(sc, sc + widths[f]);
        sc += widths[f];
        int64_t sz = 1;
        for (int v : s) {
            if (v < 0 || v >= n_vars) return set_err(BNPP_ERR_INVALID, "scope id out of range");
            sz *= m->d.cards[v];
        }
        m->d.scopes.push_back(s);
        m->d.values.emplace_back(vals, vals + sz);
        vals += sz;
    }
    std::string err;
    if (!validate(m->d, &err)) return set_err(BNPP_ERR_INVALID, err);
    *out = m.release();
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_model_free(bnpp_model *m) {
    if (!m) return BNPP_OK;
    // every live context drops the model's uploaded sources and a cached
    // one-shot job planned for it (a context in the middle of a call keeps
    // its job until its next one-shot call replaces it)
    // The contexts holding such a job are collected under the context list's
    // lock; their jobs are destroyed after it is released (destroy_job waits
    // for the device: other threads' ctx_create / ctx_destroy / model_free do
    // not wait with it), each under its own context's cache lock, and the
    // caller's current device is restored afterwards.
    std::vector<std::pair<bnpp_ctx *, std::unique_lock<std::mutex>>> evict;
    {
        std::lock_guard<std::mutex> g(g_ctxs_mu);
        for (bnpp_ctx *ctx : g_ctxs) {
            {
                std::lock_guard<std::mutex> gs(ctx->src_mu);
                ctx->srcs.erase(std::remove_if(ctx->srcs.begin(), ctx->srcs.end(),
                                               [&](const bnpp_ctx::Src &e) { return e.uid == m->uid; }),
                                ctx->srcs.end());
            }
            std::unique_lock<std::mutex> lk(ctx->cache_mu, std::try_to_lock);
            if (lk.owns_lock() && ctx->job_cached && ctx->job_cached->model_uid == m->uid)
                evict.emplace_back(ctx, std::move(lk));
        }
    }
    if (!evict.empty()) {
        int dev = -1;
        const bool had = hipGetDevice(&dev) == hipSuccess;
        for (auto &e : evict) evict_cached_job(e.first);
        if (had) (void)hipSetDevice(dev);
    }
    delete m;
    return BNPP_OK;
}

int bnpp_model_info(const bnpp_model *m, int *is_bayes, int *n_vars, int *n_factors) {
    if (!m) return set_err(BNPP_ERR_INVALID, "null model");
    if (is_bayes) *is_bayes = m->d.is_bayes ? 1 : 0;
    if (n_vars) *n_vars = (int)m->d.cards.size();
    if (n_factors) *n_factors = (int)m->d.scopes.size();
    return BNPP_OK;
}

int bnpp_model_cards(const bnpp_model *m, int *cards) {
    if (!m || !cards) return set_err(BNPP_ERR_INVALID, "null argument");
    std::copy(m->d.cards.begin(), m->d.cards.end(), cards);
    return BNPP_OK;
}

int bnpp_evidence_load(const char *path, int cap, int *n, int *vars, int *vals) {
    BNPP_GUARD_BEGIN
    if (!path || !n) return set_err(BNPP_ERR_INVALID, "null argument");
    std::vector<std::pair<int, int>> ev;
    if (load_evidence(path, ev)) return set_err(BNPP_ERR_IO, std::string("couldn't read file ") + path);
    *n = (int)ev.size();
    if ((int)ev.size() > cap) return set_err(BNPP_ERR_INVALID, "evidence larger than cap");
    for (size_t i = 0; i < ev.size(); ++i) {
        vars[i] = ev[i].first;
        vals[i] = ev[i].second;
    }
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_ordering(const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals, int n_vars,
                  const int *vars, int heuristic, int *order_out, int *width_out) {
    BNPP_GUARD_BEGIN
    if (!m || !order_out) return set_err(BNPP_ERR_INVALID, "null argument");
    if (heuristic < BNPP_ORDER_GIVEN || heuristic > BNPP_MIN_DEGREE) return set_err(BNPP_ERR_INVALID, "unknown heuristic");
    const ModelData &d = m->d;
    std::vector<int> ev;
    std::string msg;
    if (!evidence_array(d, n_ev, ev_vars, ev_vals, ev, msg)) return set_err(BNPP_ERR_INVALID, msg);
    std::vector<int> vs;
    if (vars) {
        for (int i = 0; i < n_vars; ++i) {
            if (vars[i] < 0 || vars[i] >= (int)d.cards.size()) return set_err(BNPP_ERR_INVALID, "bad variable");
            vs.push_back(vars[i]);
        }
    } else {
        for (int v = 0; v < (int)d.cards.size(); ++v)
            if (ev[v] < 0) vs.push_back(v);
    }
    std::vector<int> ord;
    int w = elimination_order((int)d.cards.size(), d.cards, conditioned_scopes(d, ev), vs, (Heuristic)heuristic, ord);
    std::copy(ord.begin(), ord.end(), order_out);
    if (width_out) *width_out = w;
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_job_create(bnpp_ctx *ctx, const bnpp_model *m, int kind, int n_ev, const int *ev_vars, const int *ev_vals,
                    int heuristic, const int *order, int n_order, int n_targets, const int *targets, int dtype,
                    bnpp_job **out) {
    BNPP_GUARD_BEGIN
    if (!out) return set_err(BNPP_ERR_INVALID, "null output");
    *out = nullptr;
    if (kind != 0 && kind != 1 && kind != 3)
        return set_err(BNPP_ERR_INVALID, "kind must be 0 (partition), 1 (marginals) or 3 (bucket-tree marginals)");
    std::unique_ptr<bnpp_job> job;
    int rc = create_job(ctx, m, kind, n_ev, ev_vars, ev_vals, heuristic, order, n_order, n_targets, targets, dtype, job);
    if (rc) {
        if (job) destroy_job(job.release());
        return rc;
    }
    *out = job.release();
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_variable_elimination(bnpp_ctx *ctx, const bnpp_model *m, int n_vars, const int *vars, int heuristic,
                              int dtype, int cap_vars, int *out_ndims, int *out_vars, int64_t cap_values,
                              int64_t *out_size, double *out_values, int64_t *exp2) {
    BNPP_GUARD_BEGIN
    if (!out_ndims || !out_size || !exp2 || (n_vars > 0 && !vars)) return set_err(BNPP_ERR_INVALID, "null argument");
    std::unique_ptr<bnpp_job> job;
    std::unique_lock<std::mutex> lk;
    if (ctx) lk = std::unique_lock<std::mutex>(ctx->cache_mu, std::try_to_lock);
    int rc = create_job(ctx, m, 2, 0, nullptr, nullptr, heuristic, vars, n_vars, 0, nullptr, dtype, job, 0, 1,
                        lk.owns_lock());
    if (rc == BNPP_OK) rc = from_ctx(ctx, launch_program(ctx->c, job->pg, ctx->c.stream));
    std::vector<std::vector<double>> vals;
    std::vector<int64_t> e2;
    if (rc == BNPP_OK) rc = from_ctx(ctx, fetch_program(ctx->c, job->pg, ctx->c.stream, vals, e2));
    if (rc == BNPP_OK) {
        const std::vector<int> &rv = job->pg.parts[0].sched.plan_result_vars[0];
        *out_ndims = (int)rv.size();
        *out_size = (int64_t)vals[0].size();
        *exp2 = e2[0];
        if ((int)rv.size() > cap_vars || (int64_t)vals[0].size() > cap_values) {
            rc = set_err(BNPP_ERR_INVALID, "result larger than the output capacity");
        } else {
            std::copy(rv.begin(), rv.end(), out_vars);
            std::copy(vals[0].begin(), vals[0].end(), out_values);
        }
    }
    if (job) destroy_job(job.release());
    return rc;
    BNPP_GUARD_END
}

int bnpp_plan_stats(const bnpp_model *m, int kind, int n_ev, const int *ev_vars, const int *ev_vals, int heuristic,
                    const int *order, int n_order, int dtype, double *stats, int n_stats) {
    BNPP_GUARD_BEGIN
    if (!m || !stats) return set_err(BNPP_ERR_INVALID, "null argument");
    if (kind != 0 && kind != 1 && kind != 3) return set_err(BNPP_ERR_INVALID, "kind must be 0, 1 or 3");
    std::vector<int> ev, targets;
    std::string msg;
    if (!evidence_array(m->d, n_ev, ev_vars, ev_vals, ev, msg)) return set_err(BNPP_ERR_INVALID, msg);
    if (kind == 1 || kind == 3)
        for (int v = 0; v < (int)m->d.cards.size(); ++v) targets.push_back(v);
    std::vector<Schedule> batches;
    double st[10] = {0};
    int rc = plan_schedules(m->d, ev, kind, heuristic, order, n_order, targets, dtype, memory_budget(nullptr), batches, st);
    if (rc) return rc;
    for (int i = 0; i < n_stats && i < 8; ++i) stats[i] = st[i];
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_plan_tree_part(const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals, int heuristic,
                        const int *order, int n_order, int part, int n_parts, int dtype, int *owned, double *stats,
                        int n_stats) {
    BNPP_GUARD_BEGIN
    if (!m || !owned) return set_err(BNPP_ERR_INVALID, "null argument");
    if (n_parts < 1 || part < 0 || part >= n_parts) return set_err(BNPP_ERR_INVALID, "bad part / n_parts");
    std::vector<int> ev, targets;
    std::string msg;
    if (!evidence_array(m->d, n_ev, ev_vars, ev_vals, ev, msg)) return set_err(BNPP_ERR_INVALID, msg);
    for (int v = 0; v < (int)m->d.cards.size(); ++v) targets.push_back(v);
    std::vector<Schedule> batches;
    double st[10] = {0};
    int rc = plan_schedules(m->d, ev, 3, heuristic, order, n_order, targets, dtype, memory_budget(nullptr), batches, st,
                            part, n_parts);
    if (rc) return rc;
    size_t i = 0;
    for (auto &s : batches)
        for (char c : s.plan_result_owned) owned[i++] = c ? 1 : 0;
    for (int k = 0; stats && k < n_stats && k < 8; ++k) stats[k] = st[k];
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_job_stats(const bnpp_job *job, double *stats, int n_stats) {
    if (!job || !stats) return set_err(BNPP_ERR_INVALID, "null argument");
    for (int i = 0; i < n_stats && i < 8; ++i) stats[i] = job->stats[i];
    return BNPP_OK;
}

int bnpp_job_launch(bnpp_job *job, void *stream) {
    BNPP_GUARD_BEGIN
    if (!job) return set_err(BNPP_ERR_INVALID, "null job");
    (void)hipSetDevice(job->ctx->c.device);
    return from_ctx(job->ctx, launch_program(job->ctx->c, job->pg, pick_stream(job->ctx, stream)));
    BNPP_GUARD_END
}

int bnpp_job_results(bnpp_job *job, void *stream, double *out) {
    BNPP_GUARD_BEGIN
    if (!job || !out) return set_err(BNPP_ERR_INVALID, "null argument");
    (void)hipSetDevice(job->ctx->c.device);
    return job_results(job, pick_stream(job->ctx, stream), out, nullptr);
    BNPP_GUARD_END
}

int bnpp_job_free(bnpp_job *job) {
    destroy_job(job);
    return BNPP_OK;
}

int bnpp_partition(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                   int heuristic, const int *order, int n_order, int dtype, double *log10_z, double *z,
                   double *uptime_ms) {
    BNPP_GUARD_BEGIN
    double t0 = now_ms();
    if (!ctx || !m) return set_err(BNPP_ERR_INVALID, "null context or model");
    bnpp_job *job = nullptr;
    std::unique_lock<std::mutex> lk(ctx->cache_mu, std::try_to_lock);
    const bool cache_ok = lk.owns_lock();
    const int64_t budget = memory_budget(ctx, true);
    const uint64_t key = cache_ok ? call_key(m, 0, n_ev, ev_vars, ev_vals, heuristic, order, n_order, 0, nullptr, dtype,
                                             0, 1) : 0;
    int rc = oneshot_job(ctx, cache_ok, key, budget, [&](std::unique_ptr<bnpp_job> &j) {
        return create_job(ctx, m, 0, n_ev, ev_vars, ev_vals, heuristic, order, n_order, 0, nullptr, dtype, j, 0, 1,
                          cache_ok);
    }, job);
    const double t1 = now_ms();
    if (rc == BNPP_OK) rc = from_ctx(ctx, launch_program(ctx->c, job->pg, ctx->c.stream));
    const double t2 = now_ms();
    double lz = 0, zz = 0;
    if (rc == BNPP_OK) rc = job_results(job, ctx->c.stream, &lz, &zz);
    const double t3 = now_ms();
    oneshot_done(ctx, cache_ok, key, budget, job, rc);
    record_call_timing(t0, t1, t2, t3);
    if (rc) return rc;
    if (log10_z) *log10_z = lz;
    if (z) *z = zz;
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_marginals(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                   int heuristic, int n_targets, const int *targets, int dtype, double *out, double *uptime_ms) {
    BNPP_GUARD_BEGIN
    if (!out) return set_err(BNPP_ERR_INVALID, "null output");
    double t0 = now_ms();
    if (!ctx || !m) return set_err(BNPP_ERR_INVALID, "null context or model");
    bnpp_job *job = nullptr;
    std::unique_lock<std::mutex> lk(ctx->cache_mu, std::try_to_lock);
    const bool cache_ok = lk.owns_lock();
    const int64_t budget = memory_budget(ctx, true);
    const uint64_t key = cache_ok ? call_key(m, 1, n_ev, ev_vars, ev_vals, heuristic, nullptr, 0, n_targets, targets,
                                             dtype, 0, 1) : 0;
    int rc = oneshot_job(ctx, cache_ok, key, budget, [&](std::unique_ptr<bnpp_job> &j) {
        return create_job(ctx, m, 1, n_ev, ev_vars, ev_vals, heuristic, nullptr, 0, n_targets, targets, dtype, j, 0, 1,
                          cache_ok);
    }, job);
    const double t1 = now_ms();
    if (rc == BNPP_OK) rc = from_ctx(ctx, launch_program(ctx->c, job->pg, ctx->c.stream));
    const double t2 = now_ms();
    if (rc == BNPP_OK) rc = job_results(job, ctx->c.stream, out, nullptr);
    const double t3 = now_ms();
    oneshot_done(ctx, cache_ok, key, budget, job, rc);
    record_call_timing(t0, t1, t2, t3);
    if (std::getenv("BNPP_TIMING"))
        std::fprintf(stderr, "[bnpp] marginals: create %.1f ms, launch %.1f ms, run+fetch %.1f ms, free %.1f ms\n",
                     t1 - t0, t2 - t1, t3 - t2, now_ms() - t3);
    if (rc) return rc;
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_marginals_tree(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                        int heuristic, const int *order, int n_order, int n_targets, const int *targets, int dtype,
                        double *out, double *uptime_ms) {
    return bnpp_marginals_tree_part(ctx, m, n_ev, ev_vars, ev_vals, heuristic, order, n_order, n_targets, targets, 0,
                                    1, dtype, out, nullptr, uptime_ms);
}

int bnpp_marginals_tree_part(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                             int heuristic, const int *order, int n_order, int n_targets, const int *targets,
                             int part, int n_parts, int dtype, double *out, int *owned, double *uptime_ms) {
    BNPP_GUARD_BEGIN
    if (!out) return set_err(BNPP_ERR_INVALID, "null output");
    double t0 = now_ms();
    if (!ctx || !m) return set_err(BNPP_ERR_INVALID, "null context or model");
    const bool timing = std::getenv("BNPP_TIMING") != nullptr;
    bnpp_job *job = nullptr;
    std::unique_lock<std::mutex> lk(ctx->cache_mu, std::try_to_lock);
    const bool cache_ok = lk.owns_lock();
    const int64_t budget = memory_budget(ctx, true);
    const uint64_t key = cache_ok ? call_key(m, 3, n_ev, ev_vars, ev_vals, heuristic, order, n_order, n_targets,
                                             targets, dtype, part, n_parts) : 0;
    int rc = oneshot_job(ctx, cache_ok, key, budget, [&](std::unique_ptr<bnpp_job> &j) {
        return create_job(ctx, m, 3, n_ev, ev_vars, ev_vals, heuristic, order, n_order, n_targets, targets, dtype, j,
                          part, n_parts, cache_ok);
    }, job);
    const double t1 = now_ms();
    if (rc == BNPP_OK) rc = from_ctx(ctx, launch_program(ctx->c, job->pg, ctx->c.stream));
    const double t2 = now_ms();
    if (rc == BNPP_OK) rc = job_results(job, ctx->c.stream, out, nullptr, owned);
    const double t3 = now_ms();
    oneshot_done(ctx, cache_ok, key, budget, job, rc);
    record_call_timing(t0, t1, t2, t3);
    if (timing)
        std::fprintf(stderr, "[bnpp] tree marginals: create %.1f ms, launch %.1f ms, run+fetch %.1f ms, free %.1f ms\n",
                     t1 - t0, t2 - t1, t3 - t2, now_ms() - t3);
    if (rc) return rc;
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return BNPP_OK;
    BNPP_GUARD_END
}

int bnpp_marginals_tree_sliced(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                               int heuristic, const int *order, int n_order, int n_targets, const int *targets,
                               int rank, int n_ranks, bnpp_collective_fn coll, void *user, double budget_gb,
                               int dtype, double *out, int64_t *out_exp2, double *uptime_ms) {
    BNPP_GUARD_BEGIN
    if (!out || !out_exp2 || !coll) return set_err(BNPP_ERR_INVALID, "null output or collective");
    if (n_ranks < 2) return set_err(BNPP_ERR_INVALID, "sliced runs need n_ranks >= 2 (bnpp_marginals_tree otherwise)");
    double t0 = now_ms();
    if (!ctx || !m) return set_err(BNPP_ERR_INVALID, "null context or model");
    // an identical call (same model, evidence, order, targets, dtype, rank,
    // world and budget) relaunches the job the previous one planned, as the
    // one-GPU tree marginals do; the collective is bound per call
    bnpp_job *job = nullptr;
    std::unique_lock<std::mutex> lk(ctx->cache_mu, std::try_to_lock);
    const bool cache_ok = lk.owns_lock();
    const int64_t fixed = budget_gb > 0 ? (int64_t)(budget_gb * 1e9) : 0;
    const int64_t budget = fixed ? fixed : memory_budget(ctx, true);
    const uint64_t key = cache_ok ? call_key(m, 4, n_ev, ev_vars, ev_vals, heuristic, order, n_order, n_targets, targets,
                                             dtype, rank, n_ranks) : 0;
    int rc = oneshot_job(ctx, cache_ok, key, budget, [&](std::unique_ptr<bnpp_job> &j) {
        return create_job(ctx, m, 3, n_ev, ev_vars, ev_vals, heuristic, order, n_order, n_targets, targets, dtype, j,
                          0, 1, cache_ok, n_ranks, rank, fixed);
    }, job);
    const double t1 = now_ms();
    if (rc == BNPP_OK) {
        job->pg.hooks.fn = coll;
        job->pg.hooks.user = user;
        rc = from_ctx(ctx, launch_program(ctx->c, job->pg, ctx->c.stream));
    }
    const double t2 = now_ms();
    if (rc == BNPP_OK) rc = job_results_sliced(job, ctx->c.stream, out, out_exp2);
    const double t3 = now_ms();
    oneshot_done(ctx, cache_ok, key, budget, job, rc);
    record_call_timing(t0, t1, t2, t3);
    if (std::getenv("BNPP_TIMING"))
        std::fprintf(stderr, "[bnpp] sliced tree marginals (rank %d of %d): create %.1f ms, launch %.1f ms, run+fetch %.1f ms\n",
                     rank, n_ranks, t1 - t0, t2 - t1, t3 - t2);
    if (rc) return rc;
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return BNPP_OK;
    BNPP_GUARD_END
}

// a world of n_ranks identical ranks (user: int[4] = {n_ranks, flags,
// link MB/s, latency us}): every block this rank would receive is a copy of
// what it sends -- the timing of one rank's share of a sliced run on one GPU,
// the data movement local; flags & 1: no bytes move; flags & 2: the stream
// waits the transfer's modelled xGMI time (latency + bytes sent over
// min(n_ranks - 1, 7) links at the given rate each)
int bnpp_collective_loopback(void *user, int op, const void *send, void *recv, int64_t bytes, void *stream) {
    if (!user || !send || !recv || bytes < 0) return 1;
    const int *u = static_cast<const int *>(user);
    const int R = u[0];
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (u[1] & 2) {                                          // a modelled transfer: the stream waits its duration
        const double links = R - 1 < 7 ? R - 1 : 7, sent = (double)bytes * (R - 1);
        const double ns = u[3] * 1e3 + sent / (links * (double)u[2] * 1e6) * 1e9;
        if (launch_delay(ns, s) != hipSuccess) return 1;
    }
    if (u[1] & 1) return 0;                                  // no data movement: the compute alone
    if (op == BNPP_COLL_ALLGATHER) {
        for (int r = 0; r < R; ++r)
            if (hipMemcpyAsync(static_cast<char *>(recv) + (int64_t)r * bytes, send, (size_t)bytes,
                               hipMemcpyDeviceToDevice, s) != hipSuccess)
                return 1;
        return 0;
    }
    if (op == BNPP_COLL_ALLTOALL)
        return hipMemcpyAsync(recv, send, (size_t)bytes * R, hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : 1;
    return 1;
}

int bnpp_plan_tree_sliced(const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals, int heuristic,
                          const int *order, int n_order, int rank, int n_ranks, int dtype, int *slice_bit,
                          double *stats, int n_stats) {
    BNPP_GUARD_BEGIN
    if (!m) return set_err(BNPP_ERR_INVALID, "null argument");
    if (n_ranks < 2 || rank < 0 || rank >= n_ranks) return set_err(BNPP_ERR_INVALID, "bad rank / n_ranks");
    std::vector<int> ev, targets;
    std::string msg;
    if (!evidence_array(m->d, n_ev, ev_vars, ev_vals, ev, msg)) return set_err(BNPP_ERR_INVALID, msg);
    for (int v = 0; v < (int)m->d.cards.size(); ++v) targets.push_back(v);
    std::vector<Schedule> batches;
    double st[10] = {0};
    int rc = plan_schedules(m->d, ev, 3, heuristic, order, n_order, targets, dtype, memory_budget(nullptr), batches, st,
                            0, 1, n_ranks, rank);
    if (rc) return rc;
    size_t i = 0;
    for (auto &s : batches)
        for (int b : s.plan_result_slice_bit)
            if (slice_bit) slice_bit[i++] = b;
    for (int k = 0; stats && k < n_stats && k < 10; ++k) stats[k] = st[k];
    return BNPP_OK;
    BNPP_GUARD_END
}

// Loopy BP as one launch per phase and iteration (bp.hip bp_flood_*, the
// layout of BpFlood): the choice for models whose iteration is too much work
// for one workgroup and for tables of 2^31 entries or more.  The host checks
// the per-iteration maxima every kBpErrChunk iterations; launches after the
// converging iteration return at once on the device.
// one-workgroup loop up to this much work per iteration (f2v terms x scope
// size + v2f products), the flood beyond (tools/bp_modes.py: a 12x12 Ising
// grid, work 1.2e4, 11 us per iteration in one workgroup against 24 us
// flooded; 32x32, 8.3e4: 61 against 22 us)
constexpr double kBpMultiWork = 32768.0;

static int sum_product_flood(bnpp_ctx *ctx, const ModelData &d, int max_iter, double eps, double *out,
                             int *iterations, double *uptime_ms, double t0) {
    const int nv = (int)d.cards.size(), nf = (int)d.scopes.size();
    std::vector<int32_t> f_edge_off(nf + 1, 0), edge_var, edge_fac, msg_off(1, 0), item_edge, v_edge_off(nv + 1, 0),
        v_edges, marg_off(nv + 1, 0);
    std::vector<uint64_t> edge_stride;
    std::vector<int64_t> tab_off(nf + 1, 0);
    for (int f = 0; f < nf; ++f) {
        const std::vector<int> &sc = d.scopes[f];
        uint64_t size = 1;
        for (int v : sc) size *= (uint64_t)d.cards[v];
        uint64_t st = size;
        for (size_t j = 0; j < sc.size(); ++j) {
            st /= (uint64_t)d.cards[sc[j]];
            const int e = (int)edge_var.size();
            edge_var.push_back(sc[j]);
            edge_fac.push_back(f);
            edge_stride.push_back(st);
            for (int x = 0; x < d.cards[sc[j]]; ++x) item_edge.push_back(e);
            if ((int64_t)msg_off.back() + d.cards[sc[j]] >= INT32_MAX)
                return set_err(BNPP_ERR_UNSUPPORTED, "sum-product: more than 2^31 message entries");
            msg_off.push_back(msg_off.back() + d.cards[sc[j]]);
            ++v_edge_off[sc[j] + 1];
        }
        f_edge_off[f + 1] = (int32_t)edge_var.size();
        tab_off[f + 1] = tab_off[f] + (int64_t)size;
    }
    const int ne = (int)edge_var.size(), nmsg = msg_off.back();
    for (int v = 0; v < nv; ++v) {
        v_edge_off[v + 1] += v_edge_off[v];
        marg_off[v + 1] = marg_off[v] + d.cards[v];
    }
    v_edges.resize(ne);
    {
        std::vector<int32_t> fill(v_edge_off.begin(), v_edge_off.end() - 1);
        for (int e = 0; e < ne; ++e) v_edges[fill[edge_var[e]]++] = msg_off[e];   // ascending edge = factor id
    }
    // segments in entry order, then their lane classes
    std::vector<int64_t> seg_off(nmsg + 1, 0);
    for (int t = 0; t < nmsg; ++t) {
        const int e = item_edge[t];
        const uint64_t terms = (uint64_t)(tab_off[edge_fac[e] + 1] - tab_off[edge_fac[e]]) / d.cards[edge_var[e]];
        seg_off[t + 1] = seg_off[t] + (int64_t)std::max<uint64_t>(1, (terms + kBpSegTerms - 1) / kBpSegTerms);
    }
    const int64_t nseg = seg_off[nmsg];
    if (nseg >= INT32_MAX) return set_err(BNPP_ERR_UNSUPPORTED, "sum-product: more than 2^31 segments");
    std::vector<int32_t> seg_item(nseg), cls[4];
    std::vector<uint64_t> seg_q0(nseg);
    for (int t = 0; t < nmsg; ++t) {
        const int e = item_edge[t];
        const uint64_t terms = (uint64_t)(tab_off[edge_fac[e] + 1] - tab_off[edge_fac[e]]) / d.cards[edge_var[e]];
        for (int64_t s = seg_off[t]; s < seg_off[t + 1]; ++s) {
            const uint64_t q0 = (uint64_t)(s - seg_off[t]) * kBpSegTerms;
            seg_item[s] = t;
            seg_q0[s] = q0;
            cls[bp_lane_class((int64_t)std::min<uint64_t>(kBpSegTerms, terms - std::min(q0, terms)))].push_back((int32_t)s);
        }
    }
    std::vector<int32_t> cls_seg;
    cls_seg.reserve(nseg);
    BpFlood a{};
    const int lanes[4] = {1, 4, 16, 64};
    for (int c = 0; c < 4; ++c) {
        a.cls_pos[c] = (int64_t)cls_seg.size();
        cls_seg.insert(cls_seg.end(), cls[c].begin(), cls[c].end());
        a.cls_pos[c + 1] = (int64_t)cls_seg.size();
        const int64_t per_block = kBpFloodBlock / lanes[c];
        const int64_t blocks = ((int64_t)cls[c].size() + per_block - 1) / per_block;
        if ((int64_t)a.cls_blk[c] + blocks >= INT32_MAX) return set_err(BNPP_ERR_UNSUPPORTED, "sum-product: grid too large");
        a.cls_blk[c + 1] = a.cls_blk[c] + (int32_t)blocks;
    }
    // device block: index arrays (256-B aligned pieces), tables, messages
    size_t off = 0;
    auto place = [&](size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_cards = place(4 * (size_t)nv), o_tab_off = place(8 * (size_t)(nf + 1)),
                 o_feo = place(4 * (size_t)(nf + 1)), o_ev = place(4 * (size_t)ne), o_ef = place(4 * (size_t)ne),
                 o_es = place(8 * (size_t)ne), o_mo = place(4 * (size_t)(ne + 1)), o_ie = place(4 * (size_t)nmsg),
                 o_so = place(8 * (size_t)(nmsg + 1)), o_si = place(4 * (size_t)nseg), o_sq = place(8 * (size_t)nseg),
                 o_cs = place(4 * (size_t)nseg), o_veo = place(4 * (size_t)(nv + 1)), o_ve = place(4 * (size_t)ne),
                 o_mgo = place(4 * (size_t)(nv + 1));
    const size_t idx_bytes = off;
    const size_t o_tabs = place(8 * (size_t)tab_off[nf]);
    const size_t o_v2f = place(8 * (size_t)nmsg), o_f2v = place(8 * (size_t)nmsg), o_raw = place(8 * (size_t)nmsg),
                 o_part = place(8 * (size_t)nseg), o_marg = place(8 * (size_t)marg_off[nv]),
                 o_err = place(8 * (size_t)kBpErrRing);
    std::vector<unsigned char> host(idx_bytes);
    auto put = [&](size_t o, const void *src, size_t bytes) {
        if (bytes) std::memcpy(host.data() + o, src, bytes);
    };
    std::vector<int32_t> cards32(d.cards.begin(), d.cards.end());
    put(o_cards, cards32.data(), 4 * (size_t)nv);
    put(o_tab_off, tab_off.data(), 8 * tab_off.size());
    put(o_feo, f_edge_off.data(), 4 * f_edge_off.size());
    put(o_ev, edge_var.data(), 4 * (size_t)ne);
    put(o_ef, edge_fac.data(), 4 * (size_t)ne);
    put(o_es, edge_stride.data(), 8 * (size_t)ne);
    put(o_mo, msg_off.data(), 4 * msg_off.size());
    put(o_ie, item_edge.data(), 4 * (size_t)nmsg);
    put(o_so, seg_off.data(), 8 * seg_off.size());
    put(o_si, seg_item.data(), 4 * (size_t)nseg);
    put(o_sq, seg_q0.data(), 8 * (size_t)nseg);
    put(o_cs, cls_seg.data(), 4 * (size_t)nseg);
    put(o_veo, v_edge_off.data(), 4 * v_edge_off.size());
    put(o_ve, v_edges.data(), 4 * (size_t)ne);
    put(o_mgo, marg_off.data(), 4 * marg_off.size());

    hipStream_t s = ctx->c.stream;
    unsigned char *dev = nullptr;
    if (hipSetDevice(ctx->c.device) != hipSuccess) return set_err(BNPP_ERR_HIP, "sum-product: hipSetDevice");
    if (hipMalloc(&dev, off) != hipSuccess) return set_err(BNPP_ERR_OOM, "sum-product: device allocation");
    struct Free {
        unsigned char *p;
        ~Free() { (void)hipFree(p); }
    } guard{dev};
    a.n_vars = nv;
    a.n_edges = ne;
    a.n_msg = nmsg;
    a.idx64 = std::getenv("BNPP_BP_IDX64") ? 1 : 0;
    a.one_seg = nseg == nmsg ? 1 : 0;
    a.eps = eps;
    a.cards = reinterpret_cast<const int32_t *>(dev + o_cards);
    a.tables = reinterpret_cast<const double *>(dev + o_tabs);
    a.tab_off = reinterpret_cast<const int64_t *>(dev + o_tab_off);
    a.f_edge_off = reinterpret_cast<const int32_t *>(dev + o_feo);
    a.edge_var = reinterpret_cast<const int32_t *>(dev + o_ev);
    a.edge_fac = reinterpret_cast<const int32_t *>(dev + o_ef);
    a.edge_stride = reinterpret_cast<const uint64_t *>(dev + o_es);
    a.msg_off = reinterpret_cast<const int32_t *>(dev + o_mo);
    a.item_edge = reinterpret_cast<const int32_t *>(dev + o_ie);
    a.seg_off = reinterpret_cast<const int64_t *>(dev + o_so);
    a.seg_item = reinterpret_cast<const int32_t *>(dev + o_si);
    a.seg_q0 = reinterpret_cast<const uint64_t *>(dev + o_sq);
    a.cls_seg = reinterpret_cast<const int32_t *>(dev + o_cs);
    a.v_edge_off = reinterpret_cast<const int32_t *>(dev + o_veo);
    a.v_moff = reinterpret_cast<const int32_t *>(dev + o_ve);
    a.marg_off = reinterpret_cast<const int32_t *>(dev + o_mgo);
    a.v2f = reinterpret_cast<double *>(dev + o_v2f);
    a.f2v = reinterpret_cast<double *>(dev + o_f2v);
    a.raw = reinterpret_cast<double *>(dev + o_raw);
    a.part = reinterpret_cast<double *>(dev + o_part);
    a.marg = reinterpret_cast<double *>(dev + o_marg);
    a.err = reinterpret_cast<unsigned long long *>(dev + o_err);
    hipError_t e = hipMemcpyAsync(dev, host.data(), idx_bytes, hipMemcpyHostToDevice, s);
    // tables: small ones gathered into a bounded staging buffer (one copy per
    // 256 MB: a grid has ~10^5 factors, and a copy per factor costs ~3 us of
    // host time), tables of 64 MB and more copied straight from the model
    {
        constexpr size_t kStage = (size_t)256 << 20, kDirect = (size_t)64 << 20;
        std::vector<unsigned char> stage;
        size_t at = o_tabs;                                   // device offset of stage[0]
        auto flush = [&]() {
            if (!stage.empty() && e == hipSuccess) {
                e = hipMemcpyAsync(dev + at, stage.data(), stage.size(), hipMemcpyHostToDevice, s);
                if (e == hipSuccess) e = hipStreamSynchronize(s);      // stage is reused
            }
            at += stage.size();
            stage.clear();
        };
        for (int f = 0; f < nf && e == hipSuccess; ++f) {
            const size_t bytes = 8 * d.values[f].size();
            if (bytes >= kDirect) {
                flush();
                e = hipMemcpyAsync(dev + at, d.values[f].data(), bytes, hipMemcpyHostToDevice, s);
                at += bytes;
                continue;
            }
            if (stage.size() + bytes > kStage) flush();
            const unsigned char *p = reinterpret_cast<const unsigned char *>(d.values[f].data());
            stage.insert(stage.end(), p, p + bytes);
        }
        flush();
    }
    if (e == hipSuccess) e = hipMemsetAsync(a.err, 0, 8 * (size_t)kBpErrRing, s);
    if (e == hipSuccess) e = launch_bp_flood_init(a, s);
    int it_done = max_iter;
    std::vector<unsigned long long> chunk(kBpErrChunk);
    for (int c = 0; e == hipSuccess && (int64_t)c * kBpErrChunk < max_iter; ++c) {
        const int it0 = c * kBpErrChunk, it1 = std::min(max_iter, it0 + kBpErrChunk);
        unsigned long long *half = a.err + (c % 2) * kBpErrChunk;
        e = hipMemsetAsync(half, 0, 8 * (size_t)kBpErrChunk, s);
        for (int it = it0; it < it1 && e == hipSuccess; ++it) e = launch_bp_flood_iteration(a, it, s);
        if (e == hipSuccess) e = hipMemcpyAsync(chunk.data(), half, 8 * (size_t)(it1 - it0), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        bool done = false;
        for (int it = it0; e == hipSuccess && it < it1; ++it) {
            double m;
            std::memcpy(&m, &chunk[it - it0], 8);
            if (m < eps) {                        // graph.cpp:328
                it_done = it;
                done = true;
                break;
            }
        }
        if (done) break;
    }
    if (e == hipSuccess) e = launch_bp_flood_marginals(a, s);
    if (e == hipSuccess) e = hipMemcpyAsync(out, a.marg, 8 * (size_t)marg_off[nv], hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return set_err(BNPP_ERR_HIP, std::string("sum-product: ") + hipGetErrorString(e));
    if (iterations) *iterations = it_done;
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return BNPP_OK;
}

// BN::marginals with options["sum-product"] (model.cpp:313-317): loopy BP on
// the factor graph of the model's own factors (evidence is not used on this
// path, as in the reference), FactorGraph::update(max_iter, eps) then one
// marginal per variable (graph.cpp:256-403).  One workgroup runs the whole
// loop (bp.hip) unless the iteration's work calls for the multi-workgroup
// flood above.
int bnpp_sum_product(bnpp_ctx *ctx, const bnpp_model *m, int max_iter, double eps, double *out, int *iterations,
                     double *uptime_ms) {
    BNPP_GUARD_BEGIN
    if (!ctx || !m || !out) return set_err(BNPP_ERR_INVALID, "null argument");
    if (max_iter < 0) return set_err(BNPP_ERR_INVALID, "max_iter must be >= 0");
    const double t0 = now_ms();
    const ModelData &d = m->d;
    const int nv = (int)d.cards.size(), nf = (int)d.scopes.size();
    // one workgroup for the whole loop, or one launch per phase and iteration
    // (BNPP_BP_MODE=single|multi overrides the choice by work per iteration)
    bool big_table = false;
    double work = 0.0;
    {
        std::vector<double> deg(nv, 0.0);
        for (int f = 0; f < nf; ++f) {
            double size = 1.0;
            for (int v : d.scopes[f]) {
                size *= d.cards[v];
                deg[v] += 1.0;
            }
            const double m = (double)d.scopes[f].size();
            work += size * m * m;
            big_table |= size >= 2147483648.0;
        }
        for (int v = 0; v < nv; ++v) work += deg[v] * deg[v] * d.cards[v];
    }
    const char *mode = std::getenv("BNPP_BP_MODE");
    bool multi = big_table || work > kBpMultiWork;
    if (mode && !std::strcmp(mode, "multi")) multi = true;
    if (mode && !std::strcmp(mode, "single")) {
        if (big_table) return set_err(BNPP_ERR_UNSUPPORTED, "sum-product: one-workgroup loop needs tables < 2^31 entries");
        multi = false;
    }
    if (multi) return sum_product_flood(ctx, d, max_iter, eps, out, iterations, uptime_ms, t0);
    // host image of every input array, laid out as on the device
    std::vector<int32_t> f_edge_off(nf + 1, 0), edge_var, edge_fac, msg_off(1, 0), item_edge, v_edge_off(nv + 1, 0),
        v_edges, marg_off(nv + 1, 0);
    std::vector<uint32_t> edge_stride;
    std::vector<int64_t> tab_off(nf + 1, 0);
    for (int f = 0; f < nf; ++f) {
        const std::vector<int> &sc = d.scopes[f];
        int64_t size = 1;
        for (int v : sc) size *= d.cards[v];
        int64_t st = size;
        for (size_t j = 0; j < sc.size(); ++j) {
            st /= d.cards[sc[j]];
            const int e = (int)edge_var.size();
            edge_var.push_back(sc[j]);
            edge_fac.push_back(f);
            edge_stride.push_back((uint32_t)st);
            for (int x = 0; x < d.cards[sc[j]]; ++x) item_edge.push_back(e);
            msg_off.push_back(msg_off.back() + d.cards[sc[j]]);
            ++v_edge_off[sc[j] + 1];
        }
        f_edge_off[f + 1] = (int32_t)edge_var.size();
        tab_off[f + 1] = tab_off[f] + size;
    }
    const int ne = (int)edge_var.size(), nmsg = msg_off.back();
    std::vector<int32_t> cls[4], cls_items;
    for (int t = 0; t < nmsg; ++t) {
        const int e = item_edge[t];
        cls[bp_lane_class((tab_off[edge_fac[e] + 1] - tab_off[edge_fac[e]]) / d.cards[edge_var[e]])].push_back(t);
    }
    int32_t cls_off[5] = {0};
    for (int c = 0; c < 4; ++c) {
        cls_items.insert(cls_items.end(), cls[c].begin(), cls[c].end());
        cls_off[c + 1] = (int32_t)cls_items.size();
    }
    for (int v = 0; v < nv; ++v) {
        v_edge_off[v + 1] += v_edge_off[v];
        marg_off[v + 1] = marg_off[v] + d.cards[v];
    }
    v_edges.resize(ne);
    {
        std::vector<int32_t> fill(v_edge_off.begin(), v_edge_off.end() - 1);
        for (int e = 0; e < ne; ++e) v_edges[fill[edge_var[e]]++] = e;     // ascending edge = factor id
    }
    // one device block: inputs, then messages and outputs (256-B aligned pieces)
    std::vector<unsigned char> host;
    size_t off = 0;
    auto place = [&](size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t o_cards = place(4 * (size_t)nv), o_tabs = place(8 * (size_t)tab_off[nf]),
                 o_tab_off = place(8 * (size_t)(nf + 1)), o_feo = place(4 * (size_t)(nf + 1)),
                 o_ev = place(4 * (size_t)ne), o_ef = place(4 * (size_t)ne), o_es = place(4 * (size_t)ne),
                 o_mo = place(4 * (size_t)(ne + 1)), o_ie = place(4 * (size_t)nmsg), o_veo = place(4 * (size_t)(nv + 1)),
                 o_ve = place(4 * (size_t)ne), o_mgo = place(4 * (size_t)(nv + 1)),
                 o_ci = place(4 * cls_items.size());
    const size_t in_bytes = off;
    const size_t o_v2f = place(8 * (size_t)nmsg), o_f2v = place(8 * (size_t)nmsg), o_raw = place(8 * (size_t)nmsg),
                 o_marg = place(8 * (size_t)marg_off[nv]), o_it = place(4);
    host.resize(in_bytes);
    auto put = [&](size_t o, const void *src, size_t bytes) {
        if (bytes) std::memcpy(host.data() + o, src, bytes);
    };
    std::vector<int32_t> cards32(d.cards.begin(), d.cards.end());
    put(o_cards, cards32.data(), 4 * (size_t)nv);
    for (int f = 0; f < nf; ++f) put(o_tabs + 8 * (size_t)tab_off[f], d.values[f].data(), 8 * d.values[f].size());
    put(o_tab_off, tab_off.data(), 8 * tab_off.size());
    put(o_feo, f_edge_off.data(), 4 * f_edge_off.size());
    put(o_ev, edge_var.data(), 4 * (size_t)ne);
    put(o_ef, edge_fac.data(), 4 * (size_t)ne);
    put(o_es, edge_stride.data(), 4 * (size_t)ne);
    put(o_mo, msg_off.data(), 4 * msg_off.size());
    put(o_ie, item_edge.data(), 4 * (size_t)nmsg);
    put(o_veo, v_edge_off.data(), 4 * v_edge_off.size());
    put(o_ve, v_edges.data(), 4 * (size_t)ne);
    put(o_mgo, marg_off.data(), 4 * marg_off.size());
    put(o_ci, cls_items.data(), 4 * cls_items.size());

    hipStream_t s = ctx->c.stream;
    unsigned char *dev = nullptr;
    if (hipSetDevice(ctx->c.device) != hipSuccess) return set_err(BNPP_ERR_HIP, "sum-product: hipSetDevice");
    if (hipMalloc(&dev, off) != hipSuccess) return set_err(BNPP_ERR_OOM, "sum-product: device allocation");
    struct Free {
        unsigned char *p;
        ~Free() { (void)hipFree(p); }
    } guard{dev};
    BpArgs a{};
    a.n_vars = nv;
    a.n_edges = ne;
    a.n_msg = nmsg;
    a.max_iter = max_iter;
    a.eps = eps;
    a.cards = reinterpret_cast<const int32_t *>(dev + o_cards);
    a.tables = reinterpret_cast<const double *>(dev + o_tabs);
    a.tab_off = reinterpret_cast<const int64_t *>(dev + o_tab_off);
    a.f_edge_off = reinterpret_cast<const int32_t *>(dev + o_feo);
    a.edge_var = reinterpret_cast<const int32_t *>(dev + o_ev);
    a.edge_fac = reinterpret_cast<const int32_t *>(dev + o_ef);
    a.edge_stride = reinterpret_cast<const uint32_t *>(dev + o_es);
    a.msg_off = reinterpret_cast<const int32_t *>(dev + o_mo);
    a.item_edge = reinterpret_cast<const int32_t *>(dev + o_ie);
    for (int c = 0; c < 5; ++c) a.cls_off[c] = cls_off[c];
    a.cls_items = reinterpret_cast<const int32_t *>(dev + o_ci);
    a.msgs_in_lds = nmsg <= kBpLdsMsgMax && !std::getenv("BNPP_BP_NO_LDS");
    a.v_edge_off = reinterpret_cast<const int32_t *>(dev + o_veo);
    a.v_edges = reinterpret_cast<const int32_t *>(dev + o_ve);
    a.marg_off = reinterpret_cast<const int32_t *>(dev + o_mgo);
    a.v2f = reinterpret_cast<double *>(dev + o_v2f);
    a.f2v = reinterpret_cast<double *>(dev + o_f2v);
    a.raw = reinterpret_cast<double *>(dev + o_raw);
    a.marg = reinterpret_cast<double *>(dev + o_marg);
    a.iterations = reinterpret_cast<int32_t *>(dev + o_it);
    int32_t it = 0;
    hipError_t e = hipMemcpyAsync(dev, host.data(), in_bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = launch_sum_product(a, s);
    if (e == hipSuccess) e = hipMemcpyAsync(out, a.marg, 8 * (size_t)marg_off[nv], hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&it, a.iterations, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return set_err(BNPP_ERR_HIP, std::string("sum-product: ") + hipGetErrorString(e));
    if (iterations) *iterations = it;
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return BNPP_OK;
    BNPP_GUARD_END
}

}  // extern "C"
