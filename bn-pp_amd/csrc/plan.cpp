// Host-side planning: scope rules, descriptor compilation, symbolic VE, schedule.
#include "plan.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <map>
#include <memory_resource>
#include <set>
#include <thread>
#include <unistd.h>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>

namespace bnpp {

// Persistent host workers (spawning 15 threads per call cost ~1 ms of a
// millisecond-scale PR plan).  One parallel_for at a time uses the pool; a
// concurrent call (another context's thread) runs on threads of its own, a
// nested one (a body that itself calls parallel_for) serially.
namespace {
struct HostPool {
    std::mutex run_mu;                         // held by the one call using the pool
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::vector<std::thread> workers;
    const std::function<void(int64_t)> *body = nullptr;
    std::atomic<int64_t> next{0};
    int64_t n = 0;
    uint64_t gen = 0;
    int want = 0, active = 0;
    bool stop = false;
    static thread_local bool in_worker;
    explicit HostPool(int nw) {
        for (int i = 0; i < nw; ++i) workers.emplace_back([this, i] { loop(i); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : workers) t.join();
    }
    void drain() {
        for (int64_t i = next++; i < n; i = next++) (*body)(i);
    }
    void loop(int id) {
        in_worker = true;
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || (gen != seen && id < want); });
            if (stop) return;
            seen = gen;
            lk.unlock();
            drain();
            lk.lock();
            if (--active == 0) done_cv.notify_all();
        }
    }
    void run(int64_t count, const std::function<void(int64_t)> &fn, int helpers) {
        {
            std::lock_guard<std::mutex> g(mu);
            body = &fn;
            n = count;
            next = 0;
            want = helpers;
            active = helpers;
            ++gen;
        }
        cv.notify_all();
        in_worker = true;                      // the caller drains too: its nested calls run serially
        drain();
        in_worker = false;
        std::unique_lock<std::mutex> lk(mu);
        done_cv.wait(lk, [&] { return active == 0; });
        body = nullptr;
    }
};
thread_local bool HostPool::in_worker = false;
}  // namespace

thread_local int t_host_threads = 0;            // ScopedHostThreads

void parallel_for(int64_t n, const std::function<void(int64_t)> &body, int threads) {
    if (threads <= 0) threads = t_host_threads;
    if (threads <= 0) {
        threads = (int)std::thread::hardware_concurrency();
        if (const char *e = std::getenv("BNPP_HOST_THREADS")) threads = std::atoi(e);
        threads = std::max(1, std::min(threads, 16));
    }
    // a body already running on the pool (a worker, or the calling thread
    // draining with them) loops serially: the pool's threads are busy with
    // the outer loop, and spawning more per nested call oversubscribes the
    // host (eight parallel slot probes each splitting their own loops)
    if (n <= 1 || threads == 1 || HostPool::in_worker) {
        for (int64_t i = 0; i < n; ++i) body(i);
        return;
    }
    const int nt = (int)std::min<int64_t>(threads, n);
    // never destroyed (workers may outlive static teardown); a forked child
    // has the object but not its threads, so it uses threads of its own
    static HostPool *pool = new HostPool(15);
    static const pid_t pool_pid = getpid();
    if (!HostPool::in_worker && nt - 1 <= (int)pool->workers.size() && getpid() == pool_pid) {
        std::unique_lock<std::mutex> g(pool->run_mu, std::try_to_lock);
        if (g.owns_lock()) {
            pool->run(n, body, nt - 1);
            return;
        }
    }
    std::atomic<int64_t> next(0);
    auto worker = [&]() {
        for (int64_t i = next++; i < n; i = next++) body(i);
    };
    std::vector<std::thread> extra;
    for (int t = 1; t < nt; ++t) extra.emplace_back(worker);
    worker();
    for (auto &t : extra) t.join();
}

std::vector<int64_t> natural_strides(const std::vector<int> &vars, const std::vector<int> &cards) {
    std::vector<int64_t> s(vars.size());
    int64_t acc = 1;
    for (int i = (int)vars.size() - 1; i >= 0; --i) {
        s[i] = acc;
        acc = sat_mul(acc, cards[vars[i]]);
    }
    return s;
}

int64_t table_size(const std::vector<int> &vars, const std::vector<int> &cards) {
    int64_t s = 1;
    for (int v : vars) s = sat_mul(s, cards[v]);
    return s;
}

View natural_view(int table, const std::vector<int> &vars, const std::vector<int> &cards) {
    View v;
    v.table = table;
    v.vars = vars;
    v.strides = natural_strides(vars, cards);
    return v;
}

View conditioned_view(int table, const std::vector<int> &vars, const std::vector<int> &cards,
                      const std::vector<int> &ev_val) {
    std::vector<int64_t> st = natural_strides(vars, cards);
    View v;
    v.table = table;
    for (size_t i = 0; i < vars.size(); ++i) {
        int e = vars[i] < (int)ev_val.size() ? ev_val[vars[i]] : -1;
        if (e >= 0) {
            v.base += (int64_t)e * st[i];
        } else {
            v.vars.push_back(vars[i]);
            v.strides.push_back(st[i]);
        }
    }
    return v;
}

static bool contains(const std::vector<int> &s, int v) { return std::find(s.begin(), s.end(), v) != s.end(); }

std::vector<int> union_scope(const std::vector<int> &a, const std::vector<int> &b) {
    std::vector<int> u = a;
    for (int v : b)
        if (!contains(a, v)) u.push_back(v);
    return u;
}

std::vector<int> chain_scope(const std::vector<View> &in) {
    std::vector<int> u;                      // Factor(1.0) has the empty scope
    for (const View &v : in) u = union_scope(u, v.vars);
    return u;
}

std::vector<int> remove_var(const std::vector<int> &s, int v) {
    std::vector<int> r;
    for (int x : s)
        if (x != v) r.push_back(x);
    return r;
}

namespace {
struct Dim {
    uint64_t card;
    int64_t s[kMaxIn];
};

void magic_for(uint32_t d, uint32_t &shift, uint32_t &magic, bool &pow2) {
    pow2 = (d & (d - 1)) == 0;
    uint32_t l = 0;
    while (((uint64_t)1 << l) < d) ++l;
    shift = l;
    if (pow2) {
        magic = 0;
    } else {
        magic = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
    }
}
}  // namespace

// Descriptor of a fused chain run (chain.cuh).  Returns false when the run's
// layout fits neither kernel form.
static bool build_chain_desc(const BucketSpec &b, const std::vector<int> &cards, int max_vec, BucketDesc &d,
                             std::vector<int64_t> &pool, std::string *msg) {
    auto fail = [&](const char *m) {
        if (msg) *msg = m;
        return false;
    };
    const int F = (int)b.chain_x.size();
    if (F < 1 || (int)b.chain_n.size() != F || b.in.empty()) return fail("chain: bad run");
    const int K = cards[b.chain_x[0]];
    const int eb = max_vec == 2 ? 8 : 4;
    const bool sum = b.chain_n[0] < 0;                // every bucket only sums (no new variable)
    int N = 1;
    for (int j = 0; j < F; ++j) {
        if ((b.chain_n[j] < 0) != sum) return fail("chain: mixed summing and swapping buckets");
        if (cards[b.chain_x[j]] != K || (!sum && cards[b.chain_n[j]] != K)) return fail("chain: mixed cardinalities");
        N *= K;
    }
    // split form (chainsplit.cuh): binary runs of 5..8 buckets over 2^(F-4)
    // waves (fp64 runs of 8 without a fused belief)
    const char *nsp = std::getenv("BNPP_NO_SPLIT");
    const char *smf = std::getenv("BNPP_SPLIT_MIN_F");
    const int split_min = smf ? std::max(5, std::atoi(smf)) : 5;
    const bool split_ok = !(nsp && *nsp == '1') && K == 2 && F >= split_min && F <= split_max_f(eb);
    if ((N > 64 && !split_ok) || (K != 2 && K != 4)) return fail("chain: register table too large");
    std::vector<int> gidx(F, -1);                     // input index of G_j (-1: absent)
    int ni = 1;
    for (int j = 0; j < F; ++j)
        if ((b.chain_gmask >> j) & 1) gidx[j] = ni++;
    const int nb = b.bel_table >= 0 ? 1 : 0;          // the belief's forward message follows the G tables
    if (ni + nb != (int)b.in.size() || ni + nb > kMaxDescIn) return fail("chain: G tables do not match the mask");
    if (ni > kMaxIn && !split_ok) return fail("chain: more than 8 inputs need the split form");
    auto stride_of = [](const View &v, int var) -> int64_t {
        for (size_t i = 0; i < v.vars.size(); ++i)
            if (v.vars[i] == var) return v.strides[i];
        return 0;
    };
    const View &big = b.in[0];
    std::vector<int64_t> ostr = natural_strides(b.out_vars, cards);
    auto out_stride = [&](int var) -> int64_t {
        for (size_t i = 0; i < b.out_vars.size(); ++i)
            if (b.out_vars[i] == var) return ostr[i];
        return -1;
    };
    std::vector<int64_t> is(F), os(F);
    for (int p = 0; p < F; ++p) {
        is[p] = stride_of(big, b.chain_x[p]);
        os[p] = sum ? 0 : out_stride(b.chain_n[p]);
        if (is[p] <= 0 || os[p] < 0) return fail("chain: slot variable missing");
    }
    // rest dims (fastest first by output stride): in, out, G_j strides
    struct RDim { uint64_t card; int64_t in, out; int64_t g[8]; };
    std::vector<RDim> rd;
    for (size_t i = b.out_vars.size(); i-- > 0;) {
        const int v = b.out_vars[i];
        if (std::find(b.chain_n.begin(), b.chain_n.end(), v) != b.chain_n.end() || cards[v] == 1) continue;
        RDim r{(uint64_t)cards[v], stride_of(big, v), ostr[i], {0}};
        if (r.in == 0) return fail("chain: rest variable missing from the message");
        for (int j = 0; j < F; ++j) r.g[j] = gidx[j] >= 0 ? stride_of(b.in[gidx[j]], v) : 0;
        rd.push_back(r);
    }
    std::vector<RDim> md;                             // merged
    for (const RDim &r : rd) {
        if (!md.empty()) {
            RDim &bk = md.back();
            const int64_t c = (int64_t)bk.card;
            bool ok = bk.card * r.card <= (uint64_t)INT32_MAX && r.in == bk.in * c && r.out == bk.out * c;
            for (int j = 0; ok && j < F; ++j) ok = r.g[j] == bk.g[j] * c;
            if (ok) {
                bk.card *= r.card;
                continue;
            }
        }
        md.push_back(r);
    }
    int64_t rest = 1;
    for (const RDim &r : md) rest = sat_mul(rest, (int64_t)r.card);
    if (rest >= (kSatMax >> 8)) return fail("chain: message beyond any device");
    // kernel form
    int form = 0, V = 1;
    bool fwd_v = false;
    bool fwd = false, bwd = false;                    // one-thread forms fit (the split forms' fallbacks)
    int bv = 1;
    if (sum) {
        // summing run: the thread's V rest entries are contiguous in the input
        // (vector loads, one per slot assignment) and in the output
        V = 16 / eb;
        const int64_t W = V;
        bool ok = !md.empty() && md[0].in == 1 && md[0].out == 1 && md[0].card % (uint64_t)V == 0 &&
                  big.base % W == 0 && rest >= 256 * V;
        for (const RDim &r : md) ok = ok && (r.in % W == 0 || &r == &md[0]) && (r.out % W == 0 || &r == &md[0]);
        for (int p = 0; ok && p < F; ++p) ok = is[p] % W == 0;
        for (int j = 0; ok && j < F; ++j) ok = md[0].g[j] == 0;
        if (!ok) return fail("chain: summing run layout fits no kernel form");
        form = kChainSum;
    } else {
        fwd = N * eb <= 256;                         // rows staged through LDS in 128-B parts
        for (int p = 0; fwd && p < F; ++p) {
            int64_t pl = 1;
            for (int q = p + 1; q < F; ++q) pl *= K;
            fwd = os[p] == pl;
        }
        if (fwd && !md.empty()) fwd = md[0].out == N;
        bwd = true;
        const int W = eb == 4 ? (N % 4 == 0 ? 4 : N % 2 == 0 ? 2 : 1) : (N % 2 == 0 ? 2 : 1);   // load_n width
        bv = chain_bwd_v(N, eb);
        int64_t pk = 1;
        for (int p = 0; bwd && p < F; ++p, pk *= K) bwd = is[p] == pk;
        bwd = bwd && !md.empty() && md[0].out == 1 && md[0].card % (uint64_t)bv == 0 && big.base % W == 0;
        if (bv == 1) bwd = bwd && !md.empty() && md[0].out == 1;
        for (const RDim &r : md) bwd = bwd && r.in % W == 0 && (r.out % bv == 0 || &r == &md[0]);
        for (int p = 0; bwd && p < F; ++p) bwd = os[p] % bv == 0;
        for (int j = 0; bwd && bv > 1 && j < F; ++j) bwd = md[0].g[j] == 0;   // G constant along a thread's V entries
        // V-wide forward: the thread's V rest entries contiguous in input and
        // output (rest dim 0 innermost in the input), G constant along them
        const int fv = chain_fwd_v(N, eb);
        fwd_v = fwd && fv > 1 && !md.empty() && md[0].in == 1 && md[0].card % (uint64_t)fv == 0 &&
                big.base % fv == 0 && rest >= 256 * fv;
        for (const RDim &r : md) fwd_v = fwd_v && (r.in % fv == 0 || &r == &md[0]);
        for (int p = 0; fwd_v && p < F; ++p) fwd_v = is[p] % fv == 0;
        for (int j = 0; fwd_v && j < F; ++j) fwd_v = md[0].g[j] == 0;
        // split forms: 64 consecutive rest entries per workgroup along rest dim 0;
        // forward rows contiguous (2^F entries, slot 0 slowest), backward rows
        // read by 16-B loads (slot 0 fastest), slab stores along rest dim 0
        bool fwd_s = split_ok && !md.empty() && md[0].card % (uint64_t)kSplitRowsHost == 0 && md[0].out == N;
        for (int p = 0; fwd_s && p < F; ++p) fwd_s = os[p] == ((int64_t)1 << (F - 1 - p));
        bool bwd_s = split_ok && !md.empty() && md[0].card % (uint64_t)kSplitRowsHost == 0 && md[0].out == 1 &&
                     big.base % 4 == 0;
        for (int p = 0; bwd_s && p < F; ++p) bwd_s = is[p] == ((int64_t)1 << p);
        for (const RDim &r : md) bwd_s = bwd_s && r.in % 4 == 0;
        // every bucket of a split run has its G table (no summing-only steps)
        if (b.chain_gmask != (1 << F) - 1) fwd_s = bwd_s = false;
        if (fwd_s) form = kChainFwdS;
        else if (bwd_s) form = kChainBwdS;
        else if (N > 64) return fail("chain: split form does not fit the layout");
        else if (fwd) form = kChainFwd;
        else if (bwd) { form = kChainBwd; V = bv; }
        else return fail("chain: layout fits no kernel form");
    }
    // which other slot each G_j varies with (ChainDep)
    int dep = kDepAny;
    {
        bool next = true, prev = true;
        for (int j = 0; j < F; ++j) {
            if (gidx[j] < 0) continue;
            for (int p = 0; p < F; ++p) {
                if (p == j) continue;
                const int var = p < j ? b.chain_n[p] : b.chain_x[p];
                if (var < 0 || stride_of(b.in[gidx[j]], var) == 0) continue;
                if (p != j + 1) next = false;
                if (p != j - 1) prev = false;
            }
        }
        dep = next ? kDepNext : prev ? kDepPrev : kDepAny;
    }
    // split forms stage G_j packed (kSplitPack entries per base offset)
    int64_t g_pk = 0;
    for (int i = 1; i < ni; ++i) {
        int64_t sp = 1;
        for (size_t q = 0; q < b.in[i].vars.size(); ++q) sp += (int64_t)(cards[b.in[i].vars[q]] - 1) * b.in[i].strides[q];
        g_pk += sp * kSplitPack;
    }
    const bool pk_fits = g_pk * eb <= split_g_budget_bytes(F, eb);
    if (chain_split_form(form) && (dep == kDepAny || !pk_fits)) {
        if (N > 64) return fail(pk_fits ? "chain: split form needs G_j to depend on one neighbouring slot"
                                        : "chain: packed G tables exceed the split form's LDS");
        // the one-thread form, only where its own layout conditions hold
        if (form == kChainFwdS) {
            if (!fwd) return fail("chain: split forward run falls back to a layout the one-thread form rejects");
            form = kChainFwd;
        } else {
            if (!bwd) return fail("chain: split backward run falls back to a layout the one-thread form rejects");
            form = kChainBwd;
            V = bv;
        }
    }
    // dense addressing (chainsplit.cuh DENSE): rest of <= 2 dims, dim 0 a power
    // of two contiguous on the streamed side, G constant along it, slot strides
    // one dense block
    if (form == kChainFwdS || form == kChainBwdS) {
        const bool fw = form == kChainFwdS;
        const char *nd = std::getenv("BNPP_NO_DENSE");
        bool dense = !(nd && *nd == '1') && !md.empty() && md.size() <= 2 && md[0].card >= (uint64_t)kSplitRowsHost &&
                     (md[0].card & (md[0].card - 1)) == 0 && (fw ? md[0].in == 1 : md[0].in == N);
        for (int j = 0; dense && j < F; ++j) dense = md[0].g[j] == 0;
        // along rest dim 1 only the boundary bucket's G may vary (chainsplit.cuh JR)
        for (int j = 0; dense && md.size() == 2 && j < F; ++j)
            dense = j == (fw ? F - 1 : 0) || md[1].g[j] == 0;
        const int64_t S = fw ? is[F - 1] : os[0];
        for (int p = 0; dense && p < F; ++p) dense = S > 0 && (fw ? is[p] : os[p]) == (S << (fw ? F - 1 - p : p));
        const int dform = fw ? kChainFwdSD : kChainBwdSD;
        if (dense && chain_supported(eb, chain_key(dform, K, F, dep))) form = dform;
    }
    if (fwd_v && !std::getenv("BNPP_NO_CHAIN_FWDV") && chain_supported(eb, chain_key(kChainFwdV, K, F, dep))) {
        form = kChainFwdV;
        V = chain_fwd_v(N, eb);
    }
    if (!chain_supported(eb, chain_key(form, K, F, dep))) return fail("chain: shape not instantiated");
    if (nb) {
        // the belief (kChainBel): the dense backward form, the output's rest one
        // dense block below the slot stride S (belief entry r = output rest
        // offset), the forward message laid out exactly as the output
        if (form != kChainBwdSD || !chain_supported(eb, chain_key(form, K, F, dep) + kChainBelKey))
            return fail("chain: a fused belief needs the dense backward form");
        const View &lam = b.in[ni];
        bool same = lam.vars.size() == b.out_vars.size() && rest == os[0];
        for (size_t i = 0; same && i < b.out_vars.size(); ++i) same = stride_of(lam, b.out_vars[i]) == ostr[i];
        if (!same) return fail("chain: the belief's forward message is not laid out as the run's output");
    }
    if (std::getenv("BNPP_DEBUG_CHAIN"))
        std::fprintf(stderr, "[chain] run form %d K=%d F=%d dep %d V=%d rest %lld\n", form, K, F, dep, V, (long long)rest);
    d = BucketDesc{};
    d.out_size = rest * N;
    d.n_tiles = rest / V;
    d.v1 = V;
    d.v2 = 1;
    d.n_in = ni;
    d.n_dims = (int)md.size();
    d.k = K;
    d.out_table = b.out_table;
    d.flags = kScale | kTrackMax | (nb ? kChainBel : 0);
    d.aux_out = nb ? b.bel_table : 0;
    d.big = -1;
    d.chain = F | (b.chain_gmask << 8) | (form << 16) | (dep << 20);
    {
        // the streamed side linear in the thread index: a wave spans 64 * V
        // consecutive rest entries -> uniform base + 32-bit lane byte offset
        bool lin = !md.empty();
        const bool fwdf = form == kChainFwd || form == kChainFwdV || form == kChainSum || form == kChainFwdS ||
                          form == kChainFwdSD;
        int64_t s0 = md.empty() ? 0 : (fwdf ? md[0].in : md[0].out);
        for (size_t q = 0; lin && q + 1 < md.size(); ++q) {
            const int64_t a = fwdf ? md[q].in : md[q].out, nb = fwdf ? md[q + 1].in : md[q + 1].out;
            lin = nb == a * (int64_t)md[q].card;
        }
        if (lin && s0 > 0 && 64 * (int64_t)V * s0 * eb < ((int64_t)1 << 31)) d.flags |= kChainLo32;
        else return fail("chain: streamed side not linear in the thread index");
    }
    int32_t lo = 0;
    for (int i = 0; i < kMaxDescIn; ++i) {
        d.in_table[i] = i < ni ? b.in[i].table : 0;
        d.in_base[i] = i < ni ? b.in[i].base : 0;
        if (i >= 1 && i < ni) {
            int64_t sp = 1;
            for (size_t q = 0; q < b.in[i].vars.size(); ++q)
                sp += (int64_t)(cards[b.in[i].vars[q]] - 1) * b.in[i].strides[q];
            if (sp > kStreamSmallMax) return fail("chain: G table too large for LDS");
            d.in_span[i] = (int32_t)sp;
            d.in_lds_off[i] = lo;
            lo += chain_split_form(form) ? (int32_t)(sp * kSplitPack) : (int32_t)((sp + 3) & ~3);
        }
    }
    if (nb) {
        d.in_table[ni] = b.in[ni].table;
        d.in_base[ni] = b.in[ni].base;
    }
    d.small_elems = lo;
    if ((int64_t)lo * eb > (chain_split_form(form) ? split_g_budget_bytes(F, eb) : kStreamLdsBudget))
        return fail("chain: G tables exceed the LDS budget");
    {
        uint32_t shift, magic;
        bool pow2;
        const uint64_t c0 = md.empty() ? 1 : md[0].card / (uint64_t)V;
        magic_for((uint32_t)c0, shift, magic, pow2);
        d.tdiv0[0] = pack_dim_header((uint32_t)c0, shift, pow2);
        d.tdiv0[1] = (int64_t)magic;
        d.tdiv1[0] = pack_dim_header(1, 0, true);
        d.tdiv1[1] = 0;
    }
    d.dim_off = (int64_t)pool.size();
    for (const RDim &r : md) {
        uint32_t shift, magic;
        bool pow2;
        magic_for((uint32_t)r.card, shift, magic, pow2);
        pool.push_back(pack_dim_header((uint32_t)r.card, shift, pow2));
        pool.push_back((int64_t)magic);
        pool.push_back(r.in);
        pool.push_back(r.out);
        for (int j = 0; j < F; ++j) pool.push_back(r.g[j]);
    }
    for (int p = 0; p < F; ++p) {
        pool.push_back(is[p]);
        pool.push_back(os[p]);
    }
    for (int j = 0; j < F; ++j) {
        const View *g = gidx[j] >= 0 ? &b.in[gidx[j]] : nullptr;
        for (int p = 0; p < F; ++p) {
            const int var = p < j ? b.chain_n[p] : b.chain_x[p];
            pool.push_back(g && var >= 0 ? stride_of(*g, var) : 0);
        }
        pool.push_back(g && b.chain_n[j] >= 0 ? stride_of(*g, b.chain_n[j]) : 0);
    }
    return true;
}

bool build_desc(const BucketSpec &b, const std::vector<int> &cards, int max_vec, BucketDesc &d,
                std::vector<int64_t> &pool, std::string *msg, bool slab_outer) {
    if (!b.chain_x.empty()) return build_chain_desc(b, cards, max_vec, d, pool, msg);
    const int n = (int)b.in.size();
    if (n < 1 || n > kMaxIn) {
        if (msg) *msg = "bucket needs 1.." + std::to_string(kMaxIn) + " inputs, got " + std::to_string(n);
        return false;
    }
    if (b.elim_var >= 0 && contains(b.out_vars, b.elim_var)) {
        if (msg) *msg = "summed variable appears in the output scope";
        return false;
    }
    for (const View &v : b.in) {
        if (v.vars.size() != v.strides.size()) {
            if (msg) *msg = "view vars/strides length mismatch";
            return false;
        }
        for (int x : v.vars)
            if (x != b.elim_var && !contains(b.out_vars, x)) {
                if (msg) *msg = "input variable " + std::to_string(x) + " is neither kept nor summed";
                return false;
            }
    }
    std::vector<Dim> dims;    // slowest first
    int64_t out_size = 1;
    for (int u : b.out_vars) {
        int c = cards[u];
        if (c < 1) {
            if (msg) *msg = "cardinality must be >= 1";
            return false;
        }
        out_size = sat_mul(out_size, (int64_t)c);
        if (c == 1) continue;
        Dim dm;
        dm.card = (uint64_t)c;
        for (int i = 0; i < kMaxIn; ++i) dm.s[i] = 0;
        for (int i = 0; i < n; ++i)
            for (size_t j = 0; j < b.in[i].vars.size(); ++j)
                if (b.in[i].vars[j] == u) dm.s[i] = b.in[i].strides[j];
        dims.push_back(dm);
    }
    // merge adjacent dims that are contiguous in every input (fastest first)
    std::vector<Dim> merged;
    for (int j = (int)dims.size() - 1; j >= 0; --j) {
        const Dim &dm = dims[j];
        bool ok = !merged.empty();
        if (ok) {
            Dim &bk = merged.back();
            if (bk.card * dm.card > (uint64_t)INT32_MAX) ok = false;
            for (int i = 0; ok && i < n; ++i)
                if (dm.s[i] != bk.s[i] * (int64_t)bk.card) ok = false;
            if (ok) bk.card *= dm.card;
        }
        if (!ok) merged.push_back(dm);
    }
    if (out_size >= (kSatMax >> 6)) {
        if (msg) *msg = "bucket output beyond any device";
        return false;
    }
    std::vector<int64_t> out_strides;     // kOutStrided: output stride per (permuted) dim
    std::vector<int64_t> outer_tab;       // slab form, outer dims: base offsets per combination and input
    int k = 1;
    int64_t es[kMaxIn] = {0};
    if (b.elim_var >= 0) {
        for (int i = 0; i < n; ++i)
            for (size_t j = 0; j < b.in[i].vars.size(); ++j)
                if (b.in[i].vars[j] == b.elim_var) {
                    es[i] = b.in[i].strides[j];
                    k = cards[b.elim_var];
                }
    }
    // register tile: v1 entries of the fastest dim (vector loads for stride-1
    // inputs), then v2 entries of the next dim when v1 covers the whole fastest
    // dim (the tile is then v1*v2 contiguous output entries)
    int max_tile = max_vec == 2 ? 8 : 16;
    if (const char *e = tuning_knob("BNPP_MAX_TILE")) max_tile = std::max(1, std::min(max_tile, std::atoi(e)));
    if (b.simple) max_tile = 1;
    auto aligned = [&](int dim, int v) {
        for (int i = 0; i < n; ++i) {
            if (merged[dim].s[i] != 1) continue;
            bool lower_zero = true;           // stride-1 on `dim`, absent on faster dims
            for (int j = 0; j < dim; ++j)
                if (merged[j].s[i] != 0) lower_zero = false;
            if (!lower_zero) continue;
            if (b.in[i].base % v || es[i] % v) return false;
            for (size_t j = dim + 1; j < merged.size(); ++j)
                if (merged[j].s[i] % v) return false;
        }
        return true;
    };
    int v1 = 1, v2 = 1;
    if (!merged.empty()) {
        for (int v = 4; v >= 2; v >>= 1)
            if (v <= max_tile && merged[0].card % (uint64_t)v == 0 && aligned(0, v)) { v1 = v; break; }
        if (merged.size() >= 2 && (uint64_t)v1 == merged[0].card) {
            const int v2_max = (v1 == 2 && max_tile == 16) ? 8 : 4;   // instantiated tiles (kernels.hip)
            for (int v = max_tile / v1; v >= 2; v >>= 1)
                if (v <= v2_max && merged[1].card % (uint64_t)v == 0 && aligned(1, v)) { v2 = v; break; }
        }
    }
    d = BucketDesc{};
    d.out_size = out_size;
    d.v1 = v1;
    d.v2 = v2;
    d.n_tiles = out_size / (v1 * v2);
    d.n_in = n;
    d.n_dims = (int)merged.size();
    d.k = k;
    d.out_table = b.out_table;
    d.flags = kScale | kTrackMax;
    for (int i = 0; i < kMaxIn; ++i) {
        d.in_table[i] = i < n ? b.in[i].table : 0;
        d.in_base[i] = i < n ? b.in[i].base : 0;
        d.elim_stride[i] = es[i];
    }
    auto divisor = [&](uint64_t c, int64_t *hdr) {
        uint32_t shift, magic;
        bool pow2;
        magic_for((uint32_t)c, shift, magic, pow2);
        hdr[0] = pack_dim_header((uint32_t)c, shift, pow2);
        hdr[1] = (int64_t)magic;
    };
    divisor(merged.empty() ? 1 : merged[0].card / v1, d.tdiv0);
    divisor(merged.size() < 2 ? 1 : merged[1].card / v2, d.tdiv1);
    // stream form: exactly one input too big for LDS, the rest small enough
    d.big = -1;
    {
        int big = -1, n_big = 0;
        int64_t small_total = 0;
        int64_t span[kMaxIn];
        for (int i = 0; i < n; ++i) {
            int64_t sp = 1 + es[i] * (k - 1);
            for (size_t j = 0; j < b.in[i].vars.size(); ++j)
                if (b.in[i].vars[j] != b.elim_var) sp += (int64_t)(cards[b.in[i].vars[j]] - 1) * b.in[i].strides[j];
            span[i] = sp;
            if (sp > kStreamSmallMax) { big = i; ++n_big; }
            else small_total += sp;
        }
        const int eb = max_vec == 2 ? 8 : 4;
        const char *off = tuning_knob("BNPP_NO_STREAM");
        // a fastest output dim of card 3, 5, 6 or 7 leaves the stream form at
        // 1x1 tiles (a decode over every dim per output); the generic kernel's
        // whole-dim tiles (below) serve it instead
        const uint64_t c0 = merged.empty() ? 0 : merged[0].card;
        const char *os = tuning_knob("BNPP_ODD_STREAM");                 // A/B knob: 1 = keep the stream form
        const bool odd_rows = v1 == 1 && (c0 == 3 || c0 == 5 || c0 == 7 || (c0 == 6 && aligned(0, 2))) && (int)c0 <= max_tile &&
                              !(os && *os == '1');
        // 5-8 inputs: their own stream instantiations (kStream8In), every tile but 2x8
        const bool nin_ok = n <= 4 || (n <= kMaxIn && !(v1 == 2 && v2 == 8));
        if (!b.simple && !b.divide && n_big == 1 && nin_ok && small_total * eb <= kStreamLdsBudget && d.n_tiles >= 1024 &&
            !(off && *off == '1') && !odd_rows) {
            int64_t s0 = merged.empty() ? 0 : merged[0].s[big];
            int64_t s1 = merged.size() < 2 ? 0 : merged[1].s[big];
            // slab form (slab.cuh): the big input is k slabs contiguous along the
            // output's slab dim (dim 0, or dim 1 after a dim of card 2/4 it does
            // not vary along), every small input is constant along the slab dim.
            // Output dims slower than the slab dim ("outer", level launches only)
            // are enumerated as whole runs of virtual blocks: per combination the
            // inputs' bases move (a column sweep's first buckets multiply a
            // message by factors over new variables: [2^30 slab][2][2])
            int slab_v = 0, slab_c0 = 1, slab_dim = -1;
            int64_t slab_outer_n = 1;
            {
                const char *ns = std::getenv("BNPP_NO_SLAB");
                const char *no = std::getenv("BNPP_NO_SLAB_OUTER");
                if (!merged.empty() && merged[0].s[big] == 1) slab_dim = 0;
                else if (merged.size() >= 2 && merged[0].s[big] == 0 && merged[1].s[big] == 1) slab_dim = 1;
                // a row over two binary dims the big input does not vary along
                // (slab_y2): the conditioned 32x32 PR's 5-input bucket
                // [2][2][2^29 slab][2], 46 ms on the generic kernel
                else if (merged.size() >= 3 && merged[0].s[big] == 0 && merged[1].s[big] == 0 && merged[2].s[big] == 1 &&
                         merged[0].card == 2 && merged[1].card == 2)
                    slab_dim = 2;
                if (slab_dim >= 0)
                    for (size_t j = (size_t)slab_dim + 1; j < merged.size(); ++j)
                        slab_outer_n = sat_mul(slab_outer_n, (int64_t)merged[j].card);
                // outer dims with C0 <= 2: measured on the 32x32 sweep, [2^30 slab][2][2]
                // k=1 buckets went 1.7 -> 5.4 TB/s (6.1 with two passes per block),
                // [2 y][2^30 slab][2] k=2 ones ran 3.8 TB/s as one-pass slab tiles against
                // 4.2 for the stream kernel, 4.5 with two passes (profiles/r04_slab_outer_ab.txt,
                // r04_slab_passes_ab.txt)
                const char *oc = tuning_knob("BNPP_SLAB_OUTER_MAXC0");      // A/B knob
                const int64_t max_c0 = oc ? std::atoll(oc) : 2;
                if (slab_outer_n > 1 && (!slab_outer || (no && *no == '1') || slab_outer_n > kSlabMaxOuter ||
                                         (slab_dim == 1 && (int64_t)merged[0].card > max_c0)))
                    slab_dim = -1;
                const Dim *sd = slab_dim >= 0 ? &merged[slab_dim] : nullptr;
                slab_c0 = slab_dim == 1 ? (int)merged[0].card : slab_dim == 2 ? 4 : 1;
                // (slab kernels: up to 4 inputs in every shape, 5-8 with one
                // slab entry per lane -- slab.cuh kSlabMaxIn / BNPP_SLAB8_*)
                bool ok = !(ns && *ns == '1') && sd && n <= kMaxIn && k >= 1 && k <= 4 &&
                          (slab_c0 == 1 || slab_c0 == 2 || slab_c0 == 4);
                for (int i = 0; ok && i < n; ++i)
                    if (i != big && sd->s[i] != 0) ok = false;
                if (ok) {
                    int vn = eb == 4 ? (slab_c0 == 1 ? 4 : slab_c0 == 2 ? 2 : 1) : (slab_c0 == 1 ? 2 : 1);
                    // A/B knob: slow-dim entries per tile (instantiated: f32 c0=1 {1,4}, 2 {1,2},
                    // 4 {1,2}; f64 c0=1 {1,2}, 2 {1,2}, 4 {1}; slab.cuh)
                    if (const char *sv = tuning_knob("BNPP_SLAB_V")) {
                        const int want = std::atoi(sv);
                        const bool inst = want == 1 || (want == 2 && slab_c0 != 1 && (eb == 4 || slab_c0 == 2)) ||
                                          (want == 2 && eb == 8 && slab_c0 == 1) || (want == 4 && eb == 4 && slab_c0 == 1);
                        if (inst) vn = want;
                    }
                    if (n > 4 || slab_dim == 2) vn = 1;            // the 8-input-class instantiations
                    if ((int64_t)sd->card % vn || b.in[big].base % vn || es[big] % vn) vn = 1;
                    for (size_t j = (size_t)slab_dim + 1; j < merged.size(); ++j)
                        if (merged[j].s[big] % vn) vn = 1;
                    if (slab_outer_n > 1) {
                        // every combination's tiles fill whole virtual blocks
                        auto fits = [&](int v) {
                            const char *sl = tuning_knob("BNPP_SLAB_LANES");
                            const int lanes = slab_c0 * v * eb == 32 && !(sl && *sl == '1') ? 2 : 1;
                            return ((int64_t)sd->card / v) % (kBlock / lanes) == 0;
                        };
                        // (two passes per block need twice that: checked below)
                        if (!fits(vn)) vn = fits(1) ? 1 : 0;
                    }
                    slab_v = vn;
                }
            }
            if (slab_v > 0) {
                v1 = slab_c0;
                v2 = slab_v;
                d.v1 = v1;
                d.v2 = v2;
                d.n_tiles = out_size / (v1 * v2);
                d.big = big;
                d.bcls = kBigSlab;
                d.slab_y2 = slab_dim == 2 ? 2 : 0;
                // 32-B rows (f64 c0 * v = 4, f32 8): two lanes per tile, 16 B each
                const char *sl = tuning_knob("BNPP_SLAB_LANES");     // A/B knob: 1 = one lane per tile
                d.lanes = v1 * v2 * eb == 32 && !(sl && *sl == '1') ? 2 : 1;
                for (int i = 0; i < n; ++i) {
                    d.in_span[i] = (int32_t)std::min<int64_t>(span[i], INT32_MAX);
                    d.in_lds_off[i] = 0;
                }
                d.small_elems = 0;
                // level launches: two passes of tiles per block, both passes' loads
                // issued first (instantiated: f32 (C0, V) = (1, 4), (2, 2); f64 (1, 2); H = 1)
                d.slab_r = 1;
                {
                    const char *sr = tuning_knob("BNPP_SLAB_R");          // A/B knob: 1 = one pass
                    const bool inst = d.lanes == 1 && ((eb == 4 && ((v1 == 1 && v2 == 4) || (v1 == 2 && v2 == 2))) ||
                                                       (eb == 8 && v1 == 1 && v2 == 2));
                    if (slab_outer && !(sr && std::atoi(sr) == 1) && inst && n <= 4 && slab_dim < 2 &&
                        (slab_outer_n == 1 || ((int64_t)merged[slab_dim].card / v2) % (2 * kBlock) == 0))
                        d.slab_r = 2;
                    // the 8-input class (5-8 inputs, or rows over two dims): one
                    // slab entry per lane leaves a block 256 lanes x K loads of
                    // 4-8 B beside its per-block setup (descriptor, exponents of
                    // every input, the small tables by scalar loads); R passes
                    // per block, every pass's loads issued first (instantiated:
                    // R = 2, 4; level launches).  The conditioned 32x32 PR's
                    // 5-input bucket: fp32 13.6 / 11.4 / 10.5 ms at R = 1 / 2 / 4
                    // (9.7 with the setup through the scalar cache), fp64 (two
                    // lanes per 32-B row) 27.3 / 28.9 / 35.7 ms -- fp64 keeps one
                    // pass (profiles/r06_slab8_passes_ab.txt)
                    if (slab_outer && (n > 4 || slab_dim == 2) && eb == 4 && !(sr && std::atoi(sr) == 1)) {
                        const int want = sr ? std::atoi(sr) : 4;
                        for (int r = want == 2 || want == 4 ? want : 4; r >= 2; r /= 2)
                            if (slab_outer_n == 1 || ((int64_t)merged[slab_dim].card / v2) % (r * kBlock / d.lanes) == 0) {
                                d.slab_r = r;
                                break;
                            }
                    }
                }
                if (slab_outer_n > 1) {
                    const int64_t S = (int64_t)merged[slab_dim].card;
                    const int64_t per_vb = kBlock / d.lanes * d.slab_r;
                    uint32_t shift, magic;
                    bool pow2;
                    magic_for((uint32_t)(S / v2 / per_vb), shift, magic, pow2);
                    d.outer_n = (int32_t)slab_outer_n;
                    d.outer_div[0] = pack_dim_header((uint32_t)(S / v2 / per_vb), shift, pow2);
                    d.outer_div[1] = (int64_t)magic;
                    outer_tab.resize((size_t)(slab_outer_n * n));
                    for (int64_t o = 0; o < slab_outer_n; ++o) {
                        int64_t rem = o;
                        for (int i = 0; i < n; ++i) outer_tab[o * n + i] = i == big ? -o * S : 0;
                        for (size_t j = (size_t)slab_dim + 1; j < merged.size(); ++j) {
                            const int64_t x = rem % (int64_t)merged[j].card;
                            rem /= (int64_t)merged[j].card;
                            for (int i = 0; i < n; ++i) outer_tab[o * n + i] += x * merged[j].s[i];
                        }
                    }
                }
            } else {
            // optional narrow tile: when the big input is constant along the
            // fastest output dim and v1 entries already fill a 16-B store, drop
            // v2 (one scalar big load per summed value, stores coalesced as is)
            const char *nw = tuning_knob("BNPP_NARROW");
            if (nw && *nw == '1' && v2 > 1 && s0 == 0 && v1 * eb >= 16) {
                v2 = 1;
                d.v2 = 1;
                d.n_tiles = out_size / v1;
                divisor(merged.size() < 2 ? 1 : merged[1].card, d.tdiv1);
            }
            // interleaved: the summed variable is the big input's fastest dim and
            // output dim 0 follows it, so a V1-entry tile reads V1*k contiguous values
            bool inter = false;
            if (n <= 4 && (k == 2 || k == 4) && es[big] == 1 && s0 == k && v1 >= 2 && !merged.empty()) {
                const int64_t vw = 16 / eb;
                inter = b.in[big].base % vw == 0 && (int64_t)(v1 * k) % vw == 0;
                for (size_t j = 1; inter && j < merged.size(); ++j)
                    if (merged[j].s[big] % vw) inter = false;
                // wider tiles keep more bytes in flight per thread: 8 entries of dim 0
                const char *iv = tuning_knob("BNPP_INTER_V1");
                const int want_v1 = iv ? std::atoi(iv) : 8;
                int nv1 = v1;
                if (want_v1 == 8 && merged[0].card % 8 == 0 && (int64_t)(8 * k) % vw == 0) nv1 = 8;
                // a dim the big input does not vary along (a variable only the small
                // inputs hold): the tile spans it, so one load of the big values
                // serves every row; it becomes dim 1 and the output offsets come
                // from per-dim output strides (kOutStrided)
                int bdim = -1;
                for (size_t j = 1; inter && j < merged.size(); ++j)
                    if (merged[j].s[big] == 0 && (merged[j].card == 2 || merged[j].card == 4)) {
                        bdim = (int)j;
                        break;
                    }
                const char *nb = tuning_knob("BNPP_NO_BCAST_ROWS");
                if (nb && *nb == '1') bdim = -1;
                if (inter && bdim >= 1) {
                    const int cb = (int)merged[bdim].card;
                    const int max_ts = eb == 4 ? 16 : 8;
                    int rv1 = nv1;
                    while (rv1 * cb > max_ts) rv1 /= 2;
                    if (rv1 >= 2 && merged[0].card % (uint64_t)rv1 == 0 && (int64_t)(rv1 * k) % vw == 0) {
                        std::vector<int64_t> os(merged.size());
                        int64_t acc_s = 1;
                        for (size_t j = 0; j < merged.size(); ++j) {
                            os[j] = acc_s;
                            acc_s *= (int64_t)merged[j].card;
                        }
                        Dim mb = merged[bdim];
                        int64_t ob = os[bdim];
                        merged.erase(merged.begin() + bdim);
                        os.erase(os.begin() + bdim);
                        merged.insert(merged.begin() + 1, mb);
                        os.insert(os.begin() + 1, ob);
                        out_strides = os;
                        v1 = rv1;
                        v2 = cb;
                        d.v1 = v1;
                        d.v2 = v2;
                        d.n_tiles = out_size / (v1 * v2);
                        d.flags |= kOutStrided;
                        divisor(merged[0].card / v1, d.tdiv0);
                        divisor(1, d.tdiv1);
                    } else {
                        bdim = -1;
                    }
                }
                if (inter && bdim < 1 && (v2 > 1 || nv1 != v1)) {
                    v1 = nv1;
                    v2 = 1;
                    d.v1 = v1;
                    d.v2 = 1;
                    d.n_tiles = out_size / v1;
                    divisor(merged[0].card / v1, d.tdiv0);
                    divisor(merged.size() < 2 ? 1 : merged[1].card, d.tdiv1);
                }
            }
            int bc;
            if (inter) bc = k == 2 ? kBigInter2 : kBigInter4;
            else if (s0 == 0 && (v2 == 1 || s1 == 0)) bc = kBigOne;
            else if (v1 > 1 && s0 == 1 && (v2 == 1 || s1 == 0)) bc = kBigRow;
            else if (v2 > 1 && s0 == 0 && s1 == 1) bc = kBigCol;
            else if (v1 > 1 && v2 > 1 && s0 == 1 && s1 == v1) bc = kBigFull;
            else bc = kBigDirect;
            d.big = big;
            d.bcls = bc;
            int32_t o = 0;
            for (int i = 0; i < n; ++i) {
                d.in_span[i] = (int32_t)span[i];
                d.in_lds_off[i] = i == big ? 0 : o;
                if (i != big) o += (int32_t)((span[i] + 3) & ~3);       // keep 16-B alignment
            }
            d.small_elems = o;
            }
        }
    }
    // generic kernel, a fastest dim of card 3, 5, 6 or 7 (Munin1's card-7
    // variables): 1x1 tiles paid a mixed-radix decode over every dim and one
    // load per input per output; whole-dim tiles decode once per card0
    // outputs and load stride-1 inputs as runs (scalar for odd cards, so no
    // alignment; card 6 as pairs)
    if (d.big < 0 && v1 == 1 && !merged.empty() && !b.simple) {
        const uint64_t c0 = merged[0].card;
        if ((c0 == 3 || c0 == 5 || c0 == 7 || (c0 == 6 && aligned(0, 2))) && (int)c0 <= max_tile) {
            v1 = (int)c0;
            v2 = 1;
            d.v1 = v1;
            d.v2 = 1;
            d.n_tiles = out_size / v1;
            divisor(1, d.tdiv0);
            divisor(merged.size() < 2 ? 1 : merged[1].card, d.tdiv1);
        }
    }
    if (b.divide) {
        if (n != 2 || b.elim_var >= 0) {
            if (msg) *msg = "divide takes two inputs and sums nothing";
            return false;
        }
        d.flags |= kDivide;
    }
    d.dim_off = (int64_t)pool.size();
    for (const Dim &dm : merged) {
        uint32_t shift, magic;
        bool pow2;
        magic_for((uint32_t)dm.card, shift, magic, pow2);
        pool.push_back(pack_dim_header((uint32_t)dm.card, shift, pow2));
        pool.push_back((int64_t)magic);
        for (int i = 0; i < n; ++i) pool.push_back(dm.s[i]);
    }
    if (d.flags & kOutStrided)
        for (int64_t o : out_strides) pool.push_back(o);
    if (d.outer_n > 0) {
        d.outer_rel = (int32_t)((int64_t)pool.size() - d.dim_off);
        pool.insert(pool.end(), outer_tab.begin(), outer_tab.end());
    }
    return true;
}

// ---------------------------------------------------------------- VE plan
constexpr int kChainRunMax = 8;                   // longest fused run tried (split form: binary fp32; fp64: 7)
// BNPP_CHAIN_RUN_MAX (tests): a shorter cap, to exercise the short-run kernels
inline int chain_run_max() {
    const char *e = std::getenv("BNPP_CHAIN_RUN_MAX");
    const int v = e ? std::atoi(e) : kChainRunMax;
    return v >= 2 && v <= kChainRunMax ? v : kChainRunMax;
}
// first run length to try for `rem` remaining buckets: never leave a single
// bucket behind when a split into runs >= 2 exists (5 -> 3 + 2, not 4 + 1)
inline int chain_first_try(int rem) {
    const int mx = chain_run_max();
    return rem == mx + 1 && mx > 2 ? mx - 1 : std::min(mx, rem);
}

namespace {
// Emits buckets and message tables into a VEPlan (shared by plan_ve and
// plan_bucket_tree).  Levels: a bucket runs one level after its latest input.
struct PlanBuilder {
    std::vector<int> cards;                 // model cards + virtual composite variables
    int n_real = 0;
    VEPlan &p;
    bool canonical;
    std::vector<int> rank;
    std::vector<int> level;                 // per table
    bool sequential = false;                // every bucket one level after the previous (program order)
    // reductions of a delivered kept table (<= 2^25 entries, read once each):
    // placed one level after their own input (and after free_base, the level
    // the delivery's reductions start from), not in program order, so the
    // reductions at one depth of a delivery's tree share a level and a launch
    // (the 32x32 MAR made ~3,000 launches of a few microseconds each per call);
    // the next big bucket still follows them all (its arena is unchanged)
    bool free_small = false;
    int64_t free_max = 0;                   // ... tables up to the delivered kept table's size
    int free_base = 0;
    int last_level = 0;
    int lane = 0;                           // BucketSpec::lane of the buckets emitted now

    PlanBuilder(const std::vector<int> &c, VEPlan &plan, const std::vector<View> &sources,
                const std::vector<int> &order, bool canon_layout)
        : cards(c), n_real((int)c.size()), p(plan), canonical(canon_layout) {
        p.n_src = (int)sources.size();
        rank.assign(cards.size(), -1);
        for (int i = (int)order.size() - 1; i >= 0; --i) rank[order[i]] = i;
        level.assign(p.n_src, 0);
    }
    // layout key: earlier-eliminated variables are slower; kept variables last
    std::vector<int> canon(std::vector<int> s) const {
        if (!canonical) return s;
        const int64_t nv = (int64_t)cards.size();
        std::stable_sort(s.begin(), s.end(), [&](int a, int b) {
            int64_t ka = rank[a] >= 0 ? rank[a] : nv + a;
            int64_t kb = rank[b] >= 0 ? rank[b] : nv + b;
            return ka < kb;
        });
        return s;
    }
    int new_msg(const std::vector<int> &vars) {
        MsgTable t;
        t.vars = vars;
        t.size = table_size(vars, cards);
        p.max_table = std::max(p.max_table, t.size);
        p.msgs.push_back(t);
        level.push_back(0);
        return p.n_src + (int)p.msgs.size() - 1;
    }
    View view(int id) const { return natural_view(id, p.msgs[id - p.n_src].vars, cards); }
    double entries_of(const std::vector<View> &in) const {
        double e = 1;
        for (int v : chain_scope(in)) e *= cards[v];
        return e;
    }
    double moved_of(const std::vector<View> &in, int out_table) const {
        double e = (double)p.msgs[out_table - p.n_src].size;
        for (const View &v : in) e += (double)table_size(v.vars, cards);
        return e;
    }
    int push_bucket(const std::vector<View> &in, int x, const std::vector<int> &ov, bool free_level = false) {
        BucketSpec b;
        b.lane = lane;
        b.in = in;
        b.elim_var = x;
        b.out_vars = ov;
        b.out_table = new_msg(ov);
        const bool small = free_small && table_size(ov, cards) <= free_max;
        int lv = sequential && !free_level ? (small ? free_base : last_level) : 0;
        for (const View &v : in) lv = std::max(lv, level[v.table]);
        b.level = lv + 1;
        last_level = std::max(last_level, b.level);
        level[b.out_table] = b.level;
        p.entries += entries_of(in);
        p.elems_moved += moved_of(in, b.out_table);
        p.buckets.push_back(b);
        return b.out_table;
    }
    // one step of a message exchange (BucketSpec::xchg): no arithmetic, its
    // traffic counted (the sync step's few bytes are not)
    int push_xchg(const std::vector<View> &in, const std::vector<int> &ov, int kind, int mode, int blocks) {
        BucketSpec b;
        b.lane = lane;
        b.in = in;
        b.elim_var = -1;
        b.out_vars = ov;
        b.out_table = new_msg(ov);
        b.xchg = kind;
        b.xchg_mode = mode;
        b.xchg_blocks = blocks;
        int lv = sequential ? last_level : 0;
        for (const View &v : in) lv = std::max(lv, level[v.table]);
        b.level = lv + 1;
        last_level = std::max(last_level, b.level);
        level[b.out_table] = b.level;
        if (kind != kXchgSync) p.elems_moved += moved_of({in[0]}, b.out_table);
        p.buckets.push_back(b);
        return b.out_table;
    }
    // a bucket over `in` (any length) summing out `x` (-1: none); inputs past
    // kMaxIn are folded into materialised products left to right, like the
    // reference's chain
    int emit(std::vector<View> in, int x, bool final_result) {
        while ((int)in.size() > kMaxIn) {
            std::vector<View> head(in.begin(), in.begin() + kMaxIn);
            int t = push_bucket(head, -1, canon(chain_scope(head)));
            std::vector<View> rest;
            rest.push_back(view(t));
            rest.insert(rest.end(), in.begin() + kMaxIn, in.end());
            in.swap(rest);
        }
        std::vector<int> u = chain_scope(in);
        std::vector<int> ov = x >= 0 ? remove_var(u, x) : u;
        if (!final_result) ov = canon(ov);
        int t = push_bucket(in, x, ov);
        p.width = std::max(p.width, (int)ov.size());
        return t;
    }
    // ---- fused chain runs (chain.cuh) ----
    int chain_eb = 0;                                   // element bytes of the run's dtype (0: no fusion)
    std::map<std::vector<int64_t>, int> gcache;         // G product tables, by their factor views
    struct ChainStep {
        std::vector<View> smalls;                       // the bucket's factor tables, chain order
        int x;                                          // the variable it sums out
    };
    // Buckets steps[0..F) as one fused run over the message `big` (each
    // bucket's chain is smalls..., then the message, model.cpp:414-418).
    // Returns the run's output table, or -1 when the run does not fit a
    // chain kernel (the caller then emits the buckets one by one).
    int emit_chain(const View &big, const std::vector<ChainStep> &steps) {
        const int F = (int)steps.size();
        if (chain_eb == 0 || F < 2) return -1;
        std::vector<int> vars = big.vars, xs, ns;
        for (const ChainStep &st : steps) {
            std::vector<int> u = vars;
            for (const View &v : st.smalls) {
                if (table_size(v.vars, cards) > kStreamSmallMax) {
                    if (std::getenv("BNPP_DEBUG_CHAIN")) std::fprintf(stderr, "[chain] F=%d: large factor table\n", F);
                    return -1;
                }
                for (int w : v.vars)
                    if (!contains(u, w)) u.push_back(w);
            }
            const bool dbg = std::getenv("BNPP_DEBUG_CHAIN") != nullptr;
            if (!contains(vars, st.x) || !contains(big.vars, st.x) || contains(ns, st.x)) {
                if (dbg) std::fprintf(stderr, "[chain] F=%d: summed var %d not an input slot\n", F, st.x);
                return -1;
            }
            std::vector<int> nw;
            for (int w : u)
                if (!contains(vars, w)) nw.push_back(w);
            // every bucket swaps one variable, or every bucket only sums one out
            const bool swap_ok = nw.size() == 1 && nw[0] != st.x && (ns.empty() || ns[0] >= 0);
            const bool sum_ok = nw.empty() && (ns.empty() || ns[0] < 0);
            if (!swap_ok && !sum_ok) {
                if (dbg) std::fprintf(stderr, "[chain] F=%d: bucket brings %zu new variables\n", F, nw.size());
                return -1;
            }
            xs.push_back(st.x);
            ns.push_back(sum_ok ? -1 : nw[0]);
            vars = remove_var(u, st.x);
        }
        BucketSpec b;
        b.lane = lane;
        b.in.push_back(big);
        b.out_vars = canon(vars);
        b.chain_x = xs;
        b.chain_n = ns;
        std::vector<int> prod_of;                       // input index -> step whose smalls need a product
        for (int j = 0; j < F; ++j) {
            const std::vector<View> &sm = steps[j].smalls;
            if (sm.empty()) continue;
            b.chain_gmask |= 1 << j;
            if (sm.size() == 1) {
                b.in.push_back(sm[0]);
                prod_of.push_back(-1);
            } else {
                b.in.push_back(natural_view(-1, canon(chain_scope(sm)), cards));
                prod_of.push_back(j);
            }
        }
        {
            BucketDesc d;
            std::vector<int64_t> pool;
            std::string why;
            if (!build_desc(b, cards, chain_eb == 8 ? 2 : 4, d, pool, &why)) {
                if (std::getenv("BNPP_DEBUG_CHAIN")) std::fprintf(stderr, "[chain] F=%d rejected: %s\n", F, why.c_str());
                return -1;
            }
        }
        double moved = (double)table_size(big.vars, cards);
        for (size_t i = 1; i < b.in.size(); ++i) {
            const int j = prod_of[i - 1];
            if (j >= 0) {
                const std::vector<View> &sm = steps[j].smalls;
                std::vector<int64_t> key;
                for (const View &v : sm) {
                    key.push_back(v.table);
                    key.push_back(v.base);
                    key.insert(key.end(), v.vars.begin(), v.vars.end());
                    key.push_back(-1);
                }
                auto it = gcache.find(key);
                int t = it != gcache.end() ? it->second : push_bucket(sm, -1, canon(chain_scope(sm)), true);
                gcache[key] = t;
                b.in[i] = view(t);
            }
            moved += (double)table_size(b.in[i].vars, cards);
        }
        b.out_table = new_msg(b.out_vars);
        int lv = sequential ? last_level : 0;
        for (const View &v : b.in) lv = std::max(lv, level[v.table]);
        b.level = lv + 1;
        last_level = std::max(last_level, b.level);
        level[b.out_table] = b.level;
        if (ns[0] >= 0) {
            const double rest = (double)table_size(b.out_vars, cards) / std::pow((double)cards[xs[0]], F);
            p.entries += F * rest * std::pow((double)cards[xs[0]], F + 1);
        } else {                                        // bucket j of a summing run: rest * K^(F-j)
            const double rest = (double)table_size(b.out_vars, cards);
            for (int j = 0; j < F; ++j) p.entries += rest * std::pow((double)cards[xs[0]], F - j);
        }
        p.elems_moved += moved + (double)p.msgs[b.out_table - p.n_src].size;
        p.width = std::max(p.width, (int)b.out_vars.size());
        p.buckets.push_back(b);
        return b.out_table;
    }
    // A delivery's belief folded into the backward run that just made its
    // message pi (kChainBel, chainsplit.cuh): the run also reads lam (laid out
    // as pi) and writes bel[r] = sum over its slot combinations s, ascending,
    // of lam[r + s S] * pi[r + s S] -- the separate belief pass re-read all of
    // pi (17 GB per delivery on the 32x32 sweep) and lam.  slow: the summed
    // (slowest) variables, which must be the run's slots.  Returns the belief
    // table, or -1 (the caller then emits the belief bucket).
    int attach_belief(const View &pi, const View &lam, const std::vector<int> &slow) {
        const char *off = std::getenv("BNPP_NO_BEL_FUSE");
        if (p.buckets.empty() || (off && *off == '1')) return -1;
        BucketSpec &b = p.buckets.back();
        const int F = (int)b.chain_n.size();
        if (b.chain_x.empty() || b.bel_table >= 0 || b.out_table != pi.table || pi.base != 0 || lam.base != 0 ||
            (int)slow.size() != F || (int)pi.vars.size() <= F || lam.vars != pi.vars || lam.strides != pi.strides ||
            lam.table < p.n_src || level[lam.table] >= b.level) {
            if (std::getenv("BNPP_DEBUG_CHAIN"))
                std::fprintf(stderr, "[chain] belief not fused: run F=%d (out %d, pi %d), %zu slow variables\n", F,
                             b.out_table, pi.table, slow.size());
            return -1;
        }
        for (int i = 0; i < F; ++i)
            if (!contains(slow, pi.vars[i]) || !contains(b.chain_n, pi.vars[i])) return -1;
        const std::vector<int> kv(pi.vars.begin() + F, pi.vars.end());
        if (canon(kv) != kv) return -1;
        {
            BucketSpec t = b;                           // the run's descriptor with the belief attached
            t.in.push_back(lam);
            t.bel_table = pi.table;
            BucketDesc d;
            std::vector<int64_t> pool;
            std::string why;
            if (!build_desc(t, cards, chain_eb == 8 ? 2 : 4, d, pool, &why)) {
                if (std::getenv("BNPP_DEBUG_CHAIN")) std::fprintf(stderr, "[chain] belief not fused: %s\n", why.c_str());
                return -1;
            }
        }
        b.in.push_back(lam);
        b.bel_table = new_msg(kv);
        level[b.bel_table] = b.level;
        p.entries += (double)table_size(pi.vars, cards);
        p.elems_moved += (double)table_size(lam.vars, cards) + (double)p.msgs[b.bel_table - p.n_src].size;
        return b.bel_table;
    }
    // first bucket (by elimination rank >= from) whose variable is in `vars`
    int first_bucket(const std::vector<int> &vars, int from) const {
        int best = -1;
        for (int v : vars) {
            int r = v < (int)cards.size() ? rank[v] : -1;
            if (r >= from && (best < 0 || r < best)) best = r;
        }
        return best;
    }
    // Merge variables `g` (slow to fast) into one virtual variable in every
    // input: each input must hold all of them as one contiguous mixed-radix
    // block in that order, or none.  Returns the virtual id, or -1.
    int merge_group(std::vector<View> &in, const std::vector<int> &g) {
        if (g.empty()) return -1;
        int64_t prod = 1;
        for (int v : g) prod *= cards[v];
        if (prod > (int64_t)INT32_MAX) return -1;
        std::vector<View> out = in;
        for (View &w : out) {
            std::vector<int> pos;
            for (int v : g) {
                auto it = std::find(w.vars.begin(), w.vars.end(), v);
                pos.push_back(it == w.vars.end() ? -1 : (int)(it - w.vars.begin()));
            }
            int present = 0;
            for (int q : pos) present += q >= 0;
            if (present == 0) continue;
            if (present != (int)g.size()) return -1;
            for (size_t k = 0; k + 1 < g.size(); ++k)
                if (w.strides[pos[k]] != w.strides[pos[k + 1]] * cards[g[k + 1]]) return -1;
            const int64_t fast = w.strides[pos.back()];
            View nw;
            nw.table = w.table;
            nw.base = w.base;
            for (size_t j = 0; j < w.vars.size(); ++j)
                if (std::find(g.begin(), g.end(), w.vars[j]) == g.end()) {
                    nw.vars.push_back(w.vars[j]);
                    nw.strides.push_back(w.strides[j]);
                }
            nw.vars.push_back((int)cards.size());
            nw.strides.push_back(fast);
            w = nw;
        }
        cards.push_back((int)prod);
        rank.push_back(-1);
        in.swap(out);
        return (int)cards.size() - 1;
    }
    // Sum everything in `in` except `t` down to a table over {t}.  When the
    // summed variables are contiguous in every input (messages in canonical
    // layout, t slowest), they are summed in a few composite passes of
    // <= ~2K values each (about one read of the inputs); otherwise one
    // variable at a time in elimination-rank order.
    int reduce_to(std::vector<View> in, int t) { return reduce_keep(std::move(in), {t}); }
    // the marginals of several targets of one table: the targets are split in
    // two halves (by position in the table's layout), each half's joint is
    // summed out of the table once, and the halves recurse; every big table
    // is read twice instead of once per target
    void reduce_many(const View &v, std::vector<int> tg, std::vector<int> &result_of) {
        if (tg.size() <= 2 || table_size(v.vars, cards) <= 4096) {
            for (int t : tg) result_of[t] = reduce_to({v}, t);
            return;
        }
        auto pos = [&](int t) { return std::find(v.vars.begin(), v.vars.end(), t) - v.vars.begin(); };
        std::sort(tg.begin(), tg.end(), [&](int a, int b) { return pos(a) < pos(b); });
        const size_t h = tg.size() / 2;
        for (int side = 0; side < 2; ++side) {
            std::vector<int> part(side ? tg.begin() + h : tg.begin(), side ? tg.end() : tg.begin() + h);
            reduce_many(view(reduce_keep({v}, part)), part, result_of);
        }
    }
    // sum every variable outside `keep` out of the product of `in`
    int reduce_keep(std::vector<View> in, const std::vector<int> &keep) {
        std::vector<int> y;
        for (int v : chain_scope(in))
            if (!contains(keep, v)) y.push_back(v);
        std::sort(y.begin(), y.end(), [&](int a, int b) { return rank[a] < rank[b]; });
        if (y.empty()) return emit(in, -1, false);
        while (!y.empty()) {
            int64_t P = 1;
            for (int v : y) P *= cards[v];
            // one stage sums kk values per output: up to 2048 while the output
            // keeps >= 2^20 entries, else 32 (small stages stay parallel)
            int64_t kk = P > ((int64_t)1 << 22) ? std::min<int64_t>(2048, P >> 20) : std::min<int64_t>(P, 32);
            int64_t want_lo = std::max<int64_t>(1, P / kk);
            size_t cut = y.size();
            int64_t lo = 1;
            while (cut > 0 && lo * cards[y[cut - 1]] <= want_lo) lo *= cards[y[--cut]];
            if (cut == 0) cut = 1;
            std::vector<int> g(y.begin(), y.begin() + cut);
            std::vector<View> merged = in;
            int vv = g.size() >= 2 ? merge_group(merged, g) : -1;
            int tb;
            if (vv >= 0) {
                tb = emit(merged, vv, false);
                y.erase(y.begin(), y.begin() + cut);
            } else {
                tb = emit(in, y[0], false);
                y.erase(y.begin());
            }
            in = {view(tb)};
        }
        return in[0].table;
    }
    void finish() {
        if ((int)cards.size() > n_real) p.cards_ext = cards;
        std::stable_sort(p.buckets.begin(), p.buckets.end(),
                         [](const BucketSpec &a, const BucketSpec &b) { return a.level < b.level; });
        p.n_levels = p.buckets.empty() ? 0 : p.buckets.back().level;
    }
};
}  // namespace

VEPlan plan_ve(const std::vector<int> &cards, const std::vector<View> &sources, const std::vector<int> &order,
               bool canonical, int chain_eb) {
    VEPlan p;
    PlanBuilder B(cards, p, sources, order, canonical);
    B.chain_eb = canonical ? chain_eb : 0;
    const int nord = (int)order.size();
    auto is_msg = [&](const View &v) { return v.table >= p.n_src; };
    std::vector<std::vector<View>> buckets(nord);
    std::vector<View> result;
    for (const View &s : sources) {                                   // model.cpp:394-406
        int bi = B.first_bucket(s.vars, 0);
        if (bi >= 0) buckets[bi].push_back(s);
        else result.push_back(s);
    }
    for (int i = 0; i < nord; ++i) {                                  // model.cpp:409-439
        if (buckets[i].empty()) continue;   // Factor(1.0).sum_out(x) == 1: result *= 1 is exact
        // a sweep: bucket i holds factor tables and ONE message (last in its
        // chain), its message goes to bucket i+1, which holds only factor
        // tables, and so on -> one fused run (chain.cuh), same arithmetic
        int fused = 0;
        if (B.chain_eb && is_msg(buckets[i].back())) {
            int n_msg = 0;
            for (const View &v : buckets[i]) n_msg += is_msg(v);
            for (int F = chain_first_try(nord - i); F >= 2 && n_msg == 1 && !fused; --F) {
                    if ((nord - i) - F == 1 && F > 2) continue;   // never strand one bucket
                const View big = buckets[i].back();
                std::vector<PlanBuilder::ChainStep> steps;
                std::vector<int> vars = big.vars;
                bool ok = true;
                for (int k = 0; k < F && ok; ++k) {
                    std::vector<View> sm = buckets[i + k];
                    if (k == 0) sm.pop_back();
                    for (const View &v : sm) ok = ok && !is_msg(v);
                    if (k > 0) ok = ok && !sm.empty() && B.first_bucket(vars, i + k) == i + k;
                    for (const View &v : sm)
                        for (int w : v.vars)
                            if (!contains(vars, w)) vars.push_back(w);
                    vars = remove_var(vars, order[i + k]);
                    steps.push_back({sm, order[i + k]});
                }
                if (!ok) continue;
                const int t = B.emit_chain(big, steps);
                if (t < 0) continue;
                View mv = B.view(t);
                int bi = B.first_bucket(mv.vars, i + F);
                if (bi >= 0) buckets[bi].push_back(mv);
                else result.push_back(mv);
                fused = F;
            }
        }
        if (fused) {
            i += fused - 1;
            continue;
        }
        int t = B.emit(buckets[i], order[i], false);
        View mv = B.view(t);
        int bi = B.first_bucket(mv.vars, i + 1);
        if (bi >= 0) buckets[bi].push_back(mv);
        else result.push_back(mv);
    }
    if (!result.empty()) {
        p.result_table = B.emit(result, -1, true);
        p.result_vars = p.msgs[p.result_table - p.n_src].vars;
    }
    B.finish();
    return p;
}

VEPlan plan_bucket_tree(const std::vector<int> &cards, const std::vector<View> &sources,
                        const std::vector<int> &order, const std::vector<int> &targets, int part, int n_parts) {
    VEPlan p;
    PlanBuilder B(cards, p, sources, order, true);
    const int nord = (int)order.size();
    // forward (collect) pass: exactly the VE buckets of plan_ve, remembering the tree
    std::vector<std::vector<View>> src_in(nord);
    std::vector<std::vector<int>> children(nord);
    std::vector<int> lam(nord, -1);
    for (const View &s : sources) {
        int bi = B.first_bucket(s.vars, 0);
        if (bi >= 0) src_in[bi].push_back(s);   // else: a constant, cancels in every marginal
    }
    auto lam_view = [&](int c) { return B.view(lam[c]); };
    for (int i = 0; i < nord; ++i) {
        std::vector<View> in = src_in[i];
        for (int c : children[i]) in.push_back(lam_view(c));
        if (in.empty()) continue;
        lam[i] = B.emit(in, order[i], false);
        int par = B.first_bucket(p.msgs[lam[i] - p.n_src].vars, i + 1);
        if (par >= 0) children[par].push_back(i);
    }
    // sum everything in `in` except `keep` (elimination-rank order): one fused
    // bucket for the first variable, then single-input sums
    auto reduce = [&](const std::vector<View> &in, const std::vector<int> &keep, bool materialise) -> View {
        std::vector<int> y;
        for (int v : chain_scope(in))
            if (std::find(keep.begin(), keep.end(), v) == keep.end()) y.push_back(v);
        std::sort(y.begin(), y.end(), [&](int a, int b) { return B.rank[a] < B.rank[b]; });
        if (y.empty()) {
            if (in.size() == 1 && !(materialise && (in[0].table < p.n_src || in[0].base != 0))) return in[0];
            return B.view(B.emit(in, -1, false));
        }
        int t = B.emit(in, y[0], false);
        for (size_t j = 1; j < y.size(); ++j) t = B.emit({B.view(t)}, y[j], false);
        return B.view(t);
    };
    // backward (distribute) pass, parents before children:
    // pi_i = sum_{scope(p) \ sep_i} F_p * pi_p * prod_{c != i} lam_c
    std::vector<View> pi(nord);
    std::vector<char> has_pi(nord, 0);
    for (int q = nord - 1; q >= 0; --q) {
        if (lam[q] < 0) continue;
        for (int i : children[q]) {
            std::vector<View> in = src_in[q];
            if (has_pi[q]) in.push_back(pi[q]);
            for (int c : children[q])
                if (c != i) in.push_back(lam_view(c));
            if (in.empty()) continue;                    // constant 1
            pi[i] = reduce(in, p.msgs[lam[i] - p.n_src].vars, false);
            has_pi[i] = 1;
        }
    }
    // marginals: the belief of the target's bucket, or of the smallest
    // separator below it (lam_c * pi_c), summed down to the target
    for (size_t ti = 0; ti < targets.size(); ++ti) {
        const int t = targets[ti];
        const bool mine = (int)(ti % (size_t)n_parts) == part;
        p.results_owned.push_back(mine);
        int i = t >= 0 && t < (int)cards.size() ? B.rank[t] : -1;
        if (!mine || i < 0 || lam[i] < 0) {              // other part / evidence / in no factor
            p.results.push_back(-1);
            p.results_vars.push_back({});
            continue;
        }
        std::vector<View> best = src_in[i];
        if (has_pi[i]) best.push_back(pi[i]);
        for (int c : children[i]) best.push_back(lam_view(c));
        double best_size = (double)table_size(chain_scope(best), cards);
        for (int c : children[i]) {
            double sz = (double)p.msgs[lam[c] - p.n_src].size;
            if (sz < best_size) {
                best = {lam_view(c)};
                if (has_pi[c]) best.push_back(pi[c]);
                best_size = sz;
            }
        }
        int rt = B.reduce_to(best, t);
        p.results.push_back(rt);
        p.results_vars.push_back(p.msgs[rt - p.n_src].vars);
    }
    B.finish();
    return p;
}

// ------------------------------------------- chain bucket tree, checkpointed
namespace {
int64_t binom_capped(int n, int k) {             // C(n, k), saturating at 2^40
    if (k < 0 || k > n) return 0;
    k = std::min(k, n - k);
    double r = 1;
    for (int i = 1; i <= k; ++i) {
        r = r * (n - k + i) / i;
        if (r > 1099511627776.0) return (int64_t)1 << 40;
    }
    return (int64_t)(r + 0.5);
}
}  // namespace

bool plan_bucket_tree_chain(const std::vector<int> &cards, const std::vector<View> &sources,
                            const std::vector<int> &order, const std::vector<int> &targets, int slots,
                            int part, int n_parts, VEPlan &out, std::string *msg, int chain_eb, int n_slices,
                            int slice_rank, bool lanes, int elem_bytes) {
    if (n_parts < 1 || part < 0 || part >= n_parts) {
        if (msg) *msg = "bad part";
        return false;
    }
    int sbits = 0;
    while ((1 << sbits) < n_slices && sbits < 16) ++sbits;
    if (n_slices < 1 || (1 << sbits) != n_slices || slice_rank < 0 || slice_rank >= n_slices ||
        (n_slices > 1 && n_parts != 1)) {
        if (msg) *msg = "bad slicing: n_slices must be a power of two, 0 <= rank < n_slices, one part";
        return false;
    }
    VEPlan p;
    p.n_slices = n_slices;
    p.slice_rank = slice_rank;
    PlanBuilder B(cards, p, sources, order, true);
    B.sequential = true;
    B.chain_eb = chain_eb;
    const int nord = (int)order.size();
    // symbolic forward pass: bucket contents, message scopes, tree shape
    std::vector<std::vector<View>> src_in(nord);
    std::vector<int> child(nord, -1), parent(nord, -1);
    std::vector<char> has(nord, 0);
    std::vector<std::vector<int>> lam_vars(nord);
    for (const View &sv : sources) {
        int bi = B.first_bucket(sv.vars, 0);
        if (bi >= 0) src_in[bi].push_back(sv);
    }
    for (int i = 0; i < nord; ++i) {
        std::vector<View> in = src_in[i];
        if (child[i] >= 0) in.push_back(natural_view(0, lam_vars[child[i]], cards));
        if (in.empty()) continue;
        has[i] = 1;
        lam_vars[i] = B.canon(remove_var(chain_scope(in), order[i]));
        int par = B.first_bucket(lam_vars[i], i + 1);
        parent[i] = par;
        if (par >= 0) {
            if (child[par] >= 0) {
                if (msg) *msg = "bucket tree is not a chain (a bucket has two children)";
                return false;
            }
            child[par] = i;
        }
    }
    std::vector<int> result_of(cards.size(), -1), slice_bit_of(cards.size(), -1);
    bool ok = true;
    std::string fail_msg;
    auto reduce_to = [&](std::vector<View> in, int t) { return B.reduce_to(std::move(in), t); };
    // paths (leaf ... root); marginals are owned by contiguous segments of the
    // concatenated paths, one segment per part
    std::vector<std::vector<int>> paths;
    for (int top = 0; top < nord; ++top) {
        if (!has[top] || parent[top] >= 0) continue;
        std::vector<int> path;
        for (int b = top; b >= 0; b = child[b]) path.push_back(b);
        std::reverse(path.begin(), path.end());
        paths.push_back(path);
    }
    int64_t total = 0;
    for (auto &pa : paths) total += (int64_t)pa.size();
    const int64_t g_lo = total * part / n_parts, g_hi = total * (part + 1) / n_parts;
    std::vector<char> owned_var(cards.size(), part == 0 ? 1 : 0);   // variables on no path: part 0
    // Deliveries: positions j where lam_j * pi_j (the belief over sep_j) is
    // formed.  One belief gives, in one pass that sums its slowest variables
    // (a composite of card <= kSlowMax), a small table over its fastest
    // variables (kept set K_j, <= kKeepMax entries); every owned target in K_j
    // takes its marginal from that table.  The deliveries are a minimum set of
    // positions stabbing every target's interval {j : x_q in K_j} (greedy by
    // right end), so a 32-wide column sweep needs one delivery per ~20
    // positions, and the forward messages are only recomputed to reach those.
    // 2^24 kept entries (measured on the 32x32 column sweep: 2^21 -> 2^24 cuts
    // the plan from 14.6 to 13.3 TB and the MAR from 2.96 to 2.73 s; kept sets
    // matter only for separators above 2^24 entries).  A delivery's belief is
    // formed inside the backward run that ends there when that run's slots
    // are the summed variables (attach_belief): fp32 runs of 8, fp64 runs of
    // at most 7, so fp64 beliefs of a 32-wide separator (8 summed variables)
    // stay separate passes -- fp64 used 2^25 kept entries until round 6 to
    // fuse them, but with four checkpoint slots (plan.cpp place_levels) 2^24
    // moves 31.85 TB against 34.27 and the fp64 32x32 MAR runs 5.93 s against
    // 6.44-6.50 (fused fp64 runs of 8, BNPP_F64_BEL8: 5.95 s;
    // profiles/r06_f64_keep_ab.txt).  BNPP_KEEP_LOG2 / BNPP_SLOW_LOG2
    // override them (tests use tiny values on small grids).
    const char *ke = std::getenv("BNPP_KEEP_LOG2"), *se = std::getenv("BNPP_SLOW_LOG2");
    const int64_t kKeepMax = (int64_t)1 << (ke ? std::atoi(ke) : 24),
                  kSlowMax = (int64_t)1 << (se ? std::atoi(se) : 13);
    auto slow_part = [&](const std::vector<int> &sep) {     // slowest vars summed in the first pass
        std::vector<int> slow;
        int64_t P = 1;
        for (int v : sep) P *= cards[v];
        int64_t sp = 1;
        for (int v : sep) {
            if (P / sp <= kKeepMax || sp * cards[v] > kSlowMax) break;
            sp *= cards[v];
            slow.push_back(v);
        }
        return slow;
    };
    int64_t off = 0;
    for (const std::vector<int> &path : paths) {
        const int m = (int)path.size();
        for (int q = 0; q < m; ++q) owned_var[order[path[q]]] = 0;
        const int a = (int)std::max<int64_t>(0, std::min<int64_t>(m, g_lo - off));
        const int b = (int)std::max<int64_t>(0, std::min<int64_t>(m, g_hi - off));
        off += m;
        if (a >= b) continue;
        for (int q = a; q < b; ++q) owned_var[order[path[q]]] = 1;
        B.lane = 0;
        // ---- message slicing (n_slices > 1) ----
        // windows: win[j] = the window of position j (-1: every rank holds the
        // whole message), Sw[k] its slice variables (canonical order; S[i]'s
        // value on rank r is bit sbits-1-i of r, so the rank is the block index
        // of the slice variables read as a mixed-radix number, slowest first).
        // A window opens at a boundary position e with the b latest-eliminated
        // variables of sep_e (binary), and lasts while they stay in the
        // separators: on a grid's column sweep ~30 positions.
        std::vector<int> win(m, -1);
        std::vector<std::vector<int>> Sw;
        if (sbits > 0) {
            const char *mw = tuning_knob("BNPP_SLICE_MIN_WIN");
            const int min_win = mw ? std::max(1, std::atoi(mw)) : 8;
            auto top_b = [&](int j, std::vector<int> &S) {
                const std::vector<int> &sep = lam_vars[path[j]];
                if ((int)sep.size() < 2 * sbits) return false;
                S.assign(sep.end() - sbits, sep.end());
                for (int v : S)
                    if (cards[v] != 2 || B.rank[v] < 0) return false;
                return true;
            };
            auto in_sep = [&](int j, const std::vector<int> &S) {
                for (int v : S)
                    if (!contains(lam_vars[path[j]], v)) return false;
                return true;
            };
            int j = 0;
            while (j + 1 < m) {
                std::vector<int> S;
                bool can = top_b(j, S);
                if (can && win[j] >= 0)                          // re-slice: the new set avoids the old
                    for (int v : S) can = can && !contains(Sw[win[j]], v);
                int f = j;
                while (can && f + 1 < m && in_sep(f + 1, S)) ++f;
                if (!can || f - j < min_win) {
                    ++j;
                    continue;
                }
                for (int q = j + 1; q <= f; ++q) win[q] = (int)Sw.size();
                Sw.push_back(S);
                j = f;
            }
        }
        static const std::vector<int> kNoSlice;
        auto Sof = [&](int w) -> const std::vector<int> & { return w < 0 ? kNoSlice : Sw[w]; };
        // a view with the slice variables S fixed to this rank's bits
        auto cond = [&](const View &v, const std::vector<int> &S) {
            if (S.empty()) return v;
            View w;
            w.table = v.table;
            w.base = v.base;
            for (size_t i = 0; i < v.vars.size(); ++i) {
                auto it = std::find(S.begin(), S.end(), v.vars[i]);
                if (it == S.end()) {
                    w.vars.push_back(v.vars[i]);
                    w.strides.push_back(v.strides[i]);
                } else {
                    const int bit = sbits - 1 - (int)(it - S.begin());
                    w.base += (int64_t)((slice_rank >> bit) & 1) * v.strides[i];
                }
            }
            return w;
        };
        // the factor tables of the bucket at position q, as its window's ranks see them
        auto src_at = [&](int q) {
            std::vector<View> r;
            for (const View &v : src_in[path[q]]) r.push_back(cond(v, Sof(win[q])));
            return r;
        };
        // the message at position pos (sliced for window wf) re-sliced for window wt
        auto xchg = [&](View cur, int pos, int wf, int wt) -> View {
            if (wf == wt || !ok) return cur;
            const std::vector<int> &So = Sof(wf), &Sn = Sof(wt);
            if (So.empty()) return cond(cur, Sn);             // whole -> slice: a conditioned view
            if (cur.table < p.n_src || cur.base != 0 || cur.vars != p.msgs[cur.table - p.n_src].vars)
                cur = B.view(B.emit({cur}, -1, false));        // exchange whole message tables only
            const std::vector<int> &A = cur.vars;
            std::vector<int> rest, sendv;
            int pmode = 0;
            if (!Sn.empty()) {
                for (int v : A)
                    if (!contains(Sn, v)) rest.push_back(v);
                const bool slow = A.size() >= Sn.size() && std::equal(Sn.begin(), Sn.end(), A.begin());
                const bool fast = A.size() >= Sn.size() && std::equal(Sn.begin(), Sn.end(), A.end() - Sn.size());
                if (!slow && !fast) {
                    ok = false;
                    fail_msg = "slicing: the new slice variables are not the slowest or fastest of the message";
                    return cur;
                }
                pmode = slow ? 0 : 1;
                sendv = Sn;
                sendv.insert(sendv.end(), rest.begin(), rest.end());
            } else {
                sendv = A;
            }
            // scratch: (E_r, exp2_r) int64 pairs of n_slices + 1 ranks (xchg.hip)
            const int vx = (int)B.cards.size();
            B.cards.push_back(4 * (n_slices + 1));
            B.rank.push_back(-1);
            const std::vector<int> &within = Sn.empty() ? A : rest;
            std::vector<int> recvv = So;
            recvv.insert(recvv.end(), within.begin(), within.end());
            std::vector<int> want;
            for (int v : lam_vars[path[pos]])
                if (!contains(Sn, v)) want.push_back(v);
            want = B.canon(want);
            std::vector<int> tl = within;                      // source blocks fastest: a transpose
            tl.insert(tl.end(), So.begin(), So.end());
            if (want != recvv && want != tl) {
                ok = false;
                fail_msg = "slicing: the old slice variables are not the slowest or fastest of the message";
                return cur;
            }
            // the destination blocks already slowest (pmode 0: the pack would
            // only scale) and a transpose after the collective anyway (the
            // backward lane's re-slices, gathers at the chain's ends): the raw
            // message travels and the unpack scales each source block as it
            // transposes -- one data pass instead of two, the same arithmetic
            const bool late_scale = pmode == 0 && sendv == A && want != recvv;
            const int X = B.push_xchg({cur}, {vx}, kXchgSync, 0, n_slices);
            const View send = late_scale ? cur : B.view(B.push_xchg({cur, B.view(X)}, sendv, kXchgPack, pmode, n_slices));
            const int Tr = B.push_xchg({send}, recvv, kXchgComm, Sn.empty() ? 1 : 0, n_slices);
            ++p.n_xchg;
            const double ssz = (double)table_size(sendv, B.cards);
            p.xchg_elems += Sn.empty() ? ssz * (n_slices - 1) : ssz * (n_slices - 1) / n_slices;
            if (want == recvv) return B.view(Tr);
            if (late_scale) return B.view(B.push_xchg({B.view(Tr), B.view(X)}, want, kXchgUnpack, 2, n_slices));
            return B.view(B.push_xchg({B.view(Tr)}, want, kXchgUnpack, 1, n_slices));
        };
        // the forward message of the bucket at position q from the previous one's (or none)
        auto forward = [&](int q, const View *lam_child) {
            std::vector<View> in = src_at(q);
            if (lam_child) in.push_back(*lam_child);
            return B.view(B.emit(in, order[path[q]], false));
        };
        // kept sets K_j and the slow parts, per position
        std::vector<std::vector<int>> slow(std::max(m - 1, 0));
        for (int j = 0; j + 1 < m; ++j) slow[j] = slow_part(lam_vars[path[j]]);
        auto kept = [&](int j, int v) {
            const std::vector<int> &sep = lam_vars[path[j]];
            if (std::find(sep.begin(), sep.end(), v) == sep.end()) return false;
            return std::find(slow[j].begin(), slow[j].end(), v) == slow[j].end();
        };
        // targets x_q (q >= 1) and their intervals
        struct Tgt { int q, lo, hi; };
        std::vector<Tgt> tg;
        std::map<int, std::vector<int>> multi, direct;       // delivery position -> targets
        for (int q = std::max(a, 1); q < b; ++q) {
            const int v = order[path[q]];
            int lo = -1, hi = -1;
            for (int j = q - 1; j >= 0; --j) {
                const std::vector<int> &sep = lam_vars[path[j]];
                if (std::find(sep.begin(), sep.end(), v) == sep.end()) break;
                if (kept(j, v)) {
                    if (hi < 0) hi = j;
                    lo = j;
                }
            }
            if (hi < 0) direct[q - 1].push_back(v);          // never in a kept set: its own reduction
            else tg.push_back({q, lo, hi});
        }
        std::sort(tg.begin(), tg.end(), [](const Tgt &x, const Tgt &y) { return x.hi < y.hi; });
        std::vector<char> done(tg.size(), 0);
        for (size_t t = 0; t < tg.size(); ++t) {
            if (done[t]) continue;
            const int j = tg[t].hi;
            for (size_t u = t; u < tg.size(); ++u)
                if (!done[u] && tg[u].lo <= j && j <= tg[u].hi && kept(j, order[path[tg[u].q]])) {
                    multi[j].push_back(order[path[tg[u].q]]);
                    done[u] = 1;
                }
        }
        std::vector<int> D;
        for (auto &kv : multi) D.push_back(kv.first);
        for (auto &kv : direct)
            if (!multi.count(kv.first)) D.push_back(kv.first);
        std::sort(D.begin(), D.end());
        // backward sweep: pi_cur = pi_{pi_pos} (message from path[pi_pos + 1])
        View pi_cur;
        bool have_pi = false;                        // pi of the root: constant 1
        int pi_pos = m - 1;
        auto pi_step = [&](int j) {                  // pi_j = sum F_{j+1} * pi_{j+1} down to sep_j
            const std::vector<int> &sep_j = lam_vars[path[j]];
            std::vector<View> in = src_at(j + 1);
            if (have_pi) in.push_back(pi_cur);
            if (in.empty()) {
                have_pi = false;
                return;
            }
            std::vector<int> y;
            for (int v : chain_scope(in))
                if (std::find(sep_j.begin(), sep_j.end(), v) == sep_j.end()) y.push_back(v);
            std::sort(y.begin(), y.end(), [&](int u, int w) { return B.rank[u] < B.rank[w]; });
            if (y.empty() && in.size() == 1) {
                pi_cur = in[0];
            } else {
                int tb = B.emit(in, y.empty() ? -1 : y[0], false);
                for (size_t k = 1; k < y.size(); ++k) tb = B.emit({B.view(tb)}, y[k], false);
                pi_cur = B.view(tb);
            }
            have_pi = true;
        };
        // last: the length the run ending at j should have (a delivery's
        // belief fuses into that run only when its slots are exactly the
        // belief's summed variables, attach_belief); 0: any partition
        auto pi_down_to = [&](int j, int last = 0) {
            int jj = pi_pos - 1;
            while (jj >= j) {
                // buckets jj+1, jj, ... of one slicing window (a run may not cross an exchange)
                int span = 1;
                while (jj - span >= j && win[jj + 1 - span] == win[jj + 1]) ++span;
                // longest fusable run of backward buckets jj, jj-1, ... (chain.cuh)
                int fused = 0;
                int first = chain_first_try(span);
                const int rem = jj - j + 1;                       // buckets left down to j
                if (last >= 2 && rem > last) first = std::min(first, rem - last);
                else if (last >= 2 && rem == last) first = std::min(first, last);
                for (int F = first; F >= 2 && have_pi && !fused; --F) {
                    if (span - F == 1 && F > 2) continue;   // never strand one bucket
                    std::vector<PlanBuilder::ChainStep> steps;
                    std::vector<int> vars = pi_cur.vars;
                    for (int i = 0; i < F; ++i) {
                        const std::vector<int> &sep = lam_vars[path[jj - i]];
                        const std::vector<View> sm = src_at(jj - i + 1);
                        std::vector<int> u = vars, y;
                        for (const View &v : sm)
                            for (int w : v.vars)
                                if (!contains(u, w)) u.push_back(w);
                        for (int w : u)
                            if (!contains(sep, w)) y.push_back(w);
                        if (y.size() != 1) break;
                        steps.push_back({sm, y[0]});
                        vars = sep;
                    }
                    if ((int)steps.size() != F) continue;
                    const int t = B.emit_chain(pi_cur, steps);
                    if (t >= 0) {
                        pi_cur = B.view(t);
                        fused = F;
                    }
                }
                const int pos = fused ? jj - fused + 1 : jj;      // the message just made: pi_pos
                if (!fused) pi_step(jj);
                jj = pos - 1;
                // pi_pos's message in its own window's slicing (it was made in pos+1's)
                if (have_pi && win[pos] != win[pos + 1]) pi_cur = xchg(pi_cur, pos, win[pos + 1], win[pos]);
            }
            pi_pos = std::min(pi_pos, j);
        };
        int next_deliver = (int)D.size() - 1;
        if (std::getenv("BNPP_DEBUG_CHAIN_PLAN")) {
            std::fprintf(stderr, "[chain plan] path of %d buckets, segment [%d, %d), %zu deliveries, %d slots, lanes %d:", m, a,
                         b, D.size(), slots, (int)lanes);
            for (int d : D) std::fprintf(stderr, " %d", d);
            std::fprintf(stderr, "\n");
        }
        // the marginals delivered at position j from its belief (lam_j, pi_j)
        auto deliver_bel = [&](int j, const std::vector<View> &bel) {
            const std::vector<int> &Sj = Sof(win[j]);          // conditioned away on this rank
            std::vector<int> slow_j;
            for (int v : slow[j])
                if (!contains(Sj, v)) slow_j.push_back(v);
            auto mark = [&](const std::vector<int> &ts) {
                for (int t : ts) {
                    auto it = std::find(Sj.begin(), Sj.end(), t);
                    if (it != Sj.end()) slice_bit_of[t] = sbits - 1 - (int)(it - Sj.begin());
                }
            };
            auto mit = multi.find(j);
            if (mit != multi.end()) {
                mark(mit->second);
                int tb = -1;                                   // one pass: sum the slow vars
                if (slow_j.size() >= 2) {
                    // folded into the backward run that made pi_j, when it can be
                    // (sliced runs too: slow_j leaves out the slice variables,
                    // and attach_belief checks that lam and pi share the run's
                    // slicing and layout)
                    if (bel.size() == 2) tb = B.attach_belief(bel[1], bel[0], slow_j);
                    if (tb < 0) {
                        std::vector<View> mg = bel;
                        int vv = B.merge_group(mg, slow_j);
                        if (vv >= 0) tb = B.emit(mg, vv, false);
                    }
                } else {
                    tb = B.emit(bel, slow_j.empty() ? -1 : slow_j[0], false);
                }
                if (tb >= 0 && !std::getenv("BNPP_NO_REDUCE_MANY")) {
                    const char *nf = std::getenv("BNPP_NO_FREE_REDUCE");
                    // (breadth-first: a depth's tables are live together, so only
                    // where they are small beside the messages -- a kept table of
                    // <= 1/64 of the largest -- else the arena would grow)
                    const int64_t kt = B.p.msgs[tb - B.p.n_src].size;
                    B.free_small = !(nf && *nf == '1') && kt <= ((int64_t)1 << 25) && kt * 64 <= B.p.max_table;
                    B.free_max = kt;
                    B.free_base = B.last_level;
                    B.reduce_many(B.view(tb), mit->second, result_of);
                    B.free_small = false;
                } else {
                    for (int t : mit->second)
                        result_of[t] = tb >= 0 ? B.reduce_to({B.view(tb)}, t) : B.reduce_to(bel, t);
                }
            }
            auto dit = direct.find(j);
            if (dit != direct.end()) {
                mark(dit->second);
                for (int t : dit->second) result_of[t] = B.reduce_to(bel, t);
            }
        };
        // the run length that lets delivery j's belief fuse (attach_belief)
        const char *nbf = std::getenv("BNPP_NO_BEL_FUSE");
        const bool bel_fuse = !(nbf && *nbf == '1');
        auto bel_run = [&](int j) {
            if (!bel_fuse || !multi.count(j) || B.chain_eb == 0) return 0;
            int f = 0;                                         // the belief's summed variables on this rank
            for (int v : slow[j])
                if (!contains(Sof(win[j]), v)) ++f;
            return f >= 5 && f <= split_max_bel_f(B.chain_eb) ? f : 0;
        };
        auto deliver = [&](int i, const View &lam_j) {
            if (i != next_deliver) return false;
            const int j = D[i];
            pi_down_to(j, bel_run(j));
            std::vector<View> bel{lam_j};
            if (have_pi) bel.push_back(pi_cur);
            deliver_bel(j, bel);
            --next_deliver;
            return true;
        };
        // lam at position `to` from lam at `from` (-1: from the path's start), streamed
        auto advance = [&](const View *start, int from, int to) {
            View cur;
            int k = from + 1;
            if (start) {
                cur = *start;
            } else {                                   // the path's first bucket: no incoming message
                cur = forward(k, nullptr);
                ++k;
            }
            while (k <= to) {
                // lam_{k-1} in bucket k's slicing; a run stays in one window
                if (win[k] != win[k - 1]) cur = xchg(cur, k - 1, win[k - 1], win[k]);
                int span = 1;
                while (k + span <= to && win[k + span] == win[k]) ++span;
                // longest fusable run of forward buckets k, k+1, ... (chain.cuh)
                int fused = 0;
                for (int F = chain_first_try(span); F >= 2 && !fused; --F) {
                    if (span - F == 1 && F > 2) continue;   // never strand one bucket
                    std::vector<PlanBuilder::ChainStep> steps;
                    for (int i = 0; i < F; ++i) steps.push_back({src_at(k + i), order[path[k + i]]});
                    const int t = B.emit_chain(cur, steps);
                    if (t >= 0) {
                        cur = B.view(t);
                        fused = F;
                    }
                }
                if (fused) {
                    k += fused;
                } else {
                    if (std::getenv("BNPP_DEBUG_CHAIN"))
                        std::fprintf(stderr, "[chain] single forward bucket at %d (run %d..%d) vars %zu\n", k, from, to,
                                     cur.vars.size());
                    cur = forward(k, &cur);
                    ++k;
                }
            }
            return cur;
        };
        // reverse(lo, hi, start, spos, s): deliver D[hi-1] ... D[lo] (binomial
        // checkpointing over the deliveries); `start` = lam at spos < D[lo]
        // Where to checkpoint: the split of [lo, hi) with sl slots that
        // minimises the forward work, each step weighted by its message's
        // entries (a chain's first deliveries are one bucket apart over tiny
        // messages, the rest ~24 buckets apart over 2^32-entry ones: the
        // uniform-step binomial rule spent the slots on the cheap ones and
        // recomputed the expensive tail; 32x32: 213 -> ~140 forward runs).
        // cost(lo, hi, s), start = D[lo-1] (the prefix end for lo = 0):
        //   s = 0: sum_i adv(start, D[i]);  else min_c adv(start, D[c]) +
        //   cost(c+1, hi, s-1) + cost(lo, c, s).  O(n^3 s / 6); long delivery
        // lists (> 256) keep the binomial rule.
        const int nD = (int)D.size();
        const int sp0 = nD ? D[0] - 1 : -1;
        std::vector<double> Wc(m + 1, 0.0);                    // Wc[i + 1] = entries of lam_0..lam_i
        for (int i = 0; i < m; ++i) Wc[i + 1] = Wc[i] + (double)table_size(lam_vars[path[i]], cards);
        auto adv_cost = [&](int from, int to) { return Wc[to + 1] - Wc[from + 1]; };
        const bool use_dp = !lanes && nD > 0 && nD <= 256 && !tuning_knob("BNPP_BINOMIAL_REVOLVE");
        const int S = use_dp ? std::min(slots, nD) : 0;
        std::vector<double> cost;
        std::vector<int16_t> arg;
        auto at = [&](int lo, int hi, int sl) { return ((size_t)lo * (nD + 1) + hi) * (S + 1) + sl; };
        if (use_dp) {
            cost.assign((size_t)(nD + 1) * (nD + 1) * (S + 1), 0.0);
            arg.assign(cost.size(), -1);
            for (int len = 1; len <= nD; ++len)
                for (int lo = 0; lo + len <= nD; ++lo) {
                    const int hi = lo + len, st = lo ? D[lo - 1] : sp0;
                    double c0 = 0;
                    for (int i = lo; i < hi; ++i) c0 += adv_cost(st, D[i]);
                    cost[at(lo, hi, 0)] = c0;
                    for (int sl = 1; sl <= S; ++sl) {
                        double best = c0;
                        int bc = -1;
                        for (int c = lo; c < hi; ++c) {
                            const double v = adv_cost(st, D[c]) + cost[at(c + 1, hi, sl - 1)] + cost[at(lo, c, sl)];
                            if (v < best) {
                                best = v;
                                bc = c;
                            }
                        }
                        cost[at(lo, hi, sl)] = best;
                        arg[at(lo, hi, sl)] = (int16_t)bc;
                    }
                }
        }
        std::function<void(int, int, const View *, int, int)> reverse = [&](int rlo, int rhi, const View *start,
                                                                             int spos, int sl) {
            const int len = rhi - rlo;
            if (len <= 0 || !ok) return;
            int c = -1;
            if (use_dp) {
                c = arg[at(rlo, rhi, std::min(sl, S))];
            } else if (len > 1 && sl > 0) {
                int r = 1;
                while (binom_capped(sl + r, sl) < len) ++r;
                int64_t right_cap = binom_capped(sl - 1 + r, sl - 1);
                int d = (int)std::max<int64_t>(1, len - std::min<int64_t>(right_cap, len - 1));
                c = rlo + d - 1;
            }
            if (c < 0) {                                       // no checkpoint: every delivery from `start`
                for (int i = rhi - 1; i >= rlo; --i) ok = ok && deliver(i, advance(start, spos, D[i]));
                return;
            }
            View ck = advance(start, spos, D[c]);
            reverse(c + 1, rhi, &ck, D[c], sl - 1);
            ok = ok && deliver(c, ck);
            reverse(rlo, c, start, spos, sl);
        };
        if (lanes && !D.empty()) {
            // Two fronts, no recomputation: lane 0 streams the forward messages
            // up the chain, lane 1 the backward messages down it, concurrently
            // (the executor runs the lanes on two streams, so one lane's
            // exchanges overlap the other's buckets).  At a delivery position
            // the front that arrives first (fewer buckets from its end) keeps
            // its message; the second one forms the belief and delivers.
            struct Ev { int dist, lane, i; };
            std::vector<Ev> evs;
            for (int i = 0; i < (int)D.size(); ++i) {
                evs.push_back({D[i] + 1, 0, i});
                evs.push_back({m - 1 - D[i], 1, i});
            }
            std::sort(evs.begin(), evs.end(), [](const Ev &x, const Ev &y) {
                return x.dist != y.dist ? x.dist < y.dist : x.lane > y.lane;
            });
            std::vector<char> seen(D.size(), 0);
            std::vector<View> lam_kept(D.size()), pi_kept(D.size());
            std::vector<char> pi_kept_has(D.size(), 0);
            View lam_cur;
            int lam_pos = -1;
            const bool dbg = std::getenv("BNPP_DEBUG_LANES") != nullptr;
            for (const Ev &e : evs) {
                const int j = D[e.i];
                if (dbg) std::fprintf(stderr, "[lanes] lane %d pos %d dist %d (lam_pos %d pi_pos %d)\n", e.lane, j, e.dist, lam_pos, pi_pos);
                B.lane = e.lane;
                if (e.lane == 0) {
                    lam_cur = advance(lam_pos >= 0 ? &lam_cur : nullptr, lam_pos, j);
                    lam_pos = j;
                } else {
                    // arriving second, the backward front ends its run at j with
                    // the belief's summed variables as slots, so the belief forms
                    // inside it (attach_belief; lam comes from the other lane)
                    pi_down_to(j, seen[e.i] ? bel_run(j) : 0);
                }
                if (!seen[e.i]) {                              // first arrival: keep this front's message
                    seen[e.i] = 1;
                    if (e.lane == 0) lam_kept[e.i] = lam_cur;
                    else {
                        pi_kept[e.i] = pi_cur;
                        pi_kept_has[e.i] = have_pi;
                    }
                    continue;
                }
                std::vector<View> bel{e.lane == 0 ? lam_cur : lam_kept[e.i]};
                if (e.lane == 0 ? pi_kept_has[e.i] : have_pi) bel.push_back(e.lane == 0 ? pi_kept[e.i] : pi_cur);
                deliver_bel(j, bel);
            }
            B.lane = 1;
            next_deliver = -1;
        } else if (!D.empty()) {
            View start;                                        // prefix: stream to D[0] - 1, kept throughout
            const int sp = D[0] - 1;
            if (sp >= 0) start = advance(nullptr, -1, sp);
            reverse(0, (int)D.size(), sp >= 0 ? &start : nullptr, sp, slots);
        }
        if (!ok || next_deliver != -1) {
            if (msg) *msg = fail_msg.empty() ? "internal: checkpoint schedule out of order" : fail_msg;
            return false;
        }
        if (a == 0) {                                          // the leaf: its own bucket and pi_0
            pi_down_to(0);
            std::vector<View> bel = src_at(0);
            if (have_pi) bel.push_back(pi_cur);
            result_of[order[path[0]]] = reduce_to(bel, order[path[0]]);
        }
    }
    for (int t : targets) {
        bool in_range = t >= 0 && t < (int)cards.size();
        int r = in_range ? result_of[t] : -1;
        p.results.push_back(r);
        p.results_vars.push_back(r >= 0 ? p.msgs[r - p.n_src].vars : std::vector<int>{});
        p.results_owned.push_back(in_range ? owned_var[t] : (part == 0));
        p.results_slice_bit.push_back(r >= 0 ? slice_bit_of[t] : -1);
    }
    B.finish();
    out = std::move(p);
    return true;
}

int64_t plan_peak_bytes(const VEPlan &p, int elem_bytes) {
    const int nt = p.n_src + (int)p.msgs.size();
    std::vector<int> born(nt, 0), last(nt, -1);
    for (const BucketSpec &b : p.buckets) {
        born[b.out_table] = b.level;
        if (b.bel_table >= 0) born[b.bel_table] = b.level;
        for (const View &v : b.in) last[v.table] = std::max(last[v.table], b.level);
    }
    if (p.result_table >= 0) last[p.result_table] = p.n_levels + 1;
    for (int r : p.results)
        if (r >= 0) last[r] = p.n_levels + 1;
    std::vector<int64_t> delta(p.n_levels + 3, 0);
    for (int t = p.n_src; t < nt; ++t) {
        const int64_t bytes = sat_add(sat_mul(p.msgs[t - p.n_src].size, elem_bytes), 255) / 256 * 256;
        delta[born[t]] = sat_add(delta[born[t]], bytes);
        delta[std::max(last[t], born[t]) + 1] -= bytes;
    }
    int64_t live = 0, peak = 0;
    for (int64_t d : delta) {
        live = sat_add(live, d);
        peak = std::max(peak, live);
    }
    return peak;
}

// ------------------------------------------------------------- schedule
namespace {
struct Arena {
    // free blocks indexed by offset (merging) and by (length, offset) (best
    // fit); tree nodes come from a pool (a per-target MAR schedule makes ~10^5
    // allocations and releases)
    std::pmr::unsynchronized_pool_resource pool_;
    std::pmr::map<int64_t, int64_t> free_{&pool_};            // offset -> length
    std::pmr::set<std::pair<int64_t, int64_t>> by_len_{&pool_};   // (length, offset)
    int64_t top = 0;
    // a plan beyond any device (sizes saturated at kSatMax): stop placing
    // tables (offsets would collide at the saturated top), report kSatMax
    bool saturated = false;
    void add_free(int64_t off, int64_t len) {
        free_[off] = len;
        by_len_.insert({len, off});
    }
    void erase_free(std::pmr::map<int64_t, int64_t>::iterator it) {
        by_len_.erase({it->second, it->first});
        free_.erase(it);
    }
    int64_t alloc(int64_t n) {
        if (saturated || n >= kSatMax / 4 || top >= kSatMax / 4) {
            saturated = true;
            top = kSatMax;
            return 0;
        }
        n = (n + 255) & ~(int64_t)255;
        // best fit: the smallest free block that holds n, lowest offset among
        // equals (small temporaries go into small holes instead of splitting
        // the holes big messages need); O(log blocks)
        auto b = by_len_.lower_bound({n, INT64_MIN});
        if (b != by_len_.end()) {
            const int64_t off = b->second, len = b->first;
            erase_free(free_.find(off));
            if (len > n) add_free(off + n, len - n);
            return off;
        }
        // extend: merge with a trailing free block if present
        if (!free_.empty()) {
            auto last = std::prev(free_.end());
            if (last->first + last->second == top) {
                int64_t off = last->first;
                erase_free(last);
                top = off + n;
                return off;
            }
        }
        int64_t off = top;
        top += n;
        return off;
    }
    void release(int64_t off, int64_t n) {
        if (saturated) return;
        n = (n + 255) & ~(int64_t)255;
        auto nx = free_.lower_bound(off);
        if (nx != free_.end() && off + n == nx->first) {     // merge the next block
            n += nx->second;
            erase_free(nx);
        }
        auto it = free_.lower_bound(off);
        if (it != free_.begin()) {
            auto pv = std::prev(it);
            if (pv->first + pv->second == off) {            // merge into the previous block
                const int64_t po = pv->first, pl = pv->second;
                erase_free(pv);
                add_free(po, pl + n);
                return;
            }
        }
        add_free(off, n);
    }
};

// Place the tables of one arena level by level (born_at[L] allocated, then
// dies_at[L] released): off[t - t_base] for every table t placed.  Two
// placements are made and the one with the lower top kept: (a) one best-fit
// arena; (b) the tables of the largest size first, by interval colouring into
// K slots of that size (K = the most of them live at once: no fragmentation
// among them), then every smaller table, in level order, into a slot that no
// large table occupies during its whole lifetime (a best-fit arena per slot),
// or else into a region above the slots.  In one arena a small table left in
// a freed message's hole can leave the next message no room -- the fp64
// 32x32 bucket tree with four checkpoint slots: 240.8 GB live at its peak,
// 275.0 GB placed in one arena (one 34-GB message more).
template <class Bytes>
int64_t place_levels(int n_levels, const std::vector<std::vector<int>> &born_at,
                     const std::vector<std::vector<int>> &dies_at, Bytes &&bytes, int t_base, std::vector<int64_t> &off,
                     bool &saturated) {
    auto rnd = [](int64_t n) { return (n + 255) & ~(int64_t)255; };
    int64_t big = 0;
    size_t n_tab = 0;
    for (int L = 1; L <= n_levels; ++L) {
        n_tab += born_at[L].size();
        for (int t : born_at[L]) big = std::max(big, rnd(bytes(t)));
    }
    Arena one;
    for (int L = 1; L <= n_levels; ++L) {
        for (int t : born_at[L]) off[t - t_base] = one.alloc(bytes(t));
        for (int t : dies_at[L]) one.release(off[t - t_base], bytes(t));
    }
    saturated = one.saturated;
    // (b) only where a large table exists beside others and the walk stays cheap
    if (one.saturated || big <= 0 || one.top <= big || big >= kSatMax / 4 || n_tab > 50000) return one.top;
    const int kLive = INT_MAX;
    std::vector<int> die(off.size(), kLive);
    for (int L = 1; L <= n_levels; ++L)
        for (int t : dies_at[L]) die[t - t_base] = L;
    auto is_big = [&](int t) { return rnd(bytes(t)) == big; };
    // large tables: interval colouring (allocations of a level before its releases)
    std::vector<int> slot(off.size(), -1);
    std::vector<std::vector<std::pair<int, int>>> busy;          // per slot: (born, dies) of its large tables
    std::vector<int> free_slots;                                 // a min-heap of slot ids
    for (int L = 1; L <= n_levels; ++L) {
        for (int t : born_at[L]) {
            if (!is_big(t)) continue;
            int k;
            if (!free_slots.empty()) {
                std::pop_heap(free_slots.begin(), free_slots.end(), std::greater<int>());
                k = free_slots.back();
                free_slots.pop_back();
            } else {
                k = (int)busy.size();
                busy.emplace_back();
            }
            slot[t - t_base] = k;
            busy[k].push_back({L, die[t - t_base]});
        }
        for (int t : dies_at[L]) {
            if (!is_big(t)) continue;
            free_slots.push_back(slot[t - t_base]);
            std::push_heap(free_slots.begin(), free_slots.end(), std::greater<int>());
        }
    }
    const int K = (int)busy.size();
    std::vector<Arena> in_slot(K);
    Arena above;
    std::vector<int64_t> off2(off.size(), 0);
    for (int L = 1; L <= n_levels; ++L) {
        for (int t : born_at[L]) {
            const int i = t - t_base;
            if (is_big(t)) {
                off2[i] = (int64_t)slot[i] * big;
                continue;
            }
            const int64_t n = bytes(t);
            const int d = die[i];
            int got = -1;
            for (int k = 0; k < K && got < 0; ++k) {
                bool clear = true;
                for (const auto &iv : busy[k])
                    if (iv.first <= d && L <= iv.second) {
                        clear = false;
                        break;
                    }
                if (!clear) continue;
                const int64_t o = in_slot[k].alloc(n);
                if (o + rnd(n) <= big) {
                    got = k;
                    off2[i] = (int64_t)k * big + o;
                } else {
                    in_slot[k].release(o, n);
                }
            }
            if (got < 0) {
                slot[i] = -2;                               // above the slots
                off2[i] = above.alloc(n);
            } else {
                slot[i] = got;
            }
        }
        for (int t : dies_at[L]) {
            const int i = t - t_base;
            if (is_big(t)) continue;
            if (slot[i] == -2) above.release(off2[i], bytes(t));
            else in_slot[slot[i]].release(off2[i] - (int64_t)slot[i] * big, bytes(t));
        }
    }
    // near-ties (within 1 %) go to the slots: the messages then sit at
    // multiples of their own size, where the split runs are fastest (§7 round 6)
    const int64_t base_above = (int64_t)K * big;
    if (std::getenv("BNPP_DEBUG_ARENA"))
        std::fprintf(stderr, "[bnpp] placement: one arena %.2f GB, %d slots of %.2f GB + %.2f GB above\n", one.top / 1e9,
                     K, big / 1e9, above.top / 1e9);
    if (above.saturated || sat_add(base_above, above.top) > one.top + one.top / 100) return one.top;
    for (int L = 1; L <= n_levels; ++L)
        for (int t : born_at[L]) {
            const int i = t - t_base;
            off[i] = slot[i] == -2 ? base_above + off2[i] : off2[i];
        }
    return base_above + above.top;
}
}  // namespace

int64_t plan_arena_bytes(const VEPlan &p, int elem_bytes) {
    const int nt = p.n_src + (int)p.msgs.size();
    std::vector<int> born(nt, 0), last(nt, -1);
    for (const BucketSpec &b : p.buckets) {
        born[b.out_table] = b.level;
        if (b.bel_table >= 0) born[b.bel_table] = b.level;
        for (const View &v : b.in) last[v.table] = std::max(last[v.table], b.level);
    }
    std::vector<char> keep(nt, 0);
    if (p.result_table >= 0) keep[p.result_table] = 1;
    for (int r : p.results)
        if (r >= 0) keep[r] = 1;
    std::vector<std::vector<int>> born_at(p.n_levels + 2), dies_at(p.n_levels + 2);
    for (int t = p.n_src; t < nt; ++t) {
        born_at[born[t]].push_back(t);
        if (!keep[t]) dies_at[std::max(last[t], born[t])].push_back(t);
    }
    std::vector<int64_t> off(nt, 0);
    auto bytes = [&](int t) { return sat_mul(p.msgs[t - p.n_src].size, elem_bytes); };
    bool sat = false;
    const int64_t top = place_levels(p.n_levels, born_at, dies_at, bytes, 0, off, sat);
    if (std::getenv("BNPP_DEBUG_ARENA")) {
        int64_t live = 0, peak = 0;
        for (int L = 1; L <= p.n_levels; ++L) {
            for (int t : born_at[L]) live += bytes(t);
            peak = std::max(peak, live);
            for (int t : dies_at[L]) live -= bytes(t);
        }
        std::fprintf(stderr, "[bnpp] arena %.2f GB, ideal live peak %.2f GB\n", top / 1e9, peak / 1e9);
    }
    return sat ? kSatMax : top;
}

bool build_schedule(const std::vector<const VEPlan *> &plans, const std::vector<int> &cards,
                    const std::vector<int64_t> &src_sizes, int elem_bytes, int max_vec, Schedule &s,
                    std::string *msg, int64_t arena_cap) {
    s = Schedule{};
    const bool timing = std::getenv("BNPP_TIMING") != nullptr;
    auto clk = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double T0 = clk();
    // small schedules (a PR over a few thousand buckets) build faster on one
    // thread than the workers' hand-off costs
    int64_t n_buckets_all = 0;
    for (const VEPlan *p : plans) n_buckets_all += (int64_t)p->buckets.size();
    ScopedHostThreads one_thread(n_buckets_all < 8192 ? 1 : 0);
    s.n_src = (int)src_sizes.size();
    s.table_size = src_sizes;
    s.table_offset.assign(src_sizes.size(), -1);
    std::vector<int> msg_base;
    int n_levels = 0;
    for (const VEPlan *p : plans) {
        if (p->n_src != s.n_src) {
            if (msg) *msg = "plans disagree on the number of sources";
            return false;
        }
        msg_base.push_back((int)s.table_size.size());
        for (const MsgTable &t : p->msgs) s.table_size.push_back(t.size);
        n_levels = std::max(n_levels, p->n_levels);
        s.entries += p->entries;
        s.elems_moved += p->elems_moved;
        s.width = std::max(s.width, p->width);
    }
    s.n_tables = (int)s.table_size.size();
    s.table_offset.resize(s.n_tables, -1);
    // Many plans (per-target MAR, BN::marginals's one VE per target): a bucket
    // structurally identical to one of an earlier plan -- the same summed
    // variable, output layout, level and inputs (sources or identical buckets'
    // outputs, with the same views) -- computes the same table bit for bit, so
    // it runs once and every plan reads its output.  Targets whose min-fill
    // orders share a prefix share those buckets (about half of the 12x32 grid's
    // 147,456).  canon[t]: the table every later reference to t reads.
    std::vector<int> canon(s.n_tables);
    for (int t = 0; t < s.n_tables; ++t) canon[t] = t;
    const char *nd = std::getenv("BNPP_NO_DEDUP");
    const bool dedup = plans.size() > 1 && !(nd && *nd == '1');
    if (dedup) {
        struct Key {
            uint64_t h1, h2;
            int t;
        };
        std::vector<Key> keys(s.n_tables - s.n_src);
        parallel_for((int64_t)plans.size(), [&](int64_t pi) {
            const VEPlan &p = *plans[pi];
            std::vector<std::pair<uint64_t, uint64_t>> th(p.msgs.size(), {0, 0});
            for (const BucketSpec &b : p.buckets) {
                uint64_t h1 = 0x9e3779b97f4a7c15ull, h2 = 0xc2b2ae3d27d4eb4full;
                auto mix = [&](uint64_t x) {
                    h1 = (h1 ^ x) * 0x100000001b3ull;
                    h1 ^= h1 >> 29;
                    h2 = (h2 + x + 0x632be59bd9b4e019ull) * 0x9e3779b97f4a7c15ull;
                    h2 ^= h2 >> 31;
                };
                mix((uint64_t)(uint32_t)b.elim_var);
                mix((uint64_t)b.level);
                mix((uint64_t)(b.xchg * 16 + b.xchg_mode));
                mix(b.divide ? 1 : 0);
                mix(b.out_vars.size());
                for (int v : b.out_vars) mix((uint64_t)v);
                mix(b.chain_x.size() * 131 + b.chain_n.size() * 7 + (uint64_t)b.chain_gmask);
                for (int v : b.chain_x) mix((uint64_t)(uint32_t)v);
                for (int v : b.chain_n) mix((uint64_t)(uint32_t)v);
                mix(p.cards_ext.size());
                for (const View &v : b.in) {
                    if (v.table < p.n_src) {
                        mix(0xabcdull);
                        mix((uint64_t)v.table);
                    } else {
                        mix(th[v.table - p.n_src].first);
                        mix(th[v.table - p.n_src].second);
                    }
                    mix((uint64_t)v.base);
                    for (size_t j = 0; j < v.vars.size(); ++j) {
                        mix((uint64_t)v.vars[j]);
                        mix((uint64_t)v.strides[j]);
                    }
                }
                th[b.out_table - p.n_src] = {h1, h2};
                if (b.bel_table >= 0) th[b.bel_table - p.n_src] = {h1 ^ 0x5bd1e9955bd1e995ull, h2 + 0x27d4eb2f165667c5ull};
            }
            for (size_t i = 0; i < p.msgs.size(); ++i) {
                const int g = msg_base[pi] + (int)i;
                keys[g - s.n_src] = {th[i].first, th[i].second, g};
            }
        });
        // equal keys share their top bits: 64 shards sorted and grouped in parallel
        constexpr int kShards = 64;
        std::vector<std::vector<Key>> shard(kShards);
        {
            std::vector<size_t> cnt(kShards, 0);
            for (const Key &k : keys) ++cnt[k.h1 >> 58];
            for (int sh = 0; sh < kShards; ++sh) shard[sh].reserve(cnt[sh]);
            for (const Key &k : keys) shard[k.h1 >> 58].push_back(k);
        }
        parallel_for(kShards, [&](int64_t sh) {
            std::vector<Key> &v = shard[sh];
            std::sort(v.begin(), v.end(), [](const Key &a, const Key &b) {
                return a.h1 != b.h1 ? a.h1 < b.h1 : a.h2 != b.h2 ? a.h2 < b.h2 : a.t < b.t;
            });
            for (size_t i = 1; i < v.size(); ++i)
                if (v[i].h1 == v[i - 1].h1 && v[i].h2 == v[i - 1].h2 && (v[i].h1 | v[i].h2) != 0)
                    canon[v[i].t] = canon[v[i - 1].t];  // the first occurrence (lowest id) of the group
        });
    }
    const double Td = clk();
    auto remap = [&](size_t pi, int t) { return t < s.n_src ? t : canon[msg_base[pi] + (t - s.n_src)]; };
    // a bucket runs when it produces its table's canonical copy
    auto kept = [&](size_t pi, const BucketSpec &b) {
        const int g = msg_base[pi] + (b.out_table - s.n_src);
        return canon[g] == g;
    };
    if (dedup) {
        // work actually scheduled: the kept buckets' factor-entries and traffic
        // (plain buckets; a schedule with fused runs keeps the plans' sums)
        std::vector<double> pe(plans.size(), 0), pm(plans.size(), 0);
        std::vector<char> pplain(plans.size(), 1);
        parallel_for((int64_t)plans.size(), [&](int64_t pi) {
            const std::vector<int> &pc = plans[pi]->cards_ext.empty() ? cards : plans[pi]->cards_ext;
            for (const BucketSpec &b : plans[pi]->buckets) {
                if (!b.chain_x.empty()) {
                    pplain[pi] = 0;
                    break;
                }
                if (!kept(pi, b)) continue;
                // factor-entries: prod(card) over the union scope = output x summed card
                const double out = (double)table_size(b.out_vars, pc);
                pe[pi] += out * (b.elim_var >= 0 ? pc[b.elim_var] : 1);
                pm[pi] += out;
                for (const View &v : b.in) pm[pi] += (double)table_size(v.vars, pc);
            }
        });
        bool plain = true;
        double e = 0, mv = 0;
        for (size_t pi = 0; pi < plans.size(); ++pi) {
            plain = plain && pplain[pi];
            e += pe[pi];
            mv += pm[pi];
        }
        if (plain) {
            s.entries = e;
            s.elems_moved = mv;
        }
    }

    // lifetimes: produced level, last consuming level
    const int kForever = INT_MAX;
    std::vector<int> born(s.n_tables, 0), last(s.n_tables, -1);
    // per plan in parallel: a canonical table is born once; its last use is
    // the latest level of any plan's kept consumer (atomic max)
    parallel_for((int64_t)plans.size(), [&](int64_t pi) {
        for (const BucketSpec &b : plans[pi]->buckets) {
            if (!kept(pi, b)) continue;
            born[remap(pi, b.out_table)] = b.level;
            if (b.bel_table >= 0) born[remap(pi, b.bel_table)] = b.level;
            for (const View &v : b.in) {
                int *lt = &last[remap(pi, v.table)];
                int cur = __atomic_load_n(lt, __ATOMIC_RELAXED);
                while (cur < b.level &&
                       !__atomic_compare_exchange_n(lt, &cur, b.level, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
                }
            }
        }
    });
    // lanes (sliced two-front schedules): a table is placed in its producer's
    // lane's arena; one read by another lane is kept to the end (the lanes
    // run concurrently, so a later level of the producer's lane may not
    // reuse memory the other lane has yet to read)
    std::vector<int> lane_of(s.n_tables, 0);
    int n_lanes = 1;
    for (size_t pi = 0; pi < plans.size(); ++pi)
        for (const BucketSpec &b : plans[pi]->buckets) {
            if (!kept(pi, b)) continue;
            lane_of[remap(pi, b.out_table)] = b.lane;
            if (b.bel_table >= 0) lane_of[remap(pi, b.bel_table)] = b.lane;
            n_lanes = std::max(n_lanes, b.lane + 1);
        }
    if (n_lanes > 1)
        for (size_t pi = 0; pi < plans.size(); ++pi)
            for (const BucketSpec &b : plans[pi]->buckets) {
                if (!kept(pi, b)) continue;
                for (const View &v : b.in) {
                    const int t = remap(pi, v.table);
                    if (t >= s.n_src && lane_of[t] != b.lane) last[t] = kForever;
                }
            }
    for (size_t pi = 0; pi < plans.size(); ++pi) {
        std::vector<int> res = plans[pi]->results;
        std::vector<std::vector<int>> res_vars = plans[pi]->results_vars;
        if (res.empty()) {                      // single-result plan (PR / one MAR target / VE)
            res.push_back(plans[pi]->result_table);
            res_vars.push_back(plans[pi]->result_vars);
        }
        for (size_t r = 0; r < res.size(); ++r) {
            if (res[r] >= 0) last[remap(pi, res[r])] = kForever;
            s.plan_result_table.push_back(res[r] >= 0 ? remap(pi, res[r]) : -1);
            s.plan_result_vars.push_back(res_vars[r]);
            s.plan_result_owned.push_back(r < plans[pi]->results_owned.size() ? plans[pi]->results_owned[r] : 1);
            s.plan_result_slice_bit.push_back(r < plans[pi]->results_slice_bit.size() ? plans[pi]->results_slice_bit[r] : -1);
        }
    }
    std::vector<std::vector<int>> born_at(n_levels + 2), dies_at(n_levels + 2);
    for (int t = s.n_src; t < s.n_tables; ++t) {
        if (canon[t] != t) continue;                  // an alias: never placed
        born_at[born[t]].push_back(t);
        if (last[t] != kForever) dies_at[std::max(last[t], born[t])].push_back(t);
    }
    const double Tl = clk();
    // Many plans (per-target MAR): each plan's tables are placed in an arena
    // of its own, in parallel, and the arenas laid side by side -- when their
    // sum fits arena_cap.  One shared arena (below) reuses memory across plans
    // and is the fallback; it is a serial best-fit walk over every table
    // (136 ms for the 147,456 buckets of the 12x32 per-target MAR).
    bool placed = false;
    const char *sa = tuning_knob("BNPP_SHARED_ARENA");
    if (plans.size() > 1 && !(sa && *sa == '1')) {
        std::vector<int64_t> tops(plans.size(), 0);
        std::vector<char> sat(plans.size(), 0);
        std::vector<int64_t> offs(s.n_tables, 0);
        parallel_for((int64_t)plans.size(), [&](int64_t pi) {
            const int t0 = msg_base[pi], t1 = t0 + (int)plans[pi]->msgs.size();
            std::vector<std::vector<int>> ba(n_levels + 2), da(n_levels + 2);
            for (int t = t0; t < t1; ++t) {
                if (canon[t] != t) continue;
                ba[born[t]].push_back(t);
                if (last[t] != kForever) da[std::max(last[t], born[t])].push_back(t);
            }
            std::vector<int64_t> lo(t1 - t0, 0);
            bool st = false;
            tops[pi] = place_levels(n_levels, ba, da, [&](int t) { return sat_mul(s.table_size[t], elem_bytes); }, t0,
                                    lo, st);
            for (int L = 1; L <= n_levels; ++L)
                for (int t : ba[L]) offs[t] = lo[t - t0];
            sat[pi] = st;
        });
        int64_t total = 0;
        bool any_sat = false;
        for (size_t pi = 0; pi < plans.size(); ++pi) {
            total = sat_add(total, tops[pi]);
            any_sat = any_sat || sat[pi];
        }
        if (!any_sat && total <= arena_cap) {
            int64_t base = 0;
            for (size_t pi = 0; pi < plans.size(); ++pi) {
                const int t0 = msg_base[pi], t1 = t0 + (int)plans[pi]->msgs.size();
                for (int t = t0; t < t1; ++t)
                    if (canon[t] == t) s.table_offset[t] = base + offs[t];
                base += tops[pi];
            }
            s.arena_bytes = total;
            placed = true;
        }
    }
    if (!placed) {
        int64_t base = 0;
        bool sat = false;
        std::vector<int64_t> lane_base(n_lanes, 0);
        for (int l = 0; l < n_lanes; ++l) {
            std::vector<std::vector<int>> ba(n_levels + 2), da(n_levels + 2);
            for (int L = 0; L < n_levels + 2; ++L) {
                for (int t : born_at[L])
                    if (lane_of[t] == l) ba[L].push_back(t);
                for (int t : dies_at[L])
                    if (lane_of[t] == l) da[L].push_back(t);
            }
            std::vector<int64_t> lo(s.n_tables - s.n_src, 0);
            bool st = false;
            const int64_t top = place_levels(n_levels, ba, da, [&](int t) { return sat_mul(s.table_size[t], elem_bytes); },
                                             s.n_src, lo, st);
            for (int L = 1; L <= n_levels; ++L)
                for (int t : ba[L]) s.table_offset[t] = lo[t - s.n_src];
            // a lane's arena starts at a multiple of its largest table (up to
            // 1 GiB): its messages keep the alignment place_levels gave them
            int64_t big = 256;
            for (int L = 1; L <= n_levels; ++L)
                for (int t : ba[L]) big = std::max(big, sat_mul(s.table_size[t], elem_bytes));
            big = std::min<int64_t>(big, (int64_t)1 << 30);
            if (l > 0 && base % big) base = sat_add(base, big - base % big);
            lane_base[l] = base;
            base = sat_add(base, top);
            sat = sat || st;
        }
        if (n_lanes > 1)
            for (int t = s.n_src; t < s.n_tables; ++t)
                if (canon[t] == t && s.table_offset[t] >= 0) s.table_offset[t] += lane_base[lane_of[t]];
        s.arena_bytes = base;
        if (sat) {                           // tables of 2^58+ bytes: no descriptors for those
            if (msg) *msg = "the plan's tables exceed any device (more than 2^58 bytes); use a narrower elimination order";
            return false;
        }
    }
    s.n_lanes = n_lanes;
    for (int t = s.n_src; t < s.n_tables; ++t)
        if (canon[t] != t) s.table_offset[t] = s.table_offset[canon[t]];
    const double T1 = clk();

    // descriptors: built in parallel (one per bucket, private dims-pool rows),
    // then grouped per level by kernel variant and concatenated
    struct Item {
        int level;
        size_t plan;
        const BucketSpec *b;
        BucketDesc d;
        std::vector<int64_t> pool;
        int key;
        bool ok;
        std::string msg;
    };
    std::vector<Item> items;
    for (size_t pi = 0; pi < plans.size(); ++pi)
        for (const BucketSpec &b : plans[pi]->buckets)
            if (kept(pi, b)) items.push_back(Item{b.level, pi, &b, BucketDesc{}, {}, 0, true, {}});
    // small plain buckets of levels holding several buckets (per-target MAR:
    // ~9 tile / input-count variants per level, 1018 launches at 12x32) share
    // one generic 1x1 launch per level: launches, not bytes, bound them
    int64_t simple_max = 4096;                         // output entries (BNPP_SIMPLE_MAX: tuning)
    if (const char *e = tuning_knob("BNPP_SIMPLE_MAX")) simple_max = std::atoll(e);
    std::vector<int> lvl_n(n_levels + 2, 0);
    for (const Item &it : items) ++lvl_n[it.level];
    const char *ns = tuning_knob("BNPP_NO_SIMPLE_LEVELS");
    const bool simplify = !(ns && *ns == '1');
    // BNPP_NO_O32=1: generic kernels with 64-bit offsets only (tests compare the two bit for bit)
    const char *no32 = std::getenv("BNPP_NO_O32");
    const bool no_o32 = no32 && *no32 == '1';
    parallel_for((int64_t)items.size(), [&](int64_t idx) {
        Item &it = items[idx];
        BucketSpec b = *it.b;
        b.simple = simplify && lvl_n[it.level] > 1 && b.chain_x.empty() && !b.divide && !b.xchg &&
                   plans[it.plan]->msgs[b.out_table - s.n_src].size <= simple_max;
        for (View &v : b.in) v.table = remap(it.plan, v.table);
        b.out_table = remap(it.plan, b.out_table);
        if (b.bel_table >= 0) b.bel_table = remap(it.plan, b.bel_table);
        if (b.xchg) {                        // an exchange step: the executor's, no kernel descriptor
            it.d = BucketDesc{};
            it.d.n_in = (int)b.in.size();
            for (int i = 0; i < it.d.n_in && i < kMaxDescIn; ++i) it.d.in_table[i] = b.in[i].table;
            it.d.out_table = b.out_table;
            it.d.k = b.xchg_blocks;
            it.d.out_size = s.table_size[b.out_table];
            it.key = kXchgKeyBase + b.xchg * 16 + b.xchg_mode;
            it.ok = b.in.size() <= (size_t)kMaxDescIn;
            return;
        }
        const std::vector<int> &pc = plans[it.plan]->cards_ext.empty() ? cards : plans[it.plan]->cards_ext;
        it.ok = build_desc(b, pc, max_vec, it.d, it.pool, &it.msg);
        auto max_in_bytes = [&](const BucketSpec &bs) {
            int64_t m = 0;
            for (const View &v : bs.in) m = std::max(m, sat_mul(s.table_size[v.table], elem_bytes));
            return m;
        };
        it.key = it.d.chain ? chain_key((it.d.chain >> 16) & 0xf, it.d.k, it.d.chain & 0xff, (it.d.chain >> 20) & 0xf) +
                                  ((it.d.flags & kChainBel) ? kChainBelKey : 0)
                 : it.d.big >= 0 && it.d.bcls == kBigSlab ? slab_key(it.d.k, it.d.v1, it.d.v2, it.d.lanes, it.d.slab_r, it.d.slab_y2 ? 8 : it.d.n_in)
                 : it.d.big >= 0 ? stream_key(it.d.bcls, it.d.v1, it.d.v2, it.d.n_in)
                 : b.simple ? generic_variant(kMaxIn, 1, 1, max_in_bytes(b), no_o32)   // the widest input class runs any input count
                            : generic_variant(it.d.n_in, it.d.v1, it.d.v2, max_in_bytes(b), no_o32);
    });
    const double T2 = clk();
    for (const Item &it : items)
        if (!it.ok) {
            if (msg) *msg = it.msg;
            return false;
        }
    // order by (level, variant), ties by item index (stable), on compact keys
    std::vector<std::pair<uint64_t, int>> sk(items.size());
    for (size_t i = 0; i < items.size(); ++i)
        sk[i] = {((uint64_t)(uint32_t)items[i].level << 32) | ((uint64_t)items[i].b->lane << 28) | (uint32_t)items[i].key,
                 (int)i};
    std::sort(sk.begin(), sk.end());
    std::vector<int> ord(items.size());
    std::vector<int64_t> pool_at(items.size() + 1, 0);
    for (size_t i = 0; i < sk.size(); ++i) {
        ord[i] = sk[i].second;
        pool_at[i + 1] = pool_at[i] + (int64_t)items[ord[i]].pool.size();
    }
    s.pool.resize((size_t)pool_at.back());
    s.descs.resize(items.size());
    parallel_for((int64_t)ord.size(), [&](int64_t i) {
        const Item &it = items[ord[i]];
        std::copy(it.pool.begin(), it.pool.end(), s.pool.begin() + pool_at[i]);
        s.descs[i] = it.d;
        s.descs[i].dim_off = pool_at[i];
    });
    const bool dump = std::getenv("BNPP_DUMP_PLAN") != nullptr;
    for (size_t i = 0; i < ord.size();) {
        const Item &first = items[ord[i]];
        Schedule::Group g{first.level, first.key, (int)i, 0, 0, 0, first.b->lane};
        int64_t vb = 0;
        for (; i < ord.size() && items[ord[i]].level == g.level && items[ord[i]].key == g.variant &&
               items[ord[i]].b->lane == g.lane;
             ++i) {
            const Item &it = items[ord[i]];
            BucketDesc &d = s.descs[i];
            d.vblk_begin = vb;
            const int64_t per_vb = d.chain && chain_split_form((d.chain >> 16) & 0xf) ? kSplitRowsHost
                                   : d.big >= 0 && d.bcls == kBigSlab ? kBlock / (d.lanes == 2 ? 2 : 1) * std::max(1, d.slab_r)
                                                                          : kBlock;
            vb += (d.n_tiles + per_vb - 1) / per_vb;
            g.small_elems = std::max(g.small_elems, d.big >= 0 || d.chain ? d.small_elems : 0);
            if (dump && d.chain) {
                // chain run: per rest dim (card, in, out, G_j strides), then per slot (in, out)
                const int F = d.chain & 0xff;
                std::fprintf(stderr, "L%d chain F=%d form=%d dep=%d gmask=%x tiles=%lld base=%lld rest:", g.level, F,
                             (d.chain >> 16) & 0xf, (d.chain >> 20) & 0xf, (d.chain >> 8) & 0xff, (long long)d.n_tiles,
                             (long long)d.in_base[0]);
                const int64_t *pl = it.pool.data();
                for (int j = 0; j < d.n_dims; ++j, pl += 4 + F) {
                    std::fprintf(stderr, " [%u:%lld,%lld|", (unsigned)((uint64_t)pl[0] & 0xffffffffu), (long long)pl[2],
                                 (long long)pl[3]);
                    for (int q = 0; q < F; ++q) std::fprintf(stderr, "%s%lld", q ? "," : "", (long long)pl[4 + q]);
                    std::fprintf(stderr, "]");
                }
                std::fprintf(stderr, " slots:");
                for (int q = 0; q < F; ++q) std::fprintf(stderr, " %lld/%lld", (long long)pl[2 * q], (long long)pl[2 * q + 1]);
                if (d.flags & kChainBel) std::fprintf(stderr, " belief: %d x %d -> %d", d.in_table[d.n_in], d.out_table, d.aux_out);
                std::fprintf(stderr, "\n");
            } else if (dump && g.variant >= kXchgKeyBase) {
                std::fprintf(stderr, "L%d xchg kind=%d mode=%d blocks=%d tables:%d->%d entries=%lld\n", g.level,
                             (g.variant - kXchgKeyBase) / 16, (g.variant - kXchgKeyBase) % 16, d.k, d.in_table[0],
                             d.out_table, (long long)d.out_size);
            } else if (dump) {
                std::fprintf(stderr, "L%d n_in=%d k=%d tile=%dx%d big=%d bcls=%d tiles=%lld dims:", g.level, d.n_in, d.k,
                             d.v1, d.v2, d.big, d.big >= 0 ? d.bcls : 0, (long long)d.n_tiles);
                for (int j = 0; j < d.n_dims; ++j) {
                    const int64_t *row = it.pool.data() + (int64_t)j * (2 + d.n_in);
                    std::fprintf(stderr, " [%u:", (unsigned)((uint64_t)row[0] & 0xffffffffu));
                    for (int q = 0; q < d.n_in; ++q) std::fprintf(stderr, "%s%lld", q ? "," : "", (long long)row[2 + q]);
                    std::fprintf(stderr, "]");
                }
                std::fprintf(stderr, " es:");
                for (int q = 0; q < d.n_in; ++q) std::fprintf(stderr, "%s%lld", q ? "," : "", (long long)d.elim_stride[q]);
                std::fprintf(stderr, " tables:");
                for (int q = 0; q < d.n_in; ++q) std::fprintf(stderr, "%s%d", q ? "," : "", d.in_table[q]);
                std::fprintf(stderr, "->%d", d.out_table);
                if (d.outer_n > 0) std::fprintf(stderr, " outer=%d", d.outer_n);
                if (d.slab_r > 1) std::fprintf(stderr, " passes=%d", d.slab_r);
                std::fprintf(stderr, "\n");
            }
        }
        g.end = (int)i;
        g.vblocks = vb;
        s.groups.push_back(g);
    }
    s.n_levels = n_levels;
    // one dims-pool vector per bucket: freed on the worker threads
    parallel_for((int64_t)items.size(), [&](int64_t i) { std::vector<int64_t>().swap(items[i].pool); });
    if (timing)
        std::fprintf(stderr, "[bnpp] build_schedule: dedup %.1f ms, lifetimes %.1f ms, arena %.1f ms, descriptors %.1f ms, "
                     "grouping %.1f ms\n", Td - T0, Tl - Td, T1 - Tl, T2 - T1, clk() - T2);
    return true;
}

}  // namespace bnpp
