// Device runtime: source upload, executable schedules, launches, result fetch.
#include <chrono>
#include "runtime.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>

#include "lane_order.hpp"

namespace bnpp {
namespace {

int fail(Context &ctx, hipError_t e, const char *what) {
    ctx.last_error = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? -3 : -4;
}

template <typename T>
uint64_t bits_of(T x) {
    uint64_t b = 0;
    std::memcpy(&b, &x, sizeof(T));
    return b;
}

}  // namespace

hipError_t get_buffer(Context &ctx, size_t bytes, void **p, size_t *cap) {
    bytes = bytes ? bytes : 256;
    {
        std::lock_guard<std::mutex> g(ctx.buf_mu);
        size_t best = ctx.buf_free.size();
        for (size_t i = 0; i < ctx.buf_free.size(); ++i) {
            const size_t c = ctx.buf_free[i].second;
            if (c >= bytes && c <= 4 * bytes + 65536 && (best == ctx.buf_free.size() || c < ctx.buf_free[best].second))
                best = i;
        }
        if (best < ctx.buf_free.size()) {
            *p = ctx.buf_free[best].first;
            *cap = ctx.buf_free[best].second;
            ctx.buf_free_bytes -= *cap;
            ctx.buf_free.erase(ctx.buf_free.begin() + best);
            return hipSuccess;
        }
    }
    const size_t c = (bytes + 65535) & ~(size_t)65535;       // 64-KiB granules: fewer distinct sizes
    hipError_t e = hipMalloc(p, c);
    *cap = e == hipSuccess ? c : 0;
    return e;
}

void put_buffer(Context &ctx, void *p, size_t cap) {
    if (!p) return;
    constexpr size_t kMaxCached = (size_t)1 << 30, kMaxCount = 64;
    {
        std::lock_guard<std::mutex> g(ctx.buf_mu);
        if (cap > 0 && ctx.buf_free_bytes + cap <= kMaxCached && ctx.buf_free.size() < kMaxCount) {
            ctx.buf_free.push_back({p, cap});
            ctx.buf_free_bytes += cap;
            return;
        }
    }
    (void)hipFree(p);
}

void drop_buffer_cache(Context &ctx) {
    std::lock_guard<std::mutex> g(ctx.buf_mu);
    for (auto &b : ctx.buf_free) (void)hipFree(b.first);
    ctx.buf_free.clear();
    ctx.buf_free_bytes = 0;
}

int upload_sources(Context &ctx, const std::vector<std::vector<double>> &values, DType dt, DeviceSources &out) {
    const size_t eb = dt == kF32 ? 4 : 8;
    out = DeviceSources{};
    out.dtype = dt;
    std::vector<size_t> off(values.size());
    size_t total = 0;
    for (size_t f = 0; f < values.size(); ++f) {
        off[f] = total;
        total += ((values[f].size() * eb + 255) / 256) * 256;
    }
    std::vector<unsigned char> host(total ? total : 256, 0);
    out.meta.resize(values.size());
    out.size.resize(values.size());
    for (size_t f = 0; f < values.size(); ++f) {
        double mx = 0;
        for (double v : values[f]) mx = v > mx ? v : mx;
        int e = 0;
        if (mx > 0) std::frexp(mx, &e);            // mx = m * 2^e, m in [0.5, 1)
        double smax = 0;
        float fmax = 0;
        for (size_t j = 0; j < values[f].size(); ++j) {
            double s = std::ldexp(values[f][j], -e);   // exact power-of-two rescale
            if (dt == kF32) {
                float x = (float)s;
                std::memcpy(host.data() + off[f] + j * 4, &x, 4);
                fmax = x > fmax ? x : fmax;
            } else {
                std::memcpy(host.data() + off[f] + j * 8, &s, 8);
                smax = s > smax ? s : smax;
            }
        }
        out.meta[f].maxbits = dt == kF32 ? bits_of(fmax) : bits_of(smax);
        out.meta[f].exp2 = e;
        out.meta[f].size = (int64_t)values[f].size();
        out.size[f] = (int64_t)values[f].size();
    }
    hipError_t err = hipSetDevice(ctx.device);
    if (err != hipSuccess) return fail(ctx, err, "hipSetDevice");
    err = get_buffer(ctx, host.size(), &out.buf, &out.buf_cap);
    if (err != hipSuccess) return fail(ctx, err, "hipMalloc(sources)");
    err = hipMemcpy(out.buf, host.data(), host.size(), hipMemcpyHostToDevice);
    if (err != hipSuccess) return fail(ctx, err, "hipMemcpy(sources)");
    for (size_t f = 0; f < values.size(); ++f) out.meta[f].ptr = static_cast<unsigned char *>(out.buf) + off[f];
    return 0;
}

void free_sources(Context &ctx, DeviceSources &s) {
    put_buffer(ctx, s.buf, s.buf_cap);
    s = DeviceSources{};
}

int make_executable(Context &ctx, const DeviceSources &src, Schedule &&s, Executable &ex, void *shared_arena) {
    ex = Executable{};
    ex.dtype = src.dtype;
    ex.sched = std::move(s);
    Schedule &sc = ex.sched;
    hipError_t err = hipSetDevice(ctx.device);
    if (err != hipSuccess) return fail(ctx, err, "hipSetDevice");
    if (sc.n_src != (int)src.meta.size()) {
        ctx.last_error = "schedule/source count mismatch";
        return -1;
    }
    if (shared_arena) {
        ex.arena = shared_arena;
        ex.own_arena = false;
    } else {
        err = hipMalloc(&ex.arena, sc.arena_bytes > 0 ? (size_t)sc.arena_bytes : 256);
        if (err != hipSuccess) return fail(ctx, err, "hipMalloc(arena)");
    }
    ex.h_meta.resize(sc.n_tables);
    for (int t = 0; t < sc.n_tables; ++t) {
        if (t < sc.n_src) {
            ex.h_meta[t] = src.meta[t];
        } else {
            TableMeta m{};
            m.ptr = static_cast<unsigned char *>(ex.arena) + sc.table_offset[t];
            m.maxbits = 0;
            m.exp2 = 0;
            m.size = sc.table_size[t];
            ex.h_meta[t] = m;
        }
    }
    const size_t mb = sizeof(TableMeta) * (size_t)sc.n_tables;
    void *pm = nullptr, *pm0 = nullptr, *pd = nullptr, *pp = nullptr;
    if ((err = get_buffer(ctx, mb + 16, &pm, &ex.cap_meta)) != hipSuccess) return fail(ctx, err, "hipMalloc(meta)");
    ex.d_meta = static_cast<TableMeta *>(pm);
    if ((err = get_buffer(ctx, mb + 16, &pm0, &ex.cap_meta0)) != hipSuccess) return fail(ctx, err, "hipMalloc(meta0)");
    ex.d_meta0 = static_cast<TableMeta *>(pm0);
    if ((err = get_buffer(ctx, sizeof(BucketDesc) * sc.descs.size() + 16, &pd, &ex.cap_desc)) != hipSuccess)
        return fail(ctx, err, "hipMalloc(desc)");
    ex.d_desc = static_cast<BucketDesc *>(pd);
    if ((err = get_buffer(ctx, sizeof(int64_t) * sc.pool.size() + 16, &pp, &ex.cap_pool)) != hipSuccess)
        return fail(ctx, err, "hipMalloc(pool)");
    ex.d_pool = static_cast<int64_t *>(pp);
    if (mb && (err = hipMemcpy(ex.d_meta0, ex.h_meta.data(), mb, hipMemcpyHostToDevice)) != hipSuccess)
        return fail(ctx, err, "hipMemcpy(meta)");
    if (!sc.descs.empty() && (err = hipMemcpy(ex.d_desc, sc.descs.data(), sizeof(BucketDesc) * sc.descs.size(),
                                              hipMemcpyHostToDevice)) != hipSuccess)
        return fail(ctx, err, "hipMemcpy(desc)");
    if (!sc.pool.empty() && (err = hipMemcpy(ex.d_pool, sc.pool.data(), sizeof(int64_t) * sc.pool.size(),
                                             hipMemcpyHostToDevice)) != hipSuccess)
        return fail(ctx, err, "hipMemcpy(pool)");
    if (sc.n_lanes > 1) {
        if (sc.n_lanes > 2) return fail(ctx, hipErrorInvalidValue, "more than two lanes");
        if (!ctx.lane_stream && (err = hipStreamCreateWithFlags(&ctx.lane_stream, hipStreamNonBlocking)) != hipSuccess)
            return fail(ctx, err, "hipStreamCreate(lane)");
        // producer group of every table; a group consuming a table made on the
        // other lane waits for the producer's event
        std::vector<int> prod(sc.n_tables, -1);
        const int ng = (int)sc.groups.size();
        ex.g_record.assign(ng, -1);
        ex.g_wait.assign(ng, {});
        int n_ev = 2;
        for (int gi = 0; gi < ng; ++gi) {
            const Schedule::Group &g = sc.groups[gi];
            for (int k = g.begin; k < g.end; ++k) {
                const BucketDesc &d = sc.descs[k];
                const int n_read = d.n_in + ((d.flags & kChainBel) ? 1 : 0);   // + a fused belief's forward message
                for (int i = 0; i < n_read && i < kMaxDescIn; ++i) {
                    const int t = d.in_table[i], pg = t >= 0 ? prod[t] : -1;
                    if (pg < 0 || sc.groups[pg].lane == g.lane) continue;
                    if (ex.g_record[pg] < 0) ex.g_record[pg] = n_ev++;
                    std::vector<int> &w = ex.g_wait[gi];
                    if (std::find(w.begin(), w.end(), ex.g_record[pg]) == w.end()) w.push_back(ex.g_record[pg]);
                }
            }
            for (int k = g.begin; k < g.end; ++k) {
                prod[sc.descs[k].out_table] = gi;
                if (sc.descs[k].flags & kChainBel) prod[sc.descs[k].aux_out] = gi;
            }
        }
        // the lanes' windows alternate (lane_order.hpp)
        std::vector<int> lane(ng);
        std::vector<char> is_x(ng);
        std::vector<int64_t> work(ng);
        for (int gi = 0; gi < ng; ++gi) {
            lane[gi] = sc.groups[gi].lane;
            is_x[gi] = sc.groups[gi].variant >= kXchgKeyBase;
            work[gi] = sc.groups[gi].vblocks;
        }
        const char *alt = tuning_knob("BNPP_LANE_ALT");
        ex.g_order = lane_order(lane, is_x, work, ex.g_record, ex.g_wait, n_ev, alt ? std::atof(alt) : kLaneAltDefault);
        ex.events.assign(n_ev, nullptr);
        for (hipEvent_t &e : ex.events)
            if ((err = hipEventCreateWithFlags(&e, hipEventDisableTiming)) != hipSuccess)
                return fail(ctx, err, "hipEventCreate");
    }
    return 0;
}

// one exchange step of a sliced run (plan.hpp BucketSpec::xchg, xchg.hip)
static int run_xchg(Context &ctx, Executable &ex, const Schedule::Group &g, hipStream_t stream, const XchgHooks *hooks) {
    const Schedule &sc = ex.sched;
    const BucketDesc &d = sc.descs[g.begin];
    const int kind = (g.variant - kXchgKeyBase) / 16, mode = (g.variant - kXchgKeyBase) % 16, R = d.k;
    const bool f32 = ex.dtype == kF32;
    const int64_t eb = f32 ? 4 : 8;
    const int in_t = d.in_table[0], out_t = d.out_table;
    auto call = [&](int op, const void *send, void *recv, int64_t bytes) {
        if (!hooks || !hooks->fn) return fail(ctx, hipErrorInvalidValue, "sliced run without a collective");
        if (hooks->fn(hooks->user, op, send, recv, bytes, stream) != 0)
            return fail(ctx, hipErrorUnknown, "the exchange collective failed");
        return 0;
    };
    hipError_t err = hipSuccess;
    switch (kind) {
        case kXchgSync: {
            err = launch_xchg_sync(f32, ex.d_meta, in_t, out_t, R, stream);
            if (err != hipSuccess) break;
            int64_t *x = static_cast<int64_t *>(ex.h_meta[out_t].ptr);
            return call(0, x + 2 * R, x, 16);                // (E_r, exp2_r) of every rank
        }
        case kXchgPack:
            err = launch_xchg_pack(f32, ex.d_meta, in_t, d.in_table[1], out_t, R, mode, sc.table_size[out_t], stream);
            break;
        case kXchgComm: {
            const int64_t n = sc.table_size[in_t];
            int rc = mode == 0 ? call(1, ex.h_meta[in_t].ptr, ex.h_meta[out_t].ptr, n / R * eb)
                               : call(0, ex.h_meta[in_t].ptr, ex.h_meta[out_t].ptr, n * eb);
            if (rc) return rc;
            err = launch_xchg_meta(ex.d_meta, in_t, out_t, stream);
            break;
        }
        case kXchgUnpack:
            // mode 2: the pack was skipped, in[1] holds the gathered exponents
            err = launch_xchg_unpack(f32, ex.d_meta, in_t, mode == 2 ? d.in_table[1] : -1, out_t, R,
                                     sc.table_size[in_t], stream);
            break;
        default:
            return fail(ctx, hipErrorInvalidValue, "unknown exchange step");
    }
    if (err != hipSuccess) return fail(ctx, err, "exchange step");
    return 0;
}

int launch(Context &ctx, Executable &ex, hipStream_t stream, const XchgHooks *hooks) {
    const Schedule &sc = ex.sched;
    hipError_t err = hipMemcpyAsync(ex.d_meta, ex.d_meta0, sizeof(TableMeta) * (size_t)sc.n_tables,
                                    hipMemcpyDeviceToDevice, stream);
    if (err != hipSuccess) return fail(ctx, err, "hipMemcpyAsync(meta reset)");
    const bool lanes = sc.n_lanes > 1 && !ex.events.empty();
    hipStream_t ls[2] = {stream, lanes ? ctx.lane_stream : stream};
    if (lanes && ((err = hipEventRecord(ex.events[0], stream)) != hipSuccess ||
                  (err = hipStreamWaitEvent(ls[1], ex.events[0], 0)) != hipSuccess))
        return fail(ctx, err, "lane start");
    const bool reorder = lanes && ex.g_order.size() == sc.groups.size();
    for (size_t oi = 0; oi < sc.groups.size(); ++oi) {
        const size_t gi = reorder ? (size_t)ex.g_order[oi] : oi;
        const Schedule::Group &g = sc.groups[gi];
        hipStream_t st = ls[lanes ? g.lane & 1 : 0];
        if (lanes)
            for (int e : ex.g_wait[gi])
                if ((err = hipStreamWaitEvent(st, ex.events[e], 0)) != hipSuccess) return fail(ctx, err, "lane wait");
        if (g.variant >= kXchgKeyBase) {
            int rc = run_xchg(ctx, ex, g, st, hooks);
            if (rc) return rc;
        } else {
            err = launch_level(ex.dtype == kF32, g.variant, ex.d_desc + g.begin, g.end - g.begin, ex.d_pool, ex.d_meta,
                               g.vblocks, g.small_elems, ctx.max_grid, st);
            if (err != hipSuccess) return fail(ctx, err, "launch_level");
        }
        if (lanes && ex.g_record[gi] >= 0 && (err = hipEventRecord(ex.events[ex.g_record[gi]], st)) != hipSuccess)
            return fail(ctx, err, "lane record");
    }
    if (lanes && ((err = hipEventRecord(ex.events[1], ls[1])) != hipSuccess ||
                  (err = hipStreamWaitEvent(stream, ex.events[1], 0)) != hipSuccess))
        return fail(ctx, err, "lane join");
    return 0;
}

int fetch_results(Context &ctx, Executable &ex, hipStream_t stream, std::vector<std::vector<double>> &vals,
                  std::vector<int64_t> &exp2) {
    hipError_t err = hipStreamSynchronize(stream);
    if (err != hipSuccess) return fail(ctx, err, "hipStreamSynchronize");
    const Schedule &sc = ex.sched;
    const size_t np = sc.plan_result_table.size();
    vals.assign(np, {});
    exp2.assign(np, 0);
    const size_t eb = ex.dtype == kF32 ? 4 : 8;
    for (size_t p = 0; p < np; ++p) {
        int t = sc.plan_result_table[p];
        if (t < 0) {                         // no factors at all: Factor(1.0)
            vals[p] = {1.0};
            continue;
        }
        TableMeta m;
        err = hipMemcpy(&m, ex.d_meta + t, sizeof(TableMeta), hipMemcpyDeviceToHost);
        if (err != hipSuccess) return fail(ctx, err, "hipMemcpy(meta)");
        exp2[p] = m.exp2;
        std::vector<unsigned char> raw((size_t)sc.table_size[t] * eb);
        err = hipMemcpy(raw.data(), m.ptr, raw.size(), hipMemcpyDeviceToHost);
        if (err != hipSuccess) return fail(ctx, err, "hipMemcpy(result)");
        vals[p].resize((size_t)sc.table_size[t]);
        for (size_t j = 0; j < vals[p].size(); ++j) {
            if (eb == 4) {
                float x;
                std::memcpy(&x, raw.data() + j * 4, 4);
                vals[p][j] = x;
            } else {
                std::memcpy(&vals[p][j], raw.data() + j * 8, 8);
            }
        }
    }
    return 0;
}

void free_executable(Context &ctx, Executable &ex) {
    for (hipEvent_t e : ex.events)
        if (e) (void)hipEventDestroy(e);
    if (ex.arena && ex.own_arena) (void)hipFree(ex.arena);
    put_buffer(ctx, ex.d_meta, ex.cap_meta);
    put_buffer(ctx, ex.d_meta0, ex.cap_meta0);
    put_buffer(ctx, ex.d_desc, ex.cap_desc);
    put_buffer(ctx, ex.d_pool, ex.cap_pool);
    put_buffer(ctx, ex.d_copies, ex.cap_copies);
    ex = Executable{};
}

void drop_arena_cache(Context &ctx) {
    if (ctx.arena_cache) (void)hipFree(static_cast<char *>(ctx.arena_cache) - ctx.arena_cache_pad);
    ctx.arena_cache = nullptr;
    ctx.arena_cache_bytes = 0;
    ctx.arena_cache_pad = 0;
}

// alignment of the arena's base: hipMalloc returns 32-MiB-aligned addresses
// for arenas this size; BNPP_ARENA_ALIGN_MB (tuning builds) asks for more
static int64_t arena_align() {
    int64_t a = 0;
    if (const char *e = tuning_knob("BNPP_ARENA_ALIGN_MB")) a = std::atoll(e) << 20;
    return a > 0 ? a : 0;
}

int make_program(Context &ctx, const DeviceSources &src, std::vector<Schedule> &&batches, Program &pg,
                 bool use_cache) {
    pg = Program{};
    pg.dtype = src.dtype;
    const int64_t eb = src.dtype == kF32 ? 4 : 8;
    for (const Schedule &s : batches) pg.arena_bytes = std::max(pg.arena_bytes, s.arena_bytes);
    hipError_t err = hipSetDevice(ctx.device);
    if (err != hipSuccess) return fail(ctx, err, "hipSetDevice");
    const int64_t need = std::max<int64_t>(pg.arena_bytes, 256);
    if (use_cache && ctx.arena_cache && ctx.arena_cache_bytes >= need) {
        pg.arena = ctx.arena_cache;
        pg.arena_cached = true;
        pg.arena_reused = true;
    } else {
        if (use_cache) drop_arena_cache(ctx);            // too small: replace it
        // the plan's own size (not the budget).  This hipMalloc is where a
        // cold call waits for the driver to clear HBM another process (or
        // this one) freed shortly before -- ~36 GB/s of backlog, one wait
        // whatever the size asked (tools/map_probe.hip,
        // profiles/r04_map_probe.log) -- so it is timed on its own
        const auto ta = std::chrono::steady_clock::now();
        const int64_t al = arena_align();
        void *raw = nullptr;
        if ((err = hipMalloc(&raw, (size_t)(need + al))) != hipSuccess) return fail(ctx, err, "hipMalloc(arena)");
        pg.arena_pad = al ? (int64_t)((al - (uintptr_t)raw % (uint64_t)al) % (uint64_t)al) : 0;
        pg.arena = static_cast<char *>(raw) + pg.arena_pad;
        pg.arena_alloc_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
        if (use_cache) {
            ctx.arena_cache = pg.arena;
            ctx.arena_cache_bytes = need;
            ctx.arena_cache_pad = pg.arena_pad;
            pg.arena_cached = true;
        }
    }
    for (const Schedule &s : batches) {
        std::vector<int64_t> off, sz;
        for (int t : s.plan_result_table) {
            if (t < 0) {
                off.push_back(-1);
                sz.push_back(1);
            } else {
                off.push_back(pg.results_bytes);
                sz.push_back(s.table_size[t]);
                pg.results_bytes += ((s.table_size[t] * eb + 255) / 256) * 256;
            }
        }
        pg.res_off.push_back(off);
        pg.res_size.push_back(sz);
    }
    if ((err = get_buffer(ctx, pg.results_bytes > 0 ? (size_t)pg.results_bytes : 256, &pg.results, &pg.results_cap)) !=
        hipSuccess)
        return fail(ctx, err, "hipMalloc(results)");
    pg.parts.resize(batches.size());
    for (size_t b = 0; b < batches.size(); ++b) {
        int rc = make_executable(ctx, src, std::move(batches[b]), pg.parts[b], pg.arena);
        if (rc) return rc;
        // the part's result tables, copied into `results` by one launch after it runs
        Executable &ex = pg.parts[b];
        std::vector<CopyItem> cp;
        for (size_t p = 0; p < ex.sched.plan_result_table.size(); ++p) {
            const int t = ex.sched.plan_result_table[p];
            if (t < 0) continue;
            cp.push_back({ex.h_meta[t].ptr, static_cast<unsigned char *>(pg.results) + pg.res_off[b][p],
                          ex.sched.table_size[t] * eb});
        }
        ex.n_copies = (int)cp.size();
        for (const CopyItem &c : cp) ex.copy_max_bytes = std::max(ex.copy_max_bytes, c.bytes);
        if (!cp.empty()) {
            void *pc = nullptr;
            if ((err = get_buffer(ctx, sizeof(CopyItem) * cp.size(), &pc, &ex.cap_copies)) != hipSuccess)
                return fail(ctx, err, "hipMalloc(copies)");
            ex.d_copies = static_cast<CopyItem *>(pc);
            if ((err = hipMemcpy(ex.d_copies, cp.data(), sizeof(CopyItem) * cp.size(), hipMemcpyHostToDevice)) !=
                hipSuccess)
                return fail(ctx, err, "hipMemcpy(copies)");
        }
    }
    return 0;
}

int launch_program(Context &ctx, Program &pg, hipStream_t stream) {
    const int64_t eb = pg.dtype == kF32 ? 4 : 8;
    (void)eb;
    for (size_t b = 0; b < pg.parts.size(); ++b) {
        Executable &ex = pg.parts[b];
        int rc = launch(ctx, ex, stream, &pg.hooks);
        if (rc) return rc;
        if (ex.n_copies > 0) {
            hipError_t err = launch_copies(ex.d_copies, ex.n_copies, ex.copy_max_bytes, stream);
            if (err != hipSuccess) return fail(ctx, err, "launch_copies");
        }
    }
    return 0;
}

int fetch_program(Context &ctx, Program &pg, hipStream_t stream, std::vector<std::vector<double>> &vals,
                  std::vector<int64_t> &exp2) {
    hipError_t err = hipStreamSynchronize(stream);
    if (err != hipSuccess) return fail(ctx, err, "hipStreamSynchronize");
    const int64_t eb = pg.dtype == kF32 ? 4 : 8;
    std::vector<unsigned char> raw((size_t)std::max<int64_t>(pg.results_bytes, 1));
    if (pg.results_bytes > 0 &&
        (err = hipMemcpy(raw.data(), pg.results, (size_t)pg.results_bytes, hipMemcpyDeviceToHost)) != hipSuccess)
        return fail(ctx, err, "hipMemcpy(results)");
    vals.clear();
    exp2.clear();
    for (size_t b = 0; b < pg.parts.size(); ++b) {
        Executable &ex = pg.parts[b];
        std::vector<TableMeta> meta(ex.sched.n_tables);
        if (!meta.empty() &&
            (err = hipMemcpy(meta.data(), ex.d_meta, sizeof(TableMeta) * meta.size(), hipMemcpyDeviceToHost)) != hipSuccess)
            return fail(ctx, err, "hipMemcpy(meta)");
        for (size_t p = 0; p < ex.sched.plan_result_table.size(); ++p) {
            int t = ex.sched.plan_result_table[p];
            if (t < 0) {
                vals.push_back({1.0});
                exp2.push_back(0);
                continue;
            }
            std::vector<double> v((size_t)pg.res_size[b][p]);
            const unsigned char *src = raw.data() + pg.res_off[b][p];
            for (size_t j = 0; j < v.size(); ++j) {
                if (eb == 4) {
                    float x;
                    std::memcpy(&x, src + j * 4, 4);
                    v[j] = x;
                } else {
                    std::memcpy(&v[j], src + j * 8, 8);
                }
            }
            vals.push_back(std::move(v));
            exp2.push_back(meta[t].exp2);
        }
    }
    return 0;
}

void free_program(Context &ctx, Program &pg) {
    for (Executable &ex : pg.parts) free_executable(ctx, ex);
    if (pg.arena && !pg.arena_cached) (void)hipFree(static_cast<char *>(pg.arena) - pg.arena_pad);
    put_buffer(ctx, pg.results, pg.results_cap);
    pg = Program{};
}

}  // namespace bnpp
