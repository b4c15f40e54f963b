// Device runtime: source upload, executable schedules, launches, result fetch.
#include <chrono>
#include "runtime.hpp"

#include <climits>
#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstring>

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

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

hipMemAllocationProp vmm_prop(int device) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    return prop;
}

}  // namespace

// ------------------------------------------------------------ VMM arena
bool vmm_reserve(int device, size_t bytes, VmmArena &a) {
    int ok = 0;
    if (hipDeviceGetAttribute(&ok, hipDeviceAttributeVirtualMemoryManagementSupported, device) != hipSuccess || !ok)
        return false;
    hipMemAllocationProp prop = vmm_prop(device);
    size_t g = 0;
    if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended) != hipSuccess || g == 0)
        return false;
    // 2-GiB chunks: a 258-GB arena is ~120 of them (0.2-0.3 ms each to map),
    // fine enough that a level waits only for the chunks it touches
    const size_t chunk = (((size_t)2 << 30) + g - 1) / g * g;
    const size_t n = (std::max<size_t>(bytes, 1) + chunk - 1) / chunk;
    void *base = nullptr;
    if (hipMemAddressReserve(&base, n * chunk, 0, nullptr, 0) != hipSuccess || !base) return false;
    a.base = base;
    a.bytes = n * chunk;
    a.chunk = chunk;
    a.device = device;
    a.handles.assign(n, hipMemGenericAllocationHandle_t{});
    a.created.assign(n, 0);
    return true;
}

void vmm_set_order(VmmArena &a, std::vector<int> order) {
    const int n = (int)a.handles.size();
    std::vector<char> seen(n, 0);
    for (int c : order) seen[c] = 1;
    for (int c = 0; c < n; ++c)
        if (!seen[c]) order.push_back(c);
    a.order = std::move(order);
}

hipError_t vmm_map_to(VmmArena &a, int prefix, double *ms) {
    if (a.mapped >= prefix) return hipSuccess;
    const auto t0 = std::chrono::steady_clock::now();
    const hipMemAllocationProp prop = vmm_prop(a.device);
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    hipError_t e = hipSuccess;
    for (; a.mapped < prefix && a.mapped < (int)a.order.size(); ++a.mapped) {
        const int c = a.order[a.mapped];
        void *p = static_cast<unsigned char *>(a.base) + (size_t)c * a.chunk;
        // the driver hands out HBM cleared: this is where a chunk waits for
        // the clearing of memory freed shortly before
        if ((e = hipMemCreate(&a.handles[c], a.chunk, &prop, 0)) != hipSuccess) break;
        a.created[c] = 1;
        if ((e = hipMemMap(p, a.chunk, 0, a.handles[c], 0)) != hipSuccess) break;
        a.created[c] = 2;
        if ((e = hipMemSetAccess(p, a.chunk, &acc, 1)) != hipSuccess) break;
    }
    if (ms) *ms += ms_since(t0);
    return e;
}

void vmm_release(VmmArena &a) {
    (void)hipSetDevice(a.device);
    for (size_t c = 0; c < a.handles.size(); ++c) {
        void *p = static_cast<unsigned char *>(a.base) + c * a.chunk;
        if (a.created[c] == 2) (void)hipMemUnmap(p, a.chunk);
        if (a.created[c] >= 1) (void)hipMemRelease(a.handles[c]);
        a.created[c] = 0;
    }
    if (a.base) (void)hipMemAddressFree(a.base, a.bytes);
    a.base = nullptr;
    a.bytes = 0;
}

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
            return call(0, x + R, x, 8);
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
            err = launch_xchg_unpack(f32, ex.d_meta, in_t, out_t, R, sc.table_size[in_t], stream);
            break;
        default:
            return fail(ctx, hipErrorInvalidValue, "unknown exchange step");
    }
    if (err != hipSuccess) return fail(ctx, err, "exchange step");
    return 0;
}

int launch(Context &ctx, Executable &ex, hipStream_t stream, const XchgHooks *hooks, VmmArena *vmm,
           const std::vector<int> *need, double *map_ms, double *first_ms) {
    const Schedule &sc = ex.sched;
    hipError_t err = hipMemcpyAsync(ex.d_meta, ex.d_meta0, sizeof(TableMeta) * (size_t)sc.n_tables,
                                    hipMemcpyDeviceToDevice, stream);
    if (err != hipSuccess) return fail(ctx, err, "hipMemcpyAsync(meta reset)");
    const bool lanes = sc.n_lanes > 1 && !ex.events.empty();
    hipStream_t ls[2] = {stream, lanes ? ctx.lane_stream : stream};
    if (lanes && ((err = hipEventRecord(ex.events[0], stream)) != hipSuccess ||
                  (err = hipStreamWaitEvent(ls[1], ex.events[0], 0)) != hipSuccess))
        return fail(ctx, err, "lane start");
    for (size_t gi = 0; gi < sc.groups.size(); ++gi) {
        const Schedule::Group &g = sc.groups[gi];
        hipStream_t st = ls[lanes ? g.lane & 1 : 0];
        // a VMM arena not fully mapped: the group's chunks are mapped before
        // it is enqueued (the device keeps running the levels before it)
        if (vmm && need && gi < need->size() &&
            (err = vmm_map_to(*vmm, (*need)[gi], gi == 0 ? first_ms : map_ms)) != hipSuccess)
            return fail(ctx, err, "arena mapping (hipMemCreate / hipMemMap)");
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
    if (ctx.arena_cache_vmm) ctx.arena_cache_vmm.reset();       // the last owner releases it
    else if (ctx.arena_cache) (void)hipFree(ctx.arena_cache);
    ctx.arena_cache = nullptr;
    ctx.arena_cache_bytes = 0;
}

namespace {

// VMM arenas from this size up (smaller ones map at once, nothing to hide);
// BNPP_NO_VMM=1 keeps one hipMalloc (A/B, and the tests' comparison)
bool use_vmm(int64_t need) {
    const char *e = std::getenv("BNPP_NO_VMM");
    return !(e && *e == '1') && need >= ((int64_t)8 << 30);
}

// Mapping order of a VMM arena's chunks and, per part and group, how many of
// them (a prefix of the order) must be mapped before the group is enqueued:
// chunks ordered by the first group (parts in order) that reads or writes a
// table in them.
void vmm_plan(const Program &pg, int64_t eb, std::vector<int> &order, std::vector<std::vector<int>> &need) {
    const VmmArena &a = *pg.vmm;
    const int n = (int)a.handles.size();
    const int64_t kNever = INT64_MAX;
    std::vector<int64_t> first(n, kNever);
    int64_t gidx = 0;
    for (const Executable &ex : pg.parts) {
        const Schedule &sc = ex.sched;
        auto touch = [&](int t) {
            if (t < sc.n_src || t >= sc.n_tables) return;
            const int64_t lo = sc.table_offset[t], hi = lo + std::max<int64_t>(sc.table_size[t], 1) * eb;
            for (int64_t c = lo / (int64_t)a.chunk; c <= (hi - 1) / (int64_t)a.chunk && c < n; ++c)
                first[c] = std::min(first[c], gidx);
        };
        for (const Schedule::Group &g : sc.groups) {
            for (int k = g.begin; k < g.end; ++k) {
                const BucketDesc &d = sc.descs[k];
                const int n_read = d.n_in + ((d.flags & kChainBel) ? 1 : 0);
                for (int i = 0; i < n_read && i < kMaxDescIn; ++i) touch(d.in_table[i]);
                touch(d.out_table);
                if (d.flags & kChainBel) touch(d.aux_out);
            }
            ++gidx;
        }
    }
    order.clear();
    for (int c = 0; c < n; ++c)
        if (first[c] != kNever) order.push_back(c);
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return first[x] < first[y]; });
    need.assign(pg.parts.size(), {});
    gidx = 0;
    size_t k = 0;
    for (size_t b = 0; b < pg.parts.size(); ++b) {
        for (size_t gi = 0; gi < pg.parts[b].sched.groups.size(); ++gi, ++gidx) {
            while (k < order.size() && first[order[k]] <= gidx) ++k;
            need[b].push_back((int)k);
        }
    }
}

}  // namespace

int make_program(Context &ctx, const DeviceSources &src, std::vector<Schedule> &&batches, Program &pg,
                 bool use_cache) {
    pg = Program{};
    pg.dtype = src.dtype;
    const int64_t eb = src.dtype == kF32 ? 4 : 8;
    for (const Schedule &s : batches) pg.arena_bytes = std::max(pg.arena_bytes, s.arena_bytes);
    hipError_t err = hipSetDevice(ctx.device);
    if (err != hipSuccess) return fail(ctx, err, "hipSetDevice");
    const int64_t need = std::max<int64_t>(pg.arena_bytes, 256);
    if (use_cache && ctx.arena_cache && ctx.arena_cache_bytes >= need && ctx.arena_cache_vmm &&
        ctx.arena_cache_vmm->mapped < (int)ctx.arena_cache_vmm->handles.size())
        drop_arena_cache(ctx);                           // an earlier call failed to map it all
    if (use_cache && ctx.arena_cache && ctx.arena_cache_bytes >= need) {
        pg.arena = ctx.arena_cache;
        pg.vmm = ctx.arena_cache_vmm;
        pg.arena_cached = true;
        pg.arena_reused = true;
    } else {
        if (use_cache) drop_arena_cache(ctx);            // too small: replace it
        // the plan's own size (not the budget).  A hipMalloc here is where a
        // cold call waits for the driver to clear HBM another process (or
        // this one) freed shortly before -- ~36 GB/s of backlog, one wait
        // whatever the size asked (tools/map_probe.hip,
        // profiles/r04_map_probe.log) -- so it is timed on its own.  Large
        // arenas are reserved instead and mapped by a helper while the run
        // goes (VmmArena); the reservation is what is timed then
        const auto ta = std::chrono::steady_clock::now();
        std::shared_ptr<VmmArena> v;
        if (use_vmm(need)) {
            // released by its last owner (the program, or the context's cache)
            v = std::shared_ptr<VmmArena>(new VmmArena, [](VmmArena *a) {
                if (a->base) {
                    (void)hipSetDevice(a->device);
                    (void)hipDeviceSynchronize();          // nothing may still run in it
                }
                vmm_release(*a);
                delete a;
            });
            if (!vmm_reserve(ctx.device, (size_t)need, *v)) v.reset();
        }
        if (v) {
            pg.arena = v->base;
            pg.vmm = v;
        } else if ((err = hipMalloc(&pg.arena, (size_t)need)) != hipSuccess) {
            return fail(ctx, err, "hipMalloc(arena)");
        }
        pg.arena_alloc_ms = ms_since(ta);
        if (use_cache) {
            ctx.arena_cache = pg.arena;
            ctx.arena_cache_bytes = need;
            ctx.arena_cache_vmm = pg.vmm;
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
    // a new VMM arena: chunks mapped by the launch as levels first need them
    if (pg.vmm && !pg.arena_reused) {
        std::vector<int> order;
        vmm_plan(pg, eb, order, pg.vmm_need);
        vmm_set_order(*pg.vmm, std::move(order));
        pg.vmm_pending = true;
    }
    return 0;
}

int launch_program(Context &ctx, Program &pg, hipStream_t stream) {
    const int64_t eb = pg.dtype == kF32 ? 4 : 8;
    (void)eb;
    pg.vmm_map_ms = pg.vmm_first_ms = 0;
    VmmArena *vmm = pg.vmm_pending ? pg.vmm.get() : nullptr;
    for (size_t b = 0; b < pg.parts.size(); ++b) {
        Executable &ex = pg.parts[b];
        int rc = launch(ctx, ex, stream, &pg.hooks, vmm, vmm ? &pg.vmm_need[b] : nullptr, &pg.vmm_map_ms,
                        b == 0 ? &pg.vmm_first_ms : &pg.vmm_map_ms);
        if (rc) return rc;
        if (ex.n_copies > 0) {
            hipError_t err = launch_copies(ex.d_copies, ex.n_copies, ex.copy_max_bytes, stream);
            if (err != hipSuccess) return fail(ctx, err, "launch_copies");
        }
    }
    if (vmm) {
        // the rest of the range (chunks no level touched): later launches of
        // this program, and later programs in the cached arena, map nothing
        hipError_t err = vmm_map_to(*vmm, (int)vmm->handles.size(), &pg.vmm_map_ms);
        if (err != hipSuccess) return fail(ctx, err, "arena mapping (hipMemCreate / hipMemMap)");
        pg.vmm_map_ms += pg.vmm_first_ms;
        pg.vmm_pending = false;
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
    if (pg.arena && !pg.arena_cached && !pg.vmm) (void)hipFree(pg.arena);
    pg.vmm.reset();                                  // a VMM arena: released by its last owner
    put_buffer(ctx, pg.results, pg.results_cap);
    pg = Program{};
}

}  // namespace bnpp
