// Device runtime: source upload, executable schedules, launches, result fetch.
#include "runtime.hpp"

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

}  // namespace

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
    err = hipMalloc(&out.buf, host.size());
    if (err != hipSuccess) return fail(ctx, err, "hipMalloc(sources)");
    err = hipMemcpy(out.buf, host.data(), host.size(), hipMemcpyHostToDevice);
    if (err != hipSuccess) return fail(ctx, err, "hipMemcpy(sources)");
    for (size_t f = 0; f < values.size(); ++f) out.meta[f].ptr = static_cast<unsigned char *>(out.buf) + off[f];
    return 0;
}

void free_sources(DeviceSources &s) {
    if (s.buf) (void)hipFree(s.buf);
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
    if ((err = hipMalloc(&ex.d_meta, mb + 16)) != hipSuccess) return fail(ctx, err, "hipMalloc(meta)");
    if ((err = hipMalloc(&ex.d_meta0, mb + 16)) != hipSuccess) return fail(ctx, err, "hipMalloc(meta0)");
    if ((err = hipMalloc(&ex.d_desc, sizeof(BucketDesc) * sc.descs.size() + 16)) != hipSuccess)
        return fail(ctx, err, "hipMalloc(desc)");
    if ((err = hipMalloc(&ex.d_pool, sizeof(int64_t) * sc.pool.size() + 16)) != hipSuccess)
        return fail(ctx, err, "hipMalloc(pool)");
    if (mb && (err = hipMemcpy(ex.d_meta0, ex.h_meta.data(), mb, hipMemcpyHostToDevice)) != hipSuccess)
        return fail(ctx, err, "hipMemcpy(meta)");
    if (!sc.descs.empty() && (err = hipMemcpy(ex.d_desc, sc.descs.data(), sizeof(BucketDesc) * sc.descs.size(),
                                              hipMemcpyHostToDevice)) != hipSuccess)
        return fail(ctx, err, "hipMemcpy(desc)");
    if (!sc.pool.empty() && (err = hipMemcpy(ex.d_pool, sc.pool.data(), sizeof(int64_t) * sc.pool.size(),
                                             hipMemcpyHostToDevice)) != hipSuccess)
        return fail(ctx, err, "hipMemcpy(pool)");
    return 0;
}

int launch(Context &ctx, Executable &ex, hipStream_t stream) {
    const Schedule &sc = ex.sched;
    hipError_t err = hipMemcpyAsync(ex.d_meta, ex.d_meta0, sizeof(TableMeta) * (size_t)sc.n_tables,
                                    hipMemcpyDeviceToDevice, stream);
    if (err != hipSuccess) return fail(ctx, err, "hipMemcpyAsync(meta reset)");
    for (const Schedule::Group &g : sc.groups) {
        err = launch_level(ex.dtype == kF32, g.variant, ex.d_desc + g.begin, g.end - g.begin, ex.d_pool, ex.d_meta,
                           g.vblocks, g.small_elems, ctx.max_grid, stream);
        if (err != hipSuccess) return fail(ctx, err, "launch_level");
    }
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

void free_executable(Executable &ex) {
    if (ex.arena && ex.own_arena) (void)hipFree(ex.arena);
    if (ex.d_meta) (void)hipFree(ex.d_meta);
    if (ex.d_meta0) (void)hipFree(ex.d_meta0);
    if (ex.d_desc) (void)hipFree(ex.d_desc);
    if (ex.d_pool) (void)hipFree(ex.d_pool);
    ex = Executable{};
}

void drop_arena_cache(Context &ctx) {
    if (ctx.arena_cache) (void)hipFree(ctx.arena_cache);
    ctx.arena_cache = nullptr;
    ctx.arena_cache_bytes = 0;
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
    } else {
        if (use_cache) drop_arena_cache(ctx);            // too small: replace it
        if ((err = hipMalloc(&pg.arena, (size_t)need)) != hipSuccess) return fail(ctx, err, "hipMalloc(arena)");
        if (use_cache) {
            ctx.arena_cache = pg.arena;
            ctx.arena_cache_bytes = need;
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
    if ((err = hipMalloc(&pg.results, pg.results_bytes > 0 ? (size_t)pg.results_bytes : 256)) != hipSuccess)
        return fail(ctx, err, "hipMalloc(results)");
    pg.parts.resize(batches.size());
    for (size_t b = 0; b < batches.size(); ++b) {
        int rc = make_executable(ctx, src, std::move(batches[b]), pg.parts[b], pg.arena);
        if (rc) return rc;
    }
    return 0;
}

int launch_program(Context &ctx, Program &pg, hipStream_t stream) {
    const int64_t eb = pg.dtype == kF32 ? 4 : 8;
    for (size_t b = 0; b < pg.parts.size(); ++b) {
        Executable &ex = pg.parts[b];
        int rc = launch(ctx, ex, stream);
        if (rc) return rc;
        for (size_t p = 0; p < ex.sched.plan_result_table.size(); ++p) {
            int t = ex.sched.plan_result_table[p];
            if (t < 0) continue;
            hipError_t err = hipMemcpyAsync(static_cast<unsigned char *>(pg.results) + pg.res_off[b][p],
                                            ex.h_meta[t].ptr, (size_t)(ex.sched.table_size[t] * eb),
                                            hipMemcpyDeviceToDevice, stream);
            if (err != hipSuccess) return fail(ctx, err, "hipMemcpyAsync(result)");
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

void free_program(Program &pg) {
    for (Executable &ex : pg.parts) free_executable(ex);
    if (pg.arena && !pg.arena_cached) (void)hipFree(pg.arena);
    if (pg.results) (void)hipFree(pg.results);
    pg = Program{};
}

}  // namespace bnpp
