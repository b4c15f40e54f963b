// Device runtime: context, source upload, schedule execution (HIP).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "bnpp_device.h"
#include "model_io.hpp"
#include "plan.hpp"

namespace bnpp {

hipError_t launch_level(int is_f32, int variant, const BucketDesc *descs, int n_desc, const int64_t *pool,
                        TableMeta *meta, int64_t total_vblocks, int small_elems, int max_grid, hipStream_t stream);

// single bucket with the descriptor passed by value (no device-side metadata,
// no rescaling): the exact Factor::product / sum_out / conditioning semantics.
constexpr int kMaxPool = 320;   // dims-pool words that fit the kernel-argument segment
struct SingleArgs {
    // slab form: the big input's first entry and summed-variable stride,
    // resolved on the host so the kernel's first loads wait on one kernarg read
    const void *big_ptr;
    int64_t big_es;
    BucketDesc d;
    TableMeta meta[kMaxIn + 1];  // inputs 0..n_in-1, output at index n_in
    int64_t pool[kMaxPool];
};
hipError_t launch_single(int is_f32, const SingleArgs &a, int max_grid, hipStream_t stream);
// the reference's running sum of a single-op call (seqsum.hip): the terms
// prod_n in[n][pos_n(i, val)] (or in[0] / in[1]) for i over the output dims
// (reference scope order, last fastest) and val < k inner, added in order
constexpr int kSeqMaxDims = 32;
struct SeqSumArgs {
    const void *in[kMaxIn];                        // input tables, base offsets applied
    double *out;                                   // device
    int64_t n_terms;                               // output entries * k
    int64_t k;                                     // card of the summed variable (1: none)
    int n_in, n_dims, divide, pad;
    int64_t card[kSeqMaxDims];
    int64_t stride[kMaxIn][kSeqMaxDims + 1];       // per input: on each output dim, then on the summed variable
};
hipError_t launch_seq_sum(bool f32, const SeqSumArgs &a, hipStream_t stream);
// message exchange steps of sliced runs (xchg.hip; plan.hpp BucketSpec::xchg)
hipError_t launch_xchg_sync(bool f32, TableMeta *meta, int in_t, int x_t, int R, hipStream_t s);
hipError_t launch_xchg_pack(bool f32, TableMeta *meta, int in_t, int x_t, int out_t, int R, int mode, int64_t n,
                            hipStream_t s);
hipError_t launch_xchg_unpack(bool f32, TableMeta *meta, int in_t, int x_t, int out_t, int R, int64_t n,
                              hipStream_t s);
hipError_t launch_xchg_meta(TableMeta *meta, int in_t, int out_t, hipStream_t s);
// stream `s` waits `ns` nanoseconds on the device (one sleeping wave)
hipError_t launch_delay(double ns, hipStream_t s);
// the collective a sliced run's exchanges call (bnpp_collective_fn, include/bnpp.h)
struct XchgHooks {
    int (*fn)(void *user, int op, const void *send, void *recv, int64_t bytes, void *stream) = nullptr;
    void *user = nullptr;
};
// loopy BP, one workgroup (bp.hip)
hipError_t launch_sum_product(const BpArgs &a, hipStream_t stream);
// multi-workgroup flood (bp.hip): messages set to 1/|x|; one iteration (three
// launches); the marginals
hipError_t launch_bp_flood_init(const BpFlood &a, hipStream_t stream);
hipError_t launch_bp_flood_iteration(const BpFlood &a, int it, hipStream_t stream);
hipError_t launch_bp_flood_marginals(const BpFlood &a, hipStream_t stream);

enum DType { kF64 = 0, kF32 = 1 };

struct Context {
    int device = 0;
    hipStream_t stream = nullptr;
    int max_grid = 2048;
    std::string last_error;
    // arena kept between one-shot calls (partition / marginals): mapping and
    // unmapping a few hundred GB of HBM costs ~1 s each way, like a caching
    // allocator the context holds on to it until it is destroyed
    void *arena_cache = nullptr;
    int64_t arena_cache_pad = 0;        // bytes between the hipMalloc'd pointer and arena_cache (alignment)
    int64_t arena_cache_bytes = 0;
    // small device buffers (sources, descriptors, dims pool, metadata, results)
    // kept for reuse: a one-shot call otherwise pays ~10 hipMalloc / hipFree
    // pairs (hipFree synchronises), several ms of a small model's PR
    std::mutex buf_mu;
    std::vector<std::pair<void *, size_t>> buf_free;   // (buffer, capacity)
    size_t buf_free_bytes = 0;
    // the second lane of two-front schedules (Schedule::n_lanes), made on first use
    hipStream_t lane_stream = nullptr;
};

// a device buffer of at least `bytes` from the context's cache (or hipMalloc);
// `cap` receives its capacity, to hand back with put_buffer
hipError_t get_buffer(Context &ctx, size_t bytes, void **p, size_t *cap);
void put_buffer(Context &ctx, void *p, size_t cap);
void drop_buffer_cache(Context &ctx);

// Sources uploaded for one dtype: one device buffer, each factor pre-scaled by
// an exact power of two so its max lies in [0.5, 1).
struct DeviceSources {
    DType dtype = kF64;
    void *buf = nullptr;
    size_t buf_cap = 0;
    std::vector<TableMeta> meta;
    std::vector<int64_t> size;
};

// one result table copied out of the arena (launch_copies: one launch for all)
struct CopyItem {
    const void *src;
    void *dst;
    int64_t bytes;
};

// A schedule bound to device buffers, launchable many times.
struct Executable {
    DType dtype = kF64;
    bool own_arena = true;
    Schedule sched;
    void *arena = nullptr;
    TableMeta *d_meta = nullptr;        // live metadata
    TableMeta *d_meta0 = nullptr;       // pristine copy, restored before every launch
    BucketDesc *d_desc = nullptr;
    int64_t *d_pool = nullptr;
    std::vector<TableMeta> h_meta;
    CopyItem *d_copies = nullptr;       // result tables -> the program's results buffer
    int n_copies = 0;
    int64_t copy_max_bytes = 0;         // the largest of them
    // lanes: events a group records (-1: none) and the events it waits for
    // (producers of its inputs on the other lane); events[0] starts lane 1
    // after the metadata reset, events[1] joins it back before the results
    std::vector<hipEvent_t> events;
    std::vector<int> g_record;
    std::vector<std::vector<int>> g_wait;
    // lanes: the order the groups are enqueued in (empty: schedule order), the
    // lanes' windows alternating (lane_order.hpp)
    std::vector<int> g_order;
    size_t cap_meta = 0, cap_meta0 = 0, cap_desc = 0, cap_pool = 0, cap_copies = 0;   // buffer capacities
};

// Several schedules (target batches of one MAR job) run back to back in one
// shared arena; each batch's result tables are copied into a persistent
// results buffer before the next batch reuses the arena.
struct Program {
    DType dtype = kF64;
    std::vector<Executable> parts;
    void *arena = nullptr;
    int64_t arena_pad = 0;              // bytes between the hipMalloc'd pointer and arena (alignment)
    int64_t arena_bytes = 0;
    bool arena_cached = false;          // arena is the context's cache (not freed with the program)
    bool arena_reused = false;          // ... and was already allocated before this program
    double arena_alloc_ms = 0;          // hipMalloc of the arena (0 when reused), incl. the driver's HBM clearing wait
    void *results = nullptr;
    size_t results_cap = 0;
    int64_t results_bytes = 0;
    std::vector<std::vector<int64_t>> res_off;    // per part, per plan: byte offset (-1: constant 1)
    std::vector<std::vector<int64_t>> res_size;   // per part, per plan: entries
    XchgHooks hooks;                              // sliced runs: the ranks' collective
};

int upload_sources(Context &ctx, const std::vector<std::vector<double>> &values, DType dt, DeviceSources &out);
void free_sources(Context &ctx, DeviceSources &s);
int make_executable(Context &ctx, const DeviceSources &src, Schedule &&s, Executable &ex, void *shared_arena = nullptr);
int launch(Context &ctx, Executable &ex, hipStream_t stream, const XchgHooks *hooks = nullptr);
// waits for `stream`, downloads result tables: values as stored (double) and the exp2 scale
int fetch_results(Context &ctx, Executable &ex, hipStream_t stream, std::vector<std::vector<double>> &vals,
                  std::vector<int64_t> &exp2);
void free_executable(Context &ctx, Executable &ex);

int make_program(Context &ctx, const DeviceSources &src, std::vector<Schedule> &&batches, Program &pg,
                 bool use_cache = false);
// copy n result tables (device array of CopyItem) in one launch (launch.hip)
hipError_t launch_copies(const CopyItem *items, int n, int64_t max_bytes, hipStream_t stream);
// release the context's cached arena
void drop_arena_cache(Context &ctx);
int launch_program(Context &ctx, Program &pg, hipStream_t stream);
// result values (as stored, double) and exp2 of every plan, batches in order
int fetch_program(Context &ctx, Program &pg, hipStream_t stream, std::vector<std::vector<double>> &vals,
                  std::vector<int64_t> &exp2);
void free_program(Context &ctx, Program &pg);

}  // namespace bnpp
