// Host-side launchers: route a descriptor to the translation unit that holds
// its kernel instantiation (k_generic_f32/f64, k_stream_f32/f64, k_slab_f32/f64,
// k_chain_f32/f64).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bnpp_device.h"
#include "runtime.hpp"

namespace bnpp {

hipError_t dispatch_level_f32(int key, const LevelArgs &a, int max_grid, hipStream_t stream);
hipError_t dispatch_single_f32(int key, const SingleArgs &a, int max_grid, hipStream_t stream);
hipError_t dispatch_level_f64(int key, const LevelArgs &a, int max_grid, hipStream_t stream);
hipError_t dispatch_single_f64(int key, const SingleArgs &a, int max_grid, hipStream_t stream);
hipError_t dispatch_stream_level_f32(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream);
hipError_t dispatch_stream_single_f32(int key, const SingleArgs &a, int max_grid, hipStream_t stream);
hipError_t dispatch_stream_level_f64(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream);
hipError_t dispatch_stream_single_f64(int key, const SingleArgs &a, int max_grid, hipStream_t stream);

hipError_t dispatch_chain_level_f32(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream);
hipError_t dispatch_chain_level_f64(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream);

hipError_t dispatch_slab_single_f32(int key, const SingleArgs &a, hipStream_t stream);
hipError_t dispatch_slab_single_f64(int key, const SingleArgs &a, hipStream_t stream);
hipError_t dispatch_slab_level_f32(int key, const LevelArgs &a, hipStream_t stream);
hipError_t dispatch_slab_level_f64(int key, const LevelArgs &a, hipStream_t stream);

// Result tables out of the arena: blockIdx.x picks the table, the
// kCopyParts workgroups along y share it grid-stride (a multi-GB
// variable_elimination result would crawl through one workgroup); 16-B moves
// while both ends allow them (tables are 256-B aligned in the arena and the
// results buffer), 4-B ones for the tail (sizes are whole fp32 / fp64 entries).
constexpr int kCopyParts = 64;
__global__ __launch_bounds__(256) void copy_tables_kernel(const CopyItem *__restrict__ items, int n) {
    const CopyItem c = items[blockIdx.x];
    const int64_t n16 = c.bytes / 16;
    const int64_t first = (int64_t)blockIdx.y * blockDim.x + threadIdx.x, step = (int64_t)gridDim.y * blockDim.x;
    const uint4 *s16 = static_cast<const uint4 *>(c.src);
    uint4 *d16 = static_cast<uint4 *>(c.dst);
    for (int64_t i = first; i < n16; i += step) d16[i] = s16[i];
    const uint32_t *s4 = static_cast<const uint32_t *>(c.src);
    uint32_t *d4 = static_cast<uint32_t *>(c.dst);
    for (int64_t i = n16 * 4 + first; i < c.bytes / 4; i += step) d4[i] = s4[i];
    (void)n;
}

hipError_t launch_copies(const CopyItem *items, int n, int64_t max_bytes, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    // a workgroup per 64 KiB of the largest table, up to kCopyParts
    const int64_t parts = std::min<int64_t>(kCopyParts, std::max<int64_t>(1, max_bytes >> 16));
    hipLaunchKernelGGL(copy_tables_kernel, dim3((unsigned)n, (unsigned)parts), dim3(256), 0, stream, items, n);
    return hipGetLastError();
}

hipError_t launch_single(int is_f32, const SingleArgs &a, int max_grid, hipStream_t stream) {
    if (a.d.n_tiles <= 0) return hipSuccess;
    if (a.d.big >= 0 && a.d.bcls == kBigSlab) {
        const int key = slab_key(a.d.k, a.d.v1, a.d.v2, a.d.lanes, 1, a.d.slab_y2 ? 8 : a.d.n_in);
        return is_f32 ? dispatch_slab_single_f32(key, a, stream) : dispatch_slab_single_f64(key, a, stream);
    }
    if (a.d.big >= 0) {
        const int key = stream_key(a.d.bcls, a.d.v1, a.d.v2, a.d.n_in);
        return is_f32 ? dispatch_stream_single_f32(key, a, max_grid, stream)
                      : dispatch_stream_single_f64(key, a, max_grid, stream);
    }
    int64_t in_bytes = 0;
    for (int i = 0; i < a.d.n_in && i < kMaxIn; ++i)
        in_bytes = std::max<int64_t>(in_bytes, a.meta[i].size * (is_f32 ? 4 : 8));
    const int key = variant_key(a.d.n_in, a.d.v1, a.d.v2) + (generic_o32(in_bytes) ? kGenericO32 : 0);   // plan.hpp generic_variant
    return is_f32 ? dispatch_single_f32(key, a, max_grid, stream) : dispatch_single_f64(key, a, max_grid, stream);
}

hipError_t launch_level(int is_f32, int variant, const BucketDesc *descs, int n_desc, const int64_t *pool,
                        TableMeta *meta, int64_t total_vblocks, int small_elems, int max_grid, hipStream_t stream) {
    if (n_desc <= 0 || total_vblocks <= 0) return hipSuccess;
    LevelArgs a{descs, n_desc, pool, meta, total_vblocks};
    if (variant >= 16384)                               // slab form: flat grid, one workgroup per virtual block
        return is_f32 ? dispatch_slab_level_f32(variant, a, stream) : dispatch_slab_level_f64(variant, a, stream);
    if (variant >= 8192)
        return is_f32 ? dispatch_chain_level_f32(variant, a, small_elems, max_grid, stream)
                      : dispatch_chain_level_f64(variant, a, small_elems, max_grid, stream);
    if (variant >= 4096)
        return is_f32 ? dispatch_stream_level_f32(variant, a, small_elems, max_grid, stream)
                      : dispatch_stream_level_f64(variant, a, small_elems, max_grid, stream);
    return is_f32 ? dispatch_level_f32(variant, a, max_grid, stream) : dispatch_level_f64(variant, a, max_grid, stream);
}

}  // namespace bnpp
