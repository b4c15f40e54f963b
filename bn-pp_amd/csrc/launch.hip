// Host-side launchers: route a descriptor to the translation unit that holds
// its kernel instantiation (k_generic_f32/f64, k_stream_f32/f64, k_slab_f32/f64,
// k_chain_f32/f64).
#include <hip/hip_runtime.h>

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

hipError_t launch_single(int is_f32, const SingleArgs &a, int max_grid, hipStream_t stream) {
    if (a.d.n_tiles <= 0) return hipSuccess;
    if (a.d.big >= 0 && a.d.bcls == kBigSlab) {
        const int key = slab_key(a.d.k, a.d.v1, a.d.v2);
        return is_f32 ? dispatch_slab_single_f32(key, a, stream) : dispatch_slab_single_f64(key, a, stream);
    }
    if (a.d.big >= 0) {
        const int key = stream_key(a.d.bcls, a.d.v1, a.d.v2);
        return is_f32 ? dispatch_stream_single_f32(key, a, max_grid, stream)
                      : dispatch_stream_single_f64(key, a, max_grid, stream);
    }
    const int key = variant_key(a.d.n_in, a.d.v1, a.d.v2);
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
