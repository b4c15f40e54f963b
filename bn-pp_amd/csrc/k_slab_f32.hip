// Slab-form kernel instantiations (float), a separate translation unit (parallel build).
#include "slab.cuh"

namespace bnpp {

hipError_t dispatch_slab_single_f32(int key, const SingleArgs &a, hipStream_t stream) {
    switch (key) { BNPP_SLAB_F32(BNPP_CASE_SLAB_SINGLE, float) BNPP_SLAB8_F32(BNPP_CASE_SLAB8_SINGLE, float) default: break; }
    return hipErrorInvalidValue;
}
hipError_t dispatch_slab_level_f32(int key, const LevelArgs &a, hipStream_t stream) {
    switch (key) { BNPP_SLAB_F32(BNPP_CASE_SLAB_LEVEL, float) BNPP_SLAB_R2_F32(BNPP_CASE_SLAB_LEVEL_R2, float)
                   BNPP_SLAB8_F32(BNPP_CASE_SLAB8_LEVEL, float) default: break; }
    return hipErrorInvalidValue;
}
}  // namespace bnpp
