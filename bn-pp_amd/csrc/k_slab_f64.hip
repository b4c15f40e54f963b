// Slab-form kernel instantiations (double), a separate translation unit (parallel build).
#include "slab.cuh"

namespace bnpp {

hipError_t dispatch_slab_single_f64(int key, const SingleArgs &a, hipStream_t stream) {
    switch (key) { BNPP_SLAB_F64(BNPP_CASE_SLAB_SINGLE, double) BNPP_SLAB8_F64(BNPP_CASE_SLAB8_SINGLE, double) default: break; }
    return hipErrorInvalidValue;
}
hipError_t dispatch_slab_level_f64(int key, const LevelArgs &a, hipStream_t stream) {
    switch (key) { BNPP_SLAB_F64(BNPP_CASE_SLAB_LEVEL, double) BNPP_SLAB_R2_F64(BNPP_CASE_SLAB_LEVEL_R2, double)
                   BNPP_SLAB8_F64(BNPP_CASE_SLAB8_LEVEL, double) default: break; }
    return hipErrorInvalidValue;
}
}  // namespace bnpp
