// Kernel instantiations compiled as a separate translation unit (parallel build).
#include "kernels.cuh"

namespace bnpp {

hipError_t dispatch_stream_level_f32(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_STREAM_F32(BNPP_CASE_SLEVEL, float) BNPP_STREAM8_F32(BNPP_CASE_SLEVEL8, float) default: break; }
    return hipErrorInvalidValue;
}
hipError_t dispatch_stream_single_f32(int key, const SingleArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_STREAM_F32(BNPP_CASE_SSINGLE, float) BNPP_STREAM8_F32(BNPP_CASE_SSINGLE8, float) default: break; }
    return hipErrorInvalidValue;
}
}  // namespace bnpp
