// Kernel instantiations compiled as a separate translation unit (parallel build).
#include "kernels.cuh"

namespace bnpp {

hipError_t dispatch_stream_level_f64(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_STREAM_F64(BNPP_CASE_SLEVEL, double) BNPP_STREAM8_F64(BNPP_CASE_SLEVEL8, double) default: break; }
    return hipErrorInvalidValue;
}
hipError_t dispatch_stream_single_f64(int key, const SingleArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_STREAM_F64(BNPP_CASE_SSINGLE, double) BNPP_STREAM8_F64(BNPP_CASE_SSINGLE8, double) default: break; }
    return hipErrorInvalidValue;
}
}  // namespace bnpp
