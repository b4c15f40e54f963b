// Kernel instantiations compiled as a separate translation unit (parallel build).
#include "kernels.cuh"

namespace bnpp {

hipError_t dispatch_level_f64(int key, const LevelArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_ALL(BNPP_CASE_LEVEL, BNPP_TILES_F64, double) default: break; }
    return hipErrorInvalidValue;
}
hipError_t dispatch_single_f64(int key, const SingleArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_ALL(BNPP_CASE_SINGLE, BNPP_TILES_F64, double) default: break; }
    return hipErrorInvalidValue;
}
}  // namespace bnpp
