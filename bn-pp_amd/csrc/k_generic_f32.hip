// Kernel instantiations compiled as a separate translation unit (parallel build).
// Generic gather kernels, tiles along one output dim; two-dim tiles are in
// k_generic2_f32.hip.
#include "kernels.cuh"

namespace bnpp {

hipError_t dispatch_level_f32_2d(int key, const LevelArgs &a, int max_grid, hipStream_t stream);
hipError_t dispatch_single_f32_2d(int key, const SingleArgs &a, int max_grid, hipStream_t stream);

hipError_t dispatch_level_f32(int key, const LevelArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_ALL(BNPP_CASE_LEVEL, BNPP_TILES_1D, float) default: break; }
    return dispatch_level_f32_2d(key, a, max_grid, stream);
}
hipError_t dispatch_single_f32(int key, const SingleArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_ALL(BNPP_CASE_SINGLE, BNPP_TILES_1D, float) default: break; }
    return dispatch_single_f32_2d(key, a, max_grid, stream);
}
}  // namespace bnpp
