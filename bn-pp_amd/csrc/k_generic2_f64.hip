// Kernel instantiations compiled as a separate translation unit (parallel build).
// Generic gather kernels, tiles along two output dims.  Built with
// -mllvm -sink-common-insts=false (Makefile): SimplifyCFG otherwise merges the
// stores load_tile's stride cases have in common into one store whose tile
// slot is selected at run time, and the whole tile then lives in scratch
// memory (80-272 B per lane, each load waited for at once).  The one-dim
// tiles measured slower without the sinking and keep the default.
#include "kernels.cuh"

namespace bnpp {

hipError_t dispatch_level_f64_2d(int key, const LevelArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_ALL(BNPP_CASE_LEVEL, BNPP_TILES_F64_2D, double) default: break; }
    return hipErrorInvalidValue;
}
hipError_t dispatch_single_f64_2d(int key, const SingleArgs &a, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_ALL(BNPP_CASE_SINGLE, BNPP_TILES_F64_2D, double) default: break; }
    return hipErrorInvalidValue;
}
}  // namespace bnpp
