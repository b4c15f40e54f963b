// Chain (sweep) kernel instantiations, float (separate translation unit).
#include "chain.cuh"

namespace bnpp {

hipError_t dispatch_chain_level_f32(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_CHAIN_F32(BNPP_CASE_CHAIN, float) default: break; }
    return hipErrorInvalidValue;
}
bool chain_supported_f32(int key) {
    switch (key) { BNPP_CHAIN_F32(BNPP_CASE_CHAIN_OK, float) default: break; }
    return false;
}
}  // namespace bnpp
