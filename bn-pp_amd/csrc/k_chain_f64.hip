// Chain (sweep) kernel instantiations, double (separate translation unit).
#include "chainsplit.cuh"

namespace bnpp {

hipError_t dispatch_chain_level_f64(int key, const LevelArgs &a, int small_elems, int max_grid, hipStream_t stream) {
    switch (key) { BNPP_CHAIN_F64(BNPP_CASE_CHAIN, double) BNPP_CHAIN_SPLIT_F64(BNPP_CASE_CHAIN_SPLIT) default: break; }
    return hipErrorInvalidValue;
}
bool chain_supported_f64(int key) {
    switch (key) { BNPP_CHAIN_F64(BNPP_CASE_CHAIN_OK, double) BNPP_CHAIN_SPLIT_F64(BNPP_CASE_CHAIN_SPLIT_OK) default: break; }
    return false;
}
}  // namespace bnpp
