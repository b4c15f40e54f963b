// Host-side check of the generic kernels' offset-width choice at the 4-GiB
// boundary: a view whose reachable span passes 2^32 bytes must
// get the 64-bit-offset kernel, one just below it the 32-bit one.  Headers
// only: the same inline functions the planner (plan.cpp) and the single-op
// path (capi.cpp run_single -> launch.hip) use.  No allocation, no GPU.
#include <cstdio>
#include <vector>

#include "plan.hpp"

using namespace bnpp;

static int fails = 0;
#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                               \
        }                                                          \
    } while (0)

static View binary_view(int n, int64_t base) {
    View v;
    v.base = base;
    for (int j = 0; j < n; ++j) {
        v.vars.push_back(j);
        v.strides.push_back((int64_t)1 << (n - 1 - j));
    }
    return v;
}

int main() {
    std::vector<int> cards(40, 2);
    CHECK(generic_o32(0xffffffffll));
    CHECK(!generic_o32(0x100000000ll));
    // fp32: 2^30 entries = 2^32 bytes -> 64-bit offsets; 2^30 - 1 entries -> 32-bit
    const View full30 = binary_view(30, 0);
    CHECK(view_span(full30, cards) == ((int64_t)1 << 30));
    CHECK(!generic_o32(view_span(full30, cards) * 4));
    View below = binary_view(29, 0);
    below.base = ((int64_t)1 << 29) - 1;                  // reaches entry 2^30 - 2: span 2^30 - 1
    CHECK(view_span(below, cards) == ((int64_t)1 << 30) - 1);
    CHECK(generic_o32(view_span(below, cards) * 4));
    // a conditioned view (evidence in the base) past the boundary: base 2^29 + 2^29 entries
    const View cond = binary_view(29, (int64_t)1 << 29);
    CHECK(view_span(cond, cards) == ((int64_t)1 << 30));
    CHECK(!generic_o32(view_span(cond, cards) * 4));
    // fp64: 2^29 entries = 2^32 bytes
    CHECK(!generic_o32(view_span(binary_view(29, 0), cards) * 8));
    CHECK(generic_o32(view_span(binary_view(28, 0), cards) * 8));
    // the variant keys: the O32 bit exactly when the offsets fit (and never under BNPP_NO_O32)
    CHECK(generic_variant(5, 2, 2, view_span(full30, cards) * 4) == variant_key(5, 2, 2));
    CHECK(generic_variant(5, 2, 2, view_span(below, cards) * 4) == variant_key(5, 2, 2) + kGenericO32);
    CHECK(generic_variant(5, 2, 2, view_span(below, cards) * 4, true) == variant_key(5, 2, 2));
    // saturation: a span past any device stays "too big", never wraps into the 32-bit range
    const View huge = binary_view(40, (int64_t)1 << 62);
    CHECK(view_span(huge, cards) == kSatMax);
    CHECK(!generic_o32(sat_mul(view_span(huge, cards), 8)));
    if (fails) return 1;
    std::printf("o32 keys ok\n");
    return 0;
}
