// The reference's running sum of a single-op call (Factor::_partition,
// factor.hh:47): every Factor operation returns, beside its table, the fp64
// sum of its terms added one at a time from 0.0 in the reference's loop order
//   product / divide   the output entries in linear order  (factor.cpp:129-139, 161-172)
//   sum_out            the INPUT entries in (i, val) order  (factor.cpp:196-208)
//   conditioning       the output entries in linear order  (factor.cpp:226-236)
// A fused bucket (Factor(1.0) *= f_0 ... ; .sum_out(v), model.cpp:414-418)
// returns sum_out's: its terms are the chain products p(i, val).
//
// Floating-point addition is not associative, so reproducing those bits
// means adding the terms in that order, one at a time: the sum is sequential
// by construction.  One wave does it: each lane computes one term of the next
// 64 (the mixed-radix decode of its index and the chain product, in the
// reference's arithmetic, so the term is bit-identical to the table entry the
// bucket kernel produced), and the 64 terms are added in order as uniform
// values.  The cost is a chain of dependent fp64 adds (~2e8 terms/s), so the
// ABI computes it only when the caller asks for it (out_sum != NULL).
#include <hip/hip_runtime.h>

#include "runtime.hpp"

namespace bnpp {

template <typename T>
__global__ __launch_bounds__(64) void seq_sum_kernel(SeqSumArgs a) {
    const int lane = threadIdx.x;
    double s = 0.0;
    for (int64_t base = 0; base < a.n_terms; base += 64) {
        const int64_t q = base + lane;
        double t = 0.0;
        if (q < a.n_terms) {
            int64_t i = q / a.k;
            const int64_t val = q - i * a.k;
            int64_t pos[kMaxIn];
#pragma unroll
            for (int n = 0; n < kMaxIn; ++n) pos[n] = val * a.stride[n][kSeqMaxDims];
            for (int d = a.n_dims - 1; d >= 0; --d) {        // last scope variable fastest
                const int64_t c = a.card[d], qd = i / c, r = i - qd * c;
                i = qd;
#pragma unroll
                for (int n = 0; n < kMaxIn; ++n) pos[n] += r * a.stride[n][d];
            }
            T p = static_cast<const T *>(a.in[0])[pos[0]];
#pragma unroll
            for (int n = 1; n < kMaxIn; ++n) {
                if (n >= a.n_in) break;
                const T x = static_cast<const T *>(a.in[n])[pos[n]];
                p = a.divide ? p / x : p * x;
            }
            t = (double)p;
        }
        // the 64 terms in order, one add at a time (uniform)
        const int64_t left = a.n_terms - base;
        for (int j = 0; j < 64; ++j) {
            if (j >= left) break;
            s = s + __shfl(t, j, 64);
        }
    }
    if (lane == 0) *a.out = s;
}

hipError_t launch_seq_sum(bool f32, const SeqSumArgs &a, hipStream_t stream) {
    if (f32)
        hipLaunchKernelGGL(seq_sum_kernel<float>, dim3(1), dim3(64), 0, stream, a);
    else
        hipLaunchKernelGGL(seq_sum_kernel<double>, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace bnpp
