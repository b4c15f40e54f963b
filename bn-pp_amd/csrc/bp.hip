// Loopy belief propagation on the factor graph (the `-sp` path of
// BN::marginals, model.cpp:313-317 -> BN::sum_product, model.cpp:736-753 ->
// FactorGraph, graph.cpp:256-403).
//
// The reference's flooding schedule is Jacobi-style: all variable->factor
// messages of an iteration read only the previous factor->variable messages,
// all factor->variable messages read only the new variable->factor ones.  So
// each phase is one parallel sweep over independent messages with a barrier
// between phases.  BN message sets are tiny (KiB), the iteration count small
// and data-dependent (stop on the largest relative change), so the whole loop
// runs inside ONE workgroup: no launch per iteration, no host round trip for
// the convergence test; the messages live in LDS when they fit (else L1/L2).
// A factor->variable message entry is a sum over the factor's table with one
// variable fixed: short sums take one lane, longer ones 4 / 16 / 64 lanes with
// a butterfly reduction (large CPTs), so no lane walks a long serial chain of
// dependent loads.
//
// Arithmetic: fp64, as the reference.  Products run by ascending factor id
// (variable side) and scope order (factor side); the reference walks
// unordered_maps (graph.hh:50-51), so values agree up to rounding.
#include <hip/hip_runtime.h>

#include "bnpp_device.h"

namespace bnpp {

constexpr int kBpBlock = 1024;

// largest value over the workgroup (every thread gets it); NaN never enters,
// as in the reference (`if (err > maxerror)`, graph.cpp:353)
__device__ double bp_block_max(double v, double *red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double m = red[0];
    for (int w = 1; w < kBpBlock / 64; ++w) m = red[w] > m ? red[w] : m;
    __syncthreads();               // red is rewritten by the next call
    return m;
}

// terms q0, q0 + step, ... of factor->variable message entry t
__device__ __forceinline__ double bp_f2v_terms(const BpArgs &a, const double *v2f, int t, uint32_t q0,
                                               uint32_t step) {
    const int e = a.item_edge[t], o = a.msg_off[e], x = t - o;
    const int f = a.edge_fac[e], k0 = a.f_edge_off[f], k1 = a.f_edge_off[f + 1];
    const uint32_t r = (uint32_t)a.cards[a.edge_var[e]], low = a.edge_stride[e];
    const double *tab = a.tables + a.tab_off[f];
    const uint32_t n = (uint32_t)((a.tab_off[f + 1] - a.tab_off[f]) / r);
    double acc = 0.0;
    for (uint32_t q = q0; q < n; q += step) {
        const uint32_t i = (q / low) * (low * r) + (uint32_t)x * low + q % low;
        double term = tab[i];
        for (int k = k0; k < k1; ++k) {
            if (k == e) continue;
            const uint32_t d = (i / a.edge_stride[k]) % (uint32_t)a.cards[a.edge_var[k]];
            term = term * v2f[a.msg_off[k] + d];
        }
        acc += term;
    }
    return acc;
}

// the factor->variable sums of one lane class: G lanes per sum, butterfly
// reduction (the same bits on every lane of the group)
template <int G>
__device__ __forceinline__ void bp_f2v_class(const BpArgs &a, const double *v2f, int c) {
    const int grp = threadIdx.x / G, lane = threadIdx.x % G;
    for (int q = a.cls_off[c] + grp; q < a.cls_off[c + 1]; q += kBpBlock / G) {
        const int t = a.cls_items[q];
        double acc = bp_f2v_terms(a, v2f, t, (uint32_t)lane, G);
#pragma unroll
        for (int off = G / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (lane == 0) a.raw[t] = acc;
    }
}

// LDS: v2f and f2v live in LDS (2 * n_msg doubles of dynamic shared memory)
template <bool LDS>
__global__ __launch_bounds__(kBpBlock) void sum_product_kernel(const BpArgs a) {
    __shared__ double red[kBpBlock / 64];
    extern __shared__ double lds_msgs[];
    double *v2f = LDS ? lds_msgs : a.v2f;
    double *f2v = LDS ? lds_msgs + a.n_msg : a.f2v;
    const int tid = threadIdx.x;
    // messages start uniform: 1 / |x| (graph.cpp:265-273)
    for (int t = tid; t < a.n_msg; t += kBpBlock) {
        const double u = 1.0 / a.cards[a.edge_var[a.item_edge[t]]];
        v2f[t] = u;
        f2v[t] = u;
    }
    __syncthreads();
    int it = 0;
    for (; it < a.max_iter; ++it) {
        double lmax = 0.0;
        // variable -> factor, one thread per edge (graph.cpp:335-362):
        // Factor(x, 1.0) *= every other factor's message, normalize
        for (int e = tid; e < a.n_edges; e += kBpBlock) {
            const int v = a.edge_var[e], r = a.cards[v], o = a.msg_off[e];
            const int b0 = a.v_edge_off[v], b1 = a.v_edge_off[v + 1];
            double s = 0.0;
            for (int x = 0; x < r; ++x) {
                double p = 1.0;
                for (int q = b0; q < b1; ++q) {
                    const int e2 = a.v_edges[q];
                    if (e2 != e) p = p * f2v[a.msg_off[e2] + x];
                }
                a.raw[o + x] = p;
                s += p;
            }
            for (int x = 0; x < r; ++x) {
                const double nw = a.raw[o + x] / s, old = v2f[o + x];
                const double err = fabs(old - nw) / old;
                if (err > lmax) lmax = err;
                v2f[o + x] = nw;
            }
        }
        __syncthreads();
        // factor -> variable (graph.cpp:364-373): sum over the factor's
        // entries with x_j fixed of F * the other variables' messages
        bp_f2v_class<1>(a, v2f, 0);
        bp_f2v_class<4>(a, v2f, 1);
        bp_f2v_class<16>(a, v2f, 2);
        bp_f2v_class<64>(a, v2f, 3);
        __syncthreads();
        // normalize (graph.cpp:374) and the relative change (graph.cpp:376-385)
        for (int e = tid; e < a.n_edges; e += kBpBlock) {
            const int o = a.msg_off[e], r = a.msg_off[e + 1] - o;
            double s = 0.0;
            for (int x = 0; x < r; ++x) s += a.raw[o + x];
            for (int x = 0; x < r; ++x) {
                const double nw = a.raw[o + x] / s, old = f2v[o + x];
                const double err = fabs(old - nw) / old;
                if (err > lmax) lmax = err;
                f2v[o + x] = nw;
            }
        }
        // (the barriers inside bp_block_max order these writes before the next reads)
        if (bp_block_max(lmax, red) < a.eps) break;          // graph.cpp:328, uniform
    }
    __syncthreads();
    // FactorGraph::marginal (graph.cpp:393-403): Factor(1.0) *= every message, normalize
    for (int v = tid; v < a.n_vars; v += kBpBlock) {
        const int r = a.cards[v], o = a.marg_off[v], b0 = a.v_edge_off[v], b1 = a.v_edge_off[v + 1];
        double s = 0.0;
        for (int x = 0; x < r; ++x) {
            double p = 1.0;
            for (int q = b0; q < b1; ++q) p = p * f2v[a.msg_off[a.v_edges[q]] + x];
            a.marg[o + x] = p;
            s += p;
        }
        for (int x = 0; x < r; ++x) a.marg[o + x] = a.marg[o + x] / s;
    }
    if (tid == 0) *a.iterations = it;
}

// ---------------------------------------------------------------------------
// Multi-workgroup flood (BpFlood, bnpp_device.h).  Same phases and arithmetic
// as the loop above, one launch per phase: v2f (a thread per edge), f2v
// partial sums (a lane group per segment), finish (a thread per edge: parts
// summed in order, normalised, relative change).  64-bit table indices where
// a factor has 2^32 entries or more.

// true when iteration it-1 met the tolerance: every launch of iteration it
// returns without touching a message (graph.cpp:328, `maxerror < epsilon`)
__device__ __forceinline__ bool bp_flood_done(const BpFlood &a, int it) {
    return it > 0 && __longlong_as_double((long long)a.err[(it - 1) % kBpErrRing]) < a.eps;
}

// wave maximum of a non-negative (or NaN-free) error, one atomic per wave
__device__ __forceinline__ void bp_flood_err(const BpFlood &a, int it, double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    if ((threadIdx.x & 63) == 0 && v > 0.0)
        atomicMax(a.err + it % kBpErrRing, (unsigned long long)__double_as_longlong(v));
}

__global__ __launch_bounds__(kBpFloodBlock) void bp_flood_init_kernel(const BpFlood a) {
    const int t = blockIdx.x * kBpFloodBlock + threadIdx.x;
    if (t < a.n_msg) {
        const double u = 1.0 / a.cards[a.edge_var[a.item_edge[t]]];       // graph.cpp:265-273
        a.v2f[t] = u;
        a.f2v[t] = u;
    }
}

// variable -> factor (graph.cpp:335-362), one thread per edge
__global__ __launch_bounds__(kBpFloodBlock) void bp_flood_v2f_kernel(const BpFlood a, int it) {
    if (bp_flood_done(a, it)) return;
    const int e = blockIdx.x * kBpFloodBlock + threadIdx.x;
    double lmax = 0.0;
    if (e < a.n_edges) {
        const int v = a.edge_var[e], r = a.cards[v], o = a.msg_off[e];
        const int b0 = a.v_edge_off[v], b1 = a.v_edge_off[v + 1];
        double s = 0.0;
        if (b1 - b0 <= 8) {
            // up to 8 edges (grids, most networks): the offsets, then each x's
            // messages, as independent loads rather than a dependent chain
            int mo[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) mo[q] = b0 + q < b1 ? a.v_moff[b0 + q] : -1;
            for (int x = 0; x < r; ++x) {
                double m[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) m[q] = mo[q] >= 0 && mo[q] != o ? a.f2v[mo[q] + x] : 1.0;
                double p = 1.0;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (mo[q] >= 0 && mo[q] != o) p = p * m[q];
                a.raw[o + x] = p;
                s += p;
            }
        } else {
            for (int x = 0; x < r; ++x) {
                double p = 1.0;
                for (int q = b0; q < b1; ++q) {
                    const int o2 = a.v_moff[q];
                    if (o2 != o) p = p * a.f2v[o2 + x];
                }
                a.raw[o + x] = p;
                s += p;
            }
        }
        for (int x = 0; x < r; ++x) {
            const double nw = a.raw[o + x] / s, old = a.v2f[o + x];
            const double err = fabs(old - nw) / old;
            if (err > lmax) lmax = err;
            a.v2f[o + x] = nw;
        }
    }
    bp_flood_err(a, it, lmax);
}

// terms q0 + lane, q0 + lane + G, ... < q1 of factor->variable entry t
template <typename I>
__device__ __forceinline__ double bp_flood_terms(const BpFlood &a, int t, uint64_t q0, uint64_t q1, uint32_t lane,
                                                 uint32_t G) {
    const int e = a.item_edge[t], x = t - a.msg_off[e];
    const int f = a.edge_fac[e], k0 = a.f_edge_off[f], k1 = a.f_edge_off[f + 1];
    const I r = (I)a.cards[a.edge_var[e]], low = (I)a.edge_stride[e];
    const double *tab = a.tables + a.tab_off[f];
    double acc = 0.0;
    for (I q = (I)q0 + lane; q < (I)q1; q += G) {
        const I i = (q / low) * (low * r) + (I)x * low + q % low;
        double term = tab[i];
        for (int k = k0; k < k1; ++k) {
            if (k == e) continue;
            const I d = (i / (I)a.edge_stride[k]) % (I)a.cards[a.edge_var[k]];
            term = term * a.v2f[a.msg_off[k] + (int)d];
        }
        acc += term;
    }
    return acc;
}

template <int G>
__device__ __forceinline__ void bp_flood_class(const BpFlood &a, int c) {
    const int64_t pos = a.cls_pos[c] + (int64_t)(blockIdx.x - a.cls_blk[c]) * (kBpFloodBlock / G) + threadIdx.x / G;
    const uint32_t lane = threadIdx.x % G;
    double acc = 0.0;
    int s = -1;
    if (pos < a.cls_pos[c + 1]) {
        s = a.cls_seg[pos];
        const int t = a.seg_item[s];
        const uint64_t q0 = a.seg_q0[s];
        const int e = a.item_edge[t], f = a.edge_fac[e];
        const uint64_t n = (uint64_t)(a.tab_off[f + 1] - a.tab_off[f]), terms = n / (uint64_t)a.cards[a.edge_var[e]];
        const uint64_t q1 = q0 + kBpSegTerms < terms ? q0 + kBpSegTerms : terms;
        acc = (a.idx64 || (n >> 32)) ? bp_flood_terms<uint64_t>(a, t, q0, q1, lane, G) : bp_flood_terms<uint32_t>(a, t, q0, q1, lane, G);
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (s >= 0 && lane == 0) a.part[s] = acc;
}

// factor -> variable partial sums (graph.cpp:364-373): the blocks of lane
// class c are [cls_blk[c], cls_blk[c+1])
__global__ __launch_bounds__(kBpFloodBlock) void bp_flood_f2v_kernel(const BpFlood a, int it) {
    if (bp_flood_done(a, it)) return;
    const int b = blockIdx.x;
    if (b < a.cls_blk[1]) bp_flood_class<1>(a, 0);
    else if (b < a.cls_blk[2]) bp_flood_class<4>(a, 1);
    else if (b < a.cls_blk[3]) bp_flood_class<16>(a, 2);
    else bp_flood_class<64>(a, 3);
}

// normalize (graph.cpp:374) and the relative change (graph.cpp:376-385)
__global__ __launch_bounds__(kBpFloodBlock) void bp_flood_finish_kernel(const BpFlood a, int it) {
    if (bp_flood_done(a, it)) return;
    const int e = blockIdx.x * kBpFloodBlock + threadIdx.x;
    double lmax = 0.0;
    if (e < a.n_edges) {
        const int o = a.msg_off[e], r = a.msg_off[e + 1] - o;
        double s = 0.0;
        for (int x = 0; x < r; ++x) {
            double v = 0.0;
            if (a.one_seg) {
                v = a.part[o + x];                      // segment t = entry t
            } else {
                for (int64_t p = a.seg_off[o + x]; p < a.seg_off[o + x + 1]; ++p) v += a.part[p];
            }
            a.raw[o + x] = v;
            s += v;
        }
        for (int x = 0; x < r; ++x) {
            const double nw = a.raw[o + x] / s, old = a.f2v[o + x];
            const double err = fabs(old - nw) / old;
            if (err > lmax) lmax = err;
            a.f2v[o + x] = nw;
        }
    }
    bp_flood_err(a, it, lmax);
}

// FactorGraph::marginal (graph.cpp:393-403), one thread per variable
__global__ __launch_bounds__(kBpFloodBlock) void bp_flood_marginal_kernel(const BpFlood a) {
    const int v = blockIdx.x * kBpFloodBlock + threadIdx.x;
    if (v >= a.n_vars) return;
    const int r = a.cards[v], o = a.marg_off[v], b0 = a.v_edge_off[v], b1 = a.v_edge_off[v + 1];
    double s = 0.0;
    for (int x = 0; x < r; ++x) {
        double p = 1.0;
        for (int q = b0; q < b1; ++q) p = p * a.f2v[a.v_moff[q] + x];
        a.marg[o + x] = p;
        s += p;
    }
    for (int x = 0; x < r; ++x) a.marg[o + x] = a.marg[o + x] / s;
}

static inline unsigned bp_blocks(int64_t n) { return (unsigned)((n + kBpFloodBlock - 1) / kBpFloodBlock); }

hipError_t launch_bp_flood_init(const BpFlood &a, hipStream_t stream) {
    if (a.n_msg > 0) hipLaunchKernelGGL(bp_flood_init_kernel, dim3(bp_blocks(a.n_msg)), dim3(kBpFloodBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_bp_flood_iteration(const BpFlood &a, int it, hipStream_t stream) {
    if (a.n_edges == 0) return hipSuccess;
    hipLaunchKernelGGL(bp_flood_v2f_kernel, dim3(bp_blocks(a.n_edges)), dim3(kBpFloodBlock), 0, stream, a, it);
    if (a.cls_blk[4] > 0)
        hipLaunchKernelGGL(bp_flood_f2v_kernel, dim3((unsigned)a.cls_blk[4]), dim3(kBpFloodBlock), 0, stream, a, it);
    hipLaunchKernelGGL(bp_flood_finish_kernel, dim3(bp_blocks(a.n_edges)), dim3(kBpFloodBlock), 0, stream, a, it);
    return hipGetLastError();
}

hipError_t launch_bp_flood_marginals(const BpFlood &a, hipStream_t stream) {
    if (a.n_vars > 0)
        hipLaunchKernelGGL(bp_flood_marginal_kernel, dim3(bp_blocks(a.n_vars)), dim3(kBpFloodBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_sum_product(const BpArgs &a, hipStream_t stream) {
    if (a.msgs_in_lds && a.n_msg <= kBpLdsMsgMax)
        hipLaunchKernelGGL(sum_product_kernel<true>, dim3(1), dim3(kBpBlock), 2 * sizeof(double) * (size_t)a.n_msg,
                           stream, a);
    else
        hipLaunchKernelGGL(sum_product_kernel<false>, dim3(1), dim3(kBpBlock), 0, stream, a);
    return hipGetLastError();
}

}  // namespace bnpp
