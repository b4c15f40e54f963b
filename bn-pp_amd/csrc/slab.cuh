// Slab form of the fused bucket (gfx950): the bench bucket and its relatives.
//
//   out[s, y] = sum_{v < K}  prod_i in_i        (model.cpp:414-418, chain order)
//
// where exactly one input is big and holds the summed variable as K slabs that
// are contiguous along the output's slow index s:  big[base + v * es + s],
// and every other (small) input depends only on (v, y):  g_i[base_i + v * es_i
// + y * sy_i].  The output row of one s is C0 consecutive entries (y fastest,
// domain.cpp:15-26).  Examples: a column-sweep forward message m(x, S) * f(x, y)
// -> sum_x (C0 = card y), the BASELINE config-5 bucket (K = C0 = 4), a plain
// sum-out of a table's slowest variable (C0 = 1).
//
// Why a separate kernel: a float4 copy reads+writes HBM at 6.3 TB/s when every
// workgroup moves one 4-KiB chunk (flat grid) and at 5.5-5.7 TB/s grid-stride
// (tools/membw4/5/6.hip; vmcnt counts loads and stores in order, so a grid-stride
// loop's next loads wait for its own stores).  This kernel is that flat shape:
// one workgroup per 256 tiles, a tile = V consecutive s values, the K slab loads
// issued back to back before any use (V * K entries in flight per lane), small
// tables read by wave-uniform (scalar) loads, no LDS, no barrier in the single
// form, ~40 VGPRs so 8 waves per SIMD stay resident.
//
// Arithmetic is the reference's, in the reference's order: p = 1; p *= in_0;
// ...; acc += p for v = 0..K-1 (factor.cpp:131-143, 199-205).  The inputs before
// the big one are folded left to right into `pre` (exactly what the chain does
// before it reaches the big input: 1 * in_0 * in_1 ...), the ones after it are
// multiplied one at a time, so fp64 results stay bit-identical.
#pragma once
#include "kernels.cuh"

namespace bnpp {

constexpr int kSlabMaxIn = 4;       // inputs of the default class; NI = 8: buckets of 5-8 inputs (kSlab8In)

// tile outputs per lane: C0 * V consecutive entries
template <typename T, int K, int C0, int V, int NI = kSlabMaxIn>
struct SlabTile {
    static constexpr int N = C0 * V;

    // small input i's values at (v, y) -> g[v][y] (wave-uniform loads); the
    // row's y spans output dim 0 (stride sy) or -- the 8-input class only
    // (NI = 8), when y2 > 0 -- dims 0 and 1 (y % 2 along dim 0, y / 2 along
    // dim 1 at stride sy1; C0 = 4, y2 = 2).  The default class keeps the
    // one-dim form: the bench bucket's kernel lost 5 % to the run-time select
    static __device__ __forceinline__ void load_small(const T *p, int64_t es, int64_t sy, T (&g)[K][C0], int y2 = 0,
                                                      int64_t sy1 = 0) {
#pragma unroll
        for (int v = 0; v < K; ++v)
#pragma unroll
            for (int y = 0; y < C0; ++y) {
                int64_t oy = (int64_t)y * sy;
                if constexpr (NI > kSlabMaxIn)
                    if (y2 == 2) oy = (int64_t)(y & 1) * sy + (int64_t)(y >> 1) * sy1;
                g[v][y] = gload(p + (int64_t)v * es + oy);
            }
    }

    // acc[j * C0 + y] for s = s0 + j:  inputs in chain order around the big one
    template <typename SmallAt>
    static __device__ __forceinline__ void compute(const T (&m)[K][V], int big, int n_in, SmallAt &&small,
                                                   T (&acc)[N]) {
        T pre[K][C0];
        bool has_pre = false;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (i >= n_in || i >= big) break;               // uniform
            T g[K][C0];
            small(i, g);
#pragma unroll
            for (int v = 0; v < K; ++v)
#pragma unroll
                for (int y = 0; y < C0; ++y) pre[v][y] = has_pre ? pre[v][y] * g[v][y] : g[v][y];   // 1 * in_0 = in_0
            has_pre = true;
        }
        T p[K][N];
#pragma unroll
        for (int v = 0; v < K; ++v)
#pragma unroll
            for (int j = 0; j < V; ++j)
#pragma unroll
                for (int y = 0; y < C0; ++y) p[v][j * C0 + y] = has_pre ? pre[v][y] * m[v][j] : m[v][j];
#pragma unroll
        for (int i = 1; i < NI; ++i) {
            if (i >= n_in) break;                           // uniform
            if (i <= big) continue;
            T g[K][C0];
            small(i, g);
#pragma unroll
            for (int v = 0; v < K; ++v)
#pragma unroll
                for (int j = 0; j < V; ++j)
#pragma unroll
                    for (int y = 0; y < C0; ++y) p[v][j * C0 + y] = p[v][j * C0 + y] * g[v][y];
        }
#pragma unroll
        for (int e = 0; e < N; ++e) {
            T a = T(0);
#pragma unroll
            for (int v = 0; v < K; ++v) a = a + p[v][e];
            acc[e] = a;
        }
    }
};

// stride of small input i along y (output dim 0 when C0 = v1 > 1), and along
// output dim 1 when the row spans two dims (slab_y2: launched as the 8-input
// class whatever the input count, slab_key)
__device__ __forceinline__ int64_t slab_sy(const BucketDesc &d, const int64_t *dims, int i) {
    return d.v1 > 1 ? dims[2 + i] : 0;
}
__device__ __forceinline__ int64_t slab_sy1(const BucketDesc &d, const int64_t *dims, int i) {
    return d.slab_y2 ? dims[(2 + d.n_in) + 2 + i] : 0;
}

template <typename T, int K, int C0, int V, bool NTL>
__device__ __forceinline__ void slab_load_big(const T *bp, int64_t es, T (&m)[K][V]) {
#pragma unroll
    for (int v = 0; v < K; ++v) load_n<T, V, NTL, true>(bp + (int64_t)v * es, m[v]);
}

// H lanes share one tile (H = 2 for 32-B tile rows): both load the tile's K * V
// big entries (the same addresses: one transaction) and compute it whole; lane
// h stores entries [h * N/H, (h+1) * N/H), so a wave's store instruction writes
// one contiguous run (a 32-B row per lane would write 16-B pieces at a 32-B
// stride per instruction: 0.68 of HBM peak for the f64 bench bucket)
template <typename T, int N, int H, bool NT>
__device__ __forceinline__ void slab_store(T *row, const T (&acc)[N], int h) {
    if constexpr (H == 1) {
        store_n<T, N, NT, true>(row, acc);
    } else {
        T part[N / H];
#pragma unroll
        for (int e = 0; e < N / H; ++e) part[e] = h ? acc[N / H + e] : acc[e];
        store_n<T, N / H, NT, true>(row + h * (N / H), part);
    }
}

template <typename T, int K, int C0, int V, int H, int NI>
__global__ __launch_bounds__(kBlock) void slab_single_kernel(const SingleArgs args) {
#if defined(__HIP_DEVICE_COMPILE__)
    (void)args;
    const SingleArgs &a = *(const __attribute__((address_space(4))) SingleArgs *)__builtin_amdgcn_kernarg_segment_ptr();
#else
    const SingleArgs &a = args;
#endif
    using ST = SlabTile<T, K, C0, V, NI>;
    const BucketDesc &d = a.d;
    const int64_t gt = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t t = H == 1 ? gt : gt / H;
    if (t >= d.n_tiles) return;
    const int big = d.big;
    T m[K][V];
    slab_load_big<T, K, C0, V, true>(static_cast<const T *>(a.big_ptr) + t * V, a.big_es, m);
    T acc[ST::N];
    ST::compute(m, big, d.n_in, [&](int i, T (&g)[K][C0]) {
        ST::load_small(static_cast<const T *>(a.meta[i].ptr) + d.in_base[i], d.elim_stride[i], slab_sy(d, a.pool, i), g,
                       d.slab_y2, slab_sy1(d, a.pool, i));
    }, acc);
    slab_store<T, ST::N, H, true>(static_cast<T *>(a.meta[d.n_in].ptr) + t * ST::N, acc, (int)(gt & (H - 1)));
}

// Level form: one workgroup per virtual block of a level's slab buckets (flat
// grid), with the VE rescaling (kScale) and the max tracking (kTrackMax) of
// the other level kernels.
template <typename T, int K, int C0, int V, int H, int R, int NI>
__global__ __launch_bounds__(kBlock) void slab_level_kernel(const BucketDesc *__restrict__ descs, int n_desc,
                                                            const int64_t *__restrict__ pool,
                                                            TableMeta *__restrict__ meta) {
    using ST = SlabTile<T, K, C0, V, NI>;
    __shared__ T red[kBlock / 64];
    const int64_t vb = blockIdx.x;
    const int bi = n_desc == 1 ? 0 : find_bucket(descs, n_desc, vb);
    // descriptor, dims pool and the inputs' metadata through the scalar cache
    // (read-only while the launch runs; the one store below, the output's
    // exp2, is never read back here): read as plain global memory, every use
    // after that store re-read them, a chain of dependent scalar loads ahead
    // of each pass's big loads (the 8-input class's 5-input bucket of the
    // conditioned 32x32 PR: 13.6 ms fp32 for 25.8 GB)
    cst_t<BucketDesc> &d = *as_const(descs + bi);
    cst_t<int64_t> *dims = as_const(pool) + d.dim_off;
    cst_t<TableMeta> *cmeta = as_const(meta);
    const int big = d.big;
    // H lanes per tile; R passes of kBlock / H tiles per block, every pass's
    // loads issued before the first tile is computed
    constexpr int TPP = kBlock / H;
    const int64_t t0 = (vb - d.vblk_begin) * (TPP * R) + threadIdx.x / H;
    // outer dims: this block's combination (uniform) moves every input's base
    cst_t<int64_t> *adj = nullptr;
    if (d.outer_n > 0) {
        uint64_t q, r;
        divmod_dim((uint64_t)(vb - d.vblk_begin), d.outer_div[0], d.outer_div[1], q, r);
        adj = dims + d.outer_rel + (int64_t)q * d.n_in;
    }
    auto base_of = [&](int i) { return adj ? d.in_base[i] + adj[i] : d.in_base[i]; };
    const T *bigp = static_cast<const T *>(cmeta[d.in_table[big]].ptr) + base_of(big);
    const int64_t big_es = d.elim_stride[big];
    T m[R][K][V];
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (t0 + r * TPP < d.n_tiles)
            slab_load_big<T, K, C0, V, kNtLoad>(bigp + (t0 + r * TPP) * V, big_es, m[r]);
    int64_t e_sum = 0, x_sum = 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        if (i >= d.n_in) break;
        cst_t<TableMeta> &mi = cmeta[d.in_table[i]];
        const int e = FBits<T>::exponent(mi.maxbits);
        if (d.flags & kScale) {
            e_sum += e;
            x_sum += mi.exp2 + e;
        } else {
            x_sum += mi.exp2;
        }
    }
    if (vb == d.vblk_begin && threadIdx.x == 0) meta[d.out_table].exp2 = x_sum;
    T lmax = T(0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t t = t0 + r * TPP;
        if (t >= d.n_tiles) break;
        T acc[ST::N];
        ST::compute(m[r], big, d.n_in, [&](int i, T (&g)[K][C0]) {
            ST::load_small(static_cast<const T *>(cmeta[d.in_table[i]].ptr) + base_of(i), d.elim_stride[i],
                           d.v1 > 1 ? dims[2 + i] : 0, g, d.slab_y2, d.slab_y2 ? dims[(2 + d.n_in) + 2 + i] : 0);
        }, acc);
        if (d.flags & kScale) {
#pragma unroll
            for (int e = 0; e < ST::N; ++e) acc[e] = ldexp_t(acc[e], (int)(-e_sum));
        }
#pragma unroll
        for (int e = 0; e < ST::N; ++e) lmax = acc[e] > lmax ? acc[e] : lmax;
        slab_store<T, ST::N, H, kNtStore>(static_cast<T *>(cmeta[d.out_table].ptr) + t * ST::N, acc,
                                           (int)(threadIdx.x & (H - 1)));
    }
    if (d.flags & kTrackMax) {
        // one atomic per workgroup at most, skipped when the table's max
        // already covers this block (a stale read only costs a needless atomic)
        T w = wave_max(lmax);
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        if (lane == 0) red[wid] = w;
        __syncthreads();
        if (threadIdx.x == 0) {
            T mx = red[0];
            for (int i = 1; i < kBlock / 64; ++i) mx = red[i] > mx ? red[i] : mx;
            using U = typename FBits<T>::U;
            U *mb = reinterpret_cast<U *>(&meta[d.out_table].maxbits);
            const U mine = FBits<T>::bits(mx);
            if (mx > T(0) && __hip_atomic_load(mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < mine)
                atomicMax(mb, mine);
        }
    }
}

template <typename T, int K, int C0, int V, int H, int NI = kSlabMaxIn>
static hipError_t go_slab_single(const SingleArgs &a, hipStream_t stream) {
    const int64_t blocks = (a.d.n_tiles * H + kBlock - 1) / kBlock;
    hipLaunchKernelGGL((slab_single_kernel<T, K, C0, V, H, NI>), dim3((unsigned)blocks), dim3(kBlock), 0, stream, a);
    return hipGetLastError();
}

template <typename T, int K, int C0, int V, int H, int R, int NI = kSlabMaxIn>
static hipError_t go_slab_level(const LevelArgs &a, hipStream_t stream) {
    hipLaunchKernelGGL((slab_level_kernel<T, K, C0, V, H, R, NI>), dim3((unsigned)a.vblocks), dim3(kBlock), 0, stream,
                       a.descs, a.n_desc, a.pool, a.meta);
    return hipGetLastError();
}

// instantiated shapes: K = 1..4 summed values; (C0, V, H): f32 (1,1) (1,4)
// (2,1) (2,2) (4,1) (4,2) and (4,2,2); f64 (1,1) (1,2) (2,1) (4,1) (2,2) and
// the 32-B rows again as (2,2,2) (4,1,2) -- H = 2 where a tile row is 32 B
// (planner; BNPP_SLAB_LANES=1 keeps H = 1 for A/B)
#define BNPP_SLAB_K(X, T, C0, V, H) X(T, 1, C0, V, H) X(T, 2, C0, V, H) X(T, 3, C0, V, H) X(T, 4, C0, V, H)
#define BNPP_SLAB_F32(X, T) BNPP_SLAB_K(X, T, 1, 1, 1) BNPP_SLAB_K(X, T, 1, 4, 1) BNPP_SLAB_K(X, T, 2, 1, 1) \
    BNPP_SLAB_K(X, T, 2, 2, 1) BNPP_SLAB_K(X, T, 4, 1, 1) BNPP_SLAB_K(X, T, 4, 2, 1) BNPP_SLAB_K(X, T, 4, 2, 2)
#define BNPP_SLAB_F64(X, T) BNPP_SLAB_K(X, T, 1, 1, 1) BNPP_SLAB_K(X, T, 1, 2, 1) BNPP_SLAB_K(X, T, 2, 1, 1) \
    BNPP_SLAB_K(X, T, 4, 1, 1) BNPP_SLAB_K(X, T, 2, 2, 1) BNPP_SLAB_K(X, T, 2, 2, 2) BNPP_SLAB_K(X, T, 4, 1, 2)
#define BNPP_CASE_SLAB_SINGLE(T, K, C0, V, H) \
    case slab_key(K, C0, V, H): return go_slab_single<T, K, C0, V, H>(a, stream);
#define BNPP_CASE_SLAB_LEVEL(T, K, C0, V, H) \
    case slab_key(K, C0, V, H): return go_slab_level<T, K, C0, V, H, 1>(a, stream);
// level launches with two passes per block (BucketDesc::slab_r; four measured
// slower, profiles/r04_slab_passes_ab.txt)
#define BNPP_SLAB_R2_F32(X, T) BNPP_SLAB_K(X, T, 1, 4, 1) BNPP_SLAB_K(X, T, 2, 2, 1)
#define BNPP_SLAB_R2_F64(X, T) BNPP_SLAB_K(X, T, 1, 2, 1)
#define BNPP_CASE_SLAB_LEVEL_R2(T, K, C0, V, H) \
    case slab_key(K, C0, V, H, 2): return go_slab_level<T, K, C0, V, H, 2>(a, stream);
// 5-8 inputs (kSlab8In): one entry of the slab dim per lane (V = 1), one pass;
// H = 2 where the tile row is 32 B (f64 C0 = 4)
#define BNPP_SLAB8_F32(X, T) BNPP_SLAB_K(X, T, 1, 1, 1) BNPP_SLAB_K(X, T, 2, 1, 1) BNPP_SLAB_K(X, T, 4, 1, 1)
#define BNPP_SLAB8_F64(X, T) BNPP_SLAB_K(X, T, 1, 1, 1) BNPP_SLAB_K(X, T, 2, 1, 1) BNPP_SLAB_K(X, T, 4, 1, 2)
#define BNPP_CASE_SLAB8_SINGLE(T, K, C0, V, H) \
    case slab_key(K, C0, V, H, 1, 8): return go_slab_single<T, K, C0, V, H, 8>(a, stream);
#define BNPP_CASE_SLAB8_LEVEL(T, K, C0, V, H) \
    case slab_key(K, C0, V, H, 1, 8): return go_slab_level<T, K, C0, V, H, 1, 8>(a, stream); \
    case slab_key(K, C0, V, H, 2, 8): return go_slab_level<T, K, C0, V, H, 2, 8>(a, stream); \
    case slab_key(K, C0, V, H, 4, 8): return go_slab_level<T, K, C0, V, H, 4, 8>(a, stream);

}  // namespace bnpp
