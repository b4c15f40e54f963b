/*
 * bnpp.h — C ABI of the MI355X-native bn-pp variable-elimination engine.
 *
 * The reference (GEO-IASS/bn-pp) has no FFI: its hot path sits behind the C++
 * class API of code/factor.hh and code/model.hh.  Every entry point below names
 * the reference interface it replaces (file:line into the reference's code/).
 * The C++ mirror of that class API (bn::Variable/Domain/Factor/BN/MN) lives in
 * include/bnpp/bn.hpp and is implemented on top of these calls.
 *
 * Conventions
 *   - Plain pointers and sizes; no C++ types; no exceptions cross the ABI.
 *   - Every call returns an int status (BNPP_OK == 0, negative on error);
 *     bnpp_strerror(status) names it, bnpp_last_error() gives the detail of the
 *     last failure on the calling thread.
 *   - Tables are row-major over their scope with the LAST variable fastest
 *     (domain.cpp:15-26).  Scopes are arrays of variable ids; `cards` is indexed
 *     by variable id and holds n_cards entries: an id outside [0, n_cards)
 *     anywhere in a call is BNPP_ERR_INVALID (the array is never read past).
 *   - Device tables passed to the single-op calls are caller-owned device
 *     buffers (bnpp_malloc, hipMalloc or a torch tensor's data_ptr); the engine
 *     never frees them.  `stream` is a hipStream_t (NULL: the context stream).
 *     Single-op calls only enqueue work.
 *   - No CPU fallback: without a usable MI355X every compute call fails with
 *     BNPP_ERR_NO_DEVICE.  Model loading, evidence loading, ordering and scope
 *     rules are host-only and work everywhere.
 *   - Thread safety: one context per device; calls on distinct contexts or
 *     distinct streams may run concurrently; model objects are read-only after
 *     creation.
 */
#ifndef BNPP_H
#define BNPP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BNPP_VERSION 202   /* 200: single ops take n_cards (the length of cards); 201: sliced bucket-tree marginals;
                              202: single ops return the reference's partition sum (out_sum) */

enum bnpp_status {
    BNPP_OK = 0,
    BNPP_ERR_INVALID = -1,      /* bad shape / argument  (reference: throw const char*, assert) */
    BNPP_ERR_NO_DEVICE = -2,    /* no usable GPU */
    BNPP_ERR_OOM = -3,
    BNPP_ERR_HIP = -4,
    BNPP_ERR_IO = -5,           /* cannot open / parse a file (io.cpp:124, 150, 177: return -1/-2) */
    BNPP_ERR_UNSUPPORTED = -6
};

enum bnpp_dtype { BNPP_F64 = 0, BNPP_F32 = 1 };

/* elimination-order heuristics: bn flags -mf / -wmf / -md (bn.cpp:183-191) */
enum bnpp_heuristic { BNPP_ORDER_GIVEN = 0, BNPP_MIN_FILL = 1, BNPP_WEIGHTED_MIN_FILL = 2, BNPP_MIN_DEGREE = 3 };

const char *bnpp_strerror(int status);
const char *bnpp_last_error(void);
int bnpp_version(void);
/* 1 when the loaded library speaks the ABI this header declares.  Callers
 * check it once: a library of another version links (the symbol names are
 * unchanged) but would read shifted arguments. */
static inline int bnpp_abi_matches(void) { return bnpp_version() == BNPP_VERSION; }
/* Phase split (ms) of this thread's last bnpp_partition / bnpp_marginals /
 * bnpp_marginals_tree[_part] call -- the reference times these tasks as one
 * "uptime" (model.cpp:258/296, 309/343):
 *   out[0] ordering + planning + schedule (host)   out[1] source upload
 *   out[2] device program (arena, descriptors)     out[3] launch enqueue
 *   out[4] device run + result fetch                out[5] free
 *   out[6] total                                    out[7] 1 if the context's cached arena was reused
 *   out[8] of out[2]: the arena's hipMalloc (0 when reused) -- where a call
 *          waits for the driver to clear HBM that was freed shortly before
 *          (by any process: ~36 GB/s of backlog on MI355X)
 * Writes min(n, 9) values. */
int bnpp_last_timing(double *out, int n);

/* ------------------------------------------------------------- device */
typedef struct bnpp_ctx bnpp_ctx;

int bnpp_device_count(int *n);
int bnpp_ctx_create(int device, bnpp_ctx **out);
int bnpp_ctx_destroy(bnpp_ctx *ctx);
int bnpp_ctx_stream(bnpp_ctx *ctx, void **stream);
/* release the device memory the context keeps between calls (the cached arena
 * of the last partition / marginals call and the small-buffer cache) */
int bnpp_ctx_trim(bnpp_ctx *ctx);
int bnpp_malloc(bnpp_ctx *ctx, size_t bytes, void **dptr);
int bnpp_free(bnpp_ctx *ctx, void *dptr);
int bnpp_memcpy_h2d(bnpp_ctx *ctx, void *dst, const void *src, size_t bytes);
int bnpp_memcpy_d2h(bnpp_ctx *ctx, void *dst, const void *src, size_t bytes);
int bnpp_synchronize(bnpp_ctx *ctx, void *stream);

/* ------------------------------------------------- scope rules (host) */
/* Output scope of ((Factor(1.0) * in_0) * in_1) ... .sum_out(elim_var):
 * Domain(d1,d2) union order (domain.cpp:32-52) then Domain(d,v) removal
 * (domain.cpp:54-72).  elim_var < 0: pure product.  Writes *out_ndims ids. */
int bnpp_out_scope(int n_in, const int *in_ndims, const int *const *in_vars, int elim_var, int cap,
                   int *out_ndims, int *out_vars);

/* --------------------------------------------- single ops (device)
 * out_sum (every single op): NULL, or a DEVICE double that receives, when the
 * stream reaches it, the reference's running sum of the op (Factor::_partition,
 * factor.hh:26/47) with its bits: the op's terms added one at a time from 0.0
 * in fp64 in the reference's loop order -- product / divide / conditioning:
 * the output entries in linear order of the reference's output scope
 * (factor.cpp:129-139, 161-172, 226-236); sum_out and a fused bucket: the
 * INPUT (chain-product) entries in (output entry, summed value) order
 * (factor.cpp:196-208).  A sequential sum by definition (one wave, ~2e8
 * terms/s): ask for it only where the caller reads partition().  Single ops
 * compute the reference's unscaled values, so there is no log10 scale to
 * return (the VE entry points below carry theirs).  fp32 tables: the fp32
 * terms, widened, summed in fp64.  At most 32 output variables with out_sum
 * (BNPP_ERR_UNSUPPORTED otherwise, checked before the op is launched).  One
 * case the ABI cannot reproduce: Factor::sum_out of a variable NOT in the
 * scope returns a copy that keeps the input's STORED _partition
 * (factor.cpp:185-188), which may differ from the linear sum of its entries
 * (e.g. 1.0 after normalize); out_sum is always the linear sum -- a caller
 * that tracks _partition (the C++ mirror does) keeps its own value there. */
/* Fused bucket:  out = sum_{elim_var} prod_i in_i   — replaces the bucket body of
 * BN::variable_elimination (model.cpp:414-418):
 *     Factor prod(1.0); for (pf : bucket) prod *= *pf; prod.sum_out(var)
 * i.e. Factor::operator*= (factor.cpp:77-81) + Factor::product (factor.cpp:117-147)
 * + Factor::sum_out (factor.cpp:182-212) in one pass with no intermediate table.
 * fp64 results are bit-identical to that chain evaluated in input order.
 * out_vars must be the layout from bnpp_out_scope (or any permutation of it).
 * 1 <= n_in <= 8; elim_var < 0 means no summation; elim_var absent from every
 * input makes it a copy (factor.cpp:185-188). */
int bnpp_bucket_eliminate(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, int n_in,
                          const void *const *in_tables, const int *in_ndims, const int *const *in_vars,
                          int elim_var, void *out_table, int out_ndims, const int *out_vars, double *out_sum);

/* Factor::product (factor.cpp:117-147; factor.hh:35) */
int bnpp_product(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *a, int a_ndims,
                 const int *a_vars, const void *b, int b_ndims, const int *b_vars, void *out, int out_ndims,
                 const int *out_vars, double *out_sum);

/* Factor::divide (factor.cpp:149-180; factor.hh:36): out = a / b over the
 * union scope (out_vars: any order of it).  The reference asserts on a zero
 * divisor (factor.cpp:165); here it yields inf / nan in that entry. */
int bnpp_divide(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *a, int a_ndims,
                const int *a_vars, const void *b, int b_ndims, const int *b_vars, void *out, int out_ndims,
                const int *out_vars, double *out_sum);

/* Factor::sum_out (factor.cpp:182-212; factor.hh:34) */
int bnpp_sum_out(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *in, int ndims,
                 const int *vars, int var, void *out, int out_ndims, const int *out_vars, double *out_sum);

/* Factor::conditioning (factor.cpp:214-242; factor.hh:38): out scope = vars minus
 * evidence vars, order preserved (domain.cpp:74-90) */
int bnpp_condition(bnpp_ctx *ctx, void *stream, int dtype, int n_cards, const int *cards, const void *in, int ndims,
                   const int *vars, int n_ev, const int *ev_vars, const int *ev_vals, void *out, double *out_sum);

/* ------------------------------------------------------ models (host) */
typedef struct bnpp_model bnpp_model;

/* read_uai_model (io.cpp:102-154) without the BAYES/MARKOV split: both kinds load */
int bnpp_model_load_uai(const char *path, bnpp_model **out);
/* the same data from arrays: scopes concatenated, values concatenated (row-major) */
int bnpp_model_from_arrays(int is_bayes, int n_vars, const int *cards, int n_factors, const int *widths,
                           const int *scopes, const double *values, bnpp_model **out);
/* Frees the model; every live context also drops what it caches for it (its
 * uploaded sources and a cached one-shot job planned for it -- a context in the
 * middle of a call keeps its job until its next one-shot call replaces it).
 * The contexts' cached arena is not the model's and stays: bnpp_ctx_trim. */
int bnpp_model_free(bnpp_model *m);
int bnpp_model_info(const bnpp_model *m, int *is_bayes, int *n_vars, int *n_factors);
int bnpp_model_cards(const bnpp_model *m, int *cards);
/* read_uai_evidence (io.cpp:157-180): *n pairs (0 unless the first integer is 1) */
int bnpp_evidence_load(const char *path, int cap, int *n, int *vars, int *vals);

/* Graph::ordering (graph.cpp:41-101) over the graph of the evidence-conditioned
 * factors, as BN::variable_elimination builds it (model.cpp:360-369).
 * vars NULL: all non-evidence variables.  *width_out: induced width. */
int bnpp_ordering(const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals, int n_vars,
                  const int *vars, int heuristic, int *order_out, int *width_out);

/* ------------------------------------------------ inference (device) */
/* BN::partition (model.cpp:250-301), VE branch: conditioning + VE.  Messages are
 * kept resident in HBM and rescaled by exact powers of two, so Z is returned as
 * log10 (always finite unless Z == 0) and as a double (may overflow to inf, as
 * the reference's would).  order: explicit order (heuristic BNPP_ORDER_GIVEN),
 * NULL otherwise.  uptime_ms covers ordering + planning + device run, like the
 * reference's steady_clock scope (model.cpp:258/296). */
int bnpp_partition(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                   int heuristic, const int *order, int n_order, int dtype, double *log10_z, double *z,
                   double *uptime_ms);

/* BN::marginals (model.cpp:303-346), VE branch: one VE per target with every
 * other variable eliminated, then Factor::normalize (factor.cpp:244-255).  All
 * targets run as one batched device schedule.  targets NULL: all variables.
 * out receives sum(card[t]) values target-major; an evidence variable's marginal
 * is written one-hot (the UAI MAR format; the reference prints a width-0 factor). */
int bnpp_marginals(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                   int heuristic, int n_targets, const int *targets, int dtype, double *out, double *uptime_ms);

/* All marginals from ONE two-pass bucket tree (Shafer-Shenoy message passing
 * on the VE bucket tree of the partition's elimination order) instead of one VE
 * per target (model.cpp:326-334): about three VE passes of device work and one
 * host ordering, whatever the number of targets.  Same output as
 * bnpp_marginals (normalised, evidence one-hot); values agree with the
 * reference to rounding (not bit-exact: the sums are associated differently).
 * order: explicit elimination order covering every non-evidence variable
 * (heuristic BNPP_ORDER_GIVEN), or NULL.  BNPP_ERR_OOM when every forward
 * message cannot stay resident within the memory budget. */
int bnpp_marginals_tree(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                        int heuristic, const int *order, int n_order, int n_targets, const int *targets, int dtype,
                        double *out, double *uptime_ms);

/* One part of bnpp_marginals_tree for multi-GPU runs (one process per GPU,
 * part = rank, n_parts = world size): this part computes only the marginals it
 * owns (a contiguous segment of a chain-shaped bucket tree, else every
 * n_parts-th target) and writes zeros for the others; owned[i] (optional)
 * flags targets[i].  Summing `out` over the parts gives bnpp_marginals_tree's
 * output (one all-reduce, no other exchange). */
int bnpp_marginals_tree_part(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                             int heuristic, const int *order, int n_order, int n_targets, const int *targets,
                             int part, int n_parts, int dtype, double *out, int *owned, double *uptime_ms);

/* Message-sliced bucket-tree marginals for multi-GPU runs (no reference
 * counterpart: the reference is single-process; this replaces the N
 * independent VEs of BN::marginals, model.cpp:303-346, across N ranks).  Every
 * message of the chain-shaped bucket tree is split into n_ranks blocks by
 * log2(n_ranks) binary variables that stay in the separators for a window of
 * the chain; rank r holds and computes the block whose slice variables read r
 * (slowest first), and between windows a message is re-sliced by one
 * all-to-all through `coll` (at the chain's ends an all-gather).  n_ranks: a
 * power of two >= 2; every rank calls this with the same model, evidence,
 * order, targets and budget_gb (> 0: the device memory in GB the plan must
 * fit, which sets its checkpoint count -- it must agree across ranks, e.g. the
 * smallest free memory; <= 0: this device's).  The collective is called synchronously from this
 * thread, in the same sequence on every rank (two-lane schedules: the lanes'
 * windows alternately, each lane on its own stream), and must be complete (or
 * enqueued on `stream`) when it returns:
 *   op BNPP_COLL_ALLGATHER: each rank contributes `bytes` at send; recv gets
 *                           rank r's at recv + r * bytes
 *   op BNPP_COLL_ALLTOALL:  send holds n_ranks blocks of `bytes`, block d for
 *                           rank d; recv gets rank s's block at recv + s * bytes
 * Output: this rank's share of each target's unnormalised marginal, as
 * mantissas (out, sum(card) doubles) times 2^out_exp2[i] per target
 * (out_exp2 = -2^40 for an all-zero share); the marginal is the normalised sum
 * of the shares over the ranks (bnpp.dist.sliced_tree_marginals).  Trees that
 * are not chains, or chains without such windows: BNPP_ERR_UNSUPPORTED.  As
 * bnpp_marginals_tree, the planned job stays with the context, and an
 * identical call (same model, evidence, order, targets, dtype, rank, n_ranks
 * and budget) relaunches it; coll / user are bound per call. */
#define BNPP_COLL_ALLGATHER 0
#define BNPP_COLL_ALLTOALL 1
typedef int (*bnpp_collective_fn)(void *user, int op, const void *send, void *recv, int64_t bytes, void *stream);
int bnpp_marginals_tree_sliced(bnpp_ctx *ctx, const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                               int heuristic, const int *order, int n_order, int n_targets, const int *targets,
                               int rank, int n_ranks, bnpp_collective_fn coll, void *user, double budget_gb,
                               int dtype, double *out, int64_t *out_exp2, double *uptime_ms);
/* A collective for one GPU (user: const int[4] = {n_ranks, flags, link MB/s,
 * latency us}): every received block is a copy of the sent one -- a world of
 * identical ranks, for timing one rank's share of a sliced run (the data it
 * computes is not a real world's); flags & 1: nothing is copied (the compute
 * alone); flags & 2: the calling stream waits the transfer's modelled time,
 * latency + bytes sent / (min(n_ranks - 1, 7) links x MB/s). */
int bnpp_collective_loopback(void *user, int op, const void *send, void *recv, int64_t bytes, void *stream);

/* BN::marginals with options["sum-product"] (model.cpp:313-317; the `bn -sp`
 * flag): loopy BP on the factor graph of the model's factors,
 * FactorGraph::update(max_iter, eps) (graph.cpp:298-332; the reference uses
 * 10000, 0.001, model.cpp:749) then FactorGraph::marginal per variable
 * (graph.cpp:393-403).  Evidence is not used, as in the reference.  fp64.
 * out: sum(card) values, var-major; *iterations = update's return value
 * (max_iter when it did not converge).  Small models run in one workgroup,
 * larger ones (or any factor table of 2^31+ entries, indexed in 64 bits) as a
 * multi-workgroup flood (BNPP_BP_MODE=single|multi forces either). */
int bnpp_sum_product(bnpp_ctx *ctx, const bnpp_model *m, int max_iter, double eps, double *out, int *iterations,
                     double *uptime_ms);

/* BN::variable_elimination (model.cpp:348-446) over the factors of `m` taken
 * as given (already conditioned by the caller): eliminates `vars` (heuristic
 * order, or exactly this order with BNPP_ORDER_GIVEN) and returns the result
 * factor: *out_ndims scope ids in out_vars (reference chain order), *out_size
 * values in out_values, scaled: true value = out_values[i] * 2^(*exp2). */
int bnpp_variable_elimination(bnpp_ctx *ctx, const bnpp_model *m, int n_vars, const int *vars, int heuristic,
                              int dtype, int cap_vars, int *out_ndims, int *out_vars, int64_t cap_values,
                              int64_t *out_size, double *out_values, int64_t *exp2);

/* Host-only planning statistics (no device needed): kind 0 partition (explicit
 * order if `order` is non-NULL), 1 marginals of all variables (one VE each),
 * 3 bucket-tree marginals of all variables.  stats as
 * bnpp_job_stats. */
int bnpp_plan_stats(const bnpp_model *m, int kind, int n_ev, const int *ev_vars, const int *ev_vals, int heuristic,
                    const int *order, int n_order, int dtype, double *stats, int n_stats);

/* Host-only planning of one part of bnpp_marginals_tree_part (all variables
 * as targets): owned[v] = 1 when this part computes v's marginal; stats as
 * bnpp_job_stats for this part's plan (may be NULL).  The memory budget is
 * BNPP_MEM_BUDGET_GB or 64 GB (no device is consulted). */
int bnpp_plan_tree_part(const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals, int heuristic,
                        const int *order, int n_order, int part, int n_parts, int dtype, int *owned, double *stats,
                        int n_stats);

/* Host-only planning of one rank of bnpp_marginals_tree_sliced (all
 * variables as targets): slice_bit[v] (may be NULL) = the rank bit that
 * indexes v's scalar share (-1: a table over v); stats as bnpp_job_stats, then
 * [8] message exchanges, [9] bytes this rank sends per call. */
int bnpp_plan_tree_sliced(const bnpp_model *m, int n_ev, const int *ev_vars, const int *ev_vals, int heuristic,
                          const int *order, int n_order, int rank, int n_ranks, int dtype, int *slice_bit,
                          double *stats, int n_stats);

/* ------------------------------------------- prepared jobs (benchmark) */
/* A planned, device-resident inference that can be launched repeatedly. */
typedef struct bnpp_job bnpp_job;
/* kind 0: partition (targets ignored)   kind 1: marginals of `targets` (one VE
 * each)   kind 3: marginals of `targets` from one bucket tree */
int bnpp_job_create(bnpp_ctx *ctx, const bnpp_model *m, int kind, int n_ev, const int *ev_vars,
                    const int *ev_vals, int heuristic, const int *order, int n_order, int n_targets,
                    const int *targets, int dtype, bnpp_job **out);
/* stats: [0] factor-entries per launch, [1] arena bytes, [2] levels, [3] buckets,
 *        [4] max induced width, [5] largest message entries, [6] algorithmic bytes,
 *        [7] target batches */
int bnpp_job_stats(const bnpp_job *job, double *stats, int n_stats);
int bnpp_job_launch(bnpp_job *job, void *stream);
/* waits on stream; partition: out[0] = log10 Z; marginals: sum(card) values */
int bnpp_job_results(bnpp_job *job, void *stream, double *out);
int bnpp_job_free(bnpp_job *job);

#ifdef __cplusplus
}
#endif
#endif
