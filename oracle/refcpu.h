/*
 * refcpu — CPU restatement of bn-pp's variable-elimination hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle and the "port" CPU
 * baseline.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product library (bn-pp_amd/) never links it.
 *
 * Pinning: checked against the reference's own fixtures
 * (models/markovnets/{grid3x3,network}.uai.{PR,MAR}) and against golden
 * vectors produced by the reference itself, compiled from
 * /root/reference/code by oracle/Makefile into oracle/_ref/ and driven by
 * oracle/ref_harness.cpp (tests/golden/make_golden.py).
 *
 * Restated reference semantics (file:line into /root/reference/code):
 *   layout      row-major over the scope, last variable fastest   domain.cpp:15-26
 *   union scope d1 order, then d2 vars not in d1 (d2 order)        domain.cpp:32-52
 *   remove var  order preserved                                    domain.cpp:54-72
 *   evidence    drop evidence vars, order preserved                domain.cpp:74-90
 *   odometer    next_valuation (last digit fastest)                domain.cpp:113-123
 *   positions   position_consistent_valuation 2-/4-arg             domain.cpp:162-190
 *   product     per-entry odometer walk, sequential partition sum  factor.cpp:117-147
 *   sum_out     for i, for val: out[i] += in[pos]; copy if absent  factor.cpp:182-212
 *   condition   evidence slice                                     factor.cpp:214-242
 *   normalize   values / partition                                 factor.cpp:244-255
 *   divide      as product with '/'                                factor.cpp:149-180
 *   VE          bucket elimination                                 model.cpp:348-446
 *   PR / MAR    conditioning + VE (+ normalize)                    model.cpp:250-346
 *   ordering    min-fill / weighted-min-fill / min-degree          graph.cpp:41-195
 *   UAI I/O     token reader, '#' comments, evidence               io.cpp:14-180
 *   loopy BP    flooding sum-product, relative-change stop         graph.cpp:256-403
 *
 * Deliberate, documented deviations (none changes a value beyond fp
 * rounding of >=3-factor chains):
 *   - bucket contents are iterated in insertion order; the reference iterates
 *     an unordered_set<const Factor*> (pointer-hash order, model.cpp:385,415);
 *   - heuristic ties are broken by ascending variable id; the reference
 *     iterates an unordered_set<unsigned> (graph.cpp:50-58,109,128);
 *   - sizes are 64-bit (reference: 32-bit unsigned, domain.hh:21-22);
 *   - a variable absent from the moral graph has no neighbours (the
 *     reference dereferences end(), graph.hh:18 — the -mar -mf crash).
 */
#ifndef BNPP_ORACLE_REFCPU_H
#define BNPP_ORACLE_REFCPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rc_factor {
    int width;
    int *vars;          /* variable ids, scope order */
    int *cards;         /* cardinality per scope position */
    uint64_t size;
    double *values;
    double partition;   /* sequential fp64 sum of values (factor.hh:47) */
} rc_factor;

typedef struct rc_model {
    int is_bayes;
    int n_vars;
    int *cards;
    int n_factors;
    rc_factor **factors;
} rc_model;

enum { RC_ORDER_GIVEN = 0, RC_MIN_FILL = 1, RC_WEIGHTED_MIN_FILL = 2, RC_MIN_DEGREE = 3 };

/* factor algebra */
rc_factor *rc_factor_new(int width, const int *vars, const int *cards, const double *values);
rc_factor *rc_factor_copy(const rc_factor *f);
void rc_factor_free(rc_factor *f);
int rc_factor_width(const rc_factor *f);
uint64_t rc_factor_size(const rc_factor *f);
void rc_factor_scope(const rc_factor *f, int *vars_out);
void rc_factor_values(const rc_factor *f, double *out);
double rc_factor_partition(const rc_factor *f);

rc_factor *rc_product(const rc_factor *a, const rc_factor *b);
rc_factor *rc_divide(const rc_factor *a, const rc_factor *b);
rc_factor *rc_sum_out(const rc_factor *f, int var, int card);
rc_factor *rc_conditioning(const rc_factor *f, int n_ev, const int *ev_vars, const int *ev_vals);
rc_factor *rc_normalize(const rc_factor *f);
/* one bucket of model.cpp:414-418: ((1 * f_1) * f_2) ... * f_m, then sum_out(var) */
rc_factor *rc_bucket(int n_in, const rc_factor *const *in, int var, int card);

/* model + I/O */
rc_model *rc_model_load_uai(const char *path);
rc_model *rc_model_new(int is_bayes, int n_vars, const int *cards, int n_factors,
                       const int *widths, const int *scopes, const double *values);
void rc_model_free(rc_model *m);
int rc_model_n_vars(const rc_model *m);
int rc_model_n_factors(const rc_model *m);
int rc_model_card(const rc_model *m, int v);
/* returns number of evidence pairs (0 if the sample count is not 1), -1 on error */
int rc_load_evidence(const char *path, int cap, int *vars, int *vals);

/* heuristic ordering of `vars` over the graph of `factors` (graph.cpp:41-101) */
int rc_ordering(const rc_model *m, int n_factors, const rc_factor *const *factors,
                int n_vars, const int *vars, int heuristic, int *order_out);
int rc_order_width(const rc_model *m, int n_factors, const rc_factor *const *factors,
                   int n_vars, const int *order);

/* VE over an explicit or heuristic order (model.cpp:348-446) */
rc_factor *rc_variable_elimination(const rc_model *m, int n_vars, const int *vars,
                                   int n_factors, const rc_factor *const *factors, int heuristic);
/* BN::partition (model.cpp:250-301): returns Z; *uptime_ms like the reference */
double rc_partition(const rc_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                    int heuristic, double *uptime_ms);
/* BN::marginals (model.cpp:303-346): writes sum(card) values, var-major */
int rc_marginals(const rc_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                 int heuristic, double *out, double *uptime_ms);
/* marginal of one variable (one VE of the MAR loop, model.cpp:326-334) */
int rc_marginal_one(const rc_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                    int heuristic, int target, double *out);

/* loopy BP, BN::sum_product + FactorGraph::marginal (model.cpp:313-317,
   736-753; graph.cpp:256-403); evidence is not used on this path.  Writes
   sum(card) values, var-major; *iterations = FactorGraph::update's result */
int rc_sum_product(const rc_model *m, int max_iter, double eps, double *out, int *iterations, double *uptime_ms);

/* bucket micro-benchmark: m(x,S_1..S_w)*f(x,y) -> sum_x, all cards = k.
   Returns factor-entries processed per second (k^(w+2) / seconds), fp64. */
double rc_micro_bucket(int k, int w, int reps, double *seconds_out);

#ifdef __cplusplus
}
#endif
#endif
