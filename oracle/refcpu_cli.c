/* refcpu_cli — command-line front end of the CPU restatement (test infrastructure).
 *   pr    <uai> <evid|-> <given|mf|wmf|md>
 *   mar   <uai> <evid|-> <given|mf|wmf|md>
 *   width <uai> <mf|wmf|md>
 *   micro <k> <w> <reps>
 * Output lines match oracle/ref_harness so the two can be diffed. */
#include "refcpu.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int heur(const char *s) {
    if (!strcmp(s, "mf")) return RC_MIN_FILL;
    if (!strcmp(s, "wmf")) return RC_WEIGHTED_MIN_FILL;
    if (!strcmp(s, "md")) return RC_MIN_DEGREE;
    return RC_ORDER_GIVEN;
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: refcpu_cli pr|mar|width|micro ...\n"); return 1; }
    static int ev_vars[1 << 16], ev_vals[1 << 16];
    if ((!strcmp(argv[1], "pr") || !strcmp(argv[1], "mar")) && argc >= 5) {
        rc_model *m = rc_model_load_uai(argv[2]);
        if (!m) { fprintf(stderr, "cannot load %s\n", argv[2]); return 2; }
        int n_ev = strcmp(argv[3], "-") ? rc_load_evidence(argv[3], 1 << 16, ev_vars, ev_vals) : 0;
        if (n_ev < 0) return 3;
        double up = 0;
        if (!strcmp(argv[1], "pr")) {
            double z = rc_partition(m, n_ev, ev_vars, ev_vals, heur(argv[4]), &up);
            printf("Z %.17g\nlog10Z %.17g\nuptime_ms %.6f\n", z, log10(z), up);
        } else {
            size_t tot = 0;
            for (int v = 0; v < m->n_vars; ++v) tot += (size_t)m->cards[v];
            double *out = (double *)malloc(sizeof(double) * tot);
            rc_marginals(m, n_ev, ev_vars, ev_vals, heur(argv[4]), out, &up);
            size_t o = 0;
            for (int v = 0; v < m->n_vars; ++v) {
                printf("M%d", v);
                for (int s = 0; s < m->cards[v]; ++s) printf(" %.17g", out[o + s]);
                printf("\n");
                o += (size_t)m->cards[v];
            }
            printf("uptime_ms %.6f\n", up);
            free(out);
        }
        rc_model_free(m);
        return 0;
    }
    if (!strcmp(argv[1], "width") && argc >= 4) {
        rc_model *m = rc_model_load_uai(argv[2]);
        if (!m) return 2;
        int *vars = (int *)malloc(sizeof(int) * (size_t)m->n_vars), *order = (int *)malloc(sizeof(int) * (size_t)m->n_vars);
        for (int v = 0; v < m->n_vars; ++v) vars[v] = v;
        int w = rc_ordering(m, m->n_factors, (const rc_factor *const *)m->factors, m->n_vars, vars, heur(argv[3]), order);
        printf("width %d\norder", w);
        for (int i = 0; i < m->n_vars; ++i) printf(" %d", order[i]);
        printf("\n");
        free(vars); free(order);
        rc_model_free(m);
        return 0;
    }
    if (!strcmp(argv[1], "micro") && argc >= 5) {
        double sec = 0;
        double eps = rc_micro_bucket(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), &sec);
        printf("entries_per_s %.6g\nseconds %.6f\n", eps, sec);
        return 0;
    }
    fprintf(stderr, "bad command\n");
    return 1;
}
