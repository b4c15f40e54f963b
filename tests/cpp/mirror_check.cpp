// Exercises the C++ class mirror (include/bnpp/bn.hpp) the way INTEGRATION.md
// shows a bn-pp caller using it.  Device results are checked against plain
// loops written here (test code, not a product path).  Prints "OK" and exits 0
// on success.  Usage: mirror_check <models dir>
#include <cmath>
#include <cstdio>
#include <iostream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "bnpp/bn.hpp"

using namespace bn;

static int fails = 0;
#define CHECK(c) do { if (!(c)) { std::fprintf(stderr, "FAIL line %d: %s\n", __LINE__, #c); ++fails; } } while (0)

int main(int argc, char **argv) {
    std::string dir = argc > 1 ? argv[1] : "tests/golden/models";
    // Factor::product / sum_out against explicit loops: f(a,b) * g(b,c), sum over b
    Variable a(0, 2), b(1, 3), c(2, 2);
    std::vector<double> fv{1, 2, 3, 4, 5, 6}, gv{0.5, 1.5, 2.5, 3.5, 4.5, 5.5};
    Factor f(new Domain({&a, &b}), fv, 21.0), g(new Domain({&b, &c}), gv, 18.0);
    Factor p = f.product(g);                         // scope (a, b, c), c fastest
    CHECK(p.width() == 3 && p.size() == 12);
    for (unsigned ia = 0; ia < 2; ++ia)
        for (unsigned ib = 0; ib < 3; ++ib)
            for (unsigned ic = 0; ic < 2; ++ic) CHECK(p[(ia * 3 + ib) * 2 + ic] == fv[ia * 3 + ib] * gv[ib * 2 + ic]);
    Factor s = p.sum_out(&b);                        // scope (a, c)
    CHECK(s.width() == 2 && s.size() == 4);
    for (unsigned ia = 0; ia < 2; ++ia)
        for (unsigned ic = 0; ic < 2; ++ic) {
            double want = 0;
            for (unsigned ib = 0; ib < 3; ++ib) want += fv[ia * 3 + ib] * gv[ib * 2 + ic];
            CHECK(s[ia * 2 + ic] == want);
        }
    Factor prod(1.0);                                // bucket chain Factor(1.0) *= f_i (model.cpp:414-417)
    prod *= f;
    prod *= g;
    CHECK(prod.values() == p.values());
    // sum_out's partition(): the input's terms in (output entry, summed value)
    // order (factor.cpp:196-208), for an input summed lazily (small) and one
    // summed at once (2^23 entries, past the mirror's lazy-copy limit)
    for (unsigned big : {0u, 1u}) {
        const unsigned nx = 3, ny = big ? 2048 : 5, nz = big ? 1366 : 7;
        Variable x(0, nx), y(1, ny), z(2, nz);
        std::vector<double> hv((size_t)nx * ny * nz);
        for (size_t i = 0; i < hv.size(); ++i) hv[i] = 0.25 + (double)((i * 2654435761u) % 1000) * 1e-3;
        Factor h(new Domain({&x, &y, &z}), hv, 0.0);
        Factor hs = h.sum_out(&y);                   // scope (x, z)
        double want = 0;
        for (unsigned ix = 0; ix < nx; ++ix)
            for (unsigned iz = 0; iz < nz; ++iz)
                for (unsigned iy = 0; iy < ny; ++iy) want += hv[((size_t)ix * ny + iy) * nz + iz];
        CHECK(hs.partition() == want);
        CHECK(hs.size() == (size_t)nx * nz);
    }

    // BN::partition / marginals on the reference's grid3x3 fixtures
    std::string path = dir + "/grid3x3.uai", ev_pr = dir + "/grid3x3-PR.uai.evid", ev_mar = dir + "/grid3x3-MAR.uai.evid";
    MN *mn = nullptr;
    CHECK(read_uai_model(path, &mn) == 0);
    std::unordered_map<unsigned, unsigned> ev;
    CHECK(read_uai_evidence(ev_pr, ev) == 0);
    std::unordered_map<std::string, bool> options{{"min-fill", true}};
    double up = 0;
    double lz = mn->log10_partition(ev, options, up);
    CHECK(std::fabs(lz - 14.8899) < 5e-5);          // grid3x3.uai.PR
    ev.clear();
    CHECK(read_uai_evidence(ev_mar, ev) == 0);
    std::vector<const Factor *> m1 = mn->marginals(ev, options, up);
    options["bucket-tree"] = true;
    std::vector<const Factor *> m2 = mn->marginals(ev, options, up);
    CHECK(m1.size() == 9 && m2.size() == 9);
    for (size_t i = 0; i < m1.size() && i < m2.size(); ++i) {
        CHECK(m1[i]->size() == m2[i]->size());
        for (uint64_t j = 0; j < m1[i]->size() && j < m2[i]->size(); ++j)
            CHECK(std::fabs((*m1[i])[j] - (*m2[i])[j]) < 1e-12);
        delete m1[i];
        delete m2[i];
    }
    delete mn;

    // Factor::divide (factor.cpp:149-180) against the explicit loop: scope (a, b, c)
    Factor q = p.divide(g);
    CHECK(q.width() == 3 && q.size() == 12);
    for (unsigned ia = 0; ia < 2; ++ia)
        for (unsigned ib = 0; ib < 3; ++ib)
            for (unsigned ic = 0; ic < 2; ++ic)
                CHECK(q[(ia * 3 + ib) * 2 + ic] == p[(ia * 3 + ib) * 2 + ic] / gv[ib * 2 + ic]);

    // BN::query_ve (model.cpp:205-248) on asia: P(t | e) as a table over (t, e);
    // each column e = v equals the marginal of t under evidence {e: v}
    std::string asia = dir + "/asia.uai";
    BN *bn = nullptr;
    CHECK(read_uai_model(asia, &bn) == 0);
    if (bn) {
        const std::vector<Variable *> &vs = bn->variables();
        const Variable *t = vs[1], *e = vs[5];
        std::unordered_set<const Variable *> target{t}, evidence{e};
        std::unordered_map<std::string, bool> opt{{"min-fill", true}};
        Factor qv = bn->query_ve(target, evidence, opt, up);
        CHECK(qv.width() == 2 && qv.size() == t->size() * e->size());
        const bool t_first = qv.domain()[0] == t;
        for (unsigned v = 0; v < e->size(); ++v) {
            std::unordered_map<unsigned, unsigned> evv{{e->id(), v}};
            std::vector<const Factor *> mv = bn->marginals(evv, opt, up);
            double colsum = 0;
            for (unsigned x = 0; x < t->size(); ++x) {
                double got = t_first ? qv[x * e->size() + v] : qv[v * t->size() + x];
                colsum += got;
                CHECK(std::fabs(got - (*mv[t->id()])[x]) < 1e-12);
            }
            CHECK(std::fabs(colsum - 1.0) < 1e-12);
            for (auto m : mv) delete m;
        }
        delete bn;
    }
    if (fails) return 1;
    std::cout << "OK" << std::endl;
    return 0;
}
