// Runs the reference's single-op known-answer cases through the C++ class
// mirror (include/bnpp/bn.hpp): Factor::product / sum_out / conditioning /
// divide on the device, partition() computed on first read.  Reads cases on
// stdin (written by tests/test_cpp_mirror.py from tests/golden/kat_golden.json),
// prints per case "scope ids | values %.17g | partition %.17g" (test code).
//   input:  CARDS n c_0 .. c_{n-1}
//           then per case: OP name / A w ids.. n vals.. / [B ...] / [VAR id] / [EV n (id val)..] / END
#include <cstdio>
#include <iostream>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "bnpp/bn.hpp"

using namespace bn;

static std::vector<std::unique_ptr<Variable>> vars;

static Factor read_factor(std::istream &in) {
    unsigned w;
    in >> w;
    std::vector<const Variable *> scope(w);
    for (unsigned i = 0; i < w; ++i) {
        unsigned id;
        in >> id;
        scope[i] = vars[id].get();
    }
    size_t n;
    in >> n;
    std::vector<double> v(n);
    double p = 0;
    for (size_t i = 0; i < n; ++i) {
        in >> v[i];
        p += v[i];
    }
    return Factor(new Domain(scope), v, p);
}

int main() {
    std::string tok;
    std::cin >> tok;                                 // CARDS
    unsigned n;
    std::cin >> n;
    for (unsigned i = 0; i < n; ++i) {
        unsigned c;
        std::cin >> c;
        vars.emplace_back(new Variable(i, c));
    }
    std::cout.precision(17);
    while (std::cin >> tok) {                        // OP
        std::string op;
        std::cin >> op;
        std::unique_ptr<Factor> a, b;
        int var = -1;
        std::unordered_map<unsigned, unsigned> ev;
        while (std::cin >> tok && tok != "END") {
            if (tok == "A") a.reset(new Factor(read_factor(std::cin)));
            else if (tok == "B") b.reset(new Factor(read_factor(std::cin)));
            else if (tok == "VAR") std::cin >> var;
            else if (tok == "EV") {
                unsigned k;
                std::cin >> k;
                for (unsigned i = 0; i < k; ++i) {
                    unsigned id, val;
                    std::cin >> id >> val;
                    ev[id] = val;
                }
            }
        }
        Factor r = op == "product" ? a->product(*b)
                 : op == "divide"  ? a->divide(*b)
                 : op == "sum_out" ? a->sum_out(vars[var].get())
                                   : a->conditioning(ev);
        const Factor &c = r;                         // const reads: the partition stays pending until asked
        for (const Variable *x : c.domain().scope()) std::printf("%u ", x->id());
        std::printf("|");
        for (double x : c.values()) std::printf(" %.17g", x);
        std::printf(" | %.17g\n", c.partition());
    }
    return 0;
}
