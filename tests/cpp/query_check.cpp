// query_check — BN::query_ve (model.cpp:204-248) through the C++ class mirror
// (include/bnpp/bn.hpp) for every `query T | E` line of a query file (the
// reference REPL's syntax, bn.cpp:263).  Prints each result like
// oracle/ref_harness `query` ("Q<i> w ids.. | size partition | values..") so
// tests/test_cpp_mirror.py can compare them with the reference's answers.
//   query_check <model.uai> <queryfile> [mf|wmf|md|given]
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "bnpp.h"
#include "bnpp/bn.hpp"

using namespace bn;

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: query_check model.uai queryfile [mf|wmf|md|given]\n");
        return 1;
    }
    if (!bnpp_abi_matches()) {
        std::fprintf(stderr, "libbnpp ABI version differs from include/bnpp.h\n");
        return 1;
    }
    std::string path = argv[1], h = argc > 3 ? argv[3] : "mf";
    BN *m = nullptr;
    if (read_uai_model(path, &m)) return 2;
    std::unordered_map<std::string, bool> opt{{"min-fill", h == "mf"}, {"weighted-min-fill", h == "wmf"},
                                              {"min-degree", h == "md"}, {"variable-elimination", true}};
    auto ids = [&](std::string s) {
        std::unordered_set<const Variable *> out;
        for (char &c : s)
            if (c == ',') c = ' ';
        std::istringstream ss(s);
        unsigned id;
        while (ss >> id) out.insert(m->variables().at(id));
        return out;
    };
    std::ifstream in(argv[2]);
    std::string line;
    int qi = 0;
    while (std::getline(in, line)) {
        if (line.compare(0, 6, "query ") != 0) continue;
        std::string body = line.substr(6), t = body, e;
        const size_t bar = body.find('|');
        if (bar != std::string::npos) {
            t = body.substr(0, bar);
            e = body.substr(bar + 1);
        }
        double up = 0;
        Factor q = m->query_ve(ids(t), ids(e), opt, up);
        std::printf("Q%d %u", qi++, q.width());
        for (unsigned i = 0; i < q.width(); ++i) std::printf(" %u", q.domain()[i]->id());
        std::printf(" | %llu %.17g |", (unsigned long long)q.size(), q.partition());
        for (uint64_t i = 0; i < q.size(); ++i) std::printf(" %.17g", q[i]);
        std::printf("\n");
    }
    delete m;
    return 0;
}
