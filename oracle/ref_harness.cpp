// ref_harness — drives the REFERENCE bn-pp implementation (compiled from
// /root/reference/code by oracle/Makefile into oracle/_ref/) to produce golden
// vectors and CPU-baseline timings.  TEST INFRASTRUCTURE ONLY.
//
// This file contains no reference code: it only calls the reference's public
// classes (Variable, Domain, Factor, BN) and the UAI reader functions that
// have external linkage in io.cpp:43-100 but are not declared in io.hh.
//
//   pr    <uai> <evid|-> <given|mf|wmf|md>     BN::partition (model.cpp:250)
//   mar   <uai> <evid|-> <given|mf|wmf|md> [t..] per-target BN::variable_elimination
//                                              + normalize (model.cpp:326-334),
//                                              evidence vars left out of the order
//                                              (dodges the -mar -mf crash);
//                                              optional target ids: only those
//   ve    <uai> <evid|-> v1 v2 ...             VE with an explicit order
//   width <uai> <mf|wmf|md>                    Graph::ordering induced width
//   kat   <opfile>                             single Factor ops (product, sum_out, ...)
//   micro <k> <w> <reps>                       m(x,S)*f(x,y) -> sum_x, timed
//   sp    <uai> [max] [eps]                    loopy BP (FactorGraph, graph.cpp:256-403)
//   query <uai> <given|mf|wmf|md> <queryfile>  BN::query_ve (model.cpp:204-248) for every
//                                              `query T | E` line (REPL syntax, bn.cpp:263)
#include "variable.hh"
#include "domain.hh"
#include "factor.hh"
#include "model.hh"
#include "graph.hh"
#include "io.hh"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace bn {
std::string read_file_header(std::ifstream &input_file);
void read_variables(std::ifstream &input_file, std::vector<Variable *> &variables);
void read_factors(std::ifstream &input_file, std::vector<Variable *> &variables, std::vector<Factor *> &factors);
}  // namespace bn

using namespace bn;

static BN *load(const std::string &path) {
    std::ifstream in(path);
    if (!in.is_open()) { std::fprintf(stderr, "cannot open %s\n", path.c_str()); std::exit(2); }
    std::vector<Variable *> vars;
    std::vector<Factor *> factors;
    read_file_header(in);
    read_variables(in, vars);
    read_factors(in, vars, factors);
    return new BN(path, vars, factors);
}

static std::unordered_map<unsigned, unsigned> load_ev(const std::string &path) {
    std::unordered_map<unsigned, unsigned> ev;
    if (path != "-") {
        std::string p = path;
        if (read_uai_evidence(p, ev)) std::exit(3);
    }
    return ev;
}

static std::unordered_map<std::string, bool> opts_for(const std::string &h) {
    std::unordered_map<std::string, bool> o;
    o["min-fill"] = h == "mf";
    o["weighted-min-fill"] = h == "wmf";
    o["min-degree"] = h == "md";
    o["verbose"] = false;
    return o;
}

static void print_factor(const char *tag, const Factor &f) {
    std::printf("%s %u", tag, f.width());
    for (unsigned i = 0; i < f.width(); ++i) std::printf(" %u", f.domain()[i]->id());
    std::printf(" | %u %.17g |", f.size(), f.partition());
    for (unsigned i = 0; i < f.size(); ++i) std::printf(" %.17g", f[i]);
    std::printf("\n");
}

int main(int argc, char **argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: ref_harness pr|mar|ve|width|kat|micro ...\n"); return 1; }
    std::string cmd = argv[1];
    if (cmd == "pr" && argc >= 5) {
        BN *m = load(argv[2]);
        auto ev = load_ev(argv[3]);
        auto o = opts_for(argv[4]);
        double up = 0;
        double p = m->partition(ev, o, up);
        std::printf("Z %.17g\nlog10Z %.17g\nuptime_ms %.6f\n", p, std::log10(p), up);
        delete m;
        return 0;
    }
    if (cmd == "mar" && argc >= 5) {
        BN *m = load(argv[2]);
        auto ev = load_ev(argv[3]);
        auto o = opts_for(argv[4]);
        auto t0 = std::chrono::steady_clock::now();
        std::vector<const Factor *> fs;
        for (auto pf : m->factors()) fs.push_back(new Factor(pf->conditioning(ev)));
        std::vector<const Variable *> targets;
        for (int i = 5; i < argc; ++i) targets.push_back(m->variables().at(std::atoi(argv[i])));
        if (targets.empty()) targets.assign(m->variables().begin(), m->variables().end());
        for (auto pv : targets) {
            std::vector<const Variable *> vars;
            for (auto pv2 : m->variables())
                if (pv2 != pv && !ev.count(pv2->id())) vars.push_back(pv2);
            Factor r = m->variable_elimination(vars, fs, o).normalize();
            char tag[32];
            std::snprintf(tag, sizeof tag, "M%u", pv->id());
            print_factor(tag, r);
        }
        auto t1 = std::chrono::steady_clock::now();
        std::printf("uptime_ms %.6f\n", std::chrono::duration<double, std::milli>(t1 - t0).count());
        for (auto pf : fs) delete pf;
        delete m;
        return 0;
    }
    if (cmd == "ve" && argc >= 4) {
        BN *m = load(argv[2]);
        auto ev = load_ev(argv[3]);
        std::vector<const Variable *> vars;
        for (int i = 4; i < argc; ++i) vars.push_back(m->variables().at(std::atoi(argv[i])));
        std::vector<const Factor *> fs;
        for (auto pf : m->factors()) fs.push_back(new Factor(pf->conditioning(ev)));
        auto o = opts_for("given");
        Factor r = m->variable_elimination(vars, fs, o);
        print_factor("R", r);
        for (auto pf : fs) delete pf;
        delete m;
        return 0;
    }
    if (cmd == "width" && argc >= 4) {
        BN *m = load(argv[2]);
        auto o = opts_for(argv[3]);
        std::vector<const Variable *> mv(m->variables().begin(), m->variables().end());
        std::vector<const Factor *> fs(m->factors().begin(), m->factors().end());
        Graph g(mv, fs);
        unsigned w = 0;
        std::vector<unsigned> ids = g.ordering(mv, w, o);
        std::printf("width %u\norder", w);
        for (auto id : ids) std::printf(" %u", id);
        std::printf("\n");
        delete m;
        return 0;
    }
    if (cmd == "kat" && argc >= 3) {
        // opfile lines:
        //   var <id> <card>
        //   factor <name> <width> <ids...> <values...>
        //   product <out> <a> <b> | divide <out> <a> <b> | sum_out <out> <a> <var>
        //   cond <out> <a> <n> <id val>... | normalize <out> <a> | print <name>
        std::ifstream in(argv[2]);
        std::map<unsigned, Variable *> vars;
        std::map<std::string, Factor *> fs;
        std::string line;
        while (std::getline(in, line)) {
            std::istringstream ss(line);
            std::string op;
            if (!(ss >> op)) continue;
            if (op == "var") {
                unsigned id, card;
                ss >> id >> card;
                vars[id] = new Variable(id, card);
            } else if (op == "factor") {
                std::string name;
                unsigned w;
                ss >> name >> w;
                std::vector<const Variable *> scope;
                for (unsigned i = 0; i < w; ++i) { unsigned id; ss >> id; scope.push_back(vars.at(id)); }
                Domain *d = new Domain(scope);
                std::vector<double> vals(d->size());
                double p = 0;
                for (auto &v : vals) { ss >> v; p += v; }
                fs[name] = new Factor(d, vals, p);
            } else if (op == "product" || op == "divide") {
                std::string out, a, b;
                ss >> out >> a >> b;
                Factor r = op == "product" ? fs.at(a)->product(*fs.at(b)) : fs.at(a)->divide(*fs.at(b));
                fs[out] = new Factor(r);
            } else if (op == "sum_out") {
                std::string out, a;
                unsigned id;
                ss >> out >> a >> id;
                fs[out] = new Factor(fs.at(a)->sum_out(vars.at(id)));
            } else if (op == "cond") {
                std::string out, a;
                unsigned n;
                ss >> out >> a >> n;
                std::unordered_map<unsigned, unsigned> ev;
                for (unsigned i = 0; i < n; ++i) { unsigned id, val; ss >> id >> val; ev[id] = val; }
                fs[out] = new Factor(fs.at(a)->conditioning(ev));
            } else if (op == "normalize") {
                std::string out, a;
                ss >> out >> a;
                fs[out] = new Factor(fs.at(a)->normalize());
            } else if (op == "print") {
                std::string name;
                ss >> name;
                print_factor(name.c_str(), *fs.at(name));
            }
        }
        for (auto &kv : fs) delete kv.second;
        for (auto &kv : vars) delete kv.second;
        return 0;
    }
    if (cmd == "sp" && argc >= 3) {
        // loopy BP as BN::sum_product (model.cpp:736-753) + marginals
        // (model.cpp:313-317); the iteration count FactorGraph::update returns
        BN *m = load(argv[2]);
        const unsigned max_it = argc >= 4 ? (unsigned)std::atoi(argv[3]) : 10000;
        const double eps = argc >= 5 ? std::atof(argv[4]) : 0.001;
        std::vector<const Variable *> mv(m->variables().begin(), m->variables().end());
        std::vector<const Factor *> fs(m->factors().begin(), m->factors().end());
        auto t0 = std::chrono::steady_clock::now();
        FactorGraph g(mv, fs);
        const unsigned it = g.update(max_it, eps);
        std::vector<Factor> marg;
        for (auto pv : mv) marg.push_back(g.marginal(pv));
        auto t1 = std::chrono::steady_clock::now();
        std::printf("iterations %u\n", it);
        for (size_t i = 0; i < marg.size(); ++i) {
            char tag[32];
            std::snprintf(tag, sizeof tag, "M%u", mv[i]->id());
            print_factor(tag, marg[i]);
        }
        std::printf("uptime_ms %.6f\n", std::chrono::duration<double, std::milli>(t1 - t0).count());
        delete m;
        return 0;
    }
    if (cmd == "query" && argc >= 5) {
        BN *m = load(argv[2]);
        auto o = opts_for(argv[3]);
        std::ifstream in(argv[4]);
        std::string line;
        int qi = 0;
        auto ids = [&](std::string s) {
            std::unordered_set<const Variable *> out;
            for (char &c : s)
                if (c == ',') c = ' ';
            std::istringstream ss(s);
            unsigned id;
            while (ss >> id) out.insert(m->variables().at(id));
            return out;
        };
        while (std::getline(in, line)) {
            if (line.compare(0, 6, "query ") != 0) continue;
            std::string body = line.substr(6), t = body, e;
            size_t bar = body.find('|');
            if (bar != std::string::npos) {
                t = body.substr(0, bar);
                e = body.substr(bar + 1);
            }
            double up = 0;
            Factor q = m->query_ve(ids(t), ids(e), o, up);
            char tag[32];
            std::snprintf(tag, sizeof tag, "Q%d", qi++);
            print_factor(tag, q);
        }
        delete m;
        return 0;
    }
    if (cmd == "micro" && argc >= 5) {
        unsigned k = (unsigned)std::atoi(argv[2]), w = (unsigned)std::atoi(argv[3]);
        int reps = std::atoi(argv[4]);
        std::vector<Variable *> vs;
        for (unsigned i = 0; i < w + 2; ++i) vs.push_back(new Variable(i, k));
        std::vector<const Variable *> sm(vs.begin(), vs.begin() + w + 1);
        std::vector<const Variable *> sf = {vs[0], vs[w + 1]};
        std::mt19937 gen(42);
        std::uniform_real_distribution<double> U(0.5, 2.0);
        Domain *dm = new Domain(sm), *df = new Domain(sf);
        std::vector<double> vm(dm->size()), vf(df->size());
        for (auto &v : vm) v = U(gen);
        for (auto &v : vf) v = U(gen);
        Factor fm(dm, vm, 0.0), ff(df, vf, 0.0);
        double entries = (double)dm->size() * k;
        auto t0 = std::chrono::steady_clock::now();
        double sink = 0;
        for (int r = 0; r < reps; ++r) {
            Factor prod(1.0);           // model.cpp:414-418
            prod *= fm;
            prod *= ff;
            Factor msg = prod.sum_out(vs[0]);
            sink += msg.partition();
        }
        auto t1 = std::chrono::steady_clock::now();
        double sec = std::chrono::duration<double>(t1 - t0).count();
        std::printf("entries_per_s %.6g\nseconds %.6f\nentries %.0f\nsink %.6g\n", entries * reps / sec, sec, entries * reps, sink);
        for (auto v : vs) delete v;
        return 0;
    }
    std::fprintf(stderr, "bad command\n");
    return 1;
}
