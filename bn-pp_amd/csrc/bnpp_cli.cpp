// bnpp — command-line front end with the reference's task flags (bn.cpp:136-258,
// mn.cpp:135-155): -pr / -mar, -mf / -wmf / -md, -sp, -v, plus -f32, -mar-tree
// and -uai <base> (UAI-competition result files <base>.PR / <base>.MAR, the
// format of the reference's models/markovnets/*.PR / *.MAR fixtures: log10 Z;
// per variable its card and probabilities, evidence variables one-hot).
// BAYES files print like `bn` (raw Z), MARKOV files like `mn` (log10 Z).
// -ve is accepted and, as in the reference, changes nothing here: bn reads it
// only for REPL queries (bn.cpp:346); partition / marginals always run VE
// (model.cpp:275, 319).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/bnpp/bn.hpp"
#include "../../include/bnpp.h"

int main(int argc, char **argv) {
    std::unordered_map<std::string, bool> options;
    std::vector<std::string> positional;
    std::string uai_out;
    for (int i = 1; i < argc; ++i) {
        std::string p(argv[i]);
        if (p == "-uai" && i + 1 < argc) uai_out = argv[++i];
        else if (p == "-pr") options["partition"] = true;
        else if (p == "-mar") options["marginals"] = true;
        else if (p == "-mar-tree") { options["marginals"] = true; options["bucket-tree"] = true; }
        else if (p == "-ve") options["variable-elimination"] = true;
        else if (p == "-sp") options["sum-product"] = true;      // bn.cpp:177-178: loopy BP marginals
        else if (p == "-mf") options["min-fill"] = true;
        else if (p == "-wmf") options["weighted-min-fill"] = true;
        else if (p == "-md") options["min-degree"] = true;
        else if (p == "-f32") options["fp32"] = true;
        else if (p == "-v") options["verbose"] = true;
        else if (p == "-h") options["help"] = true;
        else if (p[0] == '-') { std::cerr << "Error: invalid option `" << p << "'." << std::endl; return -1; }
        else positional.push_back(p);
    }
    if (positional.empty() || options["help"]) {
        std::cout << "usage: " << argv[0] << " /path/to/model.uai [/path/to/evidence.uai.evid] -pr|-mar|-mar-tree [-sp] [-mf|-wmf|-md] [-f32] [-uai base]" << std::endl;
        return positional.empty() ? 1 : 0;
    }
    bnpp_model *probe = nullptr;
    if (bnpp_model_load_uai(positional[0].c_str(), &probe) != BNPP_OK) {
        std::cerr << "Error: " << bnpp_last_error() << std::endl;
        return -1;
    }
    int is_bayes = 0;
    bnpp_model_info(probe, &is_bayes, nullptr, nullptr);
    bnpp_model_free(probe);
    std::unordered_map<unsigned, unsigned> evidence;
    if (positional.size() > 1 && bn::read_uai_evidence(positional[1], evidence)) return -2;
    bn::Model *model = nullptr;
    if (is_bayes) {
        bn::BN *m = nullptr;
        if (bn::read_uai_model(positional[0], &m)) return -1;
        model = m;
    } else {
        bn::MN *m = nullptr;
        if (bn::read_uai_model(positional[0], &m)) return -1;
        model = m;
    }
    try {
        double uptime = 0;
        if (options["partition"]) {
            double lz = 0;
            if (is_bayes) {
                double p = model->partition(evidence, options, uptime);
                std::cout << ">> Partition = " << p << std::endl;
                lz = std::log10(p);
            } else {
                lz = model->log10_partition(evidence, options, uptime);
                std::cout << "Partition = " << lz << std::endl << std::endl;
            }
            std::cout << ">> Executed in " << uptime << "ms." << std::endl << std::endl;
            if (!uai_out.empty()) {
                FILE *f = std::fopen((uai_out + ".PR").c_str(), "w");
                if (!f) throw std::runtime_error("cannot write " + uai_out + ".PR");
                std::fprintf(f, "PR\n1\n%g\n", lz);
                std::fclose(f);
            }
        }
        if (options["marginals"]) {
            std::vector<const bn::Factor *> marg = model->marginals(evidence, options, uptime);
            std::cout << ">> Marginals:" << std::endl;
            for (auto pf : marg) std::cout << *pf << std::endl;
            std::cout << ">> Executed in " << uptime << "ms." << std::endl << std::endl;
            if (!uai_out.empty()) {
                FILE *f = std::fopen((uai_out + ".MAR").c_str(), "w");
                if (!f) throw std::runtime_error("cannot write " + uai_out + ".MAR");
                std::fprintf(f, "MAR\n1\n%zu\n", marg.size());
                const std::vector<bn::Variable *> &vars = model->variables();
                for (size_t i = 0; i < marg.size(); ++i) {
                    const unsigned k = vars[i]->size();
                    std::fprintf(f, "%u", k);
                    auto ev = evidence.find(vars[i]->id());
                    for (unsigned x = 0; x < k; ++x) {
                        // an evidence variable's marginal is a width-0 factor (model.cpp:333): one-hot here
                        const double p = ev != evidence.end() && marg[i]->width() == 0 ? (x == ev->second ? 1.0 : 0.0)
                                                                                      : (*marg[i])[x];
                        std::fprintf(f, " %g", p);
                    }
                    std::fprintf(f, "\n");
                }
                std::fclose(f);
            }
            for (auto pf : marg) delete pf;
        }
    } catch (const std::exception &e) {
        std::cerr << "Error: " << e.what() << std::endl;
        delete model;
        return -3;
    }
    delete model;
    return 0;
}
