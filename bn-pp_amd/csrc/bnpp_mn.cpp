// bnpp-mn — the reference `mn` front end on the GPU engine: the same argv
// (model, evidence file, -h / -v; mn.cpp:37-94), the same stdin prompt with
// PR / MAR / quit (mn.cpp:96-133) and the same output (log10 Z, mn.cpp:135-142;
// marginals printed as Factors, mn.cpp:144-155, factor.cpp:291-321).  Inference
// runs as VE on the device (the reference forms the full joint, model.cpp:31-101;
// same quantities).
#include <iostream>
#include <regex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/bnpp.h"
#include "../../include/bnpp/bn.hpp"

namespace {

void usage(const char *prog) {
    std::cout << "usage: " << prog << " /path/to/model.uai /path/to/evidence.uai.evid [OPTIONS]" << std::endl
              << std::endl;
    std::cout << "OPTIONS:" << std::endl;
    std::cout << "-h\tdisplay help information" << std::endl;
    std::cout << "-v\tverbose" << std::endl;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        usage(argv[0]);
        return 1;
    }
    std::unordered_map<std::string, bool> options{{"verbose", false}, {"help", false}};
    for (int i = 2; i < argc; ++i) {
        const std::string o(argv[i]);
        if (o == "-h") options["help"] = true;
        else if (o == "-v") options["verbose"] = true;
    }
    if (options["help"]) {
        usage(argv[0]);
        return 0;
    }
    if (argc < 3) {                                   // mn reads argv[2] unconditionally (mn.cpp:57)
        usage(argv[0]);
        return 1;
    }
    if (!bnpp_abi_matches()) {
        std::cerr << "Error: libbnpp ABI version differs from include/bnpp.h" << std::endl;
        return -3;
    }
    std::string model_file(argv[1]), evidence_file(argv[2]);
    bn::MN *model = nullptr;
    if (bn::read_uai_model(model_file, &model)) return -1;
    std::unordered_map<unsigned, unsigned> evidence;
    if (bn::read_uai_evidence(evidence_file, evidence)) {
        delete model;
        return -2;
    }
    if (options["verbose"]) {                          // mn.cpp:96-106
        std::cout << ">> Model:" << std::endl;
        std::cout << *model << std::endl;
        std::cout << ">> Evidence:" << std::endl;
        for (auto &kv : evidence) std::cout << "Variable = " << kv.first << ", Value = " << kv.second << std::endl;
        std::cout << std::endl;
    }
    const std::regex quit_re("quit"), pr_re("PR|pr|partition"), mar_re("MAR|mar|marginals");
    std::unordered_map<std::string, bool> run_opts{{"min-fill", true}};
    int rc = 0;
    std::cout << ">> Query prompt:" << std::endl;
    while (std::cin) {
        std::cout << "? ";
        std::string line;
        std::getline(std::cin, line);
        try {
            if (std::regex_match(line, pr_re)) {
                double up = 0;
                const double lz = model->log10_partition(evidence, run_opts, up);
                std::cout << "Partition = " << lz << std::endl << std::endl;
                std::cout << ">> Executed in " << up << "ms." << std::endl << std::endl;
            } else if (std::regex_match(line, mar_re)) {
                std::cout << ">> Marginals:" << std::endl;
                double up = 0;
                std::vector<const bn::Factor *> marg = model->marginals(evidence, run_opts, up);
                for (auto pf : marg) {
                    std::cout << *pf << std::endl;
                    delete pf;
                }
                std::cout << ">> Executed in " << up << "ms." << std::endl << std::endl;
            } else if (std::regex_match(line, quit_re)) {
                break;
            } else {
                std::cout << "Error: not a valid query." << std::endl;
            }
        } catch (const std::exception &e) {
            std::cerr << "Error: " << e.what() << std::endl;
            rc = -3;
            break;
        }
    }
    delete model;
    return rc;
}
