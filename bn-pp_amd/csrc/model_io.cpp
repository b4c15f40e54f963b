#include "model_io.hpp"

#include <cstdlib>
#include <fstream>

namespace bnpp {
namespace {

// read_next_token (io.cpp:14-23): a token starting with '#' drops the rest of its line
bool next_token(std::ifstream &in, std::string &tok) {
    while (in >> tok) {
        if (tok[0] != '#') return true;
        std::string rest;
        std::getline(in, rest);
    }
    return false;
}
bool next_long(std::ifstream &in, long &v) {
    std::string t;
    if (!next_token(in, t)) return false;
    char *end = nullptr;
    v = std::strtol(t.c_str(), &end, 10);
    return end != t.c_str();
}
bool next_double(std::ifstream &in, double &v) {
    std::string t;
    if (!next_token(in, t)) return false;
    char *end = nullptr;
    v = std::strtod(t.c_str(), &end);
    return end != t.c_str();
}

}  // namespace

int load_uai(const std::string &path, ModelData &m, std::string *err) {
    std::ifstream in(path);
    if (!in.is_open()) {
        if (err) *err = "couldn't read file " + path;
        return -1;
    }
    m = ModelData{};
    m.name = path;
    std::string hdr;
    if (!next_token(in, hdr) || (hdr != "BAYES" && hdr != "MARKOV")) {
        if (err) *err = "expected 'BAYES' or 'MARKOV' file header, found: " + hdr;
        return -2;
    }
    m.is_bayes = hdr == "BAYES";
    long nv, nf;
    if (!next_long(in, nv) || nv < 0) goto bad;
    m.cards.resize(nv);
    for (long i = 0; i < nv; ++i) {
        long c;
        if (!next_long(in, c) || c < 1) goto bad;
        m.cards[i] = (int)c;
    }
    if (!next_long(in, nf) || nf < 0) goto bad;
    m.scopes.resize(nf);
    m.values.resize(nf);
    for (long f = 0; f < nf; ++f) {
        long w;
        if (!next_long(in, w) || w < 0) goto bad;
        m.scopes[f].resize(w);
        for (long j = 0; j < w; ++j) {
            long id;
            if (!next_long(in, id) || id < 0 || id >= nv) goto bad;
            m.scopes[f][j] = (int)id;
        }
    }
    for (long f = 0; f < nf; ++f) {
        long sz;
        if (!next_long(in, sz) || sz < 0) goto bad;
        m.values[f].resize(sz);
        for (long j = 0; j < sz; ++j)
            if (!next_double(in, m.values[f][j])) goto bad;
    }
    if (!validate(m, err)) return -2;
    return 0;
bad:
    if (err) *err = "malformed UAI file " + path;
    return -2;
}

int load_evidence(const std::string &path, std::vector<std::pair<int, int>> &ev) {
    std::ifstream in(path);
    if (!in.is_open()) return -1;
    ev.clear();
    long n, size;
    if (next_long(in, n) && n == 1 && next_long(in, size)) {
        for (long i = 0; i < size; ++i) {
            long id, val;
            if (!next_long(in, id) || !next_long(in, val)) break;
            bool found = false;
            for (auto &p : ev)
                if (p.first == id) { p.second = (int)val; found = true; }
            if (!found) ev.push_back({(int)id, (int)val});
        }
    }
    return 0;
}

bool validate(const ModelData &m, std::string *err) {
    for (size_t f = 0; f < m.scopes.size(); ++f) {
        long double sz = 1;
        for (int v : m.scopes[f]) {
            if (v < 0 || v >= (int)m.cards.size()) {
                if (err) *err = "factor " + std::to_string(f) + ": variable id out of range";
                return false;
            }
            sz *= m.cards[v];
        }
        if ((long double)m.values[f].size() != sz) {
            if (err) *err = "factor " + std::to_string(f) + ": table size does not match its scope";
            return false;
        }
    }
    return true;
}

}  // namespace bnpp
