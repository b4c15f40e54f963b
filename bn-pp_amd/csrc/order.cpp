// Elimination-order heuristics (graph.cpp:41-237) on bitset adjacency with
// incrementally maintained fill-in / degree caches.  Eliminating u only changes
// the scores of N(u) and of common neighbours of the new fill edges, so only
// that set is rescored; the candidate scan itself keeps the reference's rules.
#include "order.hpp"

#include <algorithm>
#include <cstdint>

namespace bnpp {
namespace {

struct BitGraph {
    int n = 0, words = 0;
    std::vector<uint64_t> adj;
    std::vector<uint8_t> present;
    int n_present = 0;

    uint64_t *row(int v) { return adj.data() + (size_t)v * words; }
    const uint64_t *row(int v) const { return adj.data() + (size_t)v * words; }
    bool has(int a, int b) const { return (row(a)[b >> 6] >> (b & 63)) & 1u; }
    void set(int a, int b) { row(a)[b >> 6] |= (uint64_t)1 << (b & 63); }
    void clr(int a, int b) { row(a)[b >> 6] &= ~((uint64_t)1 << (b & 63)); }
    int degree(int v) const {
        if (!present[v]) return 0;
        int c = 0;
        const uint64_t *r = row(v);
        for (int i = 0; i < words; ++i) c += __builtin_popcountll(r[i]);
        return c;
    }
    void neighbours(int v, std::vector<int> &out) const {
        out.clear();
        if (!present[v]) return;
        const uint64_t *r = row(v);
        for (int i = 0; i < words; ++i) {
            uint64_t b = r[i];
            while (b) {
                out.push_back(i * 64 + __builtin_ctzll(b));
                b &= b - 1;
            }
        }
    }
};

BitGraph build(int n, const std::vector<std::vector<int>> &scopes) {   // graph.cpp:9-35
    BitGraph g;
    g.n = n;
    g.words = (n + 63) / 64;
    g.adj.assign((size_t)n * g.words + 1, 0);
    g.present.assign(n + 1, 0);
    for (const auto &s : scopes) {
        for (int v : s)
            if (!g.present[v]) { g.present[v] = 1; g.n_present++; }
        for (size_t i = 0; i + 1 < s.size(); ++i)
            for (size_t j = i + 1; j < s.size(); ++j)
                if (s[i] != s[j]) { g.set(s[i], s[j]); g.set(s[j], s[i]); }
    }
    return g;
}

// non-adjacent neighbour pairs id1 < id2 (graph.cpp:131-138 / 174-180)
unsigned fill_of(const BitGraph &g, const std::vector<int> &cards, int v, bool weighted) {
    if (!g.present[v]) return 0;
    const uint64_t *r = g.row(v);
    unsigned fill = 0;
    for (int wi = 0; wi < g.words; ++wi) {
        uint64_t bits = r[wi];
        while (bits) {
            int a = wi * 64 + __builtin_ctzll(bits);
            bits &= bits - 1;
            const uint64_t *ra = g.row(a);
            for (int wj = wi; wj < g.words; ++wj) {
                uint64_t cand = r[wj] & ~ra[wj];
                if (wj == wi) cand &= ~((((uint64_t)2) << (a & 63)) - 1);
                if (!weighted) {
                    fill += (unsigned)__builtin_popcountll(cand);
                } else {
                    while (cand) {
                        int b = wj * 64 + __builtin_ctzll(cand);
                        cand &= cand - 1;
                        fill += (unsigned)cards[a] * (unsigned)cards[b];
                    }
                }
            }
        }
    }
    return fill;
}

}  // namespace

int elimination_order(int n, const std::vector<int> &cards, const std::vector<std::vector<int>> &scopes,
                      const std::vector<int> &vars, Heuristic h, std::vector<int> &order_out) {
    order_out.clear();
    if (h == kOrderGiven) {
        order_out = vars;
        return order_width(n, scopes, vars);
    }
    BitGraph g = build(n, scopes);
    std::vector<uint8_t> cand(n + 1, 0);
    int remaining = 0;
    for (int v : vars)
        if (!cand[v]) { cand[v] = 1; remaining++; }
    const bool weighted = h == kWeightedMinFill;
    std::vector<unsigned> fill(n, 0);
    std::vector<int> deg(n, 0);
    for (int v = 0; v < n; ++v) {
        deg[v] = g.degree(v);
        if (cand[v] && h != kMinDegree) fill[v] = fill_of(g, cards, v, weighted);
    }
    std::vector<int> nb, nb2;
    std::vector<uint8_t> dirty(n, 0);
    std::vector<int> dirty_list;
    int width = 0;
    int first = 0;
    while (remaining > 0) {
        while (!cand[first]) ++first;
        int next = first;
        if (h == kMinDegree) {                                          // graph.cpp:103-120
            int best = g.n_present + 1;
            for (int v = first; v < n; ++v)
                if (cand[v] && deg[v] < best) { next = v; best = deg[v]; }
        } else {                                                        // graph.cpp:122-195
            unsigned best = weighted ? fill[first] : (unsigned)g.n_present + 1;
            for (int v = first; v < n; ++v) {
                if (!cand[v]) continue;
                if (fill[v] < best) { next = v; best = fill[v]; }
                else if (fill[v] == best && deg[v] < deg[next]) { next = v; best = fill[v]; }
            }
        }
        order_out.push_back(next);
        width = std::max(width, deg[next]);
        // eliminate `next`: connect its neighbours, drop it (graph.cpp:80-97)
        g.neighbours(next, nb);
        dirty_list.clear();
        auto mark = [&](int v) {
            if (!dirty[v]) { dirty[v] = 1; dirty_list.push_back(v); }
        };
        for (int a : nb) { g.clr(a, next); mark(a); }
        for (size_t i = 0; i < nb.size(); ++i)
            for (size_t j = i + 1; j < nb.size(); ++j) {
                int a = nb[i], b = nb[j];
                if (!g.has(a, b)) {
                    g.set(a, b);
                    g.set(b, a);
                    // common neighbours of a and b now see one fewer missing pair
                    const uint64_t *ra = g.row(a), *rb = g.row(b);
                    for (int w = 0; w < g.words; ++w) {
                        uint64_t c = ra[w] & rb[w];
                        while (c) { mark(w * 64 + __builtin_ctzll(c)); c &= c - 1; }
                    }
                }
            }
        if (g.present[next]) {
            std::fill(g.row(next), g.row(next) + g.words, 0);
            g.present[next] = 0;
            g.n_present--;
        }
        cand[next] = 0;
        remaining--;
        for (int v : dirty_list) {
            dirty[v] = 0;
            deg[v] = g.degree(v);
            if (cand[v] && h != kMinDegree) fill[v] = fill_of(g, cards, v, weighted);
        }
    }
    return width;
}

int order_width(int n, const std::vector<std::vector<int>> &scopes, const std::vector<int> &order) {
    BitGraph g = build(n, scopes);
    std::vector<int> nb;
    int width = 0;
    for (int v : order) {
        width = std::max(width, g.degree(v));
        g.neighbours(v, nb);
        for (int a : nb) g.clr(a, v);
        for (size_t i = 0; i < nb.size(); ++i)
            for (size_t j = 0; j < nb.size(); ++j)
                if (i != j) g.set(nb[i], nb[j]);
        if (g.present[v]) {
            std::fill(g.row(v), g.row(v) + g.words, 0);
            g.present[v] = 0;
            g.n_present--;
        }
    }
    return width;
}

// entries of the largest table `order` makes (the product of the cards of a
// variable's neighbours when it is eliminated: its bucket's message)
double order_max_table(int n, const std::vector<int> &cards, const std::vector<std::vector<int>> &scopes,
                       const std::vector<int> &order) {
    BitGraph g = build(n, scopes);
    std::vector<int> nb;
    double big = 1;
    for (int v : order) {
        g.neighbours(v, nb);
        double t = 1;
        for (int a : nb) t *= cards[a];
        big = std::max(big, t);
        for (int a : nb) g.clr(a, v);
        for (size_t i = 0; i < nb.size(); ++i)
            for (size_t j = 0; j < nb.size(); ++j)
                if (i != j) g.set(nb[i], nb[j]);
        if (g.present[v]) {
            std::fill(g.row(v), g.row(v) + g.words, 0);
            g.present[v] = 0;
            g.n_present--;
        }
    }
    return big;
}

}  // namespace bnpp
