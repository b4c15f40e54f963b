// Host-side check of the two-lane enqueue order (bn-pp_amd/csrc/lane_order.hpp):
// on random two-lane schedules with cross-lane data dependencies, the order is
// a permutation that keeps each lane's order, every wait refers to an event a
// group enqueued earlier records, the data-dependency waits are all kept, and
// on a schedule without cross-lane inputs the windows alternate (lane 1's
// window k after lane 0's, lane 0's window k + 1 after lane 1's window k).
// Headers only, no GPU.
#include <cstdio>
#include <random>
#include <vector>

#include "lane_order.hpp"

using namespace bnpp;

static int fails = 0;
#define CHECK(c)                                                            \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                        \
        }                                                                   \
    } while (0)

struct Sched {
    std::vector<int> lane;
    std::vector<char> is_x;
    std::vector<int64_t> work;
    std::vector<int> g_record;
    std::vector<std::vector<int>> g_wait;
    int n_ev = 2;
};

// windows of `comp` compute groups and a 3-step exchange per lane, the lanes'
// groups interleaved level by level as the planner emits them (schedule
// order); with `deps`, random lane-1 groups read a lane-0 output made earlier
// in schedule order
static Sched make(std::mt19937 &rng, int windows, bool deps) {
    Sched s;
    std::vector<std::vector<std::pair<char, int64_t>>> per(2);
    for (int l = 0; l < 2; ++l)
        for (int w = 0; w < windows; ++w) {
            const int comp = 1 + (int)(rng() % 5);
            for (int c = 0; c < comp; ++c) per[l].push_back({0, 1 + (int64_t)(rng() % 1000)});
            if (w + 1 < windows || rng() % 2)
                for (int x = 0; x < 3; ++x) per[l].push_back({1, 1});
        }
    size_t i0 = 0, i1 = 0;
    while (i0 < per[0].size() || i1 < per[1].size()) {
        const bool take0 = i1 >= per[1].size() || (i0 < per[0].size() && rng() % 2);
        const int l = take0 ? 0 : 1;
        const auto &g = take0 ? per[0][i0++] : per[1][i1++];
        s.lane.push_back(l);
        s.is_x.push_back(g.first);
        s.work.push_back(g.second);
    }
    const int ng = (int)s.lane.size();
    s.g_record.assign(ng, -1);
    s.g_wait.assign(ng, {});
    if (deps)
        for (int g = 0; g < ng; ++g) {
            if (s.lane[g] == 0 || rng() % 4) continue;
            std::vector<int> prev;
            for (int p = 0; p < g; ++p)
                if (s.lane[p] == 0) prev.push_back(p);
            if (prev.empty()) continue;
            const int p = prev[rng() % prev.size()];
            if (s.g_record[p] < 0) s.g_record[p] = s.n_ev++;
            s.g_wait[g].push_back(s.g_record[p]);
        }
    return s;
}

static void check(const Sched &before, Sched &s, const std::vector<int> &order) {
    const int ng = (int)s.lane.size();
    CHECK((int)order.size() == ng);
    std::vector<int> pos(ng, -1);
    for (int i = 0; i < (int)order.size(); ++i) {
        CHECK(order[i] >= 0 && order[i] < ng && pos[order[i]] < 0);
        pos[order[i]] = i;
    }
    int last[2] = {-1, -1};                                  // per-lane order kept
    for (int g : order) {
        CHECK(g > last[s.lane[g]]);
        last[s.lane[g]] = g;
    }
    std::vector<int> rec(s.n_ev, -1);
    for (int g = 0; g < ng; ++g)
        if (s.g_record[g] >= 0) {
            CHECK(rec[s.g_record[g]] < 0);                   // one recorder per event
            rec[s.g_record[g]] = g;
        }
    for (int g = 0; g < ng; ++g) {
        for (int e : s.g_wait[g]) {
            CHECK(e >= 2 && e < s.n_ev && rec[e] >= 0);
            if (rec[e] >= 0) CHECK(pos[rec[e]] < pos[g]);   // recorded before the wait is enqueued
        }
        for (int e : before.g_wait[g]) {                     // data dependencies kept, same recorder
            bool kept = false;
            for (int f : s.g_wait[g]) kept = kept || (rec[f] >= 0 && rec[f] == [&] {
                for (int p = 0; p < ng; ++p)
                    if (before.g_record[p] == e) return p;
                return -2;
            }());
            CHECK(kept);
        }
    }
}

int main() {
    std::mt19937 rng(7);
    for (int it = 0; it < 400; ++it) {
        for (double frac : {1.0, 0.5, 0.01}) {
            Sched s = make(rng, 1 + it % 9, true);
            const Sched before = s;
            std::vector<int> order = lane_order(s.lane, s.is_x, s.work, s.g_record, s.g_wait, s.n_ev, frac);
            check(before, s, order);
        }
    }
    // frac 0: schedule order, nothing added
    {
        Sched s = make(rng, 5, true);
        const Sched before = s;
        CHECK(lane_order(s.lane, s.is_x, s.work, s.g_record, s.g_wait, s.n_ev, 0.0).empty());
        CHECK(s.n_ev == before.n_ev && s.g_wait == before.g_wait && s.g_record == before.g_record);
    }
    // no cross-lane inputs, strict alternation: window k of lane 1 waits for the
    // last compute group of lane 0's window k, window k + 1 of lane 0 for lane 1's window k
    for (int it = 0; it < 50; ++it) {
        Sched s = make(rng, 6, false);
        std::vector<int> order = lane_order(s.lane, s.is_x, s.work, s.g_record, s.g_wait, s.n_ev, 1.0);
        check(s, s, order);
        const int ng = (int)s.lane.size();
        std::vector<int> rec(s.n_ev, -1);
        for (int g = 0; g < ng; ++g)
            if (s.g_record[g] >= 0) rec[s.g_record[g]] = g;
        // windows per lane: (first compute group, last compute group)
        std::vector<std::pair<int, int>> win[2];
        for (int l = 0; l < 2; ++l) {
            int first = -1, lastc = -1;
            bool in_x = false;
            for (int g = 0; g < ng; ++g) {
                if (s.lane[g] != l) continue;
                if (!s.is_x[g]) {
                    if (in_x || first < 0) {
                        if (first >= 0) win[l].push_back({first, lastc});
                        first = g;
                    }
                    lastc = g;
                    in_x = false;
                } else {
                    in_x = true;
                }
            }
            if (first >= 0) win[l].push_back({first, lastc});
        }
        CHECK(win[0].size() == 6 && win[1].size() == 6);
        for (size_t k = 0; k < win[1].size(); ++k) {
            const int w1 = win[1][k].first;
            CHECK(s.g_wait[w1].size() == 1 && rec[s.g_wait[w1][0]] == win[0][k].second);
            if (k + 1 < win[0].size()) {
                const int w0 = win[0][k + 1].first;
                CHECK(s.g_wait[w0].size() == 1 && rec[s.g_wait[w0][0]] == win[1][k].second);
            }
        }
        CHECK(s.g_wait[win[0][0].first].empty());            // lane 0 starts free
    }
    if (fails) return 1;
    std::printf("lane order ok\n");
    return 0;
}
