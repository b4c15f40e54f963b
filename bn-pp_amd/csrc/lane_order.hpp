// Enqueue order of a two-lane sliced schedule (runtime.cpp make_executable).
// Header-only and free of HIP so tests/cpp/lane_order.cpp checks it on the host.
#pragma once
#include <algorithm>
#include <cstdint>
#include <functional>
#include <vector>

namespace bnpp {

// The share of a window's compute the other lane's next window waits for
// (two-lane sliced schedules): 1 = strict alternation, 0 = none (the lanes
// free-run).  BNPP_LANE_ALT overrides it in tuning builds.
constexpr double kLaneAltDefault = 1.0;

// Two-lane schedules: the order the groups are enqueued in, and the waits that
// make the lanes' windows alternate.  A lane's window is its compute groups up
// to an exchange plus that exchange (sync, pack, all-to-all, unpack).  Left to
// themselves the two fronts drift into phase -- both compute at half the GPU,
// then both wait on an exchange with the GPU idle (profiles/r06_mar_sliced8_
// breakdown.txt: ~73 ms of a 412-ms modelled share).  Alternating, lane 1's
// window k starts once lane 0's window k has computed (share `frac` of its
// compute groups' work), and lane 0's window k+1 once lane 1's window k has:
// each lane's exchange then runs beside the other lane's buckets.
//
// The groups are enqueued window by window alternately, because a stream wait
// only orders work enqueued before it.  A group whose input the other lane
// makes later pulls that lane's groups forward first, so every data
// dependency keeps its event; an alternation wait whose target is not yet
// enqueued is dropped.  Per-lane order is unchanged, and every rank derives
// the same order from the same schedule shape, so each lane's collectives
// keep one order across ranks.
//
//   lane[g], is_x[g] (an exchange step), work[g] (tiles): per group, schedule order
//   g_record[g]: event group g records (-1 none); g_wait[g]: events it waits for;
//   n_ev: events in use -- alternation waits add events, records and waits
// Returns the enqueue order (a permutation of the groups), or an empty vector
// (schedule order) when frac <= 0.
inline std::vector<int> lane_order(const std::vector<int> &lane, const std::vector<char> &is_x,
                                   const std::vector<int64_t> &work, std::vector<int> &g_record,
                                   std::vector<std::vector<int>> &g_wait, int &n_ev, double frac) {
    const int ng = (int)lane.size();
    std::vector<int> order;
    if (frac <= 0.0) return order;
    std::vector<int> rec_group(n_ev, -1);                    // event -> the group recording it
    for (int g = 0; g < ng; ++g)
        if (g_record[g] >= 0) rec_group[g_record[g]] = g;
    std::vector<int> seq[2];
    for (int g = 0; g < ng; ++g) seq[lane[g] & 1].push_back(g);
    struct Win { int cbegin, cend, end; };                   // seq indices: compute [cbegin, cend), exchange [cend, end)
    std::vector<Win> win[2];
    for (int l = 0; l < 2; ++l) {
        const std::vector<int> &s = seq[l];
        for (int i = 0; i < (int)s.size();) {
            Win w{i, i, i};
            while (i < (int)s.size() && !is_x[s[i]]) ++i;
            w.cend = i;
            while (i < (int)s.size() && is_x[s[i]]) ++i;
            w.end = i;
            win[l].push_back(w);
        }
    }
    std::vector<int> pos(ng, -1), lane_idx(ng, 0);
    for (int l = 0; l < 2; ++l)
        for (int i = 0; i < (int)seq[l].size(); ++i) lane_idx[seq[l][i]] = i;
    int ptr[2] = {0, 0};
    // enqueue lane l's groups up to seq index `last`, each after the other
    // lane's producers of its inputs
    std::function<void(int, int)> upto = [&](int l, int last) {
        while (ptr[l] <= last) {
            const int g = seq[l][ptr[l]];
            for (int e : g_wait[g]) {
                const int p = e < (int)rec_group.size() ? rec_group[e] : -1;
                if (p >= 0 && pos[p] < 0) upto(lane[p] & 1, lane_idx[p]);
            }
            pos[g] = (int)order.size();
            order.push_back(g);
            ++ptr[l];
        }
    };
    // the group of a window whose completion releases the other lane: where
    // `frac` of the window's compute work is done
    auto release = [&](int l, const Win &w) {
        int64_t tot = 0, acc = 0;
        for (int i = w.cbegin; i < w.cend; ++i) tot += std::max<int64_t>(1, work[seq[l][i]]);
        for (int i = w.cbegin; i < w.cend; ++i) {
            acc += std::max<int64_t>(1, work[seq[l][i]]);
            if ((double)acc >= frac * (double)tot) return seq[l][i];
        }
        return -1;
    };
    auto wait_on = [&](int waiter, int target) {
        if (target < 0 || pos[target] < 0) return;
        if (g_record[target] < 0) {
            g_record[target] = n_ev++;
            rec_group.push_back(target);
        }
        std::vector<int> &w = g_wait[waiter];
        if (std::find(w.begin(), w.end(), g_record[target]) == w.end()) w.push_back(g_record[target]);
    };
    const size_t nw = std::max(win[0].size(), win[1].size());
    for (size_t k = 0; k < nw; ++k) {
        for (int l = 0; l < 2; ++l) {
            if (k >= win[l].size()) continue;
            const Win &w = win[l][k];
            // lane 1's window k after lane 0's window k; lane 0's window k after lane 1's window k - 1
            const int ol = 1 - l, ok = l == 1 ? (int)k : (int)k - 1;
            if (w.cbegin < w.cend && ptr[l] <= w.cbegin && ok >= 0 && ok < (int)win[ol].size()) {
                upto(l, w.cbegin - 1);
                wait_on(seq[l][w.cbegin], release(ol, win[ol][ok]));
            }
            upto(l, w.end - 1);
        }
    }
    upto(0, (int)seq[0].size() - 1);
    upto(1, (int)seq[1].size() - 1);
    return order;
}

}  // namespace bnpp
