// Elimination-order heuristics over the moral graph (graph.cpp:9-237).
#pragma once
#include <vector>

namespace bnpp {

enum Heuristic { kOrderGiven = 0, kMinFill = 1, kWeightedMinFill = 2, kMinDegree = 3 };

// Graph::Graph (graph.cpp:9-35) over `scopes` (one scope per factor), then
// Graph::ordering (graph.cpp:41-101) of `vars`.  Candidates are scanned in
// ascending id order, so ties resolve deterministically; the selection rules
// (strict improvement, min-degree tie-break, initial bound |V|+1, weighted
// initial value from the first candidate) are the reference's.
// Returns the induced width; order_out receives vars.size() ids.
int elimination_order(int n_model_vars, const std::vector<int> &cards, const std::vector<std::vector<int>> &scopes,
                      const std::vector<int> &vars, Heuristic h, std::vector<int> &order_out);

// Graph::order_width (graph.cpp:197-237)
int order_width(int n_model_vars, const std::vector<std::vector<int>> &scopes, const std::vector<int> &order);

// entries of the largest message eliminating in `order` makes (a symbolic pass:
// the checkpoint-slot search's first estimate, before any plan exists)
double order_max_table(int n_model_vars, const std::vector<int> &cards, const std::vector<std::vector<int>> &scopes,
                       const std::vector<int> &order);

}  // namespace bnpp
