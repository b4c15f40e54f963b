// Host data model + UAI reader (io.cpp:14-180 token rules).
#pragma once
#include <string>
#include <utility>
#include <vector>

namespace bnpp {

struct ModelData {
    std::string name;
    bool is_bayes = false;
    std::vector<int> cards;                      // per variable
    std::vector<std::vector<int>> scopes;        // per factor, reference scope order
    std::vector<std::vector<double>> values;     // per factor, row-major (last var fastest)
};

// read_file_header / read_variables / read_factors (io.cpp:43-100).  Returns 0,
// -1 when the file cannot be opened (io.cpp:124), -2 on a malformed file.
int load_uai(const std::string &path, ModelData &m, std::string *err);
// read_uai_evidence (io.cpp:157-180): pairs are read only when the first integer
// is 1; a repeated id keeps the last value.  Returns 0 or -1 (cannot open).
int load_evidence(const std::string &path, std::vector<std::pair<int, int>> &ev);
// validate shapes (scope ids in range, table sizes = prod(card))
bool validate(const ModelData &m, std::string *err);

}  // namespace bnpp
