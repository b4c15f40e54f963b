// bn.hpp — C++ mirror of bn-pp's class API (code/variable.hh, domain.hh,
// factor.hh, model.hh, io.hh) on top of the MI355X engine.
//
// Same names, argument meaning and error behaviour as the reference, with two
// deliberate differences:
//   - sizes and positions are 64-bit (the reference's `unsigned` wraps at 2^32,
//     domain.hh:21-22);
//   - every factor-algebra operation (product, sum_out, conditioning, the VE
//     buckets) runs on the GPU through include/bnpp.h; there is no CPU
//     fallback: without a device they throw std::runtime_error.
// Index-range errors throw const char* exactly like factor.cpp:87/94 and
// domain.cpp:96.
#pragma once

#include <cstdint>
#include <memory>
#include <ostream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace bn {

class Variable {                                   // variable.hh:8-21
public:
    Variable(unsigned id, unsigned size) : _id(id), _size(size) {}
    unsigned id() const { return _id; }
    unsigned size() const { return _size; }
    friend std::ostream &operator<<(std::ostream &o, const Variable &v);

private:
    unsigned _id;
    unsigned _size;
};

class Domain {                                     // domain.hh:11-45
public:
    Domain();
    Domain(std::vector<const Variable *> scope);
    Domain(const Domain &d);
    Domain(const Domain &d1, const Domain &d2);    // union: d1 order, then new d2 vars
    Domain(const Domain &d, const Variable *v);    // remove v
    Domain(const Domain &d, const std::unordered_map<unsigned, unsigned> &evidence);

    std::vector<const Variable *> scope() const { return _scope; }
    unsigned width() const { return (unsigned)_scope.size(); }
    uint64_t size() const { return _size; }
    const Variable *operator[](unsigned i) const;
    bool in_scope(const Variable *v) const;
    bool in_scope(unsigned id) const;
    void next_valuation(std::vector<unsigned> &valuation) const;
    uint64_t position_valuation(const std::vector<unsigned> &valuation) const;
    uint64_t position_consistent_valuation(const std::vector<unsigned> &valuation, const Domain &domain) const;
    friend std::ostream &operator<<(std::ostream &o, const Domain &d);

private:
    void init();
    std::vector<const Variable *> _scope;
    std::vector<uint64_t> _offset;
    uint64_t _size = 1;
};

class Factor {                                     // factor.hh:11-48
public:
    Factor(const Domain *domain, std::vector<double> values, double partition);   // adopts domain
    Factor(const Domain *domain, double value = 0.0);
    Factor(double value = 1.0);
    Factor(const Factor &f);
    Factor(Factor &&f) noexcept;
    ~Factor();
    Factor &operator=(Factor &&f) noexcept;
    Factor &operator=(const Factor &f);
    Factor operator*(const Factor &f);
    void operator*=(const Factor &f);

    const Domain &domain() const { return *_domain; }
    uint64_t size() const { return _domain->size(); }
    unsigned width() const { return _domain->width(); }
    double partition() const;                    // factor.hh:26 (computed on first read)
    const double &operator[](uint64_t i) const;
    double &operator[](uint64_t i);
    const std::vector<double> &values() const { return _values; }
    double max() const;
    double min() const;

    Factor sum_out(const Variable *variable) const;                                  // factor.cpp:182-212
    Factor product(const Factor &f) const;                                           // factor.cpp:117-147
    Factor divide(const Factor &f) const;                                            // factor.cpp:149-180
    Factor conditioning(const std::unordered_map<unsigned, unsigned> &evidence) const;  // factor.cpp:214-242
    Factor normalize() const;                                                        // factor.cpp:244-255
    friend std::ostream &operator<<(std::ostream &os, const Factor &f);

private:
    // The reference computes _partition with every op (factor.cpp:129-139,
    // 161-172, 196-208, 226-236); here an op leaves it pending and the first
    // read (partition(), normalize(), min(), printing, a mutable operator[])
    // computes it on the host in the reference's order, so an op whose
    // partition nobody reads costs its kernel and transfers only.
    struct PendingSum;
    void resolve_partition() const;
    const Domain *_domain;
    std::vector<double> _values;
    mutable double _partition;
    mutable std::shared_ptr<const PendingSum> _pending;
};

// The GPU engine's precision for Model/BN inference (default fp64, bit-exact
// with the reference's arithmetic); options["fp32"] selects fp32 storage.
class Model {                                      // model.hh:11-38
public:
    Model(std::string name, std::vector<Variable *> &variables, std::vector<Factor *> &factors);
    virtual ~Model();
    const std::string name() const { return _name; }
    const std::vector<Variable *> &variables() const { return _variables; }
    const std::vector<Factor *> &factors() const { return _factors; }

    // VE on the GPU (the reference's Model:: versions form the full joint; the
    // result is the same quantity)
    virtual double partition(const std::unordered_map<unsigned, unsigned> &evidence,
                             std::unordered_map<std::string, bool> &options, double &uptime) const;
    // options["bucket-tree"]: all marginals from one two-pass bucket tree
    // (bnpp_marginals_tree, equal to rounding); default: one VE per target,
    // bit-exact with the reference arithmetic
    virtual std::vector<const Factor *> marginals(const std::unordered_map<unsigned, unsigned> &evidence,
                                                  std::unordered_map<std::string, bool> &options,
                                                  double &uptime) const;
    // log10 of the partition function (finite beyond the double range)
    double log10_partition(const std::unordered_map<unsigned, unsigned> &evidence,
                           std::unordered_map<std::string, bool> &options, double &uptime) const;
    virtual void write(std::ostream &) const {}

protected:
    std::string _name;
    std::vector<Variable *> _variables;
    std::vector<Factor *> _factors;
};

class BN : public Model {                          // model.hh:40-104
public:
    BN(std::string name, std::vector<Variable *> &variables, std::vector<Factor *> &factors);
    // model.cpp:348-446: bucket elimination, one fused GPU kernel per bucket
    Factor variable_elimination(std::vector<const Variable *> &variables, std::vector<const Factor *> &factors,
                                std::unordered_map<std::string, bool> &options) const;
    // model.cpp:205-248: P(target | evidence) as a table over target + evidence
    Factor query_ve(const std::unordered_set<const Variable *> &target,
                    const std::unordered_set<const Variable *> &evidence,
                    std::unordered_map<std::string, bool> &options, double &uptime) const;
    const std::unordered_set<const Variable *> parents(const Variable *v) const { return _parents.find(v)->second; }
    const std::unordered_set<const Variable *> children(const Variable *v) const { return _children.find(v)->second; }

private:
    std::unordered_map<const Variable *, std::unordered_set<const Variable *>> _parents;
    std::unordered_map<const Variable *, std::unordered_set<const Variable *>> _children;
};

class MN : public Model {                          // model.hh:106-118
public:
    MN(std::string name, std::vector<Variable *> &variables, std::vector<Factor *> &factors);
    // model.cpp:979-999: "MARKOV:", every variable with its neighbours, every factor
    void write(std::ostream &os) const override;
    friend std::ostream &operator<<(std::ostream &os, const MN &mn);

private:
    // the reference's container (model.hh:116), filled in the same order, so
    // the neighbours print in its iteration order
    std::unordered_map<const Variable *, std::unordered_set<const Variable *>> _neighbors;
};

// io.hh:10-19 (return 0 / -1 cannot open / -2 wrong network type)
int read_uai_model(std::string &filename, BN **model);
int read_uai_model(std::string &filename, MN **model);
int read_uai_evidence(std::string &filename, std::unordered_map<unsigned, unsigned> &evidence);

// Engine device used by the C++ API (default: env BNPP_DEVICE or 0).
void set_device(int device);

}  // namespace bn
