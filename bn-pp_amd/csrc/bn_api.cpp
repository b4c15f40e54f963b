// C++ mirror of bn-pp's class API (include/bnpp/bn.hpp), layered on the C ABI.
#include "../../include/bnpp/bn.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <mutex>
#include <stdexcept>

#include "../../include/bnpp.h"
#include "model_io.hpp"

namespace bn {
namespace {

std::mutex g_mu;
bnpp_ctx *g_ctx = nullptr;
int g_device = -1;

bnpp_ctx *ctx() {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ctx) {
        int dev = g_device;
        if (dev < 0) {
            const char *e = std::getenv("BNPP_DEVICE");
            dev = e ? std::atoi(e) : 0;
        }
        if (!bnpp_abi_matches()) throw std::runtime_error("bnpp: libbnpp ABI version differs from include/bnpp.h");
        if (bnpp_ctx_create(dev, &g_ctx) != BNPP_OK)
            throw std::runtime_error(std::string("bnpp: cannot create a GPU context: ") + bnpp_last_error());
    }
    return g_ctx;
}

void check(int rc, const char *what) {
    if (rc != BNPP_OK) throw std::runtime_error(std::string("bnpp: ") + what + ": " + bnpp_last_error());
}

// RAII device buffer
struct DevBuf {
    void *p = nullptr;
    explicit DevBuf(size_t bytes) { check(bnpp_malloc(ctx(), bytes, &p), "malloc"); }
    ~DevBuf() { if (p) bnpp_free(ctx(), p); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
};

std::vector<int> ids(const Domain &d) {
    std::vector<int> v;
    for (const Variable *x : d.scope()) v.push_back((int)x->id());
    return v;
}

// cardinalities indexed by variable id, covering every listed domain
std::vector<int> cards_of(std::initializer_list<const Domain *> ds) {
    std::vector<int> c;
    for (const Domain *d : ds)
        for (const Variable *x : d->scope()) {
            if (c.size() <= x->id()) c.resize(x->id() + 1, 1);
            c[x->id()] = (int)x->size();
        }
    if (c.empty()) c.push_back(1);
    return c;
}

// sum in linear order from 0.0 (a VE result's last op is a product,
// model.cpp:423/437; a loaded table's sum as io.cpp reads it)
double seq_sum(const std::vector<double> &v) {
    double p = 0;
    for (double x : v) p += x;
    return p;
}

// an output table of n doubles
struct OutBuf : DevBuf {
    uint64_t n;
    explicit OutBuf(uint64_t n_) : DevBuf(std::max<uint64_t>(n_, 1) * sizeof(double)), n(n_) {}
};

std::vector<double> download(const OutBuf &b) {
    std::vector<double> v(std::max<uint64_t>(b.n, 1));
    check(bnpp_synchronize(ctx(), nullptr), "synchronize");
    check(bnpp_memcpy_d2h(ctx(), v.data(), b.p, v.size() * sizeof(double)), "memcpy d2h");
    v.resize(b.n);
    return v;
}

std::unique_ptr<DevBuf> upload(const std::vector<double> &v) {
    std::unique_ptr<DevBuf> b(new DevBuf(std::max<size_t>(v.size(), 1) * sizeof(double)));
    check(bnpp_memcpy_h2d(ctx(), b->p, v.data(), v.size() * sizeof(double)), "memcpy h2d");
    return b;
}

int heuristic_of(std::unordered_map<std::string, bool> &o) {      // model.cpp:360, graph.cpp:62-68
    if (o["min-degree"]) return BNPP_MIN_DEGREE;
    if (o["weighted-min-fill"]) return BNPP_WEIGHTED_MIN_FILL;
    if (o["min-fill"]) return BNPP_MIN_FILL;
    return BNPP_ORDER_GIVEN;
}

}  // namespace

void set_device(int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_device = device;
}

std::ostream &operator<<(std::ostream &o, const Variable &v) {
    return o << "Variable(id:" << v.id() << ", size:" << v.size() << ")";
}

// ----------------------------------------------------------------- Domain
Domain::Domain() { init(); }
Domain::Domain(std::vector<const Variable *> scope) : _scope(std::move(scope)) { init(); }
Domain::Domain(const Domain &d) : _scope(d._scope) { init(); }
Domain::Domain(const Domain &d1, const Domain &d2) : _scope(d1._scope) {
    for (const Variable *v : d2._scope)
        if (!d1.in_scope(v)) _scope.push_back(v);
    init();
}
Domain::Domain(const Domain &d, const Variable *v) {
    for (const Variable *x : d._scope)
        if (x != v) _scope.push_back(x);
    init();
}
Domain::Domain(const Domain &d, const std::unordered_map<unsigned, unsigned> &evidence) {
    for (const Variable *x : d._scope)
        if (!evidence.count(x->id())) _scope.push_back(x);
    init();
}
void Domain::init() {
    _offset.assign(_scope.size(), 1);
    _size = 1;
    for (int i = (int)_scope.size() - 1; i >= 0; --i) {
        _offset[i] = _size;
        _size *= _scope[i]->size();
    }
}
const Variable *Domain::operator[](unsigned i) const {
    if (i < _scope.size()) return _scope[i];
    throw "Domain::operator[unsigned i]: Index out of range!";
}
bool Domain::in_scope(const Variable *v) const { return in_scope(v->id()); }
bool Domain::in_scope(unsigned id) const {
    for (const Variable *x : _scope)
        if (x->id() == id) return true;
    return false;
}
void Domain::next_valuation(std::vector<unsigned> &val) const {
    int j;
    for (j = (int)val.size() - 1; j >= 0 && val[j] == _scope[j]->size() - 1; --j) val[j] = 0;
    if (j >= 0) val[j]++;
}
uint64_t Domain::position_valuation(const std::vector<unsigned> &val) const {
    uint64_t pos = 0;
    for (size_t i = 0; i < _scope.size(); ++i) pos += val[i] * _offset[i];
    return pos;
}
uint64_t Domain::position_consistent_valuation(const std::vector<unsigned> &val, const Domain &domain) const {
    uint64_t pos = 0;
    for (size_t i = 0; i < _scope.size(); ++i)
        for (size_t j = 0; j < domain._scope.size(); ++j)
            if (domain._scope[j]->id() == _scope[i]->id()) pos += _offset[i] * val[j];
    return pos;
}
std::ostream &operator<<(std::ostream &o, const Domain &d) {
    o << "Domain{";
    for (unsigned i = 0; i < d.width(); ++i) o << (i ? ", " : "") << d._scope[i]->id();
    return o << "}";
}

// ----------------------------------------------------------------- Factor
// A pending partition sum: `in` null -- the factor's own values in linear
// order (product / divide / conditioning: factor.cpp:129-139, 161-172,
// 226-236); otherwise sum_out's terms, the input's entries in (output entry,
// summed value) order (factor.cpp:196-208): the input seen as [hi][k][lo]
// (lo = the summed variable's stride), entry i = h * lo + l adds in[h][0..k)[l].
struct Factor::PendingSum {
    std::shared_ptr<const std::vector<double>> in;
    uint64_t k = 1, lo = 1;
};
// sum_out inputs up to this many entries (32 MiB) are copied for a lazy
// partition sum; larger ones are summed at once (a kept copy
// doubled the host memory of a large factor)
constexpr size_t kLazySumMax = size_t(1) << 22;

Factor::Factor(const Domain *domain, std::vector<double> values, double partition)
    : _domain(domain), _values(std::move(values)), _partition(partition) {}
Factor::Factor(const Domain *domain, double value)
    : _domain(domain), _values(domain->size(), value), _partition(domain->size() * value) {}
Factor::Factor(double value) : _domain(new Domain()), _values(1, value), _partition(value) {}
Factor::Factor(const Factor &f)
    : _domain(new Domain(*f._domain)), _values(f._values), _partition(f._partition), _pending(f._pending) {}
Factor::Factor(Factor &&f) noexcept
    : _domain(f._domain), _values(std::move(f._values)), _partition(f._partition), _pending(std::move(f._pending)) {
    f._domain = nullptr;
    f._partition = 0.0;
}
Factor::~Factor() { delete _domain; }
Factor &Factor::operator=(Factor &&f) noexcept {
    if (this != &f) {
        delete _domain;
        _domain = f._domain;
        _values = std::move(f._values);
        _partition = f._partition;
        _pending = std::move(f._pending);
        f._domain = nullptr;
        f._partition = 0.0;
    }
    return *this;
}
// Factor stays safe for concurrent const access (two threads reading one
// shared factor's partition()): the pending sum is resolved, and read, under
// one process-wide lock (uncontended after the first read: ~20 ns a call)
static std::mutex g_pending_mu;
void Factor::resolve_partition() const {
    std::lock_guard<std::mutex> lock(g_pending_mu);
    if (!_pending) return;
    double p = 0;                                   // sequential fp64 adds from 0.0
    if (!_pending->in) {
        for (double x : _values) p += x;
    } else {
        const std::vector<double> &in = *_pending->in;
        const uint64_t k = _pending->k, lo = _pending->lo, hi = in.size() / (k * lo);
        for (uint64_t h = 0; h < hi; ++h)
            for (uint64_t l = 0; l < lo; ++l)
                for (uint64_t v = 0; v < k; ++v) p += in[(h * k + v) * lo + l];
    }
    _partition = p;
    _pending.reset();
}
double Factor::partition() const {
    resolve_partition();
    return _partition;
}
Factor &Factor::operator=(const Factor &f) {
    if (this != &f) {
        Factor c(f);
        *this = std::move(c);
    }
    return *this;
}
Factor Factor::operator*(const Factor &f) { return product(f); }
void Factor::operator*=(const Factor &f) { *this = product(f); }
const double &Factor::operator[](uint64_t i) const {
    if (i < size()) return _values.at(i);
    throw "Factor::operator[]: Index out of range.";
}
double &Factor::operator[](uint64_t i) {
    resolve_partition();                            // the sum of the values as the op made them
    if (i < size()) return _values[i];
    throw "Factor::operator[]: Index out of range.";
}
double Factor::max() const {
    double m = 0.0;
    for (double p : _values) m = p > m ? p : m;
    return m;
}
double Factor::min() const {
    double m = partition();
    for (double p : _values) m = p < m ? p : m;
    return m;
}

Factor Factor::product(const Factor &f) const {
    Domain *nd = new Domain(*_domain, *f._domain);
    std::vector<int> cards = cards_of({_domain, f._domain});
    auto a = upload(_values), b = upload(f._values);
    OutBuf out(nd->size());
    std::vector<int> av = ids(*_domain), bv = ids(*f._domain), ov = ids(*nd);
    check(bnpp_product(ctx(), nullptr, BNPP_F64, (int)cards.size(), cards.data(), a->p, (int)av.size(), av.data(), b->p, (int)bv.size(),
                       bv.data(), out.p, (int)ov.size(), ov.data(), nullptr),
          "product");
    Factor r(nd, download(out), 0.0);
    r._pending = std::make_shared<PendingSum>();
    return r;
}

Factor Factor::divide(const Factor &f) const {
    Domain *nd = new Domain(*_domain, *f._domain);                 // same scope rule as product
    std::vector<int> cards = cards_of({_domain, f._domain});
    auto a = upload(_values), b = upload(f._values);
    OutBuf out(nd->size());
    std::vector<int> av = ids(*_domain), bv = ids(*f._domain), ov = ids(*nd);
    check(bnpp_divide(ctx(), nullptr, BNPP_F64, (int)cards.size(), cards.data(), a->p, (int)av.size(), av.data(), b->p, (int)bv.size(),
                      bv.data(), out.p, (int)ov.size(), ov.data(), nullptr),
          "divide");
    Factor r(nd, download(out), 0.0);
    r._pending = std::make_shared<PendingSum>();
    return r;
}

Factor Factor::sum_out(const Variable *variable) const {
    if (!_domain->in_scope(variable)) return Factor(*this);       // factor.cpp:185-188
    Domain *nd = new Domain(*_domain, variable);
    std::vector<int> cards = cards_of({_domain});
    auto a = upload(_values);
    OutBuf out(nd->size());
    std::vector<int> av = ids(*_domain), ov = ids(*nd);
    check(bnpp_sum_out(ctx(), nullptr, BNPP_F64, (int)cards.size(), cards.data(), a->p, (int)av.size(), av.data(), (int)variable->id(),
                       out.p, (int)ov.size(), ov.data(), nullptr),
          "sum_out");
    Factor r(nd, download(out), 0.0);
    auto ps = std::make_shared<PendingSum>();
    for (unsigned i = 0; i < _domain->width(); ++i)
        if ((*_domain)[i] == variable) {                 // removal by pointer identity (domain.cpp:57)
            ps->k = variable->size();
            ps->lo = 1;
            for (unsigned j = i + 1; j < _domain->width(); ++j) ps->lo *= (*_domain)[j]->size();
        }
    if (_values.size() > kLazySumMax) {
        // a large input: its terms summed now (the same order and bits) rather
        // than a host copy kept until partition() is read
        const uint64_t k = ps->k, lo = ps->lo, hi = _values.size() / (k * lo);
        double p = 0;
        for (uint64_t h = 0; h < hi; ++h)
            for (uint64_t l = 0; l < lo; ++l)
                for (uint64_t v = 0; v < k; ++v) p += _values[(h * k + v) * lo + l];
        r._partition = p;
        return r;
    }
    ps->in = std::make_shared<const std::vector<double>>(_values);
    r._pending = ps;
    return r;
}

Factor Factor::conditioning(const std::unordered_map<unsigned, unsigned> &evidence) const {
    Domain *nd = new Domain(*_domain, evidence);
    std::vector<int> cards = cards_of({_domain});
    std::vector<int> ev_vars, ev_vals;
    for (auto &kv : evidence) {
        ev_vars.push_back((int)kv.first);
        ev_vals.push_back((int)kv.second);
    }
    auto a = upload(_values);
    OutBuf out(nd->size());
    std::vector<int> av = ids(*_domain);
    check(bnpp_condition(ctx(), nullptr, BNPP_F64, (int)cards.size(), cards.data(), a->p, (int)av.size(), av.data(), (int)ev_vars.size(),
                         ev_vars.data(), ev_vals.data(), out.p, nullptr),
          "conditioning");
    Factor r(nd, download(out), 0.0);
    r._pending = std::make_shared<PendingSum>();
    return r;
}

Factor Factor::normalize() const {
    Factor f(*this);
    f.resolve_partition();
    for (double &v : f._values) v = v / f._partition;
    f._partition = 1.0;
    return f;
}

std::ostream &operator<<(std::ostream &os, const Factor &f) {      // factor.cpp:291-321
    const Domain &d = *f._domain;
    os << "Factor(width:" << f.width() << ", size:" << f.size() << ", partition:" << f.partition() << ")" << std::endl;
    for (unsigned i = 0; i < d.width(); ++i) os << d[i]->id() << " ";
    os << std::endl;
    std::vector<unsigned> val(d.width(), 0);
    for (uint64_t i = 0; i < f.size(); ++i) {
        for (unsigned j = 0; j < d.width(); ++j) os << val[j] << " ";
        os << ": " << std::fixed << std::setprecision(7) << f._values[i] << std::endl;
        d.next_valuation(val);
    }
    return os;
}

// ------------------------------------------------------------------ models
namespace {

bnpp_model *to_engine(const std::vector<Variable *> &vars, const std::vector<const Factor *> &factors) {
    std::vector<int> cards, widths, scopes;
    std::vector<double> values;
    for (const Variable *v : vars) {
        if (cards.size() <= v->id()) cards.resize(v->id() + 1, 1);
        cards[v->id()] = (int)v->size();
    }
    for (const Factor *f : factors) {
        widths.push_back((int)f->width());
        for (const Variable *x : f->domain().scope()) scopes.push_back((int)x->id());
        values.insert(values.end(), f->values().begin(), f->values().end());
    }
    bnpp_model *m = nullptr;
    check(bnpp_model_from_arrays(0, (int)cards.size(), cards.data(), (int)factors.size(), widths.data(), scopes.data(),
                                 values.data(), &m),
          "model");
    return m;
}

struct ModelGuard {
    bnpp_model *m;
    ~ModelGuard() { bnpp_model_free(m); }
};

void split_evidence(const std::unordered_map<unsigned, unsigned> &ev, std::vector<int> &vars, std::vector<int> &vals) {
    for (auto &kv : ev) {
        vars.push_back((int)kv.first);
        vals.push_back((int)kv.second);
    }
}

}  // namespace

Model::Model(std::string name, std::vector<Variable *> &variables, std::vector<Factor *> &factors)
    : _name(std::move(name)), _variables(variables), _factors(factors) {}

Model::~Model() {
    for (auto pv : _variables) delete pv;
    for (auto pf : _factors) delete pf;
}

double Model::log10_partition(const std::unordered_map<unsigned, unsigned> &evidence,
                              std::unordered_map<std::string, bool> &options, double &uptime) const {
    auto t0 = std::chrono::steady_clock::now();
    ModelGuard g{to_engine(_variables, std::vector<const Factor *>(_factors.begin(), _factors.end()))};
    std::vector<int> ev_vars, ev_vals;
    split_evidence(evidence, ev_vars, ev_vals);
    double lz = 0, z = 0, up = 0;
    int dt = options["fp32"] ? BNPP_F32 : BNPP_F64;
    check(bnpp_partition(ctx(), g.m, (int)ev_vars.size(), ev_vars.data(), ev_vals.data(), heuristic_of(options),
                         nullptr, 0, dt, &lz, &z, &up),
          "partition");
    uptime = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return lz;
}

double Model::partition(const std::unordered_map<unsigned, unsigned> &evidence,
                        std::unordered_map<std::string, bool> &options, double &uptime) const {
    auto t0 = std::chrono::steady_clock::now();
    ModelGuard g{to_engine(_variables, std::vector<const Factor *>(_factors.begin(), _factors.end()))};
    std::vector<int> ev_vars, ev_vals;
    split_evidence(evidence, ev_vars, ev_vals);
    double lz = 0, z = 0, up = 0;
    int dt = options["fp32"] ? BNPP_F32 : BNPP_F64;
    check(bnpp_partition(ctx(), g.m, (int)ev_vars.size(), ev_vars.data(), ev_vals.data(), heuristic_of(options),
                         nullptr, 0, dt, &lz, &z, &up),
          "partition");
    uptime = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return z;                                        // part.partition() (model.cpp:289)
}

std::vector<const Factor *> Model::marginals(const std::unordered_map<unsigned, unsigned> &evidence,
                                             std::unordered_map<std::string, bool> &options, double &uptime) const {
    auto t0 = std::chrono::steady_clock::now();
    ModelGuard g{to_engine(_variables, std::vector<const Factor *>(_factors.begin(), _factors.end()))};
    std::vector<int> ev_vars, ev_vals;
    split_evidence(evidence, ev_vars, ev_vals);
    size_t total = 0;
    for (auto pv : _variables) total += pv->size();
    std::vector<double> out(total);
    std::vector<int> targets;
    for (auto pv : _variables) targets.push_back((int)pv->id());
    double up = 0;
    int dt = options["fp32"] ? BNPP_F32 : BNPP_F64;
    const bool sp = options["sum-product"];
    if (sp) {                                        // loopy BP, evidence unused (model.cpp:313-317, 749)
        int it = 0;
        check(bnpp_sum_product(ctx(), g.m, 10000, 0.001, out.data(), &it, &up), "marginals (sum-product)");
    } else if (options["bucket-tree"])               // all marginals from one bucket tree (to rounding)
        check(bnpp_marginals_tree(ctx(), g.m, (int)ev_vars.size(), ev_vars.data(), ev_vals.data(),
                                  heuristic_of(options), nullptr, 0, (int)targets.size(), targets.data(), dt,
                                  out.data(), &up),
              "marginals (bucket tree)");
    else                                             // one VE per target, bit-exact (model.cpp:326-334)
        check(bnpp_marginals(ctx(), g.m, (int)ev_vars.size(), ev_vars.data(), ev_vals.data(), heuristic_of(options),
                             (int)targets.size(), targets.data(), dt, out.data(), &up),
              "marginals");
    std::vector<const Factor *> marg;
    size_t o = 0;
    for (auto pv : _variables) {
        if (!sp && evidence.count(pv->id())) {        // width-0 factor with value 1 (model.cpp:333)
            marg.push_back(new Factor(new Domain(), std::vector<double>{1.0}, 1.0));
        } else {
            std::vector<double> v(out.begin() + o, out.begin() + o + pv->size());
            marg.push_back(new Factor(new Domain(std::vector<const Variable *>{pv}), v, 1.0));
        }
        o += pv->size();
    }
    uptime = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return marg;
}

BN::BN(std::string name, std::vector<Variable *> &variables, std::vector<Factor *> &factors)
    : Model(std::move(name), variables, factors) {
    for (auto pv : _variables) _children[pv] = {};
    for (size_t i = 0; i < _variables.size() && i < _factors.size(); ++i) {   // model.cpp:111-119
        const Variable *v = _variables[i];
        std::vector<const Variable *> scope = _factors[i]->domain().scope();
        std::unordered_set<const Variable *> parents;
        if (!scope.empty()) parents.insert(scope.begin() + 1, scope.end());
        _parents[v] = parents;
        for (auto p : parents) _children[p].insert(v);
    }
}

Factor BN::variable_elimination(std::vector<const Variable *> &variables, std::vector<const Factor *> &factors,
                                std::unordered_map<std::string, bool> &options) const {
    ModelGuard g{to_engine(_variables, factors)};
    std::vector<int> vars;
    for (auto pv : variables) vars.push_back((int)pv->id());
    int cap_vars = (int)_variables.size() + 1;
    std::vector<int> out_vars(cap_vars);
    int ndims = 0;
    int64_t size = 0, exp2 = 0;
    // the result scope is what no bucket eliminated: at most every variable
    uint64_t cap = 1;
    for (auto f : factors) cap = std::max<uint64_t>(cap, f->size());
    std::vector<double> vals;
    int dt = options["fp32"] ? BNPP_F32 : BNPP_F64;
    int h = heuristic_of(options);
    for (;;) {
        vals.assign(cap, 0.0);
        int rc = bnpp_variable_elimination(ctx(), g.m, (int)vars.size(), vars.data(), h, dt, cap_vars, &ndims,
                                           out_vars.data(), (int64_t)cap, &size, vals.data(), &exp2);
        if (rc == BNPP_OK) break;
        if ((uint64_t)size > cap) { cap = (uint64_t)size; continue; }
        check(rc, "variable_elimination");
    }
    vals.resize((size_t)size);
    for (double &v : vals) v = std::ldexp(v, (int)exp2);
    std::vector<const Variable *> scope;
    for (int i = 0; i < ndims; ++i)
        for (auto pv : _variables)
            if ((int)pv->id() == out_vars[i]) scope.push_back(pv);
    double p = seq_sum(vals);
    return Factor(new Domain(scope), std::move(vals), p);
}

Factor BN::query_ve(const std::unordered_set<const Variable *> &target,
                    const std::unordered_set<const Variable *> &evidence,
                    std::unordered_map<std::string, bool> &options, double &uptime) const {
    // model.cpp:205-248: VE over every variable neither queried nor observed,
    // then P(target | evidence) = f / sum_target f.  (options["bayes-ball"]
    // only prunes non-requisite nodes there; the result is the same table.)
    auto t0 = std::chrono::steady_clock::now();
    std::vector<const Variable *> variables;
    std::vector<const Factor *> factors;
    for (auto pv : _variables) {
        if (!target.count(pv) && !evidence.count(pv)) variables.push_back(pv);
        factors.push_back(_factors[pv->id()]);
    }
    Factor f = variable_elimination(variables, factors, options);
    if (!evidence.empty()) {
        Factor g = f;
        for (auto pv : target) g = g.sum_out(pv);
        f = f.divide(g);
    }
    uptime = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return f;
}

MN::MN(std::string name, std::vector<Variable *> &variables, std::vector<Factor *> &factors)
    : Model(std::move(name), variables, factors) {
    for (auto pv : _variables) _neighbors[pv];                     // model.cpp:962-977
    for (auto pf : _factors) {
        const std::vector<const Variable *> &scope = pf->domain().scope();
        for (auto pv1 : scope)
            for (auto pv2 : scope)
                if (pv1->id() != pv2->id()) _neighbors[pv1].insert(pv2);
    }
}

void MN::write(std::ostream &os) const {                            // model.cpp:979-999
    os << "MARKOV:" << std::endl;
    os << ">> Variables" << std::endl;
    for (auto pv1 : _variables) {
        os << *pv1 << ", ";
        os << "neighbors:{";
        for (auto pv2 : _neighbors.find(pv1)->second) os << " " << pv2->id();
        os << " }" << std::endl;
    }
    os << std::endl;
    os << ">> Factors" << std::endl;
    for (auto pf : _factors) os << *pf << std::endl;
}

std::ostream &operator<<(std::ostream &os, const MN &mn) {
    mn.write(os);
    return os;
}

// -------------------------------------------------------------------- I/O
namespace {
int read_any(std::string &filename, bnpp::ModelData &d) {
    std::string err;
    int rc = bnpp::load_uai(filename, d, &err);
    if (rc) std::cerr << "Error: " << err << std::endl;
    return rc;
}
void materialise(const bnpp::ModelData &d, std::vector<Variable *> &vars, std::vector<Factor *> &factors) {
    for (size_t i = 0; i < d.cards.size(); ++i) vars.push_back(new Variable((unsigned)i, (unsigned)d.cards[i]));
    for (size_t f = 0; f < d.scopes.size(); ++f) {
        std::vector<const Variable *> scope;
        for (int v : d.scopes[f]) scope.push_back(vars[v]);
        double p = seq_sum(d.values[f]);
        factors.push_back(new Factor(new Domain(scope), d.values[f], p));
    }
}
}  // namespace

int read_uai_model(std::string &filename, BN **model) {            // io.cpp:102-127
    bnpp::ModelData d;
    int rc = read_any(filename, d);
    if (rc) return rc;
    if (!d.is_bayes) {
        std::cerr << "Error: file " << filename << " is not a BAYES net." << std::endl;
        return -2;
    }
    std::vector<Variable *> vars;
    std::vector<Factor *> factors;
    materialise(d, vars, factors);
    *model = new BN(filename, vars, factors);
    return 0;
}

int read_uai_model(std::string &filename, MN **model) {            // io.cpp:129-154
    bnpp::ModelData d;
    int rc = read_any(filename, d);
    if (rc) return rc;
    if (d.is_bayes) {
        std::cerr << "Error: file " << filename << " is not a MARKOV net." << std::endl;
        return -2;
    }
    std::vector<Variable *> vars;
    std::vector<Factor *> factors;
    materialise(d, vars, factors);
    *model = new MN(filename, vars, factors);
    return 0;
}

int read_uai_evidence(std::string &filename, std::unordered_map<unsigned, unsigned> &evidence) {   // io.cpp:157-180
    std::vector<std::pair<int, int>> ev;
    if (bnpp::load_evidence(filename, ev)) {
        std::cerr << "Error: couldn't read file " << filename << std::endl;
        return -1;
    }
    for (auto &p : ev) evidence[(unsigned)p.first] = (unsigned)p.second;
    return 0;
}

}  // namespace bn
