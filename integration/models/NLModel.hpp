// NLModel.hpp -- an ASL-free reader of AMPL .nl files (text "g" format) as a uno::Model, so the
// reference Uno core runs the reference's own example inputs (examples/hs015.nl, examples/polak5.nl)
// without the AMPL Solver Library (absent here and on the GPU box).  SURVEY.md 8(f) item 1.
//
// Conventions follow bindings/AMPL/AMPLModel.cpp:
//   - objective sign: -1 when maximizing (AMPLModel.cpp:47), gradient and value scaled by it (:75-93);
//   - Lagrangian Hessian sigma * grad^2 f - sum_j y_j grad^2 c_j (lagscale -1, :39), upper triangle,
//     column-major, rows ascending inside a column (Sphset uptri = 1, :357-368; insertion loop :171-178);
//   - constraint gradients sparse in the order of the J segment (Cgrad lists, :118-137), Jacobian
//     nonzeros = nzc of the header (:300-302);
//   - constraints ordered nonlinear first, linear constraints = [nlc, m) (:51-52);
//   - variable / constraint partitions of AMPLModel.cpp:308-347.
// Derivatives: every nonlinear expression is evaluated with second-order forward mode over its own
// variables (value, gradient, dense Hessian of the expression's variables) -- exact, and cheap for the
// small example models.  The Hessian pattern is the union over the nonlinear expressions of their
// variables' pairs (ASL's Sphset detects finer partially separable patterns; on the reference
// examples both give the full upper triangle of the nonlinear variables).
// Supported: operators + - * / ^ unary-minus abs sqrt sin cos exp log sumlist, numbers, variables;
// segments C O r b x d k J G.  Anything else (common expressions, imported functions, suffixes,
// logical operators, discrete variables) is rejected with an error.
#ifndef UNO_KKT_NLMODEL_H
#define UNO_KKT_NLMODEL_H

#include <algorithm>
#include <cmath>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>
#include "linear_algebra/RectangularMatrix.hpp"
#include "linear_algebra/SparseVector.hpp"
#include "linear_algebra/SymmetricMatrix.hpp"
#include "linear_algebra/Vector.hpp"
#include "model/Model.hpp"
#include "symbolic/CollectionAdapter.hpp"
#include "symbolic/Range.hpp"
#include "tools/Infinity.hpp"

namespace uno {
   namespace nl {
      // expression node in .nl prefix form
      struct Node {
         int op = -1;        // -1 number, -2 variable, else the .nl operator code
         double value = 0.;  // number
         size_t var = 0;     // variable
         std::vector<std::unique_ptr<Node>> args;
      };

      // value, gradient and Hessian of an expression over its local variables (size k)
      struct Taylor {
         double v = 0.;
         std::vector<double> g, H;  // g[k], H[k*k] (symmetric, full)
         explicit Taylor(size_t k = 0): g(k, 0.), H(k * k, 0.) {}
      };

      class Reader {
      public:
         explicit Reader(const std::string& path): in(path) {
            if (!in) throw std::runtime_error("cannot open " + path);
         }
         std::string line() {
            std::string s;
            if (!std::getline(in, s)) throw std::runtime_error(".nl: unexpected end of file");
            const size_t hash = s.find('#');
            if (hash != std::string::npos) s = s.substr(0, hash);
            return s;
         }
         bool next_segment(std::string& s) {
            while (std::getline(in, s)) {
               if (!s.empty()) return true;
            }
            return false;
         }
         std::unique_ptr<Node> expr() {
            std::string s = line();
            std::istringstream is(s);
            std::string tok;
            is >> tok;
            if (tok.empty()) throw std::runtime_error(".nl: empty expression line");
            auto node = std::make_unique<Node>();
            const char c = tok[0];
            if (c == 'n') {
               node->op = -1;
               node->value = std::stod(tok.substr(1));
            }
            else if (c == 'v') {
               node->op = -2;
               node->var = std::stoul(tok.substr(1));
            }
            else if (c == 'o') {
               node->op = std::stoi(tok.substr(1));
               int arity;
               switch (node->op) {
                  case 0: case 1: case 2: case 3: case 5: arity = 2; break;
                  case 15: case 16: case 39: case 41: case 43: case 44: case 46: arity = 1; break;
                  case 54: {  // sumlist: count on the next line
                     std::string cnt = line();
                     arity = std::stoi(cnt);
                     break;
                  }
                  default: throw std::runtime_error(".nl: unsupported operator o" + std::to_string(node->op));
               }
               for (int a = 0; a < arity; ++a) node->args.push_back(this->expr());
            }
            else {
               throw std::runtime_error(".nl: unsupported expression token " + tok);
            }
            return node;
         }
         std::ifstream in;
      };

      inline void collect_vars(const Node& n, std::set<size_t>& vars) {
         if (n.op == -2) vars.insert(n.var);
         for (const auto& a: n.args) collect_vars(*a, vars);
      }

      // second-order forward mode over the local variables `loc` (global index -> local position)
      inline Taylor eval(const Node& n, const double* x, const std::map<size_t, size_t>& loc) {
         const size_t k = loc.size();
         Taylor r(k);
         auto unary = [&](const Taylor& a, double f, double f1, double f2) {
            r.v = f;
            for (size_t i = 0; i < k; ++i) r.g[i] = f1 * a.g[i];
            for (size_t i = 0; i < k; ++i)
               for (size_t j = 0; j < k; ++j) r.H[i * k + j] = f1 * a.H[i * k + j] + f2 * a.g[i] * a.g[j];
         };
         auto times = [&](const Taylor& a, const Taylor& b) {
            Taylor t(k);
            t.v = a.v * b.v;
            for (size_t i = 0; i < k; ++i) t.g[i] = a.g[i] * b.v + a.v * b.g[i];
            for (size_t i = 0; i < k; ++i)
               for (size_t j = 0; j < k; ++j)
                  t.H[i * k + j] = a.H[i * k + j] * b.v + a.v * b.H[i * k + j] + a.g[i] * b.g[j] + b.g[i] * a.g[j];
            return t;
         };
         switch (n.op) {
            case -1: r.v = n.value; return r;
            case -2: r.v = x[n.var]; r.g[loc.at(n.var)] = 1.; return r;
            case 0: case 1: case 54: {
               for (size_t a = 0; a < n.args.size(); ++a) {
                  const Taylor t = eval(*n.args[a], x, loc);
                  const double s = (n.op == 1 && a == 1) ? -1. : 1.;
                  r.v += s * t.v;
                  for (size_t i = 0; i < k; ++i) r.g[i] += s * t.g[i];
                  for (size_t i = 0; i < k * k; ++i) r.H[i] += s * t.H[i];
               }
               return r;
            }
            case 2: return times(eval(*n.args[0], x, loc), eval(*n.args[1], x, loc));
            case 3: {
               const Taylor b = eval(*n.args[1], x, loc);
               Taylor inv(k);
               const double ib = 1. / b.v;
               inv.v = ib;
               for (size_t i = 0; i < k; ++i) inv.g[i] = -ib * ib * b.g[i];
               for (size_t i = 0; i < k; ++i)
                  for (size_t j = 0; j < k; ++j)
                     inv.H[i * k + j] = -ib * ib * b.H[i * k + j] + 2. * ib * ib * ib * b.g[i] * b.g[j];
               return times(eval(*n.args[0], x, loc), inv);
            }
            case 5: {
               const Taylor a = eval(*n.args[0], x, loc);
               if (n.args[1]->op == -1) {  // constant exponent
                  const double c = n.args[1]->value;
                  unary(a, std::pow(a.v, c), c * std::pow(a.v, c - 1.), c * (c - 1.) * std::pow(a.v, c - 2.));
                  return r;
               }
               // a^b = exp(b log a)
               const Taylor b = eval(*n.args[1], x, loc);
               Taylor la(k);
               la.v = std::log(a.v);
               for (size_t i = 0; i < k; ++i) la.g[i] = a.g[i] / a.v;
               for (size_t i = 0; i < k; ++i)
                  for (size_t j = 0; j < k; ++j) la.H[i * k + j] = a.H[i * k + j] / a.v - a.g[i] * a.g[j] / (a.v * a.v);
               const Taylor e = times(b, la);
               const double ev = std::exp(e.v);
               unary(e, ev, ev, ev);
               return r;
            }
            case 15: { const Taylor a = eval(*n.args[0], x, loc); const double s = a.v < 0. ? -1. : 1.; unary(a, std::fabs(a.v), s, 0.); return r; }
            case 16: { const Taylor a = eval(*n.args[0], x, loc); unary(a, -a.v, -1., 0.); return r; }
            case 39: { const Taylor a = eval(*n.args[0], x, loc); const double s = std::sqrt(a.v); unary(a, s, 0.5 / s, -0.25 / (s * a.v)); return r; }
            case 41: { const Taylor a = eval(*n.args[0], x, loc); unary(a, std::sin(a.v), std::cos(a.v), -std::sin(a.v)); return r; }
            case 43: { const Taylor a = eval(*n.args[0], x, loc); unary(a, std::log(a.v), 1. / a.v, -1. / (a.v * a.v)); return r; }
            case 44: { const Taylor a = eval(*n.args[0], x, loc); const double e = std::exp(a.v); unary(a, e, e, e); return r; }
            case 46: { const Taylor a = eval(*n.args[0], x, loc); unary(a, std::cos(a.v), -std::sin(a.v), -std::cos(a.v)); return r; }
            default: throw std::runtime_error(".nl: operator o" + std::to_string(n.op));
         }
      }

      // one function: linear part + optional nonlinear expression over its variables
      struct Function {
         std::vector<std::pair<size_t, double>> linear;  // (variable, coefficient), .nl order
         std::unique_ptr<Node> expr;
         std::vector<size_t> vars;                       // the expression's variables, ascending
         std::map<size_t, size_t> loc;
         void finish() {
            std::set<size_t> s;
            if (expr) collect_vars(*expr, s);
            vars.assign(s.begin(), s.end());
            for (size_t i = 0; i < vars.size(); ++i) loc[vars[i]] = i;
         }
         Taylor nonlinear(const double* x) const { return expr ? eval(*expr, x, loc) : Taylor(0); }
         double value(const double* x) const {
            double v = expr ? eval(*expr, x, loc).v : 0.;
            for (const auto& [j, a]: linear) v += a * x[j];
            return v;
         }
      };
   } // namespace nl

   class NLModel : public Model {
   public:
      explicit NLModel(const std::string& path): NLModel(path, read_header(path)) {}

      [[nodiscard]] double evaluate_objective(const Vector<double>& x) const override {
         return this->n_obj ? this->objective_sign * this->objective.value(x.data()) : 0.;
      }
      void evaluate_objective_gradient(const Vector<double>& x, Vector<double>& gradient) const override {
         for (size_t i = 0; i < this->number_variables; ++i) gradient[i] = 0.;
         if (!this->n_obj) return;
         for (const auto& [j, a]: this->objective.linear) gradient[j] += a;
         const nl::Taylor t = this->objective.nonlinear(x.data());
         for (size_t i = 0; i < this->objective.vars.size(); ++i) gradient[this->objective.vars[i]] += t.g[i];
         for (size_t i = 0; i < this->number_variables; ++i) gradient[i] *= this->objective_sign;
      }
      void evaluate_constraints(const Vector<double>& x, std::vector<double>& constraints) const override {
         for (size_t j = 0; j < this->number_constraints; ++j) constraints[j] = this->cons[j].value(x.data());
      }
      void evaluate_constraint_gradient(const Vector<double>& x, size_t j, SparseVector<double>& gradient) const override {
         gradient.clear();
         const nl::Function& c = this->cons[j];
         const nl::Taylor t = c.nonlinear(x.data());
         for (const auto& [v, a]: c.linear) {  // every Jacobian entry of the J segment, in its order
            const auto it = c.loc.find(v);
            gradient.insert(v, a + (it != c.loc.end() ? t.g[it->second] : 0.));
         }
      }
      void evaluate_constraint_jacobian(const Vector<double>& x, RectangularMatrix<double>& jacobian) const override {
         for (size_t j = 0; j < this->number_constraints; ++j) this->evaluate_constraint_gradient(x, j, jacobian[j]);
      }
      void evaluate_lagrangian_hessian(const Vector<double>& x, double objective_multiplier, const Vector<double>& multipliers,
            SymmetricMatrix<size_t, double>& hessian) const override {
         std::vector<double> values(this->hpattern.size(), 0.);
         this->accumulate_hessian(x.data(), objective_multiplier * this->objective_sign, multipliers, values);
         size_t q = 0;
         for (size_t col = 0; col < this->number_variables; ++col) {
            for (; q < this->hpattern.size() && this->hpattern[q].second == col; ++q) {
               hessian.insert(this->hpattern[q].first, col, values[q]);
            }
            hessian.finalize_column(col);
         }
      }
      void compute_hessian_vector_product(const double* v, double objective_multiplier, const Vector<double>& multipliers,
            double* result) const override {
         // the Hessian at the point of the last Lagrangian evaluation is not kept (AMPL's Hvcomp uses the
         // last point ASL saw); the ipopt preset never calls this
         (void)v; (void)objective_multiplier; (void)multipliers; (void)result;
         throw std::runtime_error("NLModel::compute_hessian_vector_product is not used by the ipopt preset");
      }

      [[nodiscard]] double variable_lower_bound(size_t i) const override { return this->lv[i]; }
      [[nodiscard]] double variable_upper_bound(size_t i) const override { return this->uv[i]; }
      [[nodiscard]] const Collection<size_t>& get_lower_bounded_variables() const override { return this->lower_c; }
      [[nodiscard]] const Collection<size_t>& get_upper_bounded_variables() const override { return this->upper_c; }
      [[nodiscard]] const SparseVector<size_t>& get_slacks() const override { return this->slacks; }
      [[nodiscard]] const Collection<size_t>& get_single_lower_bounded_variables() const override { return this->single_lower_c; }
      [[nodiscard]] const Collection<size_t>& get_single_upper_bounded_variables() const override { return this->single_upper_c; }
      [[nodiscard]] const Vector<size_t>& get_fixed_variables() const override { return this->fixed; }
      [[nodiscard]] double constraint_lower_bound(size_t j) const override { return this->lc[j]; }
      [[nodiscard]] double constraint_upper_bound(size_t j) const override { return this->uc[j]; }
      [[nodiscard]] const Collection<size_t>& get_equality_constraints() const override { return this->equality_c; }
      [[nodiscard]] const Collection<size_t>& get_inequality_constraints() const override { return this->inequality_c; }
      [[nodiscard]] const Collection<size_t>& get_linear_constraints() const override { return this->linear_constraints; }
      void initial_primal_point(Vector<double>& x) const override { std::copy(this->x0.begin(), this->x0.end(), x.begin()); }
      void initial_dual_point(Vector<double>& y) const override { std::copy(this->y0.begin(), this->y0.end(), y.begin()); }
      void postprocess_solution(Iterate&, IterateStatus) const override {}
      [[nodiscard]] size_t number_jacobian_nonzeros() const override { return this->nzc; }
      [[nodiscard]] size_t number_hessian_nonzeros() const override { return this->hpattern.size(); }

   private:
      struct Header {
         size_t n = 0, m = 0, nobj = 0, nlc = 0, nzc = 0;
         double sign = 1.;  // objective sense of the O segment (1: maximize -> -1)
      };
      static Header read_header(const std::string& path) {
         nl::Reader r(path);
         const std::string first = r.line();
         if (first.empty() || first[0] != 'g') throw std::runtime_error(path + ": only text (g) .nl files are supported");
         Header h;
         std::istringstream l1(r.line());
         size_t ranges = 0, eqns = 0;
         l1 >> h.n >> h.m >> h.nobj >> ranges >> eqns;
         std::istringstream l2(r.line());
         l2 >> h.nlc;
         std::string s;
         while (r.next_segment(s)) {
            if (s[0] == 'O') {
               std::istringstream is(s.substr(1));
               int index = 0, sense = 0;
               is >> index >> sense;
               h.sign = sense == 1 ? -1. : 1.;
               break;
            }
         }
         return h;
      }

      NLModel(const std::string& path, const Header& h):
            Model(path, h.n, h.m, h.sign), n_obj(h.nobj), nzc(0), cons(h.m), x0(h.n, 0.), y0(h.m, 0.),
            lv(h.n, -INF<double>), uv(h.n, INF<double>), lc(h.m, -INF<double>), uc(h.m, INF<double>),
            lower_c(this->lower), upper_c(this->upper), single_lower_c(this->single_lower), single_upper_c(this->single_upper),
            equality_c(this->equality), inequality_c(this->inequality), linear_constraints(h.nlc, h.m) {
         if (h.nobj > 1) throw std::runtime_error(path + ": more than one objective");
         nl::Reader r(path);
         std::vector<std::string> head;
         for (int q = 0; q < 10; ++q) head.push_back(r.line());
         {
            std::istringstream d(head[6]);  // discrete variables: binary, integer, nonlinear (b, c, o)
            size_t a = 0, s = 0;
            while (d >> a) s += a;
            if (s) throw std::runtime_error(path + ": discrete variables are not supported");
            std::istringstream z(head[7]);
            z >> this->nzc;
            std::istringstream ce(head[9]);  // common expressions
            s = 0;
            while (ce >> a) s += a;
            if (s) throw std::runtime_error(path + ": common expressions (defined variables) are not supported");
         }
         std::string seg;
         while (r.next_segment(seg)) {
            std::istringstream is(seg);
            std::string tag;
            is >> tag;
            const char c = tag[0];
            if (c == 'C') {
               this->cons.at(std::stoul(tag.substr(1))).expr = r.expr();
            }
            else if (c == 'O') {
               this->objective.expr = r.expr();  // sense read by read_header (objective_sign is const)
               if (this->objective.expr->op == -1 && this->objective.expr->value == 0.) this->objective.expr.reset();
            }
            else if (c == 'x' || c == 'd') {
               const size_t k = std::stoul(tag.substr(1));
               for (size_t q = 0; q < k; ++q) {
                  std::istringstream e(r.line());
                  size_t i;
                  double v;
                  e >> i >> v;
                  (c == 'x' ? this->x0 : this->y0).at(i) = v;
               }
            }
            else if (c == 'r' || c == 'b') {
               const size_t cnt = c == 'r' ? this->number_constraints : this->number_variables;
               std::vector<double>& lo = c == 'r' ? this->lc : this->lv;
               std::vector<double>& up = c == 'r' ? this->uc : this->uv;
               for (size_t q = 0; q < cnt; ++q) {
                  std::istringstream e(r.line());
                  int type;
                  double a = 0., b = 0.;
                  e >> type;
                  switch (type) {
                     case 0: e >> a >> b; lo[q] = a; up[q] = b; break;  // a <= body <= b
                     case 1: e >> b; up[q] = b; break;                  // body <= b
                     case 2: e >> a; lo[q] = a; break;                  // a <= body
                     case 3: break;                                     // free
                     case 4: e >> a; lo[q] = up[q] = a; break;          // body = a
                     default: throw std::runtime_error(path + ": complementarity constraints are not supported");
                  }
               }
            }
            else if (c == 'k') {
               const size_t k = std::stoul(tag.substr(1));
               for (size_t q = 0; q < k; ++q) r.line();  // column counts: implied by the J segments
            }
            else if (c == 'J' || c == 'G') {
               size_t idx = std::stoul(tag.substr(1)), k = 0;
               is >> k;
               nl::Function& f = c == 'J' ? this->cons.at(idx) : this->objective;
               for (size_t q = 0; q < k; ++q) {
                  std::istringstream e(r.line());
                  size_t v;
                  double a;
                  e >> v >> a;
                  f.linear.emplace_back(v, a);
               }
            }
            else {
               throw std::runtime_error(path + ": unsupported .nl segment " + tag);
            }
         }
         for (auto& f: this->cons) f.finish();
         this->objective.finish();
         // Hessian pattern: upper triangle, column-major, rows ascending (Sphset uptri = 1)
         std::set<std::pair<size_t, size_t>> pat;  // (column, row)
         auto add = [&](const nl::Function& f) {
            for (size_t a: f.vars)
               for (size_t b: f.vars)
                  if (a <= b) pat.emplace(b, a);
         };
         add(this->objective);
         for (const auto& f: this->cons) add(f);
         for (const auto& [col, row]: pat) this->hpattern.emplace_back(row, col);
         // partitions (AMPLModel.cpp:308-347)
         for (size_t i = 0; i < this->number_variables; ++i) {
            const double l = this->lv[i], u = this->uv[i];
            if (l == u) this->fixed.emplace_back(i);
            else if (is_finite(l) && is_finite(u)) { this->lower.push_back(i); this->upper.push_back(i); }
            else if (is_finite(l)) { this->lower.push_back(i); this->single_lower.push_back(i); }
            else if (is_finite(u)) { this->upper.push_back(i); this->single_upper.push_back(i); }
         }
         for (size_t j = 0; j < this->number_constraints; ++j) {
            if (this->lc[j] == this->uc[j]) this->equality.push_back(j);
            else this->inequality.push_back(j);
         }
      }

      void accumulate_hessian(const double* x, double sigma, const Vector<double>& y, std::vector<double>& values) const {
         auto add = [&](const nl::Function& f, double w) {
            if (!f.expr || w == 0.) return;
            const nl::Taylor t = f.nonlinear(x);
            const size_t k = f.vars.size();
            for (size_t a = 0; a < k; ++a)
               for (size_t b = a; b < k; ++b) {
                  const auto key = std::make_pair(f.vars[a], f.vars[b]);  // (row, column), row <= column
                  const auto it = std::lower_bound(this->hpattern.begin(), this->hpattern.end(), key,
                     [](const auto& p, const auto& q) { return p.second != q.second ? p.second < q.second : p.first < q.first; });
                  values[static_cast<size_t>(it - this->hpattern.begin())] += w * t.H[a * k + b];
               }
         };
         add(this->objective, sigma);
         for (size_t j = 0; j < this->number_constraints; ++j) add(this->cons[j], -y[j]);  // lagscale -1
      }

      size_t n_obj;
      size_t nzc;
      nl::Function objective;
      std::vector<nl::Function> cons;
      std::vector<double> x0, y0, lv, uv, lc, uc;
      std::vector<std::pair<size_t, size_t>> hpattern;  // (row, column)
      std::vector<size_t> lower, upper, single_lower, single_upper, equality, inequality;
      CollectionAdapter<std::vector<size_t>&> lower_c, upper_c, single_lower_c, single_upper_c, equality_c, inequality_c;
      ForwardRange linear_constraints;
      SparseVector<size_t> slacks{};
      Vector<size_t> fixed{};
   };
} // namespace

#endif
