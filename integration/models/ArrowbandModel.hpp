// ArrowbandModel.hpp -- the synthetic "arrowband" NLP as a uno::Model, so the reference
// Uno core runs a whole ipopt-preset solve (configs[1]: N = 1e4) through the KKT plugin:
//
//   min  1/2 x^T H x + g^T x    s.t.  A x = b,  -10 <= x <= 10
//
// with nv = 3N/4 variables and m = N - nv equality constraints, H banded (half-width 12, H_ii in
// [-1, 3]: indefinite, so the inertia-correction loop of PrimalDualRegularization.hpp:133-219 runs),
// constraint j on the 28 variables starting at min(3j, nv - 34) plus the last 6 ("arrow") variables,
// entries +-[0.5, 1.5], b = A x* for a point x* inside the box (feasible).  Its KKT matrices have the
// pattern of uno_amd/csrc/arrowband.c (the bench / parity generator): Hessian band, barrier diagonal
// on every variable, J^T with the arrow columns.  Values from splitmix64 (portable, seed fixed).
// Conventions of AMPLModel.cpp: Hessian upper triangle, column-major; constraint gradients sparse in
// ascending variable order (the window, then the arrow).
#ifndef UNO_KKT_ARROWBANDMODEL_H
#define UNO_KKT_ARROWBANDMODEL_H

#include <algorithm>
#include <cstdint>
#include <stdexcept>
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
   class ArrowbandModel : public Model {
   public:
      static constexpr size_t band = 12, window = 28, arrow = 6;

      // inequality = true: -1 <= A x - b <= 1 instead of A x = b (the ipopt preset adds slacks:
      // the inequality-constrained KKT structure of SURVEY.md 8(f) item 4's fallback measurement)
      explicit ArrowbandModel(size_t N, bool inequality = false, uint64_t seed = 0x5EED0002ull):
            Model((inequality ? "arrowband_ineq" : "arrowband") + std::to_string(N), (3 * N) / 4, N - (3 * N) / 4, 1.),
            inequality(inequality), all_collection(this->all), empty_collection(this->empty),
            equality_collection(this->equalities), inequality_collection(this->inequalities),
            linear_constraints(0, N - (3 * N) / 4) {
         const size_t nv = this->number_variables, m = this->number_constraints;
         if (nv < window + arrow + 1 || m < 1) throw std::invalid_argument("arrowband: N too small");
         uint64_t s = seed;
         // Hessian band: hcol[c] = rows max(0, c - band) .. c of column c (upper triangle, column-major)
         this->hcol_start.resize(nv + 1, 0);
         for (size_t c = 0; c < nv; ++c) {
            const size_t r0 = c > band ? c - band : 0;
            for (size_t r = r0; r <= c; ++r) {
               const double u = unif(s);
               this->hval.push_back(r == c ? -1. + 4. * u : (u - 0.5) / 12.);
            }
            this->hcol_start[c + 1] = this->hval.size();
         }
         this->g.resize(nv);
         for (size_t i = 0; i < nv; ++i) this->g[i] = 2. * unif(s) - 1.;
         // constraint rows (ascending variables) and b = A x*
         std::vector<double> xstar(nv);
         for (size_t i = 0; i < nv; ++i) xstar[i] = 4. * unif(s) - 2.;
         this->rows.resize(m);
         this->b.resize(m);
         for (size_t j = 0; j < m; ++j) {
            size_t start = std::min(3 * j, nv - arrow - window);
            double bj = 0.;
            for (size_t t = 0; t < window + arrow; ++t) {
               const size_t v = t < window ? start + t : nv - arrow + (t - window);
               const double mag = 0.5 + unif(s);
               const double a = unif(s) < 0.5 ? -mag : mag;
               this->rows[j].emplace_back(v, a);
               bj += a * xstar[v];
            }
            this->b[j] = bj;
         }
         for (size_t i = 0; i < nv; ++i) this->all.push_back(i);
         for (size_t j = 0; j < m; ++j) (inequality ? this->inequalities : this->equalities).push_back(j);
      }

      [[nodiscard]] double evaluate_objective(const Vector<double>& x) const override {
         std::vector<double> hx(this->number_variables, 0.);
         this->hessian_product(x.data(), hx.data());
         double f = 0.;
         for (size_t i = 0; i < this->number_variables; ++i) f += x[i] * (0.5 * hx[i] + this->g[i]);
         return f;
      }
      void evaluate_objective_gradient(const Vector<double>& x, Vector<double>& gradient) const override {
         std::vector<double> hx(this->number_variables, 0.);
         this->hessian_product(x.data(), hx.data());
         for (size_t i = 0; i < this->number_variables; ++i) gradient[i] = hx[i] + this->g[i];
      }
      void evaluate_constraints(const Vector<double>& x, std::vector<double>& constraints) const override {
         for (size_t j = 0; j < this->number_constraints; ++j) {
            double c = -this->b[j];
            for (const auto& [v, a]: this->rows[j]) c += a * x[v];
            constraints[j] = c;
         }
      }
      void evaluate_constraint_gradient(const Vector<double>&, size_t j, SparseVector<double>& gradient) const override {
         gradient.clear();
         for (const auto& [v, a]: this->rows[j]) gradient.insert(v, a);
      }
      void evaluate_constraint_jacobian(const Vector<double>& x, RectangularMatrix<double>& jacobian) const override {
         for (size_t j = 0; j < this->number_constraints; ++j) this->evaluate_constraint_gradient(x, j, jacobian[j]);
      }
      void evaluate_lagrangian_hessian(const Vector<double>&, double sigma, const Vector<double>&,
            SymmetricMatrix<size_t, double>& hessian) const override {
         // linear constraints: the Lagrangian Hessian is sigma * H
         for (size_t c = 0; c < this->number_variables; ++c) {
            const size_t r0 = c > band ? c - band : 0;
            for (size_t k = this->hcol_start[c]; k < this->hcol_start[c + 1]; ++k) {
               hessian.insert(r0 + (k - this->hcol_start[c]), c, sigma * this->hval[k]);
            }
            hessian.finalize_column(c);
         }
      }
      void compute_hessian_vector_product(const double* v, double sigma, const Vector<double>&, double* result) const override {
         std::fill(result, result + this->number_variables, 0.);
         this->hessian_product(v, result);
         for (size_t i = 0; i < this->number_variables; ++i) result[i] *= sigma;
      }

      [[nodiscard]] double variable_lower_bound(size_t) const override { return -10.; }
      [[nodiscard]] double variable_upper_bound(size_t) const override { return 10.; }
      [[nodiscard]] const Collection<size_t>& get_lower_bounded_variables() const override { return this->all_collection; }
      [[nodiscard]] const Collection<size_t>& get_upper_bounded_variables() const override { return this->all_collection; }
      [[nodiscard]] const SparseVector<size_t>& get_slacks() const override { return this->slacks; }
      [[nodiscard]] const Collection<size_t>& get_single_lower_bounded_variables() const override { return this->empty_collection; }
      [[nodiscard]] const Collection<size_t>& get_single_upper_bounded_variables() const override { return this->empty_collection; }
      [[nodiscard]] const Vector<size_t>& get_fixed_variables() const override { return this->fixed; }
      [[nodiscard]] double constraint_lower_bound(size_t) const override { return this->inequality ? -1. : 0.; }
      [[nodiscard]] double constraint_upper_bound(size_t) const override { return this->inequality ? 1. : 0.; }
      [[nodiscard]] const Collection<size_t>& get_equality_constraints() const override { return this->equality_collection; }
      [[nodiscard]] const Collection<size_t>& get_inequality_constraints() const override { return this->inequality_collection; }
      [[nodiscard]] const Collection<size_t>& get_linear_constraints() const override { return this->linear_constraints; }
      void initial_primal_point(Vector<double>& x) const override { std::fill(x.begin(), x.begin() + this->number_variables, 0.); }
      void initial_dual_point(Vector<double>& y) const override { std::fill(y.begin(), y.begin() + this->number_constraints, 0.); }
      void postprocess_solution(Iterate&, IterateStatus) const override {}
      [[nodiscard]] size_t number_jacobian_nonzeros() const override { return this->number_constraints * (window + arrow); }
      [[nodiscard]] size_t number_hessian_nonzeros() const override { return this->hval.size(); }

   private:
      static uint64_t next(uint64_t& s) {
         uint64_t z = (s += 0x9E3779B97F4A7C15ull);
         z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
         z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
         return z ^ (z >> 31);
      }
      static double unif(uint64_t& s) { return static_cast<double>(next(s) >> 11) * (1.0 / 9007199254740992.0); }

      void hessian_product(const double* x, double* y) const {
         for (size_t c = 0; c < this->number_variables; ++c) {
            const size_t r0 = c > band ? c - band : 0;
            for (size_t k = this->hcol_start[c]; k < this->hcol_start[c + 1]; ++k) {
               const size_t r = r0 + (k - this->hcol_start[c]);
               y[r] += this->hval[k] * x[c];
               if (r != c) y[c] += this->hval[k] * x[r];
            }
         }
      }

      std::vector<size_t> hcol_start;
      std::vector<double> hval, g, b;
      std::vector<std::vector<std::pair<size_t, double>>> rows;
      bool inequality;
      std::vector<size_t> all, empty, equalities, inequalities;
      CollectionAdapter<std::vector<size_t>&> all_collection, empty_collection, equality_collection, inequality_collection;
      ForwardRange linear_constraints;
      SparseVector<size_t> slacks{};
      Vector<size_t> fixed{};
   };
} // namespace

#endif
