// HS015Model.hpp -- examples/hs015.mod hand-coded as a uno::Model (ASL, which reads examples/hs015.nl,
// is not available here).  Conventions follow bindings/AMPL/AMPLModel.cpp: the Lagrangian Hessian is
// sigma*grad^2 f - sum_j y_j grad^2 c_j (lagscale -1, AMPLModel.cpp:39), stored upper-triangular,
// column-major (Sphset uptri=1, AMPLModel.cpp:357-368; insertion loop :171-178); the AMPL presolve
// turns "x[1] <= 1/2" into a variable bound, leaving 2 variables and 2 nonlinear constraints.
//
//   min 100 (x2 - x1^2)^2 + (1 - x1)^2   s.t.  x1 x2 >= 1,  x1 + x2^2 >= 0,  x1 <= 1/2,  x0 = (-2, 1)
#ifndef UNO_KKT_HS015MODEL_H
#define UNO_KKT_HS015MODEL_H

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
   class HS015Model : public Model {
   public:
      HS015Model(): Model("hs015", 2, 2, 1.),
            empty_collection(this->empty), upper_bounded_collection(this->upper_bounded),
            inequality_collection(this->inequalities), linear_constraints(2, 2) {}

      [[nodiscard]] double evaluate_objective(const Vector<double>& x) const override {
         const double a = x[1] - x[0] * x[0], b = 1. - x[0];
         return 100. * a * a + b * b;
      }
      void evaluate_objective_gradient(const Vector<double>& x, Vector<double>& gradient) const override {
         const double a = x[1] - x[0] * x[0];
         gradient[0] = -400. * x[0] * a - 2. * (1. - x[0]);
         gradient[1] = 200. * a;
      }
      void evaluate_constraints(const Vector<double>& x, std::vector<double>& constraints) const override {
         constraints[0] = x[0] * x[1];
         constraints[1] = x[0] + x[1] * x[1];
      }
      void evaluate_constraint_gradient(const Vector<double>& x, size_t j, SparseVector<double>& gradient) const override {
         gradient.clear();
         if (j == 0) {
            gradient.insert(0, x[1]);
            gradient.insert(1, x[0]);
         }
         else {
            gradient.insert(0, 1.);
            gradient.insert(1, 2. * x[1]);
         }
      }
      void evaluate_constraint_jacobian(const Vector<double>& x, RectangularMatrix<double>& jacobian) const override {
         for (size_t j = 0; j < 2; ++j) {
            this->evaluate_constraint_gradient(x, j, jacobian[j]);
         }
      }
      void evaluate_lagrangian_hessian(const Vector<double>& x, double sigma, const Vector<double>& y,
            SymmetricMatrix<size_t, double>& hessian) const override {
         hessian.insert(0, 0, sigma * (1200. * x[0] * x[0] - 400. * x[1] + 2.));
         hessian.finalize_column(0);
         hessian.insert(0, 1, sigma * (-400. * x[0]) - y[0]);
         hessian.insert(1, 1, sigma * 200. - 2. * y[1]);
         hessian.finalize_column(1);
      }
      void compute_hessian_vector_product(const double* v, double sigma, const Vector<double>& y, double* result) const override {
         // only called by active-set QP solvers; hs015 Hessian at the last x is not stored, so use x-free parts
         (void)v; (void)sigma; (void)y; (void)result;
         throw std::runtime_error("HS015Model::compute_hessian_vector_product is not used by the ipopt preset");
      }

      [[nodiscard]] double variable_lower_bound(size_t) const override { return -INF<double>; }
      [[nodiscard]] double variable_upper_bound(size_t i) const override { return i == 0 ? 0.5 : INF<double>; }
      [[nodiscard]] const Collection<size_t>& get_lower_bounded_variables() const override { return this->empty_collection; }
      [[nodiscard]] const Collection<size_t>& get_upper_bounded_variables() const override { return this->upper_bounded_collection; }
      [[nodiscard]] const SparseVector<size_t>& get_slacks() const override { return this->slacks; }
      [[nodiscard]] const Collection<size_t>& get_single_lower_bounded_variables() const override { return this->empty_collection; }
      [[nodiscard]] const Collection<size_t>& get_single_upper_bounded_variables() const override { return this->upper_bounded_collection; }
      [[nodiscard]] const Vector<size_t>& get_fixed_variables() const override { return this->fixed; }

      [[nodiscard]] double constraint_lower_bound(size_t j) const override { return j == 0 ? 1. : 0.; }
      [[nodiscard]] double constraint_upper_bound(size_t) const override { return INF<double>; }
      [[nodiscard]] const Collection<size_t>& get_equality_constraints() const override { return this->empty_collection; }
      [[nodiscard]] const Collection<size_t>& get_inequality_constraints() const override { return this->inequality_collection; }
      [[nodiscard]] const Collection<size_t>& get_linear_constraints() const override { return this->linear_constraints; }

      void initial_primal_point(Vector<double>& x) const override { x[0] = -2.; x[1] = 1.; }
      void initial_dual_point(Vector<double>& multipliers) const override { multipliers[0] = 0.; multipliers[1] = 0.; }
      void postprocess_solution(Iterate&, IterateStatus) const override {}

      [[nodiscard]] size_t number_jacobian_nonzeros() const override { return 4; }
      [[nodiscard]] size_t number_hessian_nonzeros() const override { return 3; }

   private:
      std::vector<size_t> empty{};
      std::vector<size_t> upper_bounded{0};
      std::vector<size_t> inequalities{0, 1};
      CollectionAdapter<std::vector<size_t>&> empty_collection;
      CollectionAdapter<std::vector<size_t>&> upper_bounded_collection;
      CollectionAdapter<std::vector<size_t>&> inequality_collection;
      ForwardRange linear_constraints;
      SparseVector<size_t> slacks{};
      Vector<size_t> fixed{};
   };
} // namespace

#endif
