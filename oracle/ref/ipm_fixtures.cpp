// ipm_fixtures.cpp -- TEST INFRASTRUCTURE ONLY.  Golden vectors for the device-side IPM vector work
//  produced by the REFERENCE code itself: the Uno core compiled from
// /root/reference by oracle/ref/Makefile (libuno_core.a).  For a model with mixed variable bounds (lower
// only, upper only, both, free) and seeded random iterates, it calls
//   PrimalDualInteriorPointProblem::evaluate_lagrangian_hessian  (PrimalDualInteriorPointProblem.cpp:56-78,
//                                                                  the barrier diagonal Sigma)
//   Subproblem::assemble_augmented_rhs                            (Subproblem.cpp:80-99)
//   Subproblem::assemble_primal_dual_direction                    (Subproblem.cpp:101-103 ->
//                                                                  PrimalDualInteriorPointProblem.cpp:173-194,
//                                                                  262-325)
// and prints one JSON object per case (inputs and the reference's outputs, %.17g: exact round trip).
// tests/golden/make_ipm_fixtures.sh writes them to tests/golden/ipm_reference_vectors.json, which
// tests/test_ipm_vectors.py checks oracle/ipm_oracle.py and the HIP kernels against, bit for bit.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "ingredients/hessian_models/HessianModel.hpp"
#include "ingredients/hessian_models/HessianModelFactory.hpp"
#include "ingredients/inequality_handling_methods/interior_point_methods/InteriorPointParameters.hpp"
#include "ingredients/inequality_handling_methods/interior_point_methods/PrimalDualInteriorPointProblem.hpp"
#include "ingredients/regularization_strategies/RegularizationStrategy.hpp"
#include "ingredients/regularization_strategies/RegularizationStrategyFactory.hpp"
#include "ingredients/subproblem/Subproblem.hpp"
#include "linear_algebra/COOFormat.hpp"
#include "linear_algebra/RectangularMatrix.hpp"
#include "linear_algebra/SparseSymmetricMatrix.hpp"
#include "linear_algebra/SparseVector.hpp"
#include "linear_algebra/Vector.hpp"
#include "model/Model.hpp"
#include "model/ModelFactory.hpp"
#include "models/ArrowbandModel.hpp"
#include "optimization/Direction.hpp"
#include "optimization/Iterate.hpp"
#include "optimization/Multipliers.hpp"
#include "optimization/OptimizationProblem.hpp"
#include "options/DefaultOptions.hpp"
#include "options/Options.hpp"
#include "options/Presets.hpp"
#include "symbolic/CollectionAdapter.hpp"
#include "symbolic/Range.hpp"
#include "tools/Infinity.hpp"
#include "tools/Statistics.hpp"

using namespace uno;

namespace {
uint64_t sm_state;
double unif() {  // splitmix64 -> [0, 1)
   uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
   z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
   z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
   z ^= z >> 31;
   return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// Only the bound queries are used by the calls above; the evaluation entry points are never reached.
class BoundsModel : public Model {
public:
   BoundsModel(std::vector<double> lb, std::vector<double> ub, size_t m):
         Model("bounds", lb.size(), m, 1.), lb(std::move(lb)), ub(std::move(ub)), lower_c(this->lower), upper_c(this->upper),
         single_lower_c(this->single_lower), single_upper_c(this->single_upper), empty_c(this->empty),
         all_c(this->all_cons), linear(0, m) {
      for (size_t i = 0; i < this->lb.size(); ++i) {
         const bool l = is_finite(this->lb[i]), u = is_finite(this->ub[i]);
         if (l) this->lower.push_back(i);
         if (u) this->upper.push_back(i);
         if (l && !u) this->single_lower.push_back(i);
         if (u && !l) this->single_upper.push_back(i);
      }
      for (size_t j = 0; j < m; ++j) this->all_cons.push_back(j);
   }
   [[nodiscard]] double evaluate_objective(const Vector<double>&) const override { throw std::runtime_error("unused"); }
   void evaluate_objective_gradient(const Vector<double>&, Vector<double>&) const override { throw std::runtime_error("unused"); }
   void evaluate_constraints(const Vector<double>&, std::vector<double>&) const override { throw std::runtime_error("unused"); }
   void evaluate_constraint_gradient(const Vector<double>&, size_t, SparseVector<double>&) const override {
      throw std::runtime_error("unused");
   }
   void evaluate_constraint_jacobian(const Vector<double>&, RectangularMatrix<double>&) const override { throw std::runtime_error("unused"); }
   void evaluate_lagrangian_hessian(const Vector<double>&, double, const Vector<double>&, SymmetricMatrix<size_t, double>& h) const override {
      for (size_t i = 0; i < this->number_variables; ++i) h.finalize_column(i);  // no model curvature: Sigma only
   }
   void compute_hessian_vector_product(const double*, double, const Vector<double>&, double*) const override {
      throw std::runtime_error("unused");
   }
   [[nodiscard]] double variable_lower_bound(size_t i) const override { return this->lb[i]; }
   [[nodiscard]] double variable_upper_bound(size_t i) const override { return this->ub[i]; }
   [[nodiscard]] const Collection<size_t>& get_lower_bounded_variables() const override { return this->lower_c; }
   [[nodiscard]] const Collection<size_t>& get_upper_bounded_variables() const override { return this->upper_c; }
   [[nodiscard]] const SparseVector<size_t>& get_slacks() const override { return this->slacks; }
   [[nodiscard]] const Collection<size_t>& get_single_lower_bounded_variables() const override { return this->single_lower_c; }
   [[nodiscard]] const Collection<size_t>& get_single_upper_bounded_variables() const override { return this->single_upper_c; }
   [[nodiscard]] const Vector<size_t>& get_fixed_variables() const override { return this->fixed; }
   [[nodiscard]] double constraint_lower_bound(size_t) const override { return 0.; }
   [[nodiscard]] double constraint_upper_bound(size_t) const override { return 0.; }
   [[nodiscard]] const Collection<size_t>& get_equality_constraints() const override { return this->all_c; }
   [[nodiscard]] const Collection<size_t>& get_inequality_constraints() const override { return this->empty_c; }
   [[nodiscard]] const Collection<size_t>& get_linear_constraints() const override { return this->linear; }
   void initial_primal_point(Vector<double>&) const override {}
   void initial_dual_point(Vector<double>&) const override {}
   void postprocess_solution(Iterate&, IterateStatus) const override {}
   [[nodiscard]] size_t number_jacobian_nonzeros() const override { return 0; }
   [[nodiscard]] size_t number_hessian_nonzeros() const override { return 0; }

private:
   std::vector<double> lb, ub;
   std::vector<size_t> lower, upper, single_lower, single_upper, empty, all_cons;
   CollectionAdapter<std::vector<size_t>&> lower_c, upper_c, single_lower_c, single_upper_c, empty_c, all_c;
   ForwardRange linear;
   SparseVector<size_t> slacks{};
   Vector<size_t> fixed{};
};

void print_array(const char* name, const double* v, size_t n, bool comma = true) {
   std::printf("\"%s\": [", name);
   for (size_t i = 0; i < n; ++i) {
      if (std::isinf(v[i])) std::printf("%s%s", i ? ", " : "", v[i] > 0 ? "\"inf\"" : "\"-inf\"");
      else std::printf("%s%.17g", i ? ", " : "", v[i]);
   }
   std::printf("]%s", comma ? ", " : "");
}
void print_index(const char* name, const std::vector<size_t>& v) {
   std::printf("\"%s\": [", name);
   for (size_t i = 0; i < v.size(); ++i) std::printf("%s%zu", i ? ", " : "", v[i]);
   std::printf("], ");
}

void one_case(const Options& options, size_t n, size_t m, size_t per_con, double mu, uint64_t seed, bool last) {
   sm_state = seed;
   std::vector<double> lb(n), ub(n), x(n), zl(n, 0.), zu(n, 0.);
   for (size_t i = 0; i < n; ++i) {
      const double kind = unif();  // lower only / upper only / both / free
      x[i] = 4. * unif() - 2.;
      const double dl = std::pow(10., -8. + 9. * unif()), du = std::pow(10., -8. + 9. * unif());
      lb[i] = (kind < 0.3 || kind >= 0.55) && kind < 0.85 ? x[i] - dl : -INF<double>;
      ub[i] = kind >= 0.3 && kind < 0.85 ? x[i] + du : INF<double>;
      if (is_finite(lb[i])) zl[i] = std::pow(10., -6. + 6. * unif());
      if (is_finite(ub[i])) zu[i] = -std::pow(10., -6. + 6. * unif());
   }
   BoundsModel model(lb, ub, m);
   const OptimizationProblem problem(model);
   const InteriorPointParameters parameters{options.get_double("barrier_tau_min"), options.get_double("barrier_k_sigma"),
      options.get_double("barrier_regularization_exponent"), options.get_double("barrier_small_direction_factor"),
      options.get_double("barrier_push_variable_to_interior_k1"), options.get_double("barrier_push_variable_to_interior_k2"),
      options.get_double("barrier_damping_factor")};
   const PrimalDualInteriorPointProblem barrier_problem(problem, mu, parameters);
   Iterate iterate(n, m);
   Multipliers multipliers(n, m);
   for (size_t i = 0; i < n; ++i) {
      iterate.primals[i] = x[i];
      multipliers.lower_bounds[i] = zl[i];
      multipliers.upper_bounds[i] = zu[i];
   }
   for (size_t j = 0; j < m; ++j) multipliers.constraints[j] = unif() < 0.2 ? 0. : 2. * unif() - 1.;
   auto hessian_model = HessianModelFactory::create(options);
   hessian_model->initialize(model);
   auto regularization = RegularizationStrategyFactory::create(options);
   const Subproblem subproblem(barrier_problem, iterate, multipliers, *hessian_model, *regularization, INF<double>);

   // A4: barrier diagonal (the Hessian is empty: the COO holds exactly Sigma, ascending bounded variables)
   Statistics statistics;
   SparseSymmetricMatrix<COOFormat<size_t, double>> hessian(n, n, 0);
   barrier_problem.evaluate_lagrangian_hessian(statistics, *hessian_model, iterate.primals, multipliers, hessian);
   std::vector<size_t> sigma_var;
   std::vector<double> sigma;
   for (const auto [r, c, v]: hessian) {
      sigma_var.push_back(r);
      sigma.push_back(v);
   }
   // A10: right-hand side (Jacobian rows in stored order, variables in random order, repeats allowed)
   Vector<double> grad(n), rhs(n + m);
   std::vector<double> cons(m);
   RectangularMatrix<double> jacobian(m, n);
   std::vector<size_t> jc, jv;
   std::vector<double> jval;
   for (size_t i = 0; i < n; ++i) grad[i] = 4. * unif() - 2.;
   for (size_t j = 0; j < m; ++j) {
      cons[j] = 2. * unif() - 1.;
      for (size_t k = 0; k < per_con; ++k) {
         const size_t var = (size_t)(unif() * (double)n) % n;
         const double d = 3. * unif() - 1.5;
         jacobian[j].insert(var, d);
         jc.push_back(j);
         jv.push_back(var);
         jval.push_back(d);
      }
   }
   subproblem.assemble_augmented_rhs(grad, cons, jacobian, rhs);
   // A11: direction and fraction-to-boundary step lengths
   Vector<double> solution(n + m);
   for (size_t i = 0; i < n + m; ++i) solution[i] = (4. * unif() - 2.) * std::pow(10., -3. + 3. * unif());
   Direction direction(n, m);
   subproblem.assemble_primal_dual_direction(solution, direction);

   std::printf("{\"n\": %zu, \"m\": %zu, \"mu\": %.17g, \"tau_min\": %.17g, \"seed\": %llu, ", n, m, mu, parameters.tau_min,
      (unsigned long long)seed);
   print_array("lb", lb.data(), n);
   print_array("ub", ub.data(), n);
   print_array("x", x.data(), n);
   print_array("zl", zl.data(), n);
   print_array("zu", zu.data(), n);
   print_array("y", multipliers.constraints.data(), m);
   print_index("sigma_var", sigma_var);
   print_array("sigma", sigma.data(), sigma.size());
   print_array("grad", grad.data(), n);
   print_array("cons", cons.data(), m);
   print_index("jac_con", jc);
   print_index("jac_var", jv);
   print_array("jac_val", jval.data(), jval.size());
   print_array("rhs", rhs.data(), n + m);
   print_array("solution", solution.data(), n + m);
   print_array("dx", direction.primals.data(), n);
   print_array("dy", direction.multipliers.constraints.data(), m);
   print_array("dzl", direction.multipliers.lower_bounds.data(), n);
   print_array("dzu", direction.multipliers.upper_bounds.data(), n, false);
   std::printf("}%s\n", last ? "" : ",");
}
// the whole augmented (KKT) value array as the reference assembles it for the synthetic
// arrowband model through the ipopt chain (ModelFactory::reformulate: slacks + bound relaxation, then
// PrimalDualInteriorPointProblem), i.e. COOFormat::reset + Subproblem::assemble_augmented_matrix
// (Subproblem.cpp:57-70) at a seeded interior iterate.  Printed with the device kernel's inputs: the model's
// Lagrangian Hessian terms at objective multiplier 1 (insertion order) and at `sigma` (a second, direct call of
// Model::evaluate_lagrangian_hessian), the reformulated problem's Jacobian entries (constraint-major), the
// relaxed bounds and the iterate.  uno_kkt_assemble_augmented must reproduce `values` bit for bit.
void augmented_case(const Options& options, size_t N, bool inequality, double sigma, uint64_t seed, bool last) {
   std::unique_ptr<Model> model = std::make_unique<ArrowbandModel>(N, inequality);
   model = ModelFactory::reformulate(std::move(model), options);
   const OptimizationProblem problem(*model);
   const size_t n = problem.number_variables, m = problem.number_constraints;
   const InteriorPointParameters parameters{options.get_double("barrier_tau_min"), options.get_double("barrier_k_sigma"),
      options.get_double("barrier_regularization_exponent"), options.get_double("barrier_small_direction_factor"),
      options.get_double("barrier_push_variable_to_interior_k1"), options.get_double("barrier_push_variable_to_interior_k2"),
      options.get_double("barrier_damping_factor")};
   const PrimalDualInteriorPointProblem barrier_problem(problem, 0.1, parameters);
   auto hessian_model = HessianModelFactory::create(options);
   hessian_model->initialize(*model);
   auto regularization = RegularizationStrategyFactory::create(options);
   sm_state = seed;
   Iterate iterate(n, m);
   Multipliers multipliers(n, m);
   std::vector<double> lb(n), ub(n);
   for (size_t i = 0; i < n; ++i) {
      lb[i] = problem.variable_lower_bound(i);
      ub[i] = problem.variable_upper_bound(i);
      const double lo = is_finite(lb[i]) ? lb[i] : -20., hi = is_finite(ub[i]) ? ub[i] : 20.;
      iterate.primals[i] = lo + (hi - lo) * (0.001 + 0.998 * unif());
      if (is_finite(lb[i])) multipliers.lower_bounds[i] = std::pow(10., -8. + 16. * unif());
      if (is_finite(ub[i])) multipliers.upper_bounds[i] = -std::pow(10., -8. + 16. * unif());
   }
   for (size_t j = 0; j < m; ++j) multipliers.constraints[j] = 2. * unif() - 1.;
   const Subproblem subproblem(barrier_problem, iterate, multipliers, *hessian_model, *regularization, INF<double>);
   RectangularMatrix<double> jacobian(m, n);
   subproblem.evaluate_jacobian(jacobian);
   // the reference: the plugin's matrix (PrimalDualInteriorPointMethod.cpp:49-57 sizing), reset, assembled
   const size_t reg_size = (regularization->performs_primal_regularization() ? problem.get_number_original_variables() : 0) +
      (regularization->performs_dual_regularization() ? problem.get_equality_constraints().size() : 0);
   const size_t nnz = barrier_problem.number_hessian_nonzeros(*hessian_model) + barrier_problem.number_jacobian_nonzeros();
   SparseSymmetricMatrix<COOFormat<size_t, double>> augmented(n + m, nnz, reg_size);
   augmented.reset();
   Statistics statistics;
   subproblem.assemble_augmented_matrix(statistics, augmented, jacobian);
   std::vector<size_t> rows, cols;
   std::vector<double> values;
   for (const auto [r, c, v]: augmented) {
      rows.push_back(r);
      cols.push_back(c);
      values.push_back(v);
   }
   // the device kernel's inputs: Hessian terms in the model's insertion order (objective multiplier 1 and sigma)
   SparseSymmetricMatrix<COOFormat<size_t, double>> h1(n, problem.number_hessian_nonzeros(*hessian_model), 0);
   SparseSymmetricMatrix<COOFormat<size_t, double>> hs(n, problem.number_hessian_nonzeros(*hessian_model), 0);
   model->evaluate_lagrangian_hessian(iterate.primals, 1., multipliers.constraints, h1);
   model->evaluate_lagrangian_hessian(iterate.primals, sigma, multipliers.constraints, hs);
   std::vector<double> hess1, hess_sigma, jac;
   for (const auto [r, c, v]: h1) { (void)r; (void)c; hess1.push_back(v); }
   for (const auto [r, c, v]: hs) { (void)r; (void)c; hess_sigma.push_back(v); }
   for (size_t j = 0; j < m; ++j) {
      for (const auto [var, d]: jacobian[j]) { (void)var; jac.push_back(d); }
   }
   std::printf("{\"model\": \"%s\", \"N\": %zu, \"n\": %zu, \"m\": %zu, \"reg_size\": %zu, \"sigma\": %.17g, \"seed\": %llu, ",
      inequality ? "arrowband_ineq" : "arrowband", N, n, m, reg_size, sigma, (unsigned long long)seed);
   print_array("lb", lb.data(), n);
   print_array("ub", ub.data(), n);
   print_array("x", iterate.primals.data(), n);
   print_array("zl", multipliers.lower_bounds.data(), n);
   print_array("zu", multipliers.upper_bounds.data(), n);
   print_array("hess", hess1.data(), hess1.size());
   print_array("hess_sigma", hess_sigma.data(), hess_sigma.size());
   print_array("jac", jac.data(), jac.size());
   print_index("rows", rows);
   print_index("cols", cols);
   print_array("values", values.data(), values.size(), false);
   std::printf("}%s\n", last ? "" : ",");
}
} // namespace

int main(int argc, char* argv[]) {
   Options options = DefaultOptions::load();
   options.overwrite_with(DefaultOptions::determine_solvers());
   options.overwrite_with(Presets::get_preset_options(std::optional<std::string>("ipopt")));
   if (argc > 1 && std::string(argv[1]) == "augmented") {
      std::printf("[\n");
      augmented_case(options, 160, false, 0.37, 0xA55E3B1Eull, false);
      augmented_case(options, 200, true, 1e-3, 0xA55E3B1Full, true);
      std::printf("]\n");
      return 0;
   }
   std::printf("[\n");
   // (n, m, Jacobian entries per constraint, barrier parameter): mu below and above 1 - tau_min
   one_case(options, 300, 120, 6, 0.1, 0x1BADB002ull, false);
   one_case(options, 500, 200, 9, 1e-9, 0x5EED0A11ull, false);
   one_case(options, 64, 40, 4, 0.5, 0x00C0FFEEull, true);
   std::printf("]\n");
   return 0;
}
