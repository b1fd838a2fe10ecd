// uno_kkt_driver.cpp -- runs the reference Uno core (libuno built from /root/reference by
// oracle/ref/Makefile) on a hand-coded model with a KKT plugin chosen by linear_solver=..., and prints
// one JSON object: status, iterations, solution and the sequence of (dimension, inertia) of every
// factorization the plugin performed.  This is the in-container stand-in for `uno_ampl model.nl -AMPL
// preset=ipopt linear_solver=HIPLDL` (bindings/AMPL/uno_ampl.cpp:78-139; ASL is not available).
//
// usage: uno_kkt_driver <model> [option=value ...]     model: hs015 (hand-coded), arrowband:<N> (synthetic NLP) or a path to a text .nl file
//        uno_kkt_driver convexify:<model> [option=value ...]   byrd-preset Hessian convexification only (see below)
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <array>
#include <fstream>
#include <sstream>
#include <vector>
#include <iostream>
#include <memory>
#include <string>

#include "KKTTrace.hpp"
#include "kkt_oracle.h"
#include "uno_kkt.h"
#include "Uno.hpp"
#include "model/ModelFactory.hpp"
#include "models/HS015Model.hpp"
#include "models/NLModel.hpp"
#include "models/ArrowbandModel.hpp"
#include "ingredients/constraint_relaxation_strategies/l1RelaxedProblem.hpp"
#include "ingredients/hessian_models/HessianModel.hpp"
#include "ingredients/hessian_models/HessianModelFactory.hpp"
#include "ingredients/regularization_strategies/PrimalRegularization.hpp"
#include "linear_algebra/COOFormat.hpp"
#include "linear_algebra/SparseSymmetricMatrix.hpp"
#include "optimization/Iterate.hpp"
#include "optimization/Multipliers.hpp"
#include "optimization/Result.hpp"
#include "options/DefaultOptions.hpp"
#include "options/Options.hpp"
#include "options/Presets.hpp"
#include "tools/Logger.hpp"
#include "tools/Statistics.hpp"
#include "tools/UserCallbacks.hpp"

using namespace uno;

// ---- inertia cross-check (UNO_KKT_CROSSCHECK="i,j,..."): at the listed factorizations of the run, the matrix
// the plugin factored is factored again by the CPU oracle and (where a GPU exists) by a fresh GPU handle, and
// also shifted by -+sigma on its diagonal for a ladder of sigma relative to ||A||_inf.  Where two solvers report
// different inertias for nearly the same matrix, the ladder shows whether an eigenvalue lies within sigma of 0
// (its sign is then decided by rounding, not by the matrix).  Test drivers only.
namespace {
   std::vector<size_t> crosscheck_targets;
   std::vector<std::string> crosscheck_records;
   // UNO_KKT_CROSSCHECK_TRACE=<file of "p q z" lines, a golden run's inertias>: cross-check where this run first
   // reports another inertia than the golden one, and where it first disagrees on whether the inertia is the
   // expected one (the golden run's last factorization), i.e. where the two runs' decisions part
   std::vector<std::array<int64_t, 3>> crosscheck_golden;
   bool crosscheck_first_done = false, crosscheck_decision_done = false;

   std::string inertia_json(int rc, int64_t p, int64_t q, int64_t z) {
      if (rc != 0) return "null";
      std::ostringstream o;
      o << "[" << p << ", " << q << ", " << z << "]";
      return o.str();
   }

   void crosscheck_hook(size_t index, size_t n, int64_t nnz, const int64_t* r, const int64_t* c, const double* v,
         int64_t p, int64_t q, int64_t z) {
      std::string tag = "listed";
      if (std::find(crosscheck_targets.begin(), crosscheck_targets.end(), index) == crosscheck_targets.end()) {
         if (index >= crosscheck_golden.size() || crosscheck_golden.empty()) return;
         const auto& g = crosscheck_golden[index];
         const auto& e = crosscheck_golden.back();
         const bool differs = g[0] != p || g[1] != q || g[2] != z;
         const bool decision = (g == e) != (p == e[0] && q == e[1] && z == e[2]);
         if (differs && !crosscheck_first_done) { crosscheck_first_done = true; tag = decision ? "first_difference+first_decision" : "first_difference"; if (decision) crosscheck_decision_done = true; }
         else if (decision && !crosscheck_decision_done) { crosscheck_decision_done = true; tag = "first_decision"; }
         else return;
      }
      std::vector<double> rowsum(n, 0.);
      std::vector<int64_t> diag(n, -1);
      for (int64_t e = 0; e < nnz; ++e) {
         rowsum[r[e]] += std::fabs(v[e]);
         if (r[e] != c[e]) rowsum[c[e]] += std::fabs(v[e]);
         else if (diag[r[e]] < 0) diag[r[e]] = e;
      }
      double anorm = 0.;
      for (double x: rowsum) anorm = std::max(anorm, x);
      bool all_diag = true;
      for (int64_t d: diag) all_diag = all_diag && d >= 0;
      oracle_kkt_t o = oracle_kkt_create();
      uno_kkt_t g = nullptr;
      const bool gpu = uno_kkt_create(&g, 0) == UNO_KKT_OK;
      int orc = oracle_kkt_analyze(o, (int64_t)n, nnz, r, c);
      int grc = gpu ? uno_kkt_analyze(g, (int64_t)n, nnz, r, c) : -1;
      auto factor_both = [&](const double* w, std::string& jo, std::string& jg) {
         int64_t a = 0, b = 0, d = 0;
         int rc = orc == 0 ? oracle_kkt_factorize(o, w) : orc;
         if (rc == 0) rc = oracle_kkt_inertia(o, &a, &b, &d);
         jo = inertia_json(rc, a, b, d);
         if (gpu && grc == 0) {
            rc = uno_kkt_factorize(g, w, 0);
            if (rc == UNO_KKT_OK || rc == UNO_KKT_ERR_PIVOT) rc = uno_kkt_inertia(g, &a, &b, &d);
            jg = inertia_json(rc, a, b, d);
         } else {
            jg = "null";
         }
      };
      std::ostringstream out;
      std::string jo, jg;
      factor_both(v, jo, jg);
      out.precision(17);
      out << "{\"index\": " << index << ", \"tag\": \"" << tag << "\"";
      if (index < crosscheck_golden.size()) out << ", \"golden_inertia\": " << inertia_json(0, crosscheck_golden[index][0], crosscheck_golden[index][1], crosscheck_golden[index][2]);
      out << ", \"run_inertia\": " << inertia_json(0, p, q, z) << ", \"oracle\": " << jo
          << ", \"gpu\": " << jg << ", \"anorm_inf\": " << anorm << ", \"shifts\": [";
      if (all_diag) {
         std::vector<double> w(v, v + nnz);
         const double rel[] = {1e-6, 1e-8, 1e-10, 1e-12, 1e-14};
         for (size_t k = 0; k < sizeof(rel) / sizeof(rel[0]); ++k) {
            const double sigma = rel[k] * anorm;
            std::string op, gp, om, gm;
            for (size_t i = 0; i < n; ++i) w[diag[i]] = v[diag[i]] + sigma;
            factor_both(w.data(), op, gp);
            for (size_t i = 0; i < n; ++i) w[diag[i]] = v[diag[i]] - sigma;
            factor_both(w.data(), om, gm);
            out << (k ? ", " : "") << "{\"sigma_rel\": " << rel[k] << ", \"oracle_plus\": " << op << ", \"oracle_minus\": " << om
                << ", \"gpu_plus\": " << gp << ", \"gpu_minus\": " << gm << "}";
         }
      }
      out << "]}";
      crosscheck_records.push_back(out.str());
      std::fprintf(stderr, "[crosscheck] %s\n", crosscheck_records.back().c_str());
      oracle_kkt_destroy(o);
      if (gpu) uno_kkt_destroy(g);
   }

   void install_crosscheck() {
      if (const char* path = std::getenv("UNO_KKT_CROSSCHECK_TRACE")) {
         std::ifstream in(path);
         int64_t a, b, c;
         while (in >> a >> b >> c) crosscheck_golden.push_back({a, b, c});
         kkt_trace::factor_hook() = crosscheck_hook;
      }
      const char* env = std::getenv("UNO_KKT_CROSSCHECK");
      if (env == nullptr) return;
      std::stringstream ss(env);
      std::string item;
      while (std::getline(ss, item, ',')) {
         if (!item.empty()) crosscheck_targets.push_back(std::stoul(item));
      }
      kkt_trace::factor_hook() = crosscheck_hook;
   }
} // namespace

// The byrd preset's use of the plugin: Hessian convexification by
// PrimalRegularization::regularize_hessian (PrimalRegularization.hpp:79-129) of the l1-relaxed problem's
// Lagrangian Hessian, exactly as Subproblem::compute_regularized_hessian (Subproblem.cpp:32-43) drives it
// from BQPD's Hessian callback (BQPDSolver.cpp:89-96, 405-407).  BQPD itself is absent (proprietary), so the
// QP iterations cannot run; instead the Hessian is convexified at a fixed sequence of primal-dual points and
// penalty parameters, reusing ONE PrimalRegularization instance (one symbolic analysis, as in a solve).
// Expected inertia (n_model, 0, n_elastic): the elastic variables have empty Hessian rows (null pivots).
static void run_convexification(const Model& model, const Options& options) {
   const auto hessian_model = HessianModelFactory::create(options);
   const double coefficient = options.get_double("l1_constraint_violation_coefficient");
   const l1RelaxedProblem shape(model, 1., coefficient);
   const size_t n = shape.number_variables, n_model = model.number_variables;
   const size_t regularization_size = shape.get_number_original_variables();  // InequalityConstrainedMethod.cpp:28-29
   SparseSymmetricMatrix<COOFormat<size_t, double>> hessian(n, shape.number_hessian_nonzeros(*hessian_model), regularization_size);
   PrimalRegularization<double> regularization(options);
   Statistics statistics;
   regularization.initialize_statistics(statistics, options);
   regularization.initialize_memory(shape, *hessian_model);
   Vector<double> x0(n, 0.), x(n, 0.);
   Vector<double> y0(model.number_constraints, 0.);
   model.initial_primal_point(x0);
   model.project_onto_variable_bounds(x0);
   model.initial_dual_point(y0);
   const double rhos[] = {1., 0.1, 1e-2, 1., 10., 1e-3};
   std::printf("{\"mode\": \"convexify\", \"linear_solver\": \"%s\", \"dimension\": %zu, \"model_variables\": %zu, \"points\": [",
      options.get_string("linear_solver").c_str(), n, n_model);
   for (size_t k = 0; k < sizeof(rhos) / sizeof(rhos[0]); ++k) {
      // deterministic primal-dual points around the initial point
      for (size_t i = 0; i < n; ++i) {
         x[i] = (i < n_model ? x0[i] : 0.) + 0.25 * static_cast<double>(k) * std::sin(1.7 * static_cast<double>(i) + 1.);
      }
      model.project_onto_variable_bounds(x);
      Multipliers multipliers(n, model.number_constraints);
      for (size_t j = 0; j < model.number_constraints; ++j) {
         multipliers.constraints[j] = y0[j] + 0.5 * static_cast<double>(k) * std::cos(1.3 * static_cast<double>(j) + 0.5);
      }
      const l1RelaxedProblem problem(model, rhos[k], coefficient);
      const size_t before = kkt_trace::events().size();
      hessian.reset();
      problem.evaluate_lagrangian_hessian(statistics, *hessian_model, x, multipliers, hessian);
      const Inertia expected_inertia{problem.get_number_original_variables(), 0, n - problem.get_number_original_variables()};
      double smallest = hessian.smallest_diagonal_entry(expected_inertia.positive);
      regularization.regularize_hessian(statistics, hessian, problem.get_primal_regularization_variables(), expected_inertia);
      std::printf("%s{\"rho\": %.17g, \"smallest_diagonal_entry\": %.17g, \"regularization\": %.17g, \"factorizations\": %zu}",
         k ? ", " : "", rhos[k], smallest, regularization.get_primal_regularization_factor(), kkt_trace::events().size() - before);
   }
   std::printf("], \"inertia_trace\": [");
   bool first = true;
   for (const auto& e: kkt_trace::events()) {
      if (e.kind != 'F') continue;
      std::printf("%s[%zu, %lld, %lld, %lld]", first ? "" : ", ", e.dimension, static_cast<long long>(e.positive),
         static_cast<long long>(e.negative), static_cast<long long>(e.zero));
      first = false;
   }
   std::printf("]}\n");
}

int main(int argc, char* argv[]) {
   if (argc < 2) {
      std::cerr << "usage: " << argv[0] << " hs015 [option=value ...]\n";
      return 2;
   }
   std::string model_name = argv[1];
   install_crosscheck();
   const bool convexify = model_name.rfind("convexify:", 0) == 0;
   if (convexify) model_name = model_name.substr(10);
   try {
      // option precedence of uno_ampl.cpp:106-128: defaults -> solvers -> preset -> command line
      Options options = DefaultOptions::load();
      options.overwrite_with(DefaultOptions::determine_solvers());
      Options command_line = Options::get_command_line_options(argc, argv, 2);
      const auto preset = command_line.get_string_optional("preset");
      options.overwrite_with(Presets::get_preset_options(preset.has_value() ? preset :
         std::optional<std::string>(convexify ? "byrd" : "ipopt")));
      options.overwrite_with(command_line);
      Logger::set_logger(options.get_string("logger"));

      std::unique_ptr<Model> model;
      if (model_name == "hs015") {
         model = std::make_unique<HS015Model>();
      }
      else if (model_name.rfind("arrowband:", 0) == 0) {  // synthetic arrowband NLP of KKT dimension N
         model = std::make_unique<ArrowbandModel>(std::stoul(model_name.substr(10)));
      }
      else if (model_name.rfind("arrowband_ineq:", 0) == 0) {  // the same with -1 <= A x - b <= 1
         model = std::make_unique<ArrowbandModel>(std::stoul(model_name.substr(15)), true);
      }
      else if (model_name.size() > 3 && model_name.compare(model_name.size() - 3, 3, ".nl") == 0) {
         model = std::make_unique<NLModel>(model_name);  // ASL-free .nl reader (models/NLModel.hpp)
      }
      else {
         throw std::invalid_argument("unknown model " + model_name);
      }
      if (convexify) {
         run_convexification(*model, options);
         return 0;
      }
      model = ModelFactory::reformulate(std::move(model), options);
      Iterate initial_iterate(model->number_variables, model->number_constraints);
      model->initial_primal_point(initial_iterate.primals);
      model->project_onto_variable_bounds(initial_iterate.primals);
      model->initial_dual_point(initial_iterate.multipliers.constraints);
      initial_iterate.feasibility_multipliers.reset();

      Uno uno{model->number_constraints, options};
      NoUserCallbacks callbacks{};
      const auto t_solve = std::chrono::steady_clock::now();
      const Result result = uno.solve(*model, initial_iterate, options, callbacks);
      const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_solve).count();

      std::printf("{\"model\": \"%s\", \"linear_solver\": \"%s\", \"status\": %d, \"iterations\": %zu, \"objective\": %.17g",
         model_name.c_str(), options.get_string("linear_solver").c_str(), static_cast<int>(result.optimization_status),
         result.iteration, result.solution.evaluations.objective);
      std::printf(", \"primals\": [");
      const size_t shown = result.number_variables <= 64 ? result.number_variables : 0;  // large models: summary only
      for (size_t i = 0; i < shown; ++i) {
         std::printf("%s%.17g", i ? ", " : "", result.solution.primals[i]);
      }
      double ps = 0., pq = 0., pm = 0.;
      for (size_t i = 0; i < result.number_variables; ++i) {
         const double v = result.solution.primals[i];
         ps += v; pq += v * v; pm = std::max(pm, std::fabs(v));
      }
      std::printf("], \"primals_summary\": [%.17g, %.17g, %.17g", ps, pq, pm);
      // dual side (north_star: primal/dual residuals): multipliers of the constraints and of the bounds,
      // and the reference's own residual measures of the final iterate (Iterate.hpp:43-46, DualResiduals.hpp)
      const auto print_vector = [](const char* name, const Vector<double>& v, size_t count, bool full) {
         std::printf("], \"%s\": [", name);
         if (full) {
            for (size_t i = 0; i < count; ++i) std::printf("%s%.17g", i ? ", " : "", v[i]);
         }
         double s = 0., q = 0., m = 0.;
         for (size_t i = 0; i < count; ++i) { s += v[i]; q += v[i] * v[i]; m = std::max(m, std::fabs(v[i])); }
         std::printf("], \"%s_summary\": [%.17g, %.17g, %.17g", name, s, q, m);
      };
      const bool full = result.number_variables <= 64 && result.number_constraints <= 64;
      print_vector("constraint_multipliers", result.solution.multipliers.constraints, result.number_constraints, full);
      print_vector("lower_bound_multipliers", result.solution.multipliers.lower_bounds, result.number_variables, full);
      print_vector("upper_bound_multipliers", result.solution.multipliers.upper_bounds, result.number_variables, full);
      std::printf("], \"residuals\": [%.17g, %.17g, %.17g", result.solution.primal_feasibility,
         result.solution.residuals.stationarity, result.solution.residuals.complementarity);
      size_t nf = 0, ns = 0;
      for (const auto& e: kkt_trace::events()) {
         (e.kind == 'F' ? nf : ns)++;
      }
      std::printf("], \"factorizations\": %zu, \"solves\": %zu, \"inertia_trace\": [", nf, ns);
      bool first = true;
      for (const auto& e: kkt_trace::events()) {
         if (e.kind != 'F') continue;
         std::printf("%s[%zu, %lld, %lld, %lld]", first ? "" : ", ", e.dimension, static_cast<long long>(e.positive),
            static_cast<long long>(e.negative), static_cast<long long>(e.zero));
         first = false;
      }
      {
         const auto& pr = kkt_trace::profile();
         const double plugin = pr.evaluate + pr.assemble + pr.regularize + pr.rhs + pr.solve + pr.direction;
         std::printf("], \"host_profile_s\": {\"wall\": %.6f, \"plugin_orchestration\": %.6f, \"evaluate\": %.6f, "
            "\"assemble_coo\": %.6f, \"regularize\": %.6f, \"factorize_inertia\": %.6f, \"rhs\": %.6f, \"solve\": %.6f, "
            "\"direction\": %.6f, \"uno_core_outside_plugin\": %.6f, \"orchestration_calls\": %zu", wall, plugin, pr.evaluate,
            pr.assemble, pr.regularize, pr.factorize, pr.rhs, pr.solve, pr.direction, wall - plugin, pr.calls);
         if (pr.assemble_profiled > 0) {  // UNO_HIPLDL_PROFILE_ASSEMBLY=1: assemble_coo split (the second pass is
                                          // outside plugin_orchestration and inside uno_core_outside_plugin)
            std::printf(", \"assemble_split\": {\"assemblies\": %zu, \"model_and_uno_loops\": %.6f, \"plugin_storage\": %.6f}",
               pr.assemble_profiled, pr.assemble_model, pr.assemble - pr.assemble_model);
         }
         std::printf("}");
      }
      std::printf(", \"crosscheck\": [");
      for (size_t k = 0; k < crosscheck_records.size(); ++k) std::printf("%s%s", k ? ", " : "", crosscheck_records[k].c_str());
      std::printf("]}\n");
   }
   catch (std::exception& exception) {
      std::printf("{\"error\": \"%s\"}\n", exception.what());
      return 1;
   }
   return 0;
}
