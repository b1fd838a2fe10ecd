// uno_kkt_driver.cpp -- runs the reference Uno core (libuno built from /root/reference by
// oracle/ref/Makefile) on a hand-coded model with a KKT plugin chosen by linear_solver=..., and prints
// one JSON object: status, iterations, solution and the sequence of (dimension, inertia) of every
// factorization the plugin performed.  This is the in-container stand-in for `uno_ampl model.nl -AMPL
// preset=ipopt linear_solver=HIPLDL` (bindings/AMPL/uno_ampl.cpp:78-139; ASL is not available).
//
// usage: uno_kkt_driver <model> [option=value ...]     model: hs015 (hand-coded), arrowband:<N> (synthetic NLP) or a path to a text .nl file
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <iostream>
#include <memory>
#include <string>

#include "KKTTrace.hpp"
#include "Uno.hpp"
#include "model/ModelFactory.hpp"
#include "models/HS015Model.hpp"
#include "models/NLModel.hpp"
#include "models/ArrowbandModel.hpp"
#include "optimization/Iterate.hpp"
#include "optimization/Result.hpp"
#include "options/DefaultOptions.hpp"
#include "options/Options.hpp"
#include "options/Presets.hpp"
#include "tools/Logger.hpp"
#include "tools/UserCallbacks.hpp"

using namespace uno;

int main(int argc, char* argv[]) {
   if (argc < 2) {
      std::cerr << "usage: " << argv[0] << " hs015 [option=value ...]\n";
      return 2;
   }
   const std::string model_name = argv[1];
   try {
      // option precedence of uno_ampl.cpp:106-128: defaults -> solvers -> preset -> command line
      Options options = DefaultOptions::load();
      options.overwrite_with(DefaultOptions::determine_solvers());
      Options command_line = Options::get_command_line_options(argc, argv, 2);
      const auto preset = command_line.get_string_optional("preset");
      options.overwrite_with(Presets::get_preset_options(preset.has_value() ? preset : std::optional<std::string>("ipopt")));
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
      model = ModelFactory::reformulate(std::move(model), options);
      Iterate initial_iterate(model->number_variables, model->number_constraints);
      model->initial_primal_point(initial_iterate.primals);
      model->project_onto_variable_bounds(initial_iterate.primals);
      model->initial_dual_point(initial_iterate.multipliers.constraints);
      initial_iterate.feasibility_multipliers.reset();

      Uno uno{model->number_constraints, options};
      NoUserCallbacks callbacks{};
      const Result result = uno.solve(*model, initial_iterate, options, callbacks);

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
      std::printf("]}\n");
   }
   catch (std::exception& exception) {
      std::printf("{\"error\": \"%s\"}\n", exception.what());
      return 1;
   }
   return 0;
}
