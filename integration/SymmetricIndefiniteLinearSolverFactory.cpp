// Overlay of uno/ingredients/subproblem_solvers/SymmetricIndefiniteLinearSolverFactory.cpp:31-84
// that registers the MI355X backend as linear_solver=HIPLDL (and, in test builds compiled with
// UNO_KKT_WITH_ORACLE, the CPU oracle as linear_solver=ORACLE).  Link this file instead of the
// reference one; nothing else in Uno changes.
#include <stdexcept>
#include <string>
#include "ingredients/subproblem_solvers/SymmetricIndefiniteLinearSolverFactory.hpp"
#include "ingredients/subproblem_solvers/DirectSymmetricIndefiniteLinearSolver.hpp"
#include "linear_algebra/Vector.hpp"
#include "HIPLDLSolver.hpp"

namespace uno {
#ifdef UNO_KKT_WITH_ORACLE
   std::unique_ptr<DirectSymmetricIndefiniteLinearSolver<size_t, double>> make_oracle_solver();
#endif

   std::unique_ptr<DirectSymmetricIndefiniteLinearSolver<size_t, double>> SymmetricIndefiniteLinearSolverFactory::create(
         const std::string& linear_solver) {
      if (linear_solver == "HIPLDL") {
         return std::make_unique<HIPLDLSolver>();
      }
#ifdef UNO_KKT_WITH_ORACLE
      if (linear_solver == "ORACLE") {
         return make_oracle_solver();
      }
#endif
      std::string message = "The linear solver ";
      message.append(linear_solver).append(" is unknown").append("\n").append("The following values are available: ")
            .append(join(SymmetricIndefiniteLinearSolverFactory::available_solvers(), ", "));
      throw std::invalid_argument(message);
   }

   std::vector<std::string> SymmetricIndefiniteLinearSolverFactory::available_solvers() {
      std::vector<std::string> solvers{"HIPLDL"};
#ifdef UNO_KKT_WITH_ORACLE
      solvers.emplace_back("ORACLE");
#endif
      return solvers;
   }
} // namespace
