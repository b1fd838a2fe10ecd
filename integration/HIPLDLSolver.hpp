// HIPLDLSolver.hpp -- Uno linear-solver plugin backed by the MI355X KKT library (include/uno_kkt.h).
//
// Drop-in replacement for uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.hpp:17-66: same base
// class (DirectSymmetricIndefiniteLinearSolver<size_t, double>,
// DirectSymmetricIndefiniteLinearSolver.hpp:11-25), same ownership (the plugin owns the augmented
// COO matrix, rhs and solution, MUMPSSolver.hpp:47-54), registered as linear_solver=HIPLDL by the
// factory overlay in SymmetricIndefiniteLinearSolverFactory.cpp.  Compiled against the reference
// headers; see INTEGRATION.md.
#ifndef UNO_HIPLDLSOLVER_H
#define UNO_HIPLDLSOLVER_H

#include <cstdint>
#include <vector>

#include "ingredients/subproblem_solvers/DirectSymmetricIndefiniteLinearSolver.hpp"
#include "linear_algebra/COOFormat.hpp"
#include "linear_algebra/RectangularMatrix.hpp"
#include "linear_algebra/SparseSymmetricMatrix.hpp"
#include "linear_algebra/SparseVector.hpp"
#include "linear_algebra/Vector.hpp"
#include "StagedCOOMatrix.hpp"
#include "uno_kkt.h"

namespace uno {
   // The factor/solve/inertia entry points the adapter binds (a C ABI; see include/uno_kkt.h).
   // The production backend is the HIP library; the CPU oracle provides the same table for tests.
   struct KKTBackend {
      const char* name;
      void* (*create)();
      void (*destroy)(void* handle);
      int (*analyze)(void* handle, int64_t n, int64_t nnz, const int64_t* row, const int64_t* col);
      int (*factorize)(void* handle, const double* values);
      // refactorization after an edit of positions [first, first + count) of the same host array
      int (*factorize_update)(void* handle, const double* values, int64_t first, int64_t count);
      int (*inertia)(void* handle, int64_t* positive, int64_t* negative, int64_t* zero);
      int (*solve)(void* handle, const double* rhs, double* x);
      const char* (*last_error)(void* handle);
      // optional: asynchronous upload of values[first, first + count) while the caller assembles the rest;
      // factorize(handle, nullptr) then factors the staged values (nullptr: no staging, host-pointer path)
      int (*stage)(void* handle, const double* values, int64_t first, int64_t count){nullptr};
   };
   const KKTBackend& hip_kkt_backend();

   class HIPLDLSolver : public DirectSymmetricIndefiniteLinearSolver<size_t, double> {
   public:
      explicit HIPLDLSolver(const KKTBackend& backend = hip_kkt_backend());
      ~HIPLDLSolver() override;

      void initialize_memory(size_t number_variables, size_t number_constraints, size_t number_hessian_nonzeros,
         size_t regularization_size) override;

      void do_symbolic_analysis(const SymmetricMatrix<size_t, double>& matrix) override;
      void do_numerical_factorization(const SymmetricMatrix<size_t, double>& matrix) override;
      void solve_indefinite_system(const SymmetricMatrix<size_t, double>& matrix, const Vector<double>& rhs,
         Vector<double>& result) override;
      void solve_indefinite_system(Statistics& statistics, const Subproblem& subproblem, Direction& direction,
         const WarmstartInformation& warmstart_information) override;

      [[nodiscard]] Inertia get_inertia() const override;
      [[nodiscard]] size_t number_negative_eigenvalues() const override;
      [[nodiscard]] size_t number_zero_eigenvalues() const;
      [[nodiscard]] bool matrix_is_singular() const override;
      [[nodiscard]] size_t rank() const override;

   protected:
      const KKTBackend& backend;
      void* handle{nullptr};
      size_t dimension{0};
      size_t analysed_nonzeros{0};
      size_t regularization_size{0};
      // inside the adapter's orchestration (solve_indefinite_system below), between the assembly and the
      // right-hand side: the first factorization uploads every value, the inertia-correction retries only
      // the regularization diagonal, which COOFormat stores first (COOFormat.hpp:102-110)
      bool in_regularization{false};
      bool values_fresh{true};
      // inertia of the last factorization, cached (one device sync per factorization)
      int64_t positive{0}, negative{0}, zero{0};

      // COO pattern handed to the device once per analysis (0-based, int64)
      std::vector<int64_t> row_indices{};
      std::vector<int64_t> column_indices{};

      // evaluations (same layout as the MUMPS adapter)
      Vector<double> objective_gradient;
      std::vector<double> constraints;
      RectangularMatrix<double> constraint_jacobian;

      // augmented system: COOFormat semantics, values staged to the device during the assembly
      StagedCOOMatrix augmented_matrix{};
      Vector<double> rhs{};
      Vector<double> solution{};

      void check(int status, const char* what) const;
   };
} // namespace

#endif // UNO_HIPLDLSOLVER_H
