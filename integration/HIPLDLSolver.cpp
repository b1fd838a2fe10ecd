// HIPLDLSolver.cpp -- see HIPLDLSolver.hpp.  Each method names the MUMPS call it replaces.
#include "HIPLDLSolver.hpp"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "KKTTrace.hpp"
#include "ingredients/subproblem/Subproblem.hpp"
#include "linear_algebra/SymmetricMatrix.hpp"
#include "optimization/WarmstartInformation.hpp"

namespace uno {
   namespace {
      double seconds_since(std::chrono::steady_clock::time_point t0) {
         return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      }
      void* hip_create() {
         uno_kkt_t h = nullptr;
         if (uno_kkt_create(&h, 0) != UNO_KKT_OK) return nullptr;
         // Inside an interior-point solve the values change at every factorization, so delayed pivots
         // (MUMPS passes them to the parent front within JOB=2) would cost the library a re-analysis per
         // new delay.  The plugin therefore relaxes the pivot threshold inside the front instead (ladder
         // u, u/10, u/100, 1e-6, 1e-10) and the library follows such a factorization with one step of
         // iterative refinement (option "refine").  UNO_KKT_OPTIONS=delay_relaxed=1 restores the delays.
         const char* env = std::getenv("UNO_KKT_OPTIONS");
         if (env == nullptr || std::strstr(env, "delay_relaxed") == nullptr) uno_kkt_set_option(h, "delay_relaxed", 0.0);
         // the plugin owns its COO storage (MUMPSSolver.hpp:52): page-lock it once for direct uploads
         if (env == nullptr || std::strstr(env, "pin_host_values") == nullptr) uno_kkt_set_option(h, "pin_host_values", 1.0);
         return h;
      }
      void hip_destroy(void* h) { uno_kkt_destroy(static_cast<uno_kkt_t>(h)); }
      int hip_analyze(void* h, int64_t n, int64_t nnz, const int64_t* r, const int64_t* c) {
         return uno_kkt_analyze(static_cast<uno_kkt_t>(h), n, nnz, r, c);
      }
      int hip_factorize(void* h, const double* v) { return uno_kkt_factorize(static_cast<uno_kkt_t>(h), v, 0); }
      int hip_factorize_update(void* h, const double* v, int64_t first, int64_t count) {
         return uno_kkt_factorize_update(static_cast<uno_kkt_t>(h), v, first, count);
      }
      int hip_inertia(void* h, int64_t* p, int64_t* q, int64_t* z) {
         return uno_kkt_inertia(static_cast<uno_kkt_t>(h), p, q, z);
      }
      int hip_solve(void* h, const double* b, double* x) { return uno_kkt_solve(static_cast<uno_kkt_t>(h), b, x, 0); }
      int hip_stage(void* h, const double* v, int64_t first, int64_t count) {
         return uno_kkt_stage_values(static_cast<uno_kkt_t>(h), v, first, count);
      }
      const char* hip_last_error(void* h) { return uno_kkt_last_error(static_cast<uno_kkt_t>(h)); }

      // UNO_HIPLDL_PROFILE_ASSEMBLY=1 (profiling runs only): the assembly is run a second time into this matrix,
      // whose insert keeps nothing, so the driver's host profile can split Subproblem::assemble_augmented_matrix
      // into the model evaluation with Uno's assembly loops and virtual dispatch (this pass) and the storage
      // cost of the plugin's matrix (the difference)
      class DiscardingMatrix : public SymmetricMatrix<size_t, double> {
      public:
         DiscardingMatrix(size_t n, size_t cap): n(n), cap(cap) {}
         void reset() override { this->nnz = 0; }
         [[nodiscard]] size_t dimension() const override { return this->n; }
         [[nodiscard]] size_t number_nonzeros() const override { return this->nnz; }
         [[nodiscard]] size_t capacity() const override { return this->cap; }
         void insert(size_t row_index, size_t column_index, double term) override {
            this->sink += term + static_cast<double>(row_index ^ column_index);  // keeps the arguments live
            this->nnz++;
         }
         void finalize_column(size_t) override {}
         [[nodiscard]] double smallest_diagonal_entry(size_t) const override { return 0.; }
         void set_regularization(const Collection<size_t>&, size_t, double) override {}
         [[nodiscard]] const double* data_pointer() const noexcept override { return &this->sink; }
         [[nodiscard]] double* data_pointer() noexcept override { return &this->sink; }
         double sink{0.};
      protected:
         [[nodiscard]] std::tuple<size_t, size_t, double> dereference_iterator(size_t, size_t) const override { return {0, 0, 0.}; }
         void increment_iterator(size_t& column_index, size_t& nonzero_index) const override {
            nonzero_index++;
            if (nonzero_index == this->nnz) column_index = this->n;
         }
      private:
         size_t n, cap, nnz{0};
      };
      bool profile_assembly() {
         static const bool on = [] {
            const char* env = std::getenv("UNO_HIPLDL_PROFILE_ASSEMBLY");
            return env != nullptr && std::atoi(env) != 0;
         }();
         return on;
      }
   } // namespace

   const KKTBackend& hip_kkt_backend() {
      static const KKTBackend backend{"HIPLDL", hip_create, hip_destroy, hip_analyze, hip_factorize, hip_factorize_update,
         hip_inertia, hip_solve, hip_last_error, hip_stage};
      return backend;
   }

   HIPLDLSolver::HIPLDLSolver(const KKTBackend& backend): DirectSymmetricIndefiniteLinearSolver(), backend(backend) {
      // MUMPSSolver.cpp:16-37 (JOB=-1, ICNTL settings): pivot threshold, null-pivot detection and
      // equilibration are the library defaults (u = 0.01, eps*1e-5*||A||, iterative scaling)
      this->handle = this->backend.create();
      if (this->handle == nullptr) {
         throw std::runtime_error(std::string(this->backend.name) + ": could not create a solver (no device?)");
      }
   }

   HIPLDLSolver::~HIPLDLSolver() {
      this->backend.destroy(this->handle);  // MUMPSSolver.cpp:46-49 (JOB=-2)
   }

   void HIPLDLSolver::check(int status, const char* what) const {
      if (status != 0) {
         std::string message = std::string(this->backend.name) + " " + what + " failed (" + std::to_string(status) + "): " +
            this->backend.last_error(this->handle);
         throw std::runtime_error(message);
      }
   }

   // MUMPSSolver.cpp:51-70
   void HIPLDLSolver::initialize_memory(size_t number_variables, size_t number_constraints, size_t number_hessian_nonzeros,
         size_t regularization_size) {
      this->dimension = number_variables + number_constraints;
      this->regularization_size = regularization_size;
      const size_t number_nonzeros = number_hessian_nonzeros + regularization_size;
      this->row_indices.reserve(number_nonzeros);
      this->column_indices.reserve(number_nonzeros);
      this->objective_gradient.resize(number_variables);
      this->constraints.resize(number_constraints);
      this->constraint_jacobian.resize(number_constraints, number_variables);
      this->augmented_matrix = StagedCOOMatrix(this->dimension, number_hessian_nonzeros, regularization_size);
      this->rhs.resize(this->dimension);
      this->solution.resize(this->dimension);
   }

   // MUMPSSolver.cpp:72-83 + save_sparsity_to_local_format :149-157 (JOB=1)
   void HIPLDLSolver::do_symbolic_analysis(const SymmetricMatrix<size_t, double>& matrix) {
      this->row_indices.clear();
      this->column_indices.clear();
      for (const auto [row_index, column_index, _]: matrix) {
         this->row_indices.emplace_back(static_cast<int64_t>(row_index));
         this->column_indices.emplace_back(static_cast<int64_t>(column_index));
      }
      this->dimension = matrix.dimension();
      this->analysed_nonzeros = matrix.number_nonzeros();
      if (&matrix == &this->augmented_matrix) {
         // the pattern is fixed from now on (SURVEY.md 8(b) invariant 1): later assemblies store values only
         this->augmented_matrix.freeze_pattern();
      }
      this->check(this->backend.analyze(this->handle, static_cast<int64_t>(matrix.dimension()),
         static_cast<int64_t>(this->row_indices.size()), this->row_indices.data(), this->column_indices.data()), "analyze");
      // from now on the plugin's matrix streams its values to the device as Uno inserts them (chunks of
      // 2^20 entries = 8 MB): the factorization only waits for the last chunk (StagedCOOMatrix.hpp)
      const char* env = std::getenv("UNO_HIPLDL_STAGE");
      const bool stage = this->backend.stage != nullptr && &matrix == &this->augmented_matrix && (env == nullptr || std::atoi(env) != 0);
      if (stage) {
         this->augmented_matrix.set_stager([this](const double* values, size_t first, size_t count) {
            this->check(this->backend.stage(this->handle, values, static_cast<int64_t>(first), static_cast<int64_t>(count)), "stage");
         }, size_t(1) << 20);
      }
      else {
         this->augmented_matrix.set_stager({}, 1);
      }
   }

   // MUMPSSolver.cpp:85-89 (JOB=2): values straight from the COO storage, no copy on the host
   void HIPLDLSolver::do_numerical_factorization(const SymmetricMatrix<size_t, double>& matrix) {
      if (matrix.number_nonzeros() != this->analysed_nonzeros) {
         throw std::runtime_error("HIPLDL: the pattern changed since the symbolic analysis");
      }
      // inertia-correction retry: only the regularization diagonal (positions [0, reg_size)) changed
      const auto t0 = std::chrono::steady_clock::now();
      const bool retry = this->in_regularization && !this->values_fresh && this->backend.factorize_update != nullptr &&
         matrix.data_pointer() == this->augmented_matrix.data_pointer();
      if (retry) {
         this->check(this->backend.factorize_update(this->handle, matrix.data_pointer(), 0,
            static_cast<int64_t>(this->regularization_size)), "factorize");
      }
      else if (&matrix == &this->augmented_matrix && this->augmented_matrix.staging()) {
         this->augmented_matrix.flush();  // the tail (and the regularization diagonal) after the staged chunks
         this->check(this->backend.factorize(this->handle, nullptr), "factorize");
      }
      else {
         this->check(this->backend.factorize(this->handle, matrix.data_pointer()), "factorize");
      }
      this->values_fresh = false;
      this->check(this->backend.inertia(this->handle, &this->positive, &this->negative, &this->zero), "inertia");
      kkt_trace::profile().factorize += seconds_since(t0);
      kkt_trace::record_factorization(this->dimension, this->positive, this->negative, this->zero);
      const size_t index = kkt_trace::factor_count()++;
      if (kkt_trace::factor_hook() != nullptr) {
         kkt_trace::factor_hook()(index, this->dimension, static_cast<int64_t>(this->row_indices.size()), this->row_indices.data(),
            this->column_indices.data(), matrix.data_pointer(), this->positive, this->negative, this->zero);
      }
   }

   // MUMPSSolver.cpp:91-96 (JOB=3): the matrix argument is ignored, the last factorization is used
   void HIPLDLSolver::solve_indefinite_system(const SymmetricMatrix<size_t, double>& /*matrix*/, const Vector<double>& rhs,
         Vector<double>& result) {
      const auto t0 = std::chrono::steady_clock::now();
      this->check(this->backend.solve(this->handle, rhs.data(), result.data()), "solve");
      kkt_trace::profile().solve += seconds_since(t0);
      kkt_trace::record_solve(this->dimension);
   }

   // MUMPSSolver.cpp:98-122: evaluate, assemble, regularize (analysis + factorizations), rhs, solve,
   // primal-dual direction -- the orchestration every Uno plugin repeats
   void HIPLDLSolver::solve_indefinite_system(Statistics& statistics, const Subproblem& subproblem, Direction& direction,
         const WarmstartInformation& warmstart_information) {
      auto& prof = kkt_trace::profile();
      prof.calls++;
      auto t0 = std::chrono::steady_clock::now();
      if (warmstart_information.objective_changed) {
         subproblem.evaluate_objective_gradient(this->objective_gradient);
      }
      if (warmstart_information.constraints_changed) {
         subproblem.evaluate_constraints(this->constraints);
         subproblem.evaluate_jacobian(this->constraint_jacobian);
      }
      prof.evaluate += seconds_since(t0);
      if (warmstart_information.objective_changed || warmstart_information.constraints_changed) {
         t0 = std::chrono::steady_clock::now();
         this->augmented_matrix.reset();
         subproblem.assemble_augmented_matrix(statistics, this->augmented_matrix, this->constraint_jacobian);
         prof.assemble += seconds_since(t0);
         if (profile_assembly()) {
            DiscardingMatrix discard(this->dimension, this->augmented_matrix.capacity());
            t0 = std::chrono::steady_clock::now();
            subproblem.assemble_augmented_matrix(statistics, discard, this->constraint_jacobian);
            prof.assemble_model += seconds_since(t0);
            prof.assemble_profiled++;
            if (discard.number_nonzeros() + this->regularization_size != this->augmented_matrix.number_nonzeros()) {
               throw std::runtime_error("HIPLDL: the profiling assembly inserted a different number of entries");
            }
         }
         this->values_fresh = true;
         struct Scope {  // also reset when the loop throws (UnstableRegularization, FeasibilityRestoration.cpp:103-105)
            bool& flag;
            explicit Scope(bool& f): flag(f) { flag = true; }
            ~Scope() { flag = false; }
         } scope(this->in_regularization);
         t0 = std::chrono::steady_clock::now();
         subproblem.regularize_augmented_matrix(statistics, this->augmented_matrix, subproblem.dual_regularization_factor(), *this);
         prof.regularize += seconds_since(t0);
         t0 = std::chrono::steady_clock::now();
         subproblem.assemble_augmented_rhs(this->objective_gradient, this->constraints, this->constraint_jacobian, this->rhs);
         prof.rhs += seconds_since(t0);
      }
      this->solve_indefinite_system(this->augmented_matrix, this->rhs, this->solution);
      t0 = std::chrono::steady_clock::now();
      subproblem.assemble_primal_dual_direction(this->solution, direction);
      prof.direction += seconds_since(t0);
   }

   // MUMPSSolver.cpp:124-147 (INFOG(12), INFOG(28))
   Inertia HIPLDLSolver::get_inertia() const {
      return {static_cast<size_t>(this->positive), static_cast<size_t>(this->negative), static_cast<size_t>(this->zero)};
   }

   size_t HIPLDLSolver::number_negative_eigenvalues() const {
      return static_cast<size_t>(this->negative);
   }

   size_t HIPLDLSolver::number_zero_eigenvalues() const {
      return static_cast<size_t>(this->zero);
   }

   bool HIPLDLSolver::matrix_is_singular() const {
      return this->zero > 0;
   }

   size_t HIPLDLSolver::rank() const {
      return this->dimension - static_cast<size_t>(this->zero);
   }
} // namespace
