// KKTTrace.hpp -- records every factorization (dimension, inertia) and solve the plugin performs, so
// a driver can compare the sequence produced by the GPU backend with the oracle's (tests only).
#ifndef UNO_KKT_TRACE_H
#define UNO_KKT_TRACE_H

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace kkt_trace {
   struct Event {
      char kind;  // 'F' factorization, 'S' solve
      size_t dimension;
      int64_t positive, negative, zero;
   };
   inline std::vector<Event>& events() {
      static std::vector<Event> e;
      return e;
   }
   inline void record_factorization(size_t n, int64_t p, int64_t q, int64_t z) { events().push_back({'F', n, p, q, z}); }
   // optional per-factorization hook (test drivers only): the factorization's index in the run, the COO
   // pattern handed to the backend and the values it factored, and the inertia it reported
   using FactorHook = void (*)(size_t index, size_t n, int64_t nnz, const int64_t* rows, const int64_t* cols,
      const double* values, int64_t positive, int64_t negative, int64_t zero);
   inline FactorHook& factor_hook() {
      static FactorHook h = nullptr;
      return h;
   }
   inline size_t& factor_count() {
      static size_t c = 0;
      return c;
   }
   inline void record_solve(size_t n) { events().push_back({'S', n, 0, 0, 0}); }

   // host-time profile of the plugin's orchestration (HIPLDLSolver::solve_indefinite_system, the
   // MUMPSSolver.cpp:98-122 sequence), seconds accumulated over the run; the driver reports it with the
   // run's wall time, so the remainder is the Uno core's own work outside the linear-solver plugin
   struct Profile {
      double evaluate{0.0};     // objective gradient, constraints, Jacobian (Subproblem::evaluate_*)
      double assemble{0.0};     // Subproblem::assemble_augmented_matrix (COO inserts into the plugin's matrix)
      double assemble_model{0.0};  // UNO_HIPLDL_PROFILE_ASSEMBLY=1: the same assembly into a discarding matrix (model
                                   // evaluation + Uno's loops + virtual insert calls; assemble - this = storage)
      size_t assemble_profiled{0};
      double regularize{0.0};   // Subproblem::regularize_augmented_matrix: inertia-correction loop, factorizations
      double factorize{0.0};    //   of which: the plugin's factorize + inertia calls (device work + value upload)
      double rhs{0.0};          // Subproblem::assemble_augmented_rhs
      double solve{0.0};        // the plugin's solves (JOB=3)
      double direction{0.0};    // Subproblem::assemble_primal_dual_direction
      size_t calls{0};
   };
   inline Profile& profile() {
      static Profile p;
      return p;
   }
} // namespace kkt_trace

#endif
