// OracleBackend.cpp -- TEST INFRASTRUCTURE ONLY: the CPU oracle (oracle/kkt_oracle.c) behind the same
// Uno plugin adapter as the GPU backend, registered as linear_solver=ORACLE in test builds.  Used to
// produce golden Uno traces (tests/golden/) that the GPU run must reproduce.
#include <cstdlib>
#include <memory>
#include "HIPLDLSolver.hpp"
#include "kkt_oracle.h"

namespace uno {
   namespace {
      // UNO_ORACLE_ORDERING=1: Cuthill-McKee instead of its reverse (a second valid ordering, to show how far
      // a whole solve's trace depends on the rounding of one ordering; tests/golden/make_c3_golden.sh)
      void* o_create() {
         oracle_kkt_t h = oracle_kkt_create();
         if (const char* o = std::getenv("UNO_ORACLE_ORDERING")) oracle_kkt_set_option(h, "ordering", std::atof(o));
         return h;
      }
      void o_destroy(void* h) { oracle_kkt_destroy(static_cast<oracle_kkt_t>(h)); }
      int o_analyze(void* h, int64_t n, int64_t nnz, const int64_t* r, const int64_t* c) {
         return oracle_kkt_analyze(static_cast<oracle_kkt_t>(h), n, nnz, r, c);
      }
      int o_factorize(void* h, const double* v) { return oracle_kkt_factorize(static_cast<oracle_kkt_t>(h), v); }
      int o_inertia(void* h, int64_t* p, int64_t* q, int64_t* z) {
         return oracle_kkt_inertia(static_cast<oracle_kkt_t>(h), p, q, z);
      }
      int o_solve(void* h, const double* b, double* x) { return oracle_kkt_solve(static_cast<oracle_kkt_t>(h), b, x); }
      const char* o_last_error(void* h) { return oracle_kkt_last_error(static_cast<oracle_kkt_t>(h)); }
      const KKTBackend& oracle_backend() {
         static const KKTBackend b{"ORACLE", o_create, o_destroy, o_analyze, o_factorize, nullptr, o_inertia, o_solve, o_last_error};
         return b;
      }
   } // namespace

   std::unique_ptr<DirectSymmetricIndefiniteLinearSolver<size_t, double>> make_oracle_solver() {
      return std::make_unique<HIPLDLSolver>(oracle_backend());
   }
} // namespace
