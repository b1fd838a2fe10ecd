// KKTTrace.hpp -- records every factorization (dimension, inertia) and solve the plugin performs, so
// a driver can compare the sequence produced by the GPU backend with the oracle's (tests only).
#ifndef UNO_KKT_TRACE_H
#define UNO_KKT_TRACE_H

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
} // namespace kkt_trace

#endif
