// StagedCOOMatrix.hpp -- the plugin-owned augmented matrix whose values travel to the GPU while Uno is still
// assembling them (the "GPU-staging SymmetricMatrix subclass" of SURVEY.md 7 step 3).
//
// A SymmetricMatrix<size_t, double> (uno/linear_algebra/SymmetricMatrix.hpp:17-95) with the storage semantics
// of SparseSymmetricMatrix<COOFormat> (COOFormat.hpp:62-127): the regularization diagonal is inserted first
// (positions [0, regularization_size)), set_regularization overwrites those positions, insert appends in
// Uno's assembly order, and iteration / data_pointer / smallest_diagonal_entry see the same entries in the
// same order -- so the analysed pattern, the values the solver factors and every Uno-side query are those of
// the MUMPS adapter's matrix (MUMPSSolver.hpp:52).
//
// What differs:
// - the upload: after every `chunk` inserted entries the new range is handed to a stager (the plugin binds
//   uno_kkt_stage_values, an asynchronous host-to-device copy on its own stream), so the PCIe transfer of the
//   ~160 MB of values at configs[2] runs under Uno's assembly of the later entries instead of after it.
//   flush() stages the tail and, when set_regularization touched them, the regularization positions again;
//   the factorization then reads the device copy (uno_kkt_factorize(h, NULL, 0)).
// - the insert after the symbolic analysis: the pattern is fixed from then on (SURVEY.md 8(b) invariant 1,
//   PrimalDualRegularization.hpp:145-149 analyses once), so freeze_pattern() keeps the analysed row / column
//   indices and every later insert stores only its value -- one store into the (page-locked) value array,
//   no row / column push_back and no capacity growth.  Option UNO_HIPLDL_CHECK_PATTERN=1 (tests) compares
//   each insert's indices with the frozen pattern and throws on a difference.
// The value storage is allocated once at the full capacity (stable address: the library may page-lock it,
// option pin_host_values).
#ifndef UNO_STAGEDCOOMATRIX_H
#define UNO_STAGEDCOOMATRIX_H

#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <functional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "linear_algebra/SymmetricMatrix.hpp"
#include "symbolic/Collection.hpp"

namespace uno {
   class StagedCOOMatrix : public SymmetricMatrix<size_t, double> {
   public:
      // stage(values, first, count): values[first, first + count) are final until the next reset()
      using Stager = std::function<void(const double* values, size_t first, size_t count)>;

      StagedCOOMatrix() = default;
      StagedCOOMatrix(size_t dimension, size_t capacity, size_t regularization_size):
            SymmetricMatrix<size_t, double>(), n(dimension), cap(capacity + regularization_size), reg_size(regularization_size) {
         this->values.assign(this->cap, 0.0);
         this->rows.reserve(this->cap);
         this->cols.reserve(this->cap);
         const char* env = std::getenv("UNO_HIPLDL_CHECK_PATTERN");
         this->check_pattern = env != nullptr && std::atoi(env) != 0;
         this->reset();
      }
      StagedCOOMatrix& operator=(StagedCOOMatrix&& other) = default;

      // bind (or unbind, with an empty function) the stager; chunk = entries per staged range
      void set_stager(Stager s, size_t chunk) {
         this->stager = std::move(s);
         this->chunk = std::max<size_t>(chunk, 1);
         this->staged = std::min(this->reg_size, this->nnz);  // entries already present: staged by the next flush()
         this->reg_dirty = true;
      }
      [[nodiscard]] bool staging() const { return static_cast<bool>(this->stager); }

      // the symbolic analysis saw the entries present now: from here on inserts store values only
      void freeze_pattern() {
         this->rows.resize(this->nnz);
         this->cols.resize(this->nnz);
         this->frozen_nnz = this->nnz;
         this->frozen = true;
      }
      [[nodiscard]] bool pattern_frozen() const { return this->frozen; }

      // stage what has not been staged since reset(): the tail, and the regularization positions if edited
      void flush() {
         if (!this->stager) return;
         const size_t reg_end = std::min(this->reg_size, this->nnz);
         if (this->reg_dirty && reg_end > 0) this->stager(this->values.data(), 0, reg_end);
         const size_t first = std::max(this->staged, reg_end);
         if (this->nnz > first) this->stager(this->values.data(), first, this->nnz - first);
         this->staged = this->nnz;
         this->reg_dirty = false;
      }

      // SymmetricMatrix interface (COOFormat semantics)
      void reset() override {
         this->nnz = 0;
         this->staged = 0;
         if (!this->frozen) {
            this->rows.clear();
            this->cols.clear();
            for (size_t i = 0; i < this->reg_size; ++i) this->push(i, i, 0.0);  // COOFormat::initialize_regularization
         }
         else {
            std::fill(this->values.begin(), this->values.begin() + static_cast<std::ptrdiff_t>(this->reg_size), 0.0);
            this->nnz = this->reg_size;
         }
         this->reg_dirty = true;  // set_regularization fills them later: staged at flush()
         this->staged = this->nnz;
      }
      [[nodiscard]] size_t dimension() const override { return this->n; }
      [[nodiscard]] size_t number_nonzeros() const override { return this->nnz; }
      [[nodiscard]] size_t capacity() const override { return this->cap; }

      void insert(size_t row_index, size_t column_index, double term) override {
         if (this->frozen) {
            if (this->nnz >= this->frozen_nnz) {
               throw std::length_error("StagedCOOMatrix: more entries than the analysed pattern");
            }
            if (this->check_pattern && (this->rows[this->nnz] != row_index || this->cols[this->nnz] != column_index)) {
               throw std::logic_error("StagedCOOMatrix: entry " + std::to_string(this->nnz) + " differs from the analysed pattern");
            }
            this->values[this->nnz++] = term;
         }
         else {
            this->push(row_index, column_index, term);
         }
         if (this->stager && this->nnz - this->staged >= this->chunk) {
            this->stager(this->values.data(), this->staged, this->nnz - this->staged);
            this->staged = this->nnz;
         }
      }
      void finalize_column(size_t /*column_index*/) override {}

      [[nodiscard]] double smallest_diagonal_entry(size_t max_dimension) const override {
         std::vector<double> diagonal(max_dimension, 0.0);  // SparseSymmetricMatrix.hpp: duplicates summed
         for (size_t e = 0; e < this->nnz; ++e) {
            if (this->rows[e] == this->cols[e] && this->rows[e] < max_dimension) diagonal[this->rows[e]] += this->values[e];
         }
         return *std::min_element(diagonal.begin(), diagonal.end());
      }

      void set_regularization(const Collection<size_t>& indices, size_t offset, double factor) override {
         for (size_t index: indices) {  // COOFormat::set_regularization: the diagonal terms stored first
            this->values[index + offset] = factor;
         }
         this->reg_dirty = true;
      }

      [[nodiscard]] const double* data_pointer() const noexcept override { return this->values.data(); }
      [[nodiscard]] double* data_pointer() noexcept override { return this->values.data(); }

   protected:
      size_t n{0}, cap{0}, reg_size{0}, nnz{0};
      std::vector<double> values{};          // cap entries, allocated once (stable address)
      std::vector<size_t> rows{}, cols{};    // the pattern (frozen after the analysis)
      Stager stager{};
      size_t chunk{1};
      size_t staged{0};       // values[0, staged) handed to the stager since reset()
      bool reg_dirty{false};  // regularization positions to stage (again) at flush()
      bool frozen{false};
      size_t frozen_nnz{0};
      bool check_pattern{false};

      void push(size_t row_index, size_t column_index, double term) {
         if (this->nnz >= this->cap) {
            throw std::length_error("StagedCOOMatrix: capacity exceeded");  // the address must stay stable
         }
         this->values[this->nnz] = term;
         this->rows.push_back(row_index);
         this->cols.push_back(column_index);
         this->nnz++;
      }

      [[nodiscard]] std::tuple<size_t, size_t, double> dereference_iterator(size_t /*column_index*/, size_t nonzero_index) const override {
         return {this->rows[nonzero_index], this->cols[nonzero_index], this->values[nonzero_index]};
      }
      void increment_iterator(size_t& column_index, size_t& nonzero_index) const override {
         nonzero_index++;
         if (nonzero_index == this->nnz) column_index = this->n;  // COOFormat::increment_iterator
      }
   };
} // namespace

#endif // UNO_STAGEDCOOMATRIX_H
