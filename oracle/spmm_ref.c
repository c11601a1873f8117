/* ORACLE (test infrastructure only): plain-C restatement of the CSR SpMM
 * C = A @ B that th.spmm(adj, support) computes (reference layer.py:106).
 * Row by row, nonzeros in CSR order.  The f64 form is the parity checker for
 * large inputs; the f32 form (sequential fp32 accumulation) is a scalar CPU
 * port used for error bounds.  Built by __graft_entry__.build() into
 * oracle/liboracle.so with gcc; never linked into the product. */
#include <stdint.h>
#include <string.h>

void oracle_spmm_csr_f64(const int64_t* rowptr, const int64_t* colind, const double* val, int64_t M,
                         const double* B, int64_t F, double* C) {
  for (int64_t r = 0; r < M; ++r) {
    double* c = C + r * F;
    memset(c, 0, (size_t)F * sizeof(double));
    for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      const double a = val[k];
      const double* b = B + colind[k] * F;
      for (int64_t j = 0; j < F; ++j) c[j] += a * b[j];
    }
  }
}

void oracle_spmm_csr_f32(const int64_t* rowptr, const int64_t* colind, const float* val, int64_t M,
                         const float* B, int64_t F, float* C) {
  for (int64_t r = 0; r < M; ++r) {
    float* c = C + r * F;
    memset(c, 0, (size_t)F * sizeof(float));
    for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      const float a = val[k];
      const float* b = B + colind[k] * F;
      for (int64_t j = 0; j < F; ++j) c[j] += a * b[j];
    }
  }
}
