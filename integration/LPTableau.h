//
// LPTableau -- the tableau extras of Minotaur's LPEngine
// (src/base/LPEngine.h:39-73) for an engine that keeps the relaxation as a
// row-major CSR plus bounds and its basis as (head, dense B^-1).  Shared by
// HipLPEngine (the binding) and the CPU test engine oracle/ref/CpuLPEngine.
//
// OsiLPEngine answers these calls with Clp's own arrays
// (src/interfaces/OsiLPEngine.cpp:314-360); the conventions restated here
// are those of Clp 1.17 / Osi 0.108 (third-party/build_third_party:51,57;
// not vendored, absent from the image):
//   * bounds: ClpModel::loadProblem stores a bound beyond +-1e27 as
//     +-COIN_DBL_MAX (= DBL_MAX); getColLower/.../getRowUpper return them so;
//   * right-hand side (OsiSolverInterface::convertBoundToSense): the upper
//     bound of an 'E', 'R' or 'L' row, the lower bound of a 'G' row, 0 for a
//     free row;
//   * matrix by row: entries in ascending column order inside a row (the
//     term order of a Minotaur LinearFunction, Types.cpp:30-34, and of
//     CoinPackedMatrix::reverseOrderedCopyOf), starts / lengths / indices;
//   * getBasics: basic variable of each basis position, a row's slack as
//     ncols + row;
//   * getBInvARow(r): row r of B^-1 [A I] for the slacks s = rhs - Ax
//     (OsiClpSolverInterface flips the sign of the row when its basic
//     variable is a slack, because Clp's logical column is -e_r).  The
//     engines here use Clp's internal form (logical of row r = -e_r, value =
//     the row activity), so B^-1 is that of [A -I] and the same flip applies.
//
#ifndef MINOTAUR_LPTABLEAU_H
#define MINOTAUR_LPTABLEAU_H

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

namespace lptab {

inline double osi_bound(double v) {
  if (v <= -1e27) return -DBL_MAX;
  if (v >= 1e27) return DBL_MAX;
  return v;
}

inline double osi_rhs(double lo, double hi) {
  lo = osi_bound(lo);
  hi = osi_bound(hi);
  if (lo > -DBL_MAX) return hi < DBL_MAX ? hi : lo;
  return hi < DBL_MAX ? hi : 0.0;
}

// The views OsiLPEngine's getters hand out, rebuilt from the engine's mirrors
// (pointers stay valid while n and m do not change).
struct Views {
  std::vector<double> clo, chi, rlo, rhi, rhs, act;
  std::vector<int> rowlen;

  void fill(int n, int m, const int32_t *rowptr, const int32_t *colidx, const double *val,
            const double *c_lo, const double *c_hi, const double *r_lo, const double *r_hi,
            const double *x) {
    clo.resize(n);
    chi.resize(n);
    for (int j = 0; j < n; ++j) {
      clo[j] = osi_bound(c_lo[j]);
      chi[j] = osi_bound(c_hi[j]);
    }
    rlo.resize(m);
    rhi.resize(m);
    rhs.resize(m);
    act.resize(m);
    rowlen.resize(m);
    for (int i = 0; i < m; ++i) {
      rlo[i] = osi_bound(r_lo[i]);
      rhi[i] = osi_bound(r_hi[i]);
      rhs[i] = osi_rhs(r_lo[i], r_hi[i]);
      rowlen[i] = rowptr[i + 1] - rowptr[i];
      double a = 0.0;
      if (x)
        for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) a += val[k] * x[colidx[k]];
      act[i] = a;
    }
  }
};

// B^-1 (column-major [m][m]) of the basis `head` of [A -I] by Gauss-Jordan
// with partial pivoting; false when the basis is singular.
inline bool invert(int n, int m, const int32_t *rowptr, const int32_t *colidx, const double *val,
                   const int32_t *head, std::vector<double> &binv) {
  std::vector<double> B((size_t)m * m, 0.0), I((size_t)m * m, 0.0);  // row-major
  std::vector<int> pos((size_t)n, -1);
  for (int i = 0; i < m; ++i) {
    if (head[i] < 0 || head[i] >= n + m) return false;
    if (head[i] < n) pos[head[i]] = i;
    else B[(size_t)(head[i] - n) * m + i] = -1.0;
    I[(size_t)i * m + i] = 1.0;
  }
  for (int r = 0; r < m; ++r)
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k)
      if (pos[colidx[k]] >= 0) B[(size_t)r * m + pos[colidx[k]]] = val[k];
  for (int c = 0; c < m; ++c) {
    int piv = -1;
    double best = 0.0;
    for (int r = c; r < m; ++r)
      if (std::fabs(B[(size_t)r * m + c]) > best) {
        best = std::fabs(B[(size_t)r * m + c]);
        piv = r;
      }
    if (piv < 0 || best < 1e-12) return false;
    if (piv != c)
      for (int k = 0; k < m; ++k) {
        std::swap(B[(size_t)c * m + k], B[(size_t)piv * m + k]);
        std::swap(I[(size_t)c * m + k], I[(size_t)piv * m + k]);
      }
    const double inv = 1.0 / B[(size_t)c * m + c];
    for (int k = 0; k < m; ++k) {
      B[(size_t)c * m + k] *= inv;
      I[(size_t)c * m + k] *= inv;
    }
    for (int r = 0; r < m; ++r) {
      if (r == c) continue;
      const double f = B[(size_t)r * m + c];
      if (f == 0.0) continue;
      for (int k = 0; k < m; ++k) {
        B[(size_t)r * m + k] -= f * B[(size_t)c * m + k];
        I[(size_t)r * m + k] -= f * I[(size_t)c * m + k];
      }
    }
  }
  binv.assign((size_t)m * m, 0.0);
  for (int i = 0; i < m; ++i)
    for (int k = 0; k < m; ++k) binv[(size_t)k * m + i] = I[(size_t)i * m + k];
  return true;
}

// Osi's tableau row `row` (a basis position): z [n] = e B^-1 A, slack [m] =
// e B^-1, with e = -e_row when that position holds a slack (see above).
inline void binv_a_row(int n, int m, const int32_t *rowptr, const int32_t *colidx,
                       const double *val, const int32_t *head, const double *binv, int row,
                       double *z, double *slack) {
  const double sgn = head[row] >= n ? -1.0 : 1.0;
  std::vector<double> rho((size_t)m);
  for (int k = 0; k < m; ++k) rho[k] = sgn * binv[(size_t)k * m + row];
  if (z) {
    for (int j = 0; j < n; ++j) z[j] = 0.0;
    for (int k = 0; k < m; ++k) {
      if (rho[k] == 0.0) continue;
      for (int t = rowptr[k]; t < rowptr[k + 1]; ++t) z[colidx[t]] += rho[k] * val[t];
    }
  }
  if (slack)
    for (int k = 0; k < m; ++k) slack[k] = rho[k];
}

}  // namespace lptab

#endif
