// Device-side structures of the batched QP relaxation solve (qp_kkt.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mgpu {

constexpr double kQpTolMu = 1e-10;   // complementarity (oracle/qp_ipm.py TOL_MU)
constexpr double kQpTolP = 1e-9;     // primal residual, relative (oracle/qp_ipm.py TOL_P)
constexpr double kQpReg = 1e-12;     // relative regularisation of M
constexpr double kQpStep = 0.995;    // fraction to the boundary

struct DevQP {
  int n, m, np, mp;          // sizes and their multiples of 16
  const double *Q;           // [np][np] symmetric, zero padded
  const double *c;           // [np]
  const double *A;           // [mp][np]
  const double *AT;          // [np][mp]
  const double *b;           // [mp]
  double k;                  // objective constant
  double tp, td;             // primal / dual residual tolerances
};

struct QpWork {
  int B;
  const int32_t *skip;       // [B] or null: nonzero = not solved (status 12, obj +inf)
  double *l, *u;             // [B][np] node boxes (padding fixed at 0)
  double *x, *zl, *zu;       // [B][np]
  double *y;                 // [B][mp]
  double *rd;                // [B][np]
  double *rp;                // [B][mp]
  double *K;                 // [B][np][np]
  double *W;                 // [B][np][mp]
  double *WT;                // [B][mp][np] (W', for W dy)
  double *M;                 // [B][mp][mp]
  int32_t *done, *iters, *status;
  double *obj;
};

size_t qp_step_lds(int np, int mp, int m);
hipError_t launch_qp_init(const DevQP &q, const QpWork &w, hipStream_t s);
// ev (optional): four events recorded before the factor kernel, after it,
// after the W / Schur kernel and after the step kernel
hipError_t launch_qp_iteration(const DevQP &q, const QpWork &w, hipStream_t s,
                               hipEvent_t *ev = nullptr);
hipError_t launch_qp_iteration_check(const DevQP &q, const QpWork &w, hipStream_t s);
hipError_t launch_qp_final(const DevQP &q, const QpWork &w, hipStream_t s);

}  // namespace mgpu
