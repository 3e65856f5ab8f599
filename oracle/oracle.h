/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/README.md).
 * CPU restatements of the reference algorithms on the hot path.  Loaded only
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 */
#ifndef MGPU_ORACLE_H
#define MGPU_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_OBJ_LOOP_CAP 100000L

/* Shared (per batch) linear problem: CSR rows in ascending column order
 * (the reference's VariableGroup order, Types.cpp:30-34), the column->rows
 * pattern used by changeBFlag_, and the linear objective. */
typedef struct {
  int n, m;
  const int *rowptr, *colidx;
  const double *val;
  const double *rlo, *rhi;
  const int *colptr, *rowidx;
  const int *vtype;        /* Types.h:83-89 numerics */
  int nobj;
  const int *objidx;
  const double *objval;
  int cons_bad;            /* some row has lb > ub + 1e-8 (checkBounds_) */
} orc_lin_problem;

int orc_linear_fbbt_node(const orc_lin_problem *P, double *lb, double *ub,
                         int has_inc, double inc_ub, unsigned char *flag,
                         int mod_cap, int *mod_var, int *mod_lu,
                         double *mod_val, int *nmods_out);

int orc_linear_fbbt_batch(const orc_lin_problem *P, int B,
                          const double *lb_in, const double *ub_in,
                          double *lb_out, double *ub_out, int has_inc,
                          double inc_ub, int *infeas, int *nmods,
                          unsigned char *flag_scratch, int mod_cap,
                          int *mod_var, int *mod_lu, double *mod_val);

/* LP for the dual simplex restatement: CSC of A. */
typedef struct {
  int n, m;
  const int *colptr, *rowidx;
  const double *cval;
  const double *c;
  const double *rlo, *rhi;
} orc_lp;

/* path warm starts: at most this many pivots per path (= MGPU_PATH_MAX) */
#define ORC_PATH_MAX 32

int orc_dual_simplex(const orc_lp *P, const double *lb, const double *ub,
                     int *ws_head, signed char *ws_st, double *ws_binv, double *ws_d,
                     int have_ws, int have_binv, int iter_limit, double *obj_out,
                     double *x_out, double *y_out, int *iters_out);

/* Quadratic node FBBT (QuadHandler::presolveNode).  Same layout as the
 * reference driver's QSpec (oracle/ref/ref_quad.cpp). */
typedef struct {
  int nv0, nv;
  const int *vtype;
  const double *vlb, *vub;
  int nsq;
  const int *sq_x, *sq_y;
  int nbil;
  const int *bil_x0, *bil_x1, *bil_y;
  int ncon;                 /* original quadratic constraints; the objective */
  const int *lptr, *lvar;   /* is function ncon when has_obj               */
  const double *lval;
  const int *qptr, *qv1, *qv2;
  const double *qval;
  const double *clb, *cub;
  int has_obj;
  double obj_const;
} orc_qspec;

void orc_quad_rows(const orc_qspec *S, const double *lb, const double *ub, double *rows);
void orc_quad_update_rows(const orc_qspec *S, double *lb, double *ub, double *rows);
int orc_quad_fbbt_batch(const orc_qspec *S, int B, const double *lb_in, const double *ub_in,
                        double best, int qt, const double *rows_in, long rows_stride,
                        double *lb_out, double *ub_out, int *infeas, int *nmods,
                        double *rows_out, int mod_cap, int *mod_kind, int *mod_idx,
                        double *mod_v1, double *mod_v2);

#ifdef __cplusplus
}
#endif
#endif
