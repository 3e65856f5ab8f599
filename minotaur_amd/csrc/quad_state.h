// Host state of a loaded quadratic problem (mgpu_load_quad), shared by the
// K2 runtime (quad_runtime.cpp) and the glob tree (glob_runtime.cpp).
#pragma once

#include "ctx.h"

struct QuadState {
  DevQuad dq{};
  int nv0 = 0, nv = 0, R = 0;
  std::vector<int32_t> sq_x, sq_y, bil_x0, bil_x1, bil_y;
  // the original functions as loaded (function ncon = the objective when
  // has_obj) and the variable types, host copies
  int ncon = 0;
  bool has_obj = false;
  std::vector<int32_t> h_lptr, h_lvar, h_qptr, h_qv1, h_qv2, h_vtype;
  std::vector<double> h_lval, h_qval, h_clb, h_cub;
  bool obj_in_prog1 = false;
  double obj_const = 0.0;
  DevBuf vtype, sq, bil, fun[2], term[2];
  DevBuf io_lb_in, io_ub_in, io_lb_out, io_ub_out, io_rin, io_rout, io_inf, io_nm, io_kind,
      io_idx, io_v1, io_v2, scratch;
  void release() {
    for (DevBuf *b : {&vtype, &sq, &bil, &fun[0], &fun[1], &term[0], &term[1], &io_lb_in,
                      &io_ub_in, &io_lb_out, &io_ub_out, &io_rin, &io_rout, &io_inf, &io_nm,
                      &io_kind, &io_idx, &io_v1, &io_v2, &scratch})
      b->release();
  }
};

