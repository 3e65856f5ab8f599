//
// HipLinearHandler — LinearHandler whose node FBBT runs on the MI355X
// engine (mgpu_fbbt, include/mgpu.h).
//
// Keeps the Handler plugin surface (src/base/Handler.h:229-231) and every
// other LinearHandler behaviour (root presolve, relaxation building,
// separation) unchanged: only presolveNode (LinearHandler.cpp:1592-1603) is
// overridden.  The kernel returns the exact bounds, infeasibility verdict
// and VarBoundMod log of the reference's simplePresolve, and this adapter
// turns the log back into the same VarBoundMods, in the same order, applied
// to the relaxation and appended to r_mods.
//
// Compiled only against the reference headers (oracle/Makefile `integ`).
//
#ifndef MINOTAURHIPLINEARHANDLER_H
#define MINOTAURHIPLINEARHANDLER_H

#include <cstdint>
#include <vector>

#include "LinearHandler.h"

struct mgpu_ctx;

namespace Minotaur {

class HipLinearHandler : public LinearHandler {
 public:
  HipLinearHandler(EnvPtr env, ProblemPtr problem, int device = 0);
  ~HipLinearHandler();

  bool presolveNode(RelaxationPtr rel, NodePtr node, SolutionPoolPtr s_pool,
                    ModVector &p_mods, ModVector &r_mods);

  std::string getName() const;

  /// Node FBBT calls served by the GPU engine.
  UInt gpuCalls() const { return gpuCalls_; }
  /// Relaxation uploads (mgpu_load_lp): only when rows / objective changed.
  UInt gpuLoads() const { return gpuLoads_; }
  /// Engine failures (load or FBBT); each such node ran the reference's CPU
  /// LinearHandler::presolveNode instead, after an error message.
  UInt gpuErrors() const { return gpuErrors_; }

 private:
  bool loadRel_(RelaxationPtr rel);

  mgpu_ctx *ctx_;
  int device_;
  bool loaded_;
  std::vector<int32_t> rowmap_;  // kernel row -> relaxation constraint
  UInt gpuCalls_, gpuLoads_, gpuErrors_;
  // what is loaded on the device (compared before every node)
  std::vector<int32_t> rowptr_, colidx_, ctype_;
  std::vector<double> val_, rlo_, rhi_, obj_;
  double objoff_;
  std::vector<double> lb_, ub_, olb_, oub_;
  std::vector<int32_t> mvar_, mlu_;
  std::vector<double> mval_;
};

}  // namespace Minotaur
#endif
