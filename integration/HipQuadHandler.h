//
// HipQuadHandler — QuadHandler whose node FBBT (QuadHandler::presolveNode,
// src/base/QuadHandler.cpp:1204-1269) runs on the MI355X engine
// (mgpu_quad_fbbt, include/mgpu.h).
//
// Keeps the Handler plugin surface (src/base/Handler.h) and every other
// QuadHandler behaviour (registries, relaxation building, separation,
// branching, OBBT) unchanged.  QuadHandler keeps its registries and the
// original problem private, so this adapter records what the kernel needs
// through the same virtual entry points the transformer and relaxer call:
//   addConstraint  -> the y = x0*x1 / y = x^2 registries (QuadHandler.cpp:127-179)
//   relaxInitInc/Full -> the relaxation rows relax_ creates (:1549-1592)
// and reads the original problem's quadratic functions itself.
//
// presolveNode replays the kernel's mod log as the reference does: every
// bound change as a VarBoundMod / VarBoundMod2 applied to p_ (p_mods) and
// to the relaxation (r_mods), every secant / McCormick rewrite as a
// LinConMod on the relaxation (r_mods), in the reference's order.
//
// The first call (the root node) is served by the base class: it is the
// one that runs tightenQuad_ unconditionally, and keeping it there keeps the
// base's private call counter right for later fallbacks.
//
// The kernel works on ONE box; the reference reads x/y bounds from p_ in
// propSqrBnds_/propBilBnds_ and from the relaxation in tightenQuad_ and the
// row rewrites.  When p_ and the relaxation disagree on a handled variable
// (e.g. branching changed only the relaxation) the call is served by the
// base QuadHandler on the CPU; cpuCalls() counts those.
//
// Compiled only against the reference headers (oracle/Makefile `integ`).
//
#ifndef MINOTAURHIPQUADHANDLER_H
#define MINOTAURHIPQUADHANDLER_H

#include <cstdint>
#include <vector>

#include "QuadHandler.h"

struct mgpu_ctx;

namespace Minotaur {

class HipQuadHandler : public QuadHandler {
 public:
  HipQuadHandler(EnvPtr env, ProblemPtr problem, ProblemPtr orig_p, int device = 0);
  ~HipQuadHandler();

  void addConstraint(ConstraintPtr newcon);
  void relaxInitFull(RelaxationPtr rel, bool *is_inf);
  void relaxInitInc(RelaxationPtr rel, bool *is_inf);
  SolveStatus presolve(PreModQ *pre_mods, bool *changed, Solution **sol);
  bool presolveNode(RelaxationPtr rel, NodePtr node, SolutionPoolPtr s_pool,
                    ModVector &p_mods, ModVector &r_mods);
  std::string getName() const;

  UInt gpuCalls() const { return gpuCalls_; }
  UInt cpuCalls() const { return cpuCalls_; }

 private:
  struct Sq { VariablePtr x, y; };
  struct Bil { VariablePtr x0, x1, y; };
  void recordRows_(RelaxationPtr rel, UInt first);
  bool load_();

  EnvPtr env2_;
  ProblemPtr p2_, orig2_;
  mgpu_ctx *ctx_;
  std::vector<Sq> sq_;
  std::vector<Bil> bil_;
  std::vector<ConstraintPtr> rows_;   // relaxation rows: squares, then 4 per bilinear
  bool loaded_, doqt_;
  UInt calls_, gpuCalls_, cpuCalls_;
};

}  // namespace Minotaur
#endif
