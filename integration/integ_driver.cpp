// TEST INFRASTRUCTURE ONLY — drives the reference's own solver stack
// (BranchAndBound, PCBProcessor, NodeIncRelaxer, ReliabilityBrancher,
// IntVarHandler, LinearHandler; compiled from /root/reference/src/base) with
// the MI355X engine plugged in through the unchanged plugin surface:
// HipLPEngine as the LPEngine, HipLinearHandler as the linear handler.
// Mirrors the reference's own tests src/testing/AMPLOsiUT.cpp:46-170
// (testOsiLP, testOsiLP2, testOsiWarmStart, testOsiBnB), with the instances
// built programmatically from src/testing/instances/*.mod (ASL is absent).
#include <cmath>
#include <vector>

#include "BranchAndBound.h"
#include "TreeManager.h"
#include "Environment.h"
#include "Function.h"
#include "HipLPEngine.h"
#include "HipLinearHandler.h"
#include "IntVarHandler.h"
#include "LinearFunction.h"
#include "LinearHandler.h"
#include "NodeIncRelaxer.h"
#include "Objective.h"
#include "Option.h"
#include "PCBProcessor.h"
#include "Problem.h"
#include "ReliabilityBrancher.h"
#include "Variable.h"

using namespace Minotaur;

namespace {

ProblemPtr build(EnvPtr env, int n, int m, const int *rowptr, const int *colidx,
                 const double *val, const double *rlo, const double *rhi, const int *vtype,
                 const double *vlb, const double *vub, const double *obj, double objc,
                 int maximize) {
  ProblemPtr p = (ProblemPtr) new Problem(env);
  std::vector<VariablePtr> vars;
  for (int j = 0; j < n; ++j) vars.push_back(p->newVariable(vlb[j], vub[j], (VariableType)vtype[j]));
  for (int i = 0; i < m; ++i) {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) lf->addTerm(vars[colidx[k]], val[k]);
    p->newConstraint((FunctionPtr) new Function(lf), rlo[i], rhi[i]);
  }
  LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
  for (int j = 0; j < n; ++j)
    if (obj[j] != 0.0) lf->addTerm(vars[j], obj[j]);
  p->newObjective((FunctionPtr) new Function(lf), objc, maximize ? Maximize : Minimize);
  p->calculateSize();
  return p;
}

}  // namespace

extern "C" {

// AMPLOsiUT::testOsiLP + testOsiWarmStart on lp0 (Wolsey p.95):
// out[0..2] objective after solve / changeObj(NULL,2) / negateObj,
// out[3] warm re-solve objective; st[0..3] statuses; iters[0] warm iterations.
int integ_lp0(int device, double *out, int *st, int *iters) {
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  const int rowptr[] = {0, 2, 3, 5};
  const int colidx[] = {0, 1, 1, 0, 1};
  const double val[] = {7, -2, 1, 2, -2};
  const double rlo[] = {-INFINITY, -INFINITY, -INFINITY};
  const double rhi[] = {14, 3, 3};
  const int vt[] = {Continuous, Continuous};
  const double vlb[] = {-INFINITY, -INFINITY}, vub[] = {INFINITY, INFINITY};
  const double obj[] = {4, -1};
  ProblemPtr inst = build(env, 2, 3, rowptr, colidx, val, rlo, rhi, vt, vlb, vub, obj, 0.0, 1);
  HipLPEngine *e = new HipLPEngine(env, device);
  e->load(inst);
  st[0] = e->solve();
  out[0] = e->getSolutionValue();
  WarmStartPtr ws = e->getWarmStartCopy();
  // testOsiWarmStart: a second engine loads the warm start: 0 iterations
  HipLPEngine *e2 = new HipLPEngine(env, device);
  e2->load(inst);
  e2->loadFromWarmStart(ws);
  st[3] = e2->solve();
  out[3] = e2->getSolutionValue();
  iters[0] = e2->getIterationCount();
  delete e2;
  e->load(inst);
  e->solve();
  inst->changeObj(FunctionPtr(), 2.0);
  st[1] = e->solve();
  out[1] = e->getSolutionValue();
  inst->negateObj();
  st[2] = e->solve();
  out[2] = e->getSolutionValue();
  delete ws;
  delete e;
  delete inst;
  delete env;
  return 0;
}

// AMPLOsiUT::testOsiLP2: lp_eg0 is infeasible.
int integ_lp_eg0(int device) {
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  const int rowptr[] = {0, 2, 4};
  const int colidx[] = {0, 1, 0, 2};
  const double val[] = {1, 1, 1, 1};
  const double rlo[] = {-INFINITY, -INFINITY}, rhi[] = {3, 0};
  const int vt[] = {Continuous, Continuous, Continuous};
  const double vlb[] = {0, 0, 1}, vub[] = {INFINITY, INFINITY, INFINITY};
  const double obj[] = {1, 1, 1};
  ProblemPtr inst = build(env, 3, 2, rowptr, colidx, val, rlo, rhi, vt, vlb, vub, obj, 0.0, 0);
  HipLPEngine *e = new HipLPEngine(env, device);
  e->load(inst);
  int s = e->solve();
  delete e;
  delete inst;
  delete env;
  return s;
}

// AMPLOsiUT::testOsiBnB generalised: the reference BranchAndBound with
// IntVarHandler + (reference LinearHandler | HipLinearHandler), PCBProcessor,
// ReliabilityBrancher and NodeIncRelaxer, all on a HipLPEngine.
// res[0] = UB, res[1] = LB; cnt[0] = nodes processed, cnt[1] = LP solves,
// cnt[2] = GPU FBBT calls.
int integ_bnb(int device, int hip_fbbt, int n, int m, const int *rowptr, const int *colidx,
              const double *val, const double *rlo, const double *rhi, const int *vtype,
              const double *vlb, const double *vub, const double *obj, double objc,
              double *res, int *cnt) {
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  ProblemPtr p = build(env, n, m, rowptr, colidx, val, rlo, rhi, vtype, vlb, vub, obj, objc, 0);
  BranchAndBound *bab = new BranchAndBound(env, p);
  HandlerVector handlers;
  IntVarHandlerPtr v_hand = (IntVarHandlerPtr) new IntVarHandler(env, p);
  LinearHandlerPtr l_hand = hip_fbbt ? (LinearHandlerPtr) new HipLinearHandler(env, p, device)
                                     : (LinearHandlerPtr) new LinearHandler(env, p);
  handlers.push_back(v_hand);
  handlers.push_back(l_hand);
  v_hand->setModFlags(false, true);
  l_hand->setModFlags(false, true);
  HipLPEngine *e = new HipLPEngine(env, device);
  PCBProcessorPtr nproc = (PCBProcessorPtr) new PCBProcessor(env, e, handlers);
  ReliabilityBrancherPtr br = (ReliabilityBrancherPtr) new ReliabilityBrancher(env, handlers);
  br->setEngine(e);
  nproc->setBrancher(br);
  bab->setNodeProcessor(nproc);
  NodeIncRelaxerPtr nr = (NodeIncRelaxerPtr) new NodeIncRelaxer(env, handlers);
  bab->setNodeRelaxer(nr);
  nr->setEngine(e);
  nr->setModFlag(false);
  p->setNativeDer();
  bab->shouldCreateRoot(true);
  bab->setLogLevel(LogNone);
  bab->solve();
  res[0] = bab->getUb();
  res[1] = bab->getLb();
  cnt[0] = (int)bab->getTreeManager()->getSize();
  std::vector<double> lps(6, 0.0);
  e->fillStats(lps);
  cnt[1] = (int)lps[0];
  cnt[2] = hip_fbbt ? (int)((HipLinearHandler *)l_hand)->gpuCalls() : 0;
  delete v_hand;
  delete l_hand;
  delete e;
  delete p;
  delete nproc;
  delete nr;
  delete bab;
  delete env;
  return 0;
}

}  // extern "C"
