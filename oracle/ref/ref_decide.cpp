// TEST INFRASTRUCTURE ONLY — never linked into the product (minotaur_amd/).
//
// Builder-written driver that runs the REFERENCE's own node decision on
// given relaxation results:
//   * PCBProcessor::shouldPrune_ (src/base/PCBProcessor.cpp:400-523): the
//     EngineStatus switch, the incumbent / cutoff tests with solAbs_tol /
//     solRel_tol / obj_cut_off (Environment.cpp:509-528 defaults);
//   * IntVarHandler::isFeasible (src/base/IntVarHandler.cpp:54-84) for the
//     nodes shouldPrune_ keeps: is_feas and inf_meas.
// shouldPrune_ is a private member, so this file (and only this file) makes
// the reference's private members visible with the preprocessor before
// including PCBProcessor.h; no reference code is changed or copied.
// Compiled with the reference's src/base into oracle/_ref/libref_fbbt.so
// (git-ignored) by oracle/Makefile.
//
// Used by tests/golden/make_golden_decide.py (golden vectors for
// minotaur_amd/csrc/node_decide.hip).

#include <cmath>
#include <vector>

#include "Environment.h"
#include "Function.h"
#include "IntVarHandler.h"
#include "LinearFunction.h"
#include "Node.h"
#include "Objective.h"
#include "Problem.h"
#include "Relaxation.h"
#include "Solution.h"
#include "SolutionPool.h"
#include "Variable.h"
#define private public
#include "PCBProcessor.h"
#undef private

using namespace Minotaur;

extern "C" {

// vtype: reference VariableType numerics (Types.h:83-89).
// status[b]: EngineStatus numerics (Types.h:152-166); obj[b]: solution
// value; x[b*n..]: primal point.  has_inc/inc: incumbent put in the pool.
// Outputs per node: prune[b] (shouldPrune_'s return), nstat[b] (NodeStatus
// after shouldPrune_), feas[b] (isFeasible, only when not pruned; else -1),
// inf_meas[b] (isFeasible's inf_meas; 0 when not evaluated).
int ref_node_decide(int n, const int *vtype, int B, const int *status, const double *obj,
                    const double *x, int has_inc, double inc, int *prune, int *nstat,
                    int *feas, double *inf_meas)
{
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  ProblemPtr p = (ProblemPtr) new Problem(env);
  for (int j = 0; j < n; ++j) {
    const double lo = vtype[j] == Binary ? 0.0 : -1e6;
    const double hi = vtype[j] == Binary ? 1.0 : 1e6;
    p->newVariable(lo, hi, (VariableType) vtype[j]);
  }
  // Relaxation(p, env) copies the objective: give it an empty linear one
  p->newObjective((FunctionPtr) new Function((LinearFunctionPtr) new LinearFunction()), 0.0,
                  Minimize);
  p->calculateSize();
  RelaxationPtr rel = (RelaxationPtr) new Relaxation(p, env);
  rel->calculateSize();
  SolutionPoolPtr spool = (SolutionPoolPtr) new SolutionPool(env, p, 1);
  if (has_inc) {
    std::vector<double> x0(n, 0.0);
    spool->addSolution(x0.data(), inc);
  }
  HandlerVector hv;
  PCBProcessor *proc = new PCBProcessor(env, EnginePtr(), hv);
  proc->setBrancher(0);
  IntVarHandler ivh(env, p);
  for (int b = 0; b < B; ++b) {
    NodePtr node = (NodePtr) new Node();
    proc->engineStatus_ = (EngineStatus) status[b];
    const bool pr = proc->shouldPrune_(node, obj[b], spool);
    prune[b] = pr ? 1 : 0;
    nstat[b] = (int) node->getStatus();
    feas[b] = -1;
    inf_meas[b] = 0.0;
    if (!pr) {
      SolutionPtr sol = (SolutionPtr) new Solution(obj[b], x + (size_t) b * n, rel);
      bool should_prune = false;
      double meas = 0.0;
      feas[b] = ivh.isFeasible(sol, rel, should_prune, meas) ? 1 : 0;
      inf_meas[b] = meas;
      delete sol;
    }
    delete node;
  }
  delete proc;
  delete spool;
  delete rel;
  delete p;
  delete env;
  return 0;
}

}  // extern "C"
