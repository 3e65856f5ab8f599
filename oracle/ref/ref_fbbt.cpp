// TEST INFRASTRUCTURE ONLY — never linked into the product (minotaur_amd/).
//
// Builder-written driver that runs the REFERENCE's own node FBBT
// (Minotaur LinearHandler::presolveNode, src/base/LinearHandler.cpp:1592-1653)
// on problems assembled programmatically through the reference's public
// Problem API (Problem::newVariable / newConstraint / newObjective,
// src/base/Problem.h:333-437).  It is compiled together with the reference's
// src/base sources, where they lie under /root/reference, by oracle/Makefile
// into oracle/_ref/libref_fbbt.so (git-ignored).  No reference source is
// copied into this repository: this file only #includes the headers by path.
//
// Uses:
//   * tests/golden/make_golden.py — generates the committed golden vectors;
//   * bench.py cpu_baseline (kind "reference") when the prebuilt .so is present.

#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>

#include "Environment.h"
#include "Function.h"
#include "LinearFunction.h"
#include "LinearHandler.h"
#include "Modification.h"
#include "Objective.h"
#include "Problem.h"
#include "Relaxation.h"
#include "SolutionPool.h"
#include "VarBoundMod.h"
#include "Variable.h"

using namespace Minotaur;

namespace {

struct RefProblem {
  EnvPtr env;
  ProblemPtr p;
  RelaxationPtr rel;
  LinearHandler *lh;
  SolutionPoolPtr spool;
};

// vtype uses the reference's VariableType numerics (Types.h:83-89):
// 0 Binary, 1 Integer, 2 ImplBin, 3 ImplInt, 4 Continuous.
RefProblem *build(int n, int m, const int *rowptr, const int *colidx,
                  const double *val, const double *rlo, const double *rhi,
                  const int *vtype, const double *vlb, const double *vub,
                  int nobj, const int *objidx, const double *objval,
                  double objconst)
{
  RefProblem *r = new RefProblem();
  r->env = (EnvPtr) new Environment();
  int err = 0;
  r->env->startTimer(err);  // as the solvers do (e.g. src/solvers/Glob.cpp)
  r->p = (ProblemPtr) new Problem(r->env);
  std::vector<VariablePtr> vars;
  for (int j = 0; j < n; ++j) {
    vars.push_back(r->p->newVariable(vlb[j], vub[j], (VariableType) vtype[j]));
  }
  for (int i = 0; i < m; ++i) {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      lf->addTerm(vars[colidx[k]], val[k]);
    }
    FunctionPtr f = (FunctionPtr) new Function(lf);
    r->p->newConstraint(f, rlo[i], rhi[i]);
  }
  {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    for (int k = 0; k < nobj; ++k) {
      lf->addTerm(vars[objidx[k]], objval[k]);
    }
    FunctionPtr f = (FunctionPtr) new Function(lf);
    r->p->newObjective(f, objconst, Minimize);
  }
  r->p->calculateSize();
  r->rel = (RelaxationPtr) new Relaxation(r->p, r->env);
  r->rel->calculateSize();
  r->lh = new LinearHandler(r->env, r->p);
  r->lh->setModFlags(false, true);
  r->spool = (SolutionPoolPtr) new SolutionPool(r->env, r->p, 1);
  return r;
}

}  // namespace

extern "C" {

// Runs LinearHandler::presolveNode once per node box.
//   node_lb/node_ub: [B][n] input boxes; out_lb/out_ub: [B][n] tightened boxes.
//   infeas[b]: return value of presolveNode (1 = node found infeasible).
//   nmods[b]: number of VarBoundMods pushed into r_mods.
//   mod_var/mod_lu/mod_val: [B][mod_cap] mod log in push order (may be NULL).
//   has_inc/inc: when has_inc, a solution with objective value `inc` is put
//   in the pool (so varBndsFromObj_ runs, LinearHandler.cpp:1636-1640).
//   *seconds: wall time spent inside presolveNode (sum over nodes).
int ref_linear_fbbt(int n, int m, const int *rowptr, const int *colidx,
                    const double *val, const double *rlo, const double *rhi,
                    const int *vtype, const double *vlb, const double *vub,
                    int nobj, const int *objidx, const double *objval,
                    double objconst, int has_inc, double inc, int B,
                    const double *node_lb, const double *node_ub,
                    double *out_lb, double *out_ub, int *infeas, int *nmods,
                    int mod_cap, int *mod_var, int *mod_lu, double *mod_val,
                    double *seconds)
{
  RefProblem *r = build(n, m, rowptr, colidx, val, rlo, rhi, vtype, vlb, vub,
                        nobj, objidx, objval, objconst);
  if (has_inc) {
    std::vector<double> x(n, 0.0);
    r->spool->addSolution(x.data(), inc);
  }
  double total = 0.0;
  for (int b = 0; b < B; ++b) {
    for (int j = 0; j < n; ++j) {
      r->rel->changeBound(r->rel->getVariable(j), node_lb[(size_t)b * n + j],
                          node_ub[(size_t)b * n + j]);
    }
    ModVector p_mods, r_mods;
    auto t0 = std::chrono::steady_clock::now();
    bool inf = r->lh->presolveNode(r->rel, NodePtr(), r->spool, p_mods, r_mods);
    auto t1 = std::chrono::steady_clock::now();
    total += std::chrono::duration<double>(t1 - t0).count();
    infeas[b] = inf ? 1 : 0;
    nmods[b] = (int) r_mods.size();
    int k = 0;
    for (ModificationPtr mod : r_mods) {
      VarBoundModPtr vm = dynamic_cast<VarBoundModPtr>(mod);
      if (mod_var && k < mod_cap && vm) {
        mod_var[(size_t)b * mod_cap + k] = (int) vm->getVar()->getIndex();
        mod_lu[(size_t)b * mod_cap + k] = (int) vm->getLU();
        mod_val[(size_t)b * mod_cap + k] = vm->getNewVal();
      }
      ++k;
      delete mod;
    }
    for (int j = 0; j < n; ++j) {
      VariablePtr v = r->rel->getVariable(j);
      out_lb[(size_t)b * n + j] = v->getLb();
      out_ub[(size_t)b * n + j] = v->getUb();
    }
  }
  if (seconds) {
    *seconds = total;
  }
  delete r->lh;
  delete r->spool;
  delete r->rel;
  delete r->p;
  delete r->env;
  delete r;
  return 0;
}

}  // extern "C"
