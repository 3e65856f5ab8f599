//
// HipLinearHandler — see HipLinearHandler.h.
//
#include "HipLinearHandler.h"

#include <cmath>
#include <iostream>

#include "Constraint.h"
#include "Environment.h"
#include "Function.h"
#include "LinearFunction.h"
#include "Logger.h"
#include "Objective.h"
#include "Relaxation.h"
#include "SolutionPool.h"
#include "Timer.h"
#include "VarBoundMod.h"
#include "Variable.h"
#include "mgpu.h"

using namespace Minotaur;

HipLinearHandler::HipLinearHandler(EnvPtr env, ProblemPtr problem, int device)
    : LinearHandler(env, problem),
      ctx_(0),
      device_(device),
      loadedRel_(0),
      loadedCons_(0),
      loadedVars_(0),
      gpuCalls_(0) {
  if (mgpu_create(device_, &ctx_) != MGPU_OK) ctx_ = 0;
}

HipLinearHandler::~HipLinearHandler() {
  if (ctx_) mgpu_destroy(ctx_);
}

std::string HipLinearHandler::getName() const {
  return "HipLinearHandler (linear constraints, node FBBT on MI355X)";
}

// Rows the reference's varBndsFromCons_ can tighten (LinearHandler.cpp:
// 510-513, 966-968): linear, no quadratic / nonlinear part, not deleted.
void HipLinearHandler::loadRel_(RelaxationPtr rel) {
  const int n = (int)rel->getNumVars();
  std::vector<int32_t> rowptr(1, 0), colidx, ctype(n);
  std::vector<double> val, rlo, rhi, clo(n), chi(n), obj(n, 0.0);
  rowmap_.clear();
  int ci = 0;
  for (ConstraintConstIterator it = rel->consBegin(); it != rel->consEnd(); ++it, ++ci) {
    ConstraintPtr c = *it;
    if (c->getFunctionType() != Linear || c->getQuadraticFunction() != 0 ||
        c->getNonlinearFunction() != 0 || c->getState() == DeletedCons ||
        rel->isMarkedDel(c))
      continue;
    LinearFunctionPtr lf = c->getLinearFunction();
    for (VariableGroupConstIterator t = lf->termsBegin(); t != lf->termsEnd(); ++t) {
      colidx.push_back((int32_t)t->first->getIndex());
      val.push_back(t->second);
    }
    rowptr.push_back((int32_t)colidx.size());
    rlo.push_back(c->getLb());
    rhi.push_back(c->getUb());
    rowmap_.push_back(ci);
  }
  int j = 0;
  for (VariableConstIterator v = rel->varsBegin(); v != rel->varsEnd(); ++v, ++j) {
    clo[j] = (*v)->getLb();
    chi[j] = (*v)->getUb();
    ctype[j] = (int32_t)(*v)->getType();
  }
  double objoff = 0.0;
  ObjectivePtr o = rel->getObjective();
  if (o) {
    objoff = o->getConstant();
    LinearFunctionPtr lf = o->getLinearFunction();
    if (lf && o->getFunctionType() == Linear)
      for (VariableGroupConstIterator t = lf->termsBegin(); t != lf->termsEnd(); ++t)
        obj[t->first->getIndex()] = t->second;
  }
  const int m = (int)rowmap_.size();
  mgpu_load_lp(ctx_, n, m, rowptr.data(), colidx.empty() ? 0 : colidx.data(),
               val.empty() ? 0 : val.data(), rlo.data(), rhi.data(), clo.data(), chi.data(),
               ctype.data(), obj.data(), objoff);
  loadedRel_ = rel;
  loadedCons_ = rel->getNumCons();
  loadedVars_ = rel->getNumVars();
}

bool HipLinearHandler::presolveNode(RelaxationPtr rel, NodePtr, SolutionPoolPtr spool,
                                    ModVector &p_mods, ModVector &r_mods) {
  Timer *timer = env_->getNewTimer();
  timer->start();
  if (!ctx_) {
    logger_->errStream() << "HipLinearHandler: no HIP device" << std::endl;
    delete timer;
    return false;
  }
  // rows, objective or constants may have changed (cuts, McCormick rows)
  loadRel_(rel);
  const int n = (int)rel->getNumVars();
  lb_.resize(n);
  ub_.resize(n);
  olb_.resize(n);
  oub_.resize(n);
  int j = 0;
  for (VariableConstIterator v = rel->varsBegin(); v != rel->varsEnd(); ++v, ++j) {
    lb_[j] = (*v)->getLb();
    ub_[j] = (*v)->getUb();
  }
  // LinearHandler.cpp:1636-1640: incumbent only if the pool has one
  double inc = INFINITY;
  if (spool && spool->getNumSols() > 0) inc = spool->getBestSolutionValue();
  int cap = 4 * n + 64;
  int32_t infeas = 0, nmods = 0;
  for (;;) {
    mvar_.resize(cap);
    mlu_.resize(cap);
    mval_.resize(cap);
    mgpu_fbbt(ctx_, 1, lb_.data(), ub_.data(), inc, olb_.data(), oub_.data(), &infeas,
              &nmods, cap, mvar_.data(), mlu_.data(), mval_.data());
    if (nmods <= cap) break;
    cap = nmods + 16;  // log was truncated: run again with room for all
  }
  ++gpuCalls_;
  // replay the reference's VarBoundMods in push order
  for (int k = 0; k < nmods; ++k) {
    VarBoundModPtr mod = (VarBoundModPtr) new VarBoundMod(
        rel->getVariable(mvar_[k]), mlu_[k] == 0 ? Lower : Upper, mval_[k]);
    mod->applyToProblem(rel);
    r_mods.push_back(mod);
  }
  pStats_->nMods += nmods;
  if (true == modProb_) copyBndsFromRel_(rel, p_mods);
  pStats_->timeN += timer->query();
  delete timer;
  return infeas != 0;
}
