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
      loaded_(false),
      gpuCalls_(0),
      gpuLoads_(0),
      gpuErrors_(0),
      objoff_(0.0) {
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
// The rows, column types and objective are rebuilt on the host every node
// (cuts and McCormick rewrites change them through the Problem) but uploaded
// (mgpu_load_lp: device CSR, CSC and FBBT records) only when they differ
// from what is loaded.  Column bounds travel with each mgpu_fbbt call.
// Returns false when the engine refused the load.
bool HipLinearHandler::loadRel_(RelaxationPtr rel) {
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
  if (loaded_ && rowptr == rowptr_ && colidx == colidx_ && val == val_ && rlo == rlo_ &&
      rhi == rhi_ && ctype == ctype_ && obj == obj_ && objoff == objoff_)
    return true;
  const int m = (int)rowmap_.size();
  loaded_ = false;
  if (mgpu_load_lp(ctx_, n, m, rowptr.data(), colidx.empty() ? 0 : colidx.data(),
                   val.empty() ? 0 : val.data(), rlo.data(), rhi.data(), clo.data(),
                   chi.data(), ctype.data(), obj.data(), objoff) != MGPU_OK)
    return false;
  ++gpuLoads_;
  loaded_ = true;
  rowptr_.swap(rowptr);
  colidx_.swap(colidx);
  val_.swap(val);
  rlo_.swap(rlo);
  rhi_.swap(rhi);
  ctype_.swap(ctype);
  obj_.swap(obj);
  objoff_ = objoff;
  return true;
}

bool HipLinearHandler::presolveNode(RelaxationPtr rel, NodePtr node, SolutionPoolPtr spool,
                                    ModVector &p_mods, ModVector &r_mods) {
  Timer *timer = env_->getNewTimer();
  timer->start();
  // rows, objective or constants may have changed (cuts, McCormick rows)
  if (!ctx_ || !loadRel_(rel)) {
    ++gpuErrors_;
    logger_->errStream() << "HipLinearHandler: engine "
                         << (ctx_ ? mgpu_last_error(ctx_) : "not created (no HIP device)")
                         << "; node FBBT by the reference LinearHandler" << std::endl;
    delete timer;
    return LinearHandler::presolveNode(rel, node, spool, p_mods, r_mods);
  }
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
    if (mgpu_fbbt(ctx_, 1, lb_.data(), ub_.data(), inc, olb_.data(), oub_.data(), &infeas,
                  &nmods, cap, mvar_.data(), mlu_.data(), mval_.data()) != MGPU_OK) {
      // no mod of a failed call is replayed: the node runs on the host
      ++gpuErrors_;
      loaded_ = false;
      logger_->errStream() << "HipLinearHandler: mgpu_fbbt failed: " << mgpu_last_error(ctx_)
                           << "; node FBBT by the reference LinearHandler" << std::endl;
      delete timer;
      return LinearHandler::presolveNode(rel, node, spool, p_mods, r_mods);
    }
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
