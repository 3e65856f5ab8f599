//
// HipQuadHandler — see HipQuadHandler.h.
//
#include "HipQuadHandler.h"

#include <algorithm>
#include <cmath>
#include <iostream>

#include "Constraint.h"
#include "Environment.h"
#include "Function.h"
#include "LinConMod.h"
#include "LinearFunction.h"
#include "Logger.h"
#include "NonlinearFunction.h"
#include "Objective.h"
#include "Option.h"
#include "QuadraticFunction.h"
#include "Relaxation.h"
#include "SolutionPool.h"
#include "VarBoundMod.h"
#include "Variable.h"
#include "mgpu.h"

using namespace Minotaur;

HipQuadHandler::HipQuadHandler(EnvPtr env, ProblemPtr problem, ProblemPtr orig_p, int device)
    : QuadHandler(env, problem, orig_p),
      env2_(env),
      p2_(problem),
      orig2_(orig_p),
      ctx_(0),
      loaded_(false),
      doqt_(false),
      calls_(0),
      gpuCalls_(0),
      cpuCalls_(0) {
  if (mgpu_create(device, &ctx_) != MGPU_OK) ctx_ = 0;
}

HipQuadHandler::~HipQuadHandler() {
  if (ctx_) mgpu_destroy(ctx_);
}

std::string HipQuadHandler::getName() const {
  return "HipQuadHandler (y = x1*x2 terms, node FBBT on MI355X)";
}

// QuadHandler::addConstraint (QuadHandler.cpp:127-179): y is the linear
// term; the product comes from the quadratic or the nonlinear part.  The
// registries are a map keyed by x (first insert wins) and a set ordered by
// (x0, x1) ids with x0 the lower index (LinBil.cpp:26-38).
void HipQuadHandler::addConstraint(ConstraintPtr newcon) {
  QuadHandler::addConstraint(newcon);
  loaded_ = false;
  VariablePtr y = newcon->getLinearFunction()->termsBegin()->first;
  VariablePtr x0, x1;
  QuadraticFunctionPtr qf = newcon->getQuadraticFunction();
  if (qf) {
    x0 = qf->begin()->first.first;
    x1 = qf->begin()->first.second;
    if (x0->getId() == x1->getId()) x1 = x0;
  } else {
    NonlinearFunctionPtr nlf = newcon->getNonlinearFunction();
    VariableSet::iterator it = nlf->varsBegin();
    x0 = *it;
    x1 = x0;
    if (nlf->numVars() > 1) x1 = *(++it);
  }
  if (x0 == x1) {
    for (const Sq &s : sq_)
      if (s.x->getId() == x0->getId()) return;
    sq_.push_back(Sq{x0, y});
    std::sort(sq_.begin(), sq_.end(), [](const Sq &a, const Sq &b) {
      return a.x->getId() < b.x->getId();
    });
  } else {
    if (x0->getIndex() > x1->getIndex()) std::swap(x0, x1);
    for (const Bil &b : bil_)
      if (b.x0->getId() == x0->getId() && b.x1->getId() == x1->getId()) return;
    bil_.push_back(Bil{x0, x1, y});
    std::sort(bil_.begin(), bil_.end(), [](const Bil &a, const Bil &b) {
      if (a.x0->getId() == b.x0->getId()) return a.x1->getId() < b.x1->getId();
      return a.x0->getId() < b.x0->getId();
    });
  }
}

// relax_ appends one secant per square, then 4 McCormick rows per bilinear,
// in registry order (QuadHandler.cpp:1549-1592).
void HipQuadHandler::recordRows_(RelaxationPtr rel, UInt first) {
  rows_.clear();
  for (UInt i = first; i < rel->getNumCons(); ++i) rows_.push_back(rel->getConstraint(i));
}

void HipQuadHandler::relaxInitFull(RelaxationPtr rel, bool *is_inf) {
  const UInt first = rel->getNumCons();
  QuadHandler::relaxInitFull(rel, is_inf);
  recordRows_(rel, first);
}

void HipQuadHandler::relaxInitInc(RelaxationPtr rel, bool *is_inf) {
  const UInt first = rel->getNumCons();
  QuadHandler::relaxInitInc(rel, is_inf);
  recordRows_(rel, first);
}

namespace {
// A function whose tightenQuad_ pass can return true (QuadHandler.cpp:
// 2361-2427): type Quadratic, a linear part, and a square term whose
// variable is also linear.
bool has_univariate(FunctionPtr f) {
  if (!f || f->getType() != Quadratic) return false;
  LinearFunctionPtr lf = f->getLinearFunction();
  QuadraticFunctionPtr qf = f->getQuadraticFunction();
  if (!lf || !qf) return false;
  for (VariablePairGroupConstIterator it = qf->begin(); it != qf->end(); ++it)
    if (it->first.first->getId() == it->first.second->getId() && lf->hasVar(it->first.first))
      return true;
  return false;
}
}  // namespace

// presolve's tightenQuad_(bool*) (QuadHandler.cpp:2429-2682) sets doQT_ when
// one of p_'s functions passes getQfLfBnds_; the same structural test here.
SolveStatus HipQuadHandler::presolve(PreModQ *pre_mods, bool *changed, Solution **sol) {
  SolveStatus st = QuadHandler::presolve(pre_mods, changed, sol);
  ObjectivePtr o = p2_->getObjective();
  const double cut = env2_->getOptions()->findDouble("obj_cut_off")->getValue();
  if (o && cut - o->getConstant() < INFINITY && has_univariate(o->getFunction())) doqt_ = true;
  for (ConstraintConstIterator it = p2_->consBegin(); it != p2_->consEnd(); ++it)
    if (has_univariate((*it)->getFunction())) doqt_ = true;
  return st;
}

bool HipQuadHandler::load_() {
  if (loaded_) return true;
  const int nv = (int)p2_->getNumVars(), nv0 = (int)orig2_->getNumVars();
  std::vector<int32_t> vtype(nv), sx, sy, b0, b1, by, lptr(1, 0), lvar, qptr(1, 0), qv1, qv2;
  std::vector<double> lval, qval, clb, cub;
  for (int j = 0; j < nv; ++j) vtype[j] = (int32_t)p2_->getVariable(j)->getType();
  for (const Sq &s : sq_) {
    sx.push_back((int32_t)s.x->getIndex());
    sy.push_back((int32_t)s.y->getIndex());
  }
  for (const Bil &b : bil_) {
    b0.push_back((int32_t)b.x0->getIndex());
    b1.push_back((int32_t)b.x1->getIndex());
    by.push_back((int32_t)b.y->getIndex());
  }
  auto add_fun = [&](FunctionPtr f) {
    // only Quadratic functions matter to tightenQuad_; others get no terms
    if (f && f->getType() == Quadratic) {
      LinearFunctionPtr lf = f->getLinearFunction();
      QuadraticFunctionPtr qf = f->getQuadraticFunction();
      if (lf)
        for (VariableGroupConstIterator t = lf->termsBegin(); t != lf->termsEnd(); ++t) {
          lvar.push_back((int32_t)t->first->getIndex());
          lval.push_back(t->second);
        }
      if (qf)
        for (VariablePairGroupConstIterator t = qf->begin(); t != qf->end(); ++t) {
          qv1.push_back((int32_t)t->first.first->getIndex());
          qv2.push_back((int32_t)t->first.second->getIndex());
          qval.push_back(t->second);
        }
    }
    lptr.push_back((int32_t)lvar.size());
    qptr.push_back((int32_t)qv1.size());
  };
  for (ConstraintConstIterator it = orig2_->consBegin(); it != orig2_->consEnd(); ++it) {
    add_fun((*it)->getFunction());
    clb.push_back((*it)->getLb());
    cub.push_back((*it)->getUb());
  }
  ObjectivePtr o = orig2_->getObjective();
  const int has_obj = o && o->getFunction() ? 1 : 0;
  if (has_obj) add_fun(o->getFunction());
  const int rc = mgpu_load_quad(
      ctx_, nv0, nv, vtype.data(), (int)sx.size(), sx.data(), sy.data(), (int)b0.size(),
      b0.data(), b1.data(), by.data(), (int)clb.size(), lptr.data(), lvar.data(), lval.data(),
      qptr.data(), qv1.data(), qv2.data(), qval.data(), clb.data(), cub.data(), has_obj,
      o ? o->getConstant() : 0.0);
  if (rc != MGPU_OK) {
    env2_->getLogger()->msgStream(LogInfo) << "HipQuadHandler: engine refused the problem ("
                                << mgpu_last_error(ctx_) << "); node FBBT stays on the CPU"
                                << std::endl;
    return false;
  }
  loaded_ = rows_.size() == sq_.size() + 4 * bil_.size();
  return loaded_;
}

bool HipQuadHandler::presolveNode(RelaxationPtr rel, NodePtr node, SolutionPoolPtr s_pool,
                                  ModVector &p_mods, ModVector &r_mods) {
  ++calls_;
  // The first call (the root) always runs tightenQuad_ (niters <= 1,
  // QuadHandler.cpp:1241) and is left to the base class, whose private call
  // counter then stays correct for any later CPU fallback; GPU calls are
  // never the first, so tightenQuad_ runs on them exactly when doQT_ does.
  const int qt = doqt_ ? 1 : 0;
  const int nv = (int)p2_->getNumVars();
  bool gpu = calls_ > 1 && ctx_ && load_() && (int)rel->getNumVars() == nv;
  std::vector<double> lb(nv), ub(nv);
  for (int j = 0; gpu && j < nv; ++j) {
    VariablePtr pv = p2_->getVariable(j), rv = rel->getVariable(j);
    lb[j] = rv->getLb();
    ub[j] = rv->getUb();
    if (pv->getLb() != lb[j] || pv->getUb() != ub[j]) gpu = false;  // see header
  }
  const int R = (int)(2 * sq_.size() + 12 * bil_.size());
  std::vector<double> rin(R > 0 ? R : 1), rout(R > 0 ? R : 1), olb(nv), oub(nv);
  if (gpu) {
    int o = 0;
    for (size_t k = 0; k < sq_.size(); ++k) {
      ConstraintPtr c = rows_[k];
      rin[o++] = c->getLinearFunction()->getWeight(rel->getVariable(sq_[k].x->getIndex()));
      rin[o++] = c->getUb();
    }
    for (size_t k = 0; k < bil_.size(); ++k)
      for (int t = 0; t < 4; ++t) {
        ConstraintPtr c = rows_[sq_.size() + 4 * k + t];
        LinearFunctionPtr lf = c->getLinearFunction();
        rin[o++] = lf->getWeight(rel->getVariable(bil_[k].x0->getIndex()));
        rin[o++] = lf->getWeight(rel->getVariable(bil_[k].x1->getIndex()));
        rin[o++] = c->getUb();
      }
  }
  const double inc = s_pool ? s_pool->getBestSolutionValue() : INFINITY;
  int cap = 4 * nv + 12 * (int)bil_.size() + 64;
  int32_t st = 0, nmods = 0;
  std::vector<int32_t> kind, idx;
  std::vector<double> v1, v2;
  while (gpu) {
    kind.resize(cap);
    idx.resize(cap);
    v1.resize(cap);
    v2.resize(cap);
    if (mgpu_quad_fbbt(ctx_, 1, lb.data(), ub.data(), inc, qt, rin.data(), 1, olb.data(),
                       oub.data(), rout.data(), &st, &nmods, cap, kind.data(), idx.data(),
                       v1.data(), v2.data()) != MGPU_OK) {
      gpu = false;
      break;
    }
    if (nmods <= cap) break;
    cap = nmods + 16;
  }
  if (!gpu || st >= 2) {  // not representable on the engine: the reference path
    ++cpuCalls_;
    return QuadHandler::presolveNode(rel, node, s_pool, p_mods, r_mods);
  }
  ++gpuCalls_;
  // replay updatePBounds_ / upSqCon_ / upBilCon_ in the reference's order
  for (int k = 0; k < nmods; ++k) {
    if (kind[k] <= 2) {
      VariablePtr pv = p2_->getVariable(idx[k]), rv = rel->getVariable(idx[k]);
      if (kind[k] == 2) {
        VarBoundMod2Ptr m = (VarBoundMod2Ptr) new VarBoundMod2(pv, v1[k], v2[k]);
        m->applyToProblem(p2_);
        p_mods.push_back(m);
        m = (VarBoundMod2Ptr) new VarBoundMod2(rv, v1[k], v2[k]);
        m->applyToProblem(rel);
        r_mods.push_back(m);
      } else {
        const BoundType lu = kind[k] == 0 ? Lower : Upper;
        VarBoundModPtr m = (VarBoundModPtr) new VarBoundMod(pv, lu, v1[k]);
        m->applyToProblem(p2_);
        p_mods.push_back(m);
        m = (VarBoundModPtr) new VarBoundMod(rv, lu, v1[k]);
        m->applyToProblem(rel);
        r_mods.push_back(m);
      }
    } else {
      const int row = idx[k];
      LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
      double rhs;
      if (row < (int)sq_.size()) {
        lf->addTerm(rel->getVariable(sq_[row].y->getIndex()), 1.);
        const double ax = rout[2 * row];
        if (ax != 0.0) lf->addTerm(rel->getVariable(sq_[row].x->getIndex()), ax);
        rhs = rout[2 * row + 1];
      } else {
        const int kb = (row - (int)sq_.size()) / 4, t = (row - (int)sq_.size()) % 4;
        const double *r = &rout[2 * sq_.size() + 12 * kb + 3 * t];
        lf->addTerm(rel->getVariable(bil_[kb].x0->getIndex()), r[0]);
        lf->addTerm(rel->getVariable(bil_[kb].x1->getIndex()), r[1]);
        lf->addTerm(rel->getVariable(bil_[kb].y->getIndex()), t < 2 ? -1. : 1.);
        rhs = r[2];
      }
      LinConModPtr m = (LinConModPtr) new LinConMod(rows_[row], lf, -INFINITY, rhs);
      m->applyToProblem(rel);
      r_mods.push_back(m);
    }
  }
  return st == 1;
}
