//
// CpuLPEngine -- see CpuLPEngine.h (test / bench infrastructure: the CPU
// baseline of the tree search, over oracle/lp_dual.c).
//
#include "CpuLPEngine.h"

#include <cassert>
#include <chrono>
#include <cmath>
#include <cstring>
#include <iostream>

#include "Constraint.h"
#include "Environment.h"
#include "Function.h"
#include "LinearFunction.h"
#include "Logger.h"
#include "Objective.h"
#include "Problem.h"
#include "Solution.h"
#include "Timer.h"
#include "Variable.h"

extern "C" {
#include "../oracle.h"
}

using namespace Minotaur;

void CpuLPWarmStart::write(std::ostream &out) const {
  out << "CpuLPWarmStart: " << head.size() << " basic columns" << std::endl;
}

CpuLPEngine::CpuLPEngine(EnvPtr env)
    : env_(env),
      problem_(0),
      n_(0),
      m_(0),
      consChanged_(true),
      objChanged_(true),
      dStale_(false),
      binvStale_(false),
      wsValid_(false),
      sol_(0),
      iterLimit_(10000),
      lastIters_(0),
      strBr_(false),
      calls_(0),
      strCalls_(0),
      time_(0),
      strTime_(0),
      iters_(0),
      strIters_(0) {
  logger_ = env_->getLogger();
  timer_ = env_->getNewTimer();
  status_ = EngineUnknownStatus;
}

CpuLPEngine::~CpuLPEngine() {
  delete timer_;
  if (problem_) {
    problem_->unsetEngine();
    problem_ = 0;
  }
  delete sol_;
}

// CSR from the problem's rows in the order HipLPEngine reads them, then the
// CSC the oracle takes (rows ascending inside a column, as mgpu_load_lp).
void CpuLPEngine::syncRows_() {
  n_ = (int)problem_->getNumVars();
  m_ = (int)problem_->getNumCons();
  std::vector<int32_t> &rowptr = rowptr_, &colidx = colidx_;
  std::vector<double> &val = val_;
  rowptr.assign(1, 0);
  colidx.clear();
  val.clear();
  rlo_.resize(m_);
  rhi_.resize(m_);
  int i = 0;
  for (ConstraintConstIterator it = problem_->consBegin(); it != problem_->consEnd();
       ++it, ++i) {
    rlo_[i] = (*it)->getLb();
    rhi_[i] = (*it)->getUb();
    LinearFunctionPtr lf = (*it)->getLinearFunction();
    if (lf)
      for (VariableGroupConstIterator t = lf->termsBegin(); t != lf->termsEnd(); ++t) {
        colidx.push_back((int)t->first->getIndex());
        val.push_back(t->second);
      }
    rowptr.push_back((int)colidx.size());
  }
  colptr_.assign(n_ + 1, 0);
  for (int c : colidx) ++colptr_[c + 1];
  for (int j = 0; j < n_; ++j) colptr_[j + 1] += colptr_[j];
  rowidx_.assign(colidx.size(), 0);
  cval_.assign(colidx.size(), 0.0);
  std::vector<int> fill(colptr_.begin(), colptr_.end() - 1);
  for (int r = 0; r < m_; ++r)
    for (int k = rowptr[r]; k < rowptr[r + 1]; ++k) {
      const int p = fill[colidx[k]]++;
      rowidx_[p] = r;
      cval_[p] = val[k];
    }
  clo_.resize(n_);
  chi_.resize(n_);
  int j = 0;
  for (VariableConstIterator v = problem_->varsBegin(); v != problem_->varsEnd(); ++v, ++j) {
    clo_[j] = (*v)->getLb();
    chi_[j] = (*v)->getUb();
  }
}

void CpuLPEngine::load(ProblemPtr problem) {
  problem_ = problem;
  syncRows_();
  double sense = 1.0;
  LinearFunctionPtr lin = 0;
  if (problem->getObjective()) {
    lin = problem->getObjective()->getLinearFunction();
    if (problem->getObjective()->getObjectiveType() == Maximize) sense = -1.0;
  }
  obj_.assign(n_, 0.0);
  if (lin) {
    int j = 0;
    for (VariableConstIterator v = problem->varsBegin(); v != problem->varsEnd(); ++v, ++j)
      obj_[j] = sense * lin->getWeight(*v);
  }
  delete sol_;
  sol_ = new Solution(1E20, 0, problem_);
  wsValid_ = false;
  consChanged_ = objChanged_ = false;
  dStale_ = binvStale_ = false;
  problem->setEngine(this);
}

EngineStatus CpuLPEngine::solve() {
  double off = 0;
  if (problem_->getObjective()) off = problem_->getObjective()->getConstant();
  const auto t0 = std::chrono::steady_clock::now();
  calls_ += 1;
  if (consChanged_) {
    syncRows_();
    if (wsValid_) binvStale_ = true;
  }
  if (objChanged_ && wsValid_) dStale_ = true;
  const int n = n_, m = m_, N = n_ + m_;
  orc_lp P;
  P.n = n;
  P.m = m;
  P.colptr = colptr_.data();
  P.rowidx = rowidx_.empty() ? 0 : rowidx_.data();
  P.cval = cval_.empty() ? 0 : cval_.data();
  P.c = obj_.data();
  P.rlo = rlo_.data();
  P.rhi = rhi_.data();
  if (wsValid_ && ((int)ws_.head.size() != m || (int)ws_.st.size() != N)) wsValid_ = false;
  wk_ = wsValid_ ? ws_ : CpuLPWarmStart();
  wk_.head.resize(m);
  wk_.st.resize(N);
  wk_.d.resize(N);
  wk_.binv.resize((size_t)m * m);
  // have_binv: 1 inverse and reduced costs given, 2 inverse given and the
  // reduced costs rebuilt for this objective, 0 re-invert the basis
  const int have_binv = !wsValid_ ? 0 : binvStale_ ? 0 : dStale_ ? 2 : 1;
  if (!wsValid_) ++nCold_;
  else if (binvStale_) ++nRefactor_;
  x_.assign(n, 0.0);
  y_.assign(m, 0.0);
  double obj = 0.0;
  int it = 0;
  const int st = orc_dual_simplex(&P, clo_.data(), chi_.data(), wk_.head.data(), wk_.st.data(),
                                  wk_.binv.data(), wk_.d.data(), wsValid_ ? 1 : 0, have_binv,
                                  iterLimit_, &obj, x_.data(), y_.data(), &it);
  status_ = (EngineStatus)st;
  if (status_ == ProvenOptimal || status_ == EngineIterationLimit) {
    ws_ = wk_;
    wsValid_ = true;
    dStale_ = binvStale_ = false;
    rc_.assign(n, 0.0);
    for (int j = 0; j < n; ++j) rc_[j] = ws_.st[j] == 3 ? 0.0 : ws_.d[j];
    sol_->setPrimal(x_.data());
    sol_->setObjValue(obj + off);
    sol_->setDualOfCons(y_.data());
    sol_->setDualOfVars(rc_.data());
  } else if (status_ == ProvenInfeasible) {
    sol_->setObjValue(INFINITY);
  } else if (status_ == ProvenUnbounded) {
    sol_->setObjValue(-INFINITY);
  } else {
    sol_->setObjValue(INFINITY);
  }
  lastIters_ = it;
  log_.push_back({(int)status_, sol_->getObjValue(), it});
  iters_ += it;
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  time_ += dt;
  if (strBr_) {
    strCalls_ += 1;
    strIters_ += it;
    strTime_ += dt;
  }
  consChanged_ = objChanged_ = false;
  return status_;
}

void CpuLPEngine::addConstraint(ConstraintPtr) {
  if (wsValid_) {  // the new row's logical joins the basis; re-inverted
    const int N = n_ + m_;
    ws_.head.push_back(N);
    ws_.st.push_back(3);
    ws_.d.push_back(0.0);
  }
  consChanged_ = true;
}

void CpuLPEngine::removeCons(std::vector<ConstraintPtr> &delcons) {
  if (wsValid_) {  // basis kept only if every removed row's logical is basic
    std::vector<char> del(m_, 0);
    for (ConstraintPtr c : delcons) del[c->getIndex()] = 1;
    std::vector<int> newidx(m_, -1), head;
    std::vector<signed char> st;
    int nm = 0;
    for (int i = 0; i < m_; ++i)
      if (!del[i]) newidx[i] = nm++;
    for (int i = 0; i < m_; ++i) {
      const int h = ws_.head[i];
      if (h >= n_ && del[h - n_]) continue;
      head.push_back(h >= n_ ? n_ + newidx[h - n_] : h);
    }
    for (int j = 0; j < n_; ++j) st.push_back(ws_.st[j]);
    for (int i = 0; i < m_; ++i)
      if (!del[i]) st.push_back(ws_.st[n_ + i]);
    if ((int)head.size() == nm) {
      ws_.head = head;
      ws_.st = st;
    } else {
      wsValid_ = false;
    }
  }
  consChanged_ = true;
}

void CpuLPEngine::changeBound(ConstraintPtr cons, BoundType lu, double new_val) {
  if (Upper == lu) rhi_[cons->getIndex()] = new_val;
  else rlo_[cons->getIndex()] = new_val;
}

void CpuLPEngine::changeBound(VariablePtr var, BoundType lu, double new_val) {
  if (lu == Lower) clo_[var->getIndex()] = new_val;
  else if (lu == Upper) chi_[var->getIndex()] = new_val;
}

void CpuLPEngine::changeBound(VariablePtr var, double new_lb, double new_ub) {
  clo_[var->getIndex()] = new_lb;
  chi_[var->getIndex()] = new_ub;
}

void CpuLPEngine::changeConstraint(ConstraintPtr, LinearFunctionPtr, double, double) {
  consChanged_ = true;
}

void CpuLPEngine::changeConstraint(ConstraintPtr, NonlinearFunctionPtr) {
  assert(!"Cannot change a nonlinear function in CpuLPEngine");
}

void CpuLPEngine::changeObj(FunctionPtr f, double) {
  LinearFunctionPtr lf = (f) ? f->getLinearFunction() : 0;
  std::fill(obj_.begin(), obj_.end(), 0.0);
  if (lf)
    for (VariableGroupConstIterator it = lf->termsBegin(); it != lf->termsEnd(); ++it)
      obj_[it->first->getIndex()] = it->second;
  objChanged_ = true;
}

void CpuLPEngine::clear() {
  wsValid_ = false;
  if (problem_) {
    problem_->unsetEngine();
    problem_ = 0;
  }
}

ConstSolutionPtr CpuLPEngine::getSolution() { return sol_; }
double CpuLPEngine::getSolutionValue() { return sol_->getObjValue(); }

WarmStartPtr CpuLPEngine::getWarmStartCopy() {
  CpuLPWarmStart *w = new CpuLPWarmStart();
  if (wsValid_) *w = ws_;
  return w;
}

void CpuLPEngine::loadFromWarmStart(const WarmStartPtr ws) {
  const CpuLPWarmStart *w = dynamic_cast<const CpuLPWarmStart *>(ws);
  if (w && (int)w->head.size() == m_ && (int)w->st.size() == n_ + m_) {
    ws_ = *w;
    wsValid_ = true;
  }
}

void CpuLPEngine::getBasics(int *index) {
  const std::vector<int> &h = tabOn_ ? tabHead_ : ws_.head;
  for (int i = 0; i < m_ && (tabOn_ || wsValid_); ++i) index[i] = h[i];
}

bool CpuLPEngine::tableau_() {
  tabHead_.clear();
  tabBinv_.clear();
  if (consChanged_) syncRows_();
  if (!IsOptimalBasisAvailable() || (int)ws_.head.size() != m_) return false;
  tabHead_.assign(ws_.head.begin(), ws_.head.end());
  if (!lptab::invert(n_, m_, rowptr_.data(), colidx_.data(), val_.data(), tabHead_.data(),
                     tabBinv_)) {
    tabHead_.clear();
    return false;
  }
  return true;
}

void CpuLPEngine::enableFactorization() { tabOn_ = tableau_(); }

void CpuLPEngine::disableFactorization() {
  tabOn_ = false;
  tabHead_.clear();
  tabBinv_.clear();
}

void CpuLPEngine::getBInvARow(int row, double *z, double *slack) {
  if (!tabOn_ && !(tabOn_ = tableau_())) return;
  if (row < 0 || row >= m_) return;
  lptab::binv_a_row(n_, m_, rowptr_.data(), colidx_.data(), val_.data(), tabHead_.data(),
                    tabBinv_.data(), row, z, slack);
}

void CpuLPEngine::views_() {
  if (consChanged_) syncRows_();
  tab_.fill(n_, m_, rowptr_.data(), colidx_.data(), val_.data(), clo_.data(), chi_.data(),
            rlo_.data(), rhi_.data(), (int)x_.size() == n_ ? x_.data() : nullptr);
}

const double *CpuLPEngine::getColLower() { views_(); return tab_.clo.data(); }
const double *CpuLPEngine::getColUpper() { views_(); return tab_.chi.data(); }
const double *CpuLPEngine::getRowLower() { views_(); return tab_.rlo.data(); }
const double *CpuLPEngine::getRowUpper() { views_(); return tab_.rhi.data(); }
const double *CpuLPEngine::getRightHandSide() { views_(); return tab_.rhs.data(); }
const double *CpuLPEngine::getRowActivity() { views_(); return tab_.act.data(); }
const double *CpuLPEngine::getOriginalTableau() {
  if (consChanged_) syncRows_();
  return val_.data();
}
const int *CpuLPEngine::getRowStarts() {
  if (consChanged_) syncRows_();
  return rowptr_.data();
}
const int *CpuLPEngine::getIndicesofVars() {
  if (consChanged_) syncRows_();
  return colidx_.data();
}
const int *CpuLPEngine::getRowLength() { views_(); return tab_.rowlen.data(); }

void CpuLPEngine::fillStats(std::vector<double> &s) {
  if (s.size() >= 6) {
    s[0] += calls_;
    s[1] += strCalls_;
    s[2] += time_;
    s[3] += strTime_;
    s[4] += iters_;
    s[5] += strIters_;
  }
}

void CpuLPEngine::writeStats(std::ostream &out) const {
  out << "CpuLP: calls = " << calls_ << ", iterations = " << iters_ << ", time = " << time_
      << std::endl;
}
