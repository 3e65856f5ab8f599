//
// HipLPEngine — see HipLPEngine.h.  Mirrors OsiLPEngine's behaviour
// (src/interfaces/OsiLPEngine.cpp) call by call:
//   load            :390-498  row-major CSR, bounds, objective (x -1 when
//                             maximising), problem->setEngine(this)
//   edits           :152-262  set dirty flags; rows re-read lazily
//   solve           :571-652  resolve from the kept basis; status map;
//                             solution value + objective constant
//   warm start      :375-384, :500-505
//   iteration limit :561-569  (default 10000, ctor :95-137)
//
#include "HipLPEngine.h"

#include <cassert>
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
#include "mgpu.h"

using namespace Minotaur;

const std::string HipLPEngine::me_ = "HipLPEngine: ";

void HipLPWarmStart::write(std::ostream &out) const {
  out << "HipLPWarmStart: " << (dev ? dev->m : (int)head.size()) << " basic columns"
      << (dev ? " (device)" : "") << std::endl;
}

HipLPCtx::~HipLPCtx() {
  if (ctx) mgpu_destroy(ctx);
}

HipLPSlot::~HipLPSlot() {
  if (owner && owner->ctx && id >= 0) mgpu_ws_free(owner->ctx, id);
}

bool HipLPWarmStart::fetch() {
  if (!head.empty()) return true;
  if (!dev || !dev->owner || !dev->owner->ctx) return false;
  const int n = dev->n, m = dev->m;
  head.resize(m);
  st.resize(n + m);
  d.resize(n + m);
  binv.resize((size_t)m * m);
  if (mgpu_ws_read(dev->owner->ctx, dev->id, head.data(), st.data(), d.data(), binv.data()) !=
      MGPU_OK) {
    head.clear();
    return false;
  }
  return true;
}

HipLPEngine::HipLPEngine(EnvPtr env, int device)
    : env_(env),
      problem_(0),
      ctx_(0),
      device_(device),
      n_(0),
      m_(0),
      bndChanged_(true),
      consChanged_(true),
      objChanged_(true),
      needUpload_(true),
      dStale_(false),
      wsValid_(false),
      sol_(0),
      maxIterLimit_(10000),
      iterLimit_(10000),
      lastIters_(0),
      strBr_(false),
      tabOn_(false),
      tabSite_(-1) {
  logger_ = env_->getLogger();
  stats_ = new HipLPStats();
  std::memset(stats_, 0, sizeof(HipLPStats));
  timer_ = env_->getNewTimer();
  status_ = EngineUnknownStatus;
  own_ = std::make_shared<HipLPCtx>();
  if (mgpu_create(device_, &own_->ctx) != MGPU_OK) {
    own_->ctx = 0;
    logger_->errStream() << me_ << "no HIP device " << device_ << std::endl;
  }
  ctx_ = own_->ctx;
}

HipLPEngine::~HipLPEngine() {
  ws_ = HipLPWarmStart();
  own_.reset();  // the context goes with the last warm start still holding a slot
  delete stats_;
  delete timer_;
  if (problem_) {
    problem_->unsetEngine();
    problem_ = 0;
  }
  delete sol_;
}

void HipLPEngine::syncRows_() {
  n_ = (int)problem_->getNumVars();
  m_ = (int)problem_->getNumCons();
  rowptr_.assign(1, 0);
  colidx_.clear();
  val_.clear();
  rlo_.resize(m_);
  rhi_.resize(m_);
  int i = 0;
  for (ConstraintConstIterator it = problem_->consBegin(); it != problem_->consEnd();
       ++it, ++i) {
    assert((*it)->getFunctionType() == Linear);  // as OsiLPEngine.cpp:420
    rlo_[i] = (*it)->getLb();
    rhi_[i] = (*it)->getUb();
    LinearFunctionPtr lf = (*it)->getLinearFunction();
    if (lf) {
      for (VariableGroupConstIterator t = lf->termsBegin(); t != lf->termsEnd(); ++t) {
        colidx_.push_back((int32_t)t->first->getIndex());
        val_.push_back(t->second);
      }
    }
    rowptr_.push_back((int32_t)colidx_.size());
  }
  clo_.resize(n_);
  chi_.resize(n_);
  ctype_.resize(n_);
  int j = 0;
  for (VariableConstIterator v = problem_->varsBegin(); v != problem_->varsEnd(); ++v, ++j) {
    clo_[j] = (*v)->getLb();
    chi_[j] = (*v)->getUb();
    ctype_[j] = (int32_t)(*v)->getType();
  }
}

void HipLPEngine::load(ProblemPtr problem) {
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
  binvStale_ = false;
  ws_ = HipLPWarmStart();
  objChanged_ = bndChanged_ = consChanged_ = needUpload_ = true;
  problem->setEngine(this);
}

int HipLPEngine::upload_() {
  if (!ctx_) return MGPU_ERR_STATE;
  // the objective constant is added at solve time, as OsiLPEngine does
  return mgpu_load_lp(ctx_, n_, m_, rowptr_.data(), colidx_.empty() ? 0 : colidx_.data(),
                      val_.empty() ? 0 : val_.data(), rlo_.data(), rhi_.data(), clo_.data(),
                      chi_.data(), ctype_.data(), obj_.data(), 0.0);
}

// Inverse of the kept basis after the matrix changed (rows edited / added /
// removed), as Clp refactors it after OsiLPEngine::changeConstraint: on the
// device (mgpu_lp_refactor, K3R: Gauss-Jordan with partial pivoting plus the
// reduced costs) for m <= 64, else the same Gauss-Jordan on the host.  A
// singular basis is dropped for the slack basis.
void HipLPEngine::refactor_() {
  const int m = m_, n = n_;
  ws_.fetch();
  ws_.dev.reset();  // the host vectors are edited below
  if ((int)ws_.head.size() != m) {
    wsValid_ = false;
    return;
  }
  {
    HipLPWarmStart out;
    out.head.resize(m);
    out.st.resize(n + m);
    out.d.resize(n + m);
    out.binv.resize((size_t)m * m);
    int sing = 0;
    if (mgpu_lp_refactor(ctx_, ws_.head.data(), ws_.st.data(), out.head.data(), out.st.data(),
                         out.d.data(), out.binv.data(), &sing) == MGPU_OK) {
      if (sing) {
        wsValid_ = false;
      } else {
        ws_ = out;
      }
      return;
    }
  }
  if (!lptab::invert(n, m, rowptr_.data(), colidx_.data(), val_.data(), ws_.head.data(),
                     ws_.binv)) {
    wsValid_ = false;
    return;
  }
  recomputeDuals_();
}

void HipLPEngine::recomputeDuals_() {
  dStale_ = false;
  const int m = m_, n = n_, N = n_ + m_;
  std::vector<double> y(m, 0.0);
  for (int i = 0; i < m; ++i) {
    const int h = ws_.head[i];
    const double cb = h < n ? obj_[h] : 0.0;
    if (cb != 0.0)
      for (int k = 0; k < m; ++k) y[k] += cb * ws_.binv[(size_t)k * m + i];
  }
  ws_.d.assign(N, 0.0);
  std::vector<double> aty(n, 0.0);
  for (int r = 0; r < m; ++r)
    for (int k = rowptr_[r]; k < rowptr_[r + 1]; ++k) aty[colidx_[k]] += val_[k] * y[r];
  for (int j = 0; j < N; ++j) {
    if (ws_.st[j] == 3) continue;
    ws_.d[j] = j < n ? obj_[j] - aty[j] : y[j - n];
  }
}

EngineStatus HipLPEngine::solve() {
  double off = 0;
  if (problem_->getObjective()) off = problem_->getObjective()->getConstant();
  timer_->start();
  stats_->calls += 1;
  // the kept basis is refactored for edited rows into a working basis; a
  // solve that ends neither optimal nor at the iteration limit keeps the
  // basis it started from, its inverse marked stale (CpuLPEngine's wk_)
  const bool refactor = wsValid_ && (consChanged_ || binvStale_);
  HipLPWarmStart kept;
  if (refactor) kept = ws_;
  if (needUpload_ || consChanged_ || objChanged_) {
    if (consChanged_) syncRows_();
    if (upload_() != MGPU_OK) {
      status_ = EngineError;
      sol_->setObjValue(INFINITY);
      timer_->stop();
      return status_;
    }
    needUpload_ = false;
    // new objective, same basis: the kernel rebuilds the reduced costs (d = NULL)
    if (!refactor && wsValid_ && objChanged_) dStale_ = true;
  }
  if (refactor) {
    refactor_();
    ++nRefactor_;
  }
  // current column bounds (edits since the last solve); the LP starts from
  // the kept basis in its device slot and leaves its basis in a fresh slot
  const int n = n_, m = m_, N = n_ + m_;
  int32_t st = 0, it = 0;
  double obj = 0.0;
  x_.resize(n);
  rcAll_.resize(N);
  int in = -1;
  if (!wsValid_) ++nCold_;
  if (wsValid_) {
    in = devWs_();
    if (in < 0) wsValid_ = false;
  }
  std::shared_ptr<HipLPSlot> out = newSlot_();
  int rc = out ? mgpu_lp_solve1(ctx_, clo_.data(), chi_.data(), in, dStale_ ? 0 : 1, out->id,
                                iterLimit_, &st, &obj, &it, x_.data(), rcAll_.data())
               : MGPU_ERR_NOMEM;
  if (rc != MGPU_OK) {
    logger_->errStream() << me_ << (ctx_ ? mgpu_last_error(ctx_) : "no context") << std::endl;
    status_ = EngineError;
    sol_->setObjValue(INFINITY);
  } else {
    status_ = (EngineStatus)st;
    if (status_ == ProvenOptimal || status_ == EngineIterationLimit) {
      ws_ = HipLPWarmStart();
      ws_.dev = out;
      wsValid_ = true;
      dStale_ = binvStale_ = false;
      // duals from the final basis, computed in the kernel: reduced costs of
      // the structurals, and of the logicals (d_{n+r} = y_r for the row -e_r)
      rc_.assign(rcAll_.begin(), rcAll_.begin() + n);
      y_.assign(rcAll_.begin() + n, rcAll_.end());
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
  }
  if (refactor && !(rc == MGPU_OK && (status_ == ProvenOptimal || status_ == EngineIterationLimit))) {
    ws_ = kept;
    wsValid_ = true;
    binvStale_ = true;
  }
  {
    SolveRec r{-1, 0.0, (int)status_, sol_->getObjValue(), it};
    int nz = 0;
    for (int j = 0; j < n; ++j)
      if (obj_[j] != 0.0) {
        ++nz;
        r.col = j;
        r.sign = obj_[j];
      }
    if (nz != 1) r.col = -1;
    log_.push_back(r);
  }
  lastIters_ = it;
  stats_->iters += it;
  stats_->time += timer_->query();
  if (strBr_) {
    ++(stats_->strCalls);
    stats_->strIters += it;
    stats_->strTime += timer_->query();
  }
  timer_->stop();
  bndChanged_ = consChanged_ = objChanged_ = false;
  return status_;
}

void HipLPEngine::addConstraint(ConstraintPtr) {
  // the new row's logical joins the basis (refactor_ on the next solve)
  if (wsValid_ && !ws_.fetch()) wsValid_ = false;
  ws_.dev.reset();
  if (wsValid_) {
    const int N = n_ + m_;
    ws_.head.push_back(N);
    ws_.st.push_back(3);
    ws_.d.push_back(0.0);
  }
  consChanged_ = true;
}

void HipLPEngine::removeCons(std::vector<ConstraintPtr> &delcons) {
  // basis kept only if every removed row's logical is basic
  if (wsValid_ && !ws_.fetch()) wsValid_ = false;
  ws_.dev.reset();
  if (wsValid_) {
    std::vector<char> del(m_, 0);
    for (ConstraintPtr c : delcons) del[c->getIndex()] = 1;
    std::vector<int32_t> head;
    std::vector<int8_t> st;
    std::vector<int> newidx(m_, -1);
    int nm = 0;
    for (int i = 0; i < m_; ++i)
      if (!del[i]) newidx[i] = nm++;
    bool ok = true;
    for (int i = 0; i < m_; ++i) {
      const int h = ws_.head[i];
      if (h >= n_ && del[h - n_]) continue;
      if (h >= n_) head.push_back(n_ + newidx[h - n_]);
      else head.push_back(h);
    }
    if ((int)head.size() != nm) ok = false;
    for (int j = 0; j < n_; ++j) st.push_back(ws_.st[j]);
    for (int i = 0; i < m_; ++i)
      if (!del[i]) st.push_back(ws_.st[n_ + i]);
    if (ok) {
      ws_.head = head;
      ws_.st = st;
    } else {
      wsValid_ = false;
    }
  }
  consChanged_ = true;
}

void HipLPEngine::changeBound(ConstraintPtr cons, BoundType lu, double new_val) {
  if (Upper == lu) rhi_[cons->getIndex()] = new_val;
  else rlo_[cons->getIndex()] = new_val;
  needUpload_ = true;
  bndChanged_ = true;
}

void HipLPEngine::changeBound(VariablePtr var, BoundType lu, double new_val) {
  const int col = var->getIndex();
  if (lu == Lower) clo_[col] = new_val;
  else if (lu == Upper) chi_[col] = new_val;
  bndChanged_ = true;
}

void HipLPEngine::changeBound(VariablePtr var, double new_lb, double new_ub) {
  const int col = var->getIndex();
  clo_[col] = new_lb;
  chi_[col] = new_ub;
  bndChanged_ = true;
}

void HipLPEngine::changeConstraint(ConstraintPtr, LinearFunctionPtr, double, double) {
  // rows are re-read from problem_ on the next solve (the Problem applies
  // the edit before forwarding it, Problem.cpp:273-291)
  consChanged_ = true;
}

void HipLPEngine::changeConstraint(ConstraintPtr, NonlinearFunctionPtr) {
  assert(!"Cannot change a nonlinear function in HipLPEngine");
}

void HipLPEngine::changeObj(FunctionPtr f, double) {
  LinearFunctionPtr lf = (f) ? f->getLinearFunction() : 0;
  std::fill(obj_.begin(), obj_.end(), 0.0);
  if (lf)
    for (VariableGroupConstIterator it = lf->termsBegin(); it != lf->termsEnd(); ++it)
      obj_[it->first->getIndex()] = it->second;
  objChanged_ = true;
}

void HipLPEngine::negateObj() {
  // OsiLPEngine::negateObj copies the coefficients without negating them
  // (OsiLPEngine.cpp:514-522); kept as is.
  objChanged_ = true;
}

void HipLPEngine::clear() {
  wsValid_ = false;
  ws_ = HipLPWarmStart();
  needUpload_ = true;
  if (problem_) {
    problem_->unsetEngine();
    problem_ = 0;
  }
}

void HipLPEngine::disableStrBrSetup() { strBr_ = false; }
void HipLPEngine::enableStrBrSetup() { strBr_ = true; }

EnginePtr HipLPEngine::emptyCopy() { return (EnginePtr) new HipLPEngine(env_, device_); }

ConstSolutionPtr HipLPEngine::getSolution() { return sol_; }
double HipLPEngine::getSolutionValue() { return sol_->getObjValue(); }
std::string HipLPEngine::getName() const { return "HipLP"; }
EngineStatus HipLPEngine::getStatus() { return status_; }

ConstWarmStartPtr HipLPEngine::getWarmStart() { return &ws_; }

WarmStartPtr HipLPEngine::getWarmStartCopy() {
  HipLPWarmStartPtr w = new HipLPWarmStart();
  if (wsValid_) *w = ws_;
  return w;
}

void HipLPEngine::loadFromWarmStart(const WarmStartPtr ws) {
  HipLPWarmStart *w = dynamic_cast<HipLPWarmStart *>(ws);
  assert(w);
  if (!w) return;
  if (w->dev && w->dev->owner == own_ && w->dev->n == n_ && w->dev->m == m_) {
    ws_ = *w;  // shares the device slot: no device work
    wsValid_ = true;
    return;
  }
  // another engine's warm start (testOsiWarmStart): through the host
  HipLPWarmStart h = *w;
  if (!h.fetch()) return;
  h.dev.reset();
  if ((int)h.head.size() == m_ && (int)h.st.size() == n_ + m_) {
    ws_ = h;
    wsValid_ = true;
  }
}

std::shared_ptr<HipLPSlot> HipLPEngine::newSlot_() {
  int id = -1;
  if (!ctx_ || mgpu_ws_alloc(ctx_, &id) != MGPU_OK) return nullptr;
  std::shared_ptr<HipLPSlot> s = std::make_shared<HipLPSlot>();
  s->owner = own_;
  s->id = id;
  s->n = n_;
  s->m = m_;
  return s;
}

int HipLPEngine::devWs_() {
  if (ws_.dev && ws_.dev->owner == own_ && ws_.dev->n == n_ && ws_.dev->m == m_)
    return ws_.dev->id;
  if (!ws_.fetch() || (int)ws_.head.size() != m_ || (int)ws_.st.size() != n_ + m_ ||
      ws_.binv.size() != (size_t)m_ * m_)
    return -1;
  std::shared_ptr<HipLPSlot> s = newSlot_();
  if (!s ||
      mgpu_ws_write(ctx_, s->id, ws_.head.data(), ws_.st.data(),
                    (int)ws_.d.size() == n_ + m_ ? ws_.d.data() : 0, ws_.binv.data()) != MGPU_OK)
    return -1;
  ws_.dev = s;
  return s->id;
}

void HipLPEngine::getBasics(int *index) {
  if (tabOn_ && (int)tabHead_.size() == m_) {
    for (int i = 0; i < m_; ++i) index[i] = tabHead_[i];
    return;
  }
  if (wsValid_ && !ws_.fetch()) return;
  for (int i = 0; i < m_ && wsValid_; ++i) index[i] = ws_.head[i];
}

bool HipLPEngine::IsOptimalBasisAvailable() { return status_ == ProvenOptimal && wsValid_; }

// The optimal basis of the last solve, refactored from scratch (as Clp's
// factorization is fresh after an optimal resolve): the device's K3R when the
// loaded matrix is the current one, else the host Gauss-Jordan.
bool HipLPEngine::tableau_() {
  tabHead_.clear();
  tabBinv_.clear();
  tabSite_ = -1;
  if (consChanged_) syncRows_();
  if (!IsOptimalBasisAvailable() || !ws_.fetch() || (int)ws_.head.size() != m_) return false;
  const int n = n_, m = m_;
  if (ctx_ && !consChanged_ && !needUpload_ && m > 0 && m <= 64) {
    std::vector<int32_t> h((size_t)m);
    std::vector<int8_t> st((size_t)(n + m));
    std::vector<double> d((size_t)(n + m)), b((size_t)m * m);
    int sing = 1;
    if (mgpu_lp_refactor(ctx_, ws_.head.data(), ws_.st.data(), h.data(), st.data(), d.data(),
                         b.data(), &sing) == MGPU_OK &&
        !sing) {
      tabHead_ = h;
      tabBinv_ = b;
      tabSite_ = 1;
      return true;
    }
  }
  tabHead_ = ws_.head;
  if (!lptab::invert(n, m, rowptr_.data(), colidx_.data(), val_.data(), tabHead_.data(),
                     tabBinv_)) {
    tabHead_.clear();
    return false;
  }
  tabSite_ = 0;
  return true;
}

void HipLPEngine::enableFactorization() { tabOn_ = tableau_(); }

void HipLPEngine::disableFactorization() {
  tabOn_ = false;
  tabHead_.clear();
  tabBinv_.clear();
}

void HipLPEngine::getBInvARow(int row, double *z, double *slack) {
  if (!tabOn_ && !(tabOn_ = tableau_())) return;
  if (row < 0 || row >= m_) return;
  lptab::binv_a_row(n_, m_, rowptr_.data(), colidx_.data(), val_.data(), tabHead_.data(),
                    tabBinv_.data(), row, z, slack);
}

void HipLPEngine::views_() {
  if (consChanged_) syncRows_();
  tab_.fill(n_, m_, rowptr_.data(), colidx_.data(), val_.data(), clo_.data(), chi_.data(),
            rlo_.data(), rhi_.data(), (int)x_.size() == n_ ? x_.data() : nullptr);
}

const double *HipLPEngine::getColLower() { views_(); return tab_.clo.data(); }
const double *HipLPEngine::getColUpper() { views_(); return tab_.chi.data(); }
const double *HipLPEngine::getRowLower() { views_(); return tab_.rlo.data(); }
const double *HipLPEngine::getRowUpper() { views_(); return tab_.rhi.data(); }
const double *HipLPEngine::getRightHandSide() { views_(); return tab_.rhs.data(); }
const double *HipLPEngine::getRowActivity() { views_(); return tab_.act.data(); }
const double *HipLPEngine::getOriginalTableau() {
  if (consChanged_) syncRows_();
  return val_.data();
}
const int *HipLPEngine::getRowStarts() {
  if (consChanged_) syncRows_();
  return rowptr_.data();
}
const int *HipLPEngine::getIndicesofVars() {
  if (consChanged_) syncRows_();
  return colidx_.data();
}
const int *HipLPEngine::getRowLength() { views_(); return tab_.rowlen.data(); }

void HipLPEngine::resetIterationLimit() { iterLimit_ = maxIterLimit_; }
void HipLPEngine::setIterationLimit(int limit) { iterLimit_ = limit; }

void HipLPEngine::fillStats(std::vector<double> &lpStats) {
  if (lpStats.size()) {
    lpStats[0] += stats_->calls;
    lpStats[1] += stats_->strCalls;
    lpStats[2] += stats_->time;
    lpStats[3] += stats_->strTime;
    lpStats[4] += stats_->iters;
    lpStats[5] += stats_->strIters;
  }
}

void HipLPEngine::writeStats(std::ostream &out) const {
  std::string me = "HipLP: ";
  out << me << "total calls            = " << stats_->calls << std::endl
      << me << "strong branching calls = " << stats_->strCalls << std::endl
      << me << "total time in solving  = " << stats_->time << std::endl
      << me << "time in str branching  = " << stats_->strTime << std::endl
      << me << "total iterations       = " << stats_->iters << std::endl
      << me << "strong br iterations   = " << stats_->strIters << std::endl;
}
