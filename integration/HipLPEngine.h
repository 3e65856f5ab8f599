//
// HipLPEngine — Minotaur LPEngine backed by the MI355X engine (include/mgpu.h).
//
// Drop-in for OsiLPEngine (src/interfaces/OsiLPEngine.{h,cpp}) behind the
// unchanged src/base plugin surface: Engine (src/base/Engine.h:34-188) and
// LPEngine (src/base/LPEngine.h:29-74).  Drivers obtain it from
// EngineFactory::getLPEngine when the option lp_engine is "HipLP"
// (INTEGRATION.md shows the 3-line factory patch).  One engine = one
// mgpu context = one host thread (as OsiLPEngine, QGPar.cpp:712-715).
//
// This file is written against the reference headers and is compiled only
// where /root/reference exists (oracle/Makefile target `integ`); it is the
// binding a Minotaur maintainer adds, not part of the standalone engine.
//
#ifndef MINOTAURHIPLPENGINE_H
#define MINOTAURHIPLPENGINE_H

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "LPEngine.h"
#include "LPTableau.h"
#include "WarmStart.h"

struct mgpu_ctx;

namespace Minotaur {

class Environment;
class Problem;
class Solution;
class Timer;
typedef Environment *EnvPtr;
typedef Problem *ProblemPtr;
typedef Solution *SolutionPtr;

// Statistics kept like OsiLPStats (OsiLPEngine.h:35-42).
struct HipLPStats {
  UInt calls;
  UInt strCalls;
  double time;
  double strTime;
  UInt iters;
  UInt strIters;
};

// The engine's mgpu context.  Shared by the engine and every device warm
// start it handed out, so a tree node's warm start outliving the engine still
// frees its slot into a live context.
struct HipLPCtx {
  mgpu_ctx *ctx = nullptr;
  ~HipLPCtx();
};

// One device warm-start slot (mgpu_ws_alloc) of an n x m problem; freed when
// the last warm start holding it dies.
struct HipLPSlot {
  std::shared_ptr<HipLPCtx> owner;
  int id = -1, n = 0, m = 0;
  ~HipLPSlot();
};

// Warm start = the engine's basis: basic column per row, column status,
// reduced costs and the dense basis inverse (column-major).  The reference
// keeps Clp's CoinWarmStartBasis (OsiLPEngine.cpp:375-384, 500-505).  Here
// the basis normally lives in a device slot (dev), written by the solve that
// produced it and read by the next solve that starts from it; copies share
// the slot (it is never written again).  The host vectors are filled only
// when a host edit needs them (fetch), or hold a basis not yet uploaded.
class HipLPWarmStart : public WarmStart {
 public:
  HipLPWarmStart() {}
  ~HipLPWarmStart() {}
  bool hasInfo() { return dev != nullptr || !head.empty(); }
  void write(std::ostream &out) const;
  bool fetch();  // host vectors from the device slot (if empty); false if none

  std::vector<int32_t> head;
  std::vector<int8_t> st;
  std::vector<double> d;
  std::vector<double> binv;
  std::shared_ptr<HipLPSlot> dev;
};
typedef HipLPWarmStart *HipLPWarmStartPtr;

class HipLPEngine : public LPEngine {
 public:
  explicit HipLPEngine(EnvPtr env, int device = 0);
  ~HipLPEngine();

  // Engine interface (Engine.h:44-159)
  void addConstraint(ConstraintPtr con);
  void changeBound(ConstraintPtr cons, BoundType lu, double new_val);
  void changeBound(VariablePtr var, BoundType lu, double new_val);
  void changeBound(VariablePtr var, double new_lb, double new_ub);
  void changeConstraint(ConstraintPtr c, LinearFunctionPtr lf, double lb, double ub);
  void changeConstraint(ConstraintPtr c, NonlinearFunctionPtr nlf);
  void changeObj(FunctionPtr f, double cb);
  void clear();
  void disableStrBrSetup();
  EnginePtr emptyCopy();
  void enableStrBrSetup();
  ConstSolutionPtr getSolution();
  double getSolutionValue();
  EngineStatus solve();
  std::string getName() const;
  EngineStatus getStatus();
  ConstWarmStartPtr getWarmStart();
  WarmStartPtr getWarmStartCopy();
  void load(ProblemPtr problem);
  void loadFromWarmStart(const WarmStartPtr ws);
  void negateObj();
  void removeCons(std::vector<ConstraintPtr> &delcons);
  void resetIterationLimit();
  int setDualObjLimit(double) { return 0; }
  void setIterationLimit(int limit);
  void writeStats(std::ostream &out) const;
  void fillStats(std::vector<double> &lpStats);

  /// One record per solve(): the objective's single column and sign when
  /// the objective is +-x_j (the bound LPs of QuadHandler::tightenLP_),
  /// else col = -1; the status and objective value returned.
  struct SolveRec {
    int col;
    double sign;
    int status;
    double value;
    int iters;
  };
  const std::vector<SolveRec> &solveLog() const { return log_; }

  // LPEngine extras (LPEngine.h:39-73), answered as OsiLPEngine answers them
  // from Clp (OsiLPEngine.cpp:314-360; conventions in LPTableau.h).  The
  // arrays are borrowed views into the engine's host mirrors, valid until the
  // next edit or solve.  enableFactorization refactors the optimal basis of
  // the last solve (K3R on the device, mgpu_lp_refactor, for m <= 64; else
  // the same Gauss-Jordan on the host); getBasics / getBInvARow then read
  // that factorization (SimplexQuadCutGen.cpp:285-345, 366-418, 593-629).
  void enableFactorization();
  void disableFactorization();
  bool IsOptimalBasisAvailable();
  void getBasics(int *index);
  void getBInvARow(int row, double *z, double *slack);
  int getNumCols() { return n_; }
  int getNumRows() { return m_; }
  const double *getColLower();
  const double *getColUpper();
  const double *getRowLower();
  const double *getRowUpper();
  const double *getRightHandSide();
  const double *getRowActivity();
  const double *getOriginalTableau();
  const int *getRowStarts();
  const int *getIndicesofVars();
  const int *getRowLength();
  int getIterationCount() { return lastIters_; }
  /// where the last enableFactorization factored the basis: 1 device (K3R),
  /// 0 host, -1 no optimal basis
  int factorSite() const { return tabSite_; }
  /// solves that refactored the kept basis (rows edited since the basis was
  /// made) and solves that started from the slack basis
  long long refactors() const { return nRefactor_; }
  long long coldSolves() const { return nCold_; }

 private:
  void syncRows_();            // re-read every row of problem_ (after edits)
  void refactor_();            // host Gauss-Jordan of the kept basis
  void recomputeDuals_();      // d = c - A'y, y = c_B B^-1
  int upload_();
  std::shared_ptr<HipLPSlot> newSlot_();  // a free device slot for this problem
  int devWs_();                // slot id of ws_ in this context (uploads a host basis)

  EnvPtr env_;
  ProblemPtr problem_;
  std::shared_ptr<HipLPCtx> own_;
  mgpu_ctx *ctx_;
  int device_;
  int n_, m_;
  std::vector<int32_t> rowptr_, colidx_, ctype_;
  std::vector<double> val_, rlo_, rhi_, clo_, chi_, obj_;
  bool bndChanged_, consChanged_, objChanged_, needUpload_;
  bool dStale_;  // ws_.d is for an older objective: solve passes d = NULL
  // ws_'s inverse is for rows edited since: refactored before the next solve
  // (the kept basis of a solve that ended neither optimal nor at the
  // iteration limit, as CpuLPEngine keeps it)
  bool binvStale_ = false;
  HipLPWarmStart ws_;
  bool wsValid_;
  SolutionPtr sol_;
  int maxIterLimit_, iterLimit_, lastIters_;
  bool strBr_;
  HipLPStats *stats_;
  Timer *timer_;
  std::vector<double> x_, y_, rc_, rcAll_;
  std::vector<SolveRec> log_;
  bool tableau_();             // factor the optimal basis into tabHead_ / tabBinv_
  void views_();               // Osi views of the mirrors (tab_)
  long long nRefactor_ = 0, nCold_ = 0;
  bool tabOn_;                 // enableFactorization ... disableFactorization
  int tabSite_;
  std::vector<int32_t> tabHead_;
  std::vector<double> tabBinv_;  // column-major
  lptab::Views tab_;
  static const std::string me_;
};
typedef HipLPEngine *HipLPEnginePtr;

}  // namespace Minotaur
#endif
