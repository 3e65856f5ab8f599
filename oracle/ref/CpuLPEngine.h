//
// CpuLPEngine -- the tree-level CPU baseline (TEST / BENCH INFRASTRUCTURE,
// not the product): Minotaur's LPEngine (src/base/LPEngine.h:29-74) over this
// repo's C restatement of the bounded dual simplex (oracle/lp_dual.c, the
// dense explicit-inverse arithmetic K3 runs), one LP at a time on one core.
// It behaves call for call as integration/HipLPEngine (which mirrors
// OsiLPEngine, src/interfaces/OsiLPEngine.cpp): the basis of the last optimal
// solve is kept, a new objective rebuilds the reduced costs of that basis,
// edited rows re-invert it.  Driven by integ_bnb_tree(device < 0, ...) for
// bench.py's cpu_baseline of the tree_search entries: the reference's own
// BranchAndBound + LinearHandler on the CPU, timed at 1 core.
//
#ifndef MINOTAURCPULPENGINE_H
#define MINOTAURCPULPENGINE_H

#include <cstdint>
#include <string>
#include <vector>

#include "LPEngine.h"
#include "LPTableau.h"
#include "WarmStart.h"

namespace Minotaur {

class Environment;
class Problem;
class Solution;
class Timer;
typedef Environment *EnvPtr;
typedef Problem *ProblemPtr;
typedef Solution *SolutionPtr;

// Basis of the oracle's dual simplex: basic column per row, column status,
// reduced costs, dense inverse ROW-major (oracle/lp_dual.c layout).
class CpuLPWarmStart : public WarmStart {
 public:
  bool hasInfo() { return !head.empty(); }
  void write(std::ostream &out) const;
  std::vector<int> head;
  std::vector<signed char> st;
  std::vector<double> d, binv;
};

class CpuLPEngine : public LPEngine {
 public:
  explicit CpuLPEngine(EnvPtr env);
  ~CpuLPEngine();

  void addConstraint(ConstraintPtr con);
  void changeBound(ConstraintPtr cons, BoundType lu, double new_val);
  void changeBound(VariablePtr var, BoundType lu, double new_val);
  void changeBound(VariablePtr var, double new_lb, double new_ub);
  void changeConstraint(ConstraintPtr c, LinearFunctionPtr lf, double lb, double ub);
  void changeConstraint(ConstraintPtr c, NonlinearFunctionPtr nlf);
  void changeObj(FunctionPtr f, double cb);
  void clear();
  void disableStrBrSetup() { strBr_ = false; }
  EnginePtr emptyCopy() { return (EnginePtr) new CpuLPEngine(env_); }
  void enableStrBrSetup() { strBr_ = true; }
  ConstSolutionPtr getSolution();
  double getSolutionValue();
  EngineStatus solve();
  std::string getName() const { return "CpuLP"; }
  EngineStatus getStatus() { return status_; }
  ConstWarmStartPtr getWarmStart() { return &ws_; }
  WarmStartPtr getWarmStartCopy();
  void load(ProblemPtr problem);
  void loadFromWarmStart(const WarmStartPtr ws);
  void negateObj() { objChanged_ = true; }
  void removeCons(std::vector<ConstraintPtr> &delcons);
  void resetIterationLimit() { iterLimit_ = 10000; }
  int setDualObjLimit(double) { return 0; }
  void setIterationLimit(int limit) { iterLimit_ = limit; }
  void writeStats(std::ostream &out) const;
  void fillStats(std::vector<double> &lpStats);
  // LPEngine extras (LPEngine.h:39-73) with OsiLPEngine's conventions
  // (integration/LPTableau.h): the host Gauss-Jordan of the optimal basis
  void enableFactorization();
  void disableFactorization();
  bool IsOptimalBasisAvailable() { return status_ == ProvenOptimal && wsValid_; }
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
  struct SolveRec {
    int status;
    double value;
    int iters;
  };
  const std::vector<SolveRec> &solveLog() const { return log_; }
  long long refactors() const { return nRefactor_; }
  long long coldSolves() const { return nCold_; }

 private:
  void syncRows_();  // re-read every row of problem_, rebuild the CSC

  EnvPtr env_;
  ProblemPtr problem_;
  int n_, m_;
  std::vector<int> colptr_, rowidx_;
  std::vector<double> cval_, rlo_, rhi_, clo_, chi_, obj_;
  bool consChanged_, objChanged_;
  bool dStale_;     // ws_.d is for an older objective: rebuilt in the solve
  bool binvStale_;  // rows changed: the kept basis is re-inverted
  CpuLPWarmStart ws_, wk_;
  bool wsValid_;
  SolutionPtr sol_;
  int iterLimit_, lastIters_;
  bool strBr_;
  double calls_, strCalls_, time_, strTime_, iters_, strIters_;
  Timer *timer_;
  std::vector<double> x_, y_, rc_;
  std::vector<int32_t> rowptr_, colidx_;   // the rows as read (row-major)
  std::vector<double> val_;
  bool tableau_();
  void views_();
  long long nRefactor_ = 0, nCold_ = 0;
  std::vector<SolveRec> log_;
  bool tabOn_ = false;
  std::vector<int32_t> tabHead_;
  std::vector<double> tabBinv_;
  lptab::Views tab_;
};

}  // namespace Minotaur
#endif
