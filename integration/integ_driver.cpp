// TEST INFRASTRUCTURE ONLY — drives the reference's own solver stack
// (BranchAndBound, PCBProcessor, NodeIncRelaxer, ReliabilityBrancher,
// IntVarHandler, LinearHandler; compiled from /root/reference/src/base) with
// the MI355X engine plugged in through the unchanged plugin surface:
// HipLPEngine as the LPEngine, HipLinearHandler as the linear handler.
// Mirrors the reference's own tests src/testing/AMPLOsiUT.cpp:46-170
// (testOsiLP, testOsiLP2, testOsiWarmStart, testOsiBnB), with the instances
// built programmatically from src/testing/instances/*.mod (ASL is absent).
#include <chrono>
#include <cstring>
#include <cmath>
#include <vector>

#include "BranchAndBound.h"
#include "TreeManager.h"
#include "Environment.h"
#include "Function.h"
#include "CpuLPEngine.h"
#include "HipLPEngine.h"
#include "HipLinearHandler.h"
#include "HipQuadHandler.h"
#include "LinConMod.h"
#include "QuadHandler.h"
#include "QuadraticFunction.h"
#include "Relaxation.h"
#include "SolutionPool.h"
#include "VarBoundMod.h"
#include "IntVarHandler.h"
#include "LinearFunction.h"
#include "LinearHandler.h"
#include "MaxVioBrancher.h"
#include "NodeIncRelaxer.h"
#include "Objective.h"
#include "Option.h"
#include "PCBProcessor.h"
#include "Problem.h"
#include "ReliabilityBrancher.h"
#include "SimplexQuadCutGen.h"
#include "BrVarCand.h"
#include "Branch.h"
#include "Serializer.h"
#include "StrongBrancher.h"
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

// the main HipLPEngine of the last integ_glob_tree3: solves that refactored
// the kept basis, solves from the slack basis (integ_last_engine_stats)
static long long g_last_engine[2] = {0, 0};

int integ_last_engine_stats(long long *out) {
  out[0] = g_last_engine[0];
  out[1] = g_last_engine[1];
  return 0;
}

// the main engine's solves in order (status, value incl. constant, pivots)
// of the last integ_glob_tree3; returns their count (at most cap written)
struct LogRec {
  int status;
  double value;
  int iters;
};
static std::vector<LogRec> g_last_log;

int integ_last_solve_log(int cap, int *status, double *value, int *iters) {
  for (size_t k = 0; k < g_last_log.size() && (int)k < cap; ++k) {
    status[k] = g_last_log[k].status;
    value[k] = g_last_log[k].value;
    iters[k] = g_last_log[k].iters;
  }
  return (int)g_last_log.size();
}

// HipLPEngine::fillStats of the engine of the last integ_bnb / integ_bnb_tree
// run: calls, strong-branching calls, seconds in solve, strong-branching
// seconds, pivots, strong-branching pivots (integ_last_lp_stats).
static std::vector<double> g_last_lp_stats(6, 0.0);

int integ_last_lp_stats(double *out) {
  for (int k = 0; k < 6; ++k) out[k] = g_last_lp_stats[k];
  return 0;
}

// AMPLOsiUT::testOsiBnB generalised: the reference BranchAndBound with
// IntVarHandler + (reference LinearHandler | HipLinearHandler), PCBProcessor,
// ReliabilityBrancher and NodeIncRelaxer, all on a HipLPEngine.
// res[0] = UB, res[1] = LB, res[2] = wall seconds in BranchAndBound::solve;
// cnt[0] = nodes processed, cnt[1] = LP solves, cnt[2] = GPU FBBT calls,
// cnt[3] = relaxation uploads by HipLinearHandler, cnt[4] = its engine errors.
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
  const auto t0 = std::chrono::steady_clock::now();
  bab->solve();
  res[2] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  res[0] = bab->getUb();
  res[1] = bab->getLb();
  cnt[0] = (int)bab->getTreeManager()->getSize();
  std::vector<double> lps(6, 0.0);
  e->fillStats(lps);
  cnt[1] = (int)lps[0];
  g_last_lp_stats = lps;
  cnt[2] = hip_fbbt ? (int)((HipLinearHandler *)l_hand)->gpuCalls() : 0;
  cnt[3] = hip_fbbt ? (int)((HipLinearHandler *)l_hand)->gpuLoads() : 0;
  cnt[4] = hip_fbbt ? (int)((HipLinearHandler *)l_hand)->gpuErrors() : 0;
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

// BranchAndBound keeps its node count in a protected member.
class ProbeBranchAndBound : public BranchAndBound {
 public:
  ProbeBranchAndBound(EnvPtr env, ProblemPtr p) : BranchAndBound(env, p) {}
  long long nodesProcessed() const { return stats_ ? (long long)stats_->nodesProc : 0; }
};

// The reference's own tree search with the MI355X engine plugged in, set up
// for a node-for-node comparison with the batched tree at batch 1:
// tree_search "bfs" (TreeManager's NodeHeap), pres_freq 1 (LinearHandler::
// presolveNode at every node, PCBProcessor.cpp:143), brancher 0 MaxVio / 1
// reliability, guided_dive as given (reference default on).  Every other
// option keeps its default.  HipLPEngine solves the LPs; the linear handler
// is the reference's LinearHandler (hip_fbbt 0) or HipLinearHandler.
// res[0] UB, res[1] LB, res[2] seconds; cnt[0] nodes processed, cnt[1]
// nodes created, cnt[2] LP solves (strong branching included), cnt[3]
// strong-branching LPs, cnt[4] LP iterations, cnt[5] strong-branching
// iterations.
static int bnb_tree(int device, int hip_fbbt, int brancher, int guided, int n, int m,
                    const int *rowptr, const int *colidx, const double *val, const double *rlo,
                    const double *rhi, const int *vtype, const double *vlb, const double *vub,
                    const double *obj, double objc, double *res, long long *cnt,
                    double time_limit) {
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  env->getOptions()->findString("tree_search")->setValue("bfs");
  env->getOptions()->findInt("pres_freq")->setValue(1);
  env->getOptions()->findBool("guided_dive")->setValue(guided != 0);
  // (BabOptions reads the option in the BranchAndBound constructor)
  if (time_limit > 0) env->getOptions()->findDouble("time_limit")->setValue(time_limit);
  ProblemPtr p = build(env, n, m, rowptr, colidx, val, rlo, rhi, vtype, vlb, vub, obj, objc, 0);
  ProbeBranchAndBound *bab = new ProbeBranchAndBound(env, p);
  HandlerVector handlers;
  IntVarHandlerPtr v_hand = (IntVarHandlerPtr) new IntVarHandler(env, p);
  const bool cpu = device < 0;  // the tree-level CPU baseline: CpuLPEngine + LinearHandler
  LinearHandlerPtr l_hand = hip_fbbt && !cpu
                                ? (LinearHandlerPtr) new HipLinearHandler(env, p, device)
                                : (LinearHandlerPtr) new LinearHandler(env, p);
  handlers.push_back(v_hand);
  handlers.push_back(l_hand);
  v_hand->setModFlags(false, true);
  l_hand->setModFlags(false, true);
  LPEnginePtr e = cpu ? (LPEnginePtr) new CpuLPEngine(env)
                      : (LPEnginePtr) new HipLPEngine(env, device);
  PCBProcessorPtr nproc = (PCBProcessorPtr) new PCBProcessor(env, e, handlers);
  BrancherPtr br;
  if (brancher == 1) {
    ReliabilityBrancherPtr rb = (ReliabilityBrancherPtr) new ReliabilityBrancher(env, handlers);
    rb->setEngine(e);
    br = rb;
  } else {
    br = (BrancherPtr) new MaxVioBrancher(env, handlers);
  }
  nproc->setBrancher(br);
  bab->setNodeProcessor(nproc);
  NodeIncRelaxerPtr nr = (NodeIncRelaxerPtr) new NodeIncRelaxer(env, handlers);
  bab->setNodeRelaxer(nr);
  nr->setEngine(e);
  nr->setModFlag(false);
  p->setNativeDer();
  bab->shouldCreateRoot(true);
  bab->setLogLevel(LogNone);
  const auto t0 = std::chrono::steady_clock::now();
  bab->solve();
  res[2] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  res[0] = bab->getUb();
  res[1] = bab->getLb();
  cnt[0] = bab->nodesProcessed();
  cnt[1] = (long long)bab->getTreeManager()->getSize();
  std::vector<double> lps(6, 0.0);
  e->fillStats(lps);
  cnt[2] = (long long)lps[0];
  cnt[3] = (long long)lps[1];
  cnt[4] = (long long)lps[4];
  cnt[5] = (long long)lps[5];
  g_last_lp_stats = lps;
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

int integ_bnb_tree(int device, int hip_fbbt, int brancher, int guided, int n, int m,
                   const int *rowptr, const int *colidx, const double *val, const double *rlo,
                   const double *rhi, const int *vtype, const double *vlb, const double *vub,
                   const double *obj, double objc, double *res, long long *cnt) {
  if (device < 0) return -1;
  return bnb_tree(device, hip_fbbt, brancher, guided, n, m, rowptr, colidx, val, rlo, rhi,
                  vtype, vlb, vub, obj, objc, res, cnt, 0.0);
}

// The same tree search on the CPU at one core -- CpuLPEngine (the C
// restatement of the dual simplex) + the reference's LinearHandler -- for
// bench.py's tree-level cpu_baseline; time_limit > 0 bounds it (the
// reference's "time_limit" option, BranchAndBound.cpp:582), res / cnt as
// integ_bnb_tree (res[2] = seconds actually spent).
int integ_bnb_tree_cpu(int brancher, int guided, int n, int m, const int *rowptr,
                       const int *colidx, const double *val, const double *rlo,
                       const double *rhi, const int *vtype, const double *vlb, const double *vub,
                       const double *obj, double objc, double time_limit, double *res,
                       long long *cnt) {
  return bnb_tree(-1, 0, brancher, guided, n, m, rowptr, colidx, val, rlo, rhi, vtype, vlb, vub,
                  obj, objc, res, cnt, time_limit);
}

// ---- quadratic handler: reference QuadHandler vs HipQuadHandler ----------
// Same layout as oracle/ref/ref_quad.cpp's QSpec (oracle.qspec builds it).
struct QSpecI {
  int nv0, nv;
  const int *vtype;
  const double *vlb, *vub;
  int nsq;
  const int *sq_x, *sq_y;
  int nbil;
  const int *bil_x0, *bil_x1, *bil_y;
  int ncon;
  const int *lptr, *lvar;
  const double *lval;
  const int *qptr, *qv1, *qv2;
  const double *qval;
  const double *clb, *cub;
  int has_obj;
  double obj_const;
};

static FunctionPtr qfun(const QSpecI &s, ProblemPtr prob, int c) {
  LinearFunctionPtr lf = LinearFunctionPtr();
  QuadraticFunctionPtr qf = QuadraticFunctionPtr();
  if (s.lptr[c + 1] > s.lptr[c]) {
    lf = (LinearFunctionPtr) new LinearFunction();
    for (int k = s.lptr[c]; k < s.lptr[c + 1]; ++k) lf->addTerm(prob->getVariable(s.lvar[k]), s.lval[k]);
  }
  if (s.qptr[c + 1] > s.qptr[c]) {
    qf = (QuadraticFunctionPtr) new QuadraticFunction();
    for (int k = s.qptr[c]; k < s.qptr[c + 1]; ++k)
      qf->addTerm(prob->getVariable(s.qv1[k]), prob->getVariable(s.qv2[k]), s.qval[k]);
  }
  return qf ? (FunctionPtr) new Function(lf, qf) : (FunctionPtr) new Function(lf);
}

// Runs presolveNode of a QuadHandler (hip = 0 reference, 1 HipQuadHandler)
// on the root box, then on every node box with the relaxation rows reset to
// their root state; outputs the bounds, verdicts, r_mods counts, the row
// state after each call, and (hip) the GPU / CPU call counts.
int integ_quad(int device, int hip, const QSpecI *sp, int has_inc, double inc, int B,
               const double *node_lb, const double *node_ub, double *out_lb, double *out_ub,
               int *infeas, int *nmods, double *rows_out, int *calls) {
  const QSpecI &s = *sp;
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  ProblemPtr orig = (ProblemPtr) new Problem(env);
  for (int j = 0; j < s.nv0; ++j) orig->newVariable(s.vlb[j], s.vub[j], (VariableType)s.vtype[j]);
  for (int c = 0; c < s.ncon; ++c) orig->newConstraint(qfun(s, orig, c), s.clb[c], s.cub[c]);
  if (s.has_obj) orig->newObjective(qfun(s, orig, s.ncon), s.obj_const, Minimize);
  else orig->newObjective((FunctionPtr) new Function((LinearFunctionPtr) new LinearFunction()),
                          s.obj_const, Minimize);
  orig->calculateSize();
  ProblemPtr p = (ProblemPtr) new Problem(env);
  for (int j = 0; j < s.nv; ++j) p->newVariable(s.vlb[j], s.vub[j], (VariableType)s.vtype[j]);
  QuadHandler *qh = hip ? (QuadHandler *) new HipQuadHandler(env, p, orig, device)
                        : new QuadHandler(env, p, orig);
  auto add_aux = [&](int x0, int x1, int y) {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    lf->addTerm(p->getVariable(y), -1.0);
    QuadraticFunctionPtr qf = (QuadraticFunctionPtr) new QuadraticFunction();
    qf->addTerm(p->getVariable(x0), p->getVariable(x1), 1.0);
    qh->addConstraint(p->newConstraint((FunctionPtr) new Function(lf, qf), 0.0, 0.0));
  };
  for (int k = 0; k < s.nsq; ++k) add_aux(s.sq_x[k], s.sq_x[k], s.sq_y[k]);
  for (int k = 0; k < s.nbil; ++k) add_aux(s.bil_x0[k], s.bil_x1[k], s.bil_y[k]);
  p->calculateSize();
  RelaxationPtr rel = (RelaxationPtr) new Relaxation(env);
  for (int j = 0; j < s.nv; ++j) {
    VariablePtr v = p->getVariable(j);
    rel->newVariable(v->getLb(), v->getUb(), v->getType());
  }
  bool inf = false;
  qh->relaxInitInc(rel, &inf);
  rel->calculateSize();
  SolutionPoolPtr spool = (SolutionPoolPtr) new SolutionPool(env, p, 1);
  if (has_inc) {
    std::vector<double> x(s.nv, 0.0);
    spool->addSolution(x.data(), inc);
  }
  const int nrows = s.nsq + 4 * s.nbil;
  std::vector<LinearFunctionPtr> lf0(nrows);
  std::vector<double> ub0(nrows);
  for (int i = 0; i < nrows; ++i) {
    lf0[i] = rel->getConstraint(i)->getLinearFunction()->clone();
    ub0[i] = rel->getConstraint(i)->getUb();
  }
  auto set_box = [&](const double *lb, const double *ub) {
    for (int j = 0; j < s.nv; ++j) {
      p->changeBound(p->getVariable(j), lb[j], ub[j]);
      rel->changeBound(rel->getVariable(j), lb[j], ub[j]);
    }
    for (int i = 0; i < nrows; ++i)
      rel->changeConstraint(rel->getConstraint(i), lf0[i]->clone(), -INFINITY, ub0[i]);
  };
  const int R = 2 * s.nsq + 12 * s.nbil;
  for (int b = -1; b < B; ++b) {   // b = -1: the root call
    if (b < 0) set_box(s.vlb, s.vub);
    else set_box(node_lb + (size_t)b * s.nv, node_ub + (size_t)b * s.nv);
    ModVector pm, rm;
    const bool r = qh->presolveNode(rel, NodePtr(), spool, pm, rm);
    if (b < 0) {
      for (ModificationPtr m : pm) delete m;
      for (ModificationPtr m : rm) delete m;
      continue;
    }
    infeas[b] = r ? 1 : 0;
    nmods[b] = (int)rm.size();
    for (int j = 0; j < s.nv; ++j) {
      out_lb[(size_t)b * s.nv + j] = rel->getVariable(j)->getLb();
      out_ub[(size_t)b * s.nv + j] = rel->getVariable(j)->getUb();
    }
    double *ro = rows_out + (size_t)b * R;
    int o = 0;
    for (int k = 0; k < s.nsq; ++k) {
      ConstraintPtr c = rel->getConstraint(k);
      ro[o++] = c->getLinearFunction()->getWeight(rel->getVariable(s.sq_x[k]));
      ro[o++] = c->getUb();
    }
    for (int k = 0; k < s.nbil; ++k)
      for (int t = 0; t < 4; ++t) {
        ConstraintPtr c = rel->getConstraint(s.nsq + 4 * k + t);
        ro[o++] = c->getLinearFunction()->getWeight(rel->getVariable(s.bil_x0[k]));
        ro[o++] = c->getLinearFunction()->getWeight(rel->getVariable(s.bil_x1[k]));
        ro[o++] = c->getUb();
      }
    for (ModificationPtr m : pm) delete m;
    for (ModificationPtr m : rm) delete m;
  }
  calls[0] = hip ? (int)((HipQuadHandler *)qh)->gpuCalls() : 0;
  calls[1] = hip ? (int)((HipQuadHandler *)qh)->cpuCalls() : 0;
  for (LinearFunctionPtr f : lf0) delete f;
  delete qh;
  delete spool;
  delete rel;
  delete p;
  delete orig;
  delete env;
  return 0;
}

// The reference's own root OBBT, QuadHandler::postSolveRootNode (QuadHandler.
// cpp:1397-1547) -> tightenLP_ (:2218-2297), with HipLPEngine as its bound-
// tightening engine bte_ (setBTEngine, as SimpleTransformer.cpp:948-951
// wires it in mglob) and as the root relaxation's engine.  The relaxation
// is the one minotaur_amd/obbt.py relaxation_lp builds: the original
// constraints with every product replaced by its aux y, then the secant /
// McCormick rows of relaxInitInc, objective in the same form.
// Outputs: p_'s variable bounds after OBBT; info[0] root LP status,
// info[1] postSolveRootNode's return value, info[2] bound LPs solved by bte_;
// log_*[k] (k < cap): bte_'s solves in order (column, sign, status, value).
int integ_obbt(int device, const QSpecI *sp, int has_inc, double inc, double *out_lb,
               double *out_ub, int *info, int cap, int *log_col, double *log_sign,
               int *log_st, double *log_val) {
  const QSpecI &s = *sp;
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  ProblemPtr orig = (ProblemPtr) new Problem(env);
  for (int j = 0; j < s.nv0; ++j) orig->newVariable(s.vlb[j], s.vub[j], (VariableType)s.vtype[j]);
  for (int c = 0; c < s.ncon; ++c) orig->newConstraint(qfun(s, orig, c), s.clb[c], s.cub[c]);
  if (s.has_obj) orig->newObjective(qfun(s, orig, s.ncon), s.obj_const, Minimize);
  else orig->newObjective((FunctionPtr) new Function((LinearFunctionPtr) new LinearFunction()),
                          s.obj_const, Minimize);
  orig->calculateSize();
  ProblemPtr p = (ProblemPtr) new Problem(env);
  for (int j = 0; j < s.nv; ++j) p->newVariable(s.vlb[j], s.vub[j], (VariableType)s.vtype[j]);
  QuadHandler *qh = new QuadHandler(env, p, orig);
  auto add_aux = [&](int x0, int x1, int y) {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    lf->addTerm(p->getVariable(y), -1.0);
    QuadraticFunctionPtr qf = (QuadraticFunctionPtr) new QuadraticFunction();
    qf->addTerm(p->getVariable(x0), p->getVariable(x1), 1.0);
    qh->addConstraint(p->newConstraint((FunctionPtr) new Function(lf, qf), 0.0, 0.0));
  };
  for (int k = 0; k < s.nsq; ++k) add_aux(s.sq_x[k], s.sq_x[k], s.sq_y[k]);
  for (int k = 0; k < s.nbil; ++k) add_aux(s.bil_x0[k], s.bil_x1[k], s.bil_y[k]);
  p->calculateSize();
  RelaxationPtr rel = (RelaxationPtr) new Relaxation(env);
  for (int j = 0; j < s.nv; ++j) {
    VariablePtr v = p->getVariable(j);
    rel->newVariable(v->getLb(), v->getUb(), v->getType());
  }
  // original rows / objective with products replaced by their aux y
  auto yof = [&](int a, int b) {
    for (int k = 0; k < s.nsq; ++k)
      if (a == s.sq_x[k] && b == s.sq_x[k]) return s.sq_y[k];
    for (int k = 0; k < s.nbil; ++k)
      if (a == s.bil_x0[k] && b == s.bil_x1[k]) return s.bil_y[k];
    return -1;
  };
  auto ylin = [&](int c) {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    for (int k = s.lptr[c]; k < s.lptr[c + 1]; ++k)
      lf->incTerm(rel->getVariable(s.lvar[k]), s.lval[k]);
    for (int k = s.qptr[c]; k < s.qptr[c + 1]; ++k)
      lf->incTerm(rel->getVariable(yof(s.qv1[k], s.qv2[k])), s.qval[k]);
    return lf;
  };
  for (int c = 0; c < s.ncon; ++c)
    rel->newConstraint((FunctionPtr) new Function(ylin(c)), s.clb[c], s.cub[c]);
  bool inf = false;
  qh->relaxInitInc(rel, &inf);
  if (s.has_obj) rel->newObjective((FunctionPtr) new Function(ylin(s.ncon)), s.obj_const, Minimize);
  else rel->newObjective((FunctionPtr) new Function((LinearFunctionPtr) new LinearFunction()),
                         s.obj_const, Minimize);
  rel->calculateSize();
  SolutionPoolPtr spool = (SolutionPoolPtr) new SolutionPool(env, p, 1);
  if (has_inc) {
    std::vector<double> x(s.nv, 0.0);
    spool->addSolution(x.data(), inc);
  }
  HipLPEngine *root_e = new HipLPEngine(env, device);
  HipLPEngine *bte = new HipLPEngine(env, device);
  qh->setBTEngine(bte);
  root_e->load(rel);
  info[0] = (int)root_e->solve();
  info[1] = -1;
  info[2] = 0;
  if (info[0] == ProvenOptimal) {
    ModVector pm, rm;
    info[1] = qh->postSolveRootNode(rel, spool, root_e->getSolution(), pm, rm) ? 1 : 0;
    for (ModificationPtr m : pm) delete m;
    for (ModificationPtr m : rm) delete m;
    std::vector<double> st(6, 0.0);
    bte->fillStats(st);
    info[2] = (int)st[0];
    const auto &lg = bte->solveLog();
    for (size_t k = 0; k < lg.size() && (int)k < cap; ++k) {
      log_col[k] = lg[k].col;
      log_sign[k] = lg[k].sign;
      log_st[k] = lg[k].status;
      log_val[k] = lg[k].value;
    }
  }
  for (int j = 0; j < s.nv; ++j) {
    out_lb[j] = p->getVariable(j)->getLb();
    out_ub[j] = p->getVariable(j)->getUb();
  }
  root_e->clear();
  delete qh;          // QuadHandler's destructor deletes its bte_ (QuadHandler.cpp:118-120)
  delete root_e;
  delete spool;
  delete rel;
  delete p;
  delete orig;
  delete env;
  return 0;
}


// ---- the reference's own spatial branch-and-bound (Glob's tree) -----------
// QuadHandler whose fixNodeErr (PCBProcessor.cpp:311-314, NoCandToBranch)
// does what the batched glob tree does there -- closes the node without a
// solution -- and counts it: the reference calls an NLP engine here
// (QuadHandler.cpp:356-420), and none is in the image.
class NoNlpQuadHandler : public QuadHandler {
 public:
  NoNlpQuadHandler(EnvPtr env, ProblemPtr p, ProblemPtr orig) : QuadHandler(env, p, orig) {}
  int fixNodeErr(RelaxationPtr, ConstSolutionPtr, SolutionPoolPtr, bool &sol_found) {
    sol_found = false;
    ++closed;
    return 0;
  }
  long long closed = 0;
  void separate(ConstSolutionPtr sol, NodePtr node, RelaxationPtr rel, CutManager *cm,
                SolutionPoolPtr s_pool, ModVector &p_mods, ModVector &r_mods, bool *sol_found,
                SeparationStatus *status) {
    ++sepa_;
    const long long m0 = (long long)rel->getNumCons();
    QuadHandler::separate(sol, node, rel, cm, s_pool, p_mods, r_mods, sol_found, status);
    const long long add = (long long)rel->getNumCons() - m0;
    rows_ += add;
    if (!node->getParent()) rootRows_ += add;
  }
  long long sepaRounds() const { return sepa_; }
  long long sepaRows() const { return rows_; }        // rows added by separate()
  long long rootSepaRows() const { return rootRows_; }  // ... at the root (simplex cuts there)

 private:
  long long sepa_ = 0, rows_ = 0, rootRows_ = 0;
};

// MaxVioBrancher that logs each branching (variable, its LP value) in order:
// the pin tests compare it with the batched tree's branching sequence
static std::vector<std::pair<int, double>> g_last_branch;

class LogMaxVioBrancher : public MaxVioBrancher {
 public:
  LogMaxVioBrancher(EnvPtr env, HandlerVector &h) : MaxVioBrancher(env, h) {}
  Branches findBranches(RelaxationPtr rel, NodePtr node, ConstSolutionPtr sol,
                        SolutionPoolPtr s_pool, BrancherStatus &br_status, ModVector &mods) {
    Branches br = MaxVioBrancher::findBranches(rel, node, sol, s_pool, br_status, mods);
    if (br && !br->empty()) {
      BrVarCandPtr vc = dynamic_cast<BrVarCand *>((*br->begin())->getBrCand());
      if (vc) {
        const int j = (int)vc->getVar()->getIndex();
        g_last_branch.push_back({j, sol->getPrimal()[j]});
      }
    }
    return br;
  }
};

int integ_last_branch_log(int cap, int *var, double *val) {
  for (size_t k = 0; k < g_last_branch.size() && (int)k < cap; ++k) {
    var[k] = g_last_branch[k].first;
    val[k] = g_last_branch[k].second;
  }
  return (int)g_last_branch.size();
}

// LinearHandler without node presolve (flags bit 1): the batched glob
// round runs no linear FBBT at its nodes
class NoPresolveLinearHandler : public LinearHandler {
 public:
  NoPresolveLinearHandler(EnvPtr env, ProblemPtr p) : LinearHandler(env, p) {}
  bool presolveNode(RelaxationPtr, NodePtr, SolutionPoolPtr, ModVector &, ModVector &) {
    return false;
  }
};

}  // extern "C"

// The QCQP's auxiliary form, as SimpleTransformer builds it for Glob: the
// original rows with every product replaced by its aux y (LinearHandler's
// rows), and y = x0 x1 / y = x^2 for each product (QuadHandler's
// constraints: McCormick / secant rows, presolveNode, isFeasible, spatial
// candidates).  qh is constructed by the caller's factory.
template <class QH>
static QH *glob_model(EnvPtr env, const QSpecI &s, ProblemPtr &orig, ProblemPtr &p) {
  orig = (ProblemPtr) new Problem(env);
  for (int j = 0; j < s.nv0; ++j) orig->newVariable(s.vlb[j], s.vub[j], (VariableType)s.vtype[j]);
  for (int c = 0; c < s.ncon; ++c) orig->newConstraint(qfun(s, orig, c), s.clb[c], s.cub[c]);
  if (s.has_obj) orig->newObjective(qfun(s, orig, s.ncon), s.obj_const, Minimize);
  else orig->newObjective((FunctionPtr) new Function((LinearFunctionPtr) new LinearFunction()),
                          s.obj_const, Minimize);
  orig->calculateSize();
  p = (ProblemPtr) new Problem(env);
  for (int j = 0; j < s.nv; ++j) p->newVariable(s.vlb[j], s.vub[j], (VariableType)s.vtype[j]);
  auto yof = [&](int a, int b) {
    for (int k = 0; k < s.nsq; ++k)
      if (a == s.sq_x[k] && b == s.sq_x[k]) return s.sq_y[k];
    for (int k = 0; k < s.nbil; ++k)
      if (a == s.bil_x0[k] && b == s.bil_x1[k]) return s.bil_y[k];
    return -1;
  };
  auto ylin = [&](int c) {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    for (int k = s.lptr[c]; k < s.lptr[c + 1]; ++k) lf->incTerm(p->getVariable(s.lvar[k]), s.lval[k]);
    for (int k = s.qptr[c]; k < s.qptr[c + 1]; ++k)
      lf->incTerm(p->getVariable(yof(s.qv1[k], s.qv2[k])), s.qval[k]);
    return lf;
  };
  for (int c = 0; c < s.ncon; ++c)
    p->newConstraint((FunctionPtr) new Function(ylin(c)), s.clb[c], s.cub[c]);
  if (s.has_obj) p->newObjective((FunctionPtr) new Function(ylin(s.ncon)), s.obj_const, Minimize);
  else p->newObjective((FunctionPtr) new Function((LinearFunctionPtr) new LinearFunction()),
                       s.obj_const, Minimize);
  QH *qh = new QH(env, p, orig);
  auto add_aux = [&](int x0, int x1, int y) {
    LinearFunctionPtr lf = (LinearFunctionPtr) new LinearFunction();
    lf->addTerm(p->getVariable(y), -1.0);
    QuadraticFunctionPtr qf = (QuadraticFunctionPtr) new QuadraticFunction();
    qf->addTerm(p->getVariable(x0), p->getVariable(x1), 1.0);
    qh->addConstraint(p->newConstraint((FunctionPtr) new Function(lf, qf), 0.0, 0.0));
  };
  for (int k = 0; k < s.nsq; ++k) add_aux(s.sq_x[k], s.sq_x[k], s.sq_y[k]);
  for (int k = 0; k < s.nbil; ++k) add_aux(s.bil_x0[k], s.bil_x1[k], s.bil_y[k]);
  p->calculateSize();
  return qh;
}

static LPEnginePtr new_engine(EnvPtr env, int device) {
  // device < 0: CpuLPEngine (the C restatement of the dual simplex), for CPU runs
  return device < 0 ? (LPEnginePtr) new CpuLPEngine(env) : (LPEnginePtr) new HipLPEngine(env, device);
}

extern "C" {

// Glob::createBab_ (Glob.cpp:134-220) over the QCQP's auxiliary form
// (glob_model): IntVarHandler, LinearHandler, QuadHandler; PCBProcessor,
// NodeIncRelaxer (parent warm starts), HipLPEngine for the LPs (Clp is
// absent; device < 0: CpuLPEngine).  opts bits:
//   1  tree_search bfs (else dfs)
//   2  LinearHandler without node presolve (the batched glob round's shape)
//   4  simplex_cut on (Glob.cpp:311): QuadHandler's cute_ is the main engine,
//      as SimpleTransformer.cpp:953-954 wires it, so the root separation runs
//      SimplexQuadCutGen on this engine's tableau (QuadHandler.cpp:1691-1703)
//   8  root OBBT on (Environment.cpp:325-326 default; PCBProcessor.cpp:256-262
//      -> QuadHandler::postSolveRootNode) with a second engine of the same
//      kind as bte_ (SimpleTransformer.cpp:948-951)
//  16  brancher relstronger (Glob.cpp:308): StrongBrancher::reliabilitySetup
//      (20, 50, 5) (Glob.cpp:171-181), else MaxVioBrancher
// Every other option keeps its default (obj_gap_percent 0: the tree runs to
// completion).  res[0] UB, res[1] LB, res[2] seconds; cnt[0] nodes processed,
// cnt[1] nodes created, cnt[2] LP solves of the main engine, cnt[3] nodes
// closed at NoCandToBranch, cnt[4] rows QuadHandler::separate added at the
// root (the simplex cuts, and tangents of violated squares), cnt[5] bound
// LPs of OBBT, cnt[6] QuadHandler::separate calls, cnt[7] rows it added in
// the whole tree; x (nullable, nv) the
// incumbent of the auxiliary form.
int integ_glob_tree3(int device, const QSpecI *sp, int opts, int pres_freq, double *res,
                     long long *cnt, double *x) {
  const QSpecI &s = *sp;
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  env->getOptions()->findString("tree_search")->setValue((opts & 1) ? "bfs" : "dfs");
  env->getOptions()->findBool("OBBT")->setValue((opts & 8) != 0);
  env->getOptions()->findBool("simplex_cut")->setValue((opts & 4) != 0);
  env->getOptions()->findInt("pres_freq")->setValue(pres_freq);
  ProblemPtr orig = 0, p = 0;
  NoNlpQuadHandler *qh = glob_model<NoNlpQuadHandler>(env, s, orig, p);
  ProbeBranchAndBound *bab = new ProbeBranchAndBound(env, p);
  HandlerVector handlers;
  IntVarHandlerPtr v_hand = (IntVarHandlerPtr) new IntVarHandler(env, p);
  LinearHandlerPtr l_hand = (opts & 2) ? (LinearHandlerPtr) new NoPresolveLinearHandler(env, p)
                                       : (LinearHandlerPtr) new LinearHandler(env, p);
  handlers.push_back(v_hand);
  handlers.push_back(l_hand);
  handlers.push_back(qh);
  // SimpleTransformer's flags (SimpleTransformer.cpp:936-949): every handler
  // modifies the problem and the relaxation, and NodeIncRelaxer replays both
  // (modProb_ true by default, NodeIncRelaxer.cpp:28-35).  QuadHandler's
  // updatePBounds_ tightens p_ whatever its flags (QuadHandler.cpp:3268-
  // 3275) and reads p_'s bounds, so with the problem's mods not replayed the
  // tree would depend on the order nodes ran in.
  v_hand->setModFlags(true, true);
  l_hand->setModFlags(true, true);
  qh->setModFlags(true, true);
  LPEnginePtr e = new_engine(env, device);
  LPEnginePtr bte = 0;
  if (opts & 8) {
    bte = new_engine(env, device);
    qh->setBTEngine(bte);     // owned by the handler (QuadHandler.cpp:118-120)
  }
  if (opts & 4) qh->setCutEngine(e);
  PCBProcessorPtr nproc = (PCBProcessorPtr) new PCBProcessor(env, e, handlers);
  BrancherPtr br;
  if (opts & 16) {
    StrongBrancherPtr sb = (StrongBrancherPtr) new StrongBrancher(env, handlers);
    sb->setEngine(e);
    sb->reliabilitySetup(20, 50, 5);
    sb->setProblem(p);
    br = sb;
  } else {
    g_last_branch.clear();
    br = (BrancherPtr) new LogMaxVioBrancher(env, handlers);
  }
  nproc->setBrancher(br);
  bab->setNodeProcessor(nproc);
  NodeIncRelaxerPtr nr = (NodeIncRelaxerPtr) new NodeIncRelaxer(env, handlers);
  nr->setProblem(p);
  nr->setEngine(e);
  bab->setNodeRelaxer(nr);
  bab->shouldCreateRoot(true);
  bab->setLogLevel(LogNone);
  const auto t0 = std::chrono::steady_clock::now();
  bab->solve();
  res[2] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  res[0] = bab->getUb();
  res[1] = bab->getLb();
  cnt[0] = bab->nodesProcessed();
  cnt[1] = (long long)bab->getTreeManager()->getSize();
  std::vector<double> lps(6, 0.0);
  e->fillStats(lps);
  cnt[2] = (long long)lps[0];
  cnt[3] = qh->closed;
  cnt[4] = qh->rootSepaRows();
  cnt[5] = 0;
  if (bte) {
    std::vector<double> bl(6, 0.0);
    bte->fillStats(bl);
    cnt[5] = (long long)bl[0];
  }
  cnt[6] = qh->sepaRounds();
  cnt[7] = qh->sepaRows();
  g_last_log.clear();
  if (HipLPEngine *he = dynamic_cast<HipLPEngine *>(e)) {
    g_last_engine[0] = he->refactors();
    g_last_engine[1] = he->coldSolves();
    for (const auto &r : he->solveLog()) g_last_log.push_back({r.status, r.value, r.iters});
  } else if (CpuLPEngine *ce = dynamic_cast<CpuLPEngine *>(e)) {
    g_last_engine[0] = ce->refactors();
    g_last_engine[1] = ce->coldSolves();
    for (const auto &r : ce->solveLog()) g_last_log.push_back({r.status, r.value, r.iters});
  }
  if (x) {
    SolutionPtr sol = bab->getSolution();
    for (int j = 0; j < s.nv; ++j) x[j] = sol ? sol->getPrimal()[j] : NAN;
  }
  delete v_hand;
  delete l_hand;
  delete qh;
  delete e;
  delete nproc;
  delete nr;
  delete bab;
  delete p;
  delete orig;
  delete env;
  return 0;
}

// flags bit 1: LinearHandler without node presolve; pres_freq: PCBProcessor's
// node-presolve frequency (reference default 5, Environment.cpp:364); bfs:
// tree_search bfs (else dfs).  Root OBBT and simplex cuts off, MaxVio.
int integ_glob_tree2(int device, const QSpecI *sp, int bfs, int flags, int pres_freq, double *res,
                     long long *cnt) {
  long long c8[8];
  int rc = integ_glob_tree3(device, sp, (bfs ? 1 : 0) | (flags & 2), pres_freq, res, c8, nullptr);
  for (int k = 0; k < 4; ++k) cnt[k] = c8[k];
  return rc;
}

// Glob's defaults: LinearHandler presolve, pres_freq 5
int integ_glob_tree(int device, const QSpecI *sp, int bfs, double *res, long long *cnt) {
  return integ_glob_tree2(device, sp, bfs, 0, 5, res, cnt);
}

// The root of Glob's tree through the LPEngine tableau extras: the root
// relaxation (NodeIncRelaxer::createRootRelaxation over IntVar / Linear /
// Quad handlers, NodeIncRelaxer.cpp:49-67) solved by the engine (device < 0:
// CpuLPEngine), then
//   1. the engine's views as SimplexQuadCutGen::getBasicInfo_ reads them
//      (SimplexQuadCutGen.cpp:285-304): dims[0] n, dims[1] m, dims[2] nnz,
//      dims[3] root LP status, dims[4] IsOptimalBasisAvailable, dims[5] the
//      factorization site (HipLPEngine: 1 device K3R, 0 host); rowstart
//      [m+1], rowlen [m], ind [nnz], val [nnz], clo / chi [n], rlo / rhi /
//      rhs / act [m]; the relaxation's own rows for comparison: rrow [nnz],
//      rcol [nnz], rval [nnz] in iteration order, rlb / rub [m], vlb / vub [n];
//   2. enableFactorization, getBasics -> basics [m], getBInvARow for every
//      basis position -> z [m][n], slack [m][m], disableFactorization;
//   3. SimplexQuadCutGen(env, p, engine, +inf)::generateCuts(rel, sol) -- the
//      reference's own cut generator on this engine -> dims[6] cuts added;
//      each cut's dense coefficients [cap][n] and its lb / ub.  The generator
//      keeps maxCuts_ = min(max(ceil(0.2 n), ceil(0.05 m)), 20) of its
//      candidates (SimplexQuadCutGen.cpp:58-60) after std::sort on the vector
//      of SimplexCut POINTERS (:204): which ones depends on heap addresses.
//      lift != 0 gives the generator's problem 400 extra empty rows after the
//      relaxation is built, so maxCuts_ is its cap 20 and every candidate of
//      depth >= minDepth_ is added (two engines then compare as sets).
// x [n]: the root LP's primal point.  cap bounds n, m, nnz and the cuts.
int integ_simplex_cuts(int device, const QSpecI *sp, int cap, int lift, long long *dims,
                       int *rowstart,
                       int *rowlen, int *ind, double *val, double *clo, double *chi, double *rlo,
                       double *rhi, double *rhs, double *act, int *rrow, int *rcol, double *rval,
                       double *rlb, double *rub, double *vlb, double *vub, int *basics, double *z,
                       double *slack, double *x, double *cut_coef, double *cut_lb,
                       double *cut_ub) {
  const QSpecI &s = *sp;
  EnvPtr env = (EnvPtr) new Environment();
  int err = 0;
  env->startTimer(err);
  env->getOptions()->findBool("simplex_cut")->setValue(true);
  ProblemPtr orig = 0, p = 0;
  NoNlpQuadHandler *qh = glob_model<NoNlpQuadHandler>(env, s, orig, p);
  HandlerVector handlers;
  IntVarHandlerPtr v_hand = (IntVarHandlerPtr) new IntVarHandler(env, p);
  LinearHandlerPtr l_hand = (LinearHandlerPtr) new LinearHandler(env, p);
  handlers.push_back(v_hand);
  handlers.push_back(l_hand);
  handlers.push_back(qh);
  LPEnginePtr e = new_engine(env, device);
  NodeIncRelaxerPtr nr = (NodeIncRelaxerPtr) new NodeIncRelaxer(env, handlers);
  nr->setProblem(p);
  nr->setEngine(e);
  bool prune = false;
  RelaxationPtr rel = nr->createRootRelaxation(NodePtr(), prune);
  int rc = 0;
  for (int k = 0; k < 7; ++k) dims[k] = 0;
  const int n = (int)rel->getNumVars(), m = (int)rel->getNumCons();
  dims[0] = n;
  dims[1] = m;
  if (prune || n > cap || m > cap) {
    rc = -1;
  } else {
    dims[3] = (long long)e->solve();
    dims[4] = e->IsOptimalBasisAvailable() ? 1 : 0;
    const int *rs = e->getRowStarts();
    const int nnz = rs ? rs[m] : 0;
    dims[2] = nnz;
    if (!rs || nnz > cap * cap) {
      rc = -2;
    } else {
      const double *v;
      std::copy(rs, rs + m + 1, rowstart);
      std::copy(e->getRowLength(), e->getRowLength() + m, rowlen);
      std::copy(e->getIndicesofVars(), e->getIndicesofVars() + nnz, ind);
      std::copy(e->getOriginalTableau(), e->getOriginalTableau() + nnz, val);
      v = e->getColLower(); std::copy(v, v + n, clo);
      v = e->getColUpper(); std::copy(v, v + n, chi);
      v = e->getRowLower(); std::copy(v, v + m, rlo);
      v = e->getRowUpper(); std::copy(v, v + m, rhi);
      v = e->getRightHandSide(); std::copy(v, v + m, rhs);
      v = e->getRowActivity(); std::copy(v, v + m, act);
      int t = 0;
      for (int i = 0; i < m; ++i) {
        ConstraintPtr c = rel->getConstraint(i);
        rlb[i] = c->getLb();
        rub[i] = c->getUb();
        LinearFunctionPtr lf = c->getLinearFunction();
        if (lf)
          for (VariableGroupConstIterator it = lf->termsBegin(); it != lf->termsEnd(); ++it) {
            if (t < nnz) {
              rrow[t] = i;
              rcol[t] = (int)it->first->getIndex();
              rval[t] = it->second;
            }
            ++t;
          }
      }
      if (t != nnz) rc = -3;
      for (int j = 0; j < n; ++j) {
        vlb[j] = rel->getVariable(j)->getLb();
        vub[j] = rel->getVariable(j)->getUb();
      }
      if (dims[3] == ProvenOptimal) {
        const double *xp = e->getSolution()->getPrimal();
        std::copy(xp, xp + n, x);
        e->enableFactorization();
        if (HipLPEngine *he = dynamic_cast<HipLPEngine *>(e)) dims[5] = he->factorSite();
        e->getBasics(basics);
        for (int r = 0; r < m; ++r)
          e->getBInvARow(r, z + (size_t)r * n, slack + (size_t)r * m);
        e->disableFactorization();
        // the reference's cut generator on this engine (generateCuts enables
        // and disables the factorization itself, :179-190)
        if (lift) {
          LinearFunctionPtr lf0 = (LinearFunctionPtr) new LinearFunction();
          lf0->addTerm(p->getVariable(0), 1.0);
          for (int k = 0; k < 400; ++k)
            p->newConstraint((FunctionPtr) new Function(lf0->clone()), -INFINITY, INFINITY);
          delete lf0;
        }
        SimplexQuadCutGen cg(env, p, e, INFINITY);
        const int ncuts = cg.generateCuts(rel, e->getSolution());
        dims[6] = ncuts;
        for (int k = 0; k < ncuts && k < cap; ++k) {
          ConstraintPtr c = rel->getConstraint(m + k);
          cut_lb[k] = c->getLb();
          cut_ub[k] = c->getUb();
          double *row = cut_coef + (size_t)k * n;
          for (int j = 0; j < n; ++j) row[j] = 0.0;
          LinearFunctionPtr lf = c->getLinearFunction();
          if (lf)
            for (VariableGroupConstIterator it = lf->termsBegin(); it != lf->termsEnd(); ++it)
              row[it->first->getIndex()] = it->second;
        }
      }
    }
  }
  e->clear();
  delete nr;   // deletes the relaxation (NodeIncRelaxer.cpp:38-44)
  delete v_hand;
  delete l_hand;
  delete qh;
  delete e;
  delete p;
  delete orig;
  delete env;
  return rc;
}

// The reference's own Serializer / DeSerializer (src/base/Serializer.cpp:
// 26-191) for tests/test_serial_cpu.py.
// integ_serialize_path: a Problem with the root box and the root Node, then
// `steps` modifications in order: kind 0 a child whose Branch carries
// VarBoundMod(var, lu, val) (the child becomes the current node), kind 1 a
// relaxation mod of the current node (Node::addRMod, where presolve mods
// live).  Each mod's old value is the bound before it (VarBoundMod reads the
// variable; the harness then moves the bound).  Serializer::writeNode(the
// current node) -> out; returns the byte count (-1: cap too small).
long integ_serialize_path(int n, const double *root_lb, const double *root_ub, int steps,
                          const int *kind, const int *var, const int *lu, const double *val,
                          unsigned id, double nlb, unsigned char *out, long cap) {
  EnvPtr env = (EnvPtr) new Environment();
  ProblemPtr p = (ProblemPtr) new Problem(env);
  std::vector<VariablePtr> vars;
  for (int j = 0; j < n; ++j) vars.push_back(p->newVariable(root_lb[j], root_ub[j], Continuous));
  std::vector<NodePtr> path;
  NodePtr cur = (NodePtr) new Node();
  path.push_back(cur);
  for (int s = 0; s < steps; ++s) {
    VariablePtr v = vars[var[s]];
    const BoundType bt = lu[s] ? Upper : Lower;
    VarBoundModPtr md = (VarBoundModPtr) new VarBoundMod(v, bt, val[s]);
    p->changeBound(v, bt, val[s]);
    if (kind[s] == 0) {
      BranchPtr br = (BranchPtr) new Branch();
      br->addRMod(md);
      cur = (NodePtr) new Node(cur, br);
      path.push_back(cur);
    } else {
      cur->addRMod(md);
    }
  }
  cur->setId(id);
  cur->setLb(nlb);
  Serializer ser;
  ser.writeNode(cur);
  const std::string bytes = ser.get_string();
  long len = (long)bytes.size();
  if (out) {
    if (len <= cap) std::memcpy(out, bytes.data(), bytes.size());
    else len = -1;
  }
  for (size_t k = path.size(); k-- > 0;) delete path[k];
  delete p;
  delete env;
  return len;
}

// integ_deserialize_node: DeSerializer::readNode on buf against a Problem with
// the root box: the node's id, lower bound and its relaxation mods applied to
// the root box (lb / ub); returns the mod count.
int integ_deserialize_node(const unsigned char *buf, long len, int n, const double *root_lb,
                           const double *root_ub, unsigned *id, double *nlb, double *lb,
                           double *ub) {
  EnvPtr env = (EnvPtr) new Environment();
  ProblemPtr p = (ProblemPtr) new Problem(env);
  for (int j = 0; j < n; ++j) p->newVariable(root_lb[j], root_ub[j], Continuous);
  DeSerializer d(std::string((const char *)buf, (size_t)len));
  NodePtr node = d.readNode(p);
  *id = node->getId();
  *nlb = node->getLb();
  for (int j = 0; j < n; ++j) {
    lb[j] = root_lb[j];
    ub[j] = root_ub[j];
  }
  int cnt = 0;
  for (ModificationConstIterator it = node->modsrBegin(); it != node->modsrEnd(); ++it, ++cnt) {
    VarBoundModPtr md = (VarBoundModPtr) *it;
    (md->getLU() == Lower ? lb : ub)[md->getVar()->getIndex()] = md->getNewVal();
  }
  delete node;
  delete p;
  delete env;
  return cnt;
}

}  // extern "C"
