// ReliabilityBrancher's verdict on one strong-branched candidate (device
// code), shared by the round's decision (bnb_rel.hip) and K3's chained mode
// (lp_dual.hip), which stops a node's strong branching at the first verdict.
#pragma once

namespace mgpu {

constexpr double kSbETol = 1e-6;   // ReliabilityBrancher eTol_ (:43-58)

// ReliabilityBrancher::shouldPrune_ (:430-467) for one strong-branching LP
__device__ __forceinline__ bool sb_prune(double chcutoff, double change, int st, bool &is_rel) {
  switch (st) {
    case 3:   // ProvenLocalInfeasible
    case 2:   // ProvenInfeasible
    case 5:   // ProvenObjectiveCutOff
      return true;
    case 1:   // ProvenLocalOptimal
    case 0:   // ProvenOptimal (trustCutoff_)
      return change > chcutoff - kSbETol;
    case 6:   // EngineIterationLimit
      return false;
    case 7:   // ProvenFailedCQFeas / Infeas
    case 8:
      is_rel = false;
      return false;
    default:  // unexpected status (engProbs)
      is_rel = false;
      return false;
  }
}

// a candidate after both LPs (down: status sd, value od; up: su, ou): the
// changes (max(value - objval, 0), zeroed when a side is unreliable) and
// useStrongBranchInfo_'s verdict: -1 a side unreliable (no observation), 0
// none, 1 both sides pruned, 2 the up side pruned (the down branch's bound
// change), 3 the down side pruned (the up branch's); findBestCandidate_ stops
// strong branching at a verdict > 0 (:111-118)
__device__ __forceinline__ int sb_verdict(int sd, double od, int su, double ou, double objval,
                                          double maxchange, double &cd, double &cu) {
  cd = fmax(od - objval, 0.0);
  cu = fmax(ou - objval, 0.0);
  bool is_rel = true;
  const bool pd = sb_prune(maxchange, cd, sd, is_rel);
  const bool pu = sb_prune(maxchange, cu, su, is_rel);
  if (!is_rel) {
    cu = 0.0;
    cd = 0.0;
    return -1;
  }
  return (pu && pd) ? 1 : pu ? 2 : pd ? 3 : 0;
}

}  // namespace mgpu
