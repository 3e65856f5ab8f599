// Round collectives and load balancing of the node-sharded tree (SURVEY §8 e).
//
// MpiBranchAndBound (src/base/MpiBranchAndBound.cpp) runs one branch-and-bound
// per MPI rank and couples them with small collectives: the incumbent
// (MPI_Allreduce MIN :387-389, plus eager pushes :197-208), the stop flag
// (MPI_Allreduce LOR :85), the statistics (MPI_Gather :417, :442), and the
// load balancer LoadBalance_ (:78-195: an MPI_Allgather of each rank's next
// candidates' bounds, a common sort and deal, one MPI_Send per moved node).
// Here they are engine calls on the context, so a C++ host with the shape of
// MpiBranchAndBound shards the batched tree through the C ABI alone:
//   * RCCL (mgpu_comm_init): one communicator over the ranks' GPUs (xGMI
//     inside a node); the node rows move device to device in one grouped
//     send/recv exchange;
//   * a host transport (mgpu_comm_init_host): the host's own collectives on
//     host buffers (MPI, or gloo in the one-GPU rehearsal); device rows are
//     staged through host memory.
// The payloads are tiny (a few doubles per round, 50 P bounds per rebalance)
// except the migrated rows: every collective is latency-bound.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "bnb_internal.h"
#include "ctx.h"

struct CommState {
  int rank = 0, world = 1;
  ncclComm_t nccl = nullptr;
  bool host = false;
  mgpu_host_transport t{};
  DevBuf dbuf;                         // device staging of the small collectives
  double *pin = nullptr;               // pinned host staging
  size_t pin_bytes = 0;
  DevBuf send_rows, recv_rows, ord_rows, perm;   // mgpu_bnb_rebalance
};

void comm_state_free(mgpu_ctx *c) {
  if (!c || !c->comm) return;
  CommState *s = c->comm;
  if (s->nccl) (void)ncclCommDestroy(s->nccl);
  if (s->pin) (void)hipHostFree(s->pin);
  delete s;
  c->comm = nullptr;
}

namespace {

#define NCCLCHK(c, expr)                                                              \
  do {                                                                                \
    ncclResult_t r_ = (expr);                                                         \
    if (r_ != ncclSuccess)                                                            \
      return fail((c), MGPU_ERR_COMM, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_), \
                  __FILE__, __LINE__);                                                \
  } while (0)

#define HOSTCHK(c, expr)                                                              \
  do {                                                                                \
    int r_ = (expr);                                                                  \
    if (r_ != 0)                                                                      \
      return fail((c), MGPU_ERR_COMM, "host transport: %s returned %d", #expr, r_);    \
  } while (0)

ncclRedOp_t nccl_op(int op) {
  return op == MGPU_OP_MIN ? ncclMin : op == MGPU_OP_MAX ? ncclMax : ncclSum;
}

int ensure_pin(mgpu_ctx *c, CommState &s, size_t bytes) {
  if (bytes <= s.pin_bytes) return MGPU_OK;
  if (s.pin) (void)hipHostFree(s.pin);
  s.pin = nullptr;
  s.pin_bytes = 0;
  void *p = nullptr;
  HIPCHK(c, hipHostMalloc(&p, bytes, hipHostMallocDefault));
  note_dev_alloc(bytes);   // pinned host memory counts too (mgpu_alloc_stats)
  s.pin = static_cast<double *>(p);
  s.pin_bytes = bytes;
  return MGPU_OK;
}

// a communicator of one rank, or none: the collectives are identities
bool solo(const mgpu_ctx *c) { return !c->comm || (c->comm->world == 1 && !c->comm->nccl && !c->comm->host); }

int new_state(mgpu_ctx *c, int rank, int world) {
  comm_state_free(c);
  c->comm = new CommState();
  c->comm->rank = rank;
  c->comm->world = world;
  return MGPU_OK;
}

}  // namespace

extern "C" {

int mgpu_comm_unique_id(void *id) {
  if (!id) return MGPU_ERR_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return MGPU_ERR_COMM;
  std::memcpy(id, &u, sizeof u);
  return MGPU_OK;
}

int mgpu_comm_init(mgpu_ctx *c, int rank, int world, const void *id) {
  if (!c) return MGPU_ERR_ARG;
  if (world < 1 || rank < 0 || rank >= world || !id)
    return fail(c, MGPU_ERR_ARG, "mgpu_comm_init: bad rank %d / world %d", rank, world);
  static_assert(sizeof(ncclUniqueId) == MGPU_COMM_ID_BYTES, "RCCL unique id size");
  HIPCHK(c, hipSetDevice(c->device));
  new_state(c, rank, world);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRank(&comm, world, u, rank);
  if (r != ncclSuccess) {
    comm_state_free(c);
    return fail(c, MGPU_ERR_COMM, "mgpu_comm_init: ncclCommInitRank (rank %d of %d): %s", rank,
                world, ncclGetErrorString(r));
  }
  c->comm->nccl = comm;
  return MGPU_OK;
}

int mgpu_comm_init_host(mgpu_ctx *c, int rank, int world, const mgpu_host_transport *t) {
  if (!c) return MGPU_ERR_ARG;
  if (world < 1 || rank < 0 || rank >= world || !t || !t->allreduce || !t->allgather ||
      !t->alltoallv)
    return fail(c, MGPU_ERR_ARG, "mgpu_comm_init_host: bad rank / world / transport");
  new_state(c, rank, world);
  c->comm->host = true;
  c->comm->t = *t;
  return MGPU_OK;
}

int mgpu_comm_info(mgpu_ctx *c, int *rank, int *world) {
  if (!c) return MGPU_ERR_ARG;
  if (rank) *rank = c->comm ? c->comm->rank : 0;
  if (world) *world = c->comm ? c->comm->world : 1;
  return MGPU_OK;
}

int mgpu_allreduce_f64(mgpu_ctx *c, double *v, int count, int op) {
  if (!c) return MGPU_ERR_ARG;
  if (count < 0 || (count > 0 && !v) || op < MGPU_OP_SUM || op > MGPU_OP_MAX)
    return fail(c, MGPU_ERR_ARG, "mgpu_allreduce_f64: bad argument");
  if (count == 0 || solo(c)) return MGPU_OK;
  CommState &s = *c->comm;
  if (s.host) {
    HOSTCHK(c, s.t.allreduce(s.t.user, v, count, op));
    return MGPU_OK;
  }
  const size_t bytes = (size_t)count * 8;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, s.dbuf.ensure(bytes));
  int rc = ensure_pin(c, s, bytes);
  if (rc != MGPU_OK) return rc;
  std::memcpy(s.pin, v, bytes);
  HIPCHK(c, hipMemcpyAsync(s.dbuf.p, s.pin, bytes, hipMemcpyHostToDevice, c->stream));
  NCCLCHK(c, ncclAllReduce(s.dbuf.p, s.dbuf.p, (size_t)count, ncclFloat64, nccl_op(op), s.nccl,
                           c->stream));
  HIPCHK(c, hipMemcpyAsync(s.pin, s.dbuf.p, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::memcpy(v, s.pin, bytes);
  return MGPU_OK;
}

int mgpu_allreduce_min(mgpu_ctx *c, double *v) { return mgpu_allreduce_f64(c, v, 1, MGPU_OP_MIN); }

int mgpu_round_reduce(mgpu_ctx *c, double incumbent, double open, int err, double *out) {
  if (!c) return MGPU_ERR_ARG;
  if (!out) return fail(c, MGPU_ERR_ARG, "mgpu_round_reduce: out is null");
  double t[4] = {incumbent, -open, open, err ? -1.0 : 0.0};
  int rc = mgpu_allreduce_f64(c, t, 4, MGPU_OP_MIN);
  if (rc != MGPU_OK) return rc;
  out[0] = t[0];
  out[1] = -t[1];
  out[2] = t[2];
  out[3] = t[3] < 0.0 ? 1.0 : 0.0;
  return MGPU_OK;
}

int mgpu_allgather_f64(mgpu_ctx *c, const double *send, int count, double *recv) {
  if (!c) return MGPU_ERR_ARG;
  if (count < 0 || (count > 0 && (!send || !recv)))
    return fail(c, MGPU_ERR_ARG, "mgpu_allgather_f64: bad argument");
  if (count == 0) return MGPU_OK;
  if (solo(c)) {
    std::memmove(recv, send, (size_t)count * 8);
    return MGPU_OK;
  }
  CommState &s = *c->comm;
  if (s.host) {
    HOSTCHK(c, s.t.allgather(s.t.user, send, count, recv));
    return MGPU_OK;
  }
  const size_t per = (size_t)count * 8, all = per * (size_t)s.world;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, s.dbuf.ensure(all + per));
  int rc = ensure_pin(c, s, all);
  if (rc != MGPU_OK) return rc;
  char *d = s.dbuf.as<char>();
  std::memcpy(s.pin, send, per);
  HIPCHK(c, hipMemcpyAsync(d + all, s.pin, per, hipMemcpyHostToDevice, c->stream));
  NCCLCHK(c, ncclAllGather(d + all, d, (size_t)count, ncclFloat64, s.nccl, c->stream));
  HIPCHK(c, hipMemcpyAsync(s.pin, d, all, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::memcpy(recv, s.pin, all);
  return MGPU_OK;
}

int mgpu_alltoall_rows_dev(mgpu_ctx *c, int width, const double *d_send,
                           const int32_t *send_counts, double *d_recv,
                           const int32_t *recv_counts) {
  if (!c) return MGPU_ERR_ARG;
  const int P = c->comm ? c->comm->world : 1;
  if (width <= 0 || !send_counts || !recv_counts)
    return fail(c, MGPU_ERR_ARG, "mgpu_alltoall_rows_dev: bad argument");
  long long ns = 0, nr = 0;
  for (int r = 0; r < P; ++r) {
    if (send_counts[r] < 0 || recv_counts[r] < 0)
      return fail(c, MGPU_ERR_ARG, "mgpu_alltoall_rows_dev: negative count");
    ns += send_counts[r];
    nr += recv_counts[r];
  }
  if ((ns > 0 && !d_send) || (nr > 0 && !d_recv))
    return fail(c, MGPU_ERR_ARG, "mgpu_alltoall_rows_dev: null rows");
  const size_t rowb = (size_t)width * 8;
  HIPCHK(c, hipSetDevice(c->device));
  if (solo(c)) {
    if (send_counts[0] != recv_counts[0])
      return fail(c, MGPU_ERR_ARG, "mgpu_alltoall_rows_dev: one rank sends %d rows, receives %d",
                  send_counts[0], recv_counts[0]);
    if (ns > 0 && d_send != d_recv)
      HIPCHK(c, hipMemcpyAsync(d_recv, d_send, (size_t)ns * rowb, hipMemcpyDeviceToDevice,
                               c->stream));
    return MGPU_OK;
  }
  CommState &s = *c->comm;
  if (s.host) {
    std::vector<double> hs((size_t)ns * width), hr((size_t)nr * width);
    if (ns > 0) {
      HIPCHK(c, hipMemcpyAsync(hs.data(), d_send, hs.size() * 8, hipMemcpyDeviceToHost,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    HOSTCHK(c, s.t.alltoallv(s.t.user, hs.data(), send_counts, hr.data(), recv_counts, width));
    if (nr > 0) {
      HIPCHK(c, hipMemcpyAsync(d_recv, hr.data(), hr.size() * 8, hipMemcpyHostToDevice,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));   // hr is pageable and goes out of scope
    }
    return MGPU_OK;
  }
  size_t so = 0, ro = 0;
  NCCLCHK(c, ncclGroupStart());
  for (int r = 0; r < P; ++r) {
    if (send_counts[r] > 0)
      NCCLCHK(c, ncclSend(d_send + so, (size_t)send_counts[r] * width, ncclFloat64, r, s.nccl,
                          c->stream));
    if (recv_counts[r] > 0)
      NCCLCHK(c, ncclRecv(d_recv + ro, (size_t)recv_counts[r] * width, ncclFloat64, r, s.nccl,
                          c->stream));
    so += (size_t)send_counts[r] * width;
    ro += (size_t)recv_counts[r] * width;
  }
  NCCLCHK(c, ncclGroupEnd());
  return MGPU_OK;
}

int mgpu_lb_deal(int world, int S, const double *lbs, int32_t *owner, int32_t *local,
                 int32_t *recv) {
  if (world < 1 || S < 0 || (S > 0 && (!lbs || !owner || !local || !recv))) return MGPU_ERR_ARG;
  const int tot = world * S;
  std::vector<int32_t> ord((size_t)tot);
  for (int i = 0; i < tot; ++i) ord[(size_t)i] = i;
  // ascending bound, ties in rank-major order (a stable sort)
  std::stable_sort(ord.begin(), ord.end(),
                   [lbs](int32_t a, int32_t b) { return lbs[a] < lbs[b]; });
  int nd = 0;
  for (; nd < tot; ++nd) {
    const int32_t i = ord[(size_t)nd];
    if (lbs[i] == INFINITY) break;   // :137-148: the deal stops at the padding
    owner[nd] = i / S;
    local[nd] = i % S;
    recv[nd] = nd % world;
  }
  return nd;
}

int mgpu_bnb_rebalance(mgpu_ctx *c, int S, double *picked, int *npicked, double *received,
                       int *nreceived, long long *moved, int *open_after) {
  if (!c) return MGPU_ERR_ARG;
  if (S < 1) return fail(c, MGPU_ERR_ARG, "mgpu_bnb_rebalance: S = %d", S);
  const int P = c->comm ? c->comm->world : 1, me = c->comm ? c->comm->rank : 0;
  // 1. this rank's next S candidates (TreeManager::getCandidate, :93-105)
  std::vector<double> vec((size_t)S + 1, INFINITY);
  int k = 0, open = 0, spare = 0;
  int rc = mgpu_bnb_pick(c, S, vec.data(), &k);
  if (rc != MGPU_OK) return rc;
  rc = mgpu_bnb_count(c, &open, &spare);
  if (rc != MGPU_OK) return rc;
  if (picked) std::memcpy(picked, vec.data(), (size_t)k * 8);
  if (npicked) *npicked = k;
  if (P == 1) {   // solo: the deal keeps every node where it is
    if (nreceived) *nreceived = 0;
    if (moved) *moved = 0;
    if (open_after) *open_after = open;
    return MGPU_OK;
  }
  vec[(size_t)S] = (double)spare;
  // every workspace of this exchange at its worst case for S (this rank
  // sends at most the S nodes it picked and, dealt round-robin, receives at
  // most S): sized by the first rebalance, never again for the same S
  const int W = mgpu_bnb_row_width(c);
  if (W < 0) return W;
  {
    CommState &s = *c->comm;   // P > 1: a communicator is set
    const size_t rowb = (size_t)W * 8, gat = (size_t)P * (S + 1) * 8;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, s.send_rows.ensure((size_t)S * rowb));
    HIPCHK(c, s.recv_rows.ensure((size_t)S * rowb));
    HIPCHK(c, s.ord_rows.ensure((size_t)S * rowb));
    HIPCHK(c, s.perm.ensure((size_t)S * 4));
    if (!s.host) {
      HIPCHK(c, s.dbuf.ensure(gat + (size_t)(S + 1) * 8));
      rc = ensure_pin(c, s, gat);
      if (rc != MGPU_OK) return rc;
    }
    rc = bnb_reserve_migration(c, S);
    if (rc != MGPU_OK) return rc;
  }
  // 2. one all-gather of the bounds and the pool room (:107)
  std::vector<double> g((size_t)P * (S + 1));
  rc = mgpu_allgather_f64(c, vec.data(), S + 1, g.data());
  if (rc != MGPU_OK) return rc;
  std::vector<double> lbs((size_t)P * S);
  for (int r = 0; r < P; ++r)
    std::memcpy(lbs.data() + (size_t)r * S, g.data() + (size_t)r * (S + 1), (size_t)S * 8);
  // 3. the common deal (:111-188)
  std::vector<int32_t> owner((size_t)P * S), local((size_t)P * S), recv((size_t)P * S);
  const int nd = mgpu_lb_deal(P, S, lbs.data(), owner.data(), local.data(), recv.data());
  std::vector<long long> gain((size_t)P, 0);
  long long nmoved = 0;
  for (int i = 0; i < nd; ++i)
    if (owner[i] != recv[i]) {
      ++gain[(size_t)recv[i]];
      --gain[(size_t)owner[i]];
      ++nmoved;
    }
  // 4. a deal that would overflow some pool fails on every rank (same data)
  for (int r = 0; r < P; ++r)
    if ((double)gain[(size_t)r] > g[(size_t)r * (S + 1) + S])
      return fail(c, MGPU_ERR_STATE, "mgpu_bnb_rebalance: the deal would overflow rank %d's pool "
                  "(gain %lld, room %.0f)", r, gain[(size_t)r], g[(size_t)r * (S + 1) + S]);
  // 5. the rows this rank sends, grouped by receiver in deal order; the rows it
  // receives, in deal order, and where each one lands in the exchange buffer
  std::vector<int32_t> sc((size_t)P, 0), rcnt((size_t)P, 0), idx;
  std::vector<int> send_at;
  for (int i = 0; i < nd; ++i)
    if (owner[i] == me && recv[i] != me) send_at.push_back(i);
  std::stable_sort(send_at.begin(), send_at.end(),
                   [&](int a, int b) { return recv[a] < recv[b]; });
  for (int i : send_at) {
    idx.push_back(local[i]);
    ++sc[(size_t)recv[i]];
  }
  std::vector<int> got_at;
  for (int i = 0; i < nd; ++i)
    if (recv[i] == me && owner[i] != me) {
      got_at.push_back(i);
      ++rcnt[(size_t)owner[i]];
    }
  std::vector<int32_t> off((size_t)P, 0), perm;
  for (int r = 1; r < P; ++r) off[(size_t)r] = off[(size_t)r - 1] + rcnt[(size_t)r - 1];
  for (int i : got_at) perm.push_back(off[(size_t)owner[i]]++);
  if (received)
    for (size_t j = 0; j < got_at.size(); ++j) {
      const int i = got_at[j];
      received[j] = lbs[(size_t)owner[i] * S + local[i]];
    }
  if (nreceived) *nreceived = (int)got_at.size();
  CommState &s = *c->comm;
  const size_t rowb = (size_t)W * 8;
  const int ks = (int)idx.size(), kr = (int)got_at.size();
  if (ks > S || kr > S)   // the deal hands each rank at most S nodes
    return fail(c, MGPU_ERR_STATE, "mgpu_bnb_rebalance: %d sent / %d received > S = %d", ks, kr, S);
  rc = mgpu_bnb_export_dev(c, ks, ks ? idx.data() : nullptr, s.send_rows.as<double>());
  if (rc != MGPU_OK) return rc;
  rc = mgpu_alltoall_rows_dev(c, W, s.send_rows.as<double>(), sc.data(), s.recv_rows.as<double>(),
                              rcnt.data());
  if (rc != MGPU_OK) return rc;
  if (kr > 0) {
    HIPCHK(c, hipMemcpyAsync(s.perm.p, perm.data(), (size_t)kr * 4, hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, launch_bnb_gather_rows(s.recv_rows.as<unsigned char>(), s.ord_rows.as<unsigned char>(),
                                     rowb, s.perm.as<int32_t>(), kr, c->stream));
    rc = mgpu_bnb_import_dev(c, kr, s.ord_rows.as<double>());
    if (rc != MGPU_OK) return rc;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));   // perm is pageable and goes out of scope
  if (moved) *moved = nmoved;
  if (open_after) *open_after = open - ks + kr;
  return MGPU_OK;
}

}  // extern "C"
