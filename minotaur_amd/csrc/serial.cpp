// Open nodes in Minotaur's Serializer wire format (host only, no device
// work): the format MpiBranchAndBound sends nodes in (src/base/
// Serializer.cpp:26-112, DeSerializer :130-191), so a node exported from the
// batched pool (mgpu_bnb_export) can travel to a reference rank, or be
// checkpointed as a list the reference's DeSerializer reads, and back.
//
// A node is written as
//   [UInt id][double lb][size_t k] then k x [int var][short lu][double old][double new]
// packed (each field written with its own size, Serializer::writeArith), in
// the host's byte order, the k entries ascending by (var, lu): writeMods
// merges the relaxation modifications of the node's whole path into a
// std::map keyed by (variable index, BoundType) that keeps the FIRST old and
// the LAST new value of each key.  The batched pool keeps the node's box, not
// its path: the box differs from the root's box exactly in those merged
// bounds (old = the root's bound, new = the node's), so the entries are the
// bounds that differ, lower (BoundType Lower = 0) before upper (Upper = 1).
#include <cstring>

#include "mgpu.h"

namespace {

template <typename T>
void put(uint8_t *out, size_t &at, T v) {
  if (out) std::memcpy(out + at, &v, sizeof(T));
  at += sizeof(T);
}

template <typename T>
bool get(const uint8_t *buf, size_t len, size_t &at, T *v) {
  if (at + sizeof(T) > len) return false;
  std::memcpy(v, buf + at, sizeof(T));
  at += sizeof(T);
  return true;
}

}  // namespace

extern "C" {

int mgpu_node_serialize(uint32_t id, double lb, int n, const double *root_lb,
                        const double *root_ub, const double *lb_box, const double *ub_box,
                        uint8_t *out, size_t cap, size_t *len) {
  if (n < 0 || !root_lb || !root_ub || !lb_box || !ub_box || !len) return MGPU_ERR_ARG;
  size_t k = 0;
  for (int j = 0; j < n; ++j) k += (lb_box[j] != root_lb[j]) + (ub_box[j] != root_ub[j]);
  const size_t need = sizeof(uint32_t) + sizeof(double) + sizeof(size_t) +
                      k * (sizeof(int) + sizeof(short) + 2 * sizeof(double));
  *len = need;
  if (!out) return MGPU_OK;
  if (cap < need) return MGPU_ERR_ARG;
  size_t at = 0;
  put<uint32_t>(out, at, id);
  put<double>(out, at, lb);
  put<size_t>(out, at, k);
  for (int j = 0; j < n; ++j) {
    if (lb_box[j] != root_lb[j]) {
      put<int>(out, at, j);
      put<short>(out, at, 0);
      put<double>(out, at, root_lb[j]);
      put<double>(out, at, lb_box[j]);
    }
    if (ub_box[j] != root_ub[j]) {
      put<int>(out, at, j);
      put<short>(out, at, 1);
      put<double>(out, at, root_ub[j]);
      put<double>(out, at, ub_box[j]);
    }
  }
  return MGPU_OK;
}

int mgpu_node_deserialize(const uint8_t *buf, size_t len, int n, const double *root_lb,
                          const double *root_ub, uint32_t *id, double *lb, double *lb_box,
                          double *ub_box, size_t *used) {
  if (!buf || n < 0 || !root_lb || !root_ub || !id || !lb || !lb_box || !ub_box || !used)
    return MGPU_ERR_ARG;
  size_t at = 0, k = 0;
  if (!get(buf, len, at, id) || !get(buf, len, at, lb) || !get(buf, len, at, &k))
    return MGPU_ERR_ARG;
  std::memcpy(lb_box, root_lb, sizeof(double) * (size_t)n);
  std::memcpy(ub_box, root_ub, sizeof(double) * (size_t)n);
  for (size_t e = 0; e < k; ++e) {
    int var = 0;
    short lu = 0;
    double oldv = 0.0, newv = 0.0;
    if (!get(buf, len, at, &var) || !get(buf, len, at, &lu) || !get(buf, len, at, &oldv) ||
        !get(buf, len, at, &newv))
      return MGPU_ERR_ARG;
    if (var < 0 || var >= n || (lu != 0 && lu != 1)) return MGPU_ERR_ARG;
    // DeSerializer::readVarBoundMod: the new value is the node's bound
    (lu == 0 ? lb_box : ub_box)[var] = newv;
  }
  *used = at;
  return MGPU_OK;
}

}  // extern "C"
