// Internal device-side data layout of the engine (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mgpu {

// Tolerances of LinearHandler (LinearHandler.cpp:56-58): intTol_, eTol_,
// infty_.  Bit-identical constants in every kernel.
constexpr double kIntTol = 1e-6;
constexpr double kETol = 1e-8;
constexpr double kInfty = 1e20;

// Reference VariableType numerics (Types.h:83-89).
constexpr int kBinary = 0;
constexpr int kInteger = 1;

// One row term: coefficient + column, packed to 16 B so a wave-uniform term
// is one scalar dwordx4 load.
struct alignas(16) Term {
  double a;
  int32_t j;
  int32_t pad;
};

// Wave-uniform row/term records for the FBBT kernel.  A wave loads up to 64
// of them with ONE coalesced vector load (lane t holds record t) and
// broadcasts record k with v_readlane into SGPRs: no scalar-memory loads in
// the inner loops (SMEM and LDS share lgkmcnt, so mixing them serialises).
struct alignas(16) RowRec {   // 32 B
  double lo, hi;              // row bounds
  int32_t k0, nt;             // first term, term count
  int32_t pad0, pad1;
};
struct alignas(16) TermRec {  // 32 B
  double a;                   // coefficient (0 for the integer-column list)
  uint64_t cmask;             // rows holding column j (bitmask, m <= 64)
  int32_t j;                  // column
  int32_t cs, ce;             // CSC range of column j (m > 64)
  int32_t isint;              // column is Binary/Integer
};

// Batch-shared linear relaxation, resident in HBM after mgpu_load_lp.
struct DevLP {
  int n, m, nnz, nobj;
  int cons_bad;                 // checkBounds_ row test (LinearHandler.cpp:350-357)
  const int32_t *rowptr;        // [m+1]
  const Term *terms;            // [nnz] row-major, columns ascending
  const double *rlo, *rhi;      // [m]
  const int32_t *colptr;        // [n+1]  column -> rows (changeBFlag_)
  const int32_t *rowidx;        // [nnz]
  const uint8_t *vtype;         // [n]
  const Term *obj;              // [nobj] nonzero objective terms, ascending
  const double *collb, *colub;  // [n] root box
  const double *objd;           // [n] dense objective
  double objoff;
  const RowRec *rows;           // [m]
  const TermRec *trec;          // [nnz] row terms
  const TermRec *orec;          // [nobj] objective terms
  const TermRec *irec;          // [nint] integer columns (tightenInts_)
  int nint;
};

// Output/optional mod-log arguments of one FBBT launch.
struct FbbtIO {
  const double *lb_in, *ub_in;  // [B][n]
  double *lb_out, *ub_out;      // [B][n]
  int32_t *infeas, *nmods;      // [B]
  int32_t *mod_var, *mod_lu;    // [B][mod_cap] or null
  double *mod_val;
  int mod_cap;
  int batch;
  int has_inc;
  double inc_ub;                // incumbent - objective constant
  double *scratch;              // global-bounds variant: [waves][2][n][kLanes]
  uint8_t *flag_scratch;        // global-bounds variant: [waves][m][kLanes]
};

constexpr int kLanes = 64;      // wave64: one node per lane
constexpr int kLdsStride = 65;  // padded [var][lane] stride (bank spread)

hipError_t launch_fbbt_linear(const DevLP &lp, const FbbtIO &io, int variant,
                              hipStream_t stream);
size_t fbbt_lds_bytes(int n, int m);

}  // namespace mgpu
