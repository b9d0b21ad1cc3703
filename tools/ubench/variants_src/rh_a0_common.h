// rh_a0_common.h -- the constants and Xi_last layout of k_a0_sums (rh_a0.hip) that k_solve_lds
// reads in variant builds (-DRH_VARIANTS; rh_set_a0).  Not part of the shipped library.
#pragma once
#include "../../../raft-teststuff_amd/csrc/rh_common.h"

namespace rh {

#ifndef RH_A0_ABL
#define RH_A0_ABL 0   // timing ablations (tools/ubench variants): 1 no spectrum, 4 no MFMA
#endif
constexpr int kA0Cases = 16;       // cases per tile (MFMA rows)
constexpr int kA0Bins = 64;        // bins per chunk (16 MFMA steps of 4 bins)
constexpr int kA0Threads = 512;    // 8 waves, each taking 16-row blocks of the node projections
constexpr int kA0Pad = kA0Bins + 2;
constexpr int kRowP = kA0Bins + 1;          // padded staged row (complex)
constexpr int kRbLd = 16 * kA0Bins / 64;    // loads per lane per row block (one row x 64 bins each)

constexpr int kA0Cpb = 2;          // bin chunks per workgroup (setup and beta shared)

__host__ __device__ inline int a0_chunks(int nw) { return (nw + kA0Bins - 1) / kA0Bins; }
// dynamic LDS: beta [3 nn], node t [nn], member factors [18][nm], member ranges [nm + 1] (int)
__host__ __device__ inline size_t a0_smem(int nn_max, int nm_max) {
  const size_t nn = nn_max > 0 ? nn_max : 1, nm = nm_max > 0 ? nm_max : 1;
  return sizeof(double) * (4 * nn + 18 * nm) + sizeof(int) * (nm + 1);
}
// static LDS of k_a0_sums (su, sv, the wave stages, the tile's case keys)
constexpr size_t kA0StaticLds = sizeof(double) * 2 * kA0Cases * kA0Pad + 16 * (kA0Threads / 64) * 16 * kRowP +
                                sizeof(int) * 3 * kA0Cases;
// the A(0) sums of a case fit in its Xi_last block ([6][nw] complex = 12 nw doubles)
__host__ __device__ inline bool a0_fits(int nw, int nn) { return (size_t)a0_chunks(nw) * 3 * nn <= (size_t)12 * nw; }
__device__ __forceinline__ double* a0_block(const CaseArgs& a, int ic, int nw) {
  return reinterpret_cast<double*>(a.o.Xi_last + (size_t)ic * 6 * nw);
}

}  // namespace rh
