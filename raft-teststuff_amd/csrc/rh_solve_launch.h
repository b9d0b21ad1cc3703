// rh_solve_launch.h -- host launchers of the k_solve_lds instantiations compiled in
// rh_solve_fast.hip (its own translation unit and scheduler flags); called by rh_abi.hip.
#pragma once
#include "rh_common.h"

namespace rh {

enum SolveFast {
  kSolve1x128 = 0,   // k_solve_lds<1, 128, true>: nw <= 128, four cases per CU
  kSolve2x128 = 1,   // k_solve_lds<2, 128, true>: 128 < nw <= 256 (C4)
  kSolve1x256 = 2,   // k_solve_lds<1, 256>: nw <= 256 with the per-node B_drag image
  kSolve1x512 = 3,   // k_solve_lds<1, 512>: nw <= 512
  kSolve2x512 = 4,   // k_solve_lds<2, 512>: 512 < nw <= 1024 (C2)
};

hipError_t launch_solve_fast(int which, dim3 grid, dim3 block, size_t lsm, hipStream_t s, const CaseArgs& a);
hipError_t occupancy_solve_fast(int which, int* per_cu, int threads, size_t lsm);

}  // namespace rh
