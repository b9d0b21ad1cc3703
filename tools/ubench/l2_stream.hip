// l2_stream.hip -- the kproj stream of k_solve_lds with (almost) no arithmetic: what rate does
// the L2 -> CU path give this exact access pattern on gfx950?
//
// Same geometry as the C2 bench launch: 512 workgroups ("cases") of 512 threads, one per CU
// (a dynamic LDS allocation of 100 KB, as XiLast's 96 KB), case -> heading as the bench's
// design-major order, 4 headings x 53 nodes x 3 projections x 1000 bins of 16 B (2.5 MB per
// heading, L2-resident per XCD).  Each pass streams one heading table once per case, lane =
// bin (2 bins per thread), buffer loads with a 32-bit lane offset, as phases A and C do.
//   build: hipcc -O3 --offload-arch=gfx950 -I../../raft-teststuff_amd/csrc l2_stream.hip -o l2_stream
//   run:   ./l2_stream            (prints GB/s chip-wide and per CU for each variant)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "rh_device.h"

using namespace rh;

constexpr int kNW = 1000, kNN = 53, kHead = 4, kLT = 512;

// RING nodes in flight; BOTH: the two bins of a thread per node (phase A) or one bin per
// sweep (phase C, two sweeps per pass).
template <int RING, bool BOTH>
__global__ __launch_bounds__(kLT, 1) void k_stream(const rh_c128* tab, int ncase, int passes, double* out) {
  extern __shared__ double smem[];
  const int tid = threadIdx.x;
  const int ic = xcd_remap(blockIdx.x, ncase);
  const int head = ic * kHead / ncase;
  const unsigned nw16 = kNW * 16u;
  const Buf bK = mkbuf(tab + (size_t)head * kNN * 3 * kNW, (unsigned)kNN * 3u * nw16);
  auto voff = [&](int b) { return (unsigned)(b < kNW ? b : kNW - 1) * 16u; };
  double acc = 0.0;
  for (int p = 0; p < passes; ++p) {
    if (BOTH) {
      const unsigned v0 = voff(tid), v1 = voff(tid + kLT);
      for (int n = 0; n < kNN; n += RING) {
        cd K[RING][3][2];
#pragma unroll
        for (int r = 0; r < RING; ++r) {
          const unsigned so = (unsigned)(n + r < kNN ? n + r : kNN - 1) * 3u * nw16;
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            K[r][q][0] = bld(bK, v0, so + q * nw16);
            K[r][q][1] = bld(bK, v1, so + q * nw16);
          }
        }
#pragma unroll
        for (int r = 0; r < RING; ++r)
#pragma unroll
          for (int q = 0; q < 3; ++q) acc += (K[r][q][0].r + K[r][q][0].i) + (K[r][q][1].r + K[r][q][1].i);
      }
    } else {
#pragma unroll 1
      for (int j = 0; j < 2; ++j) {
        const unsigned v = voff(tid + kLT * j);
        for (int n = 0; n < kNN; n += RING) {
          cd K[RING][3];
#pragma unroll
          for (int r = 0; r < RING; ++r) {
            const unsigned so = (unsigned)(n + r < kNN ? n + r : kNN - 1) * 3u * nw16;
#pragma unroll
            for (int q = 0; q < 3; ++q) K[r][q] = bld(bK, v, so + q * nw16);
          }
#pragma unroll
          for (int r = 0; r < RING; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) acc += K[r][q].r + K[r][q].i;
        }
      }
    }
  }
  smem[tid] = acc;
  __syncthreads();
  if (tid == 0) {
    double s = 0;
    for (int i = 0; i < kLT; ++i) s += smem[i];
    out[blockIdx.x] = s;
  }
}

template <int RING, bool BOTH>
static void run(const char* name, const rh_c128* tab, double* out, int ncase, int passes) {
  const size_t lds = 100 * 1024;
  hipFuncSetAttribute((const void*)k_stream<RING, BOTH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_stream<RING, BOTH>), dim3(ncase), dim3(kLT), lds, 0, tab, ncase, passes, out);
  const int reps = 10;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_stream<RING, BOTH>), dim3(ncase), dim3(kLT), lds, 0, tab, ncase, passes, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  // bytes the lanes request (pad lanes re-read the clamped last bin, as in the solve kernel)
  const double bytes = (double)ncase * passes * kNN * 3 * (2.0 * kLT) * 16;
  const double useful = (double)ncase * passes * kNN * 3 * (double)kNW * 16;
  printf("%-22s passes %2d: %.4f ms  requested %.2f TB/s (%.1f GB/s per CU)  useful %.2f TB/s\n", name, passes, ms,
         bytes / ms * 1e-9, bytes / ms * 1e-6 / 256, useful / ms * 1e-9);
}

int main() {
  const size_t n = (size_t)kHead * kNN * 3 * kNW;
  std::vector<rh_c128> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = rh_c128{1e-3 * (double)(i % 977), 1e-3 * (double)(i % 131)};
  rh_c128* tab;
  double* out;
  hipMalloc(&tab, n * sizeof(rh_c128));
  hipMalloc(&out, 4096 * sizeof(double));
  hipMemcpy(tab, h.data(), n * sizeof(rh_c128), hipMemcpyHostToDevice);
  const int ncase = 512;
  for (int passes : {9}) {
    run<3, true>("A-shape ring3", tab, out, ncase, passes);
    run<6, true>("A-shape ring6", tab, out, ncase, passes);
    run<6, false>("C-shape ring6", tab, out, ncase, passes);
    run<12, false>("C-shape ring12", tab, out, ncase, passes);
  }
  hipFree(tab);
  hipFree(out);
  return 0;
}
