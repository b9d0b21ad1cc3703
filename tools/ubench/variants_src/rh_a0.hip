// rh_a0.hip -- k_a0_sums: phase A of the first drag iteration of a whole batch, as FP64 MFMA GEMMs.
//
// A case that starts from XiStart (no Xi_init, first_iter 0) enters iteration 0 with
// XiLast = XiStart in every DOF and bin (raft/raft_model.py:882).  Its body-motion terms in the
// phase-A sums of k_solve_lds (rh_solve.hip; raft/raft_fowt.py:1205-1211) are then the same for
// every case of a design: per node n and projection p (row j = 3 n + p) the relative velocity is
//     s_j(b) = z_b K_j(b) - i w_b beta_j,
//     beta_q = XiStart sum_c cq_c,  beta_1 = XiStart (sum_c c1_c + t sum_{c<3} c2_c),
//     beta_2 = XiStart (sum_c c2_c - t sum_{c<3} c1_c)
// (cq, c1, c2 the member factors of the node's member, t its axial coordinate), and
//     sum_b |s_j(b)|^2 = sum_b z_b^2 |K_j(b)|^2 - 2 beta_j sum_b z_b w_b Im K_j(b) + beta_j^2 sum_b w_b^2.
// The first two sums are, for the cases of one (design, heading), the product of a
// [case x bin] matrix (z^2 | z w) with a [bin x row] matrix (|K|^2 | -2 beta Im K): a GEMM that
// reads each wave-table entry once per 16 cases instead of once per case.  k_solve_lds then
// skips phase A of iteration 0 and takes these sums in phase B.  The bin sums are grouped
// differently from phase A's per-lane / butterfly order, so the two agree to rounding (the
// three terms have no cancellation to speak of: the XiStart motion term dominates most rows,
// and z^2 |K|^2 rows with beta = 0 are sums of squares).
//
// Launch: grid (ceil(ncase / 16) case tiles of the launch order, ceil(nw / 128) pairs of 64-bin chunks),
// 512 threads.  A tile's cases are handled one (design, heading) key at a time (a sorted launch
// order gives one or two keys per tile); each wave takes 16-row blocks of the key's 3 nn rows.
// Per (case, chunk) the row sums go to the case's Xi_last scratch, which the fast path does not
// otherwise use: [chunk][3 nn] doubles at the start of the case's [6][nw] complex block.
#include "rh_a0_common.h"

namespace rh {

typedef double a0d4 __attribute__((ext_vector_type(4)));

// Data flow of a workgroup (latency-bound, so loads are issued early and dependent global
// loads are avoided): the design's node axial coordinates, member factors and member ranges are
// staged in LDS with one round of loads, and beta_j of every row is formed from there (a member
// search over global memory would be a chain of dependent loads per row).  Each wave issues the
// loads of its first 16-row block (one row x 64 bins = 1 KB per load) before the workgroup
// computes the chunk's wave amplitudes; a row block then goes through the wave's LDS stage (the
// MFMA B fragment is 16 rows x 4 bins, which straight from the [row][bin] table would be 16
// scattered 64-byte pieces per load) while the wave's next row block is in flight.  A workgroup
// takes kA0Cpb chunks, so the set-up and beta serve both.
__global__ __launch_bounds__(kA0Threads) void k_a0_sums(CaseArgs a) {
  __shared__ double su[kA0Cases][kA0Pad];   // z^2 of (case, bin of the chunk)
  __shared__ double sv[kA0Cases][kA0Pad];   // z w
  __shared__ double2 stage[kA0Threads / 64][16 * kRowP];   // per wave: one 16-row block of kproj
  extern __shared__ __attribute__((aligned(16))) double dsm[];
  __shared__ int kic[kA0Cases], kd[kA0Cases], kh[kA0Cases];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = blockIdx.x;
  const int ncase = a.c.ncase;
  if (tid < kA0Cases) {
    const int slot = tile * kA0Cases + tid;
    const int ic = slot < ncase ? (a.c.order ? a.c.order[slot] : slot) : -1;
    kic[tid] = ic;
    kd[tid] = ic >= 0 ? a.c.design[ic] : -1;
    kh[tid] = ic >= 0 ? a.c.head[ic] : -1;
  }
  __syncthreads();
  int beta_for = -1;   // design whose beta is in sbeta (the same value in every thread: uniform control)
  const int nw = a.designs[kd[0]].d.nw;   // slot tile*16 < ncase; every design of a launch shares nw
  const unsigned nw16 = (unsigned)nw * 16u;
  const int nch = a0_chunks(nw);
  const int mr = lane & 15, kr = lane >> 4;
  const double xs = a.c.XiStart;
  double2* stg = stage[wv];
#pragma unroll 1
  for (int cc = 0; cc < kA0Cpb; ++cc) {
    const int chunk = blockIdx.y * kA0Cpb + cc;
    if (chunk >= nch) break;   // uniform
    const int b0 = chunk * kA0Bins;
    bool amplitudes = false;
    unsigned done = 0;
    for (;;) {   // one (design, heading) key of the tile at a time (block-uniform)
      int first = -1;
      for (int c = 0; c < kA0Cases; ++c)
        if (kic[c] >= 0 && !((done >> c) & 1u)) {
          first = c;
          break;
        }
      if (first < 0) break;
      const int kdes = kd[first], khead = kh[first];
      unsigned match = 0;
      for (int c = 0; c < kA0Cases; ++c)
        if (kic[c] >= 0 && kd[c] == kdes && kh[c] == khead) match |= 1u << c;
      done |= match;
      const rh_design& d = a.designs[kdes].d;
      const int nn = d.nn, nm = d.nm, nrow = 3 * nn, nrb = (nrow + 15) / 16;
      if (nn == 0) continue;
      const Buf bK = mkbuf(d.kproj + (size_t)khead * nrow * nw, (unsigned)nrow * nw16);
      cd L[kRbLd];
      auto load_rb = [&](int rb) {
#pragma unroll
        for (int i = 0; i < kRbLd; ++i) {
          const int row = rb * 16 + i;
          L[i] = bld(bK, (unsigned)(b0 + lane) * 16u, (unsigned)(row < nrow ? row : nrow - 1) * nw16);
        }
      };
      int rb = wv;
      if (rb < nrb) load_rb(rb);
      const double wl = b0 + lane < nw ? d.w[b0 + lane] : 0.0;
      double* sbeta = dsm;                 // [3 nn]
      double* st = sbeta + 3 * nn;         // [nn]
      double* smf = st + nn;               // [18][nm]
      int* sms = reinterpret_cast<int*>(smf + 18 * nm);   // [nm + 1]
      const bool need_beta = beta_for != kdes;   // uniform
      if (need_beta) {
        __syncthreads();   // the previous key's rows have read sbeta
        for (int n = tid; n < nn; n += kA0Threads) st[n] = d.node[RH_NF_T * nn + n];
        for (int e = tid; e < 18 * nm; e += kA0Threads) smf[e] = d.memb[e];   // fields 0..17 = cq, c1, c2
        for (int e = tid; e <= nm; e += kA0Threads) sms[e] = d.mstart[e];
      }
      if (!amplitudes) {   // the tile's wave amplitudes over the chunk (sea_amplitude, as the solve's prologue)
        amplitudes = true;
        for (int e = tid; e < kA0Cases * kA0Bins; e += kA0Threads) {
          const int c = e / kA0Bins, bl = e % kA0Bins, b = b0 + bl;
          const int ic = kic[c];
          double zz = 0.0, w = 0.0;
          if (ic >= 0 && b < nw) {
            const rh_design& dc = a.designs[kd[c]].d;
            w = dc.w[b];
#if RH_A0_ABL & 1   // timing ablation: no spectrum (wrong results)
            zz = a.c.Hs[ic];
#else
            zz = sea_amplitude(a.c.spectrum[ic], a.c.Hs[ic], a.c.Tp[ic], a.c.gamma[ic], w, dc.dw);
#endif
          }
          su[c][bl] = zz * zz;
          sv[c][bl] = zz * w;
        }
      }
      __syncthreads();   // amplitudes and the staged design tables in LDS
      if (need_beta) {
        // beta_j / XiStart: the member factors of the row's member summed over the six DOFs
        // (XiLast = XiStart (1, ..., 1)), plus t times the rotation part for the two transverse
        // projections (header comment)
        for (int j = tid; j < nrow; j += kA0Threads) {
          const int n = j / 3, p = j - 3 * n;
          int m = 0;
          while (m + 1 < nm && sms[m + 1] <= n) ++m;
          double sq = 0, s1 = 0, s2 = 0, d1 = 0, d2 = 0;
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            const double cq = smf[(RH_MF_CQ0 + c) * nm + m], c1 = smf[(RH_MF_C10 + c) * nm + m],
                         c2 = smf[(RH_MF_C20 + c) * nm + m];
            sq += cq;
            s1 += c1;
            s2 += c2;
            if (c < 3) {
              d1 += c2;
              d2 += c1;
            }
          }
          const double t = st[n];
          sbeta[j] = xs * (p == 0 ? sq : p == 1 ? s1 + t * d1 : s2 - t * d2);
        }
        __syncthreads();
        beta_for = kdes;
      }
      const bool mine = ((match >> mr) & 1u) != 0;   // A row mr belongs to this key
      const double W2 = wave_sum(wl * wl);            // this design's sum of w^2 over the chunk
      for (; rb < nrb; rb += kA0Threads / 64) {
#pragma unroll
        for (int i = 0; i < kRbLd; ++i) stg[i * kRowP + lane] = make_double2(L[i].r, L[i].i);
        if (rb + kA0Threads / 64 < nrb) load_rb(rb + kA0Threads / 64);
        const int j = rb * 16 + mr;                    // this lane's row (B column mr)
        const double beta = sbeta[j < nrow ? j : nrow - 1];
        const double m2b = -2.0 * beta;
        a0d4 accu = {0.0, 0.0, 0.0, 0.0}, accv = accu;   // two independent MFMA chains
#pragma unroll
        for (int u = 0; u < kA0Bins / 4; ++u) {
          const double2 K = stg[mr * kRowP + 4 * u + kr];
          const int bl = 4 * u + kr;
#if RH_A0_ABL & 4   // timing ablation: staged operands consumed by one add each, no MFMA (wrong results)
          accu[0] += K.x + K.y;
#else
          const double ua = mine ? su[mr][bl] : 0.0, va = mine ? sv[mr][bl] : 0.0;
          accu = __builtin_amdgcn_mfma_f64_16x16x4f64(ua, K.x * K.x + K.y * K.y, accu, 0, 0, 0);
          accv = __builtin_amdgcn_mfma_f64_16x16x4f64(va, m2b * K.y, accv, 0, 0, 0);
#endif
        }
        // C[i][j]: lane holds rows i = kr + 4 r (cases) of column j = mr (rows of the table)
        if (j < nrow) {
          const double cst = beta * beta * W2;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = kr + 4 * r;
            if ((match >> i) & 1u) a0_block(a, kic[i], nw)[(size_t)chunk * nrow + j] = (accu[r] + accv[r]) + cst;
          }
        }
      }
    }
    __syncthreads();   // this chunk's rows have read su / sv and their stages
  }
}

}  // namespace rh
