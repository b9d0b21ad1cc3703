// rh_solve_grp.hip -- k_solve_grp<CG>: the drag fixed point of CG sea-state cases that share
// one (design, heading) in one workgroup, so that every wave-table load serves CG cases.
//
// Same algorithm as k_solve_lds (rh_solve.hip; raft/raft_model.py:918-1000,
// raft/raft_fowt.py:1152-1293).  What changes is the data flow:
//   * k_solve_lds is bound by the L2 -> CU stream of the projected wave table kproj: every
//     case reads its heading's 2.5 MB table twice per drag iteration (phases A and C), with
//     ~0.5 FLOP per byte.  Here the CG cases of a group walk the same nodes
//     and bins in lock-step, so one load feeds CG cases' arithmetic.
//   * XiLast of CG cases (CG x 96 KB at nw = 1000) no longer fits in LDS: it lives in the
//     caller's Xi_last scratch, read and written only by the thread that owns the bin.
//   * Bins are processed in passes of 512 (lane = bin): phase A keeps per pass the 6-DOF
//     iterate and the member motion terms of every case in registers, so the node sums are
//     reduced over the wave once per pass (transposing butterfly over the 3 CG values).
//   * Cases converge at different iterations.  A finished case keeps its state (B_drag,
//     Bmat, Xi of its last iteration); its slot still rides along in the shared node loops
//     (that work is discarded) but skips phase B, the LU solve and every store.
// Per case the arithmetic is that of k_solve_lds except the order of the bin sums of
// phase A (pass-wise), so the two kernels agree to rounding, with identical iteration
// counts on the parity cases (tests/test_gpu_parity.py).
#include "../../../raft-teststuff_amd/csrc/rh_device.h"

namespace rh {

constexpr int kGT = 512;          // threads per group workgroup; lane = bin
constexpr int kGW = kGT / 64;     // waves
constexpr int kGRingA = 4;        // wave-table prefetch depth (nodes), phase A
constexpr int kGRingC = 4;        // ... phase C

// Transposing butterfly over 8 values: after three exchange stages (partners i^1, i^2, i^7,
// flags f0 = b0^b2, f1 = b1^b2, f2 = b2 of i = lane & 15) each lane holds the 8-lane sum of
// one value; lane i^8 holds the same value, so row_ror:8 and the two cross-row shuffles
// complete the wave total.  Lane i (< 8) ends with value tbfly8_index(i).  Fixed order.
__device__ __forceinline__ double tbfly8(double (&u)[8], int lane) {
  const int i = lane & 15;
  const bool f0 = ((i ^ (i >> 2)) & 1) != 0, f1 = (((i >> 1) ^ (i >> 2)) & 1) != 0, f2 = ((i >> 2) & 1) != 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const double keep = f0 ? u[p + 4] : u[p], send = f0 ? u[p] : u[p + 4];
    u[p] = keep + dpp_mov<0xB1>(send);
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const double keep = f1 ? u[p + 2] : u[p], send = f1 ? u[p] : u[p + 2];
    u[p] = keep + dpp_mov<0x4E>(send);
  }
  {
    const double keep = f2 ? u[1] : u[0], send = f2 ? u[0] : u[1];
    u[0] = keep + dpp_mov<0x141>(send);
  }
  double t = u[0];
  t += dpp_mov<0x128>(t);   // row_ror:8
  return xsum32(xsum16(t));
}
__device__ __forceinline__ int tbfly8_index(int lane) {
  const int i = lane & 15;
  return 4 * ((i ^ (i >> 2)) & 1) + 2 * (((i >> 1) ^ (i >> 2)) & 1) + ((i >> 2) & 1);
}

// wave totals of NV <= 16 per-lane values; lane k < P holds value index(k) (pad values 0)
template <int NV>
struct WaveSums {
  static constexpr int P = NV <= 8 ? 8 : 16;
  __device__ __forceinline__ static double run(const double (&v)[NV], int lane) {
    double u[P];
#pragma unroll
    for (int k = 0; k < P; ++k) u[k] = k < NV ? v[k] : 0.0;
    if constexpr (P == 8) return tbfly8(u, lane);
    else return tbfly16(u, lane);
  }
  __device__ __forceinline__ static int index(int lane) {
    if constexpr (P == 8) return tbfly8_index(lane);
    else return tbfly16_index(lane);
  }
};

__host__ __device__ inline size_t solve_grp_smem(int nn, int nm, int npass, int CG) {
  const size_t NWP = (size_t)kGT * npass;
  return sizeof(double) * ((size_t)CG * nn * 3 * kGW    // per-wave node sums
                           + (size_t)CG * nn * 9        // Bmat
                           + (size_t)CG * nn * 5        // member-factored drag coefficients
                           + (size_t)CG * 36            // B_drag
                           + (size_t)CG * 36 * nn       // per-node B_drag contributions
                           + 108 + (size_t)CG * kGW * 6 // M|B|C image, std partials
                           + (size_t)nn                 // node axial coordinate t
                           + (size_t)nm * 18            // member cq, c1, c2
                           + NWP * (1 + (size_t)CG))    // w, and zeta per case, per padded bin
         + sizeof(int) * ((size_t)nm + 2 + 1);          // member node ranges, convergence flags
}

// One workgroup per group g: cases order[gstart[g] .. gstart[g+1]) (1..CG of them), all with
// the same design and heading (the caller's grouping, raft/solver.py prepare_batch).
template <int CG>
__global__ __launch_bounds__(kGT, 1) void k_solve_grp(CaseArgs a, const int* __restrict__ gstart, int ngroup) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wv_s = __builtin_amdgcn_readfirstlane(wv);
  PROF_T(tp0);
  const int g = xcd_remap(blockIdx.x, ngroup);
  const int s0 = gstart[g];
  const int ncg = min(gstart[g + 1] - s0, CG);
  if (ncg <= 0) return;   // empty group (uniform, before any barrier)
  int ic[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) ic[c] = a.c.order ? a.c.order[s0 + (c < ncg ? c : 0)] : s0 + (c < ncg ? c : 0);
  const rh_design& d = a.designs[a.c.design[ic[0]]].d;
  const int nw = d.nw, nn = d.nn, nm = d.nm;
  const unsigned nw16 = (unsigned)nw * 16u;
  const double* __restrict__ node = d.node;
  const int head = a.c.head[ic[0]];
  const Buf bK = mkbuf(d.kproj + (size_t)head * nn * 3 * nw, (unsigned)nn * 3u * nw16);
  const Buf bFe = mkbuf(d.finer + (size_t)head * 6 * nw, 6u * nw16);
  const bool has_fx = a.c.fext != nullptr;
  Buf bXL[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) bXL[c] = mkbuf(a.o.Xi_last + (size_t)ic[c] * 6 * nw, 6u * nw16);
  const int npass = (nw + kGT - 1) / kGT, NWP = kGT * npass;

  double* red = smem;                              // [CG][nn*3][kGW]
  double* bm = red + CG * nn * 3 * kGW;            // [CG][nn][9]
  double* al = bm + CG * nn * 9;                   // [CG][nn][5]
  double* bd = al + CG * nn * 5;                   // [CG][36]
  double* bdn = bd + CG * 36;                      // [CG][36][nn]
  double* mbc = bdn + CG * 36 * nn;                // [108]
  double* sred = mbc + 108;                        // [CG][kGW][6]
  double* nt = sred + CG * kGW * 6;                // [nn]
  double* mbf = nt + nn;                           // [18][nm]
  double* lw = mbf + 18 * nm;                      // [NWP]
  double* lz = lw + NWP;                           // [CG][NWP]
  int* mstart = reinterpret_cast<int*>(lz + CG * NWP);   // [nm+1]
  int* flg = mstart + nm + 1;                      // convergence flag bits
  load_mbc(d, mbc, tid);
  for (int n = tid; n < nn; n += kGT) nt[n] = node[RH_NF_T * nn + n];
  for (int e = tid; e < 18 * nm; e += kGT) mbf[e] = d.memb[e];
  for (int e = tid; e <= nm; e += kGT) mstart[e] = d.mstart[e];

  auto voff = [&](int b) { return (unsigned)(b < nw ? b : nw - 1) * 16u; };
  for (int j = 0; j < npass; ++j) {
    const int b = tid + kGT * j;
    const bool okb = b < nw;
    const double w = d.w[okb ? b : nw - 1];
    lw[b] = w;
#pragma unroll
    for (int c = 0; c < CG; ++c) {
      if (c >= ncg) {
        lz[c * NWP + b] = 0.0;
        continue;
      }
      const int i = ic[c];
      const double zz = sea_amplitude(a.c.spectrum[i], a.c.Hs[i], a.c.Tp[i], a.c.gamma[i], w, d.dw);
      lz[c * NWP + b] = okb ? zz : 0.0;
      if (!okb) continue;
      if (a.o.zeta) a.o.zeta[(size_t)i * nw + b] = zz;
      const rh_c128* XI0 = a.c.Xi_init ? a.c.Xi_init + (size_t)i * 6 * nw : nullptr;
#pragma unroll
      for (int k = 0; k < 6; ++k)
        bst(bXL[c], XI0 ? ld(XI0 + k * nw + b) : mk(a.c.XiStart, 0.0), (unsigned)b * 16u, (unsigned)k * nw16);
    }
  }
  const double rho = d.rho;
  const int nloop = a.c.nIter + 1;
  const double tol = a.c.tol;
  constexpr int all = (1 << CG) - 1;
  int done = all & ~((1 << ncg) - 1);   // bit c: case c has finished or is an empty slot (uniform)
  int status[CG], iters[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) {
    status[c] = RH_CASE_NOT_CONVERGED;
    iters[c] = nloop;
  }
  __syncthreads();
  PROF_T(tp1);
  PROF_ADD(0, tp1 - tp0);

  for (int it = a.c.first_iter; it < nloop && done != all; ++it) {
    PROF_T(ta0);
    PROF_ADD(7, 1);
    // ---------------- A: per-node sums of squared relative-velocity components ----------
    // (raft/raft_fowt.py:1205-1220), member-factored as in k_solve_lds
#pragma unroll 1
    for (int j = 0; j < npass; ++j) {
      const int b = tid + kGT * j;
      const bool okb = b < nw;
      const unsigned vb = voff(b);
      const double w = lw[b];
      double z[CG];
      cd X[CG][6];
#pragma unroll
      for (int c = 0; c < CG; ++c) {
        z[c] = lz[c * NWP + b];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const cd x = bld(bXL[c], vb, (unsigned)k * nw16);
          X[c][k] = okb ? x : mk(0.0, 0.0);
        }
      }
      cd Bq[CG], B1[CG], B2[CG], E1[CG], E2[CG];
      auto member_terms = [&](int m) {
        double cq[6], c1[6], c2[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          cq[i] = mbf[(RH_MF_CQ0 + i) * nm + m];
          c1[i] = mbf[(RH_MF_C10 + i) * nm + m];
          c2[i] = mbf[(RH_MF_C20 + i) * nm + m];
        }
#pragma unroll
        for (int c = 0; c < CG; ++c) {
          cd Aq = mk(0, 0), A1 = mk(0, 0), A2 = mk(0, 0);
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            Aq = add(Aq, scl(X[c][k], cq[k]));
            A1 = add(A1, scl(X[c][k], c1[k]));
            A2 = add(A2, scl(X[c][k], c2[k]));
          }
          const cd D1 = add(add(scl(X[c][3], c2[0]), scl(X[c][4], c2[1])), scl(X[c][5], c2[2]));   // p2 . th
          const cd D2 = add(add(scl(X[c][3], c1[0]), scl(X[c][4], c1[1])), scl(X[c][5], c1[2]));   // p1 . th
          Bq[c] = iw(w, Aq);
          B1[c] = iw(w, A1);
          B2[c] = iw(w, A2);
          E1[c] = iw(w, D1);
          E2[c] = iw(-w, D2);
        }
      };
      auto load_node = [&](cd (&K)[3], int n) {
        const unsigned so = (unsigned)(n < nn ? n : nn - 1) * 3u * nw16;
#pragma unroll
        for (int p = 0; p < 3; ++p) K[p] = bld(bK, vb, so + (unsigned)p * nw16);
      };
      cd K[kGRingA][3];
#pragma unroll
      for (int r = 0; r < kGRingA; ++r) load_node(K[r], r);
      int m = -1, mnext = 0;
      for (int n = 0; n < nn; n += kGRingA) {
#pragma unroll
        for (int r = 0; r < kGRingA; ++r) {
          const int nr = n + r;
          if (nr < nn) {
            if (nr == mnext) {   // uniform: entering member m+1
              do { ++m; mnext = mstart[m + 1]; } while (mnext == nr);
              member_terms(m);
            }
            const double t = nt[nr];
            double s[3 * CG];
#pragma unroll
            for (int c = 0; c < CG; ++c) {
              const cd sq = sub(scl(K[r][0], z[c]), Bq[c]);
              const cd sp1 = sub(scl(K[r][1], z[c]), add(B1[c], scl(E1[c], t)));
              const cd sp2 = sub(scl(K[r][2], z[c]), add(B2[c], scl(E2[c], t)));
              s[3 * c] = abs2(sq);
              s[3 * c + 1] = abs2(sp1);
              s[3 * c + 2] = abs2(sp2);
            }
            load_node(K[r], nr + kGRingA);
            const int ln = lane_here();
            const double tot = WaveSums<3 * CG>::run(s, ln);
            const int k = WaveSums<3 * CG>::index(ln);
            if (ln < WaveSums<3 * CG>::P && k < 3 * CG) {
              const int c = k / 3, p = k - 3 * c;
              double* R = red + ((c * nn + nr) * 3 + p) * kGW + wv_s;
              *R = (j == 0 ? 0.0 : *R) + tot;
            }
          }
        }
      }
    }
    __syncthreads();
    PROF_T(ta1);
    PROF_ADD(1, ta1 - ta0);
    // ---------------- B: node drag matrices and B_drag, per unfinished case ---------------
    if (tid == 0) *flg = 0;
    for (int e = tid; e < CG * nn; e += kGT) {
      const int c = e / nn, n = e - c * nn;
      if ((done >> c) & 1) continue;
      double r3[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const double* R = red + (size_t)((c * nn + n) * 3 + q) * kGW;
        double s = 0;
#pragma unroll
        for (int w = 0; w < kGW; ++w) s += R[w];
        r3[q] = s;
      }
      const double qq = nrm2(node, nn, RH_NF_QX, n), pp1 = nrm2(node, nn, RH_NF_P1X, n), pp2 = nrm2(node, nn, RH_NF_P2X, n);
      const bool circ = nf(node, nn, RH_NF_CIRC, n) != 0.0;
      const double sums[3] = {r3[0] * qq, circ ? r3[1] * pp1 + r3[2] * pp2 : r3[1] * pp1, r3[2] * pp2};
      double B4[4];
      double* bmn = bm + 9 * (c * nn + n);
      node_bmat(node, nn, n, rho, sums, bmn, B4);
      const double t = nf(node, nn, RH_NF_T, n);
      double* A = al + 5 * (c * nn + n);
      A[0] = B4[0] + B4[3];
      A[1] = B4[1];
      A[2] = B4[2];
      A[3] = t * B4[1];
      A[4] = t * B4[2];
      const double rx = nf(node, nn, RH_NF_XX, n), ry = nf(node, nn, RH_NF_XY, n), rz = nf(node, nn, RH_NF_XZ, n);
#pragma unroll
      for (int q = 0; q < 36; ++q) bdn[(c * 36 + q) * nn + n] = t3to6(bmn, rx, ry, rz, q / 6, q % 6);
    }
    __syncthreads();
    if (tid < 36 * CG) {
      const int c = tid / 36;
      if (!((done >> c) & 1)) {
        const double* P = bdn + tid * nn;
        double s = 0;
        for (int n = 0; n < nn; ++n) s += P[n];
        bd[tid] = s;
      }
    }
    __syncthreads();
    PROF_T(ta2);
    PROF_ADD(2, ta2 - ta1);
#ifdef RH_PROF
    unsigned long long tc_exc = 0, tc_sol = 0;
#endif
    // ---------------- C: excitation, Z(w), LU solve, convergence flags ------------------
    int bad = 0;   // per thread: bit 3c = not converged, 3c+1 = NaN, 3c+2 = singular
#pragma unroll 1
    for (int j = 0; j < npass; ++j) {
      const int bj = tid + kGT * j;
      const unsigned vj = voff(bj);
      const bool okj = bj < nw;
      PROF_T(tc0);
      cd fe[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) fe[k] = bld(bFe, vj, k * nw16);
      cd F[CG][6];
#pragma unroll
      for (int c = 0; c < CG; ++c)
#pragma unroll
        for (int k = 0; k < 6; ++k) F[c][k] = mk(0, 0);
      {
        cd SQ[CG], S1[CG], S2[CG], T1[CG], T2[CG];
#pragma unroll
        for (int c = 0; c < CG; ++c) SQ[c] = S1[c] = S2[c] = T1[c] = T2[c] = mk(0, 0);
        auto load1 = [&](cd (&K)[3], int n) {
          const unsigned so = (unsigned)(n < nn ? n : nn - 1) * 3u * nw16;
#pragma unroll
          for (int p = 0; p < 3; ++p) K[p] = bld(bK, vj, so + (unsigned)p * nw16);
        };
        int m = 0, mnext = nn > 0 ? mstart[1] : 0;
        auto fold = [&]() {   // close member m (as k_solve_lds / drag_exc_members)
#pragma unroll
          for (int i = 0; i < 6; ++i) {
            const double cq = mbf[(RH_MF_CQ0 + i) * nm + m], c1 = mbf[(RH_MF_C10 + i) * nm + m],
                         c2 = mbf[(RH_MF_C20 + i) * nm + m];
#pragma unroll
            for (int c = 0; c < CG; ++c) F[c][i] = add(F[c][i], add(add(scl(SQ[c], cq), scl(S1[c], c1)), scl(S2[c], c2)));
          }
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const double p1 = mbf[(RH_MF_C10 + i) * nm + m], p2 = mbf[(RH_MF_C20 + i) * nm + m];
#pragma unroll
            for (int c = 0; c < CG; ++c) F[c][3 + i] = add(F[c][3 + i], sub(scl(T1[c], p2), scl(T2[c], p1)));
          }
#pragma unroll
          for (int c = 0; c < CG; ++c) SQ[c] = S1[c] = S2[c] = T1[c] = T2[c] = mk(0, 0);
        };
        auto step = [&](cd (&K)[3], int n) {
          while (n == mnext) {
            fold();
            ++m;
            mnext = mstart[m + 1];
          }
#pragma unroll
          for (int c = 0; c < CG; ++c) {
            const double* A = al + 5 * (c * nn + n);
            const double A0 = A[0], A1 = A[1], A2 = A[2], A3 = A[3], A4 = A[4];
            SQ[c] = add(SQ[c], scl(K[0], A0));
            S1[c] = add(S1[c], scl(K[1], A1));
            S2[c] = add(S2[c], scl(K[2], A2));
            T1[c] = add(T1[c], scl(K[1], A3));
            T2[c] = add(T2[c], scl(K[2], A4));
          }
          load1(K, n + kGRingC);
        };
        cd K[kGRingC][3];
#pragma unroll
        for (int r = 0; r < kGRingC; ++r) load1(K[r], r);
        for (int n = 0; n < nn; n += kGRingC) {
#pragma unroll
          for (int r = 0; r < kGRingC; ++r)
            if (n + r < nn) step(K[r], n + r);
        }
        if (nn > 0) fold();
      }
      PROF_T(tc1);
#ifdef RH_PROF
      tc_exc += tc1 - tc0;
#endif
      if (!okj) continue;
      const int b = bj;
      const double w = lw[b];
      // F_lin + F_drag of every unfinished case waits in its Xi output slot (overwritten by
      // its own solution below); the solves then run one case at a time in a rolled loop,
      // so a single LU is live and no per-case array is indexed dynamically
#pragma unroll
      for (int c = 0; c < CG; ++c) {
        if ((done >> c) & 1) continue;
        const double z = lz[c * NWP + b];
        rh_c128* Xo = a.o.Xi + (size_t)ic[c] * 6 * nw;
#pragma unroll
        for (int k = 0; k < 6; ++k) st(Xo + k * nw + b, add(scl(fe[k], z), scl(F[c][k], z)));
      }
#pragma unroll 1
      for (int c = 0; c < CG; ++c) {
        if ((done >> c) & 1) continue;   // uniform
        const int i = a.c.order ? a.c.order[s0 + c] : s0 + c;
        rh_c128* Xo = a.o.Xi + (size_t)i * 6 * nw;
        const Buf bxl = mkbuf(a.o.Xi_last + (size_t)i * 6 * nw, 6u * nw16);
        cd x[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) x[k] = ld(Xo + k * nw + b);
        if (has_fx) {
          const Buf bfx = mkbuf(a.c.fext + (size_t)i * 6 * nw, 6u * nw16);
#pragma unroll
          for (int k = 0; k < 6; ++k) x[k] = add(x[k], bld(bfx, (unsigned)b * 16u, k * nw16));
        }
        cd Z[6][6];
        {
          const int zo = opaque_zero();
          const double* zm = mbc + zo;
          const double* zb = bd + c * 36 + zo;
          const double w2 = -(w * w);
          if (d.mb_per_bin) {
            const double* M = d.M + (size_t)b * 36;
            const double* B = d.B + (size_t)b * 36;
#pragma unroll
            for (int r = 0; r < 6; ++r) {
#pragma unroll
              for (int q = 0; q < 6; ++q) Z[r][q] = mk(w2 * M[6 * r + q] + zm[72 + 6 * r + q], w * (B[6 * r + q] + zb[6 * r + q]));
              __builtin_amdgcn_sched_barrier(0);
            }
          } else {
#pragma unroll
            for (int r = 0; r < 6; ++r) {
#pragma unroll
              for (int q = 0; q < 6; ++q)
                Z[r][q] = mk(w2 * zm[6 * r + q] + zm[72 + 6 * r + q], w * (zm[36 + 6 * r + q] + zb[6 * r + q]));
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
        int f = lu_solve<6>(Z, x) ? 0 : 4;
        rh_c128* XP = a.o.Xi_prev ? a.o.Xi_prev + (size_t)i * 6 * nw : nullptr;
        bool ok = true, nan = false;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const cd xlast = bld(bxl, (unsigned)b * 16u, (unsigned)k * nw16);
          nan |= (x[k].r != x[k].r) || (x[k].i != x[k].i);
          // tolCheck = |Xi - XiLast| / (|Xi| + tol) < tol  (raft/raft_model.py:961-962)
          const double tt = sqrt(abs2(sub(x[k], xlast))) / (sqrt(abs2(x[k])) + tol);
          ok = ok && (tt < tol);
          st_nt(Xo + k * nw + b, x[k]);
          if (XP) st(XP + k * nw + b, xlast);
          // XiLast = 0.2 XiLast + 0.8 Xi  (:991)
          bst(bxl, add(scl(xlast, 0.2), scl(x[k], 0.8)), (unsigned)b * 16u, (unsigned)k * nw16);
        }
        f |= (ok ? 0 : 1) | (nan ? 2 : 0);
        bad |= f << (3 * c);
      }
#ifdef RH_PROF
      tc_sol += clock64() - tc1;
#endif
    }
    PROF_ADD(3, tc_exc);
    PROF_ADD(4, tc_sol);
    PROF_T(ta3);
    // block-wide OR of the flag bits: one LDS atomic per wave and bit group
    {
      int wbits = 0;
#pragma unroll
      for (int q = 0; q < 3 * CG; ++q)
        if (__builtin_amdgcn_ballot_w64((bad >> q) & 1) != 0) wbits |= 1 << q;
      if (lane == 0 && wbits) atomicOr(flg, wbits);
    }
    __syncthreads();
    PROF_T(ta4);
    PROF_ADD(5, ta4 - ta3);
    const int fl = *flg;
#pragma unroll
    for (int c = 0; c < CG; ++c) {
      if ((done >> c) & 1) continue;
      const int f = (fl >> (3 * c)) & 7;
      if (f & 2) status[c] = RH_CASE_NAN;
      else if (f & 4) status[c] = RH_CASE_SINGULAR;
      else if (!(f & 1)) status[c] = RH_CASE_CONVERGED;
      else continue;
      iters[c] = it + 1;
      done |= 1 << c;
    }
  }

  // ---------------- outputs, per case ------------------------------------------------------
  PROF_T(te0);
#pragma unroll
  for (int c = 0; c < CG; ++c) {
    if (c >= ncg) continue;
    const int i = ic[c];
    if (tid == 0) {
      a.o.iters[i] = iters[c];
      a.o.status[i] = status[c];
    }
    if (a.o.B_drag && tid < 36) a.o.B_drag[(size_t)i * 36 + tid] = bd[c * 36 + tid];
    if (a.o.Bmat)
      for (int e = tid; e < nn * 9; e += kGT) a.o.Bmat[(size_t)i * a.bmat_nn * 9 + e] = bm[c * nn * 9 + e];
    if (a.o.Z) {   // final impedance fowt.Z (raft/raft_model.py:1013)
#pragma unroll 1
      for (int j = 0; j < npass; ++j) {
        const int b = tid + kGT * j;
        if (b >= nw) continue;
        const double w = lw[b], w2 = -(w * w);
        rh_c128* Zo = a.o.Z + ((size_t)i * nw + b) * 36;
#pragma unroll 1
        for (int e = 0; e < 36; ++e) {
          const double M = d.mb_per_bin ? d.M[(size_t)b * 36 + e] : mbc[e];
          const double B = d.mb_per_bin ? d.B[(size_t)b * 36 + e] : mbc[36 + e];
          st(Zo + e, mk(w2 * M + mbc[72 + e], w * (B + bd[c * 36 + e])));
        }
      }
    }
    const rh_c128* Xo = a.o.Xi + (size_t)i * 6 * nw;
    double ss[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll 1
    for (int j = 0; j < npass; ++j) {
      const int b = tid + kGT * j;
      if (b >= nw) continue;
      const double z = lz[c * NWP + b];
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const cd x = ld(Xo + k * nw + b);
        const cd xd = k >= 3 ? scl(x, kRad2Deg) : x;
        const double m2 = abs2(xd);
        ss[k] += m2;
        if (a.o.psd) a.o.psd[((size_t)i * 6 + k) * nw + b] = 0.5 * m2 / d.dw;
        if (a.o.rao) st(a.o.rao + ((size_t)i * 6 + k) * nw + b, fabs(z) > 1e-6 ? cd{x.r / z, x.i / z} : mk(0, 0));
      }
    }
    if (a.o.std) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const double s = wave_sum(ss[k]);
        if (lane == 0) sred[(c * kGW + wv) * 6 + k] = s;
      }
    }
  }
  if (a.o.std) {
    __syncthreads();
    if (tid < 6 * ncg) {
      const int c = tid / 6, k = tid - 6 * c;
      double s = 0;
      for (int w = 0; w < kGW; ++w) s += sred[(c * kGW + w) * 6 + k];
      const int i = a.c.order ? a.c.order[s0 + c] : s0 + c;   // not ic[c]: no dynamic private index
      a.o.std[(size_t)i * 6 + k] = sqrt(0.5 * s);
    }
  }
  PROF_T(te1);
  PROF_ADD(6, te1 - te0);
}

}  // namespace rh
