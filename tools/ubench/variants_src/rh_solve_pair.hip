// rh_solve_pair.hip -- k_solve_pair: the per-case drag fixed point at four waves per SIMD.
//
// Same algorithm and arithmetic as k_solve_lds (rh_solve.hip; raft/raft_model.py:918-1000,
// raft/raft_fowt.py:1152-1293), re-laid-out so that one case fills a CU with 16 waves:
//   * LT threads per case (1024 for nw <= 1024, 256 for nw <= 256), one bin per lane in phase
//     C (b = tid), and at most 128 VGPRs, so the CU holds 4 waves per SIMD (k_solve_lds: 2).
//   * Each bin's 6x6 complex LU runs on a LANE PAIR (pair_lu): lane parity p holds rows p,
//     p+2, p+4, the pivot row and the partial solution are broadcast inside the pair with DPP.
//     The pair solves its two bins one after the other.  That halves the register peak of the
//     solve (the whole-matrix form needs ~170 VGPRs), which is what admits the fourth wave.
//     The pivot rule is lu_solve's: max |re|+|im|, first maximum in row order; the elimination
//     does the same operations in the same order.
//   * Phase A (per-node bin sums) with PB = 2 keeps k_solve_lds's lane layout: every lane sums
//     two bins (tid % 512, tid % 512 + 512) and the two halves of the workgroup take the two
//     halves of the node list, so the per-node wave reductions stay one per 128 bins.
//   * XiLast stays in LDS.  The unrelaxed solution of an iteration stays in registers across
//     the convergence vote and goes to HBM once, after the last iteration (k_solve_lds
//     streamed it out every iteration: ~0.2 GB per C2 launch that only the last one used).
//   * No per-lane branch anywhere around the solve: pad lanes (b >= nw) solve the clamped last
//     bin with a zero right-hand side (x = 0 exactly) and store nothing.
#include "../../../raft-teststuff_amd/csrc/rh_device.h"

namespace rh {

// DPP inside a lane pair: broadcast the value of the even (P = 0) or odd (P = 1) lane of each
// pair to both lanes (quad_perm [0,0,2,2] / [1,1,3,3]), or exchange the pair (quad_perm [1,0,3,2]).
template <int P>
__device__ __forceinline__ double pbc(double v) {
  return dpp_mov<P ? 0xF5 : 0xA0>(v);
}
template <int P>
__device__ __forceinline__ cd pbc(cd v) {
  return mk(pbc<P>(v.r), pbc<P>(v.i));
}
__device__ __forceinline__ cd pswap(cd v) { return mk(dpp_mov<0xB1>(v.r), dpp_mov<0xB1>(v.i)); }
__device__ __forceinline__ double pswap(double v) { return dpp_mov<0xB1>(v); }
__device__ __forceinline__ int pswap(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true); }
// component-wise select: a `?:` on the struct itself becomes a select of addresses plus a copy,
// which keeps the arrays it touches in scratch
__device__ __forceinline__ cd csel(bool c, cd a, cd b) { return mk(c ? a.r : b.r, c ? a.i : b.i); }

// Partially pivoted Gaussian elimination of one 6x6 complex system on a lane pair.
// A[s][c] / y[s]: row r = 2 s + par of the matrix / right-hand side held by this lane.
// On return x[0..5] is the solution in BOTH lanes.  Returns false on an exactly zero pivot.
// The arithmetic is lu_solve<6>'s (rh_device.h): the same pivot choice and the same
// operations in the same order on every element.  Call with every lane of the wave active.
template <int K>
__device__ __forceinline__ void pair_step(cd (&A)[3][6], cd (&y)[3], int par, bool& ok) {
  constexpr int kp = K & 1, ks = K >> 1;
  // pivot search: this lane's first maximum over its rows >= K, then the pair's
  double lb = 0.0;
  int lr = 6;   // 6 = no eligible row in this lane
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    if (2 * s + 1 < K) continue;   // neither lane's slot-s row is >= K
    const int row = 2 * s + par;
    const double v = cabs1(A[s][K]);
    const bool take = (row >= K) & ((lr == 6) | (v > lb));   // bitwise: no branches
    lb = take ? v : lb;
    lr = take ? row : lr;
  }
  const double ob = pswap(lb);
  const int orw = pswap(lr);
  const double be = par ? ob : lb, bo = par ? lb : ob;
  const int re = par ? orw : lr, ro = par ? lr : orw;
  // the odd lane's candidate wins if it is larger, or equal and earlier in row order (the
  // same decision in both lanes: both evaluate it on the pair's even/odd values)
  const bool take_o = (re == 6) | ((ro != 6) & ((bo > be) | ((bo == be) & (ro < re))));
  const double best = take_o ? bo : be;
  const int p = take_o ? ro : re;
  ok = ok && (best != 0.0);
  if (__builtin_amdgcn_ballot_w64(p != K) != 0) {
    // Row exchange K <-> p (columns >= K and the right-hand side).  Row K sits in lane kp,
    // slot ks; row p in lane p & 1, slot p >> 1: an in-lane select chain when the parities
    // agree, a pair exchange when they differ.
    const bool cross = (p & 1) != kp;
    const bool in_k = par == kp;
    const int ps = p >> 1;
    auto xchg = [&](cd (&v)[3]) {
      cd rowp = v[ks];
#pragma unroll
      for (int s = 0; s < 3; ++s) rowp = csel(s == ps, v[s], rowp);   // this lane's slot ps
      const cd old_k = v[ks];
      const cd rcv = pswap(csel(in_k, old_k, rowp));
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const bool is_p = s == ps;
        cd nv = v[s];
        if (s == ks) nv = csel(in_k, csel(cross, rcv, rowp), nv);
        nv = csel(cross & !in_k & is_p, rcv, nv);
        nv = csel((!cross) & in_k & is_p & (s != ks), old_k, nv);
        v[s] = nv;
      }
    };
#pragma unroll
    for (int j = K; j < 6; ++j) {   // one column at a time: the exchange is the rare path
      cd col[3] = {A[0][j], A[1][j], A[2][j]};
      xchg(col);
      A[0][j] = col[0];
      A[1][j] = col[1];
      A[2][j] = col[2];
      __builtin_amdgcn_sched_barrier(0);
    }
    xchg(y);
  }
  // 1/piv = conj(piv) / |piv|^2 (lu_solve's reciprocal); lane kp keeps it on its diagonal
  const cd pv0 = pbc<kp>(A[ks][K]);
  const cd pv = csel(best != 0.0, pv0, mk(1.0, 0.0));
  const double inv = 1.0 / (pv.r * pv.r + pv.i * pv.i);
  const cd rinv = mk(pv.r * inv, -pv.i * inv);
  cd l[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    if (2 * s + 1 <= K) continue;
    l[s] = csel(2 * s + par > K, mul(A[s][K], rinv), mk(0.0, 0.0));   // rows below K only
  }
  A[ks][K] = csel(par == kp, rinv, A[ks][K]);
#pragma unroll
  for (int j = K + 1; j < 6; ++j) {
    const cd P = pbc<kp>(A[ks][j]);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      if (2 * s + 1 <= K) continue;
      A[s][j] = sub(A[s][j], mul(l[s], P));
    }
#ifdef SBCOL
    __builtin_amdgcn_sched_barrier(0);
#endif
  }
  {
    const cd P = pbc<kp>(y[ks]);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      if (2 * s + 1 <= K) continue;
      y[s] = sub(y[s], mul(l[s], P));
    }
  }
}

template <int K>
__device__ __forceinline__ void pair_back(const cd (&A)[3][6], const cd (&y)[3], cd (&x)[6]) {
  constexpr int kp = K & 1, ks = K >> 1;
  cd s = y[ks];
#pragma unroll
  for (int j = K + 1; j < 6; ++j) s = sub(s, mul(A[ks][j], x[j]));
  x[K] = pbc<kp>(mul(s, A[ks][K]));   // computed in lane kp, which holds row K
}

#ifdef PAIR_NOINLINE
__device__ __attribute__((noinline)) bool pair_lu(
#else
__device__ __forceinline__ bool pair_lu(
#endif
cd (&A)[3][6], cd (&y)[3], cd (&x)[6], int par) {
  bool ok = true;
  pair_step<0>(A, y, par, ok);
  pair_step<1>(A, y, par, ok);
  pair_step<2>(A, y, par, ok);
  pair_step<3>(A, y, par, ok);
  pair_step<4>(A, y, par, ok);
  pair_step<5>(A, y, par, ok);
  pair_back<5>(A, y, x);
  pair_back<4>(A, y, x);
  pair_back<3>(A, y, x);
  pair_back<2>(A, y, x);
  pair_back<1>(A, y, x);
  pair_back<0>(A, y, x);
  return ok;
}

// LDS of k_solve_pair (bytes).  LT threads = padded bins; PB = bins per lane in phase A.
__host__ __device__ inline size_t solve_pair_smem(int nn, int nm, int LT, int PB) {
  const int LW = LT / 64, LWA = LW / PB;
  return sizeof(double) * ((size_t)12 * LT          // XiLast [6][LT] complex
                           + (size_t)nn * 3 * LWA   // per-wave node sums of phase A
                           + (size_t)nn * 36        // per-node B_drag contributions
                           + (size_t)nn * 9         // Bmat
                           + (size_t)nn * 5         // member-factored drag coefficients
                           + (size_t)nn             // node axial coordinate t
                           + (size_t)nm * 18        // member cq, c1, c2
                           + (size_t)2 * LT         // w and zeta per (padded) bin
                           + 36 + 108 + LW * 6 + 36  // B_drag, M|B|C image, std partials, B_lin+B_drag
                           + LW + 1)                // convergence-margin partials, closest call
         + sizeof(int) * ((size_t)nm + 2);
}

// LT threads per case, one bin per lane (nw <= LT).  PB bins per lane in phase A (PB = 2: the
// two halves of the workgroup take the two halves of the node list).  RA / RC: wave-table
// prefetch depth (nodes) of phases A / C.
template <int LT, int PB, int RA, int RC, bool HOLD>
__global__ __launch_bounds__(LT, 4) void k_solve_pair(CaseArgs a) {
  constexpr int LW = LT / 64;       // waves per case
  constexpr int TB = LT / PB;       // lanes per phase-A group (bins per pass)
  constexpr int LWA = TB / 64;      // waves per phase-A group
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x;
  // The wave index lives in an SGPR; every lane-dependent index below is recomputed from it
  // and the lane id where it is used (tnow(): v_mbcnt behind asm volatile, so it is neither
  // hoisted nor kept): a value kept live across the phases would be spilled around the
  // register-heavy pair solves, and its reload inside a node loop would drain the wave-table
  // prefetch ring (scratch loads share vmcnt with the buffer loads).
  const int wv_s = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto tnow = [&]() { return wv_s * 64 + lane_here(); };
  PROF_T(tp0);
  const int slot = xcd_remap(blockIdx.x, a.c.ncase);
  const int ic = a.c.order ? a.c.order[slot] : slot;
  const rh_design& d = a.designs[a.c.design[ic]].d;
  const int nw = d.nw, nn = d.nn, nm = d.nm;
  const unsigned nw16 = (unsigned)nw * 16u;
  const double* __restrict__ node = d.node;
  const int head = a.c.head[ic];
  const size_t c6 = (size_t)ic * 6 * nw;
  const Buf bK = mkbuf(d.kproj + (size_t)head * nn * 3 * nw, (unsigned)nn * 3u * nw16);
  const Buf bFe = mkbuf(d.finer + (size_t)head * 6 * nw, 6u * nw16);
  const bool has_fx = a.c.fext != nullptr;
  const Buf bFx = mkbuf(has_fx ? a.c.fext + c6 : nullptr, has_fx ? 6u * nw16 : 0u);

  cd* xl = reinterpret_cast<cd*>(smem);            // [6][LT]
  double* red = smem + 12 * LT;                    // [nn*3][LWA]
  double* bm = red + nn * 3 * LWA;                 // [nn][9]
  double* al = bm + nn * 9;                        // [nn][5]
  double* bd = al + nn * 5;                        // [36]
  double* mbc = bd + 36;                           // [108] M, B_lin, C
  double* sred = mbc + 108;                        // [LW][6]
  double* bsum = sred + LW * 6;                    // [36] B_lin + B_drag of this iteration
  double* bdn = bsum + 36;                         // [36][nn]
  double* nt = bdn + 36 * nn;                      // [nn]
  double* mbf = nt + nn;                           // [18][nm]
  double* lw = mbf + 18 * nm;                      // [LT] w per bin (pad bins: w[nw-1])
  double* lz = lw + LT;                            // [LT] zeta per bin (pad bins: 0)
  double* mred = lz + LT;                          // [LW] per-wave max of tolCheck, [LW] closest call
  int* mstart = reinterpret_cast<int*>(mred + LW + 1);  // [nm+1]
  load_mbc(d, mbc, tid);
  for (int n = tid; n < nn; n += LT) nt[n] = node[RH_NF_T * nn + n];
  for (int e = tid; e < 18 * nm; e += LT) mbf[e] = d.memb[e];
  for (int e = tid; e <= nm; e += LT) mstart[e] = d.mstart[e];

  auto voff = [&](int b) { return (unsigned)(b < nw ? b : nw - 1) * 16u; };
  {
    const int b = tid;                // this lane's bin in phase C
    const bool okb = b < nw;
    const int spec = a.c.spectrum[ic];
    const double Hs = a.c.Hs[ic], Tp = a.c.Tp[ic], gam = a.c.gamma[ic];
    const rh_c128* XI0 = a.c.Xi_init ? a.c.Xi_init + c6 : nullptr;
    const double w = d.w[okb ? b : nw - 1];
    const double zz = sea_amplitude(spec, Hs, Tp, gam, w, d.dw);
    lw[b] = w;
    lz[b] = okb ? zz : 0.0;
    if (okb && a.o.zeta) a.o.zeta[(size_t)ic * nw + b] = zz;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      cd x0 = mk(a.c.XiStart, 0.0);
      if (XI0) x0 = ld(XI0 + c * nw + (okb ? b : nw - 1));   // uniform branch; in-range address
      xl[c * LT + b] = csel(okb, x0, mk(0.0, 0.0));
    }
  }
  rh_c128* Xo = a.o.Xi + c6;
  rh_c128* XP = a.o.Xi_prev ? a.o.Xi_prev + c6 : nullptr;
  const double rho = d.rho;
  const int nloop = a.c.nIter + 1;
  const double tol = a.c.tol;
  int status = RH_CASE_NOT_CONVERGED, iters = nloop;
  if (tid == 0) mred[LW] = INFINITY;   // closest call of the convergence test so far (LDS)
  __syncthreads();
  // phase-A node range of this lane's group: PB = 2 splits the node list at the member
  // boundary closest to its middle (a member's terms are computed once per group)
  int na0 = 0, na1 = nn;
  if (PB == 2) {
    int split = 0, bestd = 1 << 30;
    for (int m = 0; m <= nm; ++m) {
      const int dd = abs(2 * mstart[m] - nn);
      if (dd < bestd) { bestd = dd; split = mstart[m]; }
    }
    split = __builtin_amdgcn_readfirstlane(split);   // uniform
    const int g = wv_s / LWA;
    na0 = g ? split : 0;
    na1 = g ? nn : split;
  }
  cd X[6];   // this lane's unrelaxed solution of the current iteration
  PROF_T(tp1);
  PROF_ADD(0, tp1 - tp0);
#ifdef ABL
  const bool n0_never = a.c.nIter == 12345;
#endif

  for (int it = a.c.first_iter; it < nloop; ++it) {
    PROF_T(ta0);
    PROF_ADD(7, 1);
    // ---------------- A: per-node sums of squared relative-velocity components ----------
    // (raft/raft_fowt.py:1205-1211; member-factored as in k_solve_lds)
    {
      const int tb = tnow() & (TB - 1), wg = wv_s & (LWA - 1);
      unsigned vb[PB];
      double bz[PB];
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        vb[j] = voff(tb + TB * j);
        bz[j] = lz[tb + TB * j];
      }
      cd Bq[PB], B1[PB], B2[PB], E1[PB], E2[PB];
      auto member_terms = [&](int m) {
        double cq[6], c1[6], c2[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          cq[i] = mbf[(RH_MF_CQ0 + i) * nm + m];
          c1[i] = mbf[(RH_MF_C10 + i) * nm + m];
          c2[i] = mbf[(RH_MF_C20 + i) * nm + m];
        }
#pragma unroll
        for (int j = 0; j < PB; ++j) {
          const int bb = tb + TB * j;
          cd Xl[6];
#pragma unroll
          for (int c = 0; c < 6; ++c) Xl[c] = xl[c * LT + bb];
          cd Aq = mk(0, 0), A1 = mk(0, 0), A2 = mk(0, 0);
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            Aq = add(Aq, scl(Xl[c], cq[c]));
            A1 = add(A1, scl(Xl[c], c1[c]));
            A2 = add(A2, scl(Xl[c], c2[c]));
          }
          const cd D1 = add(add(scl(Xl[3], c2[0]), scl(Xl[4], c2[1])), scl(Xl[5], c2[2]));   // p2 . th
          const cd D2 = add(add(scl(Xl[3], c1[0]), scl(Xl[4], c1[1])), scl(Xl[5], c1[2]));   // p1 . th
          const double w = lw[bb];
          Bq[j] = iw(w, Aq);
          B1[j] = iw(w, A1);
          B2[j] = iw(w, A2);
          E1[j] = iw(w, D1);
          E2[j] = iw(-w, D2);
        }
      };
      auto load_node = [&](cd (&K)[3][PB], int n) {
        const unsigned so = (unsigned)(n < nn ? n : nn - 1) * 3u * nw16;
#pragma unroll
        for (int j = 0; j < PB; ++j)
#pragma unroll
          for (int p = 0; p < 3; ++p) K[p][j] = bld(bK, vb[j], so + (unsigned)p * nw16);
      };
      auto node_sums = [&](const cd (&K)[3][PB], int n, double& s0, double& s1, double& s2) {
        const double t = nt[n];
        s0 = s1 = s2 = 0;
#pragma unroll
        for (int j = 0; j < PB; ++j) {
          const double z = bz[j];
          const cd sq = sub(scl(K[0][j], z), Bq[j]);
          const cd sp1 = sub(scl(K[1][j], z), add(B1[j], scl(E1[j], t)));
          const cd sp2 = sub(scl(K[2][j], z), add(B2[j], scl(E2[j], t)));
          s0 += abs2(sq);
          s1 += abs2(sp1);
          s2 += abs2(sp2);
        }
      };
      cd K[RA][3][PB];
#pragma unroll
      for (int r = 0; r < RA; ++r) load_node(K[r], na0 + r);
      int m = -1;
      while (m + 2 <= nm && mstart[m + 2] <= na0) ++m;   // member m + 1 holds node na0
      int mnext = na0;
#if defined(ABL) && (ABL & 1)
      if (n0_never)
#endif
      for (int n = na0; n < na1; n += RA) {
#pragma unroll
        for (int r = 0; r < RA; ++r) {
          const int nr = n + r;
          if (nr < na1) {
            if (nr == mnext) {   // uniform: entering the next member (members are node-contiguous)
              do { ++m; mnext = mstart[m + 1]; } while (mnext == nr);
              member_terms(m);
            }
            double s0, s1, s2;
            node_sums(K[r], nr, s0, s1, s2);
            load_node(K[r], nr + RA);
            const int ln = lane_here();
            const double tot = tbfly3(s0, s1, s2, ln);
            if (ln < 3) red[(nr * 3 + tbfly3_index(ln)) * LWA + wg] = tot;
          }
        }
      }
    }
    __syncthreads();
    PROF_T(ta1);
    PROF_ADD(1, ta1 - ta0);
    // ---------------- B: node drag matrices and B_drag ----------------------------------
    for (int n = tnow(); n < nn; n += LT) {
      double r3[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double* R = red + (size_t)(n * 3 + c) * LWA;
        double s = 0;
#pragma unroll
        for (int w = 0; w < LWA; ++w) s += R[w];
        r3[c] = s;
      }
      const double qq = nrm2(node, nn, RH_NF_QX, n), pp1 = nrm2(node, nn, RH_NF_P1X, n), pp2 = nrm2(node, nn, RH_NF_P2X, n);
      const bool circ = nf(node, nn, RH_NF_CIRC, n) != 0.0;
      const double sums[3] = {r3[0] * qq, circ ? r3[1] * pp1 + r3[2] * pp2 : r3[1] * pp1, r3[2] * pp2};
      double B4[4];
      node_bmat(node, nn, n, rho, sums, bm + 9 * n, B4);
      const double t = nf(node, nn, RH_NF_T, n);
      double* A = al + 5 * n;
      A[0] = B4[0] + B4[3];
      A[1] = B4[1];
      A[2] = B4[2];
      A[3] = t * B4[1];
      A[4] = t * B4[2];
      const double rx = nf(node, nn, RH_NF_XX, n), ry = nf(node, nn, RH_NF_XY, n), rz = nf(node, nn, RH_NF_XZ, n);
#pragma unroll
      for (int e = 0; e < 36; ++e) bdn[e * nn + n] = t3to6(bm + 9 * n, rx, ry, rz, e / 6, e % 6);
    }
    __syncthreads();
    if (wv_s == 0) {
      const int e = lane_here();
      if (e < 36) {
        const double* P = bdn + e * nn;
        double s = 0;
        for (int n = 0; n < nn; ++n) s += P[n];
        bd[e] = s;
        bsum[e] = mbc[36 + e] + s;
      }
    }
    __syncthreads();
    PROF_T(ta2);
    PROF_ADD(2, ta2 - ta1);
    // ---------------- C: excitation of this lane's bin ----------------------------------
    const int b = tnow();
    const bool okb = b < nw;
    const int par = b & 1;
    const unsigned vb_own = voff(b);
    cd F[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) F[c] = mk(0, 0);
    {
      cd SQ = mk(0, 0), S1 = mk(0, 0), S2 = mk(0, 0), T1 = mk(0, 0), T2 = mk(0, 0);
      auto load1 = [&](cd (&K)[3], int n) {
        const unsigned so = (unsigned)(n < nn ? n : nn - 1) * 3u * nw16;
#pragma unroll
        for (int p = 0; p < 3; ++p) K[p] = bld(bK, vb_own, so + (unsigned)p * nw16);
      };
      int m = 0, mnext = nn > 0 ? mstart[1] : 0;
      auto fold = [&]() {   // close member m: F += sum of its nodes (as drag_exc_members)
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const double cq = mbf[(RH_MF_CQ0 + i) * nm + m], c1 = mbf[(RH_MF_C10 + i) * nm + m],
                       c2 = mbf[(RH_MF_C20 + i) * nm + m];
          F[i] = add(F[i], add(add(scl(SQ, cq), scl(S1, c1)), scl(S2, c2)));
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double p1 = mbf[(RH_MF_C10 + i) * nm + m], p2 = mbf[(RH_MF_C20 + i) * nm + m];
          F[3 + i] = add(F[3 + i], sub(scl(T1, p2), scl(T2, p1)));
        }
        SQ = S1 = S2 = T1 = T2 = mk(0, 0);
      };
      auto step = [&](cd (&K)[3], int n) {
        while (n == mnext) {   // uniform: member m ended before node n
          fold();
          ++m;
          mnext = mstart[m + 1];
        }
        const double* A = al + 5 * n;
        const double A0 = A[0], A1 = A[1], A2 = A[2], A3 = A[3], A4 = A[4];
        SQ = add(SQ, scl(K[0], A0));
        S1 = add(S1, scl(K[1], A1));
        S2 = add(S2, scl(K[2], A2));
        T1 = add(T1, scl(K[1], A3));
        T2 = add(T2, scl(K[2], A4));
        load1(K, n + RC);
      };
      cd K[RC][3];
#pragma unroll
      for (int r = 0; r < RC; ++r) load1(K[r], r);
#if defined(ABL) && (ABL & 2)
      if (n0_never)
#endif
      for (int n = 0; n < nn; n += RC) {
#pragma unroll
        for (int r = 0; r < RC; ++r)
          if (n + r < nn) step(K[r], n + r);
      }
      if (nn > 0) fold();
    }
    {
      const double z = lz[b];   // 0 on pad lanes: their right-hand side is exactly zero
#pragma unroll
      for (int c = 0; c < 6; ++c) F[c] = add(scl(bld(bFe, vb_own, c * nw16), z), scl(F[c], z));   // F_lin + F_drag
      if (has_fx) {
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const cd fx = bld(bFx, vb_own, c * nw16);
          F[c] = add(F[c], csel(okb, fx, mk(0.0, 0.0)));
        }
      }
    }
    PROF_T(ta3);
    PROF_ADD(3, ta3 - ta2);
    // ---------------- C: Z(w) and the pair solves of the pair's two bins ---------------
    // Right-hand sides of both passes first, so that F is dead before the first solve: pass q
    // solves bin (tid & ~1) | q, whose rows 2s + par this lane needs.
    cd y0[3], y1[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      y0[s] = csel(par, pbc<0>(F[2 * s + 1]), F[2 * s]);
      y1[s] = csel(par, F[2 * s + 1], pbc<1>(F[2 * s]));
    }
    bool my_ok = true, my_nan = false, my_sing = false;
    double my_tmax = 0.0;
#pragma unroll 1
    for (int q = 0; q < 2; ++q) {   // not unrolled: one pass's matrix live at a time
      const int bq = (b & ~1) | q;   // the bin solved in this pass (uniform in the pair)
      cd A[3][6], x[6], y[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) y[s] = csel(q != 0, y1[s], y0[s]);
      {
        const int zo = opaque_zero();   // keep the LDS reads here, not hoisted into VGPRs
        const double* zm = mbc + zo;
        const double* zs = bsum + zo;
        const double* zb = bd + zo;
        const double w = lw[bq], w2 = -(w * w);
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int r = 2 * s + par;
          if (d.mb_per_bin) {
            const int bc = bq < nw ? bq : nw - 1;
            const double* M = d.M + (size_t)bc * 36;
            const double* B = d.B + (size_t)bc * 36;
#pragma unroll
            for (int c = 0; c < 6; ++c) A[s][c] = mk(w2 * M[6 * r + c] + zm[72 + 6 * r + c], w * (B[6 * r + c] + zb[6 * r + c]));
          } else {
#pragma unroll
            for (int c = 0; c < 6; ++c) A[s][c] = mk(w2 * zm[6 * r + c] + zm[72 + 6 * r + c], w * zs[6 * r + c]);
          }
        }
      }
#if defined(ABL) && (ABL & 4)
      bool okq = true;
      for (int c = 0; c < 6; ++c) x[c] = add(A[c % 3][c], y[c % 3]);
#else
      const bool okq = pair_lu(A, y, x, par);
#endif
      // Both lanes of the pair now hold the solution of bin bq and do the same bookkeeping
      // for it (the same values, so the duplicate flags and stores are benign).
      const bool okq_bin = bq < nw;
      my_sing = my_sing || (okq_bin && !okq);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const cd xlast = xl[c * LT + bq];
        // tolCheck = |Xi - XiLast| / (|Xi| + tol) < tol  (raft/raft_model.py:961-962)
        const double tt = sqrt(abs2(sub(x[c], xlast))) / (sqrt(abs2(x[c])) + tol);
        my_nan = my_nan || (okq_bin && ((x[c].r != x[c].r) || (x[c].i != x[c].i)));
        my_ok = my_ok && (!okq_bin || tt < tol);
        my_tmax = okq_bin ? fmax(my_tmax, tt) : my_tmax;
        if (HOLD) {
          X[c] = csel(par == q, x[c], X[c]);
        } else {
          if (okq_bin) {   // stores only (pads: the last pair of an odd grid)
            st_nt(Xo + c * nw + bq, x[c]);   // streamed: only the last iteration's value is kept
            if (XP) st(XP + c * nw + bq, xlast);
          }
          // XiLast = 0.2 XiLast + 0.8 Xi (:991), consumed only if the case goes on
          xl[c * LT + bq] = add(scl(xlast, 0.2), scl(x[c], 0.8));
        }
      }
    }
    PROF_T(ta4);
    PROF_ADD(4, ta4 - ta3);
    // ---------------- D: the convergence vote ------------------------------------------
    if (a.o.margin) {
      const double mw = wave_max(my_tmax);
      if (lane_here() == 0) mred[wv_s] = mw;
    }
    const int all_ok = __syncthreads_and(my_ok ? 1 : 0);
    if (a.o.margin && b == 0) {   // mred is rewritten only after the next iteration's solves
      double mx = mred[0];
      for (int w = 1; w < LW; ++w) mx = fmax(mx, mred[w]);
      mred[LW] = closer_call(mred[LW], mx - tol);
    }
    const int any_nan = __syncthreads_or(my_nan ? 1 : 0);
    const int any_sing = __syncthreads_or(my_sing ? 1 : 0);
    PROF_T(ta5);
    PROF_ADD(5, ta5 - ta4);
    const bool last = any_nan || any_sing || all_ok || it + 1 == nloop;
    if (last) {
      status = any_nan ? RH_CASE_NAN : any_sing ? RH_CASE_SINGULAR : all_ok ? RH_CASE_CONVERGED : RH_CASE_NOT_CONVERGED;
      iters = it + 1;
      if (HOLD && okb) {
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          st(Xo + c * nw + b, X[c]);
          if (XP) st(XP + c * nw + b, xl[c * LT + b]);
        }
      }
      break;
    }
    if (HOLD) {
#pragma unroll
      for (int c = 0; c < 6; ++c) {   // XiLast = 0.2 XiLast + 0.8 Xi  (:991)
        const cd xlast = xl[c * LT + b];
        xl[c * LT + b] = add(scl(xlast, 0.2), scl(X[c], 0.8));
      }
    }
  }
  const int b = tid;
  const bool okb = b < nw;
  const int lane = tid & 63, wv = tid >> 6;
  if (!HOLD) {   // the final unrelaxed solution, for the statistics below
#pragma unroll
    for (int c = 0; c < 6; ++c) X[c] = csel(okb, ld(Xo + c * (okb ? nw : 0) + (okb ? b : 0)), mk(0.0, 0.0));
  }

  // ---------------- outputs ------------------------------------------------------------
  PROF_T(te0);
  if (tid == 0) {
    a.o.iters[ic] = iters;
    a.o.status[ic] = status;
    if (a.o.margin) a.o.margin[ic] = mred[LW];
  }
  if (a.o.B_drag && tid < 36) a.o.B_drag[(size_t)ic * 36 + tid] = bd[tid];
  if (a.o.Bmat)
    for (int e = tid; e < nn * 9; e += LT) a.o.Bmat[(size_t)ic * a.bmat_nn * 9 + e] = bm[e];
  if (a.o.Z && okb) {   // final impedance fowt.Z (raft/raft_model.py:1013) from the last B_drag
    const double w = lw[b], w2 = -(w * w);
    rh_c128* Zo = a.o.Z + ((size_t)ic * nw + b) * 36;
#pragma unroll 1
    for (int e = 0; e < 36; ++e) {
      const double M = d.mb_per_bin ? d.M[(size_t)b * 36 + e] : mbc[e];
      const double B = d.mb_per_bin ? d.B[(size_t)b * 36 + e] : mbc[36 + e];
      st(Zo + e, mk(w2 * M + mbc[72 + e], w * (B + bd[e])));
    }
  }
  double ss[6];
  {
    const double z = lz[b];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const cd x = X[c];
      const cd xd = csel(c >= 3, scl(x, kRad2Deg), x);
      const double m2 = abs2(xd);
      ss[c] = okb ? m2 : 0.0;
      if (okb && a.o.psd) a.o.psd[((size_t)ic * 6 + c) * nw + b] = 0.5 * m2 / d.dw;
      if (okb && a.o.rao) st(a.o.rao + ((size_t)ic * 6 + c) * nw + b, fabs(z) > 1e-6 ? cd{x.r / z, x.i / z} : mk(0, 0));
    }
  }
  if (a.o.std) {
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const double s = wave_sum(ss[c]);
      if (lane == 0) sred[wv * 6 + c] = s;
    }
    __syncthreads();
    if (tid < 6) {
      double s = 0;
      for (int w = 0; w < LW; ++w) s += sred[w * 6 + tid];
      a.o.std[(size_t)ic * 6 + tid] = sqrt(0.5 * s);
    }
  }
  PROF_T(te1);
  PROF_ADD(6, te1 - te0);
}

}  // namespace rh
