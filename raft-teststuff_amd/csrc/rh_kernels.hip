// rh_kernels.hip -- gfx950 kernels of RAFT's frequency-domain response solve.
//
// Hot path:
//   k_wave_tables  : unit-amplitude Airy kinematics per (heading, node, bin) and the
//                    strip-theory inertial excitation sum over nodes
//                    (raft/raft_fowt.py:1098-1124, raft/helpers.py:105-154).
//   k_solve_cases  : one workgroup per sea-state case; the whole Borgman drag fixed point
//                    (raft/raft_model.py:918-1000) runs inside the workgroup:
//                      A  RMS of node relative velocity over all bins (raft/raft_fowt.py:1185-1220)
//                      B  per-node Bmat and B_drag = sum translateMatrix3to6DOF (:1223-1250)
//                      C  per-bin drag excitation + Z assembly + pivoted LU (raft/raft_model.py:937-947)
//                      D  convergence test / 0.2-0.8 relaxation (:961-991)
//                    then the motion statistics of saveTurbineOutputs (raft/raft_fowt.py:1831-1875).
//   k_heading_resp : extra sea states with the linearisation frozen (raft/raft_model.py:1049-1065).
//
// Work layout: lane = frequency bin (NB bins per thread, 256 threads per case), node loop
// innermost with node parameters wave-uniform (scalar loads), the per-node bin reductions
// done with 64-lane butterflies and a fixed-order cross-wave sum (deterministic).
#include "rh_common.h"

namespace rh {


__global__ __launch_bounds__(256) void k_sea_state(int nw, const double* __restrict__ w, double dw,
                                                    const int* __restrict__ spec, const double* __restrict__ Hs,
                                                    const double* __restrict__ Tp, const double* __restrict__ gam,
                                                    double* __restrict__ S, double* __restrict__ zeta) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x, ic = blockIdx.y;
  if (b >= nw) return;
  const double s = sea_spectrum(spec[ic], Hs[ic], Tp[ic], gam[ic], w[b]);
  if (S) S[(size_t)ic * nw + b] = s;
  zeta[(size_t)ic * nw + b] = sqrt(2.0 * s * dw);
}

// ----------------------------------------------------------------------------------------
// k_wave_tables: a workgroup is 64 bins x kWtN node slots of one heading.  Wave s computes
// node nb + s of every pass (the trigonometry and the uhat / kproj rows are independent per
// (node, bin)); its six force contributions go through LDS, and wave 0 adds them to F in node
// order, so F is bitwise the node-serial sum.  kWtN times the waves of a thread-per-bin
// loop: one design's tables (1000 bins) are 128 waves instead of 16.
// ----------------------------------------------------------------------------------------
#ifndef RH_WTN
#define RH_WTN 8
#endif
constexpr int kWtN = RH_WTN;

// One (heading, node, bin): the unit-amplitude Airy velocity uhat and its member-axis
// projections kproj (stored when okb), and the node's inertial-excitation contribution
// f6 = [f; r x f] (raft/raft_fowt.py:1113-1124).
__device__ __forceinline__ void wave_node(const rh_design& d, int h, int n, int b, bool okb, double w, double k,
                                          double cb, double sb, rh_c128* __restrict__ uhat,
                                          rh_c128* __restrict__ kproj, cd (&f6)[6]) {
  const int nw = d.nw, nn = d.nn;
  const double hd = d.depth;
  const double* node = d.node;
  const double x = nf(node, nn, RH_NF_RX, n), y = nf(node, nn, RH_NF_RY, n), z = nf(node, nn, RH_NF_RZ, n);
  const double th = k * (cb * x + sb * y);
  const cd e = mk(cos(th), -sin(th));      // exp(-1j*th)
  double s_sh, c_sh, c_ch;
  if (k * hd > 89.4) {                     // deep-water switch (raft/helpers.py:133-136)
    const double ez = exp(k * z);
    s_sh = ez;
    c_sh = ez;
    c_ch = ez + exp(-k * (z + 2.0 * hd));
  } else {
    const double skh = sinh(k * hd);
    s_sh = sinh(k * (z + hd)) / skh;
    c_sh = cosh(k * (z + hd)) / skh;
    c_ch = cosh(k * (z + hd)) / cosh(k * hd);
  }
  const cd we = scl(e, w);
  const cd u0 = scl(scl(we, c_sh), cb);
  const cd u1 = scl(scl(we, c_sh), sb);
  const cd u2 = scl(iw(w, e), s_sh);
  rh_c128* U = uhat + ((size_t)(h * nn + n) * 3) * nw + b;
  if (okb && uhat) {                        // (uhat NULL: a sweep block's fixed point needs kproj only)
    st(U, u0);
    st(U + nw, u1);
    st(U + 2 * nw, u2);
  }
  {  // projections on the member axes: the drag loop's only view of the wave field
    rh_c128* K = kproj + ((size_t)(h * nn + n) * 3) * nw + b;
    const int fo[3] = {RH_NF_QX, RH_NF_P1X, RH_NF_P2X};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const double e0 = nf(node, nn, fo[a], n), e1 = nf(node, nn, fo[a] + 1, n), e2 = nf(node, nn, fo[a] + 2, n);
      if (okb) st(K + a * nw, add(add(scl(u0, e0), scl(u1, e1)), scl(u2, e2)));
    }
  }
  // inertial excitation: Imat ud + pDyn a_i q, ud = i w u  (raft/raft_fowt.py:1113-1124)
  const cd ud[3] = {iw(w, u0), iw(w, u1), iw(w, u2)};
  const cd pd = scl(scl(e, d.pdyn_rho_g), c_ch);
  const double ai = nf(node, nn, RH_NF_AI, n);
  const double q[3] = {nf(node, nn, RH_NF_QX, n), nf(node, nn, RH_NF_QY, n), nf(node, nn, RH_NF_QZ, n)};
  const cd pa = scl(pd, ai);
  cd f[3];
  if (nf(node, nn, RH_NF_MCF, n) != 0.0) {
    const rh_c128* I = d.imat_mcf + (size_t)n * 9 * nw + b;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      cd s = mul(ld(I + (3 * r + 0) * nw), ud[0]);
      s = add(s, mul(ld(I + (3 * r + 1) * nw), ud[1]));
      s = add(s, mul(ld(I + (3 * r + 2) * nw), ud[2]));
      f[r] = add(s, scl(pa, q[r]));
    }
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      cd s = scl(ud[0], nf(node, nn, RH_NF_I00 + 3 * r + 0, n));
      s = add(s, scl(ud[1], nf(node, nn, RH_NF_I00 + 3 * r + 1, n)));
      s = add(s, scl(ud[2], nf(node, nn, RH_NF_I00 + 3 * r + 2, n)));
      f[r] = add(s, scl(pa, q[r]));
    }
  }
  const double rx = nf(node, nn, RH_NF_XX, n), ry = nf(node, nn, RH_NF_XY, n), rz = nf(node, nn, RH_NF_XZ, n);
  f6[0] = f[0];
  f6[1] = f[1];
  f6[2] = f[2];
  f6[3] = sub(scl(f[2], ry), scl(f[1], rz));
  f6[4] = sub(scl(f[0], rz), scl(f[2], rx));
  f6[5] = sub(scl(f[1], rx), scl(f[0], ry));
}

__device__ __forceinline__ void wave_tables_body(const rh_design& d, const double* __restrict__ beta, int h, int bx,
                                                 rh_c128* __restrict__ uhat, rh_c128* __restrict__ finer,
                                                 rh_c128* __restrict__ kproj, cd (&fs)[kWtN][6][64]) {
  const int lb = (int)threadIdx.x & 63, slot = (int)threadIdx.x >> 6;
  const int nw = d.nw, nn = d.nn;
  const int b0 = bx * 64 + lb;
  const bool okb = b0 < nw;
  const int b = okb ? b0 : nw - 1;           // pad lanes compute a valid bin and store nothing
  const double w = d.w[b], k = d.k[b];
  const double be = beta[h];
  const double cb = cos(be), sb = sin(be);
  cd F[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) F[c] = mk(0, 0);
  for (int nb = 0; nb < nn; nb += kWtN) {
    const int n = nb + slot;
    if (n < nn) {
      cd f6[6];
      wave_node(d, h, n, b, okb, w, k, cb, sb, uhat, kproj, f6);
#pragma unroll
      for (int c = 0; c < 6; ++c) fs[slot][c][lb] = f6[c];
    }
    __syncthreads();
    if (slot == 0) {
      const int ns = nn - nb < kWtN ? nn - nb : kWtN;
      for (int s2 = 0; s2 < ns; ++s2)
#pragma unroll
        for (int c = 0; c < 6; ++c) F[c] = add(F[c], fs[s2][c][lb]);
    }
    __syncthreads();
  }
  if (slot != 0 || !okb) return;
  rh_c128* Fo = finer + (size_t)h * 6 * nw + b;
#pragma unroll
  for (int c = 0; c < 6; ++c) st(Fo + c * nw, F[c]);
}

// One design's tables with the nodes spread over the grid (rh_wave_tables): a workgroup is 64
// bins x kWtN nodes of one heading (blockIdx.z = node group), one node per wave, and every node's
// six force contributions go to fw[h][n][6][nw]; k_wave_force_sum then adds them in node order
// (the same bits as wave_tables_body).  A 1000-bin, 4-heading design is 448 workgroups instead
// of 64, which left three CUs in four idle.
__global__ __launch_bounds__(64 * kWtN) void k_wave_tables_nodes(rh_design d, const double* __restrict__ beta,
                                                                  rh_c128* __restrict__ uhat, rh_c128* __restrict__ kproj,
                                                                  rh_c128* __restrict__ fw) {
  const int lb = (int)threadIdx.x & 63, slot = (int)threadIdx.x >> 6;
  const int nw = d.nw, nn = d.nn, h = (int)blockIdx.y;
  const int n = (int)blockIdx.z * kWtN + slot;
  if (n >= nn) return;                       // uniform per wave
  const int b0 = (int)blockIdx.x * 64 + lb;
  const bool okb = b0 < nw;
  const int b = okb ? b0 : nw - 1;
  const double be = beta[h];
  cd f6[6];
  wave_node(d, h, n, b, okb, d.w[b], d.k[b], cos(be), sin(be), uhat, kproj, f6);
  if (!okb) return;
  rh_c128* o = fw + ((size_t)(h * nn + n) * 6) * nw + b;
#pragma unroll
  for (int c = 0; c < 6; ++c) st(o + c * nw, f6[c]);
}

// finer[h][c][b] = sum over nodes, in node order, of fw[h][n][c][b]
__global__ __launch_bounds__(256) void k_wave_force_sum(int nw, int nn, int nhead, const rh_c128* __restrict__ fw,
                                                        rh_c128* __restrict__ finer) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= nhead * 6 * nw) return;
  const int b = t % nw, c = (t / nw) % 6, h = t / (6 * nw);
  const rh_c128* p = fw + ((size_t)h * nn * 6 + c) * nw + b;
  cd F = mk(0, 0);
  // (the loads of 16 nodes issued ahead of their in-order adds: one thread per (heading, DOF,
  // bin) is only about one wave per CU, so the loop runs on load latency)
#pragma unroll 16
  for (int n = 0; n < nn; ++n) F = add(F, ld(p + (size_t)n * 6 * nw));
  st(finer + ((size_t)h * 6 + c) * nw + b, F);
}

__global__ __launch_bounds__(64 * kWtN) void k_wave_tables(rh_design d, const double* __restrict__ beta,
                                                            rh_c128* __restrict__ uhat, rh_c128* __restrict__ finer,
                                                            rh_c128* __restrict__ kproj) {
  __shared__ cd fs[kWtN][6][64];
  wave_tables_body(d, beta, blockIdx.y, blockIdx.x, uhat, finer, kproj, fs);
}

// Every design of a batch in one launch (rh_wave_tables_batch): blockIdx.z = design, its
// headings beta[z * hstride + h] (h < its nhead), its tables at the pointers of its descriptor.
// A design sweep's tables are then one grid of ndesign x nhead x bins/64 workgroups instead of
// ndesign launches of 16 workgroups each.
__global__ __launch_bounds__(64 * kWtN) void k_wave_tables_batch(const DevDesign* __restrict__ designs,
                                                                  const double* __restrict__ beta, int hstride) {
  __shared__ cd fs[kWtN][6][64];
  const rh_design& d = designs[blockIdx.z].d;
  if ((int)blockIdx.y >= d.nhead || (int)blockIdx.x * 64 >= d.nw) return;   // uniform per workgroup
  wave_tables_body(d, beta + (size_t)blockIdx.z * hstride, blockIdx.y, blockIdx.x, const_cast<rh_c128*>(d.uhat),
                   const_cast<rh_c128*>(d.finer), const_cast<rh_c128*>(d.kproj), fs);
}


template <int NB>
__global__ __launch_bounds__(kThreads, 2) void k_solve_cases(CaseArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ncase = a.c.ncase;
  const int slot = xcd_remap(blockIdx.x, ncase);
  const int ic = a.c.order ? a.c.order[slot] : slot;
  const rh_design& d = a.designs[a.c.design[ic]].d;
  const int nw = d.nw, nn = d.nn;
  const double* node = d.node;
  const int head = a.c.head[ic];
  const int nm = d.nm;
  const rh_c128* Kp = d.kproj + (size_t)head * nn * 3 * nw;
  const rh_c128* Fe = d.finer + (size_t)head * 6 * nw;

  double* red = smem;                     // [kWaves][nn][3]
  double* bm = red + kWaves * nn * 3;     // [nn][9]
  double* bd = bm + nn * 9;               // [36]
  double* sred = bd + 36;                 // [kWaves][6]
  double* mbc = sred + kWaves * 6;        // [108] M, B_lin, C
  double* al = mbc + 108;                 // [nn][5] drag coefficients per node
  double* mred = al + nn * 5;             // [kWaves] per-wave max of tolCheck
  load_mbc(d, mbc, tid);

  const int spec = a.c.spectrum[ic];
  const double Hs = a.c.Hs[ic], Tp = a.c.Tp[ic], gam = a.c.gamma[ic];
  double zt[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int b = tid + kThreads * j;
    zt[j] = (b < nw) ? sea_amplitude(spec, Hs, Tp, gam, d.w[b], d.dw) : 0.0;
    if (b < nw && a.o.zeta) a.o.zeta[(size_t)ic * nw + b] = zt[j];
  }
  rh_c128* Xo = a.o.Xi ? a.o.Xi + (size_t)ic * 6 * nw : nullptr;   // NULL: no response wanted
  rh_c128* XL = a.o.Xi_last + (size_t)ic * 6 * nw;
  const rh_c128* XI0 = a.c.Xi_init ? a.c.Xi_init + (size_t)ic * 6 * nw : nullptr;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int b = tid + kThreads * j;
    if (b < nw)
#pragma unroll
      for (int c = 0; c < 6; ++c) st(XL + c * nw + b, XI0 ? ld(XI0 + c * nw + b) : mk(a.c.XiStart, 0.0));
  }
  rh_c128* XP = a.o.Xi_prev ? a.o.Xi_prev + (size_t)ic * 6 * nw : nullptr;

  const int nloop = a.c.nIter + 1;
  const double tol = a.c.tol;
  int status = RH_CASE_NOT_CONVERGED, iters = nloop;
  double margin = INFINITY;   // closest call of the convergence test (rh_solve_out.margin)
  for (int it = a.c.first_iter; it < nloop; ++it) {
    // ---------------- A: per-node sums of squared relative-velocity components ----------
    // Member-factored (see rh_member_field): per (member, bin) the motion terms
    //   Bq = iw cq.Xi, B1 = iw c1.Xi, B2 = iw c2.Xi, E1 = iw p2.th, E2 = -iw p1.th
    // then per node  s_q = z Kq - Bq,  s_1 = z K1 - (B1 + t E1),  s_2 = z K2 - (B2 + t E2)
    // are the relative-velocity projections of raft/raft_fowt.py:1205-1211.
    for (int m = 0; m < nm; ++m) {
      const int n0 = d.mstart[m], n1 = d.mstart[m + 1];
      double cq[6], c1[6], c2[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        cq[i] = d.memb[(RH_MF_CQ0 + i) * nm + m];
        c1[i] = d.memb[(RH_MF_C10 + i) * nm + m];
        c2[i] = d.memb[(RH_MF_C20 + i) * nm + m];
      }
      cd Bq[NB], B1[NB], B2[NB], E1[NB], E2[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int b = tid + kThreads * j;
        const int bc = b < nw ? b : nw - 1;     // unpredicated loads, pad lanes zeroed after
        cd X[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          const cd v = ld(XL + c * nw + bc);
          X[c] = (b < nw) ? v : mk(0, 0);
        }
        const double wl = d.w[bc];
        const double w = (b < nw) ? wl : 0.0;
        cd Aq = mk(0, 0), A1 = mk(0, 0), A2 = mk(0, 0);
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          Aq = add(Aq, scl(X[c], cq[c]));
          A1 = add(A1, scl(X[c], c1[c]));
          A2 = add(A2, scl(X[c], c2[c]));
        }
        const cd D1 = add(add(scl(X[3], c2[0]), scl(X[4], c2[1])), scl(X[5], c2[2]));   // p2 . th
        const cd D2 = add(add(scl(X[3], c1[0]), scl(X[4], c1[1])), scl(X[5], c1[2]));   // p1 . th
        Bq[j] = iw(w, Aq);
        B1[j] = iw(w, A1);
        B2[j] = iw(w, A2);
        E1[j] = iw(w, D1);
        E2[j] = iw(-w, D2);
      }
      for (int n = n0; n < n1; ++n) {
        const double t = nf(node, nn, RH_NF_T, n);
        const rh_c128* K = Kp + (size_t)n * 3 * nw;
        double s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          // pad lanes (b >= nw) read the last bin and add exactly 0: zeta = 0 and XiLast = 0
          const int b = tid + kThreads * j < nw ? tid + kThreads * j : nw - 1;
          const double z = zt[j];
          const cd sq = sub(scl(ld(K + b), z), Bq[j]);
          const cd sp1 = sub(scl(ld(K + nw + b), z), add(B1[j], scl(E1[j], t)));
          const cd sp2 = sub(scl(ld(K + 2 * nw + b), z), add(B2[j], scl(E2[j], t)));
          s0 += abs2(sq);
          s1 += abs2(sp1);
          s2 += abs2(sp2);
        }
        s0 = wave_sum(s0);
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        if (lane == 0) {
          double* R = red + (wv * nn + n) * 3;
          R[0] = s0;
          R[1] = s1;
          R[2] = s2;
        }
      }
    }
    __syncthreads();
    // ---------------- B: node drag matrices and B_drag ----------------------------------
    for (int n = tid; n < nn; n += kThreads) {
      double r3[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        double s = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += red[(w * nn + n) * 3 + c];
        r3[c] = s;
      }
      // sum|vrel_q|^2 = sum|s_q|^2 |q|^2 ; circular: |vrel_p|^2 = |s_1|^2|p1|^2 + |s_2|^2|p2|^2
      const double qq = nrm2(node, nn, RH_NF_QX, n), pp1 = nrm2(node, nn, RH_NF_P1X, n), pp2 = nrm2(node, nn, RH_NF_P2X, n);
      const bool circ = nf(node, nn, RH_NF_CIRC, n) != 0.0;
      const double sums[3] = {r3[0] * qq, circ ? r3[1] * pp1 + r3[2] * pp2 : r3[1] * pp1, r3[2] * pp2};
      double B4[4];
      node_bmat(node, nn, n, d.rho, sums, bm + 9 * n, B4);
      const double t = nf(node, nn, RH_NF_T, n);
      double* A = al + 5 * n;
      A[0] = B4[0] + B4[3];     // axial: side + end   (qMat terms of Bmat, raft/raft_fowt.py:1228-1248)
      A[1] = B4[1];
      A[2] = B4[2];
      A[3] = t * B4[1];
      A[4] = t * B4[2];
    }
    __syncthreads();
    if (tid < 36) {
      const int i = tid / 6, j = tid % 6;
      double s = 0;
      for (int n = 0; n < nn; ++n)
        s += t3to6(bm + 9 * n, nf(node, nn, RH_NF_XX, n), nf(node, nn, RH_NF_XY, n), nf(node, nn, RH_NF_XZ, n), i, j);
      bd[tid] = s;
    }
    __syncthreads();
    // ---------------- C: excitation, Z(w), LU solve, convergence flags ------------------
    bool my_ok = true, my_nan = false, my_sing = false;
    double my_tmax = 0.0;
    // No lane branches around the register-heavy solve: lanes past the grid (b >= nw)
    // recompute the last bin and store nothing.  (A divergent region here -- a per-lane
    // `continue` -- let the compiler's spills of SGPR-holding VGPRs run under a partial EXEC
    // mask and lose lanes: wrong tables for some cases, caught by the kernel cross-check.)
#pragma unroll 1
    for (int j = 0; j < NB; ++j) {
      const int b0 = tid + kThreads * j;
      if (!__builtin_amdgcn_ballot_w64(b0 < nw)) continue;   // whole wave past the grid: uniform
      const bool okb = b0 < nw;
      const int b = okb ? b0 : nw - 1;
      const double w = d.w[b];
      // zeta of bin j by a select chain: zt[j] with the loop index j would be a dynamic index
      // into a register array (s_set_gpr_idx), which tools/isa_check.py refuses
      double zj = zt[0];
#pragma unroll
      for (int jj = 1; jj < NB; ++jj) zj = j == jj ? zt[jj] : zj;
      cd F[6];
      drag_exc_members(d, al, Kp, nw, b, F);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        cd f = add(scl(ld(Fe + c * nw + b), zj), scl(F[c], zj));   // F_lin + F_drag
        if (a.c.fext) f = add(f, ld(a.c.fext + ((size_t)ic * 6 + c) * nw + b));
        F[c] = f;
      }
      cd Z[6][6];
      assemble_z(d, mbc, b, w, bd, Z);
      if (a.o.Z && okb) {
        rh_c128* Zo = a.o.Z + ((size_t)ic * nw + b) * 36;
#pragma unroll
        for (int e = 0; e < 36; ++e) st(Zo + e, Z[e / 6][e % 6]);
      }
      const bool ok_lu = lu_solve<6>(Z, F);
      my_sing |= okb && !ok_lu;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const cd x = F[c];
        const cd xlast = ld(XL + c * nw + b);
        // tolCheck = |Xi - XiLast| / (|Xi| + tol) < tol  (raft/raft_model.py:961-962)
        const double t = cabs(sub(x, xlast)) / (cabs(x) + tol);
        if (okb) {
          my_nan |= (x.r != x.r) || (x.i != x.i);
          my_ok = my_ok && (t < tol);
          my_tmax = fmax(my_tmax, t);
          if (Xo) st(Xo + c * nw + b, x);
          if (XP) st(XP + c * nw + b, xlast);
          // XiLast = 0.2 XiLast + 0.8 Xi  (:991), only consumed if not converged
          st(XL + c * nw + b, add(scl(xlast, 0.2), scl(x, 0.8)));
        }
      }
    }
    if (a.o.margin) {
      const double mw = wave_max(my_tmax);
      if (lane == 0) mred[wv] = mw;
    }
    const int all_ok = __syncthreads_and(my_ok ? 1 : 0);
    if (a.o.margin && tid == 0) {   // mred is rewritten only after the next phase-A barrier
      double mx = mred[0];
      for (int w = 1; w < kWaves; ++w) mx = fmax(mx, mred[w]);
      margin = closer_call(margin, mx - tol);
    }
    const int any_nan = __syncthreads_or(my_nan ? 1 : 0);
    const int any_sing = __syncthreads_or(my_sing ? 1 : 0);
    if (any_nan) {
      status = RH_CASE_NAN;
      iters = it + 1;
      break;
    }
    if (any_sing) {
      status = RH_CASE_SINGULAR;
      iters = it + 1;
      break;
    }
    if (all_ok) {
      status = RH_CASE_CONVERGED;
      iters = it + 1;
      break;
    }
  }

  // ---------------- outputs ------------------------------------------------------------
  if (tid == 0) {
    a.o.iters[ic] = iters;
    a.o.status[ic] = status;
    if (a.o.margin) a.o.margin[ic] = margin;
  }
  if (a.o.B_drag && tid < 36) a.o.B_drag[(size_t)ic * 36 + tid] = bd[tid];
  if (a.o.Bmat)
    for (int e = tid; e < nn * 9; e += kThreads) a.o.Bmat[(size_t)ic * a.bmat_nn * 9 + e] = bm[e];
  if (a.o.F_wave) {   // the excitation with the final linearisation (the arithmetic of phase C)
#pragma unroll 1
    for (int j = 0; j < NB; ++j) {
      const int b = tid + kThreads * j;
      if (b >= nw) continue;
      double zj = zt[0];   // (a select chain, as in phase C: no dynamic register index)
#pragma unroll
      for (int jj = 1; jj < NB; ++jj) zj = j == jj ? zt[jj] : zj;
      cd F[6];
      drag_exc_members(d, al, Kp, nw, b, F);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        cd f = add(scl(ld(Fe + c * nw + b), zj), scl(F[c], zj));
        if (a.c.fext) f = add(f, ld(a.c.fext + ((size_t)ic * 6 + c) * nw + b));
        F[c] = f;
      }
#pragma unroll
      for (int c = 0; c < 6; ++c) st(a.o.F_wave + ((size_t)ic * 6 + c) * nw + b, F[c]);
    }
  }
  // a case that stopped on a NaN or a singular Z has no response (the reference raises there,
  // raft/raft_model.py:957): NaN Xi, F_wave, PSD, RAO and std, as k_solve_lds writes them
  if (status == RH_CASE_NAN || status == RH_CASE_SINGULAR) {   // uniform
#pragma unroll 1
    for (int j = 0; j < NB; ++j) {
      const int b = tid + kThreads * j;
      if (b >= nw) continue;
#pragma unroll 1
      for (int c = 0; c < 6; ++c) {
        if (Xo) st(Xo + c * nw + b, mk(NAN, NAN));
        if (a.o.F_wave) st(a.o.F_wave + ((size_t)ic * 6 + c) * nw + b, mk(NAN, NAN));   // no excitation either
        if (a.o.psd) a.o.psd[((size_t)ic * 6 + c) * nw + b] = NAN;
        if (a.o.rao) st(a.o.rao + ((size_t)ic * 6 + c) * nw + b, mk(NAN, NAN));
      }
    }
    if (a.o.std && tid < 6) a.o.std[(size_t)ic * 6 + tid] = NAN;
  } else if (a.o.psd || a.o.std || a.o.rao) {
    double ss[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int b = tid + kThreads * j;
      if (b >= nw) continue;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const cd x = ld(Xo + c * nw + b);
        const cd xd = c >= 3 ? scl(x, kRad2Deg) : x;
        const double m2 = abs2(xd);
        ss[c] += m2;
        if (a.o.psd) a.o.psd[((size_t)ic * 6 + c) * nw + b] = 0.5 * m2 / d.dw;
        if (a.o.rao) {
          const double z = zt[j];
          st(a.o.rao + ((size_t)ic * 6 + c) * nw + b, fabs(z) > 1e-6 ? cd{x.r / z, x.i / z} : mk(0, 0));
        }
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
        for (int w = 0; w < kWaves; ++w) s += sred[w * 6 + tid];
        a.o.std[(size_t)ic * 6 + tid] = sqrt(0.5 * s);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// k_heading_resp: thread per (case, bin)
// ----------------------------------------------------------------------------------------
struct HeadArgs {
  const DevDesign* designs;
  int ncase;
  const int* design_idx;
  const int* head;
  const double* zeta;
  const double* B_drag;
  const double* Bmat;      // [ncase][bmat_nn][9]
  rh_c128* Xi;
  rh_c128* F;             // non-NULL: store the wave excitation only (no solve)
  int bmat_nn;            // node stride of Bmat (rh_heading_response_ext's bmat_nn)
  int ndesign;            // designs[] entries: a design index outside [0, ndesign) is not read
  const rh_c128* fext;    // [ncase][6][nw] added to the excitation (Fhydro_2nd, raft/raft_model.py:1061), or NULL
};

__global__ __launch_bounds__(kThreads, 2) void k_heading_resp(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int ic = blockIdx.y;
  const int di = a.design_idx[ic];
  if (di < 0 || di >= a.ndesign || a.head[ic] < 0 || a.head[ic] >= a.designs[di].d.nhead) {
    // uniform per block: a bad design or heading index from the caller reads no table and
    // leaves NaN in this case's rows (never plausible-looking stale memory)
    const int nw0 = a.designs[0].d.nw;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nw0) {
      const double nan = __builtin_nan("");
      rh_c128* out = a.F ? a.F : a.Xi;
#pragma unroll
      for (int c = 0; c < 6; ++c) out[((size_t)ic * 6 + c) * nw0 + b] = rh_c128{nan, nan};
    }
    return;
  }
  const rh_design& d = a.designs[di].d;
  const int nw = d.nw, nn = d.nn;
  double* bm = smem;
  double* bd = bm + 9 * nn;
  double* mbc = bd + 36;
  load_mbc(d, mbc, threadIdx.x);
  for (int e = threadIdx.x; e < nn * 9; e += blockDim.x) bm[e] = a.Bmat[(size_t)ic * a.bmat_nn * 9 + e];
  if (threadIdx.x < 36 && a.B_drag) bd[threadIdx.x] = a.B_drag[(size_t)ic * 36 + threadIdx.x];
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nw) return;
  const int head = a.head[ic];
  const rh_c128* Uh = d.uhat + (size_t)head * nn * 3 * nw;
  const rh_c128* Fe = d.finer + (size_t)head * 6 * nw;
  const double z = a.zeta[(size_t)ic * nw + b];
  cd F[6];
  drag_exc_bin(d.node, nn, bm, Uh, nw, b, F);
#pragma unroll
  for (int c = 0; c < 6; ++c) F[c] = add(scl(ld(Fe + c * nw + b), z), scl(F[c], z));
  if (a.fext) {
#pragma unroll
    for (int c = 0; c < 6; ++c) F[c] = add(F[c], ld(a.fext + ((size_t)ic * 6 + c) * nw + b));
  }
  if (a.F) {              // F_wave of raft/raft_model.py:1049-1061 for the system solve
#pragma unroll
    for (int c = 0; c < 6; ++c) st(a.F + ((size_t)ic * 6 + c) * nw + b, F[c]);
    return;
  }
  cd Z[6][6];
  assemble_z(d, mbc, b, d.w[b], bd, Z);
  lu_solve<6>(Z, F);
#pragma unroll
  for (int c = 0; c < 6; ++c) st(a.Xi + ((size_t)ic * 6 + c) * nw + b, F[c]);
}

// ----------------------------------------------------------------------------------------
// stand-alone linearisation (FOWT.calcHydroLinearization for a given Xi)
// ----------------------------------------------------------------------------------------
// pass 1: block per node, reduce over bins
// Block-wide per-node sums of |vrel_q|^2, |vrel_p|^2 (or |vrel_p1|^2, |vrel_p2|^2) over the
// bins [lo, hi) of Xi (raft/raft_fowt.py:1205-1220), bins strided over the block; returns
// the three sums in thread 0.  Fixed order (per-thread bins, butterflies, waves in order).
__device__ __forceinline__ void lin_node_sums(const rh_design& d, int head, const rh_c128* __restrict__ Xi,
                                              const double* __restrict__ zeta, int n, int lo, int hi,
                                              double (&red)[kWaves][3], double (&out)[3]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nw = d.nw, nn = d.nn;
  const double* node = d.node;
  const rh_c128* U = d.uhat + ((size_t)head * nn + n) * 3 * nw;
  const double rx = nf(node, nn, RH_NF_XX, n), ry = nf(node, nn, RH_NF_XY, n), rz = nf(node, nn, RH_NF_XZ, n);
  const double q0 = nf(node, nn, RH_NF_QX, n), q1 = nf(node, nn, RH_NF_QY, n), q2 = nf(node, nn, RH_NF_QZ, n);
  const double a0 = nf(node, nn, RH_NF_P1X, n), a1 = nf(node, nn, RH_NF_P1Y, n), a2 = nf(node, nn, RH_NF_P1Z, n);
  const double b0 = nf(node, nn, RH_NF_P2X, n), b1 = nf(node, nn, RH_NF_P2Y, n), b2 = nf(node, nn, RH_NF_P2Z, n);
  const bool circ = nf(node, nn, RH_NF_CIRC, n) != 0.0;
  double s0 = 0, s1 = 0, s2 = 0;
  for (int b = lo + tid; b < hi; b += kThreads) {
    const double w = d.w[b], z = zeta[b];
    const cd u0 = scl(ld(U + b), z), u1 = scl(ld(U + nw + b), z), u2 = scl(ld(U + 2 * nw + b), z);
    cd X[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) X[c] = ld(Xi + c * nw + b);
    const cd dr0 = add(X[0], add(scl(X[5], -ry), scl(X[4], rz)));
    const cd dr1 = add(X[1], sub(scl(X[5], rx), scl(X[3], rz)));
    const cd dr2 = add(X[2], add(scl(X[4], -rx), scl(X[3], ry)));
    const cd v0 = sub(u0, iw(w, dr0)), v1 = sub(u1, iw(w, dr1)), v2 = sub(u2, iw(w, dr2));
    const cd sq = add(add(scl(v0, q0), scl(v1, q1)), scl(v2, q2));
    const cd vq0 = scl(sq, q0), vq1 = scl(sq, q1), vq2 = scl(sq, q2);
    s0 += abs2(vq0) + abs2(vq1) + abs2(vq2);
    if (circ) {
      s1 += abs2(sub(v0, vq0)) + abs2(sub(v1, vq1)) + abs2(sub(v2, vq2));
    } else {
      const cd s_1 = add(add(scl(v0, a0), scl(v1, a1)), scl(v2, a2));
      const cd s_2 = add(add(scl(v0, b0), scl(v1, b1)), scl(v2, b2));
      s1 += abs2(scl(s_1, a0)) + abs2(scl(s_1, a1)) + abs2(scl(s_1, a2));
      s2 += abs2(scl(s_2, b0)) + abs2(scl(s_2, b1)) + abs2(scl(s_2, b2));
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  if (lane == 0) {
    red[wv][0] = s0;
    red[wv][1] = s1;
    red[wv][2] = s2;
  }
  __syncthreads();
  if (tid == 0) {
    for (int c = 0; c < 3; ++c) {
      double s = 0;
      for (int w = 0; w < kWaves; ++w) s += red[w][c];
      out[c] = s;
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_lin_sums(rh_design d, int head, const rh_c128* __restrict__ Xi,
                                                       const double* __restrict__ zeta, double* __restrict__ Bmat) {
  __shared__ double red[kWaves][3];
  double sums[3];
  const int n = blockIdx.x;
  lin_node_sums(d, head, Xi, zeta, n, 0, d.nw, red, sums);
  if (threadIdx.x == 0) node_bmat(d.node, d.nn, n, d.rho, sums, Bmat + 9 * n);
}

// ----------------------------------------------------------------------------------------
// bin-sharded drag fixed point: one case, bins split over ranks
// ----------------------------------------------------------------------------------------
// step 1: this rank's partial node sums over bins [lo, hi), block per node
__global__ __launch_bounds__(kThreads) void k_lin_partial(rh_design d, int head, const rh_c128* __restrict__ Xi,
                                                          const double* __restrict__ zeta, int lo, int hi,
                                                          double* __restrict__ sums) {
  __shared__ double red[kWaves][3];
  double s[3];
  const int n = blockIdx.x;
  lin_node_sums(d, head, Xi, zeta, n, lo, hi, red, s);
  if (threadIdx.x == 0)
    for (int c = 0; c < 3; ++c) sums[3 * n + c] = s[c];
}

// step 2 (after the caller's all-reduce of the sums): node drag matrices and B_drag from the
// global sums (every block, into LDS; block 0 also writes them out), then thread per bin of
// [lo, hi): drag + inertial excitation (+ fext), Z(w), LU, tolCheck and relaxation of XiLast
// (raft/raft_model.py:942-991, the arithmetic of k_heading_resp / k_solve_cases).
// flags (caller-zeroed): [0] some bin not converged, [1] NaN, [2] singular.
__global__ __launch_bounds__(kThreads) void k_bin_step(rh_design d, int head, const double* __restrict__ zeta,
                                                       const rh_c128* __restrict__ fext, const double* __restrict__ sums,
                                                       double tol, int lo, int hi, double* __restrict__ Bmat_out,
                                                       double* __restrict__ Bd_out, rh_c128* __restrict__ Xi,
                                                       rh_c128* __restrict__ XL, int* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nw = d.nw, nn = d.nn, tid = threadIdx.x;
  double* bm = smem;            // [nn][9]
  double* bd = bm + 9 * nn;     // [36]
  double* mbc = bd + 36;        // [108]
  load_mbc(d, mbc, tid);
  for (int n = tid; n < nn; n += blockDim.x) {
    const double s3[3] = {sums[3 * n], sums[3 * n + 1], sums[3 * n + 2]};
    node_bmat(d.node, nn, n, d.rho, s3, bm + 9 * n);
  }
  __syncthreads();
  if (tid < 36) {
    double s = 0;
    for (int n = 0; n < nn; ++n)
      s += t3to6(bm + 9 * n, nf(d.node, nn, RH_NF_XX, n), nf(d.node, nn, RH_NF_XY, n), nf(d.node, nn, RH_NF_XZ, n),
                 tid / 6, tid % 6);
    bd[tid] = s;
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    for (int e = tid; e < 9 * nn; e += blockDim.x) Bmat_out[e] = bm[e];
    if (tid < 36) Bd_out[tid] = bd[tid];
  }
  const int b = lo + blockIdx.x * blockDim.x + tid;
  int bad = 0;
  if (b < hi) {
    const rh_c128* Uh = d.uhat + (size_t)head * nn * 3 * nw;
    const rh_c128* Fe = d.finer + (size_t)head * 6 * nw;
    const double z = zeta[b];
    cd F[6];
    drag_exc_bin(d.node, nn, bm, Uh, nw, b, F);
#pragma unroll
    for (int c = 0; c < 6; ++c) F[c] = add(scl(ld(Fe + c * nw + b), z), scl(F[c], z));
    if (fext) {
#pragma unroll
      for (int c = 0; c < 6; ++c) F[c] = add(F[c], ld(fext + c * nw + b));
    }
    cd Z[6][6];
    assemble_z(d, mbc, b, d.w[b], bd, Z);
    if (!lu_solve<6>(Z, F)) bad |= 4;
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const cd x = F[c], xl = ld(XL + c * nw + b);
      if ((x.r != x.r) || (x.i != x.i)) bad |= 2;
      const double tt = sqrt(abs2(sub(x, xl))) / (sqrt(abs2(x)) + tol);   // raft/raft_model.py:961-962
      ok = ok && (tt < tol);
      st(Xi + c * nw + b, x);
      st(XL + c * nw + b, add(scl(xl, 0.2), scl(x, 0.8)));                 // :991
    }
    if (!ok) bad |= 1;
  }
#pragma unroll
  for (int q = 0; q < 3; ++q)
    if (__builtin_amdgcn_ballot_w64((bad >> q) & 1) != 0 && (tid & 63) == 0) atomicMax(flags + q, 1);
}

// pass 2: B_drag (36 threads) -- sequential node order like the reference's running sum
__global__ void k_lin_bdrag(rh_design d, const double* __restrict__ Bmat, double* __restrict__ B_drag) {
  const int t = threadIdx.x;
  if (t >= 36) return;
  const int nn = d.nn;
  double s = 0;
  for (int n = 0; n < nn; ++n)
    s += t3to6(Bmat + 9 * n, nf(d.node, nn, RH_NF_XX, n), nf(d.node, nn, RH_NF_XY, n), nf(d.node, nn, RH_NF_XZ, n),
               t / 6, t % 6);
  B_drag[t] = s;
}

// drag excitation for a given Bmat: thread per bin
__global__ __launch_bounds__(kThreads) void k_drag_exc(rh_design d, int head, const double* __restrict__ zeta,
                                                        const double* __restrict__ Bmat, rh_c128* __restrict__ Fd) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nw = d.nw, nn = d.nn;
  for (int e = threadIdx.x; e < nn * 9; e += blockDim.x) smem[e] = Bmat[e];
  __syncthreads();
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nw) return;
  const rh_c128* Uh = d.uhat + (size_t)head * nn * 3 * nw;
  cd F[6];
  drag_exc_bin(d.node, nn, smem, Uh, nw, b, F);
  const double z = zeta[b];
#pragma unroll
  for (int c = 0; c < 6; ++c) st(Fd + c * nw + b, scl(F[c], z));
}

// motion statistics over rows: block per case
__global__ __launch_bounds__(kThreads) void k_motion_stats(int nrow, int nw, double dw, const rh_c128* __restrict__ Xi,
                                                            double* __restrict__ psd, double* __restrict__ stdv) {
  __shared__ double sred[kWaves][6];
  const int ic = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double ss[6] = {0, 0, 0, 0, 0, 0};
  for (int b = tid; b < nw; b += kThreads) {
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      double p = 0;
      for (int r = 0; r < nrow; ++r) {
        const cd x = ld(Xi + (((size_t)ic * nrow + r) * 6 + c) * nw + b);
        const double m2 = abs2(c >= 3 ? scl(x, kRad2Deg) : x);
        p += 0.5 * m2 / dw;
        ss[c] += m2;
      }
      if (psd) psd[((size_t)ic * 6 + c) * nw + b] = p;
    }
  }
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    const double s = wave_sum(ss[c]);
    if (lane == 0) sred[wv][c] = s;
  }
  __syncthreads();
  if (tid < 6 && stdv) {
    double s = 0;
    for (int w = 0; w < kWaves; ++w) s += sred[w][tid];
    stdv[(size_t)ic * 6 + tid] = sqrt(0.5 * s);
  }
}

// Derived response channels (raft/raft_fowt.py:1900-1971 with zero aero loads: nacelle
// acceleration AxRNA and tower-base bending Mbase; mooring tensions J_moor Xi, :1884-1898):
// real linear combinations of the DOFs with an optional w^2 term,
//   x_k(row, b) = sum_d a[k][d] Xi[row][d][b] + w_b^2 sum_d c[k][d] Xi[row][d][b]
// psd[k][b] = sum_row 0.5 |x_k|^2 / dw (getPSD), std[k] = sqrt(0.5 sum_{row,b} |x_k|^2)
// (getRMS, raft/helpers.py:581-603).  coef: [nch][2][ndof] = {a, c}.  Block per (channel, case).
__global__ __launch_bounds__(kThreads) void k_channel_stats(int nrow, int ndof, int nw, double dw,
                                                             const double* __restrict__ w, const rh_c128* __restrict__ Xi,
                                                             int nch, const double* __restrict__ coef,
                                                             double* __restrict__ psd, double* __restrict__ stdv) {
  __shared__ double sred[kWaves];
  const int k = blockIdx.x, ic = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const double* A = coef + (size_t)k * 2 * ndof;
  const double* C = A + ndof;
  double ss = 0;
  for (int b = tid; b < nw; b += kThreads) {
    const double w2 = w[b] * w[b];
    double p = 0;
    for (int r = 0; r < nrow; ++r) {
      const rh_c128* X = Xi + ((size_t)ic * nrow + r) * ndof * nw + b;
      cd xa = mk(0, 0), xc = mk(0, 0);
      for (int dof = 0; dof < ndof; ++dof) {
        const double a = A[dof], c = C[dof];
        if (a == 0.0 && c == 0.0) continue;          // uniform: the coefficient rows are shared
        const cd x = ld(X + (size_t)dof * nw);
        xa = add(xa, scl(x, a));
        xc = add(xc, scl(x, c));
      }
      const double m2 = abs2(add(xa, scl(xc, w2)));
      p += 0.5 * m2 / dw;
      ss += m2;
    }
    if (psd) psd[((size_t)ic * nch + k) * nw + b] = p;
  }
  const double s = wave_sum(ss);
  if (lane == 0) sred[wv] = s;
  __syncthreads();
  if (tid == 0 && stdv) {
    double t = 0;
    for (int i = 0; i < kWaves; ++i) t += sred[i];
    stdv[(size_t)ic * nch + k] = sqrt(0.5 * t);
  }
}

// coupled array solve (raft/raft_model.py:1021-1065), thread per bin, matrix in LDS
// (6N x 6N with N <= 2 FOWTs is too large for registers; this path is not throughput-critical).
constexpr int kSysThreads = 32;
__global__ __launch_bounds__(kSysThreads) void k_system_solve(int N, int nw, const rh_c128* __restrict__ Z,
                                                                const double* __restrict__ K,
                                                                const rh_c128* __restrict__ F, rh_c128* __restrict__ Xi) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int t = threadIdx.x;
  const int b = blockIdx.x * blockDim.x + t;
  {                       // case blockIdx.y of a batch: [ncase][nf][nw][36], [ncase][N][nw]
    const size_t ic = blockIdx.y;
    Z += ic * (size_t)(N / 6) * nw * 36;
    F += ic * (size_t)N * nw;
    Xi += ic * (size_t)N * nw;
  }
  // A[i][j] of this thread at smem[2*((i*N + j)*kSysThreads + t)], x[i] after the matrix
  auto Ar = [&](int i, int j) -> double& { return smem[2 * ((i * N + j) * kSysThreads + t)]; };
  auto Ai = [&](int i, int j) -> double& { return smem[2 * ((i * N + j) * kSysThreads + t) + 1]; };
  double* xs = smem + 2 * N * N * kSysThreads;
  auto xr = [&](int i) -> double& { return xs[2 * (i * kSysThreads + t)]; };
  auto xi = [&](int i) -> double& { return xs[2 * (i * kSysThreads + t) + 1]; };
  if (b >= nw) return;
  const int nf = N / 6;
  for (int i = 0; i < N; ++i) {
    for (int j = 0; j < N; ++j) {
      Ar(i, j) = K ? K[i * N + j] : 0.0;
      Ai(i, j) = 0.0;
    }
    const cd f = ld(F + (size_t)i * nw + b);
    xr(i) = f.r;
    xi(i) = f.i;
  }
  for (int f = 0; f < nf; ++f)
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) {
        const cd z = ld(Z + ((size_t)f * nw + b) * 36 + 6 * i + j);
        // Z_sys[i1:i2, i1:i2] += fowt.Z then += K : the reference adds K after the blocks
        const double kr = Ar(6 * f + i, 6 * f + j);
        Ar(6 * f + i, 6 * f + j) = z.r + kr;
        Ai(6 * f + i, 6 * f + j) = z.i;
      }
  for (int k = 0; k < N; ++k) {
    int p = k;
    double best = fabs(Ar(k, k)) + fabs(Ai(k, k));
    for (int i = k + 1; i < N; ++i) {
      const double v = fabs(Ar(i, k)) + fabs(Ai(i, k));
      if (v > best) { best = v; p = i; }
    }
    if (p != k) {
      for (int j = k; j < N; ++j) {
        double tr = Ar(k, j), ti = Ai(k, j);
        Ar(k, j) = Ar(p, j); Ai(k, j) = Ai(p, j);
        Ar(p, j) = tr; Ai(p, j) = ti;
      }
      double tr = xr(k), ti = xi(k);
      xr(k) = xr(p); xi(k) = xi(p);
      xr(p) = tr; xi(p) = ti;
    }
    const cd rinv = cdiv(mk(1.0, 0.0), best != 0.0 ? mk(Ar(k, k), Ai(k, k)) : mk(1.0, 0.0));
    for (int i = k + 1; i < N; ++i) {
      const cd l = mul(mk(Ar(i, k), Ai(i, k)), rinv);
      for (int j = k + 1; j < N; ++j) {
        const cd v = sub(mk(Ar(i, j), Ai(i, j)), mul(l, mk(Ar(k, j), Ai(k, j))));
        Ar(i, j) = v.r; Ai(i, j) = v.i;
      }
      const cd v = sub(mk(xr(i), xi(i)), mul(l, mk(xr(k), xi(k))));
      xr(i) = v.r; xi(i) = v.i;
    }
  }
  for (int k = N - 1; k >= 0; --k) {
    cd s = mk(xr(k), xi(k));
    for (int j = k + 1; j < N; ++j) s = sub(s, mul(mk(Ar(k, j), Ai(k, j)), mk(xr(j), xi(j))));
    s = cdiv(s, mk(Ar(k, k), Ai(k, k)));
    xr(k) = s.r; xi(k) = s.i;
    st(Xi + (size_t)k * nw + b, s);
  }
}

// The array system per (case, bin) in registers (raft/raft_model.py:1021-1040, 1065: Z_sys =
// blockdiag(fowt.Z) + K_array, Xi = inv(Z_sys) F).  One FOWT: a 6x6 LU.  Two FOWTs: the 12x12
// system by its 6x6 blocks, Z_sys = [[A, K12], [K21, D]] (A = Z1 + K11, D = Z2 + K22):
//   X = A^-1 K12,  S = D - K21 X,  x2 = S^-1 (f2 - K21 A^-1 f1),  x1 = A^-1 f1 - X x2
// with A factored once for its 7 right-hand sides.  The same solution as the
// 12 x 12 elimination up to rounding (the reference inverts Z_sys with LAPACK); a 12 x 12
// complex matrix per lane would need 576 VGPRs.  One lane per bin, 64 lanes per block.
template <int NF>
__global__ __launch_bounds__(64) void k_system_solve_reg(int nw, const rh_c128* __restrict__ Z, const double* __restrict__ K,
                                                         const rh_c128* __restrict__ F, rh_c128* __restrict__ Xi) {
  constexpr int N = 6 * NF;
  __shared__ double ks[N * N];   // K_array staged in LDS: uniform reads, no scalar-register pressure
  for (int e = threadIdx.x; e < N * N; e += 64) ks[e] = K ? K[e] : 0.0;
  __syncthreads();
  const int b0 = blockIdx.x * 64 + threadIdx.x;
  const bool live = b0 < nw;
  const int b = live ? b0 : nw - 1;          // pad lanes solve the last bin and store nothing
  const size_t ic = blockIdx.y;
  Z += ic * (size_t)NF * nw * 36;
  F += ic * (size_t)N * nw;
  Xi += ic * (size_t)N * nw;
  int zo;                        // a zero the compiler cannot see through: the K reads stay where
  asm volatile("s_mov_b32 %0, 0" : "=s"(zo));   // they are used instead of being hoisted into registers
  const double* ksz = ks + zo;
  auto kk = [&](int i, int j) { return ksz[i * N + j]; };
  auto zload = [&](int f, cd (&A)[6][6]) {   // (0 + Z_f) + K_ff, the reference's order of additions
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const cd z = ld(Z + ((size_t)f * nw + b) * 36 + 6 * i + j);
        A[i][j] = mk(z.r + kk(6 * f + i, 6 * f + j), z.i);
      }
  };
  if constexpr (NF == 1) {
    cd A[6][6], x[6];
    zload(0, A);
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = ld(F + (size_t)i * nw + b);
    lu_solve<6>(A, x);
    if (live)
#pragma unroll
      for (int i = 0; i < 6; ++i) st(Xi + (size_t)i * nw + b, x[i]);
  } else {
    // X = A^-1 K12 goes column by column to a lane-private LDS slab [36][re, im][64 lanes], so
    // A (factored) and S never occupy registers together
    __shared__ double xs[36 * 2 * 64];
    const int ln = threadIdx.x;
    cd y[6];
    {
      cd A[6][6];
      int pa[6];
      zload(0, A);
      lu_factor<6>(A, pa);
#pragma unroll
      for (int i = 0; i < 6; ++i) y[i] = ld(F + (size_t)i * nw + b);
      lu_apply<6>(A, pa, y);                  // y = A^-1 f1
#pragma unroll 1
      for (int j = 0; j < 6; ++j) {
        cd c[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) c[i] = mk(kk(i, 6 + j), 0.0);
        lu_apply<6>(A, pa, c);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          xs[((6 * i + j) * 2) * 64 + ln] = c[i].r;
          xs[((6 * i + j) * 2 + 1) * 64 + ln] = c[i].i;
        }
      }
    }
    auto X = [&](int i, int j) { return mk(xs[((6 * i + j) * 2) * 64 + ln], xs[((6 * i + j) * 2 + 1) * 64 + ln]); };
    cd S[6][6], g[6];
    int ps[6];
    zload(1, S);                              // S = D - K21 X
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        cd t = mk(0, 0);
#pragma unroll
        for (int m = 0; m < 6; ++m) t = add(t, scl(X(m, j), kk(6 + i, m)));
        S[i][j] = sub(S[i][j], t);
      }
#pragma unroll
    for (int i = 0; i < 6; ++i) {             // g = f2 - K21 A^-1 f1
      cd t = mk(0, 0);
#pragma unroll
      for (int m = 0; m < 6; ++m) t = add(t, scl(y[m], kk(6 + i, m)));
      g[i] = sub(ld(F + (size_t)(6 + i) * nw + b), t);
    }
    lu_factor<6>(S, ps);
    lu_apply<6>(S, ps, g);                    // x2
#pragma unroll
    for (int i = 0; i < 6; ++i) {             // x1 = A^-1 f1 - X x2
      cd t = y[i];
#pragma unroll
      for (int m = 0; m < 6; ++m) t = sub(t, mul(X(i, m), g[m]));
      y[i] = t;
    }
    if (live) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        st(Xi + (size_t)i * nw + b, y[i]);
        st(Xi + (size_t)(6 + i) * nw + b, g[i]);
      }
    }
  }
}


// ----------------------------------------------------------------------------------------
// The coupled-array response of every (case, bin) (raft/raft_model.py:1021-1065 for a batch of
// single-sea-state cases), in two launches with nothing per (case, bin) in HBM but Xi:
//   k_array_exc:  for each (case, FOWT) the wave excitation with the final drag linearisation,
//                 F_f = zeta (F_iner + F_drag) (raft/raft_model.py:1049-1061), written into
//                 the FOWT's rows of Xi;
//   k_array_resp: per (case, bin) lane, each FOWT's impedance rebuilt from the design's
//                 M / B_lin / C and the case's B_drag (the expression of fowt.Z,
//                 raft/raft_model.py:944, 1013), Z_sys = blockdiag(Z_f) + K_array, and
//                 Xi = Z_sys^-1 F solved by the 6x6 blocks as in k_system_solve_reg, reading
//                 the lane's F from Xi and overwriting it with the solution; optionally the
//                 motion PSD / RMS of every FOWT from the solution in registers (k_motion_stats
//                 with one row, the same arithmetic in the same order: no read-back of Xi).
// The excitation is its own launch because the block solve's register peak and its LDS slab
// hold k_array_resp at one wave per SIMD, where the node loop of the excitation could not hide
// its wave-table loads (one fused kernel: 190 us per C4 step against 58 us for the excitation
// alone and 78 us for the rest, profiles/r04_v2).  The drag part is member-factored over the
// projected table kproj (drag_exc_members' arithmetic), the node coefficients
// {qT Bmat q, p1T Bmat p1, p2T Bmat p2} recovered from the case's Bmat
// (Bmat = a_q qqT + a_1 p1p1T + a_2 p2p2T), with the node loads 4 nodes ahead.
// ----------------------------------------------------------------------------------------
struct ArrayArgs {
  const DevDesign* designs;
  int ncase;                   // cases; entry e = ic * NF + f is FOWT f of case ic
  const int* design_idx;       // [ncase * NF] design of each entry
  const int* head;             // [ncase * NF] heading index of each entry
  const double* zeta;          // [ncase * NF][nw]
  const double* B_drag;        // [ncase * NF][36]
  const double* Bmat;          // [ncase * NF][nn_max][9] (FOWTs may differ in node count)
  const double* K;             // [6 NF][6 NF] array stiffness, or NULL
  rh_c128* Xi;                 // [ncase][6 NF][nw]: F from k_array_exc, then the response
  int nn_max, nm_max;          // largest node / member counts of the designs (dynamic LDS layout)
  double dw = 0;               // motion statistics (k_array_resp): frequency step,
  double* psd = nullptr;       // [ncase * NF][6][nw] or NULL,
  double* stdv = nullptr;      // [ncase * NF][6] or NULL
  const int* order = nullptr;  // k_array_exc: entries in launch order (design, then heading), or NULL
};
constexpr int kArrRespThreads = 256;   // k_array_resp: one case per workgroup, bins in chunks of 256
constexpr int kArrExcThreads = 256;
__host__ __device__ inline size_t array_exc_smem(int nn_max, int nm_max) {
  return sizeof(double) * (size_t)(5 * nn_max + 18 * nm_max) + sizeof(int) * (size_t)(nm_max + 1);
}

// one (case, FOWT) entry per workgroup, every bin of the grid.  With an order, an XCD's
// workgroups take a contiguous slice of it (xcd_remap): the entries of few (design, heading)
// tables, which then stay in that XCD's L2 instead of every XCD streaming every table.
template <int NF>
__global__ __launch_bounds__(kArrExcThreads) void k_array_exc(ArrayArgs a) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  const int nnA = a.nn_max, nmA = a.nm_max;
  double* alf = dyn;                                          // [nnA][5] node drag coefficients
  double* mbf = alf + (size_t)nnA * 5;                        // [18][nmA] member factors cq, c1, c2
  int* ms = reinterpret_cast<int*>(mbf + (size_t)18 * nmA);   // [nmA + 1] member node ranges
  const int tid = (int)threadIdx.x;
  const size_t e = a.order ? (size_t)a.order[xcd_remap((int)blockIdx.x, (int)gridDim.x)] : blockIdx.x;
  const int ic = (int)(e / NF), f = (int)(e % NF);
  const rh_design& d = a.designs[a.design_idx[e]].d;
  const int nn = d.nn, nm = d.nm, nw = d.nw, head = a.head[e];
  const double* Bm = a.Bmat + e * nnA * 9;
  for (int n = tid; n < nn; n += kArrExcThreads) {
    double c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {   // e^T Bmat e for e = q, p1, p2
      const int fx = k == 0 ? RH_NF_QX : k == 1 ? RH_NF_P1X : RH_NF_P2X;
      const double ex = nf(d.node, nn, fx, n), ey = nf(d.node, nn, fx + 1, n), ez = nf(d.node, nn, fx + 2, n);
      const double* B = Bm + 9 * n;
      c[k] = ex * (B[0] * ex + B[1] * ey + B[2] * ez) + ey * (B[3] * ex + B[4] * ey + B[5] * ez) +
             ez * (B[6] * ex + B[7] * ey + B[8] * ez);
    }
    const double t = nf(d.node, nn, RH_NF_T, n);
    double* A = alf + (size_t)n * 5;
    A[0] = c[0];
    A[1] = c[1];
    A[2] = c[2];
    A[3] = t * c[1];
    A[4] = t * c[2];
  }
  for (int i = tid; i < 18 * nm; i += kArrExcThreads) mbf[(size_t)(i / nm) * nmA + i % nm] = d.memb[i];
  for (int i = tid; i <= nm; i += kArrExcThreads) ms[i] = d.mstart[i];
  __syncthreads();
  const unsigned nw16 = (unsigned)nw * 16u;
  const Buf bK = mkbuf(d.kproj + (size_t)head * nn * 3 * nw, (unsigned)nn * 3u * nw16);
  const Buf bFe = mkbuf(d.finer + (size_t)head * 6 * nw, 6u * nw16);
  rh_c128* Fo = a.Xi + ((size_t)ic * 6 * NF + 6 * f) * nw;
#pragma unroll 1
  for (int b0 = 0; b0 < nw; b0 += kArrExcThreads) {
    if (!__builtin_amdgcn_ballot_w64(b0 + tid < nw)) continue;   // whole wave past the grid (uniform)
    const int b = b0 + tid < nw ? b0 + tid : nw - 1;
    const unsigned vb = (unsigned)b * 16u;
    cd fe[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) fe[c] = bld(bFe, vb, c * nw16);
    const double z = a.zeta[e * nw + b];
    cd F[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) F[c] = mk(0, 0);
    cd SQ = mk(0, 0), S1 = mk(0, 0), S2 = mk(0, 0), T1 = mk(0, 0), T2 = mk(0, 0);
    int m = 0, mnext = nn > 0 ? ms[1] : 0;
    auto fold = [&]() {   // close member m: F += its node sums (drag_exc_members)
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double cq = mbf[(RH_MF_CQ0 + i) * nmA + m], c1 = mbf[(RH_MF_C10 + i) * nmA + m],
                     c2 = mbf[(RH_MF_C20 + i) * nmA + m];
        F[i] = add(F[i], add(add(scl(SQ, cq), scl(S1, c1)), scl(S2, c2)));
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const double p1 = mbf[(RH_MF_C10 + i) * nmA + m], p2 = mbf[(RH_MF_C20 + i) * nmA + m];
        F[3 + i] = add(F[3 + i], sub(scl(T1, p2), scl(T2, p1)));
      }
      SQ = S1 = S2 = T1 = T2 = mk(0, 0);
    };
    constexpr int R = 4;
    auto load = [&](cd (&K)[3], int n) {
      const unsigned so = (unsigned)(n < nn ? n : nn - 1) * 3u * nw16;
#pragma unroll
      for (int p = 0; p < 3; ++p) K[p] = bld(bK, vb, so + (unsigned)p * nw16);
    };
    cd K[R][3];
#pragma unroll
    for (int r = 0; r < R; ++r) load(K[r], r);
    for (int n = 0; n < nn; n += R) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int nr = n + r;
        if (nr < nn) {
          while (nr == mnext) {   // uniform: member m ended before node nr
            fold();
            ++m;
            mnext = ms[m + 1];
          }
          const double* An = alf + 5 * nr;
          SQ = add(SQ, scl(K[r][0], An[0]));
          S1 = add(S1, scl(K[r][1], An[1]));
          S2 = add(S2, scl(K[r][2], An[2]));
          T1 = add(T1, scl(K[r][1], An[3]));
          T2 = add(T2, scl(K[r][2], An[4]));
          load(K[r], nr + R);
        }
      }
    }
    if (nn > 0) fold();
    if (b0 + tid < nw)
#pragma unroll
      for (int c = 0; c < 6; ++c) st(Fo + (size_t)c * nw + b, add(scl(fe[c], z), scl(F[c], z)));
  }
}

// MULTI: nw > kArrRespThreads, the bins in several chunks (the RMS sums are carried across them);
// otherwise one chunk and nothing is live across the block solve but the solution.
template <int NF, bool MULTI>
__global__ __launch_bounds__(kArrRespThreads) void k_array_resp(ArrayArgs a) {
  constexpr int N = 6 * NF;
  constexpr int W = kArrRespThreads / 64;
  __shared__ double xs[NF == 2 ? 36 * 2 * kArrRespThreads : 1];   // NF == 2: the lane-private X slab [36][re, im][lanes]
  __shared__ double ks[N * N];        // K_array (uniform reads)
  __shared__ double mz[NF][4][36];    // per FOWT: M, B_lin (frequency-independent designs), C, B_drag
  __shared__ double sred[W][N];       // motion RMS: the waves' sums
  const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ic = blockIdx.x;
  for (int e = tid; e < N * N; e += kArrRespThreads) ks[e] = a.K ? a.K[e] : 0.0;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const rh_design& d = a.designs[a.design_idx[ic * NF + f]].d;
    if (tid < 36) {
      mz[f][0][tid] = d.mb_per_bin ? 0.0 : d.M[tid];
      mz[f][1][tid] = d.mb_per_bin ? 0.0 : d.B[tid];
      mz[f][2][tid] = d.C[tid];
      mz[f][3][tid] = a.B_drag[((size_t)ic * NF + f) * 36 + tid];
    }
  }
  __syncthreads();
  const rh_design& d0 = a.designs[a.design_idx[ic * NF]].d;
  const int nw = d0.nw;
  rh_c128* Xo = a.Xi + (size_t)ic * N * nw;
  const bool stats = a.psd || a.stdv;   // uniform
  double ss[N];                         // per DOF row: this lane's sum of |x|^2 over its bins
#pragma unroll
  for (int k = 0; k < N; ++k) ss[k] = 0.0;
  // |x|^2 of a solution row (rotations in degrees) into the PSD and the lane's RMS sums
  // (k_motion_stats with nrow = 1: psd = 0 + 0.5 m2 / dw, the same bits)
  auto add_stats = [&](int k, int b, cd x) {
    const double m2 = abs2(k % 6 >= 3 ? scl(x, kRad2Deg) : x);
    if (a.psd) a.psd[((size_t)ic * N + k) * nw + b] = 0.5 * m2 / a.dw;
    ss[k] += m2;
  };
#pragma unroll 1
  for (int c0 = 0; c0 < (MULTI ? nw : 1); c0 += kArrRespThreads) {
    if (MULTI && !__builtin_amdgcn_ballot_w64(c0 + tid < nw)) continue;   // the whole wave past the grid (uniform)
    const int b0 = c0 + tid;
    const bool live = b0 < nw;
    const int b = live ? b0 : nw - 1;          // pad lanes solve the last bin and store nothing
    int zo;                        // a zero the compiler cannot see through: the LDS reads stay where
    asm volatile("s_mov_b32 %0, 0" : "=s"(zo));   // they are used instead of being hoisted into registers
    const double* ksz = ks + zo;
    auto kk = [&](int i, int j) { return ksz[i * N + j]; };
    // (0 + Z_f) + K_ff, Z_f = (-w^2 M + C) + i w (B + B_drag): the additions in the reference's order
    auto zload = [&](int f, cd (&A)[6][6]) {
      const rh_design& d = a.designs[a.design_idx[ic * NF + f]].d;
      const double w = d.w[b], w2 = -(w * w);
      const double* m = &mz[f][0][0] + zo;
      if (d.mb_per_bin) {    // uniform: per-bin M and B (aero / BEM) from the design's arrays
        const double* M = d.M + (size_t)b * 36;
        const double* B = d.B + (size_t)b * 36;
  #pragma unroll
        for (int i = 0; i < 6; ++i)
  #pragma unroll
          for (int j = 0; j < 6; ++j) {
            const int e = 6 * i + j;
            A[i][j] = mk((w2 * M[e] + m[72 + e]) + kk(6 * f + i, 6 * f + j), w * (B[e] + m[108 + e]));
          }
      } else {
  #pragma unroll
        for (int i = 0; i < 6; ++i)
  #pragma unroll
          for (int j = 0; j < 6; ++j) {
            const int e = 6 * i + j;
            A[i][j] = mk((w2 * m[e] + m[72 + e]) + kk(6 * f + i, 6 * f + j), w * (m[36 + e] + m[108 + e]));
          }
      }
    };
    auto excite = [&](int f, cd (&F)[6]) {   // F_f of this lane's bin, from k_array_exc
  #pragma unroll
      for (int c = 0; c < 6; ++c) F[c] = ld(Xo + (size_t)(6 * f + c) * nw + b);
    };
    if constexpr (NF == 1) {
      cd A[6][6], x[6];
      excite(0, x);
      zload(0, A);
      lu_solve<6>(A, x);
      if (live)
  #pragma unroll
        for (int i = 0; i < 6; ++i) {
          st(Xo + (size_t)i * nw + b, x[i]);
          if (stats) add_stats(i, b, x[i]);
        }
    } else {
      static_assert(NF == 2, "k_array_resp: one or two FOWTs");
      // X = A^-1 K12 column by column to a lane-private LDS slab [36][re, im][lanes]
      constexpr int T = kArrRespThreads;
      cd y[6];
      {
        cd A[6][6];
        int pa[6];
        excite(0, y);                           // f1
        zload(0, A);
        lu_factor<6>(A, pa);
        lu_apply<6>(A, pa, y);                  // y = A^-1 f1
  #pragma unroll 1
        for (int j = 0; j < 6; ++j) {
          cd c[6];
  #pragma unroll
          for (int i = 0; i < 6; ++i) c[i] = mk(kk(i, 6 + j), 0.0);
          lu_apply<6>(A, pa, c);
  #pragma unroll
          for (int i = 0; i < 6; ++i) {
            xs[((6 * i + j) * 2) * T + tid] = c[i].r;
            xs[((6 * i + j) * 2 + 1) * T + tid] = c[i].i;
          }
        }
      }
      auto X = [&](int i, int j) { return mk(xs[((6 * i + j) * 2) * T + tid], xs[((6 * i + j) * 2 + 1) * T + tid]); };
      cd g[6];
      excite(1, g);                             // f2, loaded once A is dead
      cd S[6][6];
      int ps[6];
      zload(1, S);                              // S = D - K21 X
  #pragma unroll
      for (int i = 0; i < 6; ++i)
  #pragma unroll
        for (int j = 0; j < 6; ++j) {
          cd t = mk(0, 0);
  #pragma unroll
          for (int m = 0; m < 6; ++m) t = add(t, scl(X(m, j), kk(6 + i, m)));
          S[i][j] = sub(S[i][j], t);
        }
  #pragma unroll
      for (int i = 0; i < 6; ++i) {             // g = f2 - K21 A^-1 f1
        cd t = mk(0, 0);
  #pragma unroll
        for (int m = 0; m < 6; ++m) t = add(t, scl(y[m], kk(6 + i, m)));
        g[i] = sub(g[i], t);
      }
      lu_factor<6>(S, ps);
      lu_apply<6>(S, ps, g);                    // x2
  #pragma unroll
      for (int i = 0; i < 6; ++i) {             // x1 = A^-1 f1 - X x2
        cd t = y[i];
  #pragma unroll
        for (int m = 0; m < 6; ++m) t = sub(t, mul(X(i, m), g[m]));
        y[i] = t;
      }
      if (live) {
  #pragma unroll
        for (int i = 0; i < 6; ++i) {
          st(Xo + (size_t)i * nw + b, y[i]);
          st(Xo + (size_t)(6 + i) * nw + b, g[i]);
        }
        if (stats) {
  #pragma unroll
          for (int i = 0; i < 6; ++i) {
            add_stats(i, b, y[i]);
            add_stats(6 + i, b, g[i]);
          }
        }
      }
    }
  }
  if (a.stdv) {   // uniform: wave sums, then the waves in order (k_motion_stats' reduction)
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const double s = wave_sum(ss[k]);
      if (lane == 0) sred[wv][k] = s;
    }
    __syncthreads();
    if (tid < N) {
      double s = 0;
      for (int w = 0; w < W; ++w) s += sred[w][tid];
      a.stdv[(size_t)ic * N + tid] = sqrt(0.5 * s);
    }
  }
}

}  // namespace rh
