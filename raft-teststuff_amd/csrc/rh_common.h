// rh_common.h -- device helpers and argument structs shared by the kernels of librafthip's
// translation units (rh_abi.hip: host boundary + most kernels; rh_solve_fast.hip: the
// single-pass k_solve_lds instantiations, compiled with the max-ilp machine scheduler).
// Nothing here defines a kernel or a __device__ variable, so it can be included by both.
#pragma once
#include "rh_device.h"

namespace rh {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr double kSqrt8Pi = 1.5957691216057308;   // np.sqrt(8/np.pi)
constexpr double kRad2Deg = 57.29577951308232;    // raft/helpers.py:25-26

struct DevDesign {
  rh_design d;
};

__device__ __forceinline__ double nf(const double* node, int nn, int f, int n) { return node[f * nn + n]; }

// Spectral density S(w) for one bin (raft/helpers.py:606-663, raft/raft_fowt.py:1000-1014)
__device__ inline double sea_spectrum(int spec, double Hs, double Tp, double gam, double w) {
  double S;
  if (spec == RH_SPEC_UNIT) {
    S = 1.0;
  } else if (spec == RH_SPEC_CONSTANT) {
    S = Hs;
  } else if (spec == RH_SPEC_NONE) {
    S = 0.0;
  } else {
    double G = gam;
    if (!(G != 0.0)) {                      // `if not Gamma:` (0 -> IEC automatic)
      const double t = Tp / sqrt(Hs);
      if (t <= 3.6) G = 5.0;
      else if (t >= 5.0) G = 1.0;
      else G = exp(5.75 - 1.15 * t);
    }
    const double f = 0.5 / M_PI * w;
    const double fp4 = pow(Tp * f, -4.0);
    const double C = 1.0 - (0.287 * log(G));
    const double sig = (f <= 1.0 / Tp) ? 0.07 : 0.09;
    const double a = (f * Tp - 1.0) / sig;
    const double Alpha = exp(-0.5 * (a * a));
    S = 0.5 / M_PI * C * 0.3125 * Hs * Hs * fp4 / f * exp(-1.25 * fp4) * pow(G, Alpha);
  }
  return S;
}

// wave amplitude zeta = sqrt(2 S dw) (raft/raft_fowt.py:1003-1009)
__device__ __forceinline__ double sea_amplitude(int spec, double Hs, double Tp, double gam, double w, double dw) {
  return sqrt(2.0 * sea_spectrum(spec, Hs, Tp, gam, w) * dw);
}

// ----------------------------------------------------------------------------------------
// shared pieces of the case solve
// ----------------------------------------------------------------------------------------

// Node drag matrix from the three bin-summed squared relative-velocity magnitudes
// (raft/raft_fowt.py:1213-1248).  sums = {sum|vrel_q|^2, sum|vrel_p or p1|^2, sum|vrel_p2|^2}.
__device__ __forceinline__ double nrm2(const double* node, int nn, int f, int n) {
  const double a = nf(node, nn, f, n), b = nf(node, nn, f + 1, n), c = nf(node, nn, f + 2, n);
  return a * a + b * b + c * c;
}

// One node's drag matrix Bmat = Bq (qq^T) + Bp1 (p1p1^T) + Bp2 (p2p2^T) + Be (qq^T) from its
// RMS sums (raft/raft_fowt.py:1205-1248); F(field) reads the node's RH_NF_* fields.
template <class Fld>
__device__ __forceinline__ void node_bmat_f(Fld F, double rho, const double* sums, double* bm, double* B4 = nullptr) {
  const bool circ = F(RH_NF_CIRC) != 0.0;
  const double vq = sqrt(0.5 * sums[0]);
  const double vp1 = sqrt(0.5 * sums[1]);
  const double vp2 = circ ? vp1 : sqrt(0.5 * sums[2]);
  const double Bq = kSqrt8Pi * vq * 0.5 * rho * F(RH_NF_AQ) * F(RH_NF_CDQ);
  const double Bp1 = kSqrt8Pi * vp1 * 0.5 * rho * F(RH_NF_AP1) * F(RH_NF_CDP1);
  const double Bp2 = kSqrt8Pi * vp2 * 0.5 * rho * F(RH_NF_AP2) * F(RH_NF_CDP2);
  const double Be = kSqrt8Pi * vq * 0.5 * rho * F(RH_NF_AEND) * F(RH_NF_CDEND);
  if (B4) {
    B4[0] = Bq;
    B4[1] = Bp1;
    B4[2] = Bp2;
    B4[3] = Be;
  }
  const double q[3] = {F(RH_NF_QX), F(RH_NF_QY), F(RH_NF_QZ)};
  const double p1[3] = {F(RH_NF_P1X), F(RH_NF_P1Y), F(RH_NF_P1Z)};
  const double p2[3] = {F(RH_NF_P2X), F(RH_NF_P2Y), F(RH_NF_P2Z)};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      bm[3 * i + j] = (Bq * (q[i] * q[j]) + Bp1 * (p1[i] * p1[j]) + Bp2 * (p2[i] * p2[j])) + Be * (q[i] * q[j]);
}
__device__ __forceinline__ void node_bmat(const double* node, int nn, int n, double rho, const double* sums,
                                          double* bm, double* B4 = nullptr) {
  node_bmat_f([&](int f) { return nf(node, nn, f, n); }, rho, sums, bm, B4);
}

// Entry (i,j) of translateMatrix3to6DOF(Bm, r) (raft/helpers.py:455-478).
__device__ __forceinline__ double t3to6(const double* Bm, double rx, double ry, double rz, int i, int j) {
  const double H[3][3] = {{0, rz, -ry}, {-rz, 0, rx}, {ry, -rx, 0}};
  auto BH = [&](int a, int c) { return Bm[3 * a + 0] * H[0][c] + Bm[3 * a + 1] * H[1][c] + Bm[3 * a + 2] * H[2][c]; };
  if (i < 3 && j < 3) return Bm[3 * i + j];
  if (i < 3) return BH(i, j - 3);
  if (j < 3) return BH(j, i - 3);
  const int a = i - 3, c = j - 3;   // (H Bm H^T)[a][c] = sum_k H[a][k] (Bm H^T)[k][c] = sum_k H[a][k] BH? -> (H (Bm H^T))
  double s = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double HB = H[a][0] * Bm[0 * 3 + k] + H[a][1] * Bm[1 * 3 + k] + H[a][2] * Bm[2 * 3 + k];  // (H Bm)[a][k]
    s += HB * H[c][k];                                                                          // * H^T[k][c]
  }
  return s;
}

// Drag excitation of one bin before the zeta factor: sum_n [Bm_n uhat_n; r_n x Bm_n uhat_n]
__device__ __forceinline__ void drag_exc_bin(const double* node, int nn, const double* bm_lds,
                                             const rh_c128* __restrict__ Uh, int nw, int b, cd (&F)[6]) {
#pragma unroll
  for (int c = 0; c < 6; ++c) F[c] = mk(0, 0);
  for (int n = 0; n < nn; ++n) {
    const rh_c128* U = Uh + (size_t)n * 3 * nw + b;
    const cd u0 = ld(U), u1 = ld(U + nw), u2 = ld(U + 2 * nw);
    const double* Bm = bm_lds + 9 * n;
    cd f[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) f[r] = add(add(scl(u0, Bm[3 * r]), scl(u1, Bm[3 * r + 1])), scl(u2, Bm[3 * r + 2]));
    const double rx = nf(node, nn, RH_NF_XX, n), ry = nf(node, nn, RH_NF_XY, n), rz = nf(node, nn, RH_NF_XZ, n);
    F[0] = add(F[0], f[0]);
    F[1] = add(F[1], f[1]);
    F[2] = add(F[2], f[2]);
    F[3] = add(F[3], sub(scl(f[2], ry), scl(f[1], rz)));
    F[4] = add(F[4], sub(scl(f[0], rz), scl(f[2], rx)));
    F[5] = add(F[5], sub(scl(f[1], rx), scl(f[0], ry)));
  }
}

// Drag excitation of one bin before the zeta factor, member-factored:
//   f_n = Bmat_n uhat_n = aq q Kq + a1 p1 K1 + a2 p2 K2,  r_n x f_n = rA x f_n + t q x f_n
// with q x p1 = p2, q x p2 = -p1 (raft/raft_fowt.py:1255-1259, 1283-1289).  al: [nn][5] LDS
// {aq, a1, a2, t a1, t a2}.
__device__ __forceinline__ void drag_exc_members(const rh_design& d, const double* al, const rh_c128* __restrict__ Kp,
                                                 int nw, int b, cd (&F)[6]) {
#pragma unroll
  for (int c = 0; c < 6; ++c) F[c] = mk(0, 0);
  const int nm = d.nm;
  for (int m = 0; m < nm; ++m) {
    const int n0 = d.mstart[m], n1 = d.mstart[m + 1];
    cd SQ = mk(0, 0), S1 = mk(0, 0), S2 = mk(0, 0), T1 = mk(0, 0), T2 = mk(0, 0);
    for (int n = n0; n < n1; ++n) {
      const rh_c128* K = Kp + (size_t)n * 3 * nw + b;
      const cd kq = ld(K), k1 = ld(K + nw), k2 = ld(K + 2 * nw);
      const double* A = al + 5 * n;
      SQ = add(SQ, scl(kq, A[0]));
      S1 = add(S1, scl(k1, A[1]));
      S2 = add(S2, scl(k2, A[2]));
      T1 = add(T1, scl(k1, A[3]));
      T2 = add(T2, scl(k2, A[4]));
    }
    const double* M = d.memb;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double cq = M[(RH_MF_CQ0 + i) * nm + m], c1 = M[(RH_MF_C10 + i) * nm + m], c2 = M[(RH_MF_C20 + i) * nm + m];
      F[i] = add(F[i], add(add(scl(SQ, cq), scl(S1, c1)), scl(S2, c2)));
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double p1 = M[(RH_MF_C10 + i) * nm + m], p2 = M[(RH_MF_C20 + i) * nm + m];
      F[3 + i] = add(F[3 + i], sub(scl(T1, p2), scl(T2, p1)));
    }
  }
}

// Z(w) = -w^2 M + i w (B + B_drag) + C (raft/raft_model.py:944).
// mbc: LDS image {M[36], B_lin[36], C[36]} of a frequency-independent design (wave-uniform
// broadcast reads); per-bin M/B (BEM added mass / radiation damping) come from global memory.
__device__ __forceinline__ void assemble_z(const rh_design& d, const double* mbc, int b, double w, const double* bd,
                                           cd (&Z)[6][6]) {
  const double w2 = -(w * w);
  if (d.mb_per_bin) {
    const double* M = d.M + (size_t)b * 36;
    const double* B = d.B + (size_t)b * 36;
#pragma unroll
    for (int e = 0; e < 36; ++e) Z[e / 6][e % 6] = mk(w2 * M[e] + mbc[72 + e], w * (B[e] + bd[e]));
  } else {
#pragma unroll
    for (int e = 0; e < 36; ++e) Z[e / 6][e % 6] = mk(w2 * mbc[e] + mbc[72 + e], w * (mbc[36 + e] + bd[e]));
  }
}

// LDS image of M_lin, B_lin, C_lin (frequency-independent parts); call with >= 36 threads.
__device__ __forceinline__ void load_mbc(const rh_design& d, double* mbc, int tid) {
  if (tid < 36) {
    mbc[tid] = d.mb_per_bin ? 0.0 : d.M[tid];
    mbc[36 + tid] = d.mb_per_bin ? 0.0 : d.B[tid];
    mbc[72 + tid] = d.C[tid];
  }
}

// ----------------------------------------------------------------------------------------
// k_solve_cases
// ----------------------------------------------------------------------------------------
struct CaseArgs {
  const DevDesign* designs;
  rh_cases c;
  rh_solve_out o;
  // two-pass launch of k_solve_lds (rh_solve_cases): pass 1 stops a case before iteration
  // stop_iter, parks its relaxed iterate in o.Xi_last and marks it kCaseStopped; pass 2
  // (resume = 1) continues only those cases from there.  The default runs one pass.
  int stop_iter = 1 << 30;
  int resume = 0;
  // 1: k_a0_sums has written every case's iteration-0 phase-A sums to its Xi_last block
  // (rh_a0.hip); k_solve_lds skips phase A of iteration 0 and reads them in phase B
  int a0 = 0;
  // node stride of the Bmat output ([ncase][bmat_nn][9]): the largest nn of the call's designs,
  // so designs with different node counts share one output array (rh_solve_cases sets it)
  int bmat_nn = 0;
};
constexpr int kCaseStopped = 9;   // internal status between the two passes (never returned)

}  // namespace rh
