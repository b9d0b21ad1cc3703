// rh_qtf.hip -- slender-body second-order QTF on gfx950.
//
//   k_qtf_tables : one launch of every per-frequency table kind:
//   qtf_freq_at  : per second-order frequency: RAO resampled from the first-order grid
//                  (np.interp, left=right=0, raft/raft_fowt.py:1415-1417), first-order force
//                  F1st = M a (:1437-1439), rotation generator i w theta (:1556-1557)
//   qtf_nodes_motion_at : per (node, frequency): incident velocity u, node displacement/velocity
//                  and their axial projections (RAO-dependent)
//   qtf_nodes_grad_at : per (node, frequency): grad u (raft/helpers.py:157-195), grad p
//                  (:202-225), dw/dz along the axis (incident wave only)
//   qtf_wl_at    : per (member, frequency): waterline kinematics (raft/raft_fowt.py:1486-1502)
//   k_qtf_pairs  : per (w1 <= w2) pair: Pinkster IV + every node term + waterline term +
//                  Kim & Yue correction, then the Hermitian fill (:1449-1640, raft_member.py:1090-1205)
//   k_force2nd   : difference-frequency force spectrum with on-the-fly bilinear resampling
//                  of the QTF (raft/raft_fowt.py:1788-1810; interp2d restated per SURVEY.md Q13)
//
// Layout: every per-frequency table is frequency-contiguous, so the lanes of a wave (64
// consecutive w2 of one w1 row) read coalesced rows for the w2 side and a broadcast for the
// w1 side.
#include "rh_bessel.h"

namespace rh {

constexpr double kDeg2Rad = 0.017453292519943295;   // raft/helpers.py:27-28
constexpr int kQtfTile = 64;
constexpr int kKayT = 8;           // doubles per (KAY row, frequency) in QtfWork::kayt

// per-(node, frequency) table fields (complex) [nq][QT_COUNT][n2]
enum { QT_U = 0, QT_VP = 3, QT_VA = 6, QT_DR = 7, QT_GU = 10, QT_GP = 19, QT_DWDZ = 22, QT_COUNT = 23 };
// per-(member, frequency) waterline fields (complex) [nmq][WT_COUNT][n2]
enum { WT_ETAR = 0, WT_UD = 1, WT_A = 4, WT_GE = 7, WT_COUNT = 10 };
// per-frequency fields (complex) [FT_COUNT][n2]
enum { FT_XI = 0, FT_F1 = 6, FT_OM = 12, FT_COUNT = 15 };

// Bilinear (MFMA) form of the pair sum, rh_qtf_mfma.hip.  Every term of the node, waterline
// and Pinkster sums is a product of a w1-side and a conj(w2-side) first-order quantity, and
// the w2-side quantities of a node are linear combinations of a few per-frequency basis
// functions (8 per node, 3 per waterline member, and the 18 motions X, w X, w^2 X shared by
// all).  So the upper triangle is Q_d(i1, i2) = sum_k L_d[k](i1) R[k](i2): one complex GEMM
// per DOF with K = 8 nq + 3 nmq + 18.  Column layout of R / L:
__host__ __device__ inline int qtf_n2p(const rh_qtf_design& q) { return (q.n2 + 15) & ~15; }
__host__ __device__ inline int qtf_kb(const rh_qtf_design& q) { return 8 * q.nq + 3 * q.nmq + 18; }
// K rounded up to 16: the GEMM loops run in groups of four k-steps of four
__host__ __device__ inline int qtf_kp(const rh_qtf_design& q) { return (qtf_kb(q) + 15) & ~15; }
__host__ __device__ inline int qtf_kq(const rh_qtf_design& q) { return (2 * q.nq + 15) & ~15; }
__host__ __device__ inline int qcol_node(int n, int j) { return 8 * n + j; }
__host__ __device__ inline int qcol_wl(const rh_qtf_design& q, int m, int j) { return 8 * q.nq + 3 * m + j; }
__host__ __device__ inline int qcol_glob(const rh_qtf_design& q, int g) { return 8 * q.nq + 3 * q.nmq + g; }
constexpr int kKayK = 24;          // real K of the Kim & Yue dots: 12 complex Hankel orders as (re, im)

struct QtfWork {
  rh_c128* node;   // [nq][QT_COUNT][n2]
  rh_c128* wl;     // [nmq][WT_COUNT][n2]
  rh_c128* freq;   // [FT_COUNT][n2]
  rh_c128* hinv;   // [nkr][n2][12] reciprocals of the Hankel-derivative table q.hank
  double* kayt;    // [nkr][n2][8] cosh(k R H), sqrt(k R H tanh(k R H)), exp(+-k (z1 + h)), exp(+-k (z2 + h)),
                   //              k R H / (sqrt(..) cosh(..)), 1 / (k R) of every KAY radius row
  // MFMA path (n2p = n2 rounded up to 16, zero padded; Kp, Kq rounded up to 16, zero rows)
  rh_c128* R;      // [Kp][n2p]   conj of the w2-side basis
  rh_c128* L;      // [6][Kp][n2p] w1-side coefficients per DOF
  rh_c128* Rp;     // [2][Kq][n2p] second-order-potential channels (+, -): b(w2), k2 b(w2)
  rh_c128* Lp;     // [2][6][Kq][n2p]
  double* KA;      // [nkr][24][n2p] Kim & Yue: (Re, Im) of the w1-side coefficients of sum omega_n
  double* KB;      // [nkr][24][n2p]                                      ... of sum n (n+1) omega_n
  double* KR;      // [nkr][24][n2p] (Im, Re) of conj(1 / D_n(k2 R))
  double* KS;      // [ntile][12][256] Kim & Yue sum of each 16 x 16 pair tile (k_qtf_kay ->
                   //                  k_qtf_kay_sum, so k_qtf_kay can run beside k_qtf_gemm)
};

// The MFMA-path operands (R, L, Rp, Lp, KA, KB, KR and the Kim & Yue tile sums KS) are
// reserved only for a sorted grid (order == 1), the only one the MFMA path runs on.
__host__ __device__ inline size_t qtf_work_elems(const rh_qtf_design& q) {   // complex elements
  const size_t n2p = (size_t)qtf_n2p(q), kp = (size_t)qtf_kp(q), kq = (size_t)qtf_kq(q);
  const size_t base = (size_t)q.nq * QT_COUNT * q.n2 + (size_t)q.nmq * WT_COUNT * q.n2 + (size_t)FT_COUNT * q.n2 +
                      (size_t)q.nkr * q.n2 * 12 + ((size_t)q.nkr * q.n2 * kKayT + 1) / 2;
  if (q.order != 1) return base;
  return base + 7 * kp * n2p + 14 * kq * n2p + ((size_t)3 * q.nkr * kKayK * n2p + 1) / 2 +
         (size_t)(n2p / 16) * (n2p / 16 + 1) / 2 * 12 * 256 / 2;
}

// carve the workspace (same order as qtf_work_elems)
__host__ inline QtfWork qtf_carve(const rh_qtf_design& q, void* work) {
  QtfWork wk;
  const size_t n2p = (size_t)qtf_n2p(q), kp = (size_t)qtf_kp(q), kq = (size_t)qtf_kq(q);
  wk.node = (rh_c128*)work;
  wk.wl = wk.node + (size_t)q.nq * QT_COUNT * q.n2;
  wk.freq = wk.wl + (size_t)q.nmq * WT_COUNT * q.n2;
  wk.hinv = wk.freq + (size_t)FT_COUNT * q.n2;
  rh_c128* after_kayt = wk.hinv + (size_t)q.nkr * q.n2 * 12 + ((size_t)q.nkr * q.n2 * kKayT + 1) / 2;
  wk.kayt = reinterpret_cast<double*>(wk.hinv + (size_t)q.nkr * q.n2 * 12);
  wk.R = after_kayt;
  wk.L = wk.R + kp * n2p;
  wk.Rp = wk.L + 6 * kp * n2p;
  wk.Lp = wk.Rp + 2 * kq * n2p;
  wk.KA = reinterpret_cast<double*>(wk.Lp + 12 * kq * n2p);
  wk.KB = wk.KA + (size_t)q.nkr * kKayK * n2p;
  wk.KR = wk.KB + (size_t)q.nkr * kKayK * n2p;
  wk.KS = wk.KR + (size_t)q.nkr * kKayK * n2p;
  if (q.order != 1) wk.R = wk.L = wk.Rp = wk.Lp = nullptr, wk.KA = wk.KB = wk.KR = wk.KS = nullptr;
  return wk;
}

// basis writers (rh_qtf_mfma.hip): called by the table kernels below for every (row, f < n2p)
__device__ void qtf_node_basis(const rh_qtf_design& q, const QtfWork& wk, int f, int n);
__device__ void qtf_wl_basis(const rh_qtf_design& q, const QtfWork& wk, int f, int m);
__device__ void qtf_kay_basis(const rh_qtf_design& q, const QtfWork& wk, int f, int ir);
__device__ void qtf_glob_basis(const rh_qtf_design& q, const QtfWork& wk, int f, const cd* X);
__host__ __device__ inline int qtf_npad(const rh_qtf_design& q);
__device__ void qtf_pad_row(const rh_qtf_design& q, const QtfWork& wk, int f, int p);

// Loads of wave-uniform table entries through the constant address space: the backend
// then issues scalar loads into SGPRs instead of 64 identical vector loads into VGPRs (the
// tables are written by earlier launches only, so they are invariant inside a kernel)
typedef const double __attribute__((address_space(4)))* f64_kp;
typedef const int __attribute__((address_space(4)))* i32_kp;
__device__ __forceinline__ cd lds(const rh_c128* p) {
  const f64_kp d = (f64_kp)(p);
  return cd{d[0], d[1]};
}
__device__ __forceinline__ double ldsd(const double* p) { return *(f64_kp)(p); }
__device__ __forceinline__ int ldsi(const int* p) { return *(i32_kp)(p); }
__device__ __forceinline__ double qn(const rh_qtf_design& q, int f, int n) { return ldsd(q.qnode + f * q.nq + n); }
__device__ __forceinline__ double qm(const rh_qtf_design& q, int f, int m) { return ldsd(q.qmemb + f * q.nmq + m); }
__device__ __forceinline__ void ldm9(const rh_qtf_design& q, int f, int n, double* M) {
#pragma unroll
  for (int i = 0; i < 9; ++i) M[i] = qn(q, f + i, n);
}

// cross products with a real vector (np.cross order)
__device__ __forceinline__ void cross_cc(const cd* a, const cd* b, cd* o) {
  o[0] = sub(mul(a[1], b[2]), mul(a[2], b[1]));
  o[1] = sub(mul(a[2], b[0]), mul(a[0], b[2]));
  o[2] = sub(mul(a[0], b[1]), mul(a[1], b[0]));
}
__device__ __forceinline__ cd cconj(cd a) { return cd{a.r, -a.i}; }
// real 3x3 (row-major, 9 consecutive fields) times complex 3-vector
__device__ __forceinline__ void rmv(const double* M, const cd* x, cd* y) {
#pragma unroll
  for (int i = 0; i < 3; ++i) y[i] = add(add(scl(x[0], M[3 * i]), scl(x[1], M[3 * i + 1])), scl(x[2], M[3 * i + 2]));
}
// complex 3x3 times complex 3-vector
__device__ __forceinline__ void cmv(const cd* M, const cd* x, cd* y) {
#pragma unroll
  for (int i = 0; i < 3; ++i) y[i] = add(add(mul(M[3 * i], x[0]), mul(M[3 * i + 1], x[1])), mul(M[3 * i + 2], x[2]));
}
// [f; r x f] accumulated into Q (translateForce3to6DOF, raft/helpers.py:386-401)
__device__ __forceinline__ void acc6(cd* Q, const cd* f, double rx, double ry, double rz) {
  Q[0] = add(Q[0], f[0]);
  Q[1] = add(Q[1], f[1]);
  Q[2] = add(Q[2], f[2]);
  Q[3] = add(Q[3], sub(scl(f[2], ry), scl(f[1], rz)));
  Q[4] = add(Q[4], sub(scl(f[0], rz), scl(f[2], rx)));
  Q[5] = add(Q[5], sub(scl(f[1], rx), scl(f[0], ry)));
}

// ---------------------------------------------------------------------------------------
// The RAO at second-order frequency f: np.interp(w2[f], w, Xi0[d], left=0, right=0)
// (raft/raft_fowt.py:1415-1417).  Every table row that needs it evaluates it itself (a binary
// search over the first-order grid), so no row waits for another.
__device__ __forceinline__ void qtf_resample(const rh_qtf_design& q, int nw, const double* __restrict__ w,
                                             const rh_c128* __restrict__ Xi0, int f, cd (&X)[6]) {
  const double x = q.w2[f];
  // j with w[j] <= x < w[j+1]
  if (x < w[0] || x > w[nw - 1]) {
#pragma unroll
    for (int d = 0; d < 6; ++d) X[d] = mk(0, 0);
  } else if (x == w[nw - 1]) {
#pragma unroll
    for (int d = 0; d < 6; ++d) X[d] = ld(Xi0 + (size_t)d * nw + nw - 1);
  } else {
    // lo with w[lo] <= x < w[lo + 1]: guessed from the first step (RAFT's grids are uniform,
    // raft/raft_model.py:66-67) and moved until the invariant holds, so any sorted grid gives
    // the interval a bisection would (two dependent loads instead of ten on a uniform grid)
    const double g = (x - w[0]) / (w[1] - w[0]);      // clamped before the conversion (NaN -> 0)
    int lo = g >= 0.0 && g < nw - 2 ? (int)g : g >= nw - 2 ? nw - 2 : 0;
    while (lo > 0 && w[lo] > x) --lo;
    while (lo < nw - 2 && w[lo + 1] <= x) ++lo;
    const double dx = w[lo + 1] - w[lo];
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      const cd a = ld(Xi0 + (size_t)d * nw + lo), b = ld(Xi0 + (size_t)d * nw + lo + 1);
      const double sr = (b.r - a.r) / dx, si = (b.i - a.i) / dx;
      X[d] = mk(sr * (x - w[lo]) + a.r, si * (x - w[lo]) + a.i);
    }
  }
}

// per second-order frequency: the resampled RAO, the first-order force F1st = M a
// (:1437-1439) and the rotation generator i w theta (:1556-1557), and the motion rows of the
// GEMM basis (the frequency row of k_qtf_tables)
__device__ __forceinline__ void qtf_freq_at(const rh_qtf_design& q, int nw, const double* __restrict__ w,
                                            const rh_c128* __restrict__ Xi0, const double* __restrict__ M66,
                                            const QtfWork& wk, int f) {
  const int n2 = q.n2;
  if (f >= n2) {
    if (wk.R && f < qtf_n2p(q)) qtf_glob_basis(q, wk, f, nullptr);   // zero padding of the GEMM operands
    return;
  }
  const double x = q.w2[f];
  cd X[6];
  qtf_resample(q, nw, w, Xi0, f, X);
  const double m2 = -(x * x);
  cd A[6];
#pragma unroll
  for (int d = 0; d < 6; ++d) A[d] = scl(X[d], m2);   // -w^2 Xi
  cd F[6];
#pragma unroll
  for (int d = 0; d < 3; ++d) F[d] = scl(A[d], M66[0]);
#pragma unroll
  for (int i = 0; i < 3; ++i)
    F[3 + i] = add(add(scl(A[3], M66[6 * (3 + i) + 3]), scl(A[4], M66[6 * (3 + i) + 4])), scl(A[5], M66[6 * (3 + i) + 5]));
#pragma unroll
  for (int d = 0; d < 6; ++d) {
    st(wk.freq + (size_t)(FT_XI + d) * n2 + f, X[d]);
    st(wk.freq + (size_t)(FT_F1 + d) * n2 + f, F[d]);
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) st(wk.freq + (size_t)(FT_OM + d) * n2 + f, iw(x, X[3 + d]));
  if (wk.R) qtf_glob_basis(q, wk, f, X);
}

// unit-amplitude Airy velocity at a point (raft/helpers.py:105-154, zeta0 = 1)
__device__ __forceinline__ void airy_u(double w, double k, double beta, double h, double x, double y, double z, cd* u,
                                       cd* eta_out = nullptr) {
  const double th = k * (cos(beta) * x + sin(beta) * y);
  const cd e = mk(cos(th), -sin(th));
  if (!(z <= 0)) {
    u[0] = u[1] = u[2] = mk(0, 0);
    if (eta_out) *eta_out = mk(0, 0);
    return;
  }
  double s_sh, c_sh, c_ch;
  if (k * h > 89.4) {
    s_sh = exp(k * z);
    c_sh = exp(k * z);
    c_ch = exp(k * z) + exp(-k * (z + 2.0 * h));
  } else {
    s_sh = sinh(k * (z + h)) / sinh(k * h);
    c_sh = cosh(k * (z + h)) / sinh(k * h);
    c_ch = cosh(k * (z + h)) / cosh(k * h);
  }
  const cd we = scl(e, w);
  u[0] = scl(scl(we, c_sh), cos(beta));
  u[1] = scl(scl(we, c_sh), sin(beta));
  u[2] = scl(iw(w, e), s_sh);
  if (eta_out) *eta_out = scl(e, c_ch);   // pDyn with rho = g = 1 (raft/raft_fowt.py:1493)
}

__device__ __forceinline__ void qtf_nodes_motion_at(const rh_qtf_design& q, const QtfWork& wk, int f, int n, const cd (&X)[6]) {
  const int n2 = q.n2;
  if (f >= n2) return;
  const double w = q.w2[f], k = q.k2[f], h = q.depth, beta = q.beta;
  const double x = qn(q, RH_QN_RX, n), y = qn(q, RH_QN_RY, n), z = qn(q, RH_QN_RZ, n);
  const double qv[3] = {qn(q, RH_QN_QX, n), qn(q, RH_QN_QY, n), qn(q, RH_QN_QZ, n)};
  // getKinematics at the node (raft/helpers.py:95-97): dr = Xi[:3] + th x r ; v = i w dr
  cd dr[3];
  dr[0] = add(X[0], add(scl(X[5], -y), scl(X[4], z)));
  dr[1] = add(X[1], sub(scl(X[5], x), scl(X[3], z)));
  dr[2] = add(X[2], add(scl(X[4], -x), scl(X[3], y)));
  cd v[3] = {iw(w, dr[0]), iw(w, dr[1]), iw(w, dr[2])};
  cd u[3];
  airy_u(w, k, beta, h, x, y, z, u);
  // nodeV_axial_rel = (u - nodeV) . q (:1482), before any projection
  const cd va = add(add(scl(sub(u[0], v[0]), qv[0]), scl(sub(u[1], v[1]), qv[1])), scl(sub(u[2], v[2]), qv[2]));
  // node velocity after _axdivAcc's in-place projection: every later use is projected
  const cd vq = add(add(scl(v[0], qv[0]), scl(v[1], qv[1])), scl(v[2], qv[2]));
  cd vp[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) vp[i] = sub(v[i], scl(vq, qv[i]));
  rh_c128* T = wk.node + (size_t)n * QT_COUNT * n2 + f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st(T + (size_t)(QT_U + i) * n2, u[i]);
    st(T + (size_t)(QT_VP + i) * n2, vp[i]);
    st(T + (size_t)(QT_DR + i) * n2, dr[i]);
  }
  st(T + (size_t)QT_VA * n2, va);
}

// the incident-wave fields of a node's table (grad u, grad p, dw/dz along the axis): no RAO in
// them, so a further RAO on the same rh_qtf_design keeps them (RH_QTF_INCIDENT_CACHED)
__device__ __forceinline__ void qtf_nodes_grad_at(const rh_qtf_design& q, const QtfWork& wk, int f, int n) {
  const int n2 = q.n2;
  if (f >= n2) return;
  const double w = q.w2[f], k = q.k2[f], h = q.depth, beta = q.beta;
  const double x = qn(q, RH_QN_RX, n), y = qn(q, RH_QN_RY, n), z = qn(q, RH_QN_RZ, n);
  const double qv[3] = {qn(q, RH_QN_QX, n), qn(q, RH_QN_QY, n), qn(q, RH_QN_QZ, n)};
  // grad u (raft/helpers.py:157-195) with the degree-converted direction cosines (Q1), Q2
  cd G[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) G[i] = mk(0, 0);
  cd gp[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
  if (z <= 0 && k > 0) {
    const double cb = cos(beta * kDeg2Rad), sb = sin(beta * kDeg2Rad);
    double kxy, kz;
    if (k * h >= 10) {
      kxy = exp(k * z);
      kz = kxy;
    } else {
      kxy = cosh(k * (z + h)) / sinh(k * h);
      kz = sinh(k * (z + h)) / sinh(k * h);
    }
    const double th = k * (cos(beta) * x + sin(beta) * y);
    const cd ph = mk(cos(th), -sin(th));
    cd aux = scl(ph, w * cb);
    const cd mi_aux = mk(aux.i, -aux.r);                         // -1j*aux
    G[0] = scl(scl(scl(mi_aux, kxy), k), cb);
    G[1] = scl(scl(scl(mi_aux, kxy), k), sb);
    G[2] = scl(scl(aux, k), kz);
    aux = scl(ph, w * sb);
    const cd mi_aux2 = mk(aux.i, -aux.r);
    G[3] = G[1];
    G[4] = scl(scl(scl(mi_aux2, kxy), k), sb);
    G[5] = scl(scl(aux, k), kz);
    aux = iw(w, ph);
    G[6] = G[2];
    G[7] = G[1];                                                 // Q2: grad[2,1] = grad[0,1]
    G[8] = scl(scl(aux, k), kxy);
    // grad p1 (raft/helpers.py:202-225): phase with the degree-converted cosines
    double pxy, pz;
    if (k * h >= 10) {
      pxy = exp(k * z);
      pz = pxy;
    } else {
      pxy = cosh(k * (z + h)) / cosh(k * h);
      pz = sinh(k * (z + h)) / cosh(k * h);
    }
    const double th2 = k * (cb * x + sb * y);
    const cd ph2 = mk(cos(th2), -sin(th2));
    const double rg = q.rho * q.g;
    const cd a0 = scl(scl(ph2, rg * pxy), 1.0);
    gp[0] = mul(a0, mk(0, -k * cb));
    gp[1] = mul(a0, mk(0, -k * sb));
    gp[2] = scl(scl(ph2, rg * pz), k);
  }
  // dw/dz along the axis for _axdivAcc: (grad u q) . q
  cd Gq[3];
  cd qc[3] = {mk(qv[0], 0), mk(qv[1], 0), mk(qv[2], 0)};
  cmv(G, qc, Gq);
  const cd dwdz = add(add(scl(Gq[0], qv[0]), scl(Gq[1], qv[1])), scl(Gq[2], qv[2]));
  rh_c128* T = wk.node + (size_t)n * QT_COUNT * n2 + f;
#pragma unroll
  for (int i = 0; i < 3; ++i) st(T + (size_t)(QT_GP + i) * n2, gp[i]);
#pragma unroll
  for (int i = 0; i < 9; ++i) st(T + (size_t)(QT_GU + i) * n2, G[i]);
  st(T + (size_t)QT_DWDZ * n2, dwdz);
}

__device__ __forceinline__ void qtf_wl_at(const rh_qtf_design& q, const QtfWork& wk, int f, int m, const cd (&X)[6]) {
  const int n2 = q.n2;
  if (f >= n2) return;
  rh_c128* T = wk.wl + (size_t)m * WT_COUNT * n2 + f;
  const double w = q.w2[f], k = q.k2[f];
  cd eta = mk(0, 0), ud[3] = {mk(0, 0), mk(0, 0), mk(0, 0)}, dr2 = mk(0, 0), a[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
  if (qm(q, RH_QM_WL, m) != 0.0) {
    const double x = qm(q, RH_QM_RIX, m), y = qm(q, RH_QM_RIY, m), z = qm(q, RH_QM_RIZ, m);
    cd u[3];
    airy_u(w, k, q.beta, q.depth, x, y, z, u, &eta);
    ud[0] = iw(w, u[0]);
    ud[1] = iw(w, u[1]);
    ud[2] = iw(w, u[2]);
    cd dr[3];
    dr[0] = add(X[0], add(scl(X[5], -y), scl(X[4], z)));
    dr[1] = add(X[1], sub(scl(X[5], x), scl(X[3], z)));
    dr[2] = add(X[2], add(scl(X[4], -x), scl(X[3], y)));
#pragma unroll
    for (int i = 0; i < 3; ++i) a[i] = iw(w, iw(w, dr[i]));
    dr2 = dr[2];
  }
  // g_e1 = -g (cross(th, p1)[2] p1 + cross(th, p2)[2] p2)   (:1497-1499)
  const double p1[3] = {qm(q, RH_QM_P1X, m), qm(q, RH_QM_P1Y, m), qm(q, RH_QM_P1Z, m)};
  const double p2[3] = {qm(q, RH_QM_P2X, m), qm(q, RH_QM_P2Y, m), qm(q, RH_QM_P2Z, m)};
  const cd c1 = sub(scl(X[3], p1[1]), scl(X[4], p1[0]));
  const cd c2 = sub(scl(X[3], p2[1]), scl(X[4], p2[0]));
  st(T + (size_t)WT_ETAR * n2, sub(eta, dr2));
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st(T + (size_t)(WT_UD + i) * n2, ud[i]);
    st(T + (size_t)(WT_A + i) * n2, a[i]);
    st(T + (size_t)(WT_GE + i) * n2, scl(add(scl(c1, p1[i]), scl(c2, p2[i])), -q.g));
  }
}

// load a 3-vector field of a table
__device__ __forceinline__ void ld3(const rh_c128* T, int field, size_t n2, int f, cd* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = ld(T + (size_t)(field + i) * n2 + f);
}
__device__ __forceinline__ void ld3s(const rh_c128* T, int field, size_t n2, int f, cd* o) {   // f wave-uniform
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = lds(T + (size_t)(field + i) * n2 + f);
}

// Per (KAY radius row, frequency) factors of the Kim & Yue correction that do not depend on
// the pair: the reciprocals R_n = 1 / D_n of the Hankel-derivative table, and the interval
// factors cosh(k R H), sqrt(k R H tanh(k R H)) of raft_member.py:1185-1190 (H = h / R), and
// the exponentials exp(+-k (z + h)) at both interval ends, from which the pair kernel forms
// sinh((k1 +- k2)(z + h)) of :1176-1183 by products instead of four sinh per (pair, row).
__device__ __forceinline__ void qtf_kay_at(const rh_qtf_design& q, const QtfWork& wk, int f, int ir) {
  if (f >= q.n2) return;
  const rh_c128* D = q.hank + ((size_t)ir * q.n2 + f) * 12;
  rh_c128* R = wk.hinv + ((size_t)ir * q.n2 + f) * 12;
#pragma unroll
  for (int n = 0; n < 12; ++n) st(R + n, cdiv(mk(1, 0), ld(D + n)));
  const double Rr = q.kray[RH_KR_R * q.nkr + ir];
  const double kh = q.k2[f] * Rr * (q.depth / Rr);
  double* t = wk.kayt + ((size_t)ir * q.n2 + f) * kKayT;
  t[0] = cosh(kh);
  t[1] = sqrt(kh * tanh(kh));
  const double x1 = q.k2[f] * (q.kray[RH_KR_Z1 * q.nkr + ir] + q.depth);
  const double x2 = q.k2[f] * (q.kray[RH_KR_Z2 * q.nkr + ir] + q.depth);
  t[2] = exp(x1);
  t[3] = exp(-x1);
  t[4] = exp(x2);
  t[5] = exp(-x2);
  t[6] = kh / (t[1] * t[0]);          // the MFMA path's separable cc = t6(k1) t6(k2)
  t[7] = 1.0 / (q.k2[f] * Rr);
}

// Bessel J_n, Y_n (n = 0..12) without library calls: rh_bessel.h (checked against scipy on the
// CPU by tests/test_bessel.py and on the device by tests/test_gpu_qtf.py)
// D_n(k R) = 0.5 (H1_{n-1}(k R) - H1_{n+1}(k R)), n = 0..11, per (row, frequency); H1_{-1} = -H1_1
__global__ __launch_bounds__(64) void k_qtf_hankel(int n2, const double* __restrict__ k2, int nkr,
                                                   const double* __restrict__ R, rh_c128* __restrict__ hank) {
  const int f = blockIdx.x * 64 + threadIdx.x, ir = blockIdx.y;
  if (f >= n2 || ir >= nkr) return;
  const double x = k2[f] * R[ir];
  double J[13], Y[13];
  bessel_jy12(x, J, Y);
  rh_c128* o = hank + ((size_t)ir * n2 + f) * 12;
  st(o, mk(-J[1], -Y[1]));
#pragma unroll
  for (int n = 1; n < 12; ++n) st(o + n, mk(0.5 * (J[n - 1] - J[n + 1]), 0.5 * (Y[n - 1] - Y[n + 1])));
}

// k_qtf_tables: every per-(node | waterline member | KAY row, frequency) table in one launch
// (blockIdx.y = node, then member, then KAY row), after k_qtf_freq.  One launch instead of
// three small ones whose grids (a few hundred waves each) left the GPU mostly idle.
__global__ __launch_bounds__(64) void k_qtf_tables(rh_qtf_design q, QtfWork wk, int nw, const double* __restrict__ w,
                                                    const rh_c128* __restrict__ Xi0, const double* __restrict__ M66,
                                                    int fb0) {
  // blockIdx.y: the frequency row (k_qtf_freq before round 4), the nodes' motion tables,
  // waterline tables, then the nodes' incident-wave gradients (grad u, grad p, dw/dz) and KAY
  // tables; on the MFMA path also the node GEMM basis and the zero K-tail rows, as rows of their
  // own (more waves in flight).  Frequencies from 64 fb0: a call that computes only the
  // pair tiles of rows i1 >= 64 fb0 reads no table entry below (i2 >= i1 on every tile).
  const int f = (fb0 + blockIdx.x) * 64 + threadIdx.x;
  const bool basis = wk.R != nullptr && f < qtf_n2p(q);   // MFMA path operands (zero padded to n2p)
  int y = blockIdx.y;
  if (y == 0) {
    qtf_freq_at(q, nw, w, Xi0, M66, wk, f);
    return;
  }
  y -= 1;
  if (y < q.nq) {
    if (f < q.n2) {
      cd X[6];
      qtf_resample(q, nw, w, Xi0, f, X);
      qtf_nodes_motion_at(q, wk, f, y, X);
    }
    return;
  }
  y -= q.nq;
  if (y < q.nmq) {
    if (f < q.n2) {
      cd X[6];
      qtf_resample(q, nw, w, Xi0, f, X);
      qtf_wl_at(q, wk, f, y, X);
    }
    if (basis) qtf_wl_basis(q, wk, f, y);
    return;
  }
  y -= q.nmq;
  // the rows from here on depend on the incident wave only (kept by RH_QTF_INCIDENT_CACHED calls)
  if (y < q.nq) {
    qtf_nodes_grad_at(q, wk, f, y);
    return;
  }
  y -= q.nq;
  if (y < q.nkr) {
    qtf_kay_at(q, wk, f, y);
    if (basis) qtf_kay_basis(q, wk, f, y);
    return;
  }
  y -= q.nkr;
  if (!basis) return;
  if (y < q.nq) {
    qtf_node_basis(q, wk, f, y);
    return;
  }
  y -= q.nq;
  if (y < qtf_npad(q)) qtf_pad_row(q, wk, f, y);
}

// omega of raft_member.py:1102-1109, 1 / (H'_{n+1}(k1R) conj H'_n(k2R)) - 1 / (H'_n(k1R) conj H'_{n+1}(k2R)),
// from the reciprocal tables R1 = 1/D(k1 R), R2 = 1/D(k2 R): division-free
__device__ __forceinline__ cd kay_omega(const rh_c128* R1, const rh_c128* R2, int n) {   // R1 wave-uniform
  return sub(mul(lds(R1 + n + 1), cconj(ld(R2 + n))), mul(lds(R1 + n), cconj(ld(R2 + n + 1))));
}

// Row k of this rank is i1 = k nrank + (k even ? rank : nrank-1-rank): a snake deal of the
// upper-triangle rows (longest first), so every rank gets the same pair count to within one
// row.  mirror = write the Hermitian lower triangle too (single device); sharded runs
// mirror after the exchange (k_qtf_fill).
//
// A workgroup is NWV (W) waves on the SAME 64 pairs (one w1 row, 64 consecutive w2).  The terms
// of a pair are split over the waves: wave w takes nodes w, w+W, ..., the waterline terms
// of members w, w+W, ... and the Kim & Yue radius rows W-1-w, 2W-1-w, ... (reversed, so the
// waves with one node fewer get the extra row), wave 0 also the Pinkster IV term.  The W
// partial sums meet in LDS and wave 0 adds them in wave order (deterministic).  With one
// wave per 64 pairs a row-sharded grid (80k pairs / 8 GPUs) is ~0.2 waves per SIMD; W waves
// multiply the resident waves by W (on one GPU, 1 to 4 waves are within 1 %).
//
// Occupancy: left alone the compiler spends 256 VGPRs + AGPRs (1 wave per SIMD).  Asking
// for 2 waves per SIMD costs ~40 spilled VGPRs (the wave-uniform w1 side and the node and
// member tables come through scalar loads, so SGPRs carry them); C3 QTF 0.71 -> 0.50 ms.
// 3 or 4 waves per SIMD spill 100-300 VGPRs and are slower (tools/ubench/run_qtf_variants.sh).
#if !defined(RH_QTF_WPE)
#define RH_QTF_WPE 2
#endif
#define RH_QTF_ATTR __attribute__((amdgpu_waves_per_eu(RH_QTF_WPE)))
template <int NWV>
__global__ __launch_bounds__(kQtfTile * NWV) RH_QTF_ATTR void k_qtf_pairs(rh_qtf_design q, QtfWork wk, rh_c128* __restrict__ qtf,
                                                            int rank, int nrank, int mirror) {
  __shared__ double red[(NWV > 1 ? NWV - 1 : 1) * 12 * kQtfTile];
  const int kr = (int)blockIdx.y;
  const int i1 = kr * nrank + ((kr & 1) ? nrank - 1 - rank : rank);
  const int lane = (int)threadIdx.x & (kQtfTile - 1);
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kQtfTile);
  // Tile t of row i1 covers w2 = i1 + 64 t .. i1 + 64 t + 63: the tiles start on the diagonal,
  // so only the last tile of a row is partial (C3: 1,456 tiles instead of 1,744 aligned ones,
  // 14 % idle lanes instead of 28 %).
  const int i2 = i1 + (int)blockIdx.x * kQtfTile + lane;
  const int n2 = q.n2;
  if (i1 >= n2 || i1 + (int)blockIdx.x * kQtfTile >= n2) return;     // block-uniform
  const bool active = i2 < n2 && q.w2[i2] >= q.w2[i1];
  const int i2s = active ? i2 : i1;         // inactive lanes compute a harmless valid pair
  const double w1 = ldsd(q.w2 + i1), w2 = q.w2[i2s], k1 = ldsd(q.k2 + i1), k2 = q.k2[i2s];
  const double h = q.depth, rho = q.rho, g = q.g, beta = q.beta;
  cd Q[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) Q[i] = mk(0, 0);
  // ---- Pinkster IV: rotation of the first-order force (:1449-1456)
  if (wv == 0) {
    cd th1[3], th2c[3], F1a[3], F1b[3], F2c[3], tmp1[3], tmp2[3];
    ld3s(wk.freq, FT_XI + 3, n2, i1, th1);
    ld3(wk.freq, FT_XI + 3, n2, i2s, th2c);
#pragma unroll
    for (int i = 0; i < 3; ++i) th2c[i] = cconj(th2c[i]);
    for (int part = 0; part < 2; ++part) {
      ld3(wk.freq, FT_F1 + 3 * part, n2, i2s, F2c);
      ld3s(wk.freq, FT_F1 + 3 * part, n2, i1, F1a);
#pragma unroll
      for (int i = 0; i < 3; ++i) F2c[i] = cconj(F2c[i]);
      cross_cc(th1, F2c, tmp1);
      cross_cc(th2c, F1a, tmp2);
#pragma unroll
      for (int i = 0; i < 3; ++i) Q[3 * part + i] = scl(add(tmp1[i], tmp2[i]), 0.25);
      (void)F1b;
    }
  }
  // ---- pair constants of the second-order potential (raft/helpers.py:254-291, Q1)
  const bool pot_on = (w1 != w2) && (k1 > 0) && (k2 > 0);
  double kx = 0, ky = 0, nk = 0, den12 = 1, den21 = 1, tnh = 0, cnh = 1, icnh = 1;
  cd aux2 = mk(0, 0);
  if (pot_on) {
    const double b = beta * kDeg2Rad, cb = cos(b), sb = sin(b);
    kx = k1 * cb - k2 * cb;
    ky = k1 * sb - k2 * sb;
    nk = sqrt(kx * kx + ky * ky);
    const double t1 = tanh(k1 * h), t2 = tanh(k2 * h);
    tnh = tanh(nk * h);
    cnh = cosh(nk * h);
    icnh = 1.0 / cnh;
    den12 = (w1 - w2) * (w1 - w2) / g - nk * tnh;
    den21 = (w2 - w1) * (w2 - w1) / g - nk * tnh;
    const double n12 = (k1 * k1) * (1 - t1 * t1) - 2 * k1 * k2 * (1 + t1 * t2);
    const double n21 = (k2 * k2) * (1 - t2 * t2) - 2 * k2 * k1 * (1 + t2 * t1);
    const cd g12 = scl(mk(0, -g / (2 * w1)), n12 / den12);
    const cd g21 = scl(mk(0, -g / (2 * w2)), n21 / den21);
    aux2 = scl(add(g21, cconj(g12)), 0.5);
  }
  cd om1[3], om2[3];
  ld3s(wk.freq, FT_OM, n2, i1, om1);
  ld3(wk.freq, FT_OM, n2, i2s, om2);
  // OMEGA = -getH(i w th):  -H = [[0,-v2,v1],[v2,0,-v0],[-v1,v0,0]]
  const cd O1[9] = {mk(0, 0), scl(om1[2], -1), om1[1], om1[2], mk(0, 0), scl(om1[0], -1), scl(om1[1], -1), om1[0], mk(0, 0)};
  const cd O2[9] = {mk(0, 0), scl(om2[2], -1), om2[1], om2[2], mk(0, 0), scl(om2[0], -1), scl(om2[1], -1), om2[0], mk(0, 0)};

  // Node terms.  The five term groups of a node share their outer operators, so they are
  // summed before those are applied (linear algebra, reassociated within FP64 rounding):
  //   f = (rv CM + rve QM) vM + rv CA vA + rv (I - QM) ax + (ai sq) q
  // vM: second-order potential acceleration (1), convective (2) and body-motion (4)
  //     accelerations, with G1 and conj(G2) each applied once to the summed vectors;
  // vA: Rainey axial divergence (3) and the CA terms of the body rotation (5);
  // ax: the (I - qMat) term of (5);  sq: the pressure terms of (1), (2) and (4).
  // One translateForce3to6DOF per node instead of five.
#pragma unroll 1
  for (int n = wv; n < q.nq; n += NWV) {
    const rh_c128* T = wk.node + (size_t)n * QT_COUNT * n2;
    const double rx = qn(q, RH_QN_RX, n), ry = qn(q, RH_QN_RY, n), rz = qn(q, RH_QN_RZ, n);
    const double qv[3] = {qn(q, RH_QN_QX, n), qn(q, RH_QN_QY, n), qn(q, RH_QN_QZ, n)};
    const double rv = rho * qn(q, RH_QN_VI, n);
    const double rve = rho * qn(q, RH_QN_VE, n) * qn(q, RH_QN_CAE, n);
    const double ai = qn(q, RH_QN_AI, n);
    cd vM[3], vA[3], sq = mk(0, 0);
    cd u1[3], u2[3], vp1[3], vp2[3], ur1[3], ur2[3];
    ld3s(T, QT_U, n2, i1, u1);
    ld3(T, QT_U, n2, i2s, u2);
    ld3s(T, QT_VP, n2, i1, vp1);
    ld3(T, QT_VP, n2, i2s, vp2);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ur1[i] = sub(u1[i], vp1[i]);
      ur2[i] = sub(u2[i], vp2[i]);
    }
    // (2) convective acceleration (:1545-1546) + (4) body motion in the first-order field
    // (:1552-1553): 0.25 [G1 (conj(u2) + i w1 conj(dr2)) + conj(G2) (u1 - i w2 dr1)]
    {
      cd dr1[3], d2c[3], x1v[3], x2v[3], c1v[3], c2v[3];
      ld3s(T, QT_DR, n2, i1, dr1);
      ld3(T, QT_DR, n2, i2s, d2c);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        d2c[i] = cconj(d2c[i]);
        x1v[i] = add(cconj(u2[i]), iw(w1, d2c[i]));
        x2v[i] = add(u1[i], iw(-w2, dr1[i]));
      }
      cd G1[9], G2c[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        G1[i] = lds(T + (size_t)(QT_GU + i) * n2 + i1);
        G2c[i] = cconj(ld(T + (size_t)(QT_GU + i) * n2 + i2s));
      }
      cmv(G1, x1v, c1v);
      cmv(G2c, x2v, c2v);
#pragma unroll
      for (int i = 0; i < 3; ++i) vM[i] = scl(add(c1v[i], c2v[i]), 0.25);
      // pressure: Bernoulli drop of (2) (:1593-1594) and grad p . dr of (4) (:1590-1592)
      double M9[9];
      cd t5[3], cu2[3], gp1[3], gp2[3];
      ldm9(q, RH_QN_P12, n, M9);
      rmv(M9, ur1, t5);
      ldm9(q, RH_QN_CA, n, M9);
      rmv(M9, ur2, cu2);
      ld3s(T, QT_GP, n2, i1, gp1);
      ld3(T, QT_GP, n2, i2s, gp2);
      cd pd = mk(0, 0), pn = mk(0, 0), pm = mk(0, 0);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        pd = add(pd, mul(t5[i], cconj(cu2[i])));
        pn = add(pn, mul(gp1[i], d2c[i]));
        pm = add(pm, mul(cconj(gp2[i]), dr1[i]));
      }
      sq = add(scl(pd, -2 * 0.25 * 0.5 * rho), add(scl(pn, 0.25), scl(pm, 0.25)));
    }
    // (1) second-order potential acceleration and pressure (f_2ndPot :1541-1542, :1587-1588)
    if (pot_on && rz <= 0) {
      const double ez = exp(nk * (rz + h)), iez = 1.0 / ez;     // cosh, sinh of nk (z + h)
      const double kxy = 0.5 * (ez + iez) * icnh, kz = 0.5 * (ez - iez) * icnh;
      const double th = kx * rx + ky * ry + 0 * rz;
      double sth, cth;
      sincos(th, &sth, &cth);
      const cd ph = mk(cth, -sth);
      const cd base = mul(scl(aux2, kxy), ph);
      vM[0] = add(vM[0], scl(base, (w1 - w2) * kx));
      vM[1] = add(vM[1], scl(base, (w1 - w2) * ky));
      vM[2] = add(vM[2], mul(mul(scl(aux2, kz), ph), mk(0, (w1 - w2) * nk)));
      sq = add(sq, mul(base, mk(0, -rho * (w1 - w2))));
    }
    // (3) Rainey axial divergence (raft/helpers.py:228-251)
    {
      const cd dz1 = lds(T + (size_t)QT_DWDZ * n2 + i1), dz2 = ld(T + (size_t)QT_DWDZ * n2 + i2s);
      const cd s1 = add(add(scl(u1[0], qv[0]), scl(u1[1], qv[1])), scl(u1[2], qv[2]));
      const cd s2 = add(add(scl(u2[0], qv[0]), scl(u2[1], qv[1])), scl(u2[2], qv[2]));
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const cd up1 = sub(u1[i], scl(s1, qv[i])), up2 = sub(u2[i], scl(s2, qv[i]));
        vA[i] = scl(add(mul(dz1, cconj(sub(up2, vp2[i]))), mul(cconj(dz2), sub(up1, vp1[i]))), 0.25);
      }
      const cd aq = add(add(scl(vA[0], qv[0]), scl(vA[1], qv[1])), scl(vA[2], qv[2]));
#pragma unroll
      for (int i = 0; i < 3; ++i) vA[i] = sub(vA[i], scl(aq, qv[i]));
    }
    // (5) Rainey body-rotation terms (:1556-1575)
    cd fr[3];
    {
      cd x1[3], x2[3], t4[3], t5[3];
      double CA[9], QM[9];
      ldm9(q, RH_QN_CA, n, CA);
      ldm9(q, RH_QN_QM, n, QM);
      const cd va1 = lds(T + (size_t)QT_VA * n2 + i1), va2 = ld(T + (size_t)QT_VA * n2 + i2s);
      const cd va2q[3] = {cconj(scl(va2, qv[0])), cconj(scl(va2, qv[1])), cconj(scl(va2, qv[2]))};
      const cd va1q[3] = {scl(va1, qv[0]), scl(va1, qv[1]), scl(va1, qv[2])};
      cd O2c[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) O2c[i] = cconj(O2[i]);
      cmv(O1, va2q, x1);
      cmv(O2c, va1q, x2);
#pragma unroll
      for (int i = 0; i < 3; ++i) vA[i] = sub(vA[i], scl(add(x1[i], x2[i]), 0.5));
      cd V1[9], V2c[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        V1[i] = add(lds(T + (size_t)(QT_GU + i) * n2 + i1), O1[i]);
        V2c[i] = cconj(add(ld(T + (size_t)(QT_GU + i) * n2 + i2s), O2[i]));
      }
      // aux = 0.25 (V1 conj(CaM u2a) + conj(V2) CaM u1a); aux -= qMat aux
      cd cu1[3], cu2c[3];
      rmv(CA, ur1, cu1);
      rmv(CA, ur2, cu2c);
#pragma unroll
      for (int i = 0; i < 3; ++i) cu2c[i] = cconj(cu2c[i]);
      cmv(V1, cu2c, x1);
      cmv(V2c, cu1, x2);
      cd ax[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) ax[i] = scl(add(x1[i], x2[i]), 0.25);
      rmv(QM, ax, t4);
#pragma unroll
      for (int i = 0; i < 3; ++i) fr[i] = sub(ax[i], t4[i]);
      // u_aux -= qMat u_aux ; aux = 0.25 (CaM V1 conj(u2a) + CaM conj(V2) u1a): into vA
      cd w1a[3], w2a[3];
      rmv(QM, ur1, t4);
      rmv(QM, ur2, t5);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        w1a[i] = sub(ur1[i], t4[i]);
        w2a[i] = cconj(sub(ur2[i], t5[i]));
      }
      cmv(V1, w2a, x1);
      cmv(V2c, w1a, x2);
#pragma unroll
      for (int i = 0; i < 3; ++i) vA[i] = sub(vA[i], scl(add(x1[i], x2[i]), 0.25));
      cd tA[3];
      rmv(CA, vA, tA);
#pragma unroll
      for (int i = 0; i < 3; ++i) fr[i] = add(fr[i], tA[i]);
    }
    {
      double CM[9], QM[9], MP[9];
      ldm9(q, RH_QN_CM, n, CM);
      ldm9(q, RH_QN_QM, n, QM);
#pragma unroll
      for (int i = 0; i < 9; ++i) MP[i] = rv * CM[i] + rve * QM[i];
      cd tM[3], f[3];
      rmv(MP, vM, tM);
      const cd sa = scl(sq, ai);
#pragma unroll
      for (int i = 0; i < 3; ++i) f[i] = add(add(tM[i], scl(fr[i], rv)), scl(sa, qv[i]));
      acc6(Q, f, rx, ry, rz);
    }
  }
  // ---- waterline relative-elevation force (:1602-1630)
#pragma unroll 1
  for (int m = wv; m < q.nmq; m += NWV) {
    if (qm(q, RH_QM_WL, m) != 0.0) {
      const rh_c128* W = wk.wl + (size_t)m * WT_COUNT * n2;
      const cd e1 = lds(W + (size_t)WT_ETAR * n2 + i1), e2c = cconj(ld(W + (size_t)WT_ETAR * n2 + i2s));
      cd ud1[3], ud2[3], a1[3], a2[3], ge1[3], ge2[3];
      ld3s(W, WT_UD, n2, i1, ud1);
      ld3(W, WT_UD, n2, i2s, ud2);
      ld3s(W, WT_A, n2, i1, a1);
      ld3(W, WT_A, n2, i2s, a2);
      ld3s(W, WT_GE, n2, i1, ge1);
      ld3(W, WT_GE, n2, i2s, ge2);
      double CM[9], CA[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        CM[i] = qm(q, RH_QM_CM + i, m);
        CA[i] = qm(q, RH_QM_CA + i, m);
      }
      const double ra = rho * qm(q, RH_QM_AWL, m);
      cd fe[3], ae[3], t3[3], t4[3], fo[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        fe[i] = scl(add(mul(ud1[i], e2c), mul(cconj(ud2[i]), e1)), 0.25);
        ae[i] = scl(add(mul(a1[i], e2c), mul(cconj(a2[i]), e1)), 0.25);
      }
      rmv(CM, fe, t3);
      rmv(CA, ae, t4);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const cd gt = add(mul(ge1[i], e2c), mul(cconj(ge2[i]), e1));
        fo[i] = sub(sub(scl(t3[i], ra), scl(t4[i], ra)), scl(gt, 0.25 * ra));
      }
      acc6(Q, fo, qm(q, RH_QM_RIX, m), qm(q, RH_QM_RIY, m), qm(q, RH_QM_RIZ, m));
    }
  }
  // ---- Kim & Yue second-order diffraction (raft/raft_member.py:1090-1205), one radius row
  // at a time; conj(F) when k1 < k2 is applied per row (conj is exact and
  // linear, so it equals conj of the member sum)
  {
    const bool cj = k1 < k2;
    const double cb = cos(beta), sb = sin(beta);
    const double kkx = k1 * cb - k2 * cb, kky = k1 * sb - k2 * sb;
    int m = 0, mph = -1;
    cd ph = mk(1, 0);
#pragma unroll 1
    for (int ir = NWV - 1 - wv; ir < q.nkr; ir += NWV) {
      while (ldsi(q.kstart + m + 1) <= ir) ++m;          // member of row ir (rows ascend)
      const int r0 = ldsi(q.kstart + m);
      const double wx = qm(q, RH_QM_WLX, m), wy = qm(q, RH_QM_WLY, m), wz = qm(q, RH_QM_WLZ, m);
      if (m != mph) {   // phase of the member's waterline point, once per member (uniform)
        const double thp = kkx * wx + kky * wy + 0 * wz;
        double sp, cp;
        sincos(thp, &sp, &cp);
        ph = mk(cp, -sp);
        mph = m;
      }
      const double pf[3] = {qm(q, RH_QM_PFX, m), qm(q, RH_QM_PFY, m), qm(q, RH_QM_PFZ, m)};
      const double R = ldsd(q.kray + RH_KR_R * q.nkr + ir);
      const rh_c128* D1 = wk.hinv + ((size_t)ir * n2 + i1) * 12;
      const rh_c128* D2 = wk.hinv + ((size_t)ir * n2 + i2s) * 12;
      const double k1R = k1 * R, k2R = k2 * R;
      double sre;
      double px, py, pz;
      if (ir == r0) {       // waterline term (:1133-1149)
        const cd c0 = mk(0, -rho * g * R * 2 / M_PI / (k1R * k2R));
        cd s = mk(0, 0);
#pragma unroll
        for (int nn = 0; nn <= 10; ++nn) s = add(s, kay_omega(D1, D2, nn));
        sre = mul(c0, s).r;
        px = wx;
        py = wy;
        pz = wz;
      } else {              // node-interval Bernoulli term (:1155-1200)
        const double z1 = ldsd(q.kray + RH_KR_Z1 * q.nkr + ir), z2 = ldsd(q.kray + RH_KR_Z2 * q.nkr + ir);
        const double H = h / R;
        const double k1h = k1R * H, k2h = k2R * H;
        const double* t1 = wk.kayt + ((size_t)ir * n2 + i1) * kKayT;
        const double* t2 = wk.kayt + ((size_t)ir * n2 + i2s) * kKayT;
        // sinh((k1 +- k2) x) = (e^{k1 x} e^{+-k2 x} - e^{-k1 x} e^{-+k2 x}) / 2 at x = z1 + h, z2 + h
        const double P1 = ldsd(t1 + 2), M1 = ldsd(t1 + 3), P2 = ldsd(t1 + 4), M2 = ldsd(t1 + 5);
        const double p1 = t2[2], m1 = t2[3], p2 = t2[4], m2 = t2[5];
        const double ia = 0.5 / (k1h + k2h);
        double Im, Ip;
        const double a2 = (P2 * p2 - M2 * m2) * ia, a1 = (P1 * p1 - M1 * m1) * ia;
        if (w1 == w2) {
          Im = 0.5 * (a2 - (z2 + h) / h - a1 + (z1 + h) / h);
          Ip = 0.5 * (a2 + (z2 + h) / h - a1 - (z1 + h) / h);
        } else {
          const double id = 0.5 / (k1h - k2h);
          const double d2 = (P2 * m2 - M2 * p2) * id, d1 = (P1 * m1 - M1 * p1) * id;
          Im = 0.5 * (a2 - d2 - a1 + d1);
          Ip = 0.5 * (a2 + d2 - a1 - d1);
        }
        // coef / (cosh(k1 R H) cosh(k2 R H)) and Ip / (k1R k2R), hoisted out of the n sum
        const double cc = k1h * k2h / (ldsd(t1 + 1) * t2[1] * ldsd(t1) * t2[0]);
        const double ipr = Ip / (k1R * k2R);
        const cd c0 = mk(0, rho * g * R * 2 / M_PI / (k1R * k2R));
        cd s = mk(0, 0);
#pragma unroll   // all 12 table entries in flight at once (0.365 -> 0.343 ms, r01_v9)
        for (int nn = 0; nn <= 10; ++nn) s = add(s, scl(kay_omega(D1, D2, nn), cc * (Im + ipr * (nn * (nn + 1)))));
        sre = mul(c0, s).r;
        px = ldsd(q.kray + RH_KR_MX * q.nkr + ir);
        py = ldsd(q.kray + RH_KR_MY * q.nkr + ir);
        pz = ldsd(q.kray + RH_KR_MZ * q.nkr + ir);
      }
      const cd Fs = scl(ph, sre);    // real part times the phase of the waterline point
      cd fv[3] = {scl(Fs, pf[0]), scl(Fs, pf[1]), scl(Fs, pf[2])};
      if (cj) {
#pragma unroll
        for (int i = 0; i < 3; ++i) fv[i] = cconj(fv[i]);
      }
      acc6(Q, fv, px, py, pz);
    }
  }
  // ---- the NWV partial sums meet in LDS; wave 0 adds them in wave order
  if (NWV > 1) {
    if (wv > 0) {
      double* r = red + (size_t)(wv - 1) * 12 * kQtfTile;
#pragma unroll
      for (int d = 0; d < 6; ++d) {
        r[(2 * d) * kQtfTile + lane] = Q[d].r;
        r[(2 * d + 1) * kQtfTile + lane] = Q[d].i;
      }
    }
    __syncthreads();
    if (wv > 0) return;
#pragma unroll 1
    for (int v = 0; v < NWV - 1; ++v) {
      const double* r = red + (size_t)v * 12 * kQtfTile;
#pragma unroll
      for (int d = 0; d < 6; ++d) Q[d] = add(Q[d], mk(r[(2 * d) * kQtfTile + lane], r[(2 * d + 1) * kQtfTile + lane]));
    }
  }
  if (!active) return;
  // Hermitian fill (:1639-1640): qtf + conj(qtf).T - diag(conj(diag(qtf)))
  rh_c128* up = qtf + ((size_t)i1 * n2 + i2) * 6;
  if (!mirror) {
#pragma unroll
    for (int d = 0; d < 6; ++d) st(up + d, Q[d]);
  } else if (i1 == i2) {
#pragma unroll
    for (int d = 0; d < 6; ++d) st(up + d, sub(add(Q[d], cconj(Q[d])), cconj(Q[d])));
  } else {
    rh_c128* lo = qtf + ((size_t)i2 * n2 + i1) * 6;
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      st(up + d, Q[d]);
      st(lo + d, cconj(Q[d]));
    }
  }
}

template __global__ void k_qtf_pairs<1>(rh_qtf_design, QtfWork, rh_c128*, int, int, int);
template __global__ void k_qtf_pairs<2>(rh_qtf_design, QtfWork, rh_c128*, int, int, int);
template __global__ void k_qtf_pairs<4>(rh_qtf_design, QtfWork, rh_c128*, int, int, int);

// Hermitian fill of a row-sharded QTF after the exchange: lower[i2][i1] = conj(upper[i1][i2]);
// the diagonal keeps q + conj(q) - conj(q) == q exactly (raft/raft_fowt.py:1639-1640)
__global__ __launch_bounds__(256) void k_qtf_fill(int n2, rh_c128* __restrict__ qtf) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n2 * n2 * 6) return;
  const int d = (int)(t % 6);
  const size_t p = t / 6;
  const int i = (int)(p / n2), j = (int)(p % n2);
  if (i <= j) return;                                  // lower triangle only
  st(qtf + p * 6 + d, cconj(ld(qtf + ((size_t)j * n2 + i) * 6 + d)));
}

// ---------------------------------------------------------------------------------------
// second-order force spectrum: block per difference-frequency index mu
// ---------------------------------------------------------------------------------------
// RegularGridInterpolator(linear): i = searchsorted(grid, x) - 1 clipped to [0, n-2]
__device__ __forceinline__ bool grid_cell(const double* g, int n, double x, int& i, double& t) {
  if (x < g[0] || x > g[n - 1]) return false;          // fill_value = 0 strictly outside
  int lo = 0, hi = n;                                     // searchsorted side='left'
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (g[mid] < x) lo = mid + 1; else hi = mid;
  }
  i = lo - 1;
  if (i < 0) i = 0;
  if (i > n - 2) i = n - 2;
  t = (x - g[i]) / (g[i + 1] - g[i]);
  return true;
}

// One difference-frequency index mu (0 = mean drift, 1..nw-1) of one (QTF, spectrum) pair, one
// 256-thread block.  kCplx: f is complex [6][nw] (the fext rows of a batched solve, imaginary part
// 0), else real [6][nw].  The same arithmetic in both forms, so the bits agree.
template <bool kCplx>
__device__ __forceinline__ void force2nd_block(int mu, int n2, const double* __restrict__ w2,
                                               const rh_c128* __restrict__ qtf, int nw, const double* __restrict__ w,
                                               double dw, const double* __restrict__ S0, double* __restrict__ fout,
                                               double* __restrict__ fmean) {
  __shared__ double red[4][6];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int i = tid; i + mu < nw; i += 256) {
    const int j = i + mu;
    int iy, ix;
    double ty, tx;
    cd v[6];
    // value at (y = w_i, x = w_j): z[y, x] orientation
    if (grid_cell(w2, n2, w[i], iy, ty) && grid_cell(w2, n2, w[j], ix, tx)) {
      const rh_c128* a = qtf + ((size_t)iy * n2 + ix) * 6;
      const rh_c128* b = qtf + ((size_t)iy * n2 + ix + 1) * 6;
      const rh_c128* c = qtf + ((size_t)(iy + 1) * n2 + ix) * 6;
      const rh_c128* e = qtf + ((size_t)(iy + 1) * n2 + ix + 1) * 6;
#pragma unroll
      for (int d = 0; d < 6; ++d) {
        const cd A = ld(a + d), B = ld(b + d), C = ld(c + d), E = ld(e + d);
        v[d] = add(add(add(scl(A, (1 - ty) * (1 - tx)), scl(B, (1 - ty) * tx)), scl(C, ty * (1 - tx))), scl(E, ty * tx));
      }
    } else {
#pragma unroll
      for (int d = 0; d < 6; ++d) v[d] = mk(0, 0);
    }
    if (mu == 0) {
#pragma unroll
      for (int d = 0; d < 6; ++d) acc[d] += S0[i] * v[d].r;
    } else {
      const double ss = S0[i] * S0[j];
#pragma unroll
      for (int d = 0; d < 6; ++d) acc[d] += ss * abs2(v[d]);
    }
  }
#pragma unroll
  for (int d = 0; d < 6; ++d) {
    const double s = wave_sum(acc[d]);
    if (lane == 0) red[wv][d] = s;
  }
  __syncthreads();
  if (tid < 6) {
    const double s = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    const int bin = mu == 0 ? nw - 1 : mu - 1;            // shifted by one bin (:1809-1810)
    const double val = mu == 0 ? 0.0 : 4 * sqrt(s) * dw;  // the last bin has no difference frequency
    if (mu == 0) fmean[tid] = 2 * s * dw;
    if (kCplx) {
      fout[2 * ((size_t)tid * nw + bin)] = val;
      fout[2 * ((size_t)tid * nw + bin) + 1] = 0.0;
    } else {
      fout[(size_t)tid * nw + bin] = val;
    }
  }
}

__global__ __launch_bounds__(256) void k_force2nd(int n2, const double* __restrict__ w2, const rh_c128* __restrict__ qtf,
                                                   int nw, const double* __restrict__ w, double dw,
                                                   const double* __restrict__ S0, double* __restrict__ fout,
                                                   double* __restrict__ fmean) {
  force2nd_block<false>(blockIdx.x, n2, w2, qtf, nw, w, dw, S0, fout, fmean);
}

// Batched form: block (mu, case); case c uses QTF qidx[c] of the stack qtf [nq][n2][n2][6] (qidx
// NULL: QTF 0) and spectrum S0[c] [nw]; f [ncase][6][nw] complex, f_mean [ncase][6].
__global__ __launch_bounds__(256) void k_force2nd_batch(int n2, const double* __restrict__ w2,
                                                         const rh_c128* __restrict__ qtf, const int* __restrict__ qidx,
                                                         int nq, int nw, const double* __restrict__ w, double dw,
                                                         const double* __restrict__ S0, rh_c128* __restrict__ f,
                                                         double* __restrict__ fmean) {
  const int c = blockIdx.y;
  const int qi = qidx ? qidx[c] : 0;
  if (qi < 0 || qi >= nq) {               // uniform per block: a bad index gives NaN, never a stray read
    if (threadIdx.x < 6) {
      const double nan = __builtin_nan("");
      const int mu = blockIdx.x;
      const int bin = mu == 0 ? nw - 1 : mu - 1;
      f[((size_t)c * 6 + threadIdx.x) * nw + bin] = rh_c128{nan, nan};
      if (mu == 0) fmean[(size_t)c * 6 + threadIdx.x] = nan;
    }
    return;
  }
  force2nd_block<true>(blockIdx.x, n2, w2, qtf + (size_t)qi * n2 * n2 * 6, nw, w, dw, S0 + (size_t)c * nw,
                       reinterpret_cast<double*>(f + (size_t)c * 6 * nw), fmean + (size_t)c * 6);
}

// ---------------------------------------------------------------------------------------
// second-order force spectrum, 'spectrum' interpolation mode (raft/raft_fowt.py:1760-1784)
// ---------------------------------------------------------------------------------------
// np.interp(x, xp, fp, left=0, right=0) for increasing xp: j with xp[j] <= x < xp[j+1];
// x == xp[j] (and x == xp[n-1]) returns fp[j] exactly, else slope (x - xp[j]) + fp[j].
__device__ __forceinline__ double np_interp0(double x, const double* xp, const double* fp, int n, int stride = 1) {
  if (!(x >= xp[0]) || x > xp[n - 1]) return 0.0;
  int lo = 0, hi = n - 1;                 // invariant xp[lo] <= x, and x < xp[hi] or hi == n-1
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (xp[mid] <= x) lo = mid; else hi = mid;
  }
  if (x == xp[n - 1]) return fp[(size_t)(n - 1) * stride];
  const double y0 = fp[(size_t)lo * stride];
  if (xp[lo] == x) return y0;
  const double y1 = fp[(size_t)hi * stride];
  const double slope = (y1 - y0) / (xp[hi] - xp[lo]);
  return slope * (x - xp[lo]) + y0;
}

// Stage 1, block per difference-frequency index mu of the QTF grid: S = interp(w2, w, S0) on
// the fly, Sf[d][mu] = 8 sum_i S_i S_{i+mu} |Q_d(i, i+mu)|^2 dw2 (mu >= 1, Sf[d][0] = 0) and the
// mean drift f_mean[d] = 2 sum_i S_i Re Q_d(i, i) dw2 (mu == 0).  Upper half of the QTF only.
__global__ __launch_bounds__(256) void k_force2nd_spec(int n2, const double* __restrict__ w2, const rh_c128* __restrict__ qtf,
                                                        int nw, const double* __restrict__ w,
                                                        const double* __restrict__ S0, double* __restrict__ Sf,
                                                        double* __restrict__ fmean) {
  __shared__ double red[4][6];
  const int mu = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const double dw2 = w2[1] - w2[0];
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int i = tid; i + mu < n2; i += 256) {
    const int j = i + mu;
    const double Si = np_interp0(w2[i], w, S0, nw);
    const rh_c128* q = qtf + ((size_t)i * n2 + j) * 6;
    if (mu == 0) {
#pragma unroll
      for (int d = 0; d < 6; ++d) acc[d] += Si * ld(q + d).r;
    } else {
      const double ss = Si * np_interp0(w2[j], w, S0, nw);
#pragma unroll
      for (int d = 0; d < 6; ++d) acc[d] += ss * abs2(ld(q + d));
    }
  }
#pragma unroll
  for (int d = 0; d < 6; ++d) {
    const double s = wave_sum(acc[d]);
    if (lane == 0) red[wv][d] = s;
  }
  __syncthreads();
  if (tid < 6) {
    const double s = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    if (mu == 0) {
      fmean[tid] = 2 * s * dw2;
      Sf[(size_t)tid * n2] = 0.0;
    } else {
      Sf[(size_t)tid * n2 + mu] = 8 * s * dw2;
    }
  }
}

// Stage 2, thread per (dof, output bin): Sf_interp = interp(w - w[0], w2 - w2[0], Sf, 0, 0),
// f = sqrt(2 Sf_interp dw), shifted by one bin with a zero last bin (:1781-1784, 1809-1810).
__global__ __launch_bounds__(256) void k_force2nd_spec_out(int n2, const double* __restrict__ w2, int nw,
                                                            const double* __restrict__ w, double dw,
                                                            const double* __restrict__ Sf, double* __restrict__ fout) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 6 * nw) return;
  const int d = t / nw, b = t % nw;
  if (b == nw - 1) {
    fout[t] = 0.0;
    return;
  }
  // the grid mu = w2 - w2[0], formed per probe (a binary search reads log2(n2) entries)
  const double x = w[b + 1] - w[0], w20 = w2[0];
  double v = 0.0;
  if (x >= 0.0 && x <= w2[n2 - 1] - w20) {
    int lo = 0, hi = n2 - 1;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (w2[mid] - w20 <= x) lo = mid; else hi = mid;
    }
    const double* S = Sf + (size_t)d * n2;
    const double xl = w2[lo] - w20, xh = w2[hi] - w20;
    if (x == w2[n2 - 1] - w20) v = S[n2 - 1];
    else if (xl == x) v = S[lo];
    else v = (S[hi] - S[lo]) / (xh - xl) * (x - xl) + S[lo];
  }
  fout[t] = sqrt(2 * v * dw);
}

}  // namespace rh
