// rh_qtf_mfma.hip -- the QTF pair sum of calcQTF_slenderBody as FP64 MFMA GEMMs on gfx950
// (raft/raft_fowt.py:1449-1640, raft/raft_member.py:1090-1205).
//
// Every node, waterline and Pinkster term of a pair (w1 <= w2) is a product of a w1-side
// first-order quantity and the conjugate of a w2-side one (raft_fowt.py:1521-1630: the
// reference multiplies w1 quantities by np.conj of w2 quantities throughout), so
//     Q_d(i1, i2) = sum_k L_d[k](i1) R[k](i2),   R[k] = conj(basis_k(w2)).
// The w2-side node quantities are linear in a small basis: the incident velocity u is
// (cos b c0, sin b c0, c1), grad u is g0 A + g1 B, grad p is (cb p0, sb p0, p1) with constant
// direction matrices (Q1/Q2 quirks included), and the body-motion terms dr, v_perp, v_axial,
// omega and the Pinkster / waterline motions are linear in X, w X and w^2 X of the RAO.
// K = 8 per node + 3 per waterline member + 18 motions (C3: 238 against the 26 x 23
// complex table entries one pair reads in the direct kernel).  L is found by probing the
// bilinear node/waterline/Pinkster functions with the basis vectors (k_qtf_lcoef), so it is
// exactly the arithmetic of the direct kernel reassociated.
//
// Two terms are not bilinear and get their own channels:
//   * the second-order potential (raft/helpers.py:254-291): its node factors
//     cosh(nk (z + h)) e^{-i (k1 - k2) s} split into exp(+-k1 ..) exp(-+k2 ..) for k2 >= k1,
//     leaving the pair scalar aux2 (w1 - w2) (alpha+ P+ + alpha- P-) with two GEMM channels;
//   * Kim & Yue (raft_member.py:1090-1205): per radius row, Im(sum omega_n) and
//     Im(sum n (n+1) omega_n) are K = 24 real GEMMs (12 Hankel orders) and the row's
//     Bernoulli integrals Im/Ip are applied per (pair, row) in the epilogue.
// Precondition (checked by the caller, rh_qtf_design.order): w2 and k2 strictly increasing,
// so the upper triangle is i2 >= i1 and nk = k2 - k1.
namespace rh {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------
// basis of the w2 side (written per (row, frequency) by the table kernels)
// ---------------------------------------------------------------------------------------
// airy_u's arithmetic (raft/helpers.py:105-154, zeta0 = 1): u = (cos b c0, sin b c0, c1), eta
__device__ __forceinline__ void airy_basis(double w, double k, double beta, double h, double x, double y, double z,
                                           cd& c0, cd& c1, cd& eta) {
  const double th = k * (cos(beta) * x + sin(beta) * y);
  const cd e = mk(cos(th), -sin(th));
  if (!(z <= 0)) {
    c0 = c1 = eta = mk(0, 0);
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
  c0 = scl(scl(e, w), c_sh);
  c1 = scl(iw(w, e), s_sh);
  eta = scl(e, c_ch);
}

__device__ __forceinline__ rh_c128* rcol(const rh_qtf_design& q, const QtfWork& wk, int col, int f) {
  return wk.R + (size_t)col * qtf_n2p(q) + f;
}

// node basis: c0, c1 (u), g0, g1 (grad u), w g0, w g1, p0, p1 (grad p); and the two
// second-order-potential channels of the node (a+-, b+- of the header)
__device__ void qtf_node_basis(const rh_qtf_design& q, const QtfWork& wk, int f, int n) {
  const int n2p = qtf_n2p(q), kq = qtf_kq(q);
  cd b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = mk(0, 0);
  cd Lpc[2][6][2], Rpc[2][2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    Rpc[c][0] = Rpc[c][1] = mk(0, 0);
#pragma unroll
    for (int d = 0; d < 6; ++d) Lpc[c][d][0] = Lpc[c][d][1] = mk(0, 0);
  }
  if (f < q.n2) {
    const double w = q.w2[f], k = q.k2[f], h = q.depth, beta = q.beta;
    const double x = qn(q, RH_QN_RX, n), y = qn(q, RH_QN_RY, n), z = qn(q, RH_QN_RZ, n);
    cd eta;
    airy_basis(w, k, beta, h, x, y, z, b[0], b[1], eta);
    const double cb = cos(beta * kDeg2Rad), sb = sin(beta * kDeg2Rad);
    if (z <= 0 && k > 0) {
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
      b[2] = scl(scl(mk(ph.i, -ph.r), w), k * kxy);     // -i w ph k kxy: G = g0 (cb^2, cb sb, ., cb sb, sb^2, ., ., cb sb, -1)
      b[3] = scl(scl(ph, w), k * kz);                  //  w ph k kz:    G = g1 (., ., cb, ., ., sb, cb, ., .)
      b[4] = scl(b[2], w);
      b[5] = scl(b[3], w);
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
      const cd a0 = scl(ph2, rg * pxy);
      b[6] = mk(a0.i * k, -a0.r * k);                 // a0 (-i k): grad p = (cb p0, sb p0, p1)
      b[7] = scl(scl(ph2, rg * pz), k);
    }
    // second-order potential channels: E ph = a(w1) b(w2) with
    //   a+ = e^{-k z} e^{-i k s}, b+ = e^{k z} e^{i k s}, a- = e^{k z} e^{-i k s}, b- = e^{-k z} e^{i k s}
    // (s = cb x + sb y), and the node's 6-DOF operators (translateForce3to6DOF of MP v + ai sq q):
    //   A1+- = T (MP e_xy -+ i MP e_z), Aq = ai T q;   L = a (k1 A1 - i rho Aq), -a A1;  R = b, k2 b
    {
      const double s = cb * x + sb * y, ekz = exp(k * z), emkz = exp(-k * z);
      double sn, cs;
      sincos(k * s, &sn, &cs);
      const cd em = mk(cs, -sn), ep = mk(cs, sn);
      const cd a[2] = {scl(em, emkz), scl(em, ekz)}, bb[2] = {scl(ep, ekz), scl(ep, emkz)};
      const double rho = q.rho, rv = rho * qn(q, RH_QN_VI, n), rve = rho * qn(q, RH_QN_VE, n) * qn(q, RH_QN_CAE, n);
      const double ai = qn(q, RH_QN_AI, n);
      double MP[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) MP[i] = rv * qn(q, RH_QN_CM + i, n) + rve * qn(q, RH_QN_QM + i, n);
      double mxy[3], mz[3], qv[3] = {qn(q, RH_QN_QX, n), qn(q, RH_QN_QY, n), qn(q, RH_QN_QZ, n)};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        mxy[i] = cb * MP[3 * i] + sb * MP[3 * i + 1];
        mz[i] = MP[3 * i + 2];
      }
      auto T6 = [&](const double* v, double* o) {   // [v; r x v]
        o[0] = v[0];
        o[1] = v[1];
        o[2] = v[2];
        o[3] = y * v[2] - z * v[1];
        o[4] = z * v[0] - x * v[2];
        o[5] = x * v[1] - y * v[0];
      };
      double Txy[6], Tz[6], Tq[6];
      T6(mxy, Txy);
      T6(mz, Tz);
      T6(qv, Tq);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const double sg = c == 0 ? -1.0 : 1.0;      // A1 = Txy + sg i Tz
        Rpc[c][0] = bb[c];
        Rpc[c][1] = scl(bb[c], k);
#pragma unroll
        for (int d = 0; d < 6; ++d) {
          Lpc[c][d][0] = mul(a[c], mk(k * Txy[d], sg * k * Tz[d] - rho * ai * Tq[d]));
          Lpc[c][d][1] = mul(a[c], mk(-Txy[d], -sg * Tz[d]));
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) st(rcol(q, wk, qcol_node(n, j), f), cconj(b[j]));
#pragma unroll
  for (int c = 0; c < 2; ++c) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      st(wk.Rp + ((size_t)c * kq + 2 * n + r) * n2p + f, Rpc[c][r]);
#pragma unroll
      for (int d = 0; d < 6; ++d) st(wk.Lp + (((size_t)c * 6 + d) * kq + 2 * n + r) * n2p + f, Lpc[c][d][r]);
    }
  }
}

// waterline member basis: eta, h0 = w c0, h1 = i w c1 at r_int (ud = (i cos b h0, i sin b h0, h1))
__device__ void qtf_wl_basis(const rh_qtf_design& q, const QtfWork& wk, int f, int m) {
  cd b[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
  if (f < q.n2 && qm(q, RH_QM_WL, m) != 0.0) {
    const double w = q.w2[f], k = q.k2[f];
    cd c0, c1;
    airy_basis(w, k, q.beta, q.depth, qm(q, RH_QM_RIX, m), qm(q, RH_QM_RIY, m), qm(q, RH_QM_RIZ, m), c0, c1, b[0]);
    b[1] = scl(c0, w);
    b[2] = iw(w, c1);
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) st(rcol(q, wk, qcol_wl(q, m, j), f), cconj(b[j]));
}

// Kim & Yue row: A = sum_n omega_n and B = sum_n n (n+1) omega_n with
// omega_n = R1[n+1] conj(R2[n]) - R1[n] conj(R2[n+1]) (R = 1 / D, raft_member.py:1102-1109) are
// sum_b LA_b(w1) conj(R2_b), LA_b = R1[b+1] - R1[b-1], LB_b = b(b+1) R1[b+1] - (b-1) b R1[b-1];
// only their imaginary parts are needed: Im(x conj y) over (re, im) pairs as one K = 24 real dot
__device__ void qtf_kay_basis(const rh_qtf_design& q, const QtfWork& wk, int f, int ir) {
  const int n2p = qtf_n2p(q);
  double* KA = wk.KA + (size_t)ir * kKayK * n2p + f;
  double* KB = wk.KB + (size_t)ir * kKayK * n2p + f;
  double* KR = wk.KR + (size_t)ir * kKayK * n2p + f;
  if (f >= q.n2) {
#pragma unroll 4
    for (int b = 0; b < kKayK; ++b) KA[(size_t)b * n2p] = KB[(size_t)b * n2p] = KR[(size_t)b * n2p] = 0.0;
    return;
  }
  const rh_c128* Rv = wk.hinv + ((size_t)ir * q.n2 + f) * 12;   // written by qtf_kay_at in this thread
  cd R[12];
#pragma unroll
  for (int b = 0; b < 12; ++b) R[b] = ld(Rv + b);
#pragma unroll
  for (int b = 0; b < 12; ++b) {
    cd la = mk(0, 0), lb = mk(0, 0);
    if (b <= 10) {
      la = R[b + 1];
      lb = scl(R[b + 1], (double)(b * (b + 1)));
    }
    if (b >= 1) {
      la = sub(la, R[b - 1]);
      lb = sub(lb, scl(R[b - 1], (double)((b - 1) * b)));
    }
    KA[(size_t)b * n2p] = la.r;
    KA[(size_t)(12 + b) * n2p] = la.i;
    KB[(size_t)b * n2p] = lb.r;
    KB[(size_t)(12 + b) * n2p] = lb.i;
    KR[(size_t)b * n2p] = -R[b].i;        // conj(R2)
    KR[(size_t)(12 + b) * n2p] = R[b].r;
  }
}

// motions X, w X, w^2 X (shared by every node and member) for frequency column f < n2p
// (X == nullptr: f >= n2, zero padding)
__device__ void qtf_glob_basis(const rh_qtf_design& q, const QtfWork& wk, int f, const cd* X) {
  const double w = X ? q.w2[f] : 0.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const cd x = X ? X[j] : mk(0, 0);
    st(rcol(q, wk, qcol_glob(q, j), f), cconj(x));
    st(rcol(q, wk, qcol_glob(q, 6 + j), f), cconj(scl(x, w)));
    st(rcol(q, wk, qcol_glob(q, 12 + j), f), cconj(scl(x, w * w)));
  }
}

// zero K-tail row p (0 .. qtf_npad - 1) of every GEMM operand plane, column f < n2p
__host__ __device__ inline int qtf_npad(const rh_qtf_design& q) { return (qtf_kp(q) - qtf_kb(q)) + (qtf_kq(q) - 2 * q.nq); }
__device__ void qtf_pad_row(const rh_qtf_design& q, const QtfWork& wk, int f, int p) {
  const int n2p = qtf_n2p(q), kb = qtf_kb(q), kp = qtf_kp(q), kq = qtf_kq(q);
  if (p < kp - kb) {
    const int k = kb + p;
    st(wk.R + (size_t)k * n2p + f, mk(0, 0));
    for (int d = 0; d < 6; ++d) st(wk.L + ((size_t)d * kp + k) * n2p + f, mk(0, 0));
    return;
  }
  const int k = 2 * q.nq + p - (kp - kb);
  for (int c = 0; c < 2; ++c) {
    st(wk.Rp + ((size_t)c * kq + k) * n2p + f, mk(0, 0));
    for (int d = 0; d < 6; ++d) st(wk.Lp + (((size_t)c * 6 + d) * kq + k) * n2p + f, mk(0, 0));
  }
}

// ---------------------------------------------------------------------------------------
// w1-side coefficients: the node / waterline / Pinkster functions of the direct kernel
// (k_qtf_pairs), written in terms of Z = conj(w2-side quantities) and probed per basis vector
// ---------------------------------------------------------------------------------------
struct NodeW1 {      // w1 side of a node (tables of k_qtf_tables at i1)
  cd u[3], vp[3], dr[3], G[9], gp[3], dz, va, om[3];
  double w;
};
struct NodeZ {       // conj of the w2-side node quantities
  cd u[3], vp[3], dr[3], G[9], wG[9], gp[3], dz, va, om[3];   // wG = w2 conj(G2)
};

__device__ __forceinline__ void load_w1(const rh_qtf_design& q, const QtfWork& wk, int n, int f, NodeW1& a) {
  const int n2 = q.n2;
  const rh_c128* T = wk.node + (size_t)n * QT_COUNT * n2 + f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    a.u[i] = ld(T + (size_t)(QT_U + i) * n2);
    a.vp[i] = ld(T + (size_t)(QT_VP + i) * n2);
    a.dr[i] = ld(T + (size_t)(QT_DR + i) * n2);
    a.gp[i] = ld(T + (size_t)(QT_GP + i) * n2);
    a.om[i] = ld(wk.freq + (size_t)(FT_OM + i) * n2 + f);
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) a.G[i] = ld(T + (size_t)(QT_GU + i) * n2);
  a.dz = ld(T + (size_t)QT_DWDZ * n2);
  a.va = ld(T + (size_t)QT_VA * n2);
  a.w = q.w2[f];
}

__device__ __forceinline__ void skew(const cd* o, cd* O) {   // -getH(o): O x = o x x
  O[0] = mk(0, 0);
  O[1] = scl(o[2], -1);
  O[2] = o[1];
  O[3] = o[2];
  O[4] = mk(0, 0);
  O[5] = scl(o[0], -1);
  O[6] = scl(o[1], -1);
  O[7] = o[0];
  O[8] = mk(0, 0);
}

enum : int { ZU = 1, ZVP = 2, ZDR = 4, ZG = 8, ZWG = 16, ZGP = 32, ZDZ = 64, ZVA = 128, ZOM = 256 };

// The node term of k_qtf_pairs (raft_fowt.py:1521-1600) for Z restricted to the groups in GM
// (the others are zero and their terms are not formed).  Adds translateForce3to6DOF(f) to Q.
template <int GM>
__device__ __forceinline__ void node_force_z(const rh_qtf_design& q, int n, const NodeW1& a, const NodeZ& z, cd* Q) {
  constexpr bool HU = GM & ZU, HVP = GM & ZVP, HDR = GM & ZDR, HG = GM & ZG, HWG = GM & ZWG, HGP = GM & ZGP,
                 HDZ = GM & ZDZ, HVA = GM & ZVA, HOM = GM & ZOM;
  const double rho = q.rho;
  const double rx = qn(q, RH_QN_RX, n), ry = qn(q, RH_QN_RY, n), rz = qn(q, RH_QN_RZ, n);
  const double qv[3] = {qn(q, RH_QN_QX, n), qn(q, RH_QN_QY, n), qn(q, RH_QN_QZ, n)};
  const double rv = rho * qn(q, RH_QN_VI, n);
  const double rve = rho * qn(q, RH_QN_VE, n) * qn(q, RH_QN_CAE, n);
  const double ai = qn(q, RH_QN_AI, n);
  cd ur1[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) ur1[i] = sub(a.u[i], a.vp[i]);
  cd vM[3] = {mk(0, 0), mk(0, 0), mk(0, 0)}, vA[3] = {mk(0, 0), mk(0, 0), mk(0, 0)},
     ax[3] = {mk(0, 0), mk(0, 0), mk(0, 0)}, sq = mk(0, 0);
  // (2) convective + (4) body motion: 0.25 [G1 (conj u2 + i w1 conj dr2) + conj(G2) (u1 - i w2 dr1)]
  if constexpr (HU || HDR) {
    cd x[3], c[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      x[i] = mk(0, 0);
      if constexpr (HU) x[i] = add(x[i], z.u[i]);
      if constexpr (HDR) x[i] = add(x[i], iw(a.w, z.dr[i]));
    }
    cmv(a.G, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) vM[i] = add(vM[i], scl(c[i], 0.25));
  }
  if constexpr (HG) {
    cd c[3];
    cmv(z.G, a.u, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) vM[i] = add(vM[i], scl(c[i], 0.25));
  }
  if constexpr (HWG) {
    cd x[3], c[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = iw(-1.0, a.dr[i]);
    cmv(z.wG, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) vM[i] = add(vM[i], scl(c[i], 0.25));
  }
  constexpr bool HUR = HU || HVP;   // terms in conj(ur2) = conj(u2) - conj(vp2)
  cd ur2[3];
  if constexpr (HUR) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      ur2[i] = mk(0, 0);
      if constexpr (HU) ur2[i] = add(ur2[i], z.u[i]);
      if constexpr (HVP) ur2[i] = sub(ur2[i], z.vp[i]);
    }
    // pressure: Bernoulli drop (:1593-1594)
    double M9[9];
    cd t5[3], cu2[3];
    ldm9(q, RH_QN_P12, n, M9);
    rmv(M9, ur1, t5);
    ldm9(q, RH_QN_CA, n, M9);
    rmv(M9, ur2, cu2);
    cd pd = mk(0, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i) pd = add(pd, mul(t5[i], cu2[i]));
    sq = add(sq, scl(pd, -0.25 * rho));
  }
  if constexpr (HDR) {   // grad p1 . conj(dr2) (:1590-1592)
    cd pn = mk(0, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i) pn = add(pn, mul(a.gp[i], z.dr[i]));
    sq = add(sq, scl(pn, 0.25));
  }
  if constexpr (HGP) {
    cd pm = mk(0, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i) pm = add(pm, mul(z.gp[i], a.dr[i]));
    sq = add(sq, scl(pm, 0.25));
  }
  // (3) Rainey axial divergence (raft/helpers.py:228-251), projected perpendicular to q
  if constexpr (HUR || HDZ) {
    cd v3[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
    if constexpr (HUR) {
      cd s2 = mk(0, 0);
      if constexpr (HU) s2 = add(add(scl(z.u[0], qv[0]), scl(z.u[1], qv[1])), scl(z.u[2], qv[2]));
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        cd up2 = mk(0, 0);
        if constexpr (HU) up2 = sub(z.u[i], scl(s2, qv[i]));
        if constexpr (HVP) up2 = sub(up2, z.vp[i]);
        v3[i] = add(v3[i], mul(a.dz, up2));
      }
    }
    if constexpr (HDZ) {
      const cd s1 = add(add(scl(a.u[0], qv[0]), scl(a.u[1], qv[1])), scl(a.u[2], qv[2]));
#pragma unroll
      for (int i = 0; i < 3; ++i) v3[i] = add(v3[i], mul(z.dz, sub(sub(a.u[i], scl(s1, qv[i])), a.vp[i])));
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) v3[i] = scl(v3[i], 0.25);
    const cd aq = add(add(scl(v3[0], qv[0]), scl(v3[1], qv[1])), scl(v3[2], qv[2]));
#pragma unroll
    for (int i = 0; i < 3; ++i) vA[i] = add(vA[i], sub(v3[i], scl(aq, qv[i])));
  }
  // (5) Rainey body rotation (:1556-1575)
  double CA[9], QM[9];
  ldm9(q, RH_QN_CA, n, CA);
  ldm9(q, RH_QN_QM, n, QM);
  cd O1[9];
  skew(a.om, O1);
  if constexpr (HVA) {   // -0.5 O1 conj(va2) q
    cd x[3], c[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = scl(z.va, qv[i]);
    cmv(O1, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) vA[i] = sub(vA[i], scl(c[i], 0.5));
  }
  cd O2c[9];
  if constexpr (HOM) {
    skew(z.om, O2c);
    cd x[3], c[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = scl(a.va, qv[i]);
    cmv(O2c, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) vA[i] = sub(vA[i], scl(c[i], 0.5));
  }
  if constexpr (HUR) {   // V1 = G1 + O1 against CaM conj(ur2) and (I - qMat) conj(ur2)
    cd V1[9], x[3], c[3], t[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) V1[i] = add(a.G[i], O1[i]);
    rmv(CA, ur2, x);
    cmv(V1, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) ax[i] = add(ax[i], scl(c[i], 0.25));
    rmv(QM, ur2, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = sub(ur2[i], t[i]);
    cmv(V1, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) vA[i] = sub(vA[i], scl(c[i], 0.25));
  }
  if constexpr (HG || HOM) {   // conj(V2) = conj(G2) + conj(O2) against CaM ur1 and (I - qMat) ur1
    cd V2[9], x[3], c[3], t[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      V2[i] = mk(0, 0);
      if constexpr (HG) V2[i] = add(V2[i], z.G[i]);
      if constexpr (HOM) V2[i] = add(V2[i], O2c[i]);
    }
    rmv(CA, ur1, x);
    cmv(V2, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) ax[i] = add(ax[i], scl(c[i], 0.25));
    rmv(QM, ur1, t);
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = sub(ur1[i], t[i]);
    cmv(V2, x, c);
#pragma unroll
    for (int i = 0; i < 3; ++i) vA[i] = sub(vA[i], scl(c[i], 0.25));
  }
  // fr = (I - qMat) ax + CaM vA ;  f = (rv CM + rve QM) vM + rv fr + ai sq q
  cd fr[3], t4[3], tA[3];
  rmv(QM, ax, t4);
  rmv(CA, vA, tA);
#pragma unroll
  for (int i = 0; i < 3; ++i) fr[i] = add(sub(ax[i], t4[i]), tA[i]);
  double CM[9], MP[9];
  ldm9(q, RH_QN_CM, n, CM);
#pragma unroll
  for (int i = 0; i < 9; ++i) MP[i] = rv * CM[i] + rve * QM[i];
  cd tM[3], f[3];
  rmv(MP, vM, tM);
  const cd sa = scl(sq, ai);
#pragma unroll
  for (int i = 0; i < 3; ++i) f[i] = add(add(tM[i], scl(fr[i], rv)), scl(sa, qv[i]));
  acc6(Q, f, rx, ry, rz);
}

struct WlSide {   // waterline member quantities: w1 side, or conj of the w2 side
  cd e, ud[3], a[3], ge[3];
};
__device__ __forceinline__ void load_wl(const rh_qtf_design& q, const QtfWork& wk, int m, int f, WlSide& s) {
  const int n2 = q.n2;
  const rh_c128* W = wk.wl + (size_t)m * WT_COUNT * n2 + f;
  s.e = ld(W + (size_t)WT_ETAR * n2);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    s.ud[i] = ld(W + (size_t)(WT_UD + i) * n2);
    s.a[i] = ld(W + (size_t)(WT_A + i) * n2);
    s.ge[i] = ld(W + (size_t)(WT_GE + i) * n2);
  }
}
// waterline relative-elevation force (:1602-1630) of member m
__device__ __forceinline__ void wl_force_z(const rh_qtf_design& q, int m, const WlSide& a, const WlSide& z, cd* Q) {
  if (qm(q, RH_QM_WL, m) == 0.0) return;
  double CM[9], CA[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    CM[i] = qm(q, RH_QM_CM + i, m);
    CA[i] = qm(q, RH_QM_CA + i, m);
  }
  const double ra = q.rho * qm(q, RH_QM_AWL, m);
  cd fe[3], ae[3], t3[3], t4[3], fo[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    fe[i] = scl(add(mul(a.ud[i], z.e), mul(z.ud[i], a.e)), 0.25);
    ae[i] = scl(add(mul(a.a[i], z.e), mul(z.a[i], a.e)), 0.25);
  }
  rmv(CM, fe, t3);
  rmv(CA, ae, t4);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const cd gt = add(mul(a.ge[i], z.e), mul(z.ge[i], a.e));
    fo[i] = sub(sub(scl(t3[i], ra), scl(t4[i], ra)), scl(gt, 0.25 * ra));
  }
  acc6(Q, fo, qm(q, RH_QM_RIX, m), qm(q, RH_QM_RIY, m), qm(q, RH_QM_RIZ, m));
}

// body-motion operator at a point: dr = X[:3] + th x r  (getKinematics, raft/helpers.py:95-97)
__device__ __forceinline__ void dlin_unit(int j, double x, double y, double z, double* o) {
  o[0] = o[1] = o[2] = 0.0;
  switch (j) {
    case 0: o[0] = 1; break;
    case 1: o[1] = 1; break;
    case 2: o[2] = 1; break;
    case 3: o[1] = -z; o[2] = y; break;
    case 4: o[0] = z; o[2] = -x; break;
    case 5: o[0] = -y; o[1] = x; break;   // not `default`: see node_probe_glob_k
    default: break;
  }
}

// global probe g (0..17) of node n: X_j -> conj(dr2); w X_j -> conj(v2) = -i conj(w dr2)
// (its projection vp and the axial part va) and conj(om2) = -i conj(w X[3:]); w^2 X: none.
// One kind of probe per instantiation: K = 0 (g < 6: X_j), 1 (6 <= g < 9: w X_j translation),
// 2 (9 <= g < 12: w X_j rotation): the same arithmetic, one node_force_z instantiation per kind
template <int K>
__device__ __forceinline__ void node_probe_glob_k(const rh_qtf_design& q, int n, int g, const NodeW1& a, cd* Q) {
  NodeZ z;
  const double x = qn(q, RH_QN_RX, n), y = qn(q, RH_QN_RY, n), zz = qn(q, RH_QN_RZ, n);
  double D[3];
  if constexpr (K == 0) {
    dlin_unit(g, x, y, zz, D);
#pragma unroll
    for (int i = 0; i < 3; ++i) z.dr[i] = mk(D[i], 0);
    node_force_z<ZDR>(q, n, a, z, Q);
  } else {
    const int j = g - 6;
    dlin_unit(j, x, y, zz, D);
    const double qv[3] = {qn(q, RH_QN_QX, n), qn(q, RH_QN_QY, n), qn(q, RH_QN_QZ, n)};
    cd v[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) v[i] = mk(0, -D[i]);
    const cd vq = add(add(scl(v[0], qv[0]), scl(v[1], qv[1])), scl(v[2], qv[2]));
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      z.vp[i] = sub(v[i], scl(vq, qv[i]));
      z.om[i] = mk(0, 0);
    }
    z.va = scl(vq, -1.0);
    if constexpr (K == 2) {
      // Written out per component.  dlin_unit's yaw row must stay an explicit `case 5`: as the
      // switch's `default` it came out of the compiler with a wrong yaw column here (g = 11;
      // g = 9, 10 right; the loop form of these three lines alone was fine), DESIGN.md §5,
      // tools/ubench/qtf_lcol_diag.py, profiles/r06_v6/yaw_variants.txt
      z.om[0] = mk(0, j == 3 ? -1.0 : 0.0);
      z.om[1] = mk(0, j == 4 ? -1.0 : 0.0);
      z.om[2] = mk(0, j == 5 ? -1.0 : 0.0);
      node_force_z<ZVP | ZVA | ZOM>(q, n, a, z, Q);
    } else {
      node_force_z<ZVP | ZVA>(q, n, a, z, Q);
    }
  }
}

// own probe j (0..7) of node n (basis order of qtf_node_basis)
__device__ __forceinline__ void node_probe_own(const rh_qtf_design& q, int n, int j, const NodeW1& a, cd* Q) {
  NodeZ z;
  const double cbr = cos(q.beta), sbr = sin(q.beta);
  const double cb = cos(q.beta * kDeg2Rad), sb = sin(q.beta * kDeg2Rad);
  const double qv[3] = {qn(q, RH_QN_QX, n), qn(q, RH_QN_QY, n), qn(q, RH_QN_QZ, n)};
  if (j < 2) {
    z.u[0] = mk(j == 0 ? cbr : 0.0, 0);
    z.u[1] = mk(j == 0 ? sbr : 0.0, 0);
    z.u[2] = mk(j == 0 ? 0.0 : 1.0, 0);
    z.va = add(add(scl(z.u[0], qv[0]), scl(z.u[1], qv[1])), scl(z.u[2], qv[2]));
    node_force_z<ZU | ZVA>(q, n, a, z, Q);
    return;
  }
  if (j < 6) {
    cd G[9];
    if ((j & 1) == 0) {   // g0 / w g0
      const double v[9] = {cb * cb, cb * sb, 0, cb * sb, sb * sb, 0, 0, cb * sb, -1};
#pragma unroll
      for (int i = 0; i < 9; ++i) G[i] = mk(v[i], 0);
    } else {              // g1 / w g1
      const double v[9] = {0, 0, cb, 0, 0, sb, cb, 0, 0};
#pragma unroll
      for (int i = 0; i < 9; ++i) G[i] = mk(v[i], 0);
    }
    if (j < 4) {
#pragma unroll
      for (int i = 0; i < 9; ++i) z.G[i] = G[i];
      cd Gq[3];
      const cd qc[3] = {mk(qv[0], 0), mk(qv[1], 0), mk(qv[2], 0)};
      cmv(G, qc, Gq);
      z.dz = add(add(scl(Gq[0], qv[0]), scl(Gq[1], qv[1])), scl(Gq[2], qv[2]));
      node_force_z<ZG | ZDZ>(q, n, a, z, Q);
    } else {
#pragma unroll
      for (int i = 0; i < 9; ++i) z.wG[i] = G[i];
      node_force_z<ZWG>(q, n, a, z, Q);
    }
    return;
  }
  z.gp[0] = mk(j == 6 ? cb : 0.0, 0);
  z.gp[1] = mk(j == 6 ? sb : 0.0, 0);
  z.gp[2] = mk(j == 6 ? 0.0 : 1.0, 0);
  node_force_z<ZGP>(q, n, a, z, Q);
}

// waterline probes: own j (eta, h0, h1) or global g (X_j: eta_r and g_e, w^2 X_j: acceleration)
__device__ __forceinline__ void wl_probe(const rh_qtf_design& q, int m, bool own, int j, const WlSide& a, cd* Q) {
  WlSide z;
  z.e = mk(0, 0);
#pragma unroll
  for (int i = 0; i < 3; ++i) z.ud[i] = z.a[i] = z.ge[i] = mk(0, 0);
  const double cbr = cos(q.beta), sbr = sin(q.beta);
  if (own) {
    if (j == 0) z.e = mk(1, 0);
    else if (j == 1) {
      z.ud[0] = mk(0, -cbr);
      z.ud[1] = mk(0, -sbr);
    } else z.ud[2] = mk(1, 0);
  } else {
    const double x = qm(q, RH_QM_RIX, m), y = qm(q, RH_QM_RIY, m), zz = qm(q, RH_QM_RIZ, m);
    double D[3];
    if (j < 6) {
      dlin_unit(j, x, y, zz, D);
      z.e = mk(-D[2], 0);                               // eta_r = eta - dr_z
      const double p1[3] = {qm(q, RH_QM_P1X, m), qm(q, RH_QM_P1Y, m), qm(q, RH_QM_P1Z, m)};
      const double p2[3] = {qm(q, RH_QM_P2X, m), qm(q, RH_QM_P2Y, m), qm(q, RH_QM_P2Z, m)};
      const double e3 = j == 3 ? 1.0 : 0.0, e4 = j == 4 ? 1.0 : 0.0;
      const double c1 = e3 * p1[1] - e4 * p1[0], c2 = e3 * p2[1] - e4 * p2[0];
#pragma unroll
      for (int i = 0; i < 3; ++i) z.ge[i] = mk(-q.g * (c1 * p1[i] + c2 * p2[i]), 0);
    } else if (j >= 12) {
      dlin_unit(j - 12, x, y, zz, D);
#pragma unroll
      for (int i = 0; i < 3; ++i) z.a[i] = mk(-D[i], 0);   // conj(a2) = -conj(w^2 dr2)
    } else {
      return;
    }
  }
  wl_force_z(q, m, a, z, Q);
}

// Pinkster IV (:1449-1456): 0.25 [th1 x conj(F2) + conj(th2) x F1], F1 = M (-w^2 X)
__device__ __forceinline__ void pinkster_probe(const rh_qtf_design& q, const QtfWork& wk, const double* M66, int g, int f, cd* Q) {
  const int n2 = q.n2;
  cd th2c[3] = {mk(0, 0), mk(0, 0), mk(0, 0)}, F2c[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) F2c[i] = mk(0, 0);
  if (g >= 3 && g < 6) {
    th2c[0] = mk(g == 3 ? 1.0 : 0.0, 0);
    th2c[1] = mk(g == 4 ? 1.0 : 0.0, 0);
    th2c[2] = mk(g == 5 ? 1.0 : 0.0, 0);
  } else if (g >= 12) {
    const int j = g - 12;
    F2c[0] = mk(j == 0 ? -M66[0] : 0.0, 0);
    F2c[1] = mk(j == 1 ? -M66[0] : 0.0, 0);
    F2c[2] = mk(j == 2 ? -M66[0] : 0.0, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i) F2c[3 + i] = mk(j >= 3 ? -M66[6 * (3 + i) + j] : 0.0, 0);
  } else {
    return;
  }
  cd th1[3], F1a[6], tmp1[3], tmp2[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) th1[i] = ld(wk.freq + (size_t)(FT_XI + 3 + i) * n2 + f);
#pragma unroll
  for (int i = 0; i < 6; ++i) F1a[i] = ld(wk.freq + (size_t)(FT_F1 + i) * n2 + f);
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    cross_cc(th1, F2c + 3 * part, tmp1);
    cross_cc(th2c, F1a + 3 * part, tmp2);
#pragma unroll
    for (int i = 0; i < 3; ++i) Q[3 * part + i] = add(Q[3 * part + i], scl(add(tmp1[i], tmp2[i]), 0.25));
  }
}

// L columns.  grid (ceil(n2p / 64), 18 + nq + nmq), 512 threads; lane = frequency f (= i1).
//   y < 18      : global motion column g = y: waves split nodes (w, w+8, ...) and members,
//                 wave 0 adds Pinkster; the 8 partial sums meet in LDS in wave order
//   y < 18 + nq : the 8 own columns of node y - 18 (wave j = probe j)
//   else        : the 3 own columns of waterline member y - 18 - nq (waves 0..2)
__device__ __forceinline__ void lcoef_block(const rh_qtf_design& q, const QtfWork& wk, const double* __restrict__ M66,
                                            int fb, int y, double (*red)[12][64]) {
  const int lane = (int)threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int f = fb * 64 + lane;
  const int n2 = q.n2, n2p = qtf_n2p(q), kp = qtf_kp(q);
  const bool live = f < n2;
  const int fs = live ? f : 0;            // pad lanes evaluate a valid column and store zeros
  cd Q[6];
#pragma unroll
  for (int d = 0; d < 6; ++d) Q[d] = mk(0, 0);
  auto store = [&](int col) {
    if (f < n2p)
#pragma unroll
      for (int d = 0; d < 6; ++d) st(wk.L + ((size_t)d * kp + col) * n2p + f, live ? Q[d] : mk(0, 0));
  };
  if (y < 18) {
    const int g = y;
    // one probe kind per node loop (the branch on g is uniform and hoisted): a loop body that
    // held every kind of node_probe_glob would need the registers of the largest one throughout
    auto node_loop = [&](auto kind) {
#pragma unroll 1
      for (int n = wv; n < q.nq; n += 8) {
        NodeW1 a;
        load_w1(q, wk, n, fs, a);
        node_probe_glob_k<decltype(kind)::value>(q, n, g, a, Q);
      }
    };
    if (g < 6) node_loop(std::integral_constant<int, 0>{});
    else if (g < 9) node_loop(std::integral_constant<int, 1>{});
    else if (g < 12) node_loop(std::integral_constant<int, 2>{});
#pragma unroll 1
    for (int m = wv; m < q.nmq; m += 8) {
      WlSide a;
      load_wl(q, wk, m, fs, a);
      wl_probe(q, m, false, g, a, Q);
    }
    if (wv == 0) pinkster_probe(q, wk, M66, g, fs, Q);
#pragma unroll
    for (int d = 0; d < 6; ++d) {
      red[wv][2 * d][lane] = Q[d].r;
      red[wv][2 * d + 1][lane] = Q[d].i;
    }
    __syncthreads();
    if (wv < 6) {
      const int d = wv;
      cd s = mk(0, 0);
#pragma unroll
      for (int v = 0; v < 8; ++v) s = add(s, mk(red[v][2 * d][lane], red[v][2 * d + 1][lane]));
      if (f < n2p) st(wk.L + ((size_t)d * kp + qcol_glob(q, g)) * n2p + f, live ? s : mk(0, 0));
    }
    return;
  }
  if (y < 18 + q.nq) {
    const int n = y - 18;
    NodeW1 a;
    load_w1(q, wk, n, fs, a);
    node_probe_own(q, n, wv, a, Q);
    store(qcol_node(n, wv));
    return;
  }
  const int m = y - 18 - q.nq;
  if (wv < 3) {
    WlSide a;
    load_wl(q, wk, m, fs, a);
    wl_probe(q, m, true, wv, a, Q);
    store(qcol_wl(q, m, wv));
  }
}

// ---------------------------------------------------------------------------------------
// pair tiles: 16 (i1) x 16 (i2), upper-triangle tiles in row-major order, dealt round robin
// over the ranks (tile t of the order goes to rank t mod nrank)
// ---------------------------------------------------------------------------------------
// Complex GEMM steps of one 16 x 16 tile: A[m = i1][k] (lane l holds A[l & 15][4 s + (l >> 4)]),
// B[k][n = i2] (B[4 s + (l >> 4)][l & 15]).  Three real MFMAs per step (Gauss):
// P1 = Ar Br, P2 = Ai Bi, P3 = (Ar + Ai)(Br + Bi); Re = P1 - P2, Im = P3 - P1 - P2.  nsteps is a
// multiple of 4: the loads of the next four steps are in flight while the MFMAs of the current
// four run.
#ifndef RH_QTF_PF
#define RH_QTF_PF 4   // k-steps per operand batch (tools/ubench variant: 8)
#endif
#ifndef RH_QTF_CHAIN
#define RH_QTF_CHAIN 1   // 1: the bilinear and potential-channel k-steps as one operand stream (cgemm_steps2)
#endif
#ifndef RH_QTF_SPLIT
#define RH_QTF_SPLIT 0   // 1: even / odd k-steps in two accumulator sets (tools/ubench variant)
#endif
__device__ __forceinline__ void cgemm_steps(const rh_c128* __restrict__ A, const rh_c128* __restrict__ B, size_t step,
                                            int nsteps, d4& p1, d4& p2, d4& p3) {
  constexpr int PF = RH_QTF_PF;
#if RH_QTF_SPLIT
  d4 q1 = {0, 0, 0, 0}, q2 = q1, q3 = q1;
#endif
  cd a[PF], b[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) {
    const int sj = (PF > 4 && j >= nsteps) ? nsteps - 1 : j;
    a[j] = ld(A + sj * step);
    b[j] = ld(B + sj * step);
  }
#pragma unroll 1
  for (int s = 0; s < nsteps; s += PF) {
    cd an[PF], bn[PF];
    const bool more = s + PF < nsteps;
    if (more) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        // nsteps is a multiple of 4: a deeper batch (variant) stops at the last step
        const int sj = (PF > 4 && s + PF + j >= nsteps) ? nsteps - 1 : s + PF + j;
        an[j] = ld(A + sj * step);
        bn[j] = ld(B + sj * step);
      }
    }
#pragma unroll
    for (int j = 0; j < PF; j += 2) {
      if (PF > 4 && s + j >= nsteps) break;   // uniform (variant only)
      p1 = mfma64(a[j].r, b[j].r, p1);
      p2 = mfma64(a[j].i, b[j].i, p2);
      p3 = mfma64(a[j].r + a[j].i, b[j].r + b[j].i, p3);
#if RH_QTF_SPLIT   // two accumulator sets (six independent MFMA chains): the round-2/3 order
      q1 = mfma64(a[j + 1].r, b[j + 1].r, q1);
      q2 = mfma64(a[j + 1].i, b[j + 1].i, q2);
      q3 = mfma64(a[j + 1].r + a[j + 1].i, b[j + 1].r + b[j + 1].i, q3);
#else              // one chain per product, the k-step order of k_qtf_gemm32: sharded == whole, bit for bit
      p1 = mfma64(a[j + 1].r, b[j + 1].r, p1);
      p2 = mfma64(a[j + 1].i, b[j + 1].i, p2);
      p3 = mfma64(a[j + 1].r + a[j + 1].i, b[j + 1].r + b[j + 1].i, p3);
#endif
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        a[j] = an[j];
        b[j] = bn[j];
      }
    }
  }
#if RH_QTF_SPLIT
  p1 += q1;
  p2 += q2;
  p3 += q3;
#endif
}

// The bilinear steps (A1, B1: n1 steps, into p) and the potential channel's (A2, B2: n2 steps,
// into c) as one operand stream: the channel's first batch is loaded while the last bilinear
// batch runs, instead of after it.  Each accumulator sees its k-steps in the same order as with
// two cgemm_steps calls (the same bits).  n1 and n2 are multiples of 4.
__device__ __forceinline__ void cgemm_steps2(const rh_c128* __restrict__ A1, const rh_c128* __restrict__ B1, int n1,
                                             const rh_c128* __restrict__ A2, const rh_c128* __restrict__ B2, int n2,
                                             size_t step, d4& p1, d4& p2, d4& p3, d4& c1, d4& c2, d4& c3) {
  constexpr int PF = 4;
  const int nt = n1 + n2;
  auto src = [&](int s, const rh_c128*& a, const rh_c128*& b) {   // operands of k-step s (uniform)
    if (s < n1) {
      a = A1 + s * step;
      b = B1 + s * step;
    } else {
      a = A2 + (s - n1) * step;
      b = B2 + (s - n1) * step;
    }
  };
  cd a[PF], b[PF];
  {
    const rh_c128 *pa, *pb;
    src(0, pa, pb);
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      a[j] = ld(pa + j * step);
      b[j] = ld(pb + j * step);
    }
  }
#pragma unroll 1
  for (int s = 0; s < nt; s += PF) {
    cd an[PF], bn[PF];
    const bool more = s + PF < nt;
    if (more) {
      const rh_c128 *pa, *pb;
      src(s + PF, pa, pb);
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        an[j] = ld(pa + j * step);
        bn[j] = ld(pb + j * step);
      }
    }
    if (s < n1) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        p1 = mfma64(a[j].r, b[j].r, p1);
        p2 = mfma64(a[j].i, b[j].i, p2);
        p3 = mfma64(a[j].r + a[j].i, b[j].r + b[j].i, p3);
      }
    } else {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        c1 = mfma64(a[j].r, b[j].r, c1);
        c2 = mfma64(a[j].i, b[j].i, c2);
        c3 = mfma64(a[j].r + a[j].i, b[j].r + b[j].i, c3);
      }
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        a[j] = an[j];
        b[j] = bn[j];
      }
    }
  }
}

// cgemm_steps2 with a ring of operand registers instead of a double buffer: k-step s + j is
// consumed from slot j, which is then refilled with k-step s + PF + j, so PF steps stay in flight
// with half the operand registers (the kernel fits 128 VGPRs: four waves per SIMD).  Same MFMA
// order per accumulator, the same bits.
__device__ __forceinline__ void cgemm_ring2(const rh_c128* __restrict__ A1, const rh_c128* __restrict__ B1, int n1,
                                            const rh_c128* __restrict__ A2, const rh_c128* __restrict__ B2, int n2,
                                            size_t step, d4& p1, d4& p2, d4& p3, d4& c1, d4& c2, d4& c3) {
  constexpr int PF = 4;
  cd a[PF], b[PF];
  auto mf = [&](const cd& x, const cd& y, d4& q1, d4& q2, d4& q3) {
    q1 = mfma64(x.r, y.r, q1);
    q2 = mfma64(x.i, y.i, q2);
    q3 = mfma64(x.r + x.i, y.r + y.i, q3);
  };
  {
    const rh_c128* pa = n1 > 0 ? A1 : A2;   // (uniform)
    const rh_c128* pb = n1 > 0 ? B1 : B2;
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      a[j] = ld(pa + j * step);
      b[j] = ld(pb + j * step);
    }
  }
  if (n1 > 0) {
    // bilinear k-steps; each slot is refilled with the step PF ahead, from the channel's first
    // steps during the last batch
#pragma unroll 1
    for (int s = 0; s < n1 - PF; s += PF) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        mf(a[j], b[j], p1, p2, p3);
        a[j] = ld(A1 + (s + PF + j) * step);
        b[j] = ld(B1 + (s + PF + j) * step);
      }
    }
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      mf(a[j], b[j], p1, p2, p3);
      a[j] = ld(A2 + j * step);
      b[j] = ld(B2 + j * step);
    }
  }
#pragma unroll 1
  for (int s = 0; s < n2; s += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      mf(a[j], b[j], c1, c2, c3);
      const int r = min(s + PF + j, n2 - 1);   // (the last batch reloads the last step: not used)
      a[j] = ld(A2 + r * step);
      b[j] = ld(B2 + r * step);
    }
  }
}

// The pair scalars of the second-order potential (raft/helpers.py:254-291) of pair (w1, w2):
// aux2 (w1 - w2) alpha+ and aux2 (w1 - w2) alpha-, with
// cosh(nk (z+h)) / cosh(nk h) = alpha+ e^{nk z} + alpha- e^{-nk z}.  t1, t2 = tanh(k1 h),
// tanh(k2 h) (per frequency, formed once per tile); tanh(nk h) = -m / (2 + m) with
// m = expm1(-2 nk h), accurate for small nk h.  Shared by both GEMM kernels, with contraction
// off, so that they produce the same bits.
__device__ __forceinline__ void qtf_pot_scalars(double w1, double k1, double t1, double w2, double k2, double t2,
                                                double cb, double sb, double h, double g, cd& sp, cd& sm) {
#pragma clang fp contract(off)
  sp = cd{0.0, 0.0};
  sm = cd{0.0, 0.0};
  if ((w1 != w2) && (k1 > 0) && (k2 > 0)) {
    const double kx = k1 * cb - k2 * cb, ky = k1 * sb - k2 * sb;
    const double nk = sqrt(kx * kx + ky * ky);
    const double em = expm1(-2.0 * nk * h), tnh = -em / (2.0 + em);
    const double den12 = (w1 - w2) * (w1 - w2) / g - nk * tnh;
    const double den21 = (w2 - w1) * (w2 - w1) / g - nk * tnh;
    const double n12 = (k1 * k1) * (1 - t1 * t1) - 2 * k1 * k2 * (1 + t1 * t2);
    const double n21 = (k2 * k2) * (1 - t2 * t2) - 2 * k2 * k1 * (1 + t2 * t1);
    const double f12 = n12 / den12, f21 = n21 / den21;
    // g12 = i (-g / (2 w1)) f12, g21 = i (-g / (2 w2)) f21: purely imaginary
    const double g12i = (-g / (2 * w1)) * f12, g21i = (-g / (2 * w2)) * f21;
    // a2w = 0.5 (g21 + conj(g12)) (w1 - w2)
    const double a2wi = ((g21i - g12i) * 0.5) * (w1 - w2);
    const double e2 = exp(-2.0 * nk * h), ap = 1.0 / (1.0 + e2), am = e2 * ap;
    sp = cd{0.0 * ap, a2wi * ap};
    sm = cd{0.0 * am, a2wi * am};
  }
}

// The final sum of a pair entry, shared by k_qtf_gemm and k_qtf_gemm32 and written out with
// contraction off, so that both kernels (the row-sharded and the whole QTF) produce the same
// bits: (bilinear part + second half) + (alpha+ P+ + alpha- P-) + Kim & Yue.
__device__ __forceinline__ cd qtf_pair_sum(double mre, double mim, double hre, double him, double ppr, double ppi,
                                           double pmr, double pmi, double spr, double spi, double smr, double smi,
                                           double ksr, double ksi) {
#pragma clang fp contract(off)
  const double pr = (spr * ppr - spi * ppi) + (smr * pmr - smi * pmi);
  const double pi = (spr * ppi + spi * ppr) + (smr * pmi + smi * pmr);
  return cd{((mre + hre) + pr) + ksr, ((mim + him) + pi) + ksi};
}

// row-major index of upper-triangle tile (T1, T2), T2 >= T1, of an nt x nt tile grid
__device__ __forceinline__ int qtf_tile_id(int T1, int T2, int nt) { return T1 * nt - T1 * (T1 - 1) / 2 + (T2 - T1); }
// tile (T1, T2) of the t-th upper-triangle tile in row-major order (block-uniform)
__device__ __forceinline__ void qtf_tile_of(int t, int nt, int& T1, int& T2) {
  T1 = 0;
  while (t >= nt - T1) {
    t -= nt - T1;
    ++T1;
  }
  T2 = T1 + t;
}


// Q_d over the bilinear terms and the two potential channels for one tile and three DOFs.
// Workgroup = 2 kGD waves: wave w takes DOF kGD dg + (w % kGD) (dg = the block's DOF group) and
// half w / kGD of the work: the first half of K and channel +, or the second half and channel -
// (the kGD waves of a half share the R tile through L1); the second half's partial sums reach
// the first through LDS.  Blocks are (tile, DOF group) pairs, remapped so that an XCD works on a
// contiguous run of tiles (their L rows stay in its L2).  kGD = 2: 4-wave workgroups at <= 128
// VGPRs, so the C3 grid (325 tiles x 3) is resident at once (four per CU); with kGD = 3 the
// 6-wave workgroups fit two per CU at three waves per SIMD, and 650 of them took two rounds.
#ifndef RH_QTF_GDOF
#define RH_QTF_GDOF 2   // DOFs per k_qtf_gemm workgroup: 2 (4 waves, 3 workgroups per tile) or 3 (6 waves, 2)
#endif
#ifndef RH_QTF_RING
#define RH_QTF_RING 1   // 1: operand ring (cgemm_ring2), 0: double buffer (cgemm_steps2)
#endif
constexpr int kGD = RH_QTF_GDOF;
constexpr int kGThreads = 128 * kGD;
static_assert(6 % kGD == 0, "the DOFs split evenly over a tile's workgroups");
static_assert(kGThreads >= 256, "the pair scalars: one pair per thread of the 16 x 16 tile");
#ifndef RH_QTF_GWPE
#define RH_QTF_GWPE 4   // k_qtf_gemm waves per SIMD asked of the register allocator (<= 128 VGPRs)
#endif
__global__ __launch_bounds__(kGThreads) __attribute__((amdgpu_waves_per_eu(RH_QTF_GWPE))) void k_qtf_gemm(rh_qtf_design q, QtfWork wk, rh_c128* __restrict__ qtf, int t0,
                                                        int mirror) {
  __shared__ double part[kGD][16][64];
  __shared__ double pscal[4][256];   // per pair: aux2 (w1 - w2) alpha+, ... alpha- (complex)
  __shared__ double tkh[32];         // tanh(k h) of the tile's rows (i1) and columns (i2)
  const int lane = (int)threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int half = w / kGD, dl = w % kGD;
  const int n2 = q.n2, n2p = qtf_n2p(q), nt = n2p / 16, kp = qtf_kp(q), kq = qtf_kq(q);
  const int slot = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  constexpr int kGB = 6 / kGD;   // workgroups per tile
  const int d = kGD * (slot % kGB) + dl;
  int T1 = 0, t = t0 + slot / kGB;   // this call's tiles: t0, t0 + 1, ... (row-major)
  while (t >= nt - T1) {   // block-uniform
    t -= nt - T1;
    ++T1;
  }
  const int T2 = T1 + t;
  const int mr = lane & 15, kr = lane >> 4;
  const int i1b = 16 * T1, i2b = 16 * T2;
  const double h = q.depth, g = q.g;
  // The pair scalars of the second-order potential (raft/helpers.py:254-291), once per pair,
  // before the GEMM (their transcendentals overlap the other waves' operand loads):
  // tanh(k h) of the tile's 16 rows and 16 columns first, then one pair per thread.
  {
    const int x = (int)threadIdx.x;
    if (x < 32) {
      const int i = min(x < 16 ? i1b + x : i2b + x - 16, n2 - 1);
      tkh[x] = tanh(q.k2[i] * h);
    }
    __syncthreads();
    if (x < 256) {
      const double bt = q.beta * kDeg2Rad, cb = cos(bt), sb = sin(bt);
      const int i1 = min(i1b + (x >> 4), n2 - 1), i2 = min(i2b + (x & 15), n2 - 1);
      cd sp, sm;
#if RH_ABL_G_NOPOT   // timing ablation (wrong results)
      sp = cd{q.w2[i1], tkh[x >> 4]}; sm = cd{q.w2[i2], tkh[16 + (x & 15)]};
#else
      qtf_pot_scalars(q.w2[i1], q.k2[i1], tkh[x >> 4], q.w2[i2], q.k2[i2], tkh[16 + (x & 15)], cb, sb, h, g, sp, sm);
#endif
      pscal[0][x] = sp.r;
      pscal[1][x] = sp.i;
      pscal[2][x] = sm.r;
      pscal[3][x] = sm.i;
    }
  }
  const size_t step = (size_t)4 * n2p;
  const int ns = kp / 4, ns0 = 4 * ((ns / 4 + 1) / 2);
  const int k0 = half == 0 ? 0 : ns0, nk = half == 0 ? ns0 : ns - ns0;
  d4 p1 = {0, 0, 0, 0}, p2 = p1, p3 = p1;
  d4 c1 = {0, 0, 0, 0}, c2 = c1, c3 = c1;   // potential channel c = half
#if RH_QTF_CHAIN && RH_QTF_RING && !RH_ABL_G_NOBIL && !RH_ABL_G_NOPCH
  cgemm_ring2(wk.L + ((size_t)d * kp + 4 * k0 + kr) * n2p + i1b + mr, wk.R + ((size_t)4 * k0 + kr) * n2p + i2b + mr, nk,
              wk.Lp + (((size_t)half * 6 + d) * kq + kr) * n2p + i1b + mr,
              wk.Rp + ((size_t)half * kq + kr) * n2p + i2b + mr, kq / 4, step, p1, p2, p3, c1, c2, c3);
#elif RH_QTF_CHAIN && !RH_ABL_G_NOBIL && !RH_ABL_G_NOPCH
  cgemm_steps2(wk.L + ((size_t)d * kp + 4 * k0 + kr) * n2p + i1b + mr, wk.R + ((size_t)4 * k0 + kr) * n2p + i2b + mr, nk,
               wk.Lp + (((size_t)half * 6 + d) * kq + kr) * n2p + i1b + mr,
               wk.Rp + ((size_t)half * kq + kr) * n2p + i2b + mr, kq / 4, step, p1, p2, p3, c1, c2, c3);
#else
#if !RH_ABL_G_NOBIL   // timing ablation: no bilinear GEMM (wrong results)
  if (nk > 0)
    cgemm_steps(wk.L + ((size_t)d * kp + 4 * k0 + kr) * n2p + i1b + mr, wk.R + ((size_t)4 * k0 + kr) * n2p + i2b + mr,
                step, nk, p1, p2, p3);
#endif
#if !RH_ABL_G_NOPCH   // timing ablation: no potential-channel GEMM (wrong results)
  cgemm_steps(wk.Lp + (((size_t)half * 6 + d) * kq + kr) * n2p + i1b + mr,
              wk.Rp + ((size_t)half * kq + kr) * n2p + i2b + mr, step, kq / 4, c1, c2, c3);
#endif
#endif
  const d4 mre = p1 - p2, mim = p3 - p1 - p2, cre = c1 - c2, cim = c3 - c1 - c2;
  if (half == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      part[dl][r][lane] = mre[r];
      part[dl][4 + r][lane] = mim[r];
      part[dl][8 + r][lane] = cre[r];
      part[dl][12 + r][lane] = cim[r];
    }
  }
  __syncthreads();
  if (half == 1) return;
  // + the tile's Kim & Yue sums (k_qtf_kay, the previous launch), then the upper-triangle entry and,
  // for a whole QTF, its Hermitian mirror (raft/raft_fowt.py:1639-1640: qtf + conj(qtf).T -
  // diag(conj(diag(qtf))))
  const double* ks = wk.KS + (size_t)qtf_tile_id(T1, T2, nt) * 12 * 256;
  const int i2 = i2b + mr;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i1 = i1b + kr + 4 * r;
    if (i1 >= n2 || i2 >= n2 || i2 < i1) continue;
    const int e = (kr + 4 * r) * 16 + mr;
    const int ek = kr * 16 + mr + 64 * r;   // kay_tile's element of this pair
    const cd Qf = qtf_pair_sum(mre[r], mim[r], part[dl][r][lane], part[dl][4 + r][lane], cre[r], cim[r],
                               part[dl][8 + r][lane], part[dl][12 + r][lane], pscal[0][e], pscal[1][e], pscal[2][e],
                               pscal[3][e], ks[(2 * d) * 256 + ek], ks[(2 * d + 1) * 256 + ek]);
    rh_c128* up = qtf + ((size_t)i1 * n2 + i2) * 6 + d;
#if RH_ABL_G_NOSTORE   // timing ablation: no stores (wrong results)
    if (Qf.r == 1.2345e300) st(up, Qf);
    continue;
#endif
#if RH_ABL_G_NOMIRROR  // timing ablation: upper triangle only (wrong results)
    st(up, Qf);
    continue;
#endif
    if (!mirror) {
      st(up, Qf);
    } else if (i1 == i2) {
      st(up, sub(add(Qf, cconj(Qf)), cconj(Qf)));
    } else {
      st(up, Qf);
      st(qtf + ((size_t)i2 * n2 + i1) * 6 + d, cconj(Qf));
    }
  }
}

// Kim & Yue correction (raft/raft_member.py:1090-1205) per 16 x 16 pair tile, plus the final
// sum with the bilinear part (k_qtf_gemm wrote it into the upper triangle) and the Hermitian
// fill (raft/raft_fowt.py:1639-1640).  A radius row's force is Re(i kap (...)) times a real
// direction, so only Im(sum omega_n) and Im(sum n (n+1) omega_n) are formed, as K = 24 real
// MFMA dots over the Hankel orders (qtf_kay_basis).  The rows of a member share its waterline
// phase and pforce: a wave takes whole members (the j-th Kim & Yue member goes to wave j % 4),
// keeps per element sum sre and sum sre p over the member's rows, and adds
// phase x [s0 pf; s x pf] (the rows' translateForce3to6DOF) to the tile's LDS sum in member
// order.  The next row's operands are loaded while the current row is reduced.

#ifndef RH_KAY_SPLIT
#define RH_KAY_SPLIT 1   // waves per member of the variants' k_qtf_kay (k_qtf_lk picks per call)
#endif
constexpr int kKayM = 4;                   // Kim & Yue members per round
// A member's rows are summed in kKayP contiguous parts, and the parts' sums added in part order,
// whether one wave takes all the parts one after the other (S = 1) or each part has a wave of
// its own (S = kKayP): the same bits either way, so the launch can pick S per call (a rank's few
// tiles of a sharded QTF: S = kKayP, more waves per tile; a whole QTF: S = 1, two tiles per block)
constexpr int kKayP = 2;
static_assert(kKayP == 2, "kay_tile: the part sums are added as P0 + P1");
template <int S>
constexpr int kay_threads() { return 64 * kKayM * S; }
constexpr int kKayS = RH_KAY_SPLIT;
constexpr int kKayThreads = kay_threads<kKayS>();
// One pair tile's Kim & Yue sums by a group of kKayW waves (tid 0 .. kKayThreads - 1 of the
// group) into acc[12][256]; live = false: the group has no tile and only joins the block's
// barriers (every group of a block runs the same member rounds).  Every __syncthreads here is
// a whole-block barrier: the caller's block is made of such groups only.  A member's rows are
// split into kKayS contiguous parts, one per wave; the parts' row sums meet in part order
// (psg, LDS) before the member's phase is applied.
template <int S>
__device__ __forceinline__ void kay_tile(const rh_qtf_design& q, const QtfWork& wk, int T1, int T2, bool live, int tid,
                                         double (*acc)[256], double* psg) {
  static_assert(S == 1 || S == kKayP, "kay_tile: one wave per member or one per part");
  constexpr int kThreads = kay_threads<S>();
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int slot = wv / S, part = wv % S;
  const int n2 = q.n2, n2p = qtf_n2p(q), nt = n2p / 16, nkr = q.nkr;
  const int mr = lane & 15, kr = lane >> 4;
  const int i1b = 16 * T1, i2b = 16 * T2;
  for (int e = tid; e < 12 * 256; e += kThreads) (&acc[0][0])[e] = 0.0;
  const double rho = q.rho, g = q.g, h = q.depth;
  const double cbr = cos(q.beta), sbr = sin(q.beta);
  const int i2s = min(i2b + mr, n2 - 1);
  const double k2 = q.k2[i2s], w2 = q.w2[i2s];
  const int e0 = kr * 16 + mr;      // element of register r: e0 + 64 r
  __syncthreads();
  int m = 0, j = 0;                 // scan state: member m is the j-th Kim & Yue member
  for (int round = 0;; ++round) {
    // this wave's member of the round: the (round * kKayM + slot)-th member with rows
    int mine = -1;
    while (m < q.nmq) {
      const bool has = ldsi(q.kstart + m + 1) > ldsi(q.kstart + m) && ldsi(q.kstart + m) < nkr;
      if (has) {
        if (j == round * kKayM + slot) mine = m;
        ++j;
      }
      ++m;
      if (j == (round + 1) * kKayM) break;
    }
    const bool any_left = j > round * kKayM;   // block-uniform: this round has at least one member
    if (!any_left) break;
    if (!live) mine = -1;                      // no tile: the rounds' barriers only
    double sg[4][4];   // [s0, sx, sy, sz][element] of this wave's part of its member
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) sg[c][r] = 0.0;
    if (mine >= 0) {
      const int r0 = ldsi(q.kstart + mine), r1m = min(ldsi(q.kstart + mine + 1), nkr);
      double va[6], vb[6], vr[6];
      auto load_row = [&](int ir, double* A, double* B, double* Rr) {
        const size_t o1 = ((size_t)ir * kKayK + kr) * n2p + i1b + mr, o2 = ((size_t)ir * kKayK + kr) * n2p + i2b + mr;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
          A[s] = wk.KA[o1 + (size_t)4 * s * n2p];
          B[s] = wk.KB[o1 + (size_t)4 * s * n2p];
          Rr[s] = wk.KR[o2 + (size_t)4 * s * n2p];
        }
      };
      // Per (row, element) factors: every table value an element's epilogue needs is loaded at
      // the start of its row, in one batch, before the row's MFMAs; the row's tail (the element
      // formulas) then runs without a memory wait, and the wave-uniform waterline / interval
      // choices are selects, not branches.  (The epilogue used to load each element's factors
      // where it used them, behind a branch: every element drained the whole vector-memory queue,
      // the next row's prefetched operands included.)
      double k1v[4], w1v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i1 = min(i1b + kr + 4 * r, n2 - 1);
        k1v[r] = q.k2[i1];
        w1v[r] = q.w2[i1];
      }
      // S = 1: all the member's rows in order, part 0's sums parked in this lane's psg slot when
      // part 1 begins (r1m > r0: a member in the scan has rows, so that happens once)
      const int rmid = r0 + (r1m - r0) / kKayP;
      const int ra = S == 1 ? r0 : r0 + (r1m - r0) * part / kKayP;
      const int r1 = S == 1 ? r1m : r0 + (r1m - r0) * (part + 1) / kKayP;
#pragma unroll 1
      for (int ir = ra; ir < r1; ++ir) {
        if (S == 1 && ir == rmid) {   // wave-uniform
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              psg[(slot * 16 + 4 * c + r) * 64 + lane] = sg[c][r];
              sg[c][r] = 0.0;
            }
        }
        load_row(ir, va, vb, vr);
        double t1[4][6], t2[6];
        {
          const double2* T2 = reinterpret_cast<const double2*>(wk.kayt + ((size_t)ir * n2 + i2s) * kKayT + 2);
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const double2 v = T2[c];
            t2[2 * c] = v.x;
            t2[2 * c + 1] = v.y;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i1 = min(i1b + kr + 4 * r, n2 - 1);
            const double2* T1 = reinterpret_cast<const double2*>(wk.kayt + ((size_t)ir * n2 + i1) * kKayT + 2);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const double2 v = T1[c];
              t1[r][2 * c] = v.x;
              t1[r][2 * c + 1] = v.y;
            }
          }
        }
        const double R = ldsd(q.kray + RH_KR_R * nkr + ir);
        const bool wl = ir == r0;
        const double px = wl ? qm(q, RH_QM_WLX, mine) : ldsd(q.kray + RH_KR_MX * nkr + ir);
        const double py = wl ? qm(q, RH_QM_WLY, mine) : ldsd(q.kray + RH_KR_MY * nkr + ir);
        const double pz = wl ? qm(q, RH_QM_WLZ, mine) : ldsd(q.kray + RH_KR_MZ * nkr + ir);
        const double z1 = ldsd(q.kray + RH_KR_Z1 * nkr + ir), z2 = ldsd(q.kray + RH_KR_Z2 * nkr + ir);
        d4 ca = {0, 0, 0, 0}, cbk = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 6; ++s) {
          ca = mfma64(va[s], vr[s], ca);
          cbk = mfma64(vb[s], vr[s], cbk);
        }
        const double p1 = t2[0], m1 = t2[1], p2 = t2[2], m2 = t2[3], c2 = t2[4], r2 = t2[5];
        const double cR = rho * g * R * 2 / M_PI;
        const double H = h / R, k2h = k2 * R * H;
        const double zz1 = (z1 + h) / h, zz2 = (z2 + h) / h;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double kap = cR * t1[r][5] * r2;   // rho g R 2/pi / (k1R k2R)
          // waterline term (:1133-1149): Re(-i kap A) = kap Im(A)
          const double s_wl = kap * ca[r];
          // node-interval Bernoulli term (:1155-1200)
          const double k1h = k1v[r] * R * H;
          const double P1 = t1[r][0], M1 = t1[r][1], P2 = t1[r][2], M2 = t1[r][3];
          const double ia = 0.5 / (k1h + k2h);
          const double a2 = (P2 * p2 - M2 * m2) * ia, a1 = (P1 * p1 - M1 * m1) * ia;
          const bool same = w1v[r] == w2;      // the diagonal pair: the (k1 - k2) terms are their limits
          const double id = 0.5 / (k1h - k2h);
          const double d2 = same ? zz2 : (P2 * m2 - M2 * p2) * id, d1 = same ? zz1 : (P1 * m1 - M1 * p1) * id;
          const double Im = 0.5 * (a2 - d2 - a1 + d1);
          const double Ip = 0.5 * (a2 + d2 - a1 - d1);
          const double s_in = -kap * (t1[r][4] * c2) * (Im * ca[r] + Ip * t1[r][5] * r2 * cbk[r]);   // Re(i kap cc (Im A + Ip/(k1R k2R) B))
          const double sre = wl ? s_wl : s_in;
          sg[0][r] += sre;
          sg[1][r] += sre * px;
          sg[2][r] += sre * py;
          sg[3][r] += sre * pz;
        }
      }
      if (S == 1) {   // P0 + P1: part 0's sums (parked) plus part 1's
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) sg[c][r] = psg[(slot * 16 + 4 * c + r) * 64 + lane] + sg[c][r];
      }
    }
    if (S > 1) {   // part 1's row sums to part 0's wave: P0 + P1
      if (part > 0 && mine >= 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) psg[(slot * 16 + 4 * c + r) * 64 + lane] = sg[c][r];
      }
      __syncthreads();
      if (part == 0 && mine >= 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) sg[c][r] += psg[(slot * 16 + 4 * c + r) * 64 + lane];
      }
    }
    // this round's members reach the tile sum in member order (deterministic): at its turn a
    // wave adds phase x [s0 pf; s x pf], the phase of its member's waterline point with
    // conj(F) when k1 < k2
#pragma unroll 1
    for (int v = 0; v < kKayM; ++v) {
      if (slot == v && part == 0 && mine >= 0) {
        const double wx = qm(q, RH_QM_WLX, mine), wy = qm(q, RH_QM_WLY, mine), wz = qm(q, RH_QM_WLZ, mine);
        const double pf0 = qm(q, RH_QM_PFX, mine), pf1 = qm(q, RH_QM_PFY, mine), pf2 = qm(q, RH_QM_PFZ, mine);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double k1 = q.k2[min(i1b + kr + 4 * r, n2 - 1)];
          const double kkx = k1 * cbr - k2 * cbr, kky = k1 * sbr - k2 * sbr;
          double sp, cp;
          sincos(kkx * wx + kky * wy + 0 * wz, &sp, &cp);
          const cd ph = (k1 < k2) ? mk(cp, sp) : mk(cp, -sp);
          const double s0 = sg[0][r], sx = sg[1][r], sy = sg[2][r], sz = sg[3][r];
          const double T[6] = {s0 * pf0, s0 * pf1, s0 * pf2, pf2 * sy - pf1 * sz, pf0 * sz - pf2 * sx, pf1 * sx - pf0 * sy};
          const int e = e0 + 64 * r;
#pragma unroll
          for (int d = 0; d < 6; ++d) {
            acc[2 * d][e] += ph.r * T[d];
            acc[2 * d + 1][e] += ph.i * T[d];
          }
        }
      }
      __syncthreads();
    }
  }
  // the tile's Kim & Yue sums to the workspace; the GEMM epilogue adds them to the pair sums
  if (live) {
    double* ks = wk.KS + (size_t)qtf_tile_id(T1, T2, nt) * 12 * 256;
    for (int e = tid; e < 12 * 256; e += kThreads) ks[e] = (&acc[0][0])[e];
  }
}


#ifndef RH_KAY_WPE
#define RH_KAY_WPE 2
#endif
// k_qtf_lcoef and k_qtf_kay in ONE launch (both read only the tables of k_qtf_tables): the
// first nkb workgroups take the Kim & Yue pair tiles (S = 1: two tiles per workgroup, one wave
// per member; S = kKayP: one tile, one wave per part of a member's rows), the rest are
// k_qtf_lcoef's (x, y) blocks, so the coefficient blocks fill the CUs the Kim & Yue tiles leave
// idle instead of running before them.  Per tile and per block the arithmetic is that of the
// two kernels, and either S gives the same bits.
template <int S>
constexpr int lk_tiles() { return 512 / kay_threads<S>(); }   // Kim & Yue tiles per k_qtf_lk block
constexpr int kLkThreads = 512;
constexpr int kPsg = kKayM * (kKayP - 1) * 16 * 64;          // one group's parked / handed part sums

static_assert(kLkThreads == 512, "k_qtf_lk: lcoef_block is a 512-thread block");
template <int S>
__global__ __launch_bounds__(kLkThreads) __attribute__((amdgpu_waves_per_eu(RH_KAY_WPE))) void k_qtf_lk(
    rh_qtf_design q, QtfWork wk, const double* __restrict__ M66, int t0, int ntile, int nkb, int bx0, int nbx) {
  constexpr int kTiles = lk_tiles<S>(), kThreads = kay_threads<S>();
  constexpr int kAcc = 12 * 256, kRed = 8 * 12 * 64;
  constexpr int kSm = 2 * kAcc > kRed ? 2 * kAcc : kRed;
  __shared__ double sm[kSm];                 // kTiles Kim & Yue tile sums, or lcoef_block's wave sums
  __shared__ double psg[kTiles * kPsg];
  const int tid = (int)threadIdx.x;
  if ((int)blockIdx.x < nkb) {               // block-uniform
    const int grp = __builtin_amdgcn_readfirstlane(tid / kThreads);   // wave-uniform: the tile indices stay scalar
    const int t = kTiles * xcd_remap((int)blockIdx.x, nkb) + grp;   // this group's tile of the rank's order
    const bool live = t < ntile;
    int T1 = 0, T2 = 0;
    if (live) qtf_tile_of(t0 + t, qtf_n2p(q) / 16, T1, T2);
    kay_tile<S>(q, wk, T1, T2, live, tid - grp * kThreads, reinterpret_cast<double(*)[256]>(sm + grp * kAcc),
                psg + grp * kPsg);
  } else {
    // (k_qtf_lcoef's block order; frequency-block-major runs per XCD cut the launch's HBM reads
    // from 52 to 31 MB but cost 3.5 us per QTF); the w1 blocks bx0 .. bx0 + nbx - 1
    // hold this call's w1 rows
    const int bl = (int)blockIdx.x - nkb;
    lcoef_block(q, wk, M66, bx0 + bl % nbx, bl / nbx, reinterpret_cast<double(*)[12][64]>(sm));
  }
}

}  // namespace rh
