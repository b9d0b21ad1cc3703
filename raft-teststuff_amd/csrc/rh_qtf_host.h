// rh_qtf_host.h -- host-only: the static slender-body QTF tables of one FOWT (rh_qtf_tables).
//
// The per-(design, grid, heading) geometry bookkeeping of FOWT.calcQTF_slenderBody
// (raft/raft_fowt.py:1461-1502, 1532-1587, 1604-1625) and Member.correction_KAY
// (raft/raft_member.py:1111-1200) that the device kernels read (include/rafthip.h
// rh_qtf_node_field / rh_qtf_member_field / rh_kay_field).  raft/qtf.py build_tables is the
// Python statement of the same tables and the parity reference of this code
// (tests/test_qtf_tables.py); a QTF of a new design then costs one call here instead of some
// hundred small NumPy operations per member.
//
// Member record (raft/qtf.py member_record writes it), float64:
//   circ, MCF, ns, nst, rA[3], rB[3], p1[3], p2[3], q[3], p1Mat[9], p2Mat[9], qMat[9],
//   r[ns][3], ls[ns], dls[ns], ds[ns][nd], drs[ns][nd], a_i[ns], stations[nst],
//   Ca_p1[nst], Ca_p2[nst], Ca_End[nst]        (nd = 1 circular, 2 rectangular)
#pragma once
#include <cmath>
#include <stdexcept>
#include <vector>

#pragma clang fp contract(off)   // NumPy rounds every product and sum separately

namespace rhq {

constexpr int kQN = 46, kQM = 36, kKR = 6;
constexpr double kPi = 3.141592653589793;

struct MemberRec {
  int circ, mcf, ns, nst, nd;
  const double *rA, *rB, *p1, *p2, *q, *p1M, *p2M, *qM, *r, *ls, *dls, *ds, *drs, *ai, *st, *cap1, *cap2, *caend;
};

// Parses one record; returns the number of doubles it spans, or -1 when it is malformed.
inline long long parse(const double* s, long long avail, MemberRec& m) {
  if (avail < 4) return -1;
  m.circ = (int)s[0];
  m.mcf = (int)s[1];
  m.ns = (int)s[2];
  m.nst = (int)s[3];
  if (m.ns < 1 || m.nst < 1 || s[2] != (double)m.ns || s[3] != (double)m.nst) return -1;
  m.nd = m.circ ? 1 : 2;
  const long long need = 4 + 15 + 27 + 3LL * m.ns + 2LL * m.ns + 2LL * m.nd * m.ns + m.ns + 4LL * m.nst;
  if (avail < need) return -1;
  const double* p = s + 4;
  auto take = [&](long long n) { const double* a = p; p += n; return a; };
  m.rA = take(3); m.rB = take(3); m.p1 = take(3); m.p2 = take(3); m.q = take(3);
  m.p1M = take(9); m.p2M = take(9); m.qM = take(9);
  m.r = take(3LL * m.ns); m.ls = take(m.ns); m.dls = take(m.ns);
  m.ds = take((long long)m.nd * m.ns); m.drs = take((long long)m.nd * m.ns); m.ai = take(m.ns);
  m.st = take(m.nst); m.cap1 = take(m.nst); m.cap2 = take(m.nst); m.caend = take(m.nst);
  return need;
}

// np.interp(x, xp, fp) with the default end values (fp[0] / fp[-1]) -- rhp::np_interp's search
inline double interp(double x, const double* xp, const double* fp, int n) {
  if (x <= xp[0]) return fp[0];
  if (x >= xp[n - 1]) return fp[n - 1];
  int lo = 0, hi = n - 1;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (xp[mid] <= x) lo = mid; else hi = mid;
  }
  if (xp[lo] == x) return fp[lo];
  const double slope = (fp[lo + 1] - fp[lo]) / (xp[lo + 1] - xp[lo]);
  return slope * (x - xp[lo]) + fp[lo];
}

inline bool above(const MemberRec& m) { return m.rA[2] > 0 && m.rB[2] > 0; }   // entirely above water (:1461)
inline bool kay_on(const MemberRec& m) { return m.mcf && (m.rA[2] * m.rB[2] < 0); }

// Table sizes: submerged nodes, members not above water, Kim & Yue radius rows.
inline void count(const std::vector<MemberRec>& mems, long long& nq, long long& nmq, long long& nkr) {
  nq = nmq = nkr = 0;
  for (const MemberRec& m : mems) {
    if (above(m)) continue;
    ++nmq;
    for (int i = 0; i < m.ns; ++i) nq += m.r[3 * i + 2] < 0;
    if (kay_on(m)) {
      ++nkr;
      for (int i = 0; i + 1 < m.ns; ++i) nkr += m.r[3 * i + 2] <= 0;
    }
  }
}

// Column-major output tables of the sizes count() gives: node [kQN][nq], memb [kQM][nmq],
// kray [kKR][nkr], qmstart / kstart [nmq + 1].
struct Tables {
  double *node, *memb, *kray;
  int *qmstart, *kstart;
  long long nq, nmq, nkr;
};

inline void build(const std::vector<MemberRec>& mems, double beta, const Tables& T) {
  long long iq = 0, im = 0, ik = 0;
  T.qmstart[0] = T.kstart[0] = 0;
  auto node = [&](int f) { return T.node + f * T.nq; };
  auto krow = [&](const double* row) {
    for (int k = 0; k < kKR; ++k) T.kray[k * T.nkr + ik] = row[k];
    ++ik;
  };
  for (const MemberRec& m : mems) {
    if (above(m)) continue;
    const double* R = m.r;
    double last_cm[9] = {0}, last_ca[9] = {0};
    int nsub = 0;
    for (int i = 0; i < m.ns; ++i) {
      if (!(R[3 * i + 2] < 0)) continue;
      ++nsub;
      const double ls = m.ls[i], dls = m.dls[i];
      const double ca1 = interp(ls, m.st, m.cap1, m.nst), ca2 = interp(ls, m.st, m.cap2, m.nst);
      const double cae = interp(ls, m.st, m.caend, m.nst);
      double vi, ve;
      if (m.circ) {
        const double d = m.ds[i], dr = m.drs[i];
        vi = 0.25 * kPi * (d * d) * dls;                                   // (:1532-1533)
        ve = kPi / 12.0 * std::fabs(std::pow(d + dr, 3.0) - std::pow(d - dr, 3.0));   // (:1580-1581)
      } else {
        const double d0 = m.ds[2 * i], d1 = m.ds[2 * i + 1], r0 = m.drs[2 * i], r1 = m.drs[2 * i + 1];
        vi = d0 * d1 * dls;
        ve = kPi / 12.0 * (std::pow(((d0 + r0) + (d1 + r1)) / 2.0, 3.0) - std::pow(((d0 - r0) + (d1 - r1)) / 2.0, 3.0));
      }
      const double rz = R[3 * i + 2];
      if (rz + 0.5 * dls > 0) vi = vi * (0.5 * dls - rz) / dls;          // partly submerged strip (Q12)
      const double col[10] = {R[3 * i], R[3 * i + 1], rz, m.q[0], m.q[1], m.q[2], vi, ve, m.ai[i], cae};
      for (int k = 0; k < 10; ++k) node(k)[iq] = col[k];
      for (int k = 0; k < 9; ++k) {
        last_cm[k] = (1. + ca1) * m.p1M[k] + (1. + ca2) * m.p2M[k];
        last_ca[k] = ca1 * m.p1M[k] + ca2 * m.p2M[k];
        node(10 + k)[iq] = last_cm[k];
        node(19 + k)[iq] = last_ca[k];
        node(28 + k)[iq] = m.p1M[k] + m.p2M[k];
        node(37 + k)[iq] = m.qM[k];
      }
      ++iq;
    }
    T.qmstart[im + 1] = T.qmstart[im] + nsub;
    const int n = m.ns;
    const bool wl = R[3 * (n - 1) + 2] * R[2] < 0;
    double rint[3] = {0, 0, 0}, awl = 0.0;
    if (wl) {
      for (int k = 0; k < 3; ++k)
        rint[k] = R[k] + (R[3 * (n - 1) + k] - R[k]) * (0. - R[2]) / (R[3 * (n - 1) + 2] - R[2]);   // (:1492)
      int iwl = -1;
      for (int i = 0; i < n; ++i)
        if (R[3 * i + 2] < 0) iwl = i;
      if (m.circ) {
        const double dwl = iwl != n - 1 ? 0.5 * (m.ds[iwl] + m.ds[iwl + 1]) : m.ds[iwl];
        awl = 0.25 * kPi * (dwl * dwl);
      } else {
        double a, b;
        if (iwl != n - 1) {
          a = 0.5 * (m.ds[2 * iwl] + m.ds[2 * (iwl + 1)]);
          b = 0.5 * (m.ds[2 * iwl + 1] + m.ds[2 * (iwl + 1) + 1]);
        } else {
          a = m.ds[2 * iwl];
          b = m.ds[2 * iwl + 1];
        }
        awl = a * b;
      }
    }
    // Kim & Yue (raft_member.py:1111-1200)
    const bool kay = kay_on(m);
    double pf[3] = {0, 0, 0}, rwl[3] = {0, 0, 0};
    if (kay) {
      const double bv[3] = {std::cos(beta), std::sin(beta), 0.0};
      // np.dot and np.linalg.norm of 3-vectors go to the BLAS ddot, whose kernel sums the
      // products as a chain of fused multiply-adds (measured: bit for bit on 20,000 random pairs)
      auto dot3 = [](const double* x, const double* y) { return std::fma(x[2], y[2], std::fma(x[1], y[1], x[0] * y[0])); };
      const double a1 = dot3(bv, m.p1), a2 = dot3(bv, m.p2);
      for (int k = 0; k < 3; ++k) pf[k] = a1 * m.p1[k] + a2 * m.p2[k];
      const double nrm = std::sqrt(dot3(pf, pf));
      for (int k = 0; k < 3; ++k) pf[k] = pf[k] / nrm;
      for (int k = 0; k < 3; ++k) rwl[k] = m.rA[k] + (m.rB[k] - m.rA[k]) * (0 - m.rA[2]) / (m.rB[2] - m.rA[2]);
      if (m.nd == 1) {          // np.interp(0, mem.r[:, 2], 0.5 * np.array(mem.ds)): a circular member
        std::vector<double> zs(2 * n);
        for (int i = 0; i < n; ++i) {
          zs[i] = R[3 * i + 2];
          zs[n + i] = 0.5 * m.ds[i];
        }
        const double Rw = interp(0.0, zs.data(), zs.data() + n, n);
        const double row[6] = {Rw, 0.0, 0.0, rwl[0], rwl[1], rwl[2]};
        krow(row);
      } else {
        throw std::invalid_argument("rh_qtf_tables: Kim & Yue correction on a rectangular member");
      }
      for (int i = 0; i + 1 < n; ++i) {                                   // intervals whose first node is wet
        if (!(R[3 * i + 2] <= 0)) continue;
        const double z1 = R[3 * i + 2];
        const double z2 = R[3 * (i + 1) + 2] > 0 ? 0.0 : R[3 * (i + 1) + 2];
        const double R1 = m.dls[i] == 0 ? m.ds[i] : m.ds[i] / 2;
        const double R2 = m.dls[i + 1] == 0 ? m.ds[i] : m.ds[i + 1] / 2;   // Q9
        const double row[6] = {0.5 * (R1 + R2), z1, z2, 0.5 * (R[3 * i] + R[3 * (i + 1)]),
                               0.5 * (R[3 * i + 1] + R[3 * (i + 1) + 1]), 0.5 * (R[3 * i + 2] + R[3 * (i + 1) + 2])};
        krow(row);
      }
    }
    T.kstart[im + 1] = (int)ik;
    const double mc[kQM] = {wl ? 1.0 : 0.0, rint[0], rint[1], rint[2], awl,
                            last_cm[0], last_cm[1], last_cm[2], last_cm[3], last_cm[4], last_cm[5], last_cm[6], last_cm[7], last_cm[8],
                            last_ca[0], last_ca[1], last_ca[2], last_ca[3], last_ca[4], last_ca[5], last_ca[6], last_ca[7], last_ca[8],
                            m.p1[0], m.p1[1], m.p1[2], m.p2[0], m.p2[1], m.p2[2],
                            kay ? 1.0 : 0.0, pf[0], pf[1], pf[2], rwl[0], rwl[1], rwl[2]};
    for (int k = 0; k < kQM; ++k) T.memb[k * T.nmq + im] = mc[k];
    ++im;
  }
}

}  // namespace rhq
