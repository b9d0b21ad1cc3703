// rh_device.h -- device-side building blocks for librafthip (gfx950, FP64 VALU).
//
// Complex FP64 arithmetic in the order NumPy uses it, the register-resident partially
// pivoted LU solve that replaces LAPACK zgesv (numpy.linalg.solve, raft/raft_model.py:947)
// and wavefront reductions for 64-lane waves.
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/rafthip.h"

namespace rh {

struct cd {
  double r, i;
};

__device__ __forceinline__ cd mk(double r, double i) { return cd{r, i}; }
__device__ __forceinline__ cd ld(const rh_c128* p) {
  const double2 v = *reinterpret_cast<const double2*>(p);
  return cd{v.x, v.y};
}
__device__ __forceinline__ void st(rh_c128* p, cd v) {
  *reinterpret_cast<double2*>(p) = make_double2(v.r, v.i);
}
// non-temporal (streaming) store: write-once data that must not displace cached tables
__device__ __forceinline__ void st_nt(rh_c128* p, cd v) {
  double* q = reinterpret_cast<double*>(p);
  __builtin_nontemporal_store(v.r, q);
  __builtin_nontemporal_store(v.i, q + 1);
}
__device__ __forceinline__ cd add(cd a, cd b) { return cd{a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cd sub(cd a, cd b) { return cd{a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cd mul(cd a, cd b) { return cd{a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
__device__ __forceinline__ cd scl(cd a, double s) { return cd{a.r * s, a.i * s}; }
// i*w*a  (NumPy: (1j*w)*a = (0,w)*(ar,ai))
__device__ __forceinline__ cd iw(double w, cd a) { return cd{-w * a.i, w * a.r}; }
__device__ __forceinline__ double abs2(cd a) { return a.r * a.r + a.i * a.i; }
__device__ __forceinline__ double cabs(cd a) { return hypot(a.r, a.i); }
__device__ __forceinline__ double cabs1(cd a) { return fabs(a.r) + fabs(a.i); }  // LAPACK dcabs1

// Smith's complex division (as LAPACK zladiv / C99), a / b.
__device__ __forceinline__ cd cdiv(cd a, cd b) {
  if (fabs(b.i) <= fabs(b.r)) {
    const double e = b.i / b.r, f = b.r + b.i * e;
    return cd{(a.r + a.i * e) / f, (a.i - a.r * e) / f};
  }
  const double e = b.r / b.i, f = b.i + b.r * e;
  return cd{(a.r * e + a.i) / f, (a.i * e - a.r) / f};
}

// In-register Gaussian elimination with partial pivoting (max |re|+|im|, first maximum
// wins as in izamax) on an N x N complex system; A and x are overwritten, x = A^-1 x.
// Returns false on an exactly zero pivot (LAPACK: info > 0 -> LinAlgError("Singular matrix")).
template <int N>
__device__ __forceinline__ bool lu_solve(cd (&A)[N][N], cd (&x)[N]) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int p = k;
    double best = cabs1(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const double v = cabs1(A[i][k]);
      if (v > best) { best = v; p = i; }
    }
    ok = ok && (best != 0.0);
    // The row exchange is a chain of per-lane selects; skip it when no lane of the wave
    // pivots off the diagonal at this step (the common case for these impedance matrices).
    // Results are the same either way.
    if (__builtin_amdgcn_ballot_w64(p != k) != 0) {
#pragma unroll
      for (int i = k + 1; i < N; ++i) {
        const bool sw = (p == i);
#pragma unroll
        for (int j = k; j < N; ++j) {
          const cd a = A[k][j], b = A[i][j];
          A[k][j] = sw ? b : a;
          A[i][j] = sw ? a : b;
        }
        const cd a = x[k], b = x[i];
        x[k] = sw ? b : a;
        x[i] = sw ? a : b;
      }
    }
    // 1/piv = conj(piv) / |piv|^2: one real division per pivot, reused by the back
    // substitution (|Z| entries are far from the overflow range of |piv|^2)
    const cd piv = best != 0.0 ? A[k][k] : mk(1.0, 0.0);
    const double inv = 1.0 / (piv.r * piv.r + piv.i * piv.i);
    const cd rinv = mk(piv.r * inv, -piv.i * inv);
    A[k][k] = rinv;   // the diagonal is only needed as its reciprocal from here on
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const cd l = mul(A[i][k], rinv);
#pragma unroll
      for (int j = k + 1; j < N; ++j) A[i][j] = sub(A[i][j], mul(l, A[k][j]));
      x[i] = sub(x[i], mul(l, x[k]));
    }
  }
#pragma unroll
  for (int k = N - 1; k >= 0; --k) {
    cd s = x[k];
#pragma unroll
    for (int j = k + 1; j < N; ++j) s = sub(s, mul(A[k][j], x[j]));
    x[k] = mul(s, A[k][k]);
  }
  return ok;
}

// Factor-once / solve-many form of lu_solve (same pivot rule: max |re|+|im|, first maximum):
// A holds L below the diagonal, U above, the reciprocal pivots on it; piv[k] the row exchanged
// with k at step k.  Rows are exchanged in columns >= k only, so the multipliers of column k
// stay where they were formed and lu_apply replays each exchange before that column's
// elimination (as lu_solve does in one pass).  Returns false on an exactly zero pivot.
template <int N>
__device__ __forceinline__ bool lu_factor(cd (&A)[N][N], int (&piv)[N]) {
  bool ok = true;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int p = k;
    double best = cabs1(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const double v = cabs1(A[i][k]);
      if (v > best) { best = v; p = i; }
    }
    ok = ok && (best != 0.0);
    piv[k] = p;
    if (__builtin_amdgcn_ballot_w64(p != k) != 0) {
#pragma unroll
      for (int i = k + 1; i < N; ++i) {
        const bool sw = (p == i);
#pragma unroll
        for (int j = k; j < N; ++j) {   // columns >= k only: lu_apply replays the swaps interleaved
          const cd a = A[k][j], b = A[i][j];
          A[k][j] = sw ? b : a;
          A[i][j] = sw ? a : b;
        }
      }
    }
    const cd pv = best != 0.0 ? A[k][k] : mk(1.0, 0.0);
    const double inv = 1.0 / (pv.r * pv.r + pv.i * pv.i);
    const cd rinv = mk(pv.r * inv, -pv.i * inv);
    A[k][k] = rinv;
#pragma unroll
    for (int i = k + 1; i < N; ++i) {
      const cd l = mul(A[i][k], rinv);
      A[i][k] = l;
#pragma unroll
      for (int j = k + 1; j < N; ++j) A[i][j] = sub(A[i][j], mul(l, A[k][j]));
    }
  }
  return ok;
}
template <int N>
__device__ __forceinline__ void lu_apply(const cd (&A)[N][N], const int (&piv)[N], cd (&x)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (__builtin_amdgcn_ballot_w64(piv[k] != k) != 0) {
#pragma unroll
      for (int i = k + 1; i < N; ++i) {
        const bool sw = (piv[k] == i);
        const cd a = x[k], b = x[i];
        x[k] = sw ? b : a;
        x[i] = sw ? a : b;
      }
    }
#pragma unroll
    for (int i = k + 1; i < N; ++i) x[i] = sub(x[i], mul(A[i][k], x[k]));
  }
#pragma unroll
  for (int k = N - 1; k >= 0; --k) {
    cd s = x[k];
#pragma unroll
    for (int j = k + 1; j < N; ++j) s = sub(s, mul(A[k][j], x[j]));
    x[k] = mul(s, A[k][k]);
  }
}

// Raw buffer access: the 128-bit resource lives in SGPRs, each lane supplies one 32-bit byte
// offset and the per-array / per-component part is a scalar offset.  This keeps the many
// (array, DOF, bin) addresses of the case solve from being materialised as 64-bit VGPR pairs,
// and bounds every access by the resource size (out-of-range loads return 0, stores drop).
struct Buf {
  __amdgpu_buffer_rsrc_t r;
};
__device__ __forceinline__ Buf mkbuf(const void* p, unsigned bytes) {
  return Buf{__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000)};
}
__device__ __forceinline__ cd bld(Buf b, unsigned voff, unsigned soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(b.r, voff, soff, 0);
  const double2 d = __builtin_bit_cast(double2, v);
  return cd{d.x, d.y};
}
__device__ __forceinline__ void bst(Buf b, cd x, unsigned voff, unsigned soff) {
  const double2 d = make_double2(x.r, x.i);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), b.r, voff,
                                         soff, 0);
}
__device__ __forceinline__ double bld1(Buf b, unsigned voff, unsigned soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(b.r, voff, soff, 0);
  return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void bst1(Buf b, double x, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, x), b.r, voff,
                                        soff, 0);
}

// full 64-lane butterfly sum (every lane ends with the total)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// full 64-lane butterfly max (every lane ends with the maximum; NaN inputs are ignored)
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// Closest call of the all-bins convergence test (raft/raft_model.py:961-962): of the
// per-iteration values m = max_bins,dof tolCheck - tol, keep the one with the smallest |m|.
// A case whose closest call is within rounding of 0 could flip its iteration count.
__device__ __forceinline__ double closer_call(double best, double m) { return fabs(m) < fabs(best) ? m : best; }

// blockIdx -> work item such that blocks dispatched to the same XCD (b % 8 under the
// observed round-robin placement) get a CONTIGUOUS range of items; bijective for any G.
// Placement only affects speed (L2 locality of the per-design/heading tables), never results.
__device__ __forceinline__ int xcd_remap(int b, int G) {
  const int x = b & 7, q = G >> 3, r = G & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

}  // namespace rh
