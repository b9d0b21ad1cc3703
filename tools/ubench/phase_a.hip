// phase_a.hip -- go/no-go microbenchmark: phase A of the drag fixed point (per-node sums of
// |relative velocity|^2 over the bins, raft/raft_fowt.py:1205-1220) as a STANDALONE kernel
// with a small register budget, several workgroups per case and several waves per SIMD,
// against the ~0.082 ms per 512-case iteration that phase A takes inside k_solve_lds<2,512>.
// Random data of the C2 shapes (53 nodes, 9 members, nw = 1000, 4 headings, 512 cases).
//   hipcc --offload-arch=gfx950 -O3 -o phase_a tools/ubench/phase_a.hip && ./phase_a
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../raft-teststuff_amd/csrc/rh_device.h"

using namespace rh;

constexpr int NN = 53, NM = 9, NW = 1000, NH = 4, NC = 512;

__device__ __forceinline__ double dmov(double v, int ctrl_dummy);

template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double xs32(double t) {
  const int lo = __double2loint(t), hi = __double2hiint(t);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double xs16(double t) {
  const int lo = __double2loint(t), hi = __double2hiint(t);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double tb3(double a, double b, double c, int lane) {
  const bool f0 = (lane & 1) != 0, f1 = (lane & 2) != 0;
  const double k0 = f0 ? c : a, s0 = f0 ? a : c;
  const double k1 = f0 ? 0.0 : b, s1 = f0 ? b : 0.0;
  const double u0 = k0 + dpp<0xB1>(s0);
  const double u1 = k1 + dpp<0xB1>(s1);
  double t = (f1 ? u1 : u0) + dpp<0x4E>(f1 ? u0 : u1);
  t += dpp<0x124>(t);
  t += dpp<0x128>(t);
  return xs32(xs16(t));
}

struct Args {
  const rh_c128* kproj;   // [NH][NN][3][NW]
  const rh_c128* xl;      // [NC][6][NW]
  const double* zeta;     // [NC][NW]
  const double* w;        // [NW]
  const int* head;        // [NC]
  const double* memb;     // [18][NM] cq, c1, c2
  const int* mstart;      // [NM+1]
  const double* nt;       // [NN]
  double* part;           // [NC][chunks][NN][3]
};

// T threads per workgroup, NB bins per lane, R-node prefetch ring; a workgroup covers T*NB bins
template <int T, int NB, int R, int WPS>
__global__ __launch_bounds__(T, WPS) void k_phase_a(Args a) {
  constexpr int LW = T / 64;
  constexpr int CB = T * NB;
  const int chunks = (NW + CB - 1) / CB;
  const int ic = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  __shared__ double red[NN * 3 * LW];
  const unsigned nw16 = NW * 16u;
  const Buf bK = mkbuf(a.kproj + (size_t)a.head[ic] * NN * 3 * NW, NN * 3u * nw16);
  unsigned vb[NB];
  double z[NB];
  cd X[NB][6];
  double w[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int b0 = ch * CB + tid + T * j;
    const bool ok = b0 < NW;
    const int b = ok ? b0 : NW - 1;
    vb[j] = (unsigned)b * 16u;
    z[j] = ok ? a.zeta[(size_t)ic * NW + b] : 0.0;
    w[j] = a.w[b];
#pragma unroll
    for (int c = 0; c < 6; ++c) X[j][c] = ld(a.xl + ((size_t)ic * 6 + c) * NW + b);
  }
  cd Bq[NB], B1[NB], B2[NB], E1[NB], E2[NB];
  auto member_terms = [&](int m) {
    double cq[6], c1[6], c2[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      cq[i] = a.memb[i * NM + m];
      c1[i] = a.memb[(6 + i) * NM + m];
      c2[i] = a.memb[(12 + i) * NM + m];
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      cd Aq = mk(0, 0), A1 = mk(0, 0), A2 = mk(0, 0);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        Aq = add(Aq, scl(X[j][c], cq[c]));
        A1 = add(A1, scl(X[j][c], c1[c]));
        A2 = add(A2, scl(X[j][c], c2[c]));
      }
      const cd D1 = add(add(scl(X[j][3], c2[0]), scl(X[j][4], c2[1])), scl(X[j][5], c2[2]));
      const cd D2 = add(add(scl(X[j][3], c1[0]), scl(X[j][4], c1[1])), scl(X[j][5], c1[2]));
      Bq[j] = iw(w[j], Aq);
      B1[j] = iw(w[j], A1);
      B2[j] = iw(w[j], A2);
      E1[j] = iw(w[j], D1);
      E2[j] = iw(-w[j], D2);
    }
  };
  auto load_node = [&](cd (&K)[3][NB], int n) {
    const unsigned so = (unsigned)(n < NN ? n : NN - 1) * 3u * nw16;
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) K[p][j] = bld(bK, vb[j], so + (unsigned)p * nw16);
  };
  cd K[R][3][NB];
#pragma unroll
  for (int r = 0; r < R; ++r) load_node(K[r], r);
  int m = -1, mnext = 0;
  for (int n = 0; n < NN; n += R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int nr = n + r;
      if (nr < NN) {
        if (nr == mnext) {
          do { ++m; mnext = a.mstart[m + 1]; } while (mnext == nr);
          member_terms(m);
        }
        const double t = a.nt[nr];
        double s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const cd sq = sub(scl(K[r][0][j], z[j]), Bq[j]);
          const cd sp1 = sub(scl(K[r][1][j], z[j]), add(B1[j], scl(E1[j], t)));
          const cd sp2 = sub(scl(K[r][2][j], z[j]), add(B2[j], scl(E2[j], t)));
          s0 += abs2(sq);
          s1 += abs2(sp1);
          s2 += abs2(sp2);
        }
        load_node(K[r], nr + R);
        const double tot = tb3(s0, s1, s2, lane);
        if (lane < 3) red[(nr * 3 + (2 * (lane & 1) + ((lane >> 1) & 1))) * LW + wv] = tot;
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < NN * 3; e += T) {
    double s = 0;
#pragma unroll
    for (int q = 0; q < LW; ++q) s += red[e * LW + q];
    a.part[((size_t)ic * chunks + ch) * NN * 3 + e] = s;
  }
}


// phase C1: drag excitation per bin (member-factored), F written to global
struct ArgsC {
  const rh_c128* kproj;   // [NH][NN][3][NW]
  const double* al;       // [NC][NN][5]
  const int* head;
  const double* memb;     // [18][NM]
  const int* mstart;
  rh_c128* F;             // [NC][6][NW]
  const rh_c128* finer;   // [NH][6][NW]
  const double* zeta;     // [NC][NW]
  const double* w;
  const double* mbc;      // [108] M, B, C
  rh_c128* xl;            // [NC][6][NW]
  rh_c128* xo;            // [NC][6][NW]
  int* flags;             // [NC]
};
template <int T, int R, int WPS>
__global__ __launch_bounds__(T, WPS) void k_phase_c1(ArgsC a) {
  const int chunks = (NW + T - 1) / T;
  const int ic = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const int b0 = ch * T + threadIdx.x;
  const int b = b0 < NW ? b0 : NW - 1;
  const unsigned nw16 = NW * 16u, vj = (unsigned)b * 16u;
  const Buf bK = mkbuf(a.kproj + (size_t)a.head[ic] * NN * 3 * NW, NN * 3u * nw16);
  const double* al = a.al + (size_t)ic * NN * 5;
  cd F[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) F[c] = mk(0, 0);
  cd SQ = mk(0, 0), S1 = mk(0, 0), S2 = mk(0, 0), T1 = mk(0, 0), T2 = mk(0, 0);
  int m = 0, mnext = a.mstart[1];
  auto fold = [&]() {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const double cq = a.memb[i * NM + m], c1 = a.memb[(6 + i) * NM + m], c2 = a.memb[(12 + i) * NM + m];
      F[i] = add(F[i], add(add(scl(SQ, cq), scl(S1, c1)), scl(S2, c2)));
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double p1 = a.memb[(6 + i) * NM + m], p2 = a.memb[(12 + i) * NM + m];
      F[3 + i] = add(F[3 + i], sub(scl(T1, p2), scl(T2, p1)));
    }
    SQ = S1 = S2 = T1 = T2 = mk(0, 0);
  };
  auto load1 = [&](cd (&K)[3], int n) {
    const unsigned so = (unsigned)(n < NN ? n : NN - 1) * 3u * nw16;
#pragma unroll
    for (int p = 0; p < 3; ++p) K[p] = bld(bK, vj, so + (unsigned)p * nw16);
  };
  cd K[R][3];
#pragma unroll
  for (int r = 0; r < R; ++r) load1(K[r], r);
  for (int n = 0; n < NN; n += R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int nr = n + r;
      if (nr < NN) {
        while (nr == mnext) { fold(); ++m; mnext = a.mstart[m + 1]; }
        const double* A = al + 5 * nr;
        SQ = add(SQ, scl(K[r][0], A[0]));
        S1 = add(S1, scl(K[r][1], A[1]));
        S2 = add(S2, scl(K[r][2], A[2]));
        T1 = add(T1, scl(K[r][1], A[3]));
        T2 = add(T2, scl(K[r][2], A[4]));
        load1(K[r], nr + R);
      }
    }
  }
  fold();
  if (b0 < NW)
#pragma unroll
    for (int c = 0; c < 6; ++c) st(a.F + ((size_t)ic * 6 + c) * NW + b, F[c]);
}
// phase C2: Z(w) assembly, LU, tolCheck, relaxation; one bin per lane
template <int T, int WPS>
__global__ __launch_bounds__(T, WPS) void k_phase_c2(ArgsC a) {
  const int chunks = (NW + T - 1) / T;
  const int ic = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const int b0 = ch * T + threadIdx.x;
  const bool okb = b0 < NW;
  const int b = okb ? b0 : NW - 1;
  const double w = a.w[b], z = okb ? a.zeta[(size_t)ic * NW + b] : 0.0, w2 = -w * w;
  cd F[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    const cd fe = ld(a.finer + ((size_t)a.head[ic] * 6 + c) * NW + b);
    const cd fd = ld(a.F + ((size_t)ic * 6 + c) * NW + b);
    F[c] = add(scl(fe, z), scl(fd, z));
  }
  cd Z[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = 0; c < 6; ++c) Z[r][c] = mk(w2 * a.mbc[6 * r + c] + a.mbc[72 + 6 * r + c], w * a.mbc[36 + 6 * r + c]);
  const bool ok = lu_solve<6>(Z, F);
  bool conv = true;
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    const cd x = F[c];
    const cd xlast = ld(a.xl + ((size_t)ic * 6 + c) * NW + b);
    const double tt = sqrt(abs2(sub(x, xlast))) / (sqrt(abs2(x)) + 0.01);
    conv = conv && tt < 0.01;
    if (okb) {
      st_nt(a.xo + ((size_t)ic * 6 + c) * NW + b, x);
      st(a.xl + ((size_t)ic * 6 + c) * NW + b, add(scl(xlast, 0.2), scl(x, 0.8)));
    }
  }
  if (!__builtin_amdgcn_ballot_w64(conv && ok) && okb) a.flags[ic] = 1;
}
template <int T, int R, int WPS>
void runc1(const char* name, ArgsC a) {
  const int chunks = (NW + T - 1) / T;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_phase_c1<T, R, WPS>), dim3(NC * chunks), dim3(T), 0, 0, a);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_phase_c1<T, R, WPS>), dim3(NC * chunks), dim3(T), 0, 0, a);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipFuncAttributes at;
  hipFuncGetAttributes(&at, (const void*)k_phase_c1<T, R, WPS>);
  printf("C1 %-25s %8.4f ms per 512-case pass  (%d regs, spill %zu B)\n", name, ms / 20, at.numRegs, at.localSizeBytes);
}
template <int T, int WPS>
void runc2(const char* name, ArgsC a) {
  const int chunks = (NW + T - 1) / T;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_phase_c2<T, WPS>), dim3(NC * chunks), dim3(T), 0, 0, a);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_phase_c2<T, WPS>), dim3(NC * chunks), dim3(T), 0, 0, a);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipFuncAttributes at;
  hipFuncGetAttributes(&at, (const void*)k_phase_c2<T, WPS>);
  printf("C2 %-25s %8.4f ms per 512-case pass  (%d regs, spill %zu B)\n", name, ms / 20, at.numRegs, at.localSizeBytes);
}

template <int T, int NB, int R, int WPS>
void run(const char* name, Args a) {
  constexpr int CB = T * NB;
  const int chunks = (NW + CB - 1) / CB;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_phase_a<T, NB, R, WPS>), dim3(NC * chunks), dim3(T), 0, 0, a);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_phase_a<T, NB, R, WPS>), dim3(NC * chunks), dim3(T), 0, 0, a);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipFuncAttributes at;
  hipFuncGetAttributes(&at, (const void*)k_phase_a<T, NB, R, WPS>);
  printf("%-28s T=%4d NB=%d R=%d  %8.4f ms per 512-case pass  (vgpr? %d regs, spill %zu B)\n", name, T, NB, R,
         ms / reps, at.numRegs, at.localSizeBytes);
}

int main() {
  srand(1);
  auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
  std::vector<rh_c128> kp((size_t)NH * NN * 3 * NW), xl((size_t)NC * 6 * NW);
  for (auto& v : kp) v = {rnd(), rnd()};
  for (auto& v : xl) v = {rnd(), rnd()};
  std::vector<double> zeta((size_t)NC * NW), w(NW), memb(18 * NM), nt(NN);
  for (auto& v : zeta) v = rnd();
  for (int i = 0; i < NW; ++i) w[i] = 0.01 + 0.001 * i;
  for (auto& v : memb) v = rnd();
  for (auto& v : nt) v = rnd();
  std::vector<int> head(NC), ms(NM + 1);
  for (int i = 0; i < NC; ++i) head[i] = i % NH;
  for (int m = 0; m <= NM; ++m) ms[m] = m * NN / NM;
  ms[NM] = NN;
  Args a;
  rh_c128 *dkp, *dxl;
  double *dz, *dw, *dm, *dnt, *dp;
  int *dh, *dms;
  hipMalloc(&dkp, kp.size() * 16);
  hipMalloc(&dxl, xl.size() * 16);
  hipMalloc(&dz, zeta.size() * 8);
  hipMalloc(&dw, w.size() * 8);
  hipMalloc(&dm, memb.size() * 8);
  hipMalloc(&dnt, nt.size() * 8);
  hipMalloc(&dh, NC * 4);
  hipMalloc(&dms, (NM + 1) * 4);
  hipMalloc(&dp, (size_t)NC * 8 * NN * 3 * 8);
  hipMemcpy(dkp, kp.data(), kp.size() * 16, hipMemcpyHostToDevice);
  hipMemcpy(dxl, xl.data(), xl.size() * 16, hipMemcpyHostToDevice);
  hipMemcpy(dz, zeta.data(), zeta.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), w.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dm, memb.data(), memb.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dnt, nt.data(), nt.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dh, head.data(), NC * 4, hipMemcpyHostToDevice);
  hipMemcpy(dms, ms.data(), (NM + 1) * 4, hipMemcpyHostToDevice);
  a = Args{dkp, dxl, dz, dw, dh, dm, dms, dnt, dp};
  run<256, 1, 3, 4>("T256 NB1 R3 (4 w/SIMD)", a);
  run<256, 1, 4, 4>("T256 NB1 R4 (4 w/SIMD)", a);
  run<256, 1, 6, 3>("T256 NB1 R6 (3 w/SIMD)", a);
  run<256, 2, 3, 3>("T256 NB2 R3 (3 w/SIMD)", a);
  run<512, 2, 3, 2>("T512 NB2 R3 (2 w/SIMD)", a);
  run<128, 1, 4, 8>("T128 NB1 R4 (8 WG/CU)", a);
  run<256, 1, 2, 5>("T256 NB1 R2 (5 w/SIMD)", a);

  {
    double *dal, *dmbc;
    rh_c128 *dF, *dfe, *dxo;
    int* dfl;
    std::vector<double> al((size_t)NC * NN * 5), mbc(108);
    for (auto& v : al) v = rnd();
    for (int i = 0; i < 108; ++i) mbc[i] = (i % 7 == 0) ? 10.0 + rnd() : rnd();
    std::vector<rh_c128> fe((size_t)NH * 6 * NW);
    for (auto& v : fe) v = {rnd(), rnd()};
    hipMalloc(&dal, al.size() * 8);
    hipMalloc(&dmbc, 108 * 8);
    hipMalloc(&dF, (size_t)NC * 6 * NW * 16);
    hipMalloc(&dfe, fe.size() * 16);
    hipMalloc(&dxo, (size_t)NC * 6 * NW * 16);
    hipMalloc(&dfl, NC * 4);
    hipMemcpy(dal, al.data(), al.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dmbc, mbc.data(), 108 * 8, hipMemcpyHostToDevice);
    hipMemcpy(dfe, fe.data(), fe.size() * 16, hipMemcpyHostToDevice);
    hipMemset(dF, 0, (size_t)NC * 6 * NW * 16);
    ArgsC c{dkp, dal, dh, dm, dms, dF, dfe, dz, dw, dmbc, dxl, dxo, dfl};
    runc1<256, 3, 4>("T256 R3", c);
    runc1<256, 6, 3>("T256 R6", c);
    runc1<256, 8, 2>("T256 R8", c);
    runc1<512, 6, 2>("T512 R6", c);
    runc2<256, 2>("T256 (2 w/SIMD)", c);
    runc2<256, 1>("T256 (1 WG req)", c);
    runc2<128, 2>("T128", c);
    runc2<64, 2>("T64", c);
  }
  return 0;
}
