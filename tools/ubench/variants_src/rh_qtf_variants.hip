// rh_qtf_variants.hip -- QTF kernels measured slower than the shipped chain and kept for A/B
// timing only (-DRH_VARIANTS, tools/build_variants.sh): k_qtf_gemm32 (32 x 32 pair
// tiles, rh_set_qtf_path(ctx, 2)) and k_qtf_lcoef + k_qtf_kay as two launches (rh_set_qtf_path(ctx, 3);
// k_qtf_lk runs both bodies in one launch).  Included by rh_abi.hip after rh_qtf_mfma.hip.

namespace rh {

// ---------------------------------------------------------------------------------------
// 32 x 32 pair tiles for a whole (unsharded) QTF: each wave computes the four 16 x 16
// sub-tiles of its DOF, so one pair of A fragments and one pair of B fragments feed 12 MFMAs
// per k-step instead of one pair feeding 3 (k_qtf_gemm is latency-bound on its operand loads,
// DESIGN.md §5).  Workgroup = 6 waves as in k_qtf_gemm (3 DOFs of the block's DOF half x two
// halves of K, the second half's partial sums reaching the first through LDS); blocks are
// (32-tile, DOF half) pairs.  Sub-tiles below the diagonal and beyond the grid are computed
// (uniform control) but not stored; the Kim & Yue sums of k_qtf_kay are per 16 x 16 tile.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void cgemm4_steps(const rh_c128* __restrict__ A0, const rh_c128* __restrict__ A1,
                                             const rh_c128* __restrict__ B0, const rh_c128* __restrict__ B1,
                                             size_t step, int nsteps, d4 (&p)[4][3]) {
  cd a[2][2], b[2][2];   // [step in batch][fragment]
  auto ldk = [&](int s, cd (&x)[2][2], cd (&y)[2][2], int j) {
    x[j][0] = ld(A0 + (size_t)s * step);
    x[j][1] = ld(A1 + (size_t)s * step);
    y[j][0] = ld(B0 + (size_t)s * step);
    y[j][1] = ld(B1 + (size_t)s * step);
  };
  ldk(0, a, b, 0);
  ldk(1, a, b, 1);
#pragma unroll 1
  for (int s = 0; s < nsteps; s += 2) {
    cd an[2][2], bn[2][2];
    const bool more = s + 2 < nsteps;
    if (more) {
      ldk(s + 2, an, bn, 0);
      ldk(s + 3, an, bn, 1);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          d4 (&q)[3] = p[2 * x + y];
          q[0] = mfma64(a[j][x].r, b[j][y].r, q[0]);
          q[1] = mfma64(a[j][x].i, b[j][y].i, q[1]);
          q[2] = mfma64(a[j][x].r + a[j][x].i, b[j][y].r + b[j][y].i, q[2]);
        }
    if (more) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          a[j][x] = an[j][x];
          b[j][x] = bn[j][x];
        }
    }
  }
}

__global__ __launch_bounds__(384) void k_qtf_gemm32(rh_qtf_design q, QtfWork wk, rh_c128* __restrict__ qtf) {
  __shared__ double part[3][4][16][64];   // half 1's partial sums: [DOF][sub-tile][value][lane]
  __shared__ double pscal[4][4][256];     // per sub-tile and pair: aux2 (w1 - w2) alpha+, alpha- (complex)
  const int lane = (int)threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int half = w / 3, dl = w % 3;
  const int n2 = q.n2, n2p = qtf_n2p(q), nt = n2p / 16, nt32 = (nt + 1) / 2, kp = qtf_kp(q), kq = qtf_kq(q);
  const int slot = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const int d = 3 * (slot & 1) + dl;
  int T1, T2;
  qtf_tile_of(slot >> 1, nt32, T1, T2);
  const int mr = lane & 15, kr = lane >> 4;
  const int i1b = 32 * T1, i2b = 32 * T2;
  const int c10 = min(i1b + mr, n2p - 1), c11 = min(i1b + 16 + mr, n2p - 1);   // operand columns (clamped
  const int c20 = min(i2b + mr, n2p - 1), c21 = min(i2b + 16 + mr, n2p - 1);   // past the padded grid)
  const size_t step = (size_t)4 * n2p;
  const int ns = kp / 4, ns0 = 4 * ((ns / 4 + 1) / 2);
  const int k0 = half == 0 ? 0 : ns0, nk = half == 0 ? ns0 : ns - ns0;
  d4 pb[4][3], pc[4][3];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int g = 0; g < 3; ++g) pb[t][g] = pc[t][g] = d4{0, 0, 0, 0};
  if (nk > 0) {
    const size_t ra = ((size_t)d * kp + 4 * k0 + kr) * n2p, rb = ((size_t)4 * k0 + kr) * n2p;
    cgemm4_steps(wk.L + ra + c10, wk.L + ra + c11, wk.R + rb + c20, wk.R + rb + c21, step, nk, pb);
  }
  {
    const size_t ra = (((size_t)half * 6 + d) * kq + kr) * n2p, rb = ((size_t)half * kq + kr) * n2p;
    cgemm4_steps(wk.Lp + ra + c10, wk.Lp + ra + c11, wk.Rp + rb + c20, wk.Rp + rb + c21, step, kq / 4, pc);
  }
  const double h = q.depth, g = q.g, bt = q.beta * kDeg2Rad, cb = cos(bt), sb = sin(bt);
  if (half == 1) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        part[dl][t][r][lane] = pb[t][0][r] - pb[t][1][r];
        part[dl][t][4 + r][lane] = pb[t][2][r] - pb[t][0][r] - pb[t][1][r];
        part[dl][t][8 + r][lane] = pc[t][0][r] - pc[t][1][r];
        part[dl][t][12 + r][lane] = pc[t][2][r] - pc[t][0][r] - pc[t][1][r];
      }
    // the pair scalars of the second-order potential (raft/helpers.py:254-291), as k_qtf_gemm
    for (int e = (int)threadIdx.x - 192; e < 1024; e += 192) {
      const int t = e >> 8, x = t >> 1, y = t & 1, el = e & 255;
      const int i1 = min(i1b + 16 * x + (el >> 4), n2 - 1), i2 = min(i2b + 16 * y + (el & 15), n2 - 1);
      cd sp, sm;
      qtf_pot_scalars(q.w2[i1], q.k2[i1], tanh(q.k2[i1] * h), q.w2[i2], q.k2[i2], tanh(q.k2[i2] * h), cb, sb, h, g, sp, sm);
      pscal[t][0][el] = sp.r;
      pscal[t][1][el] = sp.i;
      pscal[t][2][el] = sm.r;
      pscal[t][3][el] = sm.i;
    }
  }
  __syncthreads();
  if (half == 1) return;
  // + each sub-tile's Kim & Yue sums (k_qtf_kay), then the upper-triangle entry and its
  // Hermitian mirror (raft/raft_fowt.py:1639-1640), the arithmetic of k_qtf_gemm's epilogue
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int x = t >> 1, y = t & 1;
    const int s1 = 2 * T1 + x, s2 = 2 * T2 + y;   // 16 x 16 sub-tile
    if (s1 >= nt || s2 >= nt || s2 < s1) continue;   // uniform
    const double* ks = wk.KS + (size_t)qtf_tile_id(s1, s2, nt) * 12 * 256;
    const int i2 = 16 * s2 + mr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i1 = 16 * s1 + kr + 4 * r;
      if (i1 >= n2 || i2 >= n2 || i2 < i1) continue;
      const int e = (kr + 4 * r) * 16 + mr;
      const double mre = pb[t][0][r] - pb[t][1][r], mim = pb[t][2][r] - pb[t][0][r] - pb[t][1][r];
      const double cre = pc[t][0][r] - pc[t][1][r], cim = pc[t][2][r] - pc[t][0][r] - pc[t][1][r];
      const int ek = kr * 16 + mr + 64 * r;   // kay_tile's element of this pair
      const cd Qf = qtf_pair_sum(mre, mim, part[dl][t][r][lane], part[dl][t][4 + r][lane], cre, cim,
                                 part[dl][t][8 + r][lane], part[dl][t][12 + r][lane], pscal[t][0][e], pscal[t][1][e],
                                 pscal[t][2][e], pscal[t][3][e], ks[(2 * d) * 256 + ek], ks[(2 * d + 1) * 256 + ek]);
      rh_c128* up = qtf + ((size_t)i1 * n2 + i2) * 6 + d;
      if (i1 == i2) {
        st(up, sub(add(Qf, cconj(Qf)), cconj(Qf)));
      } else {
        st(up, Qf);
        st(qtf + ((size_t)i2 * n2 + i1) * 6 + d, cconj(Qf));
      }
    }
  }
}


// The w1-side GEMM coefficients: grid (ceil(n2p / 64), 18 + nq + nmq), 512 threads (lcoef_block).
__global__ __launch_bounds__(512) void k_qtf_lcoef(rh_qtf_design q, QtfWork wk, const double* __restrict__ M66) {
  __shared__ double red[8][12][64];
  lcoef_block(q, wk, M66, (int)blockIdx.x, (int)blockIdx.y, red);
}

// The Kim & Yue sums of this rank's pair tiles (kay_tile), one tile per workgroup; the GEMM
// epilogue adds them (before round 4 this kernel ran on a second stream beside k_qtf_lcoef +
// k_qtf_gemm, with two event hand-offs and a final k_qtf_kay_sum launch).
__global__ __launch_bounds__(kKayThreads) __attribute__((amdgpu_waves_per_eu(RH_KAY_WPE))) void k_qtf_kay(
    rh_qtf_design q, QtfWork wk, int t0) {
  __shared__ double acc[12][256];
  __shared__ double psg[kPsg];   // the parts' row sums
  int T1, T2;
  qtf_tile_of(t0 + xcd_remap((int)blockIdx.x, (int)gridDim.x), qtf_n2p(q) / 16, T1, T2);
  kay_tile<kKayS>(q, wk, T1, T2, true, (int)threadIdx.x, acc, psg);
}

}  // namespace rh
