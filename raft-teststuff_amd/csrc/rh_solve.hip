// rh_solve.hip -- k_solve_lds: the per-case drag fixed point with the relaxed iterate in LDS.
//
// Same algorithm and arithmetic as k_solve_cases (rh_kernels.hip; raft/raft_model.py:918-1000,
// raft/raft_fowt.py:1152-1293), re-laid-out for latency on gfx950:
//   * 512 threads (8 waves) per case, one case per CU; lane = bin, NB <= 2 bins per thread.
//   * XiLast lives in LDS ([6][512 NB] complex) for the whole solve: the thread that owns a
//     bin is the only one that reads or writes it, so no global round trip per iteration.
//     The unrelaxed solution is streamed to HBM with non-temporal stores (it is only
//     consumed after the loop), so it does not evict the wave tables from L2.
//   * The projected wave table (kproj, the only per-node stream) is read through a buffer
//     resource (one 32-bit lane offset per bin, node/projection offsets scalar) with a
//     3-slot register ring: node n+2 is in flight while node n is reduced.
//   * Per-node bin sums: a 6-step DPP wave reduction (VALU only, no LDS or SGPR traffic),
//     one partial per wave, summed in wave order.  Fixed order, so results are deterministic.
#include "rh_common.h"
#ifdef RH_VARIANTS
#include "../../tools/ubench/variants_src/rh_a0_common.h"   // k_a0_sums sums (rh_set_a0)
#endif

namespace rh {

#ifdef RH_PROF
// Phase cycle counters (s_memtime of wave 0 of every workgroup), summed over workgroups:
// [0] prologue [1] A [2] B [3] C excitation [4] C solve [5] flags [6] epilogue [7] iterations
static __device__ unsigned long long rh_prof[12];   // static: one per translation unit (rh_prof_read reads rh_solve_fast.hip's)
#define PROF_T(v) const unsigned long long v = clock64()
#define PROF_ADD(i, x) if (tid == 0) atomicAdd(&rh_prof[i], (unsigned long long)(x))
#else
#define PROF_T(v)
#define PROF_ADD(i, x)
#endif

#ifdef RH_WGTIME
// Per-workgroup wall-clock (s_memrealtime, 100 MHz) of the fixed point: [2 slot] = start,
// [2 slot + 1] = end of the loop, by dispatch slot (launch-tail analysis, tools/ubench/wg_times.py)
static __device__ unsigned long long rh_wgt[2 * 8192];
#endif

constexpr int kLT = 512;          // threads per case workgroup
constexpr int kLW = kLT / 64;     // waves per case workgroup
#ifndef RH_RING_A
#define RH_RING_A 4               // (3 in the two-pass kernel: 4 moves its spills into the streaming loops)
#endif
#ifndef RH_RING_C
#define RH_RING_C 6
#endif
constexpr int kRingA1 = RH_RING_A; // wave-table prefetch depth (nodes) of phase A
constexpr int kRingC = RH_RING_C; // ... of phase C (one bin per pass: less work per node)
#ifndef RH_ONE_VOTE
#define RH_ONE_VOTE 0                 // 1: one barrier (LDS flag word) for the three end-of-iteration votes
#endif
#ifndef RH_OVERLAP
#define RH_OVERLAP 1                  // 1: no barrier vote between phase C and the next phase A (single-pass kernels)
#endif
#ifndef RH_STATS_C
#define RH_STATS_C 1                  // 1: PSD / RAO / RMS sums formed where phase C stores Xi (no read-back)
#endif
#ifndef RH_XI_STORE
#define RH_XI_STORE 1                 // 0: per-entry stores of passing entries; 1: while the iteration may be final; 2: traffic floor (A/B)
#endif
#define XI_STORE_MODE RH_XI_STORE
#ifndef RH_A_BATCH
#define RH_A_BATCH 0                  // > 0: phase-A nodes in batches of RH_A_BATCH, one tbfly16 per batch
#endif
#ifndef RH_A_PAIR
#define RH_A_PAIR 1                   // 1: phase-A sums of two nodes per butterfly (tbfly6)
#endif
#ifndef RH_LDS_LANE_BRANCH
#define RH_LDS_LANE_BRANCH 0          // 1: the round-2 per-lane `continue` before the solve (A/B only)
#endif

// A scalar zero the compiler cannot fold (see its use in phase C).
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}

// The lane index, recomputed where it is used: a hoisted copy would be one more value kept
// live across the whole solve (and spilled, and its reload would drain the prefetch ring,
// since scratch loads share the vector-memory counter with the wave-table loads).
__device__ __forceinline__ int lane_here() {
  int r;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
  return r;
}

template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {   // full-mask permutations: every lane valid
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// t + t(lane ^ 32) and t + t(lane ^ 16) with the gfx950 row-swap instructions
// (v_permlane32_swap / v_permlane16_swap: VALU, no LDS round trip as with ds_bpermute).
// Called with both operands equal, the swap leaves {x_i, x_partner} split over its two
// results in lane-dependent order, and their sum is the pair sum (bitwise the same as
// t + __shfl_xor(t, 32 | 16): FP addition commutes).  Call with every lane active.
__device__ __forceinline__ double xsum32(double t) {
  const int lo = __double2loint(t), hi = __double2hiint(t);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double xsum16(double t) {
  const int lo = __double2loint(t), hi = __double2hiint(t);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}

// Transposing butterfly: 16 per-lane values u[k] -> lane i of EVERY row ends with the wave
// total (all 64 lanes) of value k(i) = 8 f0 + 4 f1 + 2 f2 + f3, with the lane bits
//   f0 = b0^b2, f1 = b1^b2, f2 = b2^b3, f3 = b3     (i = lane & 15, b = bits of i).
// Stage s pairs lane i with i^1 (quad_perm [1,0,3,2]), i^2 (quad_perm [2,3,0,1]), i^7
// (row_half_mirror), i^15 (row_mirror); the f_s differ across each pair and agree on the
// values both lanes still hold, so each lane keeps one half, sends the other, and the value
// count halves per stage: 15 exchanges for 16 values instead of 16 full reductions.  The
// four row sums are then combined across rows (lane^16, lane^32).  Fixed order everywhere.
__device__ __forceinline__ double tbfly16(double (&u)[16], int lane) {
  const int i = lane & 15;
  const bool f0 = ((i ^ (i >> 2)) & 1) != 0, f1 = (((i >> 1) ^ (i >> 2)) & 1) != 0;
  const bool f2 = (((i >> 2) ^ (i >> 3)) & 1) != 0, f3 = ((i >> 3) & 1) != 0;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const double keep = f0 ? u[p + 8] : u[p], send = f0 ? u[p] : u[p + 8];
    u[p] = keep + dpp_mov<0xB1>(send);
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const double keep = f1 ? u[p + 4] : u[p], send = f1 ? u[p] : u[p + 4];
    u[p] = keep + dpp_mov<0x4E>(send);
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const double keep = f2 ? u[p + 2] : u[p], send = f2 ? u[p] : u[p + 2];
    u[p] = keep + dpp_mov<0x141>(send);
  }
  {
    const double keep = f3 ? u[1] : u[0], send = f3 ? u[0] : u[1];
    u[0] = keep + dpp_mov<0x140>(send);
  }
  return xsum32(xsum16(u[0]));
}
__device__ __forceinline__ int tbfly16_index(int lane) {
  const int i = lane & 15;
  return 8 * ((i ^ (i >> 2)) & 1) + 4 * (((i >> 1) ^ (i >> 2)) & 1) + 2 * (((i >> 2) ^ (i >> 3)) & 1) + ((i >> 3) & 1);
}

// Three wave sums at once.  A 2-stage transposing butterfly inside each quad (partners i^1,
// i^2: each lane keeps one of the values {a, b, c, 0}), then the quad sums are folded over
// the row (row_ror 4, 8) and over the rows (lane^16, lane^32).  Every lane ends with the
// wave total of value tbfly3_index(lane) (0 = a, 1 = b, 2 = c, 3 = pad): lanes 0, 2, 1
// hold a, b, c.  33 instructions instead of 3 x 18 for three separate reductions.
__device__ __forceinline__ double tbfly3(double a, double b, double c, int lane) {
  const bool f0 = (lane & 1) != 0, f1 = (lane & 2) != 0;
  // stage 0: pairs (a, c) and (b, 0): keep the second of each pair if f0
  const double k0 = f0 ? c : a, s0 = f0 ? a : c;
  const double k1 = f0 ? 0.0 : b, s1 = f0 ? b : 0.0;
  const double u0 = k0 + dpp_mov<0xB1>(s0);
  const double u1 = k1 + dpp_mov<0xB1>(s1);
  // stage 1: pair (u0, u1): keep u1 if f1
  double t = (f1 ? u1 : u0) + dpp_mov<0x4E>(f1 ? u0 : u1);
  t += dpp_mov<0x124>(t);   // row_ror:4
  t += dpp_mov<0x128>(t);   // row_ror:8
  return xsum32(xsum16(t));
}
// value held by a lane after tbfly3: 2 f0 + f1 -> lane 0: a (0), lane 1: c (2), lane 2: b (1)
__device__ __forceinline__ int tbfly3_index(int lane) { return 2 * (lane & 1) + ((lane >> 1) & 1); }

// Six wave sums at once: the three sums of two nodes.  Transposing stages with tbfly16's lane
// flags (partners i^1, i^2, i^7 within the 16-lane row): (a0, a1), (b0, b1), (c0, c1) -> three
// values, (v0, v1), (v2, 0) -> two, then one; the row halves (i^15) hold the same value and
// are added, then the rows (lane^16, lane^32).  9 exchanges instead of 2 x 7 for two tbfly3.
struct Bfly6 {   // a lane's stage flags and the sum it holds after tbfly6 (formed once per phase A)
  bool f0, f1, f2;
  int vi;         // 3 node + sum, or -1 (pad; lanes >= 8 hold copies)
};
__device__ __forceinline__ Bfly6 bfly6_lane(int lane) {
  const int i = lane & 15;
  Bfly6 b;
  b.f0 = ((i ^ (i >> 2)) & 1) != 0;
  b.f1 = (((i >> 1) ^ (i >> 2)) & 1) != 0;
  b.f2 = (((i >> 2) ^ (i >> 3)) & 1) != 0;
  b.vi = lane >= 8 ? -1 : b.f2 ? (b.f1 ? -1 : 3 * b.f0 + 2) : 3 * b.f0 + b.f1;
  return b;
}
__device__ __forceinline__ double tbfly6(double a0, double b0, double c0, double a1, double b1, double c1, const Bfly6& L) {
  const bool f0 = L.f0, f1 = L.f1, f2 = L.f2;
  const double v0 = (f0 ? a1 : a0) + dpp_mov<0xB1>(f0 ? a0 : a1);
  const double v1 = (f0 ? b1 : b0) + dpp_mov<0xB1>(f0 ? b0 : b1);
  const double v2 = (f0 ? c1 : c0) + dpp_mov<0xB1>(f0 ? c0 : c1);
  const double w0 = (f1 ? v1 : v0) + dpp_mov<0x4E>(f1 ? v0 : v1);
  const double w1 = (f1 ? 0.0 : v2) + dpp_mov<0x4E>(f1 ? v2 : 0.0);
  double t = (f2 ? w1 : w0) + dpp_mov<0x141>(f2 ? w0 : w1);
  t += dpp_mov<0x140>(t);
  return xsum32(xsum16(t));
}

template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_mov_rows(double v) {   // rows outside ROWS receive 0
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum over the whole wave, complete in lane 63 only.  Call with every lane active.
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror and row_mirror give every lane
// its 16-lane row total r_k; row_bcast:15 then adds r0 into row 1 and r2 into row 3, and
// row_bcast:31 adds row 1 into row 3: lane 63 = (r3 + r2) + (r1 + r0).  VALU only, no
// LDS or SGPR traffic, fixed order.
__device__ __forceinline__ double wave_sum63(double v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  v += dpp_mov_rows<0x142, 0xA>(v);
  v += dpp_mov_rows<0x143, 0xC>(v);
  return v;
}

// One entry of translateMatrix3to6DOF by block: 0 = Bm[r][c], 1 = (Bm H)[r][c] (the upper-right
// block; the lower-left one is its transpose), 2 = (H Bm H^T)[r][c]; the expressions of t3to6
// (rh_kernels.hip), evaluated for all three and selected, so no lane branches.
__device__ __forceinline__ double t3to6_block(const double* Bm, double rx, double ry, double rz, int blk, int r, int c) {
  const double H[3][3] = {{0, rz, -ry}, {-rz, 0, rx}, {ry, -rx, 0}};
  double hc[3], hr[3];   // column c of H, row r of H (selected without dynamic register indexing)
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    hc[k] = c == 0 ? H[k][0] : c == 1 ? H[k][1] : H[k][2];
    hr[k] = r == 0 ? H[0][k] : r == 1 ? H[1][k] : H[2][k];
  }
  double hcc[3];   // row c of H
#pragma unroll
  for (int k = 0; k < 3; ++k) hcc[k] = c == 0 ? H[0][k] : c == 1 ? H[1][k] : H[2][k];
  const double b0 = Bm[3 * r + c];
  const double b1 = Bm[3 * r + 0] * hc[0] + Bm[3 * r + 1] * hc[1] + Bm[3 * r + 2] * hc[2];
  double b2 = 0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double HB = hr[0] * Bm[0 * 3 + k] + hr[1] * Bm[1 * 3 + k] + hr[2] * Bm[2 * 3 + k];
    b2 += HB * hcc[k];
  }
  return blk == 0 ? b0 : blk == 1 ? b1 : b2;
}

// Every table the loops read is staged here: a global load inside the node loops would share
// the vector-memory counter with the prefetched wave-table loads and force them to drain.
__host__ __device__ inline size_t solve_lds_smem(int nn, int nm, int NB, int LT = kLT, bool ser = false, int NP = 1) {
  const int LW = LT / 64;
  return sizeof(double) * ((size_t)(NP == 1 ? 12 * LT * NB : 0)   // XiLast [6][512 NB] complex (one pass)
                           + (size_t)(ser && nn * 3 * LW < 27 ? 27 : nn * 3 * LW)   // per-wave node sums (SER: >= 27 entries)
                           + (ser ? (size_t)0 : (size_t)nn * 36)   // per-node B_drag contributions
                           + (size_t)nn * 9           // Bmat
                           + (size_t)nn * 6           // member-factored drag coefficients (stride 6: 16-B rows)
                           + (size_t)nn               // node axial coordinate t
                           + (size_t)nm * 18          // member cq, c1, c2
                           + (size_t)2 * LT * NB * NP   // w and zeta per (padded) bin
                           + 36 + 108 + LW * 6 + 36  // B_drag, M|B|C image, std partials, B_lin+B_drag
                           + LW)                     // convergence-margin partials
         + sizeof(int) * ((size_t)nm + 6);            // member node ranges, vote words, wave counters
}

// LT threads per case: 512 (8 waves), or 256 for nw <= 256 (two cases per CU; C4 has 240 bins),
// or 128 (SER: four cases per CU, B_drag summed node-serially per entry instead of through a
// per-node LDS image, so a workgroup needs about 40 KB of LDS).
// NP > 1 (grids beyond LT NB bins, nw <= 2048): the bins are taken in NP passes of LT NB, and
// XiLast ([6][nw] complex, 192 KB at nw = 2048) no longer fits the LDS: it lives in the case's
// Xi_last block, read and written only by the thread that owns the bin.  Phase A loads a pass's
// XiLast into registers before its node loop (no global load between the ring's wave-table
// loads) and adds each pass's node sums to the LDS partials in pass order; phase C reads and
// writes it around each bin's solve.
template <int NB, int LT = kLT, bool SER = false, int NP = 1>
__global__ __launch_bounds__(LT, LT >= 256 ? 512 / LT : 2) void k_solve_lds(CaseArgs a) {
  constexpr int LW = LT / 64;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wv_s = __builtin_amdgcn_readfirstlane(wv);   // wave index in an SGPR
  PROF_T(tp0);
#ifdef RH_WGTIME
  const unsigned long long wgt0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int slot = xcd_remap(blockIdx.x, a.c.ncase);
  const int ic = a.c.order ? a.c.order[slot] : slot;
#ifdef RH_VARIANTS
  // two-pass launch (a tools/ubench variant, rh_abi.hip): pass 2 runs only the parked cases
  const bool resume = a.resume != 0;
  const int stop_iter = a.stop_iter;
  if (resume && a.o.status[ic] != kCaseStopped) return;   // uniform
#else
  constexpr bool resume = false;
  constexpr int stop_iter = 1 << 30;
#endif
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

  constexpr int NWP = LT * NB;                    // padded bins of one pass
  constexpr int NBT = NB * NP;                     // bins per thread over all passes
  constexpr bool GX = NP > 1;                      // XiLast in the Xi_last block, not in LDS
  constexpr int kRingA = GX ? 3 : kRingA1;
  // PSD / RAO / RMS sums formed in phase C (RH_STATS_C) by the 512-thread kernels; the SER
  // kernels (C4's fixed point: no response output) keep them in the epilogue
  constexpr bool kStatsC = RH_STATS_C && (XI_STORE_MODE == 1) && !SER && NB > 1;
#if RH_OVERLAP && !defined(RH_VARIANTS)
  constexpr bool kOv = !GX;                        // the vote deferred into the next phase A (below)
#else
  constexpr bool kOv = false;                      // (variants: the two-pass launch stops mid-loop)
#endif
  auto wave_maxes = [&](const double* m) {         // max of the per-wave convergence-margin partials
    double mx = m[0];
    for (int w = 1; w < LW; ++w) mx = fmax(mx, m[w]);
    return mx;
  };
  cd* xl = reinterpret_cast<cd*>(smem);            // [6][NWP] (one pass only)
  rh_c128* XL = a.o.Xi_last + c6;                  // [6][nw] (GX)
  // The member factors and the node coefficients, read at every member change and node step of
  // the loops, come first, member- / node-major with 16-byte rows (a member's 18 factors are
  // 9 ds_read_b128 at one base address instead of 18 scattered reads at nm-strided addresses).
  double* mbf = smem + (GX ? 0 : 12 * NWP);        // [nm][18] cq, c1, c2
  double* al = mbf + 18 * nm;                      // [nn][6] (5 used)
  double* red = al + 6 * nn;                       // [nn*3][LW]
  double* bm = red + (SER && nn * 3 * LW < 27 ? 27 : nn * 3 * LW);   // [nn][9]
  double* bd = bm + nn * 9;                        // [36]
  double* mbc = bd + 36;                           // [108] M, B_lin, C
  double* sred = mbc + 108;                        // [LW][6]
  double* bsum = sred + LW * 6;                   // [36] B_lin + B_drag of this iteration
  double* bdn = bsum + 36;                         // [36][nn] (not with SER)
  double* nt = bdn + (SER ? 0 : 36 * nn);          // [nn]
  double* lw = nt + nn;                            // [NP NWP] w per bin (pad bins: w[nw-1])
  double* lz = lw + NP * NWP;                      // [NP NWP] zeta per bin (pad bins: 0)
  double* mred = lz + NP * NWP;                    // [LW] per-wave max of tolCheck
  int* mstart = reinterpret_cast<int*>(mred + LW);  // [nm+1]
  int* sflag = mstart + nm + 1;                      // [2] vote words of even / odd iterations,
                                                     // [2]: it + 1 once a test of iteration it failed,
                                                     // [3 + (it & 1)]: waves done with phase C of iteration it
  load_mbc(d, mbc, tid);
  for (int n = tid; n < nn; n += LT) nt[n] = node[RH_NF_T * nn + n];
  for (int e = tid; e < 18 * nm; e += LT) mbf[e] = d.memb[(e % 18) * nm + e / 18];   // RH_MF_CQ0..C20: fields 0..17
  for (int e = tid; e <= nm; e += LT) mstart[e] = d.mstart[e];
  if (tid < 5) sflag[tid] = 0;
  const int it0 = resume ? stop_iter : a.c.first_iter;
  // Iteration 0's phase-A sums formed for the whole batch by k_a0_sums (rh_a0.hip): their
  // chunk sums (in chunk order) take the place of wave 0's partials and the other waves' are 0,
  // so phase B's wave-order sum returns them unchanged; phase A of that iteration is skipped.
  // (Read before the prologue: with GX the same Xi_last block then receives XiLast.)
#ifdef RH_VARIANTS
  bool skip_a = a.a0 != 0 && it0 == 0;   // uniform
#else
  constexpr bool skip_a = false;         // k_a0_sums is a variant kernel (tools/ubench/variants_src/rh_a0.hip)
#endif
  if (skip_a) {
#ifdef RH_VARIANTS
    const double* a0s = a0_block(a, ic, nw);
    const int nch = a0_chunks(nw);
    for (int e = tid; e < nn * 3; e += LT) {
      double s = 0;
      for (int ch = 0; ch < nch; ++ch) s += a0s[(size_t)ch * 3 * nn + e];
      red[e * LW] = s;
#pragma unroll
      for (int w = 1; w < LW; ++w) red[e * LW + w] = 0.0;
    }
    __syncthreads();
#endif
  }

  // Per-bin scalars live in LDS, not in registers: nothing per-thread stays live across the
  // phases, so the register-heavy solve of phase C does not push other values to scratch.
  // Bin j of this thread is b = tid + LT j; loads use the clamped bin min(b, nw-1) so no
  // load is predicated, and pad bins (b >= nw) carry zeta = 0 and XiLast = 0.
  auto voff = [&](int b) { return (unsigned)(b < nw ? b : nw - 1) * 16u; };
  {
    const int spec = a.c.spectrum[ic];
    const double Hs = a.c.Hs[ic], Tp = a.c.Tp[ic], gam = a.c.gamma[ic];
    const rh_c128* XI0 = resume ? a.o.Xi_last + c6 : a.c.Xi_init ? a.c.Xi_init + c6 : nullptr;
    // (the loads first, then the spectrum from LDS: a loop that both loads and evaluates the
    // spectrum's transcendentals keeps scratch stores beside its loads under the max-ilp scheduler)
#pragma unroll
    for (int j = 0; j < NBT; ++j) {
      const int b = tid + LT * j;
      const bool okb = b < nw;
      lw[b] = d.w[okb ? b : nw - 1];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const cd x0 = okb ? (XI0 ? ld(XI0 + c * nw + b) : mk(a.c.XiStart, 0.0)) : mk(0.0, 0.0);
        if constexpr (GX) {
          if (okb && !resume) st(XL + c * nw + b, x0);
        } else {
          xl[c * NWP + b] = x0;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NBT; ++j) {   // the thread reads back only its own bins: no barrier
      const int b = tid + LT * j;
      const bool okb = b < nw;
      const double zz = sea_amplitude(spec, Hs, Tp, gam, lw[b], d.dw);
      lz[b] = okb ? zz : 0.0;
      if (okb && a.o.zeta) a.o.zeta[(size_t)ic * nw + b] = zz;
    }
  }
  rh_c128* Xo = a.o.Xi ? a.o.Xi + c6 : nullptr;   // NULL: the caller wants no response (C4 fixed point)
  rh_c128* XP = a.o.Xi_prev ? a.o.Xi_prev + c6 : nullptr;
  const double rho = d.rho;
  const int nloop = a.c.nIter + 1;
  const double tol = a.c.tol;
  int status = RH_CASE_NOT_CONVERGED, iters = nloop;
  // closest call of the convergence test (rh_solve_out.margin); pass 2 continues pass 1's
  double margin = resume && a.o.margin ? a.o.margin[ic] : INFINITY;
  const int itend = resume || stop_iter >= nloop ? nloop : stop_iter;
  __syncthreads();
  PROF_T(tp1);
  PROF_ADD(0, tp1 - tp0);

  // The excitation of bin j of this thread with the current node coefficients (al, written by
  // phase B), member-factored (drag_exc_members' arithmetic):
  //   f_n = Bmat_n uhat_n = aq q Kq + a1 p1 K1 + a2 p2 K2,  r_n x f_n = rA x f_n + t q x f_n
  // with q x p1 = p2, q x p2 = -p1 (raft/raft_fowt.py:1255-1259, 1283-1289), then
  // F = zeta (F_iner + F_drag) (+ fext), phase C of every iteration.
  auto excite = [&](int bj, cd (&F)[6]) {
    const unsigned vj = voff(bj);
    const bool okj = bj < nw;
    cd fe[6];   // unit inertial excitation of this bin, in flight during the node loop
#pragma unroll
    for (int c = 0; c < 6; ++c) fe[c] = bld(bFe, vj, c * nw16);
#pragma unroll
    for (int c = 0; c < 6; ++c) F[c] = mk(0, 0);
    {
      cd SQ = mk(0, 0), S1 = mk(0, 0), S2 = mk(0, 0), T1 = mk(0, 0), T2 = mk(0, 0);
      auto load1 = [&](cd (&K)[3], int n) {
        const unsigned so = (unsigned)(n < nn ? n : nn - 1) * 3u * nw16;
#if RH_ABL_C_NOLOAD
        if (n >= kRingC) return;
#endif
#pragma unroll
        for (int p = 0; p < 3; ++p) K[p] = bld(bK, vj, so + (unsigned)p * nw16);
      };
      int m = 0, mnext = nn > 0 ? mstart[1] : 0;
      auto fold = [&]() {   // close member m: F += sum of its nodes (as drag_exc_members)
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          const double cq = mbf[18 * m + RH_MF_CQ0 + i], c1 = mbf[18 * m + RH_MF_C10 + i],
                       c2 = mbf[18 * m + RH_MF_C20 + i];
          F[i] = add(F[i], add(add(scl(SQ, cq), scl(S1, c1)), scl(S2, c2)));
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const double p1 = mbf[18 * m + RH_MF_C10 + i], p2 = mbf[18 * m + RH_MF_C20 + i];
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
        const double* A = al + 6 * n;
        const double A0 = A[0], A1 = A[1], A2 = A[2], A3 = A[3], A4 = A[4];
#if RH_ABL_C_NOCOMP
        SQ = add(SQ, K[0]); S1 = add(S1, K[1]); S2 = add(S2, K[2]);
        load1(K, n + kRingC);
        return;
#endif
        SQ = add(SQ, scl(K[0], A0));
        S1 = add(S1, scl(K[1], A1));
        S2 = add(S2, scl(K[2], A2));
        T1 = add(T1, scl(K[1], A3));
        T2 = add(T2, scl(K[2], A4));
        load1(K, n + kRingC);
      };
      cd K[kRingC][3];
#pragma unroll
      for (int r = 0; r < kRingC; ++r) load1(K[r], r);
      for (int n = 0; n < nn; n += kRingC) {
#pragma unroll
        for (int r = 0; r < kRingC; ++r)
          if (n + r < nn) step(K[r], n + r);
      }
      if (nn > 0) fold();
    }
    const double z = lz[bj];
#pragma unroll
    for (int c = 0; c < 6; ++c) F[c] = add(scl(fe[c], z), scl(F[c], z));   // F_lin + F_drag
    if (has_fx) {
      cd fx[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) fx[c] = bld(bFx, vj, c * nw16);
#pragma unroll
      for (int c = 0; c < 6; ++c) F[c] = add(F[c], mk(okj ? fx[c].r : 0.0, okj ? fx[c].i : 0.0));
    }
  };

  const double hdw = 0.5 / d.dw;   // psd = |x|^2 hdw and rao = x (1 / zeta): multiplies, not 36 divisions per thread
  for (int it = it0; it < itend; ++it) {
    PROF_T(ta0);
    PROF_ADD(7, 1);
    // ---------------- A: per-node sums of squared relative-velocity components ----------
    // Member-factored (rh_member_field): per (member, bin)
    //   Bq = iw cq.Xi, B1 = iw c1.Xi, B2 = iw c2.Xi, E1 = iw p2.th, E2 = -iw p1.th
    // and per node s_q = z Kq - Bq, s_1 = z K1 - (B1 + t E1), s_2 = z K2 - (B2 + t E2)
    // (raft/raft_fowt.py:1205-1211).
#pragma unroll 1
    for (int p = 0; p < NP; ++p) {   // passes of NWP bins (NP == 1: the whole grid)
      const int pb = tid + NWP * p;  // this thread's first bin of the pass
      unsigned vb[NB];
      double bz[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        vb[j] = voff(pb + LT * j);
        bz[j] = lz[pb + LT * j];
      }
      cd XR[GX ? NB : 1][6];         // GX: the pass's XiLast, loaded before the node loop
      if constexpr (GX) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int b = pb + LT * j, bc = b < nw ? b : nw - 1;
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            const cd v = ld(XL + c * nw + bc);
            XR[j][c] = b < nw ? v : mk(0.0, 0.0);
          }
        }
      }
      // (defined here, not just before their first use: left undefined, the register allocator
      // may keep the previous iteration's values live, and spill them, across phase C)
      cd Bq[NB], B1[NB], B2[NB], E1[NB], E2[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) Bq[j] = B1[j] = B2[j] = E1[j] = E2[j] = mk(0.0, 0.0);
      auto member_terms = [&](int m) {
        double cq[6], c1[6], c2[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          cq[i] = mbf[18 * m + RH_MF_CQ0 + i];
          c1[i] = mbf[18 * m + RH_MF_C10 + i];
          c2[i] = mbf[18 * m + RH_MF_C20 + i];
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int b = pb + LT * j;
          cd X[6];
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            if constexpr (GX) X[c] = XR[j][c];
            else X[c] = xl[c * NWP + b];
          }
          cd Aq = mk(0, 0), A1 = mk(0, 0), A2 = mk(0, 0);
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            Aq = add(Aq, scl(X[c], cq[c]));
            A1 = add(A1, scl(X[c], c1[c]));
            A2 = add(A2, scl(X[c], c2[c]));
          }
          const cd D1 = add(add(scl(X[3], c2[0]), scl(X[4], c2[1])), scl(X[5], c2[2]));   // p2 . th
          const cd D2 = add(add(scl(X[3], c1[0]), scl(X[4], c1[1])), scl(X[5], c1[2]));   // p1 . th
          const double w = lw[b];
          Bq[j] = iw(w, Aq);
          B1[j] = iw(w, A1);
          B2[j] = iw(w, A2);
          E1[j] = iw(w, D1);
          E2[j] = iw(-w, D2);
        }
      };
      auto load_node = [&](cd (&K)[3][NB], int n) {
        const unsigned so = (unsigned)(n < nn ? n : nn - 1) * 3u * nw16;
#if RH_ABL_A_NOLOAD   // timing ablation: the ring keeps its first nodes (wrong results)
        if (n >= kRingA) return;
#endif
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int p = 0; p < 3; ++p) K[p][j] = bld(bK, vb[j], so + (unsigned)p * nw16);
      };
      // this lane's partial sums over its bins of |s_q|^2, |s_1|^2, |s_2|^2 for one node
      auto node_sums = [&](const cd (&K)[3][NB], int n, double& s0, double& s1, double& s2) {
        const double t = nt[n];
        s0 = s1 = s2 = 0;
#if RH_ABL_A_NOCOMP   // timing ablation: consume the loads with one add each (wrong results)
#pragma unroll
        for (int j = 0; j < NB; ++j) { s0 += K[0][j].r + K[0][j].i; s1 += K[1][j].r + K[1][j].i; s2 += K[2][j].r + K[2][j].i; }
        return;
#endif
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const double z = bz[j];
          const cd sq = sub(scl(K[0][j], z), Bq[j]);
          const cd sp1 = sub(scl(K[1][j], z), add(B1[j], scl(E1[j], t)));
          const cd sp2 = sub(scl(K[2][j], z), add(B2[j], scl(E2[j], t)));
          s0 += abs2(sq);
          s1 += abs2(sp1);
          s2 += abs2(sp2);
        }
      };
      if constexpr (RH_A_BATCH > 0 && !GX) {
      // Nodes in batches of kB (= the ring depth): the three sums of each node of a batch are
      // independent chains, and the 3 kB values are reduced over the wave by ONE transposing
      // butterfly (tbfly16: 17 exchange steps for up to 16 values, against 8 per node for
      // tbfly3); lanes 0..15 then hold the totals.  The ring slot of node n is refilled with
      // node n + kB as soon as n is summed.
      constexpr int kB = RH_A_BATCH > 0 ? RH_A_BATCH : 1;
      static_assert(3 * kB <= 16, "tbfly16 reduces at most 16 values");
      cd K[kB][3][NB];
#pragma unroll
      for (int r = 0; r < kB; ++r) load_node(K[r], r);
      int m = -1, mnext = 0;
      for (int n = 0; n < nn; n += kB) {
        double u[16];
#pragma unroll
        for (int r = 0; r < kB; ++r) {
          const int nr = n + r;
          if (nr < nn) {
            if (nr == mnext) {   // uniform: entering member m+1 (members are node-contiguous)
              do { ++m; mnext = mstart[m + 1]; } while (mnext == nr);
              member_terms(m);
            }
            node_sums(K[r], nr, u[3 * r], u[3 * r + 1], u[3 * r + 2]);
            load_node(K[r], nr + kB);
          } else {
            u[3 * r] = u[3 * r + 1] = u[3 * r + 2] = 0.0;
          }
        }
#pragma unroll
        for (int v = 3 * kB; v < 16; ++v) u[v] = 0.0;
        const int ln = lane_here();
        const double tot = tbfly16(u, ln);
        const int vi = tbfly16_index(ln);
        if (ln < 16 && vi < 3 * kB && n + vi / 3 < nn) red[((n + vi / 3) * 3 + vi % 3) * LW + wv_s] = tot;
      }
      } else {
      // the three sums of a node are reduced over the wave together (tbfly3); lane k < 3
      // writes sum k.  The ring slot of node n is refilled with node n + kRingA.
      cd K[kRingA][3][NB];
#pragma unroll
      for (int r = 0; r < kRingA; ++r) load_node(K[r], r);
      int m = -1, mnext = 0;
      const int nA = skip_a ? 0 : nn;   // no node steps when iteration 0's sums came from k_a0_sums
      // RH_A_PAIR: the sums of nodes 2k and 2k + 1 reduced together (tbfly6; even ring depth)
      constexpr bool kPair = RH_A_PAIR && (kRingA % 2 == 0);
      double h0 = 0.0, h1 = 0.0, h2 = 0.0;   // (kPair) the even node's sums
      // (kPair) the butterfly's lane flags: formed here, live through the node loop only
      // (lane_here is not hoisted out of the iteration loop)
      const Bfly6 bl = bfly6_lane(kPair ? lane_here() : 0);
      for (int n = 0; n < nA; n += kRingA) {
#pragma unroll
        for (int r = 0; r < kRingA; ++r) {
          const int nr = n + r;
          if (nr < nA) {
            if (nr == mnext) {   // uniform: entering member m+1 (members are node-contiguous)
              do { ++m; mnext = mstart[m + 1]; } while (mnext == nr);
              member_terms(m);
            }
            double s0, s1, s2;
            node_sums(K[r], nr, s0, s1, s2);
            load_node(K[r], nr + kRingA);
            if constexpr (kPair) {
              if ((r & 1) == 0 && nr + 1 < nA) {   // uniform: held for the odd node
                h0 = s0; h1 = s1; h2 = s2;
                continue;
              }
              const int n0 = (r & 1) ? nr - 1 : nr;   // the pair's even node
              const double tot = (r & 1) ? tbfly6(h0, h1, h2, s0, s1, s2, bl)
                                         : tbfly6(s0, s1, s2, 0.0, 0.0, 0.0, bl);   // the last node alone
              if ((r & 1) ? bl.vi >= 0 : (unsigned)bl.vi < 3u) {
                double& rr = red[(n0 * 3 + bl.vi) * LW + wv_s];
                rr = (GX && p > 0) ? rr + tot : tot;   // passes add in pass order
              }
              continue;
            }
            const int ln = lane_here();
#if RH_ABL_A_NOBFLY
            const double tot = s0 + s1 + s2;
#else
            const double tot = tbfly3(s0, s1, s2, ln);
#endif
            if (ln < 3) {
              double& r = red[(nr * 3 + tbfly3_index(ln)) * LW + wv_s];
              r = (GX && p > 0) ? r + tot : tot;   // passes add in pass order
            }
          }
        }
      }
      }
    }
#ifdef RH_VARIANTS
    skip_a = false;
#endif
    __syncthreads();
    if constexpr (kOv) {
      // the deferred vote of iteration it - 1 (every wave finished its phase C before this
      // barrier; they came here because some test of it - 1 failed, so it did not converge)
      if (it > it0) {
        const int fl = sflag[(it - 1) & 1];
        if (a.o.margin && tid == 0) margin = closer_call(margin, wave_maxes(mred) - tol);
        if (fl & 6) {
          status = (fl & 2) ? RH_CASE_NAN : RH_CASE_SINGULAR;
          iters = it;
          break;
        }
      }
    }
    PROF_T(ta1);
    PROF_ADD(1, ta1 - ta0);
    // ---------------- B: node drag matrices and B_drag ----------------------------------
    for (int n = tid; n < nn; n += LT) {
      // the node's fields XX .. CIRC and T, all loads issued before any use (left to the
      // scheduler, each load waited on before the next was issued: eight serial L2 round trips)
      double fv[RH_NF_CIRC - RH_NF_XX + 2];
#pragma unroll
      for (int f = RH_NF_XX; f <= RH_NF_CIRC; ++f) fv[f - RH_NF_XX] = node[(size_t)f * nn + n];
      fv[RH_NF_CIRC - RH_NF_XX + 1] = node[(size_t)RH_NF_T * nn + n];
      __builtin_amdgcn_sched_barrier(0);
      auto F = [&](int f) { return f == RH_NF_T ? fv[RH_NF_CIRC - RH_NF_XX + 1] : fv[f - RH_NF_XX]; };
      double r3[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double* R = red + (size_t)(n * 3 + c) * LW;
        double s = 0;
#pragma unroll
        for (int w = 0; w < LW; ++w) s += R[w];
        r3[c] = s;
      }
      // sum|vrel_q|^2 = sum|s_q|^2 |q|^2 ; circular: |vrel_p|^2 = |s_1|^2|p1|^2 + |s_2|^2|p2|^2
      auto n2 = [&](int f) { const double a = F(f), b = F(f + 1), c = F(f + 2); return a * a + b * b + c * c; };
      const double qq = n2(RH_NF_QX), pp1 = n2(RH_NF_P1X), pp2 = n2(RH_NF_P2X);
      const bool circ = F(RH_NF_CIRC) != 0.0;
      const double sums[3] = {r3[0] * qq, circ ? r3[1] * pp1 + r3[2] * pp2 : r3[1] * pp1, r3[2] * pp2};
      double B4[4];
      node_bmat_f(F, rho, sums, bm + 9 * n, B4);
      const double t = F(RH_NF_T);
      double* A = al + 6 * n;
      A[0] = B4[0] + B4[3];     // axial: side + end   (qMat terms of Bmat, raft/raft_fowt.py:1228-1248)
      A[1] = B4[1];
      A[2] = B4[2];
      A[3] = t * B4[1];
      A[4] = t * B4[2];
      if (!SER) {
        // this node's translateMatrix3to6DOF (raft/helpers.py:455-478), summed below in node order
        const double rx = F(RH_NF_XX), ry = F(RH_NF_XY), rz = F(RH_NF_XZ);
#pragma unroll
        for (int e = 0; e < 36; ++e) bdn[e * nn + n] = t3to6(bm + 9 * n, rx, ry, rz, e / 6, e % 6);
      }
    }
    __syncthreads();
    if (SER) {
      // B_drag without the per-node image: the 27 distinct entries of translateMatrix3to6DOF (9 of
      // Bm, 9 of Bm H, 9 of H Bm H^T; the lower-left block is the transpose of the upper-right
      // one) of cn nodes at a time go to the node-sum buffer (free after the Bmat loop above), one
      // thread per node computing them with t3to6's expressions; lane e < 27 then adds entry e of
      // those nodes to its running sum in node order (the same bits as the image path).
      const int cn = (nn * 3 * LW) / 27 > 0 ? (nn * 3 * LW) / 27 : 1;
      double se = 0.0;
      for (int n0 = 0; n0 < nn; n0 += cn) {
        const int cnt = nn - n0 < cn ? nn - n0 : cn;
        for (int nl = tid; nl < cnt; nl += LT) {   // one node per thread: its 27 entries share the loads
          const int n = n0 + nl;
          const double rx = nf(node, nn, RH_NF_XX, n), ry = nf(node, nn, RH_NF_XY, n), rz = nf(node, nn, RH_NF_XZ, n);
          double Bn[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) Bn[k] = bm[9 * n + k];
#pragma unroll
          for (int e = 0; e < 27; ++e) red[27 * nl + e] = t3to6_block(Bn, rx, ry, rz, e / 9, (e % 9) / 3, e % 3);
        }
        __syncthreads();
        if (tid < 27)
          for (int k = 0; k < cnt; ++k) se += red[27 * k + tid];
        __syncthreads();
      }
      if (tid < 27) {
        const int blk = tid / 9, r = (tid % 9) / 3, c = tid % 3;
        if (blk == 0) bd[6 * r + c] = se;
        else if (blk == 1) bd[6 * r + 3 + c] = bd[6 * (3 + c) + r] = se;
        else bd[6 * (3 + r) + 3 + c] = se;
      }
      __syncthreads();
      if (tid < 36) bsum[tid] = mbc[36 + tid] + bd[tid];
    } else if (tid < 36) {
      double s = 0;
      const double* P = bdn + tid * nn;
      for (int n = 0; n < nn; ++n) s += P[n];
      bd[tid] = s;
      bsum[tid] = mbc[36 + tid] + s;   // the B_lin + B_drag of every bin's Z (same sum as before)
    }
    __syncthreads();
    PROF_T(ta2);
    PROF_ADD(2, ta2 - ta0 - (ta1 - ta0));
#ifdef RH_PROF
    unsigned long long tc_exc = 0, tc_sol = 0, tc_z = 0, tc_lu = 0;
#endif
    // ---------------- C: excitation, Z(w), LU solve, convergence flags ------------------
    bool my_ok = true, my_nan = false, my_sing = false;
    double tN = 0.0, tD = 1.0;   // the lane's largest tolCheck so far as tt^2 = tN / tD
    // the last allowed iteration stores every entry of the unrelaxed iterate (uniform)
    const bool last_it = __builtin_amdgcn_readfirstlane(it + 1 == nloop ? 1 : 0) != 0;
    // The outputs of the final iteration (Xi, F_wave) are stored by every iteration that may be
    // the final one: the last allowed, or one whose tests have all passed so far.  A wave that
    // sees a failed test (any lane, this bin or an earlier one) marks the iteration in LDS
    // (sflag[2]); the other waves read the mark at their next store (a stale read only stores
    // more).  (uniform)
    auto may_be_final = [&]() -> bool {
      if (last_it) return true;
      if (__builtin_amdgcn_ballot_w64(!my_ok)) {
        if (lane == 0) __hip_atomic_store(&sflag[2], it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return false;
      }
      return __builtin_amdgcn_readfirstlane(__hip_atomic_load(&sflag[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != it + 1;
    };
    if constexpr (kStatsC)
      if (lane < 6) sred[wv * 6 + lane] = 0.0;   // this wave's RMS sums: only the final iteration's are kept
    if constexpr (kOv) {
      // the words of iteration it + 1: their last readers (iteration it - 1's vote) are done
      if (tid == 0) {
        sflag[(it + 1) & 1] = 0;
        sflag[3 + ((it + 1) & 1)] = 0;
      }
    }
#pragma unroll 1
    for (int j = 0; j < NBT; ++j) {
      // per-bin scalars picked without dynamic register indexing (the loop is not unrolled,
      // so only one bin's LU is ever live)
      const int bj = tid + LT * j;
      const bool okj = bj < nw;
      PROF_T(tc0);
      cd F[6];
      excite(bj, F);
      // F_wave: the excitation of the final iteration, which every iteration's overwrites (F is
      // live for the LU anyway), skipped once the iteration is known not to be final (below)
      if (a.o.F_wave && may_be_final()) {
        if (okj) {
#pragma unroll
          for (int c = 0; c < 6; ++c) st_nt(a.o.F_wave + c6 + c * nw + bj, F[c]);
        }
      }
      PROF_T(tc1);
#ifdef RH_PROF
      tc_exc += tc1 - tc0;
#endif
#if RH_LDS_LANE_BRANCH
      if (!okj) continue;
#else
      // No lane branch around the solve (a per-lane `continue` here let the compiler's spills
      // run under a partial EXEC mask in the general kernel): only a wave whose
      // every lane is past the grid skips it (uniform); pad lanes of the last wave solve the
      // clamped last bin with a zero right-hand side (zeta = 0, x = 0 exactly) and store nothing.
      if (!__builtin_amdgcn_ballot_w64(okj)) continue;
#endif
      const int b = bj;
      const double w = lw[b];
      cd Z[6][6];
      {
        // index the LDS image with a zero the compiler cannot see through, so that its 144
        // loop-invariant reads stay here instead of being hoisted into VGPRs for the solve
        const int zo = opaque_zero();
        const double* zm = mbc + zo;
        const double* zb = bd + zo;
        const double* zs = bsum + zo;
        const double w2 = -(w * w);
        if (d.mb_per_bin) {
          const int bc = okj ? b : nw - 1;
          const double* M = d.M + (size_t)bc * 36;
          const double* B = d.B + (size_t)bc * 36;
#pragma unroll
          for (int r = 0; r < 6; ++r) {
#pragma unroll
            for (int c = 0; c < 6; ++c) Z[r][c] = mk(w2 * M[6 * r + c] + zm[72 + 6 * r + c], w * (B[6 * r + c] + zb[6 * r + c]));
            __builtin_amdgcn_sched_barrier(0);   // one row of reads in flight at a time
          }
        } else {
#pragma unroll
          for (int r = 0; r < 6; ++r) {
#pragma unroll
            for (int c = 0; c < 6; ++c)
              Z[r][c] = mk(w2 * zm[6 * r + c] + zm[72 + 6 * r + c], w * zs[6 * r + c]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
#ifdef RH_PROF
      const unsigned long long tcz = clock64();
      tc_z += tcz - tc1;
#endif
      const bool ok_lu = lu_solve<6>(Z, F);
      my_sing |= okj && !ok_lu;
#ifdef RH_PROF
      tc_lu += clock64() - tcz;
#endif
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const cd x = F[c];
        cd xlast;
        if constexpr (GX) {
          const cd v = ld(XL + c * nw + (okj ? b : nw - 1));
          xlast = okj ? v : mk(0.0, 0.0);
        } else {
          xlast = xl[c * NWP + b];
        }
        my_nan |= okj && ((x.r != x.r) || (x.i != x.i));
        // tolCheck = |Xi - XiLast| / (|Xi| + tol) < tol  (raft/raft_model.py:961-962)
        // (magnitudes as sqrt(re^2 + im^2): within an ulp of np.abs's hypot, far cheaper)
        // tt < tol as |Xi - XiLast|^2 < (tol (|Xi| + tol))^2: one square root, no division per
        // entry; the lane keeps its largest tt^2 as a fraction (compared by cross products) and
        // forms tt itself only for the convergence margin, once per iteration
        const double n2 = abs2(sub(x, xlast)), den = sqrt(abs2(x)) + tol, d2 = den * den;
        const double td = tol * den;
        my_ok = my_ok && (!okj || n2 < td * td);
        const bool gt = okj && n2 * tD > tN * d2;
        tN = gt ? n2 : tN;
        tD = gt ? d2 : tD;
        [[maybe_unused]] const bool pass = n2 < td * td;
#if RH_XI_STORE == 0
        // (round 4: an entry stored whenever it passed its own test or at the last iteration)
        if (okj && (GX || Xo) && (pass || last_it)) st_nt(Xo + c * nw + b, x);
#elif RH_XI_STORE == 2
        if (okj && (GX || Xo) && last_it) st_nt(Xo + c * nw + b, x);   // traffic floor (A/B only: wrong Xi)
#endif
        if (okj && XP) st(XP + c * nw + b, xlast);
        // XiLast = 0.2 XiLast + 0.8 Xi  (:991), only consumed if not converged (pads: 0)
        const cd xr = add(scl(xlast, 0.2), scl(x, 0.8));
        if constexpr (GX) {
          if (okj) st(XL + c * nw + b, xr);
        } else {
          xl[c * NWP + b] = xr;
        }
      }
#if RH_XI_STORE == 1
      // The unrelaxed iterate leaves the kernel only as the output of the case's final
      // iteration: the one whose test every (bin, DOF) passed, or the last allowed one
      // (raft/raft_model.py:996-1000).  So the bin's six entries are stored only while this
      // iteration may still be that one (may_be_final, with this bin's tests counted);
      // streamed: the final iteration's stores are the ones kept.  (Xi may be NULL with NP == 1.)
      if ((GX || Xo) && may_be_final()) {
        if constexpr (kStatsC) {
          // PSD, RAO and the RMS sums from x in registers (the epilogue's arithmetic,
          // k_motion_stats with one row): the final iteration's values are the ones kept, and
          // nothing is read back
          const double z = lz[b];
          const double rz = fabs(z) > 1e-6 ? 1.0 / z : 0.0;
          double m2v[6];
#pragma unroll
          for (int c = 0; c < 6; ++c) m2v[c] = okj ? abs2(c >= 3 ? scl(F[c], kRad2Deg) : F[c]) : 0.0;
          if (okj) {
#pragma unroll
            for (int c = 0; c < 6; ++c) {
              st_nt(Xo + c * nw + b, F[c]);
              if (a.o.psd) __builtin_nontemporal_store(m2v[c] * hdw, a.o.psd + ((size_t)ic * 6 + c) * nw + b);
              if (a.o.rao) st_nt(a.o.rao + ((size_t)ic * 6 + c) * nw + b, scl(F[c], rz));
            }
          }
          if (a.o.std) {   // the bin's six sums over the wave by two transposing butterflies
            const int ln = lane_here();
            const double t0 = tbfly3(m2v[0], m2v[1], m2v[2], ln), t1 = tbfly3(m2v[3], m2v[4], m2v[5], ln);
            if (ln < 3) {
              const int k = tbfly3_index(ln);
              sred[wv * 6 + k] += t0;
              sred[wv * 6 + 3 + k] += t1;
            }
          }
        } else if (okj) {
#pragma unroll
          for (int c = 0; c < 6; ++c) st_nt(Xo + c * nw + b, F[c]);
        }
      }
#endif
#ifdef RH_PROF
      tc_sol += clock64() - tc1;
#endif
    }
    PROF_ADD(3, tc_exc);
    PROF_ADD(4, tc_sol);
    PROF_ADD(8, tc_z);
    PROF_ADD(9, tc_lu);
    PROF_T(ta3);
    if (a.o.margin) {
      const double my_tmax = sqrt(tN) / sqrt(tD);
      const double mw = wave_max(my_tmax);
      if (lane == 0) mred[wv] = mw;
    }
    if constexpr (kOv) {
      // No barrier here.  Each wave ORs its flag bits (1 = a bin not converged, 2 = NaN,
      // 4 = singular) into this iteration's word and counts itself done (release: the bits, the
      // mark and mred first).  A wave that knows the loop goes on (one of its own tests failed,
      // or another wave's mark) starts the next phase A at once, overlapping the waves still in
      // phase C: phase A reads only the XiLast entries this very thread wrote, and writes only
      // the node partials, which phase B consumed before this iteration's phase C.  The vote is
      // then read after the next phase-A barrier (above).  Otherwise the wave waits for every
      // wave to be done or for a mark, whichever comes first; with all done and no mark the
      // iteration is the final one, the same verdict for every wave (a mark is written before
      // its wave's done count).  The last allowed iteration always waits for all.
      const bool last = it + 1 == nloop;
      const unsigned long long bn = __builtin_amdgcn_ballot_w64(!my_ok), bx = __builtin_amdgcn_ballot_w64(my_nan),
                               bs = __builtin_amdgcn_ballot_w64(my_sing);
      const int bits = (bn ? 1 : 0) | (bx ? 2 : 0) | (bs ? 4 : 0);
      if (lane == 0) {
        if (bits) __hip_atomic_fetch_or(&sflag[it & 1], bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (bn) __hip_atomic_store(&sflag[2], it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&sflag[3 + (it & 1)], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      bool go_on = !last && bn != 0;
      if (!go_on) {
#pragma unroll 1
        while (true) {
          const int dn = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(&sflag[3 + (it & 1)], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
          const int mk = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(&sflag[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          if (!last && mk == it + 1) {
            go_on = true;
            break;
          }
          if (dn == LW) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      PROF_T(ta4);
      PROF_ADD(5, ta4 - ta3);
      if (go_on) continue;
      // the final iteration: every wave is done and no test failed (or it was the last allowed)
      const int fl = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(&sflag[it & 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
      if (a.o.margin && tid == 0) margin = closer_call(margin, wave_maxes(mred) - tol);
      status = (fl & 2) ? RH_CASE_NAN : (fl & 4) ? RH_CASE_SINGULAR : (fl & 1) ? RH_CASE_NOT_CONVERGED : RH_CASE_CONVERGED;
      iters = it + 1;
      break;
    } else {
#if RH_ONE_VOTE
    // One barrier for the three votes: each wave ORs its flag bits (1 = a bin not converged,
    // 2 = NaN, 4 = singular) into this iteration's LDS word; tid 0 clears the other word for
    // the next iteration (everyone has read it: it was last read before this iteration's
    // phase-A barrier).
    {
      const unsigned long long bn = __builtin_amdgcn_ballot_w64(!my_ok), bx = __builtin_amdgcn_ballot_w64(my_nan),
                               bs = __builtin_amdgcn_ballot_w64(my_sing);
      const int bits = (bn ? 1 : 0) | (bx ? 2 : 0) | (bs ? 4 : 0);
      if (lane == 0 && bits) atomicOr(&sflag[it & 1], bits);
    }
    __syncthreads();
    const int fl = sflag[it & 1];
    if (tid == 0) sflag[(it + 1) & 1] = 0;
    const int all_ok = !(fl & 1), any_nan = fl & 2, any_sing = fl & 4;
    if (a.o.margin && tid == 0) {   // mred is rewritten only after the next phase-A barrier
      double mx = mred[0];
      for (int w = 1; w < LW; ++w) mx = fmax(mx, mred[w]);
      margin = closer_call(margin, mx - tol);
    }
#else
    const int all_ok = __syncthreads_and(my_ok ? 1 : 0);
    if (a.o.margin && tid == 0) {   // mred is rewritten only after the next phase-A barrier
      double mx = mred[0];
      for (int w = 1; w < LW; ++w) mx = fmax(mx, mred[w]);
      margin = closer_call(margin, mx - tol);
    }
    const int any_nan = __syncthreads_or(my_nan ? 1 : 0);
    const int any_sing = __syncthreads_or(my_sing ? 1 : 0);
#endif
    PROF_T(ta4);
    PROF_ADD(5, ta4 - ta3);
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
  }

  if (status == RH_CASE_NOT_CONVERGED && itend < nloop) {
    // pass 1 stops here: park the relaxed iterate (the next iteration's XiLast) and the margin
    // so far; pass 2 continues the case from iteration itend with the same bits
#pragma unroll 1
    for (int j = 0; j < NB && !GX; ++j) {   // (GX: XiLast is already in Xi_last)
      const int b = tid + LT * j;
      if (b >= nw) continue;
#pragma unroll 1
      for (int c = 0; c < 6; ++c) st(a.o.Xi_last + c6 + c * nw + b, xl[c * NWP + b]);
    }
    if (tid == 0) {
      a.o.status[ic] = kCaseStopped;
      if (a.o.margin) a.o.margin[ic] = margin;
    }
    return;
  }

  // ---------------- outputs ------------------------------------------------------------
#ifdef RH_WGTIME
  if (tid == 0 && blockIdx.x < 8192) {
    rh_wgt[2 * blockIdx.x] = wgt0;
    rh_wgt[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  PROF_T(te0);
  if (tid == 0) {
    a.o.iters[ic] = iters;
    a.o.status[ic] = status;
    if (a.o.margin) a.o.margin[ic] = margin;
  }
  if (a.o.B_drag && tid < 36) a.o.B_drag[(size_t)ic * 36 + tid] = bd[tid];
  if (a.o.Bmat)
    for (int e = tid; e < nn * 9; e += LT) a.o.Bmat[(size_t)ic * a.bmat_nn * 9 + e] = bm[e];
  if (a.o.Z) {   // final impedance fowt.Z (raft/raft_model.py:1013) from the last B_drag, streamed
#pragma unroll 1
    for (int j = 0; j < NBT; ++j) {
      const int b = tid + LT * j;
      if (b >= nw) continue;
      const double w = lw[b], w2 = -(w * w);
      rh_c128* Zo = a.o.Z + ((size_t)ic * nw + b) * 36;
#pragma unroll 1
      for (int e = 0; e < 36; ++e) {
        const double M = d.mb_per_bin ? d.M[(size_t)b * 36 + e] : mbc[e];
        const double B = d.mb_per_bin ? d.B[(size_t)b * 36 + e] : mbc[36 + e];
        st(Zo + e, mk(w2 * M + mbc[72 + e], w * (B + bd[e])));
      }
    }
  }
  // A case that stopped on a NaN or a singular Z has no response (the reference raises there,
  // raft/raft_model.py:957): its Xi, F_wave, PSD, RAO and std are NaN, as in k_solve_cases.  (The
  // entries of its last iterate were stored only where they passed their test.)
  const bool failed = status == RH_CASE_NAN || status == RH_CASE_SINGULAR;   // uniform
  if (failed && a.o.F_wave) {   // nor an excitation: an array solve of it gives NaN, not stale memory
#pragma unroll 1
    for (int j = 0; j < NBT; ++j) {
      const int b = tid + LT * j;
      if (b >= nw) continue;
#pragma unroll
      for (int c = 0; c < 6; ++c) st(a.o.F_wave + ((size_t)ic * 6 + c) * nw + b, mk(NAN, NAN));
    }
  }
  // (kStatsC: phase C formed PSD / RAO / the RMS sums of a case that did not fail)
  double ss[6] = {0, 0, 0, 0, 0, 0};
  if (!kStatsC || failed) {
#pragma unroll
  for (int j = 0; j < NBT; ++j) {
    const int b = tid + LT * j;
    if (b >= nw || !Xo) continue;   // (psd, std and rao need Xi: checked by the caller)
    const double z = lz[b];
    const double rz = fabs(z) > 1e-6 ? 1.0 / z : 0.0;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      cd x;
      if (failed) {
        x = mk(NAN, NAN);
        st(Xo + c * nw + b, x);
      } else {
        x = ld(Xo + c * nw + b);
      }
      const cd xd = c >= 3 ? scl(x, kRad2Deg) : x;
      const double m2 = abs2(xd);
      ss[c] += m2;
      if (a.o.psd) a.o.psd[((size_t)ic * 6 + c) * nw + b] = m2 * hdw;
      if (a.o.rao) st(a.o.rao + ((size_t)ic * 6 + c) * nw + b, failed ? x : scl(x, rz));
    }
  }
  }
  if (a.o.std) {
    if (!kStatsC || failed) {
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const double s = wave_sum(ss[c]);
        if (lane == 0) sred[wv * 6 + c] = s;
      }
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
