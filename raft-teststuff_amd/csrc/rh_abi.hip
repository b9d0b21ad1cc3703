// rh_abi.hip -- the extern "C" boundary of librafthip.so (declared in include/rafthip.h).
//
// Host-side responsibilities only: argument validation, the per-context device copy of
// the design descriptors, kernel configuration and error translation.  No numerics here.
#include <cstdarg>
#include <cstdio>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

#include <unistd.h>
#include <string>
#include <vector>

#include "rh_device.h"

#include "rh_kernels.hip"   // kernels + their host launchers (this translation unit: default scheduler)
#include "rh_qtf.hip"
#include "rh_qtf_mfma.hip"
#include "rh_solve.hip"        // k_solve_lds: only the two-pass <2, 512, false, 2> is instantiated here
#include "rh_solve_launch.h"   // ... the single-pass ones live in rh_solve_fast.hip (max-ilp scheduler)
#ifdef RH_VARIANTS
// Opt-in solve kernels that were measured slower than k_solve_lds on C2: the
// lock-step grouped kernel, the lane-pair kernel and the two-pass launch.  They are not part
// of the shipped library; tools/build_variants.sh builds them for on-box A/B timing.
#include "../../tools/ubench/variants_src/rh_solve_grp.hip"
#include "../../tools/ubench/variants_src/rh_solve_pair.hip"
#include "../../tools/ubench/variants_src/rh_a0.hip"            // k_a0_sums (rh_set_a0)
#include "../../tools/ubench/variants_src/rh_qtf_variants.hip"  // k_qtf_gemm32, k_qtf_lcoef + k_qtf_kay (rh_set_qtf_path 2, 3)
#endif
#ifndef RH_KAY_SPLIT_MAX_TILES
#define RH_KAY_SPLIT_MAX_TILES(ncu) (ncu)   // k_qtf_lk: one wave per part of a member's rows up to this many tiles
#endif
#include "rh_prep.h"       // host-only: native per-design preparation (rh_prep_designs)
#include "rh_qtf_host.h"   // host-only: the static QTF tables of a FOWT (rh_qtf_tables)

// One staging slot of the design descriptor array.  A context cycles through kDescSlots of
// them, so a launch never waits for the descriptors of the previous one: the host blocks only
// when it is kDescSlots launches ahead of the device (a pipelined sweep enqueues a block's
// tables and solve while the previous block still runs, raft/batch.py solve_sweep).
struct rh_desc_slot {
  rh::DevDesign* d = nullptr;   // device copy of the descriptor array
  rh::DevDesign* h = nullptr;   // pinned staging
  int cap = 0;
  hipEvent_t staged = nullptr;  // after the copy out of h
  hipEvent_t used = nullptr;    // after the last kernel that reads d
  int n = 0;                    // descriptors of the last staging into this slot
  hipStream_t stream = nullptr; // ... and the stream its copy ran on
};
constexpr int kDescSlots = 8;

struct rh_ctx {
  int device = 0;
  rh_desc_slot slot[kDescSlots];
  int next = 0;                         // slot of the next staging
  int cur = 0;                          // slot of the last staging
  // tuning / cross-check knobs (per context: the ABI has no mutable process globals)
  bool force_general = false;   // rh_set_solver(ctx, 1): always use k_solve_cases (parity cross-checks)
#ifdef RH_VARIANTS
  bool a0 = false;              // rh_set_a0: iteration-0 phase A of the fast path as a batch GEMM (rh_a0.hip;
                                // measured slower than the per-case phase A)
  bool no_group = false;        // rh_set_solver(ctx, 2): ignore group_start (one case per workgroup)
#ifndef RH_PAIR_ON
#define RH_PAIR_ON 0
#endif
  bool use_pair = RH_PAIR_ON;   // rh_set_solver(ctx, 3): k_solve_pair instead of k_solve_lds (cross-checks)
#ifndef RH_TWO_PASS
#define RH_TWO_PASS 0
#endif
  bool two_pass = RH_TWO_PASS;  // k_solve_lds in two passes when a batch needs more than one round
                                // (rh_set_solver(ctx, 5) on, 4 off; the default is RH_TWO_PASS)
#endif
  int ncu = 0;                  // compute units of the device (rh_ctx_create)
  int qtf_waves = 0;            // rh_set_qtf_waves: waves per 64 QTF pairs in k_qtf_pairs (0 = auto)
  bool qtf_direct = false;      // rh_set_qtf_path(ctx, 1): the per-pair kernel even on a sorted grid
#ifdef RH_VARIANTS
  bool qtf_sep = false;         // rh_set_qtf_path(ctx, 3): k_qtf_lcoef and k_qtf_kay as two launches
  bool qtf_t32 = false;         // rh_set_qtf_path(ctx, 2): 32 x 32 GEMM tiles for a whole QTF
                                // (68.7 vs 57.0 us per C3 QTF)
#endif
  // per-stream scratch of rh_wave_tables (per-node forces, k_wave_tables_nodes ->
  // k_wave_force_sum): one buffer per stream, so stream order alone protects its reuse
  struct Scratch {
    hipStream_t s;
    void* p;
    size_t bytes;
  };
  std::vector<Scratch> wt_scratch;
  std::mutex wt_mu;
};

namespace {
thread_local std::string g_err;
#ifdef RH_VARIANTS
constexpr int kGroupCases = 2;   // lock-step width of k_solve_grp
#else
constexpr int kGroupCases = 1;   // no grouped kernel in the shipped library: group_start is ignored
#endif
#ifndef RH_PAIR_RA
#define RH_PAIR_RA 2
#endif
#ifndef RH_PAIR_RC
#define RH_PAIR_RC 4
#endif
constexpr int kPairRA = RH_PAIR_RA;   // k_solve_pair wave-table prefetch depth, phase A (nodes)
constexpr int kPairRC = RH_PAIR_RC;   // ... phase C
#ifndef RH_PAIR_HOLD
#define RH_PAIR_HOLD 0
#endif
constexpr bool kPairHold = RH_PAIR_HOLD;   // k_solve_pair keeps the unrelaxed iterate in VGPRs
#ifndef RH_PAIR_PB
#define RH_PAIR_PB 2
#endif
constexpr int kPairPB = RH_PAIR_PB;   // bins per lane in phase A at 1024 threads

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define RH_HIP(call)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess) return fail(RH_EHIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

constexpr int kThreads = 256;
constexpr int kMaxNodes = 1024;
constexpr size_t kMaxLds = 160 * 1024;   // LDS per workgroup on gfx950

// need_uhat: the entry point's kernels read the velocity table (the fixed point does not: it
// reads kproj and finer only, so a sweep block may skip uhat, rh_wave_tables_batch)
int check_design(const rh_design& d, bool need_tables, bool need_uhat = true) {
  if (d.nw < 2 || d.nw > 2048) return fail(RH_EINVAL, "nw=%d outside [2, 2048]", d.nw);
  if (d.nn < 0 || d.nn > kMaxNodes) return fail(RH_EINVAL, "nn=%d outside [0, %d]", d.nn, kMaxNodes);
  if (!d.w || !d.k || (d.nn > 0 && !d.node)) return fail(RH_EINVAL, "design: null w/k/node table");
  if (!d.M || !d.B || !d.C) return fail(RH_EINVAL, "design: null M/B/C");
  if (d.nn > 0 && (d.nm < 1 || !d.memb || !d.mstart)) return fail(RH_EINVAL, "design: member table missing");
  if (need_tables && ((need_uhat && !d.uhat) || !d.finer || !d.kproj || d.nhead < 1))
    return fail(RH_EINVAL, "design: wave tables missing (call rh_wave_tables first)");
  if (!(d.dw > 0)) return fail(RH_EINVAL, "design: dw must be > 0");
  return RH_OK;
}

int stage_designs(rh_ctx* ctx, const rh_design* designs, int n, hipStream_t s) {
  {  // the same descriptors as the last staging, on the same stream: its device copy is
     // current and ordered before this call's kernels (a repeated batch, e.g. a timed step)
    const rh_desc_slot& last = ctx->slot[ctx->cur];
    if (last.d && last.n == n && last.stream == s) {
      bool same = true;
      for (int i = 0; i < n && same; ++i) same = std::memcmp(&last.h[i].d, &designs[i], sizeof(rh_design)) == 0;
      if (same) return RH_OK;
    }
  }
  rh_desc_slot& sl = ctx->slot[ctx->next];
  ctx->cur = ctx->next;
  ctx->next = (ctx->next + 1) % kDescSlots;
  if (n > sl.cap) {
    RH_HIP(hipEventSynchronize(sl.staged));
    RH_HIP(hipEventSynchronize(sl.used));   // no kernel reads this slot's old array any more
    if (sl.d) RH_HIP(hipFree(sl.d));
    if (sl.h) RH_HIP(hipHostFree(sl.h));
    sl.d = sl.h = nullptr;
    sl.cap = 0;
    int cap = n < 64 ? 64 : n;
    RH_HIP(hipMalloc(&sl.d, sizeof(rh::DevDesign) * cap));
    RH_HIP(hipHostMalloc(&sl.h, sizeof(rh::DevDesign) * cap, hipHostMallocDefault));
    sl.cap = cap;
  }
  RH_HIP(hipEventSynchronize(sl.staged));  // this slot's previous copy has left the staging buffer
  // the slot's device array may still be read by a kernel of an earlier call on another
  // stream: order the overwrite after it (a no-op on the same stream)
  RH_HIP(hipStreamWaitEvent(s, sl.used, 0));
  // the slot describes no valid device copy until the copy and its event are enqueued: a failure
  // below must not leave new descriptors in h beside a stale (n, stream) that the dedupe trusts
  sl.n = 0;
  sl.stream = nullptr;
  for (int i = 0; i < n; ++i) sl.h[i].d = designs[i];
  RH_HIP(hipMemcpyAsync(sl.d, sl.h, sizeof(rh::DevDesign) * n, hipMemcpyHostToDevice, s));
  RH_HIP(hipEventRecord(sl.staged, s));
  sl.n = n;
  sl.stream = s;
  return RH_OK;
}

// the device descriptor array of the last staging
rh::DevDesign* staged_designs(rh_ctx* ctx) { return ctx->slot[ctx->cur].d; }

// after every launch that reads the staged descriptors
int designs_used(rh_ctx* ctx, hipStream_t s) {
  RH_HIP(hipGetLastError());
  RH_HIP(hipEventRecord(ctx->slot[ctx->cur].used, s));
  return RH_OK;
}

int nb_for(int nw) {
  if (nw <= 256) return 1;
  if (nw <= 512) return 2;
  if (nw <= 1024) return 4;
  return 8;
}
}  // namespace

extern "C" {

const char* rh_last_error(void) { return g_err.c_str(); }

int rh_version(void) { return 7; }

// (rh_prof_read / rh_wgt_read of instrumented builds live in rh_solve_fast.hip, beside the counters)

int rh_set_solver(rh_ctx* ctx, int which) {
  if (!ctx) return fail(RH_EINVAL, "rh_set_solver: null context");
#ifdef RH_VARIANTS
  if (which < 0 || which > 5)
    return fail(RH_EINVAL,
                "rh_set_solver: which=%d (0 = auto, 1 = general kernel, 2 = ungrouped, 3 = k_solve_pair, "
                "4 / 5 = ungrouped, k_solve_lds in one / two passes)", which);
  ctx->no_group = which >= 2;
  ctx->use_pair = which == 3 || (which == 0 && RH_PAIR_ON);
  ctx->two_pass = which == 5 || (which != 4 && RH_TWO_PASS);
#else
  if (which < 0 || which > 1)
    return fail(RH_EINVAL, "rh_set_solver: which=%d (0 = auto, 1 = general kernel; the grouped, lane-pair and "
                "two-pass kernels are tools/ubench variant builds)", which);
#endif
  ctx->force_general = which == 1;
  return RH_OK;
}

int rh_group_cases(void) { return kGroupCases; }

int rh_solve_noxi_max_bins(void) { return 2 * rh::kLT; }

int rh_set_a0(rh_ctx* ctx, int on) {
  if (!ctx) return fail(RH_EINVAL, "rh_set_a0: null context");
  if (on != 0 && on != 1) return fail(RH_EINVAL, "rh_set_a0: on=%d (0 or 1)", on);
#ifdef RH_VARIANTS
  ctx->a0 = on != 0;
#else
  if (on) return fail(RH_EINVAL, "rh_set_a0: k_a0_sums is not in the shipped library (measured slower, DESIGN.md §5; "
                                 "tools/build_variants.sh builds it)");
#endif
  return RH_OK;
}

int rh_set_qtf_waves(rh_ctx* ctx, int waves) {
  if (!ctx) return fail(RH_EINVAL, "rh_set_qtf_waves: null context");
  if (waves != 0 && waves != 1 && waves != 2 && waves != 4)
    return fail(RH_EINVAL, "rh_set_qtf_waves: waves=%d (0 = auto, 1, 2 or 4)", waves);
  ctx->qtf_waves = waves;
  return RH_OK;
}

int rh_set_qtf_path(rh_ctx* ctx, int path) {
  if (!ctx) return fail(RH_EINVAL, "rh_set_qtf_path: null context");
  if (path < 0 || path > 3)
    return fail(RH_EINVAL, "rh_set_qtf_path: path=%d (0 = MFMA GEMMs when order == 1, 1 = per-pair kernel, "
                           "2 = MFMA GEMMs with 32 x 32 tiles for a whole QTF, 3 = the GEMM coefficients and "
                           "Kim & Yue as two launches)", path);
#ifdef RH_VARIANTS
  ctx->qtf_t32 = path == 2;
  ctx->qtf_sep = path == 3;
#else
  if (path >= 2)
    return fail(RH_EINVAL, "rh_set_qtf_path: path %d is not in the shipped library (measured slower, DESIGN.md §5; "
                           "tools/build_variants.sh builds it)", path);
#endif
  ctx->qtf_direct = path == 1;
  return RH_OK;
}

int rh_ctx_create(int device, rh_ctx** out) {
  if (!out) return fail(RH_EINVAL, "rh_ctx_create: null out");
  int n = 0;
  RH_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(RH_EINVAL, "device %d not present (%d visible)", device, n);
  RH_HIP(hipSetDevice(device));
  rh_ctx* c = new rh_ctx;
  c->device = device;
  hipError_t e = hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device);
  for (auto& sl : c->slot) {
    if (e == hipSuccess) e = hipEventCreateWithFlags(&sl.staged, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&sl.used, hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    for (auto& sl : c->slot) {
      if (sl.staged) (void)hipEventDestroy(sl.staged);
      if (sl.used) (void)hipEventDestroy(sl.used);
    }
    delete c;
    return fail(RH_EHIP, "hipEventCreate: %s", hipGetErrorString(e));
  }
  *out = c;
  return RH_OK;
}

int rh_ctx_destroy(rh_ctx* ctx) {
  if (!ctx) return RH_OK;
  for (auto& sl : ctx->slot) {
    if (sl.staged) {
      (void)hipEventSynchronize(sl.staged);
      (void)hipEventDestroy(sl.staged);
    }
    if (sl.used) {
      (void)hipEventSynchronize(sl.used);
      (void)hipEventDestroy(sl.used);
    }
    if (sl.d) (void)hipFree(sl.d);
    if (sl.h) (void)hipHostFree(sl.h);
  }
  if (!ctx->wt_scratch.empty()) (void)hipDeviceSynchronize();
  for (auto& sc : ctx->wt_scratch) (void)hipFree(sc.p);
  delete ctx;
  return RH_OK;
}

int rh_wave_tables(rh_ctx* ctx, const rh_design* d, const double* beta, rh_c128* uhat, rh_c128* finer,
                   rh_c128* kproj, rh_stream stream) {
  if (!ctx || !d || !beta || !uhat || !finer || !kproj) return fail(RH_EINVAL, "rh_wave_tables: null argument");
  if (int r = check_design(*d, false)) return r;
  if (d->nhead < 1) return fail(RH_EINVAL, "rh_wave_tables: nhead must be >= 1");
  RH_HIP(hipSetDevice(ctx->device));
  const hipStream_t s = (hipStream_t)stream;
  const int ng = (d->nn + rh::kWtN - 1) / rh::kWtN;
  if (ng > 1) {
    // nodes over the grid, per-node forces through this stream's scratch, summed in node order
    // (k_wave_tables_nodes + k_wave_force_sum: the bits of k_wave_tables)
    const size_t bytes = (size_t)d->nhead * d->nn * 6 * d->nw * sizeof(rh_c128);
    void* fw = nullptr;
    {
      std::lock_guard<std::mutex> lock(ctx->wt_mu);
      rh_ctx::Scratch* sc = nullptr;
      for (auto& e : ctx->wt_scratch)
        if (e.s == s) sc = &e;
      if (!sc) {
        ctx->wt_scratch.push_back({s, nullptr, 0});
        sc = &ctx->wt_scratch.back();
      }
      if (sc->bytes < bytes) {   // grow: the old buffer may still be read by this stream's work
        if (sc->p) {
          RH_HIP(hipStreamSynchronize(s));
          RH_HIP(hipFree(sc->p));
          sc->p = nullptr;
          sc->bytes = 0;
        }
        RH_HIP(hipMalloc(&sc->p, bytes));
        sc->bytes = bytes;
      }
      fw = sc->p;
    }
    dim3 grid((d->nw + 63) / 64, d->nhead, ng);
    hipLaunchKernelGGL(rh::k_wave_tables_nodes, grid, dim3(64 * rh::kWtN), 0, s, *d, beta, uhat, kproj, (rh_c128*)fw);
    const int tot = d->nhead * 6 * d->nw;
    hipLaunchKernelGGL(rh::k_wave_force_sum, dim3((tot + 255) / 256), dim3(256), 0, s, d->nw, d->nn, d->nhead,
                       (const rh_c128*)fw, finer);
    RH_HIP(hipGetLastError());
    return RH_OK;
  }
  dim3 grid((d->nw + 63) / 64, d->nhead);
  hipLaunchKernelGGL(rh::k_wave_tables, grid, dim3(64 * rh::kWtN), 0, s, *d, beta, uhat, finer, kproj);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_wave_tables_batch(rh_ctx* ctx, const rh_design* designs, int ndesign, const double* beta, int hstride,
                         rh_stream stream) {
  if (!ctx || !designs || !beta) return fail(RH_EINVAL, "rh_wave_tables_batch: null argument");
  if (ndesign < 1) return ndesign == 0 ? RH_OK : fail(RH_EINVAL, "rh_wave_tables_batch: ndesign=%d", ndesign);
  int nwmax = 0, nhmax = 0;
  for (int i = 0; i < ndesign; ++i) {
    const rh_design& d = designs[i];
    if (int r = check_design(d, false)) return r;
    if (d.nhead < 1 || d.nhead > hstride)
      return fail(RH_EINVAL, "rh_wave_tables_batch: design %d: nhead=%d outside [1, hstride=%d]", i, d.nhead, hstride);
    if (!d.finer || !d.kproj) return fail(RH_EINVAL, "rh_wave_tables_batch: design %d: null table", i);
    nwmax = d.nw > nwmax ? d.nw : nwmax;
    nhmax = d.nhead > nhmax ? d.nhead : nhmax;
  }
  RH_HIP(hipSetDevice(ctx->device));
  const hipStream_t s = (hipStream_t)stream;
  if (int r = stage_designs(ctx, designs, ndesign, s)) return r;
  dim3 grid((nwmax + 63) / 64, nhmax, ndesign);
  hipLaunchKernelGGL(rh::k_wave_tables_batch, grid, dim3(64 * rh::kWtN), 0, s, staged_designs(ctx), beta, hstride);
  return designs_used(ctx, s);
}

int rh_solve_cases(rh_ctx* ctx, const rh_design* designs, int ndesign, const rh_cases* cases,
                   const rh_solve_out* out, rh_stream stream) {
  if (!ctx || !designs || !cases || !out) return fail(RH_EINVAL, "rh_solve_cases: null argument");
  if (ndesign < 1) return fail(RH_EINVAL, "rh_solve_cases: ndesign=%d", ndesign);
  if (cases->ncase < 0) return fail(RH_EINVAL, "rh_solve_cases: ncase=%d", cases->ncase);
  if (cases->ncase == 0) return RH_OK;
  if (!cases->design || !cases->head || !cases->spectrum || !cases->Hs || !cases->Tp || !cases->gamma)
    return fail(RH_EINVAL, "rh_solve_cases: null case array");
  if (!out->Xi_last || !out->iters || !out->status)
    return fail(RH_EINVAL, "rh_solve_cases: Xi_last, iters and status outputs are required");
  if (!out->Xi && (out->psd || out->std || out->rao))
    return fail(RH_EINVAL, "rh_solve_cases: psd, std and rao need the Xi output");
  if (!out->Xi && designs[0].nw > rh_solve_noxi_max_bins())
    return fail(RH_EINVAL, "rh_solve_cases: grids beyond %d bins need the Xi output", rh_solve_noxi_max_bins());
  if (cases->nIter < 0) return fail(RH_EINVAL, "rh_solve_cases: nIter=%d", cases->nIter);
  if (cases->first_iter < 0 || cases->first_iter > cases->nIter)
    return fail(RH_EINVAL, "rh_solve_cases: first_iter=%d outside [0, nIter=%d]", cases->first_iter, cases->nIter);
  const int nw = designs[0].nw;
  int nnmax = 0;
  for (int i = 0; i < ndesign; ++i) {
    if (int r = check_design(designs[i], true, false)) return r;
    if (designs[i].nw != nw) return fail(RH_EINVAL, "rh_solve_cases: all designs must share nw");
    if (designs[i].nn > nnmax) nnmax = designs[i].nn;
  }
  RH_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (int r = stage_designs(ctx, designs, ndesign, s)) return r;
  rh::CaseArgs a;
  a.designs = staged_designs(ctx);
  a.c = *cases;
  a.o = *out;
  a.bmat_nn = nnmax;
  int nmmax = 0;
  for (int i = 0; i < ndesign; ++i) nmmax = designs[i].nm > nmmax ? designs[i].nm : nmmax;
#ifdef RH_VARIANTS
  // Grouped path (rh_solve_grp.hip): kGroupCases cases of one (design, heading) per workgroup.
  // (It does not report the convergence margin: with out->margin the ungrouped kernels run.)
  if (cases->group_start && cases->ngroup > 0 && !ctx->force_general && !ctx->no_group && !out->margin) {
    if (cases->ngroup > cases->ncase) return fail(RH_EINVAL, "rh_solve_cases: ngroup=%d > ncase", cases->ngroup);
    const int npass = (nw + rh::kGT - 1) / rh::kGT;
    const size_t lsm = rh::solve_grp_smem(nnmax, nmmax, npass, kGroupCases);
    if (lsm <= 160 * 1024) {
      hipLaunchKernelGGL(rh::k_solve_grp<kGroupCases>, dim3(cases->ngroup), dim3(rh::kGT), lsm, s, a,
                         cases->group_start, cases->ngroup);
      return designs_used(ctx, s);
    }
  }
  // Opt-in path (rh_solve_pair.hip, rh_set_solver(ctx, 3)): one bin per lane, lane-pair LU,
  // 4 waves per SIMD.  Parity-green but slower than k_solve_lds on C2.
  if (nw <= 1024 && !ctx->force_general && ctx->use_pair) {
    const int lt = nw <= 256 ? 256 : nw <= 512 ? 512 : 1024;
    const int pb = lt == 1024 ? kPairPB : 1;
    const size_t lsm = rh::solve_pair_smem(nnmax, nmmax, lt, pb);
    if (lsm <= kMaxLds) {
      dim3 grid(cases->ncase), block(lt);
      if (lt == 256) hipLaunchKernelGGL((rh::k_solve_pair<256, 1, kPairRA, kPairRC, kPairHold>), grid, block, lsm, s, a);
      else if (lt == 512) hipLaunchKernelGGL((rh::k_solve_pair<512, 1, kPairRA, kPairRC, kPairHold>), grid, block, lsm, s, a);
      else hipLaunchKernelGGL((rh::k_solve_pair<1024, kPairPB, kPairRA, kPairRC, kPairHold>), grid, block, lsm, s, a);
      return designs_used(ctx, s);
    }
  }
#endif
  // Cases that start from XiStart: phase A of iteration 0 for the whole batch as one GEMM
  // launch (rh_a0.hip), its sums in each case's Xi_last block (k_solve_lds reads them first).
  auto prep_a0 = [&]() -> int {
#ifdef RH_VARIANTS
    if (!ctx->a0 || cases->first_iter != 0 || cases->Xi_init || !rh::a0_fits(nw, nnmax) ||
        rh::kA0StaticLds + rh::a0_smem(nnmax, nmmax) > kMaxLds)
      return RH_OK;
    dim3 g((cases->ncase + rh::kA0Cases - 1) / rh::kA0Cases, (rh::a0_chunks(nw) + rh::kA0Cpb - 1) / rh::kA0Cpb);
    hipLaunchKernelGGL(rh::k_a0_sums, g, dim3(rh::kA0Threads), rh::a0_smem(nnmax, nmmax), s, a);
    RH_HIP(hipGetLastError());
    a.a0 = 1;
#endif
    return RH_OK;
  };
  // Fast path (rh_solve.hip): XiLast in LDS, 512 threads per case (256 for nw <= 256), nw <= 1024.
  if (nw <= 2 * rh::kLT && !ctx->force_general) {
#ifndef RH_SMALL_GRID_128
#define RH_SMALL_GRID_128 1
#endif
    // nw <= 256 on 128 threads x 2 bins (x 1 bin for nw <= 128), B_drag summed without the
    // per-node image (rh_solve.hip), four cases per CU while a workgroup's LDS stays within
    // 40 KB: C4 0.544-0.554 ms against 0.586-0.590 ms for 256 threads x 1 bin
    // (-DRH_SMALL_GRID_128=0).  The kernel depends on nw only, never on the batch's node counts,
    // so the bits of a case do not depend on which designs share its launch.
    if (RH_SMALL_GRID_128 && nw <= rh::kLT / 2) {
      const int nb128 = nw <= rh::kLT / 4 ? 1 : 2;
      const size_t lsm128 = rh::solve_lds_smem(nnmax, nmmax, nb128, rh::kLT / 4, true);
      if (lsm128 <= kMaxLds) {
        if (int r = prep_a0()) return r;
        dim3 grid(cases->ncase), block(rh::kLT / 4);
        RH_HIP(rh::launch_solve_fast(nb128 == 1 ? rh::kSolve1x128 : rh::kSolve2x128, grid, block, lsm128, s, a));
        return designs_used(ctx, s);
      }
    }
    const int nb = nw <= rh::kLT ? 1 : 2;
    const int lt = nw <= rh::kLT / 2 ? rh::kLT / 2 : rh::kLT;   // nw <= 256: 256 threads, two cases per CU
    const size_t lsm = rh::solve_lds_smem(nnmax, nmmax, nb, lt);
    if (lsm <= 160 * 1024) {
      if (int r = prep_a0()) return r;
      dim3 grid(cases->ncase), block(lt);
      const int kern = lt < rh::kLT ? rh::kSolve1x256 : nb == 1 ? rh::kSolve1x512 : rh::kSolve2x512;
#ifdef RH_VARIANTS
      // Two passes when the batch needs more than one round of workgroups (measured slower on
      // C2: 0.895 vs 0.828 ms).  Pass 1 runs every case up to its last possible
      // iteration, pass 2 finishes the cases that need it from the parked iterate.
      const int nloop = cases->nIter + 1;
      if (ctx->two_pass && nloop - 1 > cases->first_iter) {
        int per_cu = 0;
        RH_HIP(rh::occupancy_solve_fast(kern, &per_cu, lt, lsm));
        if (cases->ncase > per_cu * ctx->ncu) {
          a.stop_iter = nloop - 1;
          RH_HIP(rh::launch_solve_fast(kern, grid, block, lsm, s, a));
          a.resume = 1;
        }
      }
#endif
      RH_HIP(rh::launch_solve_fast(kern, grid, block, lsm, s, a));
      return designs_used(ctx, s);
    }
  }
  // 1024 < nw <= 2048: the same kernel in two passes of 1024 bins, XiLast in the Xi_last block
  // (192 KB at nw = 2048 is beyond the LDS), DESIGN.md §4.
  if (nw <= 4 * rh::kLT && !ctx->force_general) {
    const size_t lsm = rh::solve_lds_smem(nnmax, nmmax, 2, rh::kLT, false, 2);
    if (lsm <= kMaxLds) {
      if (int r = prep_a0()) return r;
      hipLaunchKernelGGL((rh::k_solve_lds<2, rh::kLT, false, 2>), dim3(cases->ncase), dim3(rh::kLT), lsm, s, a);
      return designs_used(ctx, s);
    }
  }
  const size_t smem = sizeof(double) * (size_t)((kThreads / 64) * nnmax * 3 + nnmax * 9 + 36 + (kThreads / 64) * 6 + 108 +
                                                nnmax * 5 + kThreads / 64);
  if (smem > kMaxLds)
    return fail(RH_EINVAL, "rh_solve_cases: %d submerged nodes need %zu B of LDS (> %zu B on gfx950)", nnmax, smem,
                kMaxLds);
  dim3 grid(cases->ncase), block(kThreads);
  switch (nb_for(nw)) {
    case 1: hipLaunchKernelGGL(rh::k_solve_cases<1>, grid, block, smem, s, a); break;
    case 2: hipLaunchKernelGGL(rh::k_solve_cases<2>, grid, block, smem, s, a); break;
    case 4: hipLaunchKernelGGL(rh::k_solve_cases<4>, grid, block, smem, s, a); break;
    default: hipLaunchKernelGGL(rh::k_solve_cases<8>, grid, block, smem, s, a); break;
  }
  return designs_used(ctx, s);
}

int rh_heading_response_ext(rh_ctx* ctx, const rh_design* designs, int ndesign, int ncase, const int* design_idx,
                            const int* head, const double* zeta, const double* B_drag, const double* Bmat, int bmat_nn,
                            const rh_c128* fext, rh_c128* Xi, rh_stream stream) {
  if (!ctx || !designs || !design_idx || !head || !zeta || !B_drag || !Bmat || !Xi)
    return fail(RH_EINVAL, "rh_heading_response: null argument");
  if (ncase <= 0) return ncase == 0 ? RH_OK : fail(RH_EINVAL, "ncase=%d", ncase);
  if (ndesign < 1) return fail(RH_EINVAL, "rh_heading_response: ndesign=%d", ndesign);
  const int nw = designs[0].nw;
  int nnmax = 0;
  for (int i = 0; i < ndesign; ++i) {
    if (int r = check_design(designs[i], true)) return r;
    if (designs[i].nw != nw) return fail(RH_EINVAL, "rh_heading_response: all designs must share nw");
    if (designs[i].nn > nnmax) nnmax = designs[i].nn;
  }
  if (bmat_nn == 0) bmat_nn = nnmax;
  if (bmat_nn < nnmax)
    return fail(RH_EINVAL, "rh_heading_response: Bmat row stride %d < %d nodes of a design passed", bmat_nn, nnmax);
  RH_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (int r = stage_designs(ctx, designs, ndesign, s)) return r;
  rh::HeadArgs a{staged_designs(ctx), ncase, design_idx, head, zeta, B_drag, Bmat, Xi, nullptr, bmat_nn, ndesign, fext};
  const size_t smem = sizeof(double) * (size_t)(nnmax * 9 + 36 + 108);
  dim3 grid((nw + kThreads - 1) / kThreads, ncase);
  hipLaunchKernelGGL(rh::k_heading_resp, grid, dim3(kThreads), smem, s, a);
  return designs_used(ctx, s);
}

int rh_heading_response(rh_ctx* ctx, const rh_design* designs, int ndesign, int ncase, const int* design_idx,
                        const int* head, const double* zeta, const double* B_drag, const double* Bmat, rh_c128* Xi,
                        rh_stream stream) {
  return rh_heading_response_ext(ctx, designs, ndesign, ncase, design_idx, head, zeta, B_drag, Bmat, 0, nullptr, Xi,
                                 stream);
}

int rh_wave_excitation(rh_ctx* ctx, const rh_design* designs, int ndesign, int ncase, const int* design_idx,
                       const int* head, const double* zeta, const double* Bmat, rh_c128* F, rh_stream stream) {
  if (!ctx || !designs || !design_idx || !head || !zeta || !Bmat || !F)
    return fail(RH_EINVAL, "rh_wave_excitation: null argument");
  if (ncase <= 0) return ncase == 0 ? RH_OK : fail(RH_EINVAL, "ncase=%d", ncase);
  const int nw = designs[0].nw;
  int nnmax = 0;
  for (int i = 0; i < ndesign; ++i) {
    if (int r = check_design(designs[i], true)) return r;
    if (designs[i].nw != nw) return fail(RH_EINVAL, "rh_wave_excitation: all designs must share nw");
    if (designs[i].nn > nnmax) nnmax = designs[i].nn;
  }
  RH_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (int r = stage_designs(ctx, designs, ndesign, s)) return r;
  rh::HeadArgs a{staged_designs(ctx), ncase, design_idx, head, zeta, nullptr, Bmat, nullptr, F, nnmax, ndesign, nullptr};
  const size_t smem = sizeof(double) * (size_t)(nnmax * 9 + 36 + 108);
  dim3 grid((nw + kThreads - 1) / kThreads, ncase);
  hipLaunchKernelGGL(rh::k_heading_resp, grid, dim3(kThreads), smem, s, a);
  return designs_used(ctx, s);
}

int rh_linearize(rh_ctx* ctx, const rh_design* d, int head, const rh_c128* Xi, const double* zeta, double* B_drag,
                 double* Bmat, rh_c128* F_drag, rh_stream stream) {
  if (!ctx || !d || !Xi || !zeta || !B_drag || !Bmat) return fail(RH_EINVAL, "rh_linearize: null argument");
  if (int r = check_design(*d, true)) return r;
  if (head < 0 || head >= d->nhead) return fail(RH_EINVAL, "rh_linearize: head %d out of range", head);
  RH_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (d->nn > 0) hipLaunchKernelGGL(rh::k_lin_sums, dim3(d->nn), dim3(kThreads), 0, s, *d, head, Xi, zeta, Bmat);
  RH_HIP(hipGetLastError());
  hipLaunchKernelGGL(rh::k_lin_bdrag, dim3(1), dim3(64), 0, s, *d, (const double*)Bmat, B_drag);
  RH_HIP(hipGetLastError());
  if (F_drag) return rh_drag_excitation(ctx, d, head, zeta, Bmat, F_drag, stream);
  return RH_OK;
}

int rh_lin_partial_sums(rh_ctx* ctx, const rh_design* d, int head, const rh_c128* Xi_last, const double* zeta,
                        int bin_lo, int bin_hi, double* sums, rh_stream stream) {
  if (!ctx || !d || !Xi_last || !zeta || !sums) return fail(RH_EINVAL, "rh_lin_partial_sums: null argument");
  if (int r = check_design(*d, true)) return r;
  if (head < 0 || head >= d->nhead) return fail(RH_EINVAL, "rh_lin_partial_sums: head %d out of range", head);
  if (bin_lo < 0 || bin_hi > d->nw || bin_lo > bin_hi)
    return fail(RH_EINVAL, "rh_lin_partial_sums: bins [%d, %d) outside [0, %d)", bin_lo, bin_hi, d->nw);
  RH_HIP(hipSetDevice(ctx->device));
  if (d->nn > 0)
    hipLaunchKernelGGL(rh::k_lin_partial, dim3(d->nn), dim3(kThreads), 0, (hipStream_t)stream, *d, head, Xi_last, zeta,
                       bin_lo, bin_hi, sums);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_bin_step(rh_ctx* ctx, const rh_design* d, int head, const double* zeta, const rh_c128* fext, const double* sums,
                double tol, int bin_lo, int bin_hi, double* Bmat, double* B_drag, rh_c128* Xi, rh_c128* Xi_last,
                int* flags, rh_stream stream) {
  if (!ctx || !d || !zeta || !sums || !Bmat || !B_drag || !Xi || !Xi_last || !flags)
    return fail(RH_EINVAL, "rh_bin_step: null argument");
  if (int r = check_design(*d, true)) return r;
  if (head < 0 || head >= d->nhead) return fail(RH_EINVAL, "rh_bin_step: head %d out of range", head);
  if (bin_lo < 0 || bin_hi > d->nw || bin_lo > bin_hi)
    return fail(RH_EINVAL, "rh_bin_step: bins [%d, %d) outside [0, %d)", bin_lo, bin_hi, d->nw);
  RH_HIP(hipSetDevice(ctx->device));
  const int n = bin_hi - bin_lo;
  const size_t smem = sizeof(double) * (size_t)(9 * d->nn + 36 + 108);
  hipLaunchKernelGGL(rh::k_bin_step, dim3(n > 0 ? (n + kThreads - 1) / kThreads : 1), dim3(kThreads), smem,
                     (hipStream_t)stream, *d, head, zeta, fext, sums, tol, bin_lo, bin_hi, Bmat, B_drag, Xi, Xi_last,
                     flags);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_drag_excitation(rh_ctx* ctx, const rh_design* d, int head, const double* zeta, const double* Bmat,
                       rh_c128* F_drag, rh_stream stream) {
  if (!ctx || !d || !zeta || !Bmat || !F_drag) return fail(RH_EINVAL, "rh_drag_excitation: null argument");
  if (int r = check_design(*d, true)) return r;
  if (head < 0 || head >= d->nhead) return fail(RH_EINVAL, "rh_drag_excitation: head %d out of range", head);
  RH_HIP(hipSetDevice(ctx->device));
  const size_t smem = sizeof(double) * (size_t)(d->nn * 9 + 2);
  hipLaunchKernelGGL(rh::k_drag_exc, dim3((d->nw + kThreads - 1) / kThreads), dim3(kThreads), smem,
                     (hipStream_t)stream, *d, head, zeta, Bmat, F_drag);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_sea_state(rh_ctx* ctx, int ncase, int nw, const double* w, double dw, const int* spectrum, const double* Hs,
                 const double* Tp, const double* gamma, double* S, double* zeta, rh_stream stream) {
  if (!ctx || !w || !spectrum || !Hs || !Tp || !gamma || !zeta) return fail(RH_EINVAL, "rh_sea_state: null argument");
  if (ncase < 0 || nw <= 0 || !(dw > 0)) return fail(RH_EINVAL, "rh_sea_state: bad sizes");
  if (ncase == 0) return RH_OK;
  RH_HIP(hipSetDevice(ctx->device));
  dim3 grid((nw + 255) / 256, ncase);
  hipLaunchKernelGGL(rh::k_sea_state, grid, dim3(256), 0, (hipStream_t)stream, nw, w, dw, spectrum, Hs, Tp, gamma, S,
                     zeta);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_motion_stats(rh_ctx* ctx, int ncase, int nrow, int nw, double dw, const rh_c128* Xi, double* psd, double* std_,
                    rh_stream stream) {
  if (!ctx || !Xi) return fail(RH_EINVAL, "rh_motion_stats: null argument");
  if (ncase <= 0 || nrow <= 0 || nw <= 0 || !(dw > 0)) return fail(RH_EINVAL, "rh_motion_stats: bad sizes");
  RH_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(rh::k_motion_stats, dim3(ncase), dim3(kThreads), 0, (hipStream_t)stream, nrow, nw, dw, Xi, psd,
                     std_);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_channel_stats(rh_ctx* ctx, int ncase, int nrow, int ndof, int nw, double dw, const double* w,
                     const rh_c128* Xi, int nch, const double* coef, double* psd, double* std_, rh_stream stream) {
  if (!ctx || !w || !Xi || !coef) return fail(RH_EINVAL, "rh_channel_stats: null argument");
  if (ncase < 0 || nrow <= 0 || ndof <= 0 || nw <= 0 || nch < 0 || !(dw > 0))
    return fail(RH_EINVAL, "rh_channel_stats: bad sizes ncase=%d nrow=%d ndof=%d nw=%d nch=%d", ncase, nrow, ndof, nw,
                nch);
  if (ncase == 0 || nch == 0) return RH_OK;
  RH_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(rh::k_channel_stats, dim3(nch, ncase), dim3(kThreads), 0, (hipStream_t)stream, nrow, ndof, nw, dw,
                     w, Xi, nch, coef, psd, std_);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_system_solve(rh_ctx* ctx, int nf, int nw, const rh_c128* Z, const double* K, const rh_c128* F, rh_c128* Xi,
                    rh_stream stream) {
  return rh_system_solve_batch(ctx, 1, nf, nw, Z, K, F, Xi, stream);
}

int rh_system_solve_batch(rh_ctx* ctx, int ncase, int nf, int nw, const rh_c128* Z, const double* K, const rh_c128* F,
                          rh_c128* Xi, rh_stream stream) {
  if (!ctx || !Z || !F || !Xi) return fail(RH_EINVAL, "rh_system_solve: null argument");
  if (nw <= 0 || ncase < 0) return fail(RH_EINVAL, "rh_system_solve: nw=%d ncase=%d", nw, ncase);
  if (nf < 1 || nf > 2) return fail(RH_EINVAL, "rh_system_solve: nf=%d (supported: 1, 2)", nf);
  if (ncase == 0) return RH_OK;
  RH_HIP(hipSetDevice(ctx->device));
  const int N = 6 * nf;
  if (!ctx->force_general) {   // register kernels (rh_set_solver(ctx, 1) keeps the LDS elimination for cross-checks)
    const dim3 g((nw + 63) / 64, ncase);
    if (nf == 1)
      hipLaunchKernelGGL(rh::k_system_solve_reg<1>, g, dim3(64), 0, (hipStream_t)stream, nw, Z, K, F, Xi);
    else
      hipLaunchKernelGGL(rh::k_system_solve_reg<2>, g, dim3(64), 0, (hipStream_t)stream, nw, Z, K, F, Xi);
    RH_HIP(hipGetLastError());
    return RH_OK;
  }
  const size_t smem = sizeof(double) * 2 * (size_t)(N * N + N) * rh::kSysThreads;
  dim3 grid((nw + rh::kSysThreads - 1) / rh::kSysThreads, ncase);
  hipLaunchKernelGGL(rh::k_system_solve, grid, dim3(rh::kSysThreads), smem, (hipStream_t)stream, N, nw, Z, K, F, Xi);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_array_response(rh_ctx* ctx, const rh_design* designs, int ndesign, int nf, int ncase, const int* design_idx,
                      const int* head, const double* zeta, const double* B_drag, const double* Bmat, const double* K,
                      rh_c128* Xi, rh_stream stream) {
  return rh_array_response_stats(ctx, designs, ndesign, nf, ncase, design_idx, head, zeta, B_drag, Bmat, K, Xi, 0.0,
                                 nullptr, nullptr, nullptr, stream);
}

int rh_array_response_stats(rh_ctx* ctx, const rh_design* designs, int ndesign, int nf, int ncase,
                            const int* design_idx, const int* head, const double* zeta, const double* B_drag,
                            const double* Bmat, const double* K, rh_c128* Xi, double dw, double* psd, double* std_,
                            const int* order, rh_stream stream) {
  if (!ctx || !designs || !design_idx || !head || !zeta || !B_drag || !Bmat || !Xi)
    return fail(RH_EINVAL, "rh_array_response: null argument");
  if ((psd || std_) && !(dw > 0)) return fail(RH_EINVAL, "rh_array_response_stats: dw=%g", dw);
  if (nf < 1 || nf > 2) return fail(RH_EINVAL, "rh_array_response: nf=%d (supported: 1, 2)", nf);
  if (ncase <= 0) return ncase == 0 ? RH_OK : fail(RH_EINVAL, "rh_array_response: ncase=%d", ncase);
  if (ndesign < 1) return fail(RH_EINVAL, "rh_array_response: ndesign=%d", ndesign);
  const int nw = designs[0].nw;
  int nn = 0, nmmax = 0;   // nn: the largest node count (the Bmat stride and the LDS layout)
  for (int i = 0; i < ndesign; ++i) {
    if (int r = check_design(designs[i], true)) return r;
    if (designs[i].nw != nw) return fail(RH_EINVAL, "rh_array_response: all designs must share nw");
    nn = designs[i].nn > nn ? designs[i].nn : nn;
    nmmax = designs[i].nm > nmmax ? designs[i].nm : nmmax;
  }
  const size_t lsm = rh::array_exc_smem(nn, nmmax);
  if (lsm > kMaxLds)
    return fail(RH_EINVAL, "rh_array_response: %d nodes / %d members need %zu B of LDS", nn, nmmax, lsm);
  RH_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (int r = stage_designs(ctx, designs, ndesign, s)) return r;
  rh::ArrayArgs a{staged_designs(ctx), ncase, design_idx, head, zeta, B_drag, Bmat, K, Xi, nn, nmmax, dw, psd, std_,
                  order};
  const dim3 ge(ncase * nf), g(ncase);   // excitation per (case, FOWT), then the solve (+ statistics) per case
  const bool multi = nw > rh::kArrRespThreads;
  const dim3 gr(rh::kArrRespThreads);
  if (nf == 1) {
    hipLaunchKernelGGL(rh::k_array_exc<1>, ge, dim3(rh::kArrExcThreads), lsm, s, a);
    RH_HIP(hipGetLastError());
    if (multi) hipLaunchKernelGGL((rh::k_array_resp<1, true>), g, gr, 0, s, a);
    else hipLaunchKernelGGL((rh::k_array_resp<1, false>), g, gr, 0, s, a);
  } else {
    hipLaunchKernelGGL(rh::k_array_exc<2>, ge, dim3(rh::kArrExcThreads), lsm, s, a);
    RH_HIP(hipGetLastError());
    if (multi) hipLaunchKernelGGL((rh::k_array_resp<2, true>), g, gr, 0, s, a);
    else hipLaunchKernelGGL((rh::k_array_resp<2, false>), g, gr, 0, s, a);
  }
  RH_HIP(hipGetLastError());
  return designs_used(ctx, s);
}

// The response step alone, with F already in Xi (rh_solve_out.F_wave of the fixed point): the
// block solve and the statistics of k_array_resp, no excitation launch.
int rh_array_solve_stats(rh_ctx* ctx, const rh_design* designs, int ndesign, int nf, int ncase, const int* design_idx,
                         const double* B_drag, const double* K, rh_c128* Xi, double dw, double* psd, double* std_,
                         rh_stream stream) {
  if (!ctx || !designs || !design_idx || !B_drag || !Xi) return fail(RH_EINVAL, "rh_array_solve_stats: null argument");
  if ((psd || std_) && !(dw > 0)) return fail(RH_EINVAL, "rh_array_solve_stats: dw=%g", dw);
  if (nf < 1 || nf > 2) return fail(RH_EINVAL, "rh_array_solve_stats: nf=%d (supported: 1, 2)", nf);
  if (ncase <= 0) return ncase == 0 ? RH_OK : fail(RH_EINVAL, "rh_array_solve_stats: ncase=%d", ncase);
  if (ndesign < 1) return fail(RH_EINVAL, "rh_array_solve_stats: ndesign=%d", ndesign);
  const int nw = designs[0].nw;
  for (int i = 0; i < ndesign; ++i) {
    if (int r = check_design(designs[i], false)) return r;
    if (designs[i].nw != nw) return fail(RH_EINVAL, "rh_array_solve_stats: all designs must share nw");
  }
  RH_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (int r = stage_designs(ctx, designs, ndesign, s)) return r;
  rh::ArrayArgs a{staged_designs(ctx), ncase, design_idx, nullptr, nullptr, B_drag, nullptr, K, Xi, 0, 0, dw, psd, std_,
                  nullptr};
  const dim3 g(ncase), gr(rh::kArrRespThreads);
  const bool multi = nw > rh::kArrRespThreads;
  if (nf == 1) {
    if (multi) hipLaunchKernelGGL((rh::k_array_resp<1, true>), g, gr, 0, s, a);
    else hipLaunchKernelGGL((rh::k_array_resp<1, false>), g, gr, 0, s, a);
  } else {
    if (multi) hipLaunchKernelGGL((rh::k_array_resp<2, true>), g, gr, 0, s, a);
    else hipLaunchKernelGGL((rh::k_array_resp<2, false>), g, gr, 0, s, a);
  }
  RH_HIP(hipGetLastError());
  return designs_used(ctx, s);
}

long long rh_qtf_workspace_bytes(const rh_qtf_design* q) {
  if (!q) return -1;
  return (long long)(rh::qtf_work_elems(*q) * sizeof(rh_c128));
}

// Rank's contiguous block [t0, t1) of the upper triangle's 16 x 16 pair tiles (row-major, T1 <=
// T2): t_r is the first tile whose preceding tiles hold at least r / nrank of the pairs (i1 <=
// i2 < n2; a diagonal tile holds 136 pairs, a full one 256), so the ranks' pair counts differ by
// at most a tile's.  raft/parallel.py qtf_tile_block is the same integer arithmetic.
static void qtf_tile_block(int n2, int rank, int nrank, int& t0, int& t1) {
  const int nt = (n2 + 15) / 16;
  std::vector<long long> cum(1, 0);   // pairs before tile t
  for (int a = 0; a < nt; ++a) {
    const long long ra = (16 * a + 16 < n2 ? 16 * a + 16 : n2) - 16 * a;
    for (int b = a; b < nt; ++b) {
      const long long cb = (16 * b + 16 < n2 ? 16 * b + 16 : n2) - 16 * b;
      cum.push_back(cum.back() + (a == b ? ra * (ra + 1) / 2 : ra * cb));
    }
  }
  const long long total = cum.back();
  auto first = [&](int r) {   // smallest t with cum[t] * nrank >= r * total
    int t = 0;
    while (cum[t] * nrank < (long long)r * total) ++t;
    return t;
  };
  t0 = first(rank);
  t1 = rank + 1 == nrank ? (int)cum.size() - 1 : first(rank + 1);
}

static int qtf_launch(rh_ctx* ctx, const rh_qtf_design* q, int nw, const double* w, const rh_c128* Xi0,
                      const double* M66, int rank, int nrank, int mirror, rh_c128* qtf, void* work,
                      long long work_bytes, rh_stream stream, const char* who, int flags = 0) {
  if (!ctx || !q || !w || !Xi0 || !M66 || !qtf || !work) return fail(RH_EINVAL, "%s: null argument", who);
  if (q->n2 < 1 || q->nq < 0 || q->nmq < 0 || q->nkr < 0 || nw < 2)
    return fail(RH_EINVAL, "%s: bad sizes n2=%d nq=%d nmq=%d nkr=%d nw=%d", who, q->n2, q->nq, q->nmq, q->nkr, nw);
  if (nrank < 1 || rank < 0 || rank >= nrank) return fail(RH_EINVAL, "%s: rank %d of %d", who, rank, nrank);
  if (!q->w2 || !q->k2 || (q->nq > 0 && !q->qnode) || (q->nmq > 0 && (!q->qmemb || !q->qmstart || !q->kstart)) ||
      (q->nkr > 0 && (!q->kray || !q->hank)))
    return fail(RH_EINVAL, "%s: null table", who);
  if (work_bytes < rh_qtf_workspace_bytes(q)) return fail(RH_EINVAL, "%s: workspace too small", who);
  if (q->order != 0 && q->order != 1) return fail(RH_EINVAL, "%s: order=%d (0 or 1)", who, q->order);
  RH_HIP(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  rh::QtfWork wk = rh::qtf_carve(*q, work);
  const bool gemm = q->order == 1 && !ctx->qtf_direct;
  if (!gemm) wk.R = nullptr;                                 // the table kernels skip the GEMM operands
  if (flags & ~RH_QTF_INCIDENT_CACHED) return fail(RH_EINVAL, "%s: unknown flags 0x%x", who, flags);
  // RH_QTF_INCIDENT_CACHED: the incident-wave parts (the nodes' grad u / grad p / dw/dz tables,
  // the Kim & Yue tables, basis and pair-tile sums, the node GEMM basis, the zero K tails) are
  // already in `work` from an earlier call
  // with this q and these tiles; only the RAO-dependent tables and coefficients are formed
  const bool cached = (flags & RH_QTF_INCIDENT_CACHED) != 0;
  if (cached && !gemm) return fail(RH_EINVAL, "%s: the incident-wave cache is kept by the MFMA path only", who);
  const int n2p = rh::qtf_n2p(*q);
  const int nb = (n2p + 63) / 64;
  // This call's pair tiles (MFMA path): the rank's contiguous block [t0, t0 + blocks) of the
  // upper triangle's 16 x 16 tiles in row-major order, cut at the pair-count quantiles
  // (qtf_tile_block; raft/parallel.py qtf_tile_block mirrors it).  Its w1 rows are tile rows
  // T1(t0) .. T1(t0 + blocks - 1); the tables and coefficients of lower frequencies are not read.
  const int nt = n2p / 16;
  int t0 = 0, t1 = 0;
  qtf_tile_block(q->n2, rank, nrank, t0, t1);
  const int blocks = t1 - t0;
  auto row_of = [&](int t) {   // tile row of the t-th tile
    int T1 = 0;
    while (t >= nt - T1) {
      t -= nt - T1;
      ++T1;
    }
    return T1;
  };
  const int R0 = blocks > 0 ? row_of(t0) : 0, R1 = blocks > 0 ? row_of(t0 + blocks - 1) + 1 : 0;
  const int fb0 = gemm ? 16 * R0 / 64 : 0;   // first 64-frequency block read (the per-pair path: all)
  // the frequency row, node, waterline and KAY tables (+ GEMM basis and zero K tails): one launch
  // (rows in this order: frequency row, nodes, waterline members -- RAO-dependent -- then the
  // Kim & Yue rows, node GEMM basis and zero tails, which depend on the incident wave only)
  const int trows = 1 + q->nq + q->nmq + (cached ? 0 : q->nq + q->nkr + (gemm ? q->nq + rh::qtf_npad(*q) : 0));
  if (nb > fb0) {
    hipLaunchKernelGGL(rh::k_qtf_tables, dim3(nb - fb0, trows), dim3(64), 0, s, *q, wk, nw, w, Xi0, M66, fb0);
    RH_HIP(hipGetLastError());
  }
  if (gemm) {
    // the w1-side GEMM coefficients of the call's rows, the Kim & Yue tile sums (both need only
    // the tables), then the pair tiles: bilinear + potential GEMMs plus the Kim & Yue sums, and
    // the Hermitian fill (rh_qtf_mfma.hip)
    const int bx0 = 16 * R0 / 64, nbx = blocks > 0 ? (16 * R1 + 63) / 64 - bx0 : 0;
#ifdef RH_VARIANTS
    const bool sep = ctx->qtf_sep, t32 = ctx->qtf_t32;
#else
    constexpr bool sep = false, t32 = false;
#endif
    if (blocks > 0 && !sep) {
      // the Kim & Yue tiles and the GEMM coefficient blocks in one launch.  A call with few
      // tiles (a rank's share of a sharded QTF) gives each tile a workgroup and each part of a
      // member's rows a wave (S = kKayP); a whole QTF two tiles per workgroup (S = 1).  The same
      // bits either way (kay_tile), so a sharded QTF still equals the single-device one.
      const bool split = blocks <= RH_KAY_SPLIT_MAX_TILES(ctx->ncu);
      const int per = split ? rh::lk_tiles<rh::kKayP>() : rh::lk_tiles<1>();
      int nkb = (blocks + per - 1) / per, nly = 18 + q->nq + q->nmq;
#if RH_ABL_LK_NOKAY    // timing ablation: no Kim & Yue tiles (wrong results)
      nkb = 0;
#endif
      if (cached) nkb = 0;   // their tile sums KS are in the workspace already
#if RH_ABL_LK_NOCOEF   // timing ablation: no coefficient blocks (wrong results)
      nly = 0;
#endif
      if (split)
        hipLaunchKernelGGL(rh::k_qtf_lk<rh::kKayP>, dim3(nkb + nbx * nly), dim3(rh::kLkThreads), 0, s, *q, wk, M66, t0,
                           blocks, nkb, bx0, nbx);
      else
        hipLaunchKernelGGL(rh::k_qtf_lk<1>, dim3(nkb + nbx * nly), dim3(rh::kLkThreads), 0, s, *q, wk, M66, t0, blocks,
                           nkb, bx0, nbx);
      RH_HIP(hipGetLastError());
    } else {
#ifdef RH_VARIANTS
      hipLaunchKernelGGL(rh::k_qtf_lcoef, dim3(nb, 18 + q->nq + q->nmq), dim3(512), 0, s, *q, wk, M66);
      RH_HIP(hipGetLastError());
      if (blocks > 0) {
        hipLaunchKernelGGL(rh::k_qtf_kay, dim3(blocks), dim3(rh::kKayThreads), 0, s, *q, wk, t0);
        RH_HIP(hipGetLastError());
      }
#endif
    }
    if (blocks > 0) {
      if (nrank == 1 && mirror && t32) {   // variant builds, a whole QTF: 32 x 32 pair tiles
#ifdef RH_VARIANTS
        const int nt32 = (nt + 1) / 2;
        hipLaunchKernelGGL(rh::k_qtf_gemm32, dim3(nt32 * (nt32 + 1)), dim3(384), 0, s, *q, wk, qtf);
#endif
      } else {
        hipLaunchKernelGGL(rh::k_qtf_gemm, dim3(6 / rh::kGD * blocks), dim3(rh::kGThreads), 0, s, *q, wk, qtf, t0, mirror);
      }
      RH_HIP(hipGetLastError());
    }
    return RH_OK;
  }
  // per-pair kernel; a sharded call computes the whole triangle (a superset of the rank's tiles)
  rank = 0;
  nrank = 1;
  const int rows = (q->n2 + nrank - 1) / nrank;     // snake rounds (k_qtf_pairs skips i1 >= n2)
  if (rows > 0) {
    const dim3 grid((q->n2 + rh::kQtfTile - 1) / rh::kQtfTile, rows);
    // waves per 64 pairs (rh_set_qtf_waves).  Auto = 4.  With the tiles starting on the
    // diagonal, 4 waves per tile are the fastest on one GPU too (C3: 0.294 ms against 0.33 ms
    // with 1 or 2 waves, profiles/r01_v11/qtf_diag_tiles_ab.txt), and a sharded grid needs
    // them to keep the CUs busy.
    const int waves = ctx->qtf_waves == 0 ? 4 : ctx->qtf_waves;
    switch (waves) {
      case 1:
        hipLaunchKernelGGL(rh::k_qtf_pairs<1>, grid, dim3(rh::kQtfTile), 0, s, *q, wk, qtf, rank, nrank, mirror);
        break;
      case 2:
        hipLaunchKernelGGL(rh::k_qtf_pairs<2>, grid, dim3(2 * rh::kQtfTile), 0, s, *q, wk, qtf, rank, nrank, mirror);
        break;
      default:
        hipLaunchKernelGGL(rh::k_qtf_pairs<4>, grid, dim3(4 * rh::kQtfTile), 0, s, *q, wk, qtf, rank, nrank, mirror);
    }
    RH_HIP(hipGetLastError());
  }
  return RH_OK;
}

int rh_qtf_slender(rh_ctx* ctx, const rh_qtf_design* q, int nw, const double* w, const rh_c128* Xi0, const double* M66,
                   rh_c128* qtf, void* work, long long work_bytes, rh_stream stream) {
  return qtf_launch(ctx, q, nw, w, Xi0, M66, 0, 1, 1, qtf, work, work_bytes, stream, "rh_qtf_slender");
}

int rh_qtf_slender_ext(rh_ctx* ctx, const rh_qtf_design* q, int nw, const double* w, const rh_c128* Xi0,
                       const double* M66, rh_c128* qtf, void* work, long long work_bytes, int flags, rh_stream stream) {
  return qtf_launch(ctx, q, nw, w, Xi0, M66, 0, 1, 1, qtf, work, work_bytes, stream, "rh_qtf_slender_ext", flags);
}

int rh_qtf_slender_rows(rh_ctx* ctx, const rh_qtf_design* q, int nw, const double* w, const rh_c128* Xi0,
                        const double* M66, int rank, int nrank, rh_c128* qtf, void* work, long long work_bytes,
                        rh_stream stream) {
  return qtf_launch(ctx, q, nw, w, Xi0, M66, rank, nrank, 0, qtf, work, work_bytes, stream, "rh_qtf_slender_rows");
}

int rh_qtf_hankel(rh_ctx* ctx, int n2, const double* k2, int nkr, const double* R, rh_c128* hank, rh_stream stream) {
  if (!ctx || n2 < 1 || nkr < 0 || (nkr > 0 && (!k2 || !R || !hank))) return fail(RH_EINVAL, "rh_qtf_hankel: bad argument");
  if (nkr == 0) return RH_OK;
  RH_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(rh::k_qtf_hankel, dim3((n2 + 63) / 64, nkr), dim3(64), 0, (hipStream_t)stream, n2, k2, nkr, R, hank);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_qtf_hermitian_fill(rh_ctx* ctx, int n2, rh_c128* qtf, rh_stream stream) {
  if (!ctx || !qtf || n2 < 1) return fail(RH_EINVAL, "rh_qtf_hermitian_fill: bad argument");
  RH_HIP(hipSetDevice(ctx->device));
  const size_t n = (size_t)n2 * n2 * 6;
  hipLaunchKernelGGL(rh::k_qtf_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n2, qtf);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_force_2nd(rh_ctx* ctx, int n2, const double* w2, const rh_c128* qtf, int nw, const double* w, double dw,
                 const double* S0, double* f, double* f_mean, rh_stream stream) {
  if (!ctx || !w2 || !qtf || !w || !S0 || !f || !f_mean) return fail(RH_EINVAL, "rh_force_2nd: null argument");
  if (n2 < 2 || nw < 2 || !(dw > 0)) return fail(RH_EINVAL, "rh_force_2nd: bad sizes");
  RH_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(rh::k_force2nd, dim3(nw), dim3(256), 0, (hipStream_t)stream, n2, w2, qtf, nw, w, dw, S0, f, f_mean);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_force_2nd_batch(rh_ctx* ctx, int ncase, int n2, const double* w2, const rh_c128* qtf, int nq, const int* qidx,
                       int nw, const double* w, double dw, const double* S0, rh_c128* f, double* f_mean,
                       rh_stream stream) {
  if (!ctx || !w2 || !qtf || !w || !S0 || !f || !f_mean) return fail(RH_EINVAL, "rh_force_2nd_batch: null argument");
  if (ncase < 0 || n2 < 2 || nw < 2 || nq < 1 || !(dw > 0)) return fail(RH_EINVAL, "rh_force_2nd_batch: bad sizes");
  if (ncase == 0) return RH_OK;
  if (ncase > 65535) return fail(RH_EINVAL, "rh_force_2nd_batch: ncase=%d > 65535 per call", ncase);
  RH_HIP(hipSetDevice(ctx->device));
  hipLaunchKernelGGL(rh::k_force2nd_batch, dim3(nw, ncase), dim3(256), 0, (hipStream_t)stream, n2, w2, qtf, qidx, nq,
                     nw, w, dw, S0, f, f_mean);
  RH_HIP(hipGetLastError());
  return RH_OK;
}

int rh_force_2nd_spectrum(rh_ctx* ctx, int n2, const double* w2, const rh_c128* qtf, int nw, const double* w,
                          double dw, const double* S0, double* Sf, double* f, double* f_mean, rh_stream stream) {
  if (!ctx || !w2 || !qtf || !w || !S0 || !Sf || !f || !f_mean)
    return fail(RH_EINVAL, "rh_force_2nd_spectrum: null argument");
  if (n2 < 2 || nw < 2 || !(dw > 0)) return fail(RH_EINVAL, "rh_force_2nd_spectrum: bad sizes");
  RH_HIP(hipSetDevice(ctx->device));
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(rh::k_force2nd_spec, dim3(n2), dim3(256), 0, s, n2, w2, qtf, nw, w, S0, Sf, f_mean);
  RH_HIP(hipGetLastError());
  hipLaunchKernelGGL(rh::k_force2nd_spec_out, dim3((6 * nw + 255) / 256), dim3(256), 0, s, n2, w2, nw, w, dw, Sf, f);
  RH_HIP(hipGetLastError());
  return RH_OK;
}


// ---------------------------------------------------------------- native design preparation
namespace {
// Worker threads kept across rh_prep_designs calls.  Spawning and joining 16 threads per call
// cost 0.3-0.7 ms of host time, paid by every design block of a sweep and in full by its first
// block, which nothing overlaps.  One job at a time (callers queue on call_mx); the caller runs the
// job too.  A forked child gets a new pool: the parent's threads do not exist there, so the old
// pool is left alone (never destroyed, as is the process-lifetime pool itself).
struct PrepPool {
  explicit PrepPool(pid_t p) : pid(p) {}
  const pid_t pid;
  std::mutex call_mx, mx;
  std::condition_variable cv_start, cv_done;
  std::vector<std::thread> th;
  const std::function<void()>* job = nullptr;
  unsigned long gen = 0;
  int want = 0, pending = 0;

  void worker(int idx) {
    unsigned long seen = 0;
    std::unique_lock<std::mutex> lk(mx);
    for (;;) {
      cv_start.wait(lk, [&] { return gen != seen; });
      seen = gen;
      if (idx >= want) continue;
      const std::function<void()>* f = job;
      lk.unlock();
      (*f)();
      lk.lock();
      if (--pending == 0) cv_done.notify_all();
    }
  }
  // fn on nt threads (the caller and nt - 1 workers), back when every one has returned
  void run(int nt, const std::function<void()>& fn) {
    std::lock_guard<std::mutex> call(call_mx);
    const int helpers = nt - 1;
    {
      std::lock_guard<std::mutex> lk(mx);
      while ((int)th.size() < helpers) {
        const int idx = (int)th.size();
        th.emplace_back([this, idx] { worker(idx); });
      }
      job = &fn;
      want = helpers;
      pending = helpers;
      ++gen;
    }
    cv_start.notify_all();
    fn();
    std::unique_lock<std::mutex> lk(mx);
    cv_done.wait(lk, [&] { return pending == 0; });
    job = nullptr;
  }
  static PrepPool& get() {   // this process's pool
    static std::mutex m;
    static PrepPool* pool = nullptr;
    std::lock_guard<std::mutex> lk(m);
    if (!pool || pool->pid != getpid()) pool = new PrepPool(getpid());
    return *pool;
  }
};
}  // namespace

int rh_prep_designs(int ndesign, const double* spec, const long long* spec_off, int nw, const double* w,
                    const double* k, int nthreads, rh_prep** out) {
  if (!out) return fail(RH_EINVAL, "rh_prep_designs: null out");
  *out = nullptr;
  if (ndesign < 0 || (ndesign > 0 && (!spec || !spec_off)) || nw < 2 || !w || !k)
    return fail(RH_EINVAL, "rh_prep_designs: bad arguments (ndesign=%d, nw=%d)", ndesign, nw);
  auto* p = new rh_prep();
  p->res.resize(ndesign);
  int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  nt = std::max(1, std::min({nt, 64, std::max(ndesign, 1)}));
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int i = next++; i < ndesign; i = next++) {
      try {   // an exception must not leave a worker thread (std::terminate): it becomes RH_EINVAL
        rhp::prep_one(spec + spec_off[i], spec_off[i + 1] - spec_off[i], nw, w, k, p->res[i]);
      } catch (const std::exception& e) {
        p->res[i].ok = 0;
        p->res[i].err = std::string("rh_prep_designs: ") + e.what();
      } catch (...) {
        p->res[i].ok = 0;
        p->res[i].err = "rh_prep_designs: unknown exception";
      }
    }
  };
  if (nt == 1) {
    work();
  } else {
    const std::function<void()> job(work);
    PrepPool::get().run(nt, job);
  }
  for (int i = 0; i < ndesign; ++i)
    if (!p->res[i].ok) {
      const std::string e = p->res[i].err;
      delete p;
      return fail(RH_EINVAL, "rh_prep_designs: design %d: %s", i, e.c_str());
    }
  long long o = 0, mo = 0;
  for (auto& r : p->res) {
    p->off.push_back(o);
    p->moff.push_back(mo);
    o += (long long)r.packed.size();
    mo += (long long)r.mstart.size();
  }
  p->off.push_back(o);
  p->moff.push_back(mo);
  *out = p;
  return RH_OK;
}

int rh_prep_layout(const rh_prep* p, long long* info) {
  if (!p || !info) return fail(RH_EINVAL, "rh_prep_layout: null argument");
  const int nd = (int)p->res.size();
  for (int i = 0; i < nd; ++i) {
    long long* r = info + 5 * i;
    r[0] = p->off[i];
    r[1] = p->off[i + 1] - p->off[i];
    r[2] = p->moff[i];
    r[3] = p->res[i].nn;
    r[4] = p->res[i].nm;
  }
  info[5 * nd] = p->off[nd];
  info[5 * nd + 1] = p->moff[nd];
  return RH_OK;
}

int rh_prep_copy(const rh_prep* p, double* packed, int* mstart, double* statics) {
  if (!p || !packed || !mstart) return fail(RH_EINVAL, "rh_prep_copy: null argument");
  for (size_t i = 0; i < p->res.size(); ++i) {
    const auto& r = p->res[i];
    std::copy(r.packed.begin(), r.packed.end(), packed + p->off[i]);
    std::copy(r.mstart.begin(), r.mstart.end(), mstart + p->moff[i]);
    if (statics) std::copy(r.statics, r.statics + 5 * 36, statics + 5 * 36 * i);
  }
  return RH_OK;
}

long long rh_prep_imat(const rh_prep* p, int design, rh_c128* imat) {
  if (!p || design < 0 || design >= (int)p->res.size()) return fail(RH_EINVAL, "rh_prep_imat: bad arguments");
  const auto& v = p->res[design].imat;
  if (imat && !v.empty()) std::memcpy(imat, v.data(), v.size() * sizeof(double));
  return (long long)(v.size() / 2);
}

// ------------------------------------------------------------------ QTF tables (host)
int rh_qtf_tables(int nmemb, const double* rec, long long rec_len, double beta, double* out, long long cap, int* iout,
                  long long capi, int* counts) {
  if (nmemb < 0 || (nmemb > 0 && !rec) || rec_len < 0 || !out || !iout || !counts)
    return fail(RH_EINVAL, "rh_qtf_tables: bad arguments (nmemb=%d)", nmemb);
  std::vector<rhq::MemberRec> mems(nmemb);
  long long off = 0;
  for (int i = 0; i < nmemb; ++i) {
    const long long n = rhq::parse(rec + off, rec_len - off, mems[i]);
    if (n < 0) return fail(RH_EINVAL, "rh_qtf_tables: malformed member record %d", i);
    off += n;
  }
  if (off != rec_len) return fail(RH_EINVAL, "rh_qtf_tables: %lld doubles after the last member record", rec_len - off);
  long long nq, nmq, nkr;
  rhq::count(mems, nq, nmq, nkr);
  if (rhq::kQN * nq + rhq::kQM * nmq + rhq::kKR * nkr > cap || 2 * (nmq + 1) > capi)
    return fail(RH_EINVAL, "rh_qtf_tables: output capacity too small (%lld doubles, %lld ints)", cap, capi);
  const rhq::Tables T{out, out + rhq::kQN * nq, out + rhq::kQN * nq + rhq::kQM * nmq, iout, iout + nmq + 1, nq, nmq, nkr};
  try {
    rhq::build(mems, beta, T);
  } catch (const std::exception& e) {
    return fail(RH_EINVAL, "%s", e.what());
  }
  counts[0] = (int)nq;
  counts[1] = (int)nmq;
  counts[2] = (int)nkr;
  return RH_OK;
}

void rh_prep_free(rh_prep* p) { delete p; }

}  // extern "C"
