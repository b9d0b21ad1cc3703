/* rafthip.h -- C-ABI of librafthip.so, the MI355X (gfx950) implementation of RAFT's
 * frequency-domain response solve (lucas-carmo/RAFT-testStuff, RAFT v1.3.1 fork).
 *
 * The reference is pure Python/NumPy: it has no FFI of its own.  Each
 * entry point below replaces one reference method (or the loop nest inside it); the
 * reference-side binding is the ctypes wrapper in raft-teststuff_amd/raft/_native.py,
 * shown for maintainers in INTEGRATION.md.
 *
 * Conventions
 *   - All array pointers inside the structs are DEVICE pointers owned by the caller
 *     (PyTorch-ROCm tensors used as plain buffers).  The library never frees them.
 *   - complex128 == interleaved {re, im} doubles (rh_c128), same as torch.complex128.
 *   - Every call is stream-ordered on the given hipStream_t (pass NULL for the null
 *     stream) and returns immediately; the caller synchronises.
 *   - Return codes: RH_OK, RH_EINVAL (-> ValueError), RH_ENAN ("Nan detected in response
 *     vector Xi.", raft/raft_model.py:956-957), RH_ESINGULAR (-> LinAlgError), RH_EHIP.
 *     rh_last_error() returns the thread-local message of the last failure.
 *   - No C++ exception crosses this boundary.
 */
#ifndef RAFTHIP_H
#define RAFTHIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define RH_OK 0
#define RH_EINVAL (-1)
#define RH_ENAN (-2)
#define RH_ESINGULAR (-3)
#define RH_EHIP (-4)

/* per-case status words written by rh_solve_cases */
#define RH_CASE_CONVERGED 1
#define RH_CASE_NOT_CONVERGED 0
#define RH_CASE_NAN (-2)
#define RH_CASE_SINGULAR (-3)

/* spectrum codes (raft/raft_fowt.py:1000-1014) */
#define RH_SPEC_JONSWAP 0
#define RH_SPEC_UNIT 1
#define RH_SPEC_CONSTANT 2
#define RH_SPEC_NONE 3

/* node-table fields: struct-of-arrays, field f of node n at node[f*nn + n].
 * Built on the host from the member strip discretisation
 * (raft/raft_member.py:169-304, 877-1088) for SUBMERGED nodes only (r_z < 0,
 * raft/raft_fowt.py:1104,1188), in reference member/node order. */
enum rh_node_field {
  RH_NF_RX = 0, RH_NF_RY, RH_NF_RZ,      /* absolute node position (wave phase / depth)   */
  RH_NF_XX, RH_NF_XY, RH_NF_XZ,          /* position relative to the PRP (moments, motion) */
  RH_NF_QX, RH_NF_QY, RH_NF_QZ,          /* member axis q                                  */
  RH_NF_P1X, RH_NF_P1Y, RH_NF_P1Z,       /* transverse p1                                  */
  RH_NF_P2X, RH_NF_P2Y, RH_NF_P2Z,       /* transverse p2                                  */
  RH_NF_AQ, RH_NF_AP1, RH_NF_AP2, RH_NF_AEND,      /* drag areas, raft/raft_fowt.py:1200-1238 */
  RH_NF_CDQ, RH_NF_CDP1, RH_NF_CDP2, RH_NF_CDEND,  /* interpolated Cd, :1191-1194           */
  RH_NF_CIRC,                            /* 1.0 circular, 0.0 rectangular                   */
  RH_NF_AI,                              /* signed axial area for dynamic pressure (a_i)    */
  RH_NF_MCF,                             /* 1.0 if Imat is frequency dependent (MacCamy-Fuchs) */
  RH_NF_I00, RH_NF_I01, RH_NF_I02, RH_NF_I10, RH_NF_I11, RH_NF_I12, RH_NF_I20, RH_NF_I21, RH_NF_I22,
  RH_NF_T,                               /* axial coordinate of the node from its member's end A */
  RH_NF_COUNT
};

/* member-table fields (struct-of-arrays [RH_MF_COUNT][nm]) for members with submerged nodes.
 * Every RAFT member is straight, so a node at axial coordinate t has r = rA + t q and
 *   q.(th x r) = th.(rA x q),  p1.(th x r) = th.(rA x p1) + t p2.th,  p2.(th x r) = th.(rA x p2) - t p1.th
 * (p2 = q x p1, raft/raft_member.py:276-277): the motion-dependent part of every node's
 * relative velocity is a per-(member, bin) quantity plus t times another one. */
enum rh_member_field {
  RH_MF_CQ0 = 0,                         /* cq = [q ; rA x q]   (6) */
  RH_MF_C10 = 6,                         /* c1 = [p1; rA x p1]  (6) */
  RH_MF_C20 = 12,                        /* c2 = [p2; rA x p2]  (6) */
  RH_MF_QQ = 18, RH_MF_PP1, RH_MF_PP2,   /* |q|^2, |p1|^2, |p2|^2 */
  RH_MF_COUNT
};

typedef struct { double re, im; } rh_c128;
typedef struct rh_ctx rh_ctx;
typedef void* rh_stream; /* hipStream_t */

/* One FOWT design on one frequency grid.  Replaces the per-FOWT state the reference
 * keeps on FOWT/Member objects (raft/raft_fowt.py:22-257, raft/raft_member.py:16-304). */
typedef struct {
  int nw;                 /* frequency bins                                   */
  int nn;                 /* submerged strip nodes                            */
  int nhead;              /* headings tabulated in uhat/finer                 */
  int mb_per_bin;         /* 0: M,B are [36]; 1: M,B are [nw][36]             */
  double dw, depth, rho, g;
  double pdyn_rho_g;      /* rho*g used for dynamic pressure: the reference calls getWaveKin
                             with its DEFAULT rho=1025, g=9.81 (raft/raft_fowt.py:1109) */
  const double* w;        /* [nw] rad/s                                       */
  const double* k;        /* [nw] wave numbers (raft/helpers.py:295)          */
  const double* node;     /* [RH_NF_COUNT][nn]                                */
  int nm;                 /* members with submerged nodes                     */
  const double* memb;     /* [RH_MF_COUNT][nm]                                */
  const int* mstart;      /* [nm+1] first node of each member (nodes are member-contiguous) */
  const rh_c128* imat_mcf;/* [nn][9][nw] frequency-dependent Imat (MCF nodes), or NULL */
  const rh_c128* uhat;    /* [nhead][nn][3][nw] unit-amplitude wave velocity (rh_wave_tables) */
  const rh_c128* finer;   /* [nhead][6][nw]     unit-amplitude inertial excitation        */
  const rh_c128* kproj;   /* [nhead][nn][3][nw] projections (q.uhat, p1.uhat, p2.uhat)    */
  const double* M;        /* mass + added mass      M_lin (raft/raft_model.py:911) */
  const double* B;        /* linear damping         B_lin (:912)                   */
  const double* C;        /* [36] stiffness         C_lin (:913)                   */
} rh_design;

/* A batch of sea-state cases (the per-case loop of Model.analyzeCases,
 * raft/raft_model.py:267-291).  All arrays are device arrays of length ncase. */
typedef struct {
  int ncase;
  const int* design;      /* index into the designs array                     */
  const int* head;        /* heading-table index of sea state 0               */
  const int* spectrum;    /* RH_SPEC_*                                         */
  const double* Hs;       /* wave_height                                       */
  const double* Tp;       /* wave_period                                       */
  const double* gamma;    /* wave_gamma (0 -> IEC automatic, raft/helpers.py:636-643) */
  int nIter;              /* settings.nIter; the loop runs nIter+1 times (raft/raft_model.py:861) */
  double XiStart;         /* settings.XiStart                                  */
  double tol;             /* solveDynamics(tol=0.01)                           */
  const rh_c128* fext;    /* [ncase][6][nw] extra excitation added to F_lin (F_BEM, Fhydro_2nd;
                             raft/raft_model.py:914), or NULL                  */
  const int* order;       /* optional launch order (a permutation of 0..ncase-1, e.g. cases sorted
                             by design/heading so each XCD's L2 holds few wave tables), or NULL */
  const rh_c128* Xi_init; /* [ncase][6][nw] initial XiLast instead of XiStart, or NULL          */
  int first_iter;         /* initial value of the iteration counter (1 for the second pass of
                             potSecOrder=1, raft/raft_model.py:973-1000), normally 0         */
  const int* group_start; /* optional [ngroup+1] device array of offsets into `order`: group g
                             is order[group_start[g] .. group_start[g+1]), 1..rh_group_cases()
                             cases that share design AND heading index, solved in lock-step by
                             one workgroup.  Ignored when rh_group_cases() == 1 (the shipped
                             library: one case per workgroup).  NULL -> one case per workgroup. */
  int ngroup;
} rh_cases;

/* Outputs of rh_solve_cases (device buffers; NULL = not wanted). */
typedef struct {
  rh_c128* Xi;            /* [ncase][6][nw] response to sea state 0, or NULL when only the
                             linearisation is wanted (then psd, std and rao must be NULL too;
                             nw <= 1024 only) */
  rh_c128* Xi_last;       /* [ncase][6][nw] scratch for the relaxed iterate (required) */
  int* iters;             /* [ncase] linear solves executed (required)         */
  int* status;            /* [ncase] RH_CASE_* (required)                      */
  double* zeta;           /* [ncase][nw] wave amplitudes sqrt(2 S dw)          */
  double* B_drag;         /* [ncase][36] final linearised drag damping         */
  double* Bmat;           /* [ncase][nn_max][9] final per-node drag matrices; nn_max = the
                             largest nn of the call's designs (a case with fewer nodes
                             leaves the rest of its rows untouched)              */
  double* psd;            /* [ncase][6][nw] motion PSD (rotations in deg^2), raft/raft_fowt.py:1836-1874 */
  double* std;            /* [ncase][6] motion RMS                             */
  rh_c128* rao;           /* [ncase][6][nw] Xi / zeta (raft/helpers.py:665)   */
  rh_c128* Z;             /* [ncase][nw][36] final impedance (fowt.Z, raft/raft_model.py:1013) */
  rh_c128* Xi_prev;       /* [ncase][6][nw] XiLast of the final iteration (the un-relaxed iterate the
                             potSecOrder=1 second pass restarts from, Q6), or NULL */
  double* margin;         /* [ncase] closest call of the convergence test, or NULL: over the
                             executed iterations, the value m = max_{bin,dof} |Xi-XiLast|/(|Xi|+tol)
                             - tol (raft/raft_model.py:961-962) with the smallest |m|.  m < 0 means
                             that iteration passed.  |m| near rounding level marks a case whose
                             iteration count could flip between implementations. */
  rh_c128* F_wave;        /* [ncase][6][nw] the wave excitation of sea state 0 with the final
                             linearisation, zeta (F_iner + F_drag(Bmat)) (+ fext), or NULL: the
                             F_wave of the coupled-array solve (raft/raft_model.py:1049-1061),
                             formed by the fixed point itself, so rh_array_solve_stats needs no
                             excitation launch */
} rh_solve_out;

const char* rh_last_error(void);
int rh_ctx_create(int device, rh_ctx** out);
int rh_ctx_destroy(rh_ctx* ctx);
int rh_version(void);

/* Kernel selection for rh_solve_cases on this context (not part of the reference API):
 * 0 = automatic (the LDS-resident fast path when nw <= 1024 and the node tables fit in LDS;
 * else the general kernel), 1 = always the general kernel.  Used by the parity tests to
 * cross-check the device paths on the same inputs.  (Builds with -DRH_VARIANTS, made by
 * tools/build_variants.sh for on-box A/B timing only, also accept 2..5: the lock-step grouped
 * kernel, the lane-pair kernel and the two-pass launch, all measured slower) */
int rh_set_solver(rh_ctx* ctx, int which);

/* Iteration-0 sums as a batch GEMM on this context (not part of the reference API; default 0).
 * The shipped library accepts only 0 (every case forms them in its own workgroup) and refuses 1
 * with RH_EINVAL: k_a0_sums, which forms phase A of the first iteration of every case that starts
 * from XiStart as one MFMA launch, was measured slower on C2 and C4 and is built
 * only into variant libraries (tools/build_variants.sh, -DRH_VARIANTS), where 1 enables it. */
int rh_set_a0(rh_ctx* ctx, int on);

/* Largest grid (bins) rh_solve_cases can solve with rh_solve_out.Xi = NULL (the linearisation
 * only); larger grids keep their iterate in the Xi output and need it (RH_EINVAL otherwise). */
int rh_solve_noxi_max_bins(void);

/* Maximum cases per group of rh_cases.group_start: 1 in the shipped library (no grouped
 * kernel; group_start is then ignored). */
int rh_group_cases(void);

/* Waves per 64 (w1, w2) pairs in the QTF pair kernel on this context (not part of the
 * reference API): 1, 2, 4, or 0 (default: auto, currently 4 waves, the fastest measured
 * both on one GPU and for a row-sharded grid).
 * The per-pair terms are split over the waves and summed in a fixed order, so the result
 * differs between settings only by rounding.
 * Used by the tests and the kernel-tuning scripts. */
int rh_set_qtf_waves(rh_ctx* ctx, int waves);

/* QTF pair-sum path of this context: 0 (default) = FP64 MFMA GEMMs on 16 x 16 pair tiles when
 * the grid is sorted (rh_qtf_design.order == 1), 1 = the per-pair kernel k_qtf_pairs (parity
 * cross-checks).  Variant libraries (tools/build_variants.sh) also take 2 = the GEMMs with
 * 32 x 32 tiles for a whole QTF and 3 = the GEMM coefficients (k_qtf_lcoef) and the Kim & Yue
 * sums (k_qtf_kay) as two launches (both measured slower, the same bits as 0); the shipped
 * library refuses them with RH_EINVAL. */
int rh_set_qtf_path(rh_ctx* ctx, int path);

/* Unit-amplitude wave kinematics and strip-theory inertial excitation per heading.
 * Replaces the node loops of FOWT.calcHydroExcitation (raft/raft_fowt.py:1098-1124)
 * and helpers.getWaveKin (raft/helpers.py:105-154):
 *   uhat[h][n][:,b]  = u(zeta0 = 1, beta[h]) at node n, bin b
 *   finer[h][:,b]    = sum_n translateForce3to6DOF(Imat_n(b) iw uhat + pDyn a_i q, r_n)
 *   kproj[h][n][:,b] = (q.uhat, p1.uhat, p2.uhat) of node n (the only form the drag loop needs)
 * so that for a sea state with amplitudes zeta(b): u = zeta*uhat, F_hydro_iner = zeta*finer.
 * beta: device [nhead] (rad).  Outputs are device buffers sized as in rh_design. */
int rh_wave_tables(rh_ctx* ctx, const rh_design* d, const double* beta,
                   rh_c128* uhat, rh_c128* finer, rh_c128* kproj, rh_stream stream);

/* rh_wave_tables for many designs in ONE launch: design i tabulates designs[i].nhead headings
 * beta[i * hstride + h] (rad) into the tables its descriptor points at (uhat, finer, kproj,
 * written).  The per-design part of a design sweep (C5) as a single grid.  A design's uhat
 * may be NULL: its velocity table is then not stored, and only rh_solve_cases (whose fixed
 * point reads kproj and finer) accepts the design afterwards; the entry points that read uhat
 * return RH_EINVAL for it. */
int rh_wave_tables_batch(rh_ctx* ctx, const rh_design* designs, int ndesign, const double* beta, int hstride,
                         rh_stream stream);

/* Drag-linearisation fixed point + per-bin Z assemble / pivoted LU solve for a batch of
 * cases, one workgroup per case.  Replaces Model.solveDynamics' per-FOWT iteration
 * (raft/raft_model.py:877-1013) including FOWT.calcHydroLinearization (raft/raft_fowt.py:
 * 1152-1266), calcDragExcitation (:1270-1293) and the motion part of saveTurbineOutputs
 * (:1831-1875).  designs: HOST array of ndesign descriptors (their pointers are device
 * pointers); all designs must share nw.  cases: HOST struct with DEVICE arrays. */
int rh_solve_cases(rh_ctx* ctx, const rh_design* designs, int ndesign, const rh_cases* cases,
                   const rh_solve_out* out, rh_stream stream);

/* Response to additional sea states of a solved case with the linearisation frozen:
 * Xi_h = Z^-1 (zeta_h finer_h + zeta_h sum_n T_n Bmat_n uhat_h,n)  (raft/raft_model.py:1049-1065).
 * zeta: device [ncase][nw]; head: device [ncase] heading-table index; B_drag [ncase][36] and
 * Bmat [ncase][nn_max][9] as produced by rh_solve_cases (nn_max: the largest nn of the designs
 * passed here); Xi out: [ncase][6][nw]. */
int rh_heading_response(rh_ctx* ctx, const rh_design* designs, int ndesign, int ncase,
                        const int* design_idx, const int* head, const double* zeta,
                        const double* B_drag, const double* Bmat, rh_c128* Xi, rh_stream stream);

/* rh_heading_response with the Bmat row stride explicit and an extra excitation:
 * Xi_h = Z^-1 (zeta_h finer_h + zeta_h sum_n T_n Bmat_n uhat_h,n + fext_h), the F_wave of
 * raft/raft_model.py:1061 with the second-order force Fhydro_2nd[ih] of that sea state
 * (:1059-1060, an external .12d QTF; FOWT.calcHydroForce_2ndOrd).  bmat_nn: the node stride of
 * Bmat (0 = the largest nn of the designs passed; RH_EINVAL when smaller than that), so a call
 * over a subset of the designs of the rh_solve_cases call that wrote Bmat reads it correctly.
 * fext: [ncase][6][nw] or NULL.  A case whose design or heading index is out of range gets NaN
 * rows (no table is read). */
int rh_heading_response_ext(rh_ctx* ctx, const rh_design* designs, int ndesign, int ncase,
                            const int* design_idx, const int* head, const double* zeta,
                            const double* B_drag, const double* Bmat, int bmat_nn, const rh_c128* fext,
                            rh_c128* Xi, rh_stream stream);

/* Wave excitation of solved cases with the final linearisation, without the solve:
 * F = zeta_h finer_h + zeta_h sum_n T_n Bmat_n uhat_h,n  -- F_wave of the system solve of an
 * array (raft/raft_model.py:1049-1061).  Arguments as rh_heading_response; F out: [ncase][6][nw]. */
int rh_wave_excitation(rh_ctx* ctx, const rh_design* designs, int ndesign, int ncase, const int* design_idx,
                       const int* head, const double* zeta, const double* Bmat, rh_c128* F, rh_stream stream);

/* Stand-alone FOWT.calcHydroLinearization(Xi) + calcDragExcitation (raft/raft_fowt.py:1152-1293)
 * for one design and one sea state: Xi [6][nw], zeta [nw] (u = zeta*uhat[head]).
 * Outputs: B_drag [36], Bmat [nn][9], F_drag [6][nw]. */
int rh_linearize(rh_ctx* ctx, const rh_design* d, int head, const rh_c128* Xi, const double* zeta,
                 double* B_drag, double* Bmat, rh_c128* F_drag, rh_stream stream);

/* Bin-sharded drag fixed point of ONE case, bins split over ranks.
 * The only coupling across bins is the per-node RMS sum (raft/raft_fowt.py:1214-1220) and
 * the all-bins convergence test (raft/raft_model.py:962).  One iteration on each rank:
 *  1. rh_lin_partial_sums: per-node sums of |vrel|^2 over this rank's bins [bin_lo, bin_hi)
 *     of Xi_last [6][nw] -> sums [nn][3] (q, p or p1, p2);
 *  2. the caller all-reduces (sums) the sums over ranks;
 *  3. rh_bin_step: Bmat [nn][9] and B_drag [36] from the global sums (raft/raft_fowt.py:
 *     1223-1250), then for bins [bin_lo, bin_hi): F_lin + F_drag (+ fext [6][nw], or NULL),
 *     Z(w) and its LU solve -> Xi, tolCheck against Xi_last and the 0.2/0.8 relaxation of
 *     Xi_last in place (raft/raft_model.py:942-991).  flags: device int[3], zeroed by the
 *     caller, set to 1 if some bin is [0] not converged, [1] NaN, [2] singular;
 *  4. the caller all-reduces (max) the flags.
 * Host driver: raft/parallel.py solve_bins_sharded. */
int rh_lin_partial_sums(rh_ctx* ctx, const rh_design* d, int head, const rh_c128* Xi_last, const double* zeta,
                        int bin_lo, int bin_hi, double* sums, rh_stream stream);
int rh_bin_step(rh_ctx* ctx, const rh_design* d, int head, const double* zeta, const rh_c128* fext,
                const double* sums, double tol, int bin_lo, int bin_hi, double* Bmat, double* B_drag,
                rh_c128* Xi, rh_c128* Xi_last, int* flags, rh_stream stream);

/* Drag excitation for given node matrices (FOWT.calcDragExcitation, raft/raft_fowt.py:1270-1293). */
int rh_drag_excitation(rh_ctx* ctx, const rh_design* d, int head, const double* zeta,
                       const double* Bmat, rh_c128* F_drag, rh_stream stream);

/* Sea-state amplitudes for ncase spectra on one grid (raft/raft_fowt.py:995-1014, JONSWAP
 * raft/helpers.py:606-663): S [ncase][nw] (may be NULL) and zeta = sqrt(2 S dw) [ncase][nw]. */
int rh_sea_state(rh_ctx* ctx, int ncase, int nw, const double* w, double dw, const int* spectrum,
                 const double* Hs, const double* Tp, const double* gamma, double* S, double* zeta,
                 rh_stream stream);

/* Motion statistics over nrow excitation rows (raft/raft_fowt.py:1831-1875):
 * Xi [ncase][nrow][6][nw] -> psd [ncase][6][nw], std [ncase][6]. */
int rh_motion_stats(rh_ctx* ctx, int ncase, int nrow, int nw, double dw, const rh_c128* Xi,
                    double* psd, double* std, rh_stream stream);

/* Derived response channels (FOWT.saveTurbineOutputs, raft/raft_fowt.py:1900-1971 with zero
 * aero loads -- nacelle acceleration AxRNA, tower-base bending moment Mbase -- and mooring
 * tensions J_moor Xi, :1884-1898).  Channel k is a real linear combination of the DOFs with
 * an optional w^2 term: x_k(row, b) = sum_d a[k][d] Xi[row][d][b] + w_b^2 sum_d c[k][d] Xi[row][d][b].
 * Xi [ncase][nrow][ndof][nw], w [nw], coef [nch][2][ndof] = {a, c} -> psd [ncase][nch][nw]
 * = sum_row 0.5|x_k|^2/dw (getPSD), std [ncase][nch] = sqrt(0.5 sum|x_k|^2) (getRMS); either
 * output may be NULL. */
int rh_channel_stats(rh_ctx* ctx, int ncase, int nrow, int ndof, int nw, double dw, const double* w,
                     const rh_c128* Xi, int nch, const double* coef, double* psd, double* std, rh_stream stream);

/* Coupled array solve (raft/raft_model.py:1021-1065) for nf FOWTs, 6nf <= 12:
 * Z_sys = blockdiag(Z_i) + K ; Xi = Z_sys^-1 F.  Z: [nf][nw][36] per-FOWT impedances,
 * K: [6nf*6nf] array mooring stiffness (or NULL), F: [6nf][nw], Xi out: [6nf][nw]. */
int rh_system_solve(rh_ctx* ctx, int nf, int nw, const rh_c128* Z, const double* K,
                    const rh_c128* F, rh_c128* Xi, rh_stream stream);

/* rh_system_solve for ncase independent cases of one array in one launch (the batched farm
 * path, Model.analyzeCasesBatch): Z [ncase][nf][nw][36], F / Xi [ncase][6nf][nw], K shared. */
int rh_system_solve_batch(rh_ctx* ctx, int ncase, int nf, int nw, const rh_c128* Z, const double* K,
                          const rh_c128* F, rh_c128* Xi, rh_stream stream);

/* The coupled-array response of a batch of single-sea-state cases in one launch
 * (raft/raft_model.py:1021-1065 with the per-heading excitation of :1049-1061): for every
 * case and bin, each FOWT's wave excitation F_f = zeta (F_iner + F_drag(Bmat)) and impedance
 * Z_f = -w^2 M + i w (B_lin + B_drag) + C (the fowt.Z of :1013, rebuilt from the design's
 * matrices and the case's B_drag), then Xi = (blockdiag(Z_f) + K)^-1 F.  Replaces the
 * rh_wave_excitation + rh_system_solve_batch pair without the per-(case, bin) Z and F arrays.
 * Entries e = ic * nf + f (case-major, FOWT-minor) index design_idx, head, zeta [.][nw],
 * B_drag [.][36] and Bmat [.][nn_max][9] (as rh_solve_cases writes them: nn_max is the largest
 * node count of the designs, which must share nw; FOWTs of an array may differ in node count).
 * K: [6nf][6nf] array stiffness or NULL.
 * Xi out: [ncase][6 nf][nw]. */
int rh_array_response(rh_ctx* ctx, const rh_design* designs, int ndesign, int nf, int ncase, const int* design_idx,
                      const int* head, const double* zeta, const double* B_drag, const double* Bmat, const double* K,
                      rh_c128* Xi, rh_stream stream);

/* rh_array_response plus the motion statistics of every (case, FOWT) from the solution while
 * it is in registers (no read-back of Xi): psd [ncase * nf][6][nw] = 0.5 |Xi|^2 / dw and
 * std [ncase * nf][6] = sqrt(0.5 sum_w |Xi|^2), rotations in degrees -- the values, bit for bit,
 * of rh_motion_stats(ctx, ncase * nf, 1, nw, dw, Xi, psd, std, stream) on the result
 * (FOWT.getPSD / getRMS, raft/helpers.py:581-603).  Either output may be NULL; dw > 0 when one
 * is requested.  order: optional device permutation of the ncase * nf (case, FOWT) entries,
 * sorted by design and heading (e.g. the rh_cases.order of the fixed point): each XCD then
 * excites a contiguous slice of it and streams few wave tables (placement only, never results). */
int rh_array_response_stats(rh_ctx* ctx, const rh_design* designs, int ndesign, int nf, int ncase,
                            const int* design_idx, const int* head, const double* zeta, const double* B_drag,
                            const double* Bmat, const double* K, rh_c128* Xi, double dw, double* psd, double* std_,
                            const int* order, rh_stream stream);

/* The response step of rh_array_response_stats alone, with each FOWT's wave excitation already
 * in Xi: Xi [ncase][6 nf][nw] holds F_wave on entry (rh_solve_out.F_wave of the (case, FOWT)
 * fixed points, entries e = ic * nf + f, which is this layout) and the response on return;
 * Z_f rebuilt from the design and B_drag [ncase * nf][36], Xi = (blockdiag(Z_f) + K)^-1 F, and
 * the statistics as rh_array_response_stats writes them (psd / std may be NULL). */
int rh_array_solve_stats(rh_ctx* ctx, const rh_design* designs, int ndesign, int nf, int ncase, const int* design_idx,
                         const double* B_drag, const double* K, rh_c128* Xi, double dw, double* psd, double* std_,
                         rh_stream stream);

/* ------------------------------------------------------------------------------------
 * Slender-body second-order QTF (FOWT.calcQTF_slenderBody, raft/raft_fowt.py:1385-1648)
 * ------------------------------------------------------------------------------------ */

/* QTF node table fields ([RH_QN_COUNT][nq]): submerged strip nodes (r_z < 0) of the
 * members that are not entirely above water, member-contiguous, reference order. */
enum rh_qtf_node_field {
  RH_QN_RX = 0, RH_QN_RY, RH_QN_RZ,      /* node position (the QTF uses mem.r, :1476)            */
  RH_QN_QX, RH_QN_QY, RH_QN_QZ,          /* member axis                                          */
  RH_QN_VI,                              /* side volume incl. partial-submergence scaling (:1532-1538) */
  RH_QN_VE,                              /* end volume (:1580-1584)                              */
  RH_QN_AI,                              /* signed end area mem.a_i (:1587)                      */
  RH_QN_CAE,                             /* Ca_End                                               */
  RH_QN_CM = 10,                         /* (1+Ca_p1) p1 p1^T + (1+Ca_p2) p2 p2^T   (9)          */
  RH_QN_CA = 19,                         /* Ca_p1 p1 p1^T + Ca_p2 p2 p2^T           (9)          */
  RH_QN_P12 = 28,                        /* p1 p1^T + p2 p2^T                       (9)          */
  RH_QN_QM = 37,                         /* q q^T                                   (9)          */
  RH_QN_COUNT = 46
};

/* QTF member table fields ([RH_QM_COUNT][nmq]) */
enum rh_qtf_member_field {
  RH_QM_WL = 0,                          /* 1: member crosses the waterline (mem.r[-1,2]*mem.r[0,2] < 0) */
  RH_QM_RIX, RH_QM_RIY, RH_QM_RIZ,       /* waterline intersection r_int (:1492)                  */
  RH_QM_AWL,                             /* waterline section area (:1608-1622)                   */
  RH_QM_CM = 5,                          /* CmM of the LAST submerged node (the reference reuses the loop's Ca, :1625) (9) */
  RH_QM_CA = 14,                         /* CaM of the last submerged node (9)                    */
  RH_QM_P1X = 23, RH_QM_P1Y, RH_QM_P1Z,  /* p1, p2 for the hydrostatic term g_e1 (:1497-1499)    */
  RH_QM_P2X, RH_QM_P2Y, RH_QM_P2Z,
  RH_QM_KAY = 29,                        /* 1: Kim & Yue correction active (MCF, piercing)        */
  RH_QM_PFX, RH_QM_PFY, RH_QM_PFZ,       /* normalised force direction pforce (raft_member.py:1130-1131) */
  RH_QM_WLX, RH_QM_WLY, RH_QM_WLZ,       /* rwl (raft_member.py:1136)                             */
  RH_QM_COUNT
};

/* Kim & Yue radius table ([RH_KR_COUNT][nkr]); for each KAY member the first entry is the
 * waterline radius, the following ones the submerged node intervals (raft_member.py:1155-1200). */
enum rh_kay_field {
  RH_KR_R = 0,                           /* radius R (waterline) or mean radius Rm (interval)    */
  RH_KR_Z1, RH_KR_Z2,                    /* interval ends (z2 clipped at 0)                      */
  RH_KR_MX, RH_KR_MY, RH_KR_MZ,          /* interval mid-point 0.5 (r1 + r2)                     */
  RH_KR_COUNT
};

typedef struct {
  int n2, nq, nmq, nkr;
  double beta, depth, rho, g;
  const double* w2;        /* [n2] second-order frequencies (rad/s)                     */
  const double* k2;        /* [n2] their wave numbers                                   */
  const double* qnode;     /* [RH_QN_COUNT][nq]                                         */
  const double* qmemb;     /* [RH_QM_COUNT][nmq]                                        */
  const int* qmstart;      /* [nmq+1] node ranges                                       */
  const int* kstart;       /* [nmq+1] ranges in the KAY radius table                    */
  const double* kray;      /* [RH_KR_COUNT][nkr]                                        */
  const rh_c128* hank;     /* [nkr][n2][12]  0.5 (H1_{n-1}(k R) - H1_{n+1}(k R)), n = 0..11 (scipy hankel1) */
  int order;               /* 1: w2 and k2 strictly increasing (checked by the caller): the pair sum
                              runs as FP64 MFMA GEMMs (rh_qtf_mfma.hip); 0: the per-pair kernel     */
} rh_qtf_design;

/* The static tables of one FOWT for a QTF at heading beta (rad), on the host: the geometry
 * bookkeeping of FOWT.calcQTF_slenderBody (raft/raft_fowt.py:1461-1502, 1532-1587, 1604-1625)
 * and Member.correction_KAY (raft/raft_member.py:1111-1200) that rh_qtf_design points at.
 * Host code only (no device, no ctx); replaces raft/qtf.py build_tables, which states the
 * same tables in NumPy.  rec: nmemb member records back to back, rec_len doubles (format:
 * csrc/rh_qtf_host.h; writer raft/qtf.py member_record).  out (cap doubles) receives
 * qnode [RH_QN_COUNT][nq], qmemb [RH_QM_COUNT][nmq] and kray [RH_KR_COUNT][nkr] back to back;
 * iout (capi ints) qmstart [nmq+1] and kstart [nmq+1]; counts = {nq, nmq, nkr}.  RH_EINVAL
 * for a malformed record or too small a capacity (46 + 6 doubles per node and 36 per member
 * always suffice). */
int rh_qtf_tables(int nmemb, const double* rec, long long rec_len, double beta, double* out, long long cap, int* iout,
                  long long capi, int* counts);

/* Device workspace (bytes) rh_qtf_slender needs for a design. */
long long rh_qtf_workspace_bytes(const rh_qtf_design* q);

/* Slender-body QTF for one heading: Xi0 [6][nw] motion RAO on the first-order grid w [nw];
 * M66 [36] structural mass matrix (F1st, :1437-1439); qtf out [n2][n2][6] (full Hermitian
 * matrix, upper triangle computed, lower filled as :1639-1640).  work: device workspace.
 * On the MFMA path the Kim & Yue kernel runs on a second stream owned by ctx, joined back to
 * `stream` by an event before the final kernel: the outputs are stream-ordered on `stream`, and
 * a ctx must not run two QTFs at once on different streams. */
int rh_qtf_slender(rh_ctx* ctx, const rh_qtf_design* q, int nw, const double* w, const rh_c128* Xi0,
                   const double* M66, rh_c128* qtf, void* work, long long work_bytes, rh_stream stream);

/* rh_qtf_slender with flags.  RH_QTF_INCIDENT_CACHED: `work` already holds the incident-wave
 * parts of this QTF -- the nodes' grad u / grad p / dw/dz tables, the Kim & Yue tables, their
 * GEMM basis and pair-tile sums, the node GEMM basis and the zero K tails, none of which depends
 * on the RAO -- from an earlier
 * rh_qtf_slender(_ext) call with the same q and work on the MFMA path (the caller vouches for
 * it); only the RAO-dependent tables, coefficients and GEMMs run.  The result equals a full call
 * bit for bit.  For a design's many QTFs with different RAOs (the second passes of
 * potSecOrder = 1 cases, raft/second_order.py).  RH_EINVAL on the per-pair path. */
#define RH_QTF_INCIDENT_CACHED 1
int rh_qtf_slender_ext(rh_ctx* ctx, const rh_qtf_design* q, int nw, const double* w, const rh_c128* Xi0,
                       const double* M66, rh_c128* qtf, void* work, long long work_bytes, int flags, rh_stream stream);

/* The upper-triangle pairs (w1 <= w2) of one rank of a QTF sharded over nrank devices, no
   Hermitian fill.  The upper triangle is cut into 16 x 16 pair tiles (i1 tile T1 <= i2 tile T2,
   n2 rounded up to 16), numbered row-major; rank r owns the tiles t with t % nrank == r
   (raft/parallel.py qtf_tiles).  Entries of other tiles are not written (order == 0: every
   rank computes the whole triangle, a superset).  The caller exchanges the shards
   (raft/parallel.py assemble_qtf: one all_gather over xGMI of every rank's packed pairs,
   scattered into place by index) and then calls rh_qtf_hermitian_fill. */
int rh_qtf_slender_rows(rh_ctx* ctx, const rh_qtf_design* q, int nw, const double* w, const rh_c128* Xi0,
                        const double* M66, int rank, int nrank, rh_c128* qtf, void* work, long long work_bytes,
                        rh_stream stream);

/* The Kim & Yue Hankel table of rh_qtf_design.hank on the device: hank[ir][f][n] =
 * 0.5 (H1_{n-1}(x) - H1_{n+1}(x)), x = k2[f] R[ir], n = 0..11 -- the values the reference takes
 * from scipy.special.hankel1 (raft/raft_member.py:1104-1107).  R: [nkr] radii (the RH_KR_R row
 * of the radius table).  J by series / Miller recurrence, Y by forward recurrence from y0, y1. */
int rh_qtf_hankel(rh_ctx* ctx, int n2, const double* k2, int nkr, const double* R, rh_c128* hank, rh_stream stream);

/* qtf[i2][i1] = conj(qtf[i1][i2]) for i2 > i1 (raft/raft_fowt.py:1639-1640). */
int rh_qtf_hermitian_fill(rh_ctx* ctx, int n2, rh_c128* qtf, rh_stream stream);

/* Second-order force spectrum, 'qtf' interpolation mode (raft/raft_fowt.py:1788-1810):
 * qtf [n2][n2][6] on grid w2 [n2] (uniform spacing), spectrum S0 [nw] on grid w [nw]
 * (uniform spacing dw) -> f [6][nw] (already shifted by one bin), f_mean [6]. */
int rh_force_2nd(rh_ctx* ctx, int n2, const double* w2, const rh_c128* qtf, int nw, const double* w, double dw,
                 const double* S0, double* f, double* f_mean, rh_stream stream);

/* rh_force_2nd for a batch of sea states in one launch (the per-case second-order loads of a
 * batched solve, Model.analyzeCasesBatch): case c uses the QTF qidx[c] of the stack
 * qtf [nq][n2][n2][6] (qidx: device [ncase], or NULL for QTF 0) and its spectrum S0 [c][nw];
 * f out: [ncase][6][nw] complex with zero imaginary part (the fext rows of rh_cases, the same
 * values as rh_force_2nd bit for bit), f_mean [ncase][6].  A qidx outside [0, nq) gives NaN. */
int rh_force_2nd_batch(rh_ctx* ctx, int ncase, int n2, const double* w2, const rh_c128* qtf, int nq,
                       const int* qidx, int nw, const double* w, double dw, const double* S0, rh_c128* f,
                       double* f_mean, rh_stream stream);

/* Second-order force spectrum, 'spectrum' interpolation mode (raft/raft_fowt.py:1760-1784,
 * 1809-1810): S = interp(w2, w, S0) (0 outside w), force spectrum on the QTF grid
 * Sf [6][n2] (device workspace, written), then f [6][nw] = sqrt(2 dw interp(w - w[0],
 * w2 - w2[0], Sf)) shifted by one bin (the reference returns it as complex with zero imaginary
 * part), f_mean [6]. */
int rh_force_2nd_spectrum(rh_ctx* ctx, int n2, const double* w2, const rh_c128* qtf, int nw, const double* w,
                          double dw, const double* S0, double* Sf, double* f, double* f_mean, rh_stream stream);

/* ---- native per-design host preparation (host code; no device calls) -------------------
 * Members, statics, added mass and the device-table layout of many single-FOWT designs on
 * host threads: the per-design work of Model/FOWT setup before a case loop
 * (raft/raft_model.py:30-170, raft/raft_fowt.py:291-565, 848-880; raft/raft_member.py:23-1050),
 * here in C++ (raft-teststuff_amd/csrc/rh_prep.h) so that a design sweep (C5) pays no
 * interpreter time per design.  spec: one float64 record per design, design i at
 * spec[spec_off[i] .. spec_off[i+1]) (format: rh_prep.h; writer: raft/native_prep.py).
 * w, k [nw]: the shared frequency grid and wave numbers.  nthreads <= 0: all host cores (at
 * most 64).  The calling thread works too; the other nthreads - 1 are kept by the library
 * across calls (created on first need, one call at a time: concurrent callers queue; a forked
 * child makes its own).
 * MacCamy-Fuchs members (raft/raft_member.py:1053-1088) get their frequency-dependent inertial
 * excitation matrices, one [9][nw] block per node: rh_prep_imat. */
typedef struct rh_prep rh_prep;
int rh_prep_designs(int ndesign, const double* spec, const long long* spec_off, int nw, const double* w,
                    const double* k, int nthreads, rh_prep** out);
/* info [ndesign][5] = (packed offset, packed length, mstart offset, nn, nm), then the totals
 * info[5 nd] = packed doubles, info[5 nd + 1] = mstart ints.  Per design the packed block is
 * w[nw], k[nw], node[RH_NF_COUNT][max(nn,1)], memb[RH_MF_COUNT][max(nm,1)], M[36], B[36], C[36]
 * (the layout of raft/prep.py host_tables). */
int rh_prep_layout(const rh_prep* p, long long* info);
/* packed [total], mstart [total]; statics (optional) [ndesign][5][36] = M_struc, B_struc,
 * C_struc, C_hydro, A_hydro_morison. */
int rh_prep_copy(const rh_prep* p, double* packed, int* mstart, double* statics);
/* Design `design`'s MacCamy-Fuchs inertia table, the rh_design.imat_mcf of raft/prep.py
 * node_table: [nn][9][nw] complex (zeros for the other nodes).  Returns its number of entries
 * (nn 9 nw; 0 when no node of the design is MacCamy-Fuchs), and copies them when imat != NULL;
 * RH_EINVAL for a bad handle or index. */
long long rh_prep_imat(const rh_prep* p, int design, rh_c128* imat);
void rh_prep_free(rh_prep* p);

#ifdef __cplusplus
}
#endif
#endif
