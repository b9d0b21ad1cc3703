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
} rh_cases;

/* Outputs of rh_solve_cases (device buffers; NULL = not wanted). */
typedef struct {
  rh_c128* Xi;            /* [ncase][6][nw] response to sea state 0 (required)  */
  rh_c128* Xi_last;       /* [ncase][6][nw] scratch for the relaxed iterate (required) */
  int* iters;             /* [ncase] linear solves executed (required)         */
  int* status;            /* [ncase] RH_CASE_* (required)                      */
  double* zeta;           /* [ncase][nw] wave amplitudes sqrt(2 S dw)          */
  double* B_drag;         /* [ncase][36] final linearised drag damping         */
  double* Bmat;           /* [ncase][nn][9] final per-node drag matrices       */
  double* psd;            /* [ncase][6][nw] motion PSD (rotations in deg^2), raft/raft_fowt.py:1836-1874 */
  double* std;            /* [ncase][6] motion RMS                             */
  rh_c128* rao;           /* [ncase][6][nw] Xi / zeta (raft/helpers.py:665)   */
  rh_c128* Z;             /* [ncase][nw][36] final impedance (fowt.Z, raft/raft_model.py:1013) */
} rh_solve_out;

const char* rh_last_error(void);
int rh_ctx_create(int device, rh_ctx** out);
int rh_ctx_destroy(rh_ctx* ctx);
int rh_version(void);

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
 * Bmat [ncase][nn][9] as produced by rh_solve_cases; Xi out: [ncase][6][nw]. */
int rh_heading_response(rh_ctx* ctx, const rh_design* designs, int ndesign, int ncase,
                        const int* design_idx, const int* head, const double* zeta,
                        const double* B_drag, const double* Bmat, rh_c128* Xi, rh_stream stream);

/* Stand-alone FOWT.calcHydroLinearization(Xi) + calcDragExcitation (raft/raft_fowt.py:1152-1293)
 * for one design and one sea state: Xi [6][nw], zeta [nw] (u = zeta*uhat[head]).
 * Outputs: B_drag [36], Bmat [nn][9], F_drag [6][nw]. */
int rh_linearize(rh_ctx* ctx, const rh_design* d, int head, const rh_c128* Xi, const double* zeta,
                 double* B_drag, double* Bmat, rh_c128* F_drag, rh_stream stream);

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

/* Coupled array solve (raft/raft_model.py:1021-1065) for nf FOWTs, 6nf <= 12:
 * Z_sys = blockdiag(Z_i) + K ; Xi = Z_sys^-1 F.  Z: [nf][nw][36] per-FOWT impedances,
 * K: [6nf*6nf] array mooring stiffness (or NULL), F: [6nf][nw], Xi out: [6nf][nw]. */
int rh_system_solve(rh_ctx* ctx, int nf, int nw, const rh_c128* Z, const double* K,
                    const rh_c128* F, rh_c128* Xi, rh_stream stream);

#ifdef __cplusplus
}
#endif
#endif
