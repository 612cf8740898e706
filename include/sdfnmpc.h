/* sdfnmpc.h -- C ABI of the MI355X-native neural-SDF NMPC evaluator (libsdfnmpc.so).
 *
 * Plain pointers and sizes only: no torch types, no C++ types.  Every entry point returns
 * SDFNMPC_OK (0) or a negative error code and never throws; sdfnmpc_last_error() gives the message
 * (thread-local).  Device pointers are HIP device pointers on the context's device; work is enqueued
 * on the context's stream (asynchronous unless stated otherwise).
 *
 * Which reference interface each entry point replaces (paths relative to the reference checkout):
 *
 *   sdfnmpc_net_load / _load_file      torch.jit.load(sdf weights) + .to(device) + .eval()
 *                                      (sdf_nmpc/gen_model.py:32-34); weights as a packed .sdfw blob
 *   sdfnmpc_net_siren                  NeuralDF(...) + init_linear_layer_sine (df_train.py:109-110,
 *                                      layer_init.py:15-25) with a counter-based PRNG
 *   sdfnmpc_sdf_eval                   NeuralDF.forward (network/neural_df.py:91-103) + autograd
 *                                      d df / d input, batched over rows -- what L4CasADi's
 *                                      sdf_l4c / jac_sdf_l4c compute one row at a time
 *                                      (gen_model.py:39,60)
 *   sdfnmpc_linearize                  the per-node evaluations acados performs in the SQP-RTI
 *                                      preparation phase of Ocp.solve (ocp.py:159-170, rti_phase 0):
 *                                      ERK4 + forward sensitivities (ocp.py:106), NONLINEAR_LS residual
 *                                      and Jacobian (model/quad_rollpitchyawrate.py:48-55), and the
 *                                      constraint vector h = [hfov, vfov, sdf] with its Jacobian
 *                                      (model/cost_const_helpers.py:48-75, gen_model.py:46-70)
 *   sdfnmpc_qp_solve                   the feedback phase of the same SQP-RTI step: the QP acados
 *                                      builds (NONLINEAR_LS Gauss-Newton + levenberg_marquardt, soft
 *                                      h rows, input boxes, ocp.py:54-120) and hands to HPIPM
 *                                      (FULL_CONDENSING_HPIPM, ocp.py:113-116), batched over instances
 *   sdfnmpc_rti_apply                  the SQP-RTI full step x <- x + dx, u <- u + du and u_0
 *                                      (solve_for_x0's return value, ocp.py:169)
 *   sdfnmpc_shooting_grid              Ocp.__init__ shooting nodes / time steps (ocp.py:18-27)
 *   sdfnmpc_solver_*                   the AcadosOcpSolver object Ocp builds (ocp.py:127) and drives:
 *                                      solver.set(k, 'x'|'u'|'p') / cost_set(k, 'yref'|'W') (ocp.py:
 *                                      146-170) -> _upload; solver.get -> _download; reset + init
 *                                      (ocp.py:144-149) -> _init; shift (ocp.py:152-156) -> _shift;
 *                                      solve_for_x0 (ocp.py:169) -> _step + _wait.  It owns the device
 *                                      workspace of B instances, so a controller needs no tensor library
 *
 * The CasADi external-function symbols that acados links (sdf_l4c, jac_sdf_l4c, ...) are in
 * sdf_l4c.h / libsdf_l4c.so.
 */
#ifndef SDFNMPC_H
#define SDFNMPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDFNMPC_ABI_VERSION 6

enum {
    SDFNMPC_OK = 0,
    SDFNMPC_E_ARG = -1,          /* invalid argument / shape */
    SDFNMPC_E_HIP = -2,          /* HIP runtime error (message has the HIP error string) */
    SDFNMPC_E_FORMAT = -3,       /* malformed weight blob */
    SDFNMPC_E_UNSUPPORTED = -4,  /* network architecture / model option not built for */
    SDFNMPC_E_NODEVICE = -5      /* no HIP device visible */
};

typedef struct sdfnmpc_ctx sdfnmpc_ctx;
typedef struct sdfnmpc_net sdfnmpc_net;

#define SDFNMPC_POLY_DEG_MAX 6 /* braking-distance polynomial: degree bound ... */
#define SDFNMPC_POLY_MAX 84    /* ... and its coefficient count (deg + 3 choose 3) */
#define SDFNMPC_NHN_MAX 8      /* terminal constraint rows (soft <= 3, hard <= 6) */
#define SDFNMPC_NHE 6          /* terminal extra functions hE (sdfnmpc_lin_args) */

/* 'att' model constants (model/quad_rollpitchyawrate.py; config robot.limits / sensor / mpc) and the
 * terminal ingredients of flags.recursive_feasibility / flags.stability (gen_model.py:72-149) */
typedef struct {
    double gamma, roll, pitch, wz; /* robot.limits.{gamma, roll, pitch, wz}: u -> physical inputs */
    double g;                      /* gravity, 9.81 (model/base_model.py:10) */
    double B_p_C[3];               /* sensor.B_p_C (utils/config.py:43) */
    double B_R_C[9];               /* sensor.B_R_C, row-major (utils/config.py:44) */
    double fov_const_offset;       /* mpc.fov_const_offset (cost_const_helpers.py:65) */
    int rec_feas;                  /* 1: the preparation phase evaluates the terminal extras hE[0..2] (below) */
    int stability;                 /* 1: hE[3..5] = v_N, and the terminal residual y_N is scaled by the flag and
                                      gains the row flag |v|^2 (quad_rollpitchyawrate.py:52-55, gen_model.py:
                                      142-149): nyN = 5 */
    int poly_deg;                  /* braking-distance polynomial degree (mpc.braking_dist.degree, <= 6) */
    double poly[SDFNMPC_POLY_MAX]; /* its coefficients in polynomial_3variate's term order (utils/math.py:
                                      307-314: total degree 0..deg, then x exponent a, then y exponent b) */
} sdfnmpc_quad_model;

/* Batched preparation phase: B instances x (N+1) shooting nodes, fp64, row-major C arrays.
 * Jacobian blocks are column-major (column j contiguous), j over (x[0..9], u[0..3]). */
typedef struct {
    int B, N;         /* instances, horizon */
    int np;           /* parameters per node, >= 17 + 128 (p layout: default.yaml mpc.p_idx) */
    int latent_mode;  /* 0: latent shared per instance (node 0's, as Nmpc.set_latent writes all
                         rows, controller.py:50-54); 1: latent read per node */
    const double* x;  /* [B][N+1][10] current iterate */
    const double* u;  /* [B][N][4] */
    const double* p;  /* [B][N+1][np] stage parameters (Ocp.solve p[k], ocp.py:165,168) */
    const double* dt; /* [N] time steps (sdfnmpc_shooting_grid) */
    double* xn;       /* [B][N][10]      x_{k+1} = RK4(x_k, u_k, dt_k) */
    double* AB;       /* [B][N][14][10]  [A_k | B_k] column-major */
    double* y;        /* [B][N][11]      NONLINEAR_LS residual */
    double* Jy;       /* [B][N][14][11]  column-major */
    double* yN;       /* [B][4]          terminal residual */
    double* JyN;      /* [B][10][4]      column-major */
    double* h;        /* [B][N+1][3]     the three node functions [hfov, vfov, sdf] in fixed columns: which
                                            of them are rows of the OCP is the QP's constraint set
                                            (sdfnmpc_qp_opts.nh / h_col) */
    double* Jh;       /* [B][N+1][10][3] column-major, d h / d x (d h / d u == 0) */
    float* sdf;       /* [B][N+1][4]     optional: (df, d df / d Co_p_B); NULL = internal buffer */
    int nyN;          /* terminal residual rows: 4, or 5 with sdfnmpc_quad_model.stability (yN [B][nyN],
                         JyN [B][10][nyN]) */
    int no_sdf;       /* 1: no constraint or cost uses the network (enable_sdf False, or neither sdf_constraint,
                         sdf_cost nor rec_feas): the SDF kernels are skipped, h[.][2] is not written and
                         net may be NULL */
    double* hE;       /* [B][6]          terminal extras (NULL unless rec_feas / stability): [-flag poly(v),
                         flag atan2(E_y, E_x), flag atan2(E_z, |E_xy|), v_x, v_y, v_z] with E = Co_p_E, the
                         camera-frame point at the braking distance ahead (gen_model.py:98-112); the
                         rec_feas constraint value is h[N][2] + hE[0] (gen_model.py:94-95) */
    double* JhE;      /* [B][10][6]      column-major d hE / d x_N */
} sdfnmpc_lin_args;

/* QP model data and solver options (defaults in sdf-nmpc_amd/model.py / ocp.py) */
typedef struct {
    double lbu[4], ubu[4]; /* input box (model/quad_rollpitchyawrate.py:58-59) */
    double lh[3], uh[3];   /* h bounds: +-fov_ratio*fov, [size.xy+bound_margin, max_df+0.2] */
    double zl[3], Zl[3];   /* L1 / L2 slack penalties of the soft h rows, lower == upper (ocp.py:85-92) */
    double lm;             /* levenberg_marquardt (ocp.py:120, mpc.lm_reg) */
    int cost_scaling;      /* 1: stage cost and slack penalties x dt_k, terminal x 1 (acados default) */
    int max_iter;          /* qp_solver_iter_max (ocp.py:115) */
    double tol;            /* IPM stop: max complementarity max_i t_i lambda_i and max primal residual below
                              tol (HPIPM's res_m / res_b tests) */
    int ny;                /* stage residuals: 11, or 12 with flags.sdf_cost (gen_model.py:65-66): the 12th,
                              (1 - s/2)^4 of the flagged SDF value s = h[2], and its Jacobian
                              -2 (1 - s/2)^3 J_h[2] are formed from h / J_h by the QP (yref, W: [B][N][ny]) */
    int lm_scaling;        /* 1: Levenberg-Marquardt term lm dt_k at stages k < N and lm at N (acados adds
                              Ts[k] * levenberg_marquardt); 0: lm at every node */
    int warm_start;        /* qp_solver_warm_start (ocp.py:116, HPIPM's primal warm start): 1 = the IPM starts
                              from the du found in sdfnmpc_qp_args.du on entry (the previous QP's solution --
                              the solver object keeps it between steps; zero after init), dx rolled out from
                              x0 under it, t / lambda by the cold start's rule; 0 = du = 0 (cold) */
    /* The constraint set (gen_model.py:26-149 under flags.enable_sdf / sdf_constraint / vfov_constraint /
     * recursive_feasibility / stability and sensor.hfov < 3.14; sdf-nmpc_amd/model.py builds it).
     * Stage rows k < N: nh rows, row j = column h_col[j] of h / J_h, with bounds / slack weights lh[j], uh[j],
     * zl[j], Zl[j] above; the first nh - nhs soft, the last nhs hard (slack weight None: add_const_stage,
     * base_model.py:142-155; zl / Zl unused).  Terminal rows: nhN rows, the first nsN soft
     * (lhN / uhN, slack weights zlN / ZlN, not cost-scaled), the rest hard; row j's value is
     * h[N][hN_col[j]] (if >= 0) + hE[hE_col[j]] (if >= 0), its Jacobian the same sum of columns. */
    int nh;                /* 0..3 (3: [hfov, vfov, sdf], the default flags) */
    int h_col[3];          /* distinct columns 0..2 */
    int nhN, nsN;          /* nhN <= SDFNMPC_NHN_MAX, nsN <= min(nhN, 3), nhN - nsN <= 6 */
    int hN_col[SDFNMPC_NHN_MAX], hE_col[SDFNMPC_NHN_MAX];
    double lhN[SDFNMPC_NHN_MAX], uhN[SDFNMPC_NHN_MAX], zlN[3], ZlN[3];
    int nyN;               /* terminal residual rows (yNref / WN [B][nyN]): 4, or 5 with flags.stability */
    int nhs;               /* hard stage rows (the last nhs of the nh), 0..nh: mpc.weights.slack_fov / slack_df
                              None (the terminal copies of those rows are then hard rows of the nhN too) */
} sdfnmpc_qp_opts;

/* Batched QP of the RTI feedback phase, built from sdfnmpc_linearize outputs. */
typedef struct {
    int B, N;
    const double *xn, *AB, *y, *Jy, *yN, *JyN, *h, *Jh; /* sdfnmpc_lin_args outputs */
    const double *hE, *JhE; /* sdfnmpc_lin_args outputs (NULL when no terminal row reads them) */
    const double* x;     /* [B][N+1][10] iterate the QP was built at */
    const double* u;     /* [B][N][4] */
    const double* x0;    /* [B][10] measured state (Ocp.solve x0) */
    const double* yref;  /* [B][N][ny] stage references (Ocp.solve y[k]) */
    const double* W;     /* [B][N][ny] diagonal weights (Ocp.solve W[k], set as np.diag) */
    const double* yNref; /* [B][nyN] */
    const double* WN;    /* [B][nyN] */
    const double* dt;    /* [N] */
    double* dx;          /* [B][N+1][10] solution: the RTI step */
    double* du;          /* [B][N][4] */
    double* slack;       /* [B][N+1][3][2] optional: (sl, su) of the soft rows (row j of node k < N; terminal
                            soft row j at node N; unused entries 0) */
    int* status;         /* [B] optional: 0 converged, 1 max_iter reached (acados status 2: the step is
                            kept), 2 numerical failure -- a NaN / Inf in the data (acados QP failure,
                            status 4: sdfnmpc_rti_apply given this array keeps the instance's iterate) */
    int* iters;          /* [B] optional */
    double* res;         /* [B][2] optional: (max complementarity, max primal residual) */
} sdfnmpc_qp_args;

/* Batched reference / parameter packing: RefGen (ref_gen.py:17-130) ->
 * formate_ref (quad_rollpitchyawrate.py:62-65) -> Nmpc.set_ref / set_latent / set_sdf_flag
 * (controller.py:45-54,133-142) for B instances x (N+1) nodes on the device. */
typedef struct {
    int mode;              /* 0 gen_ref_list_wps, 1 gen_ref_joystick, 2 from_x0, -1 latent / flag only */
    int yaw_mode;          /* path samples: 0 identity, 1 'ref', 2 'align', 3 x0 quaternion ('curent', sic) */
    int st_enable;         /* ref.stop_and_turn.enable */
    int st_mode;           /* stop-and-turn yaw: 0 current, 1 'topic', 2 'align' */
    double st_dang;        /* ref.stop_and_turn.dang_min */
    double align_off;      /* ref.align_yaw_offset */
    double dmin;           /* ref.yaw_align_dmin */
    double vref, wzref;    /* ref.vref, ref.wzref */
    double T;              /* mpc.T */
    double B_p_C[3], B_R_C[9]; /* sensor extrinsics (config.py) */
} sdfnmpc_ref_opts;

typedef struct {
    int B, N, np, ny;      /* np = 17 + latent size; ny = 11 or 12 (sdf_cost) */
    int n_wp;              /* waypoints per instance (mode 0), <= 32 */
    int L;                 /* latent size (when latent != NULL) */
    const double* x0;      /* [B][x0_stride] current state */
    int x0_stride;
    const double* wp_p;    /* [B][n_wp][3] (mode 0) */
    const double* wp_q;    /* [B][n_wp][4] (mode 0) */
    const double* vw;      /* [B][4] (vx, vy, vz, wz) in [-1, 1] (mode 1) */
    const double* wrow;    /* [ny] the W row formate_ref builds from the caller's weight set */
    const double* latent;  /* [B][L] or NULL (then W_p_Bo / W_R_Bo are ignored) */
    const double* W_p_Bo;  /* [B][3] body position at image time */
    const double* W_R_Bo;  /* [B][9] body attitude at image time, row-major */
    const double* flag;    /* [B] sdf flag or NULL */
    double* p;             /* [B][N+1][np] OCP parameters */
    double* yref;          /* [B][N][ny] */
    double* W;             /* [B][N][ny] */
    double* yNref;         /* [B][nyN] */
    double* WN;            /* [B][nyN] */
    int nyN;               /* terminal residual rows: 4, or 5 with flags.stability (y[:nyN] / W[:nyN] of the
                              last node, controller.py:141-142; 0 is taken as 4) */
} sdfnmpc_ref_args;

int sdfnmpc_abi_version(void);
const char* sdfnmpc_last_error(void);

/* ---- context: one device + one stream (+ workspaces, kernel timing) ---- */
int sdfnmpc_ctx_create(int device, void* hip_stream /* NULL: create a non-blocking stream */, sdfnmpc_ctx** out);
void sdfnmpc_ctx_destroy(sdfnmpc_ctx* ctx);
int sdfnmpc_ctx_set_stream(sdfnmpc_ctx* ctx, void* hip_stream);
/* launch on the legacy null stream (handle 0, e.g. PyTorch's default stream) */
int sdfnmpc_ctx_use_null_stream(sdfnmpc_ctx* ctx);
void* sdfnmpc_ctx_stream(sdfnmpc_ctx* ctx);
int sdfnmpc_ctx_device(const sdfnmpc_ctx* ctx);
int sdfnmpc_ctx_synchronize(sdfnmpc_ctx* ctx);
/* the feedback-phase IPM kernel: SEGMENTED runs every instance on one workgroup of four wavefronts with a
 * partitioned (parallel-in-time) Riccati recursion (csrc/rti_qp_seg.hip); SERIAL on one wavefront
 * (csrc/rti_qp.hip).  AUTO (default) = SEGMENTED for batches of at most SDFNMPC_QP_SEG_AUTO_MAX_B
 * instances (twice that from N = 48) at horizons SDFNMPC_QP_SEG_AUTO_MIN_N <= N <= 63 (8-10 % faster
 * at N = 40, 21-24 % at N = 60 up to B = 512), SERIAL otherwise (large batches at N < 48: one wavefront
 * per SIMD is the throughput regime; short horizons, where the couplings outweigh the segments).  Both solve the same QP to the same stop test; their iterates
 * agree to rounding, not bitwise.  SDFNMPC_QP_KERNEL=serial|segmented sets the default of new contexts. */
#define SDFNMPC_QP_AUTO 0
#define SDFNMPC_QP_SERIAL 1
#define SDFNMPC_QP_SEGMENTED 2
#define SDFNMPC_QP_SEG_AUTO_MAX_B 256
#define SDFNMPC_QP_SEG_AUTO_MIN_N 36
int sdfnmpc_ctx_set_qp_kernel(sdfnmpc_ctx* ctx, int kernel);
/* the kernel a QP batch of B instances at horizon N runs on this context (SDFNMPC_QP_SERIAL or
 * _SEGMENTED; -1 on bad arguments) */
int sdfnmpc_ctx_qp_kernel(const sdfnmpc_ctx* ctx, int N, int B);
/* the same for the constraint set of opts (NULL: the default set; -1 on a malformed set).  Both kernels serve
 * every constraint set sdfnmpc_qp_opts describes (soft / hard stage rows, rec_feas and stability terminal
 * rows), so the choice is the batch / horizon policy above.  Replaces acados' one HPIPM instance per solver
 * (ocp.py:113-120). */
int sdfnmpc_ctx_qp_kernel_for(const sdfnmpc_ctx* ctx, int N, int B, const sdfnmpc_qp_opts* opts);
/* LDS bytes one instance of the serial QP kernel holds at horizon N (-1: N < 1) */
long long sdfnmpc_qp_lds_bytes(int N);
/* the occupancy gate of SURVEY.md §8(e): instances the context's device solves in one wave of QP
 * workgroups at horizon N = CUs x min(LDS per CU / LDS per instance, the runtime's occupancy of the
 * kernel sdfnmpc_ctx_qp_kernel picks -- registers and waves included), from hipDeviceProp_t and
 * hipOccupancyMaxActiveBlocksPerMultiprocessor (1024 at N = 20 and 40 on an MI355X: the serial kernel's
 * registers allow four instances per CU); 0 when N does not fit one CU, -1 on bad arguments.  Replaces the reference's single acados solver per process
 * (controller.py:16 builds one Ocp): a batch larger than this is split over devices (shard.plan). */
long long sdfnmpc_qp_capacity(const sdfnmpc_ctx* ctx, int N);
/* the same for the constraint set of opts (its rows change the LDS per instance; NULL: the default set) */
long long sdfnmpc_qp_capacity_for(const sdfnmpc_ctx* ctx, int N, const sdfnmpc_qp_opts* opts);
/* rows per SDF workgroup: 32 (2 workgroups / CU) or 64 (1 workgroup / CU); default 32 */
int sdfnmpc_ctx_set_tile_rows(sdfnmpc_ctx* ctx, int rows);
/* per-kernel HIP-event timing on the context stream (off by default) */
int sdfnmpc_ctx_enable_timing(sdfnmpc_ctx* ctx, int on);
/* kernel: "sdf_mlp", "sdf_hoist", "linearize"; synchronizes the stream(s) */
int sdfnmpc_ctx_kernel_stats(sdfnmpc_ctx* ctx, const char* kernel, double* total_ms, long long* launches);
int sdfnmpc_ctx_reset_stats(sdfnmpc_ctx* ctx);

/* ---- network ---- */
int sdfnmpc_net_load(sdfnmpc_ctx* ctx, const void* blob, size_t bytes, sdfnmpc_net** out);
int sdfnmpc_net_load_file(sdfnmpc_ctx* ctx, const char* path, sdfnmpc_net** out);
int sdfnmpc_net_siren(sdfnmpc_ctx* ctx, uint64_t seed, float weight_gain, float bias_gain, sdfnmpc_net** out);
void sdfnmpc_net_free(sdfnmpc_net* net);
float sdfnmpc_net_max_df(const sdfnmpc_net* net);
int sdfnmpc_net_size_latent(const sdfnmpc_net* net);
/* FNV-1a of the fp32 parameters in torch order (identity check across ranks / files) */
uint64_t sdfnmpc_net_fingerprint(const sdfnmpc_net* net);

/* ---- SDF evaluation, device pointers ----
 * pos4[rows][4] = (Co_p_B, unused); latent[n_inst][128] fp32 with row r -> instance r / rows_per_inst;
 * out4[rows][4] = (df, d df / d pos); grad_latent[rows][128] optional (NULL to skip). */
int sdfnmpc_sdf_eval(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, long long rows, const float* pos4,
                     const float* latent, int rows_per_inst, float* out4, float* grad_latent);

/* ---- SDF evaluation, host pointers, synchronous (the CasADi external path) ----
 * in[rows][3+128] doubles (the L4CasADi input vertcat(Co_p_B, latent), gen_model.py:60) ->
 * df[rows], grad[rows][3+128] (optional). Computed in fp32 on the device, returned as fp64. */
int sdfnmpc_sdf_eval_host(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, int rows, const double* in, double* df,
                          double* grad);
/* Calls of sdfnmpc_sdf_eval_host with at most 16 rows (the CasADi external's one row per node) are
 * served by a resident server kernel: one persistent workgroup on its own stream polls a mailbox in
 * pinned host memory, so a call costs no launch, no copies and no stream synchronisation.  It exits
 * after SDFNMPC_SDF_SERVER_IDLE_MS (default 20) without a request, on sdfnmpc_ctx_destroy, or after 10 s
 * (relaunched on the next call).  on = 0 stops it and returns to one launch per call (also
 * SDFNMPC_SDF_SERVER=0); results are bitwise the same either way. */
int sdfnmpc_ctx_set_sdf_server(sdfnmpc_ctx* ctx, int on);
/* diagnostics: mean microseconds per served request since the last call -- out18[0] staging the request,
 * [1] evaluating it, [2] the caller's wait from posting to the answer; out18[3] = requests;
 * out18[4..17] the evaluation's phases (embedding, 4 x (layer GEMV, sine), the last sine, 4 backward
 * GEMVs, outputs) */
int sdfnmpc_ctx_sdf_server_stats(sdfnmpc_ctx* ctx, double* out18);

/* ---- batched preparation phase ---- */
int sdfnmpc_linearize(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* model,
                      const sdfnmpc_lin_args* args);

/* ---- batched QP (feedback phase) and the RTI step ---- */
int sdfnmpc_qp_solve(sdfnmpc_ctx* ctx, const sdfnmpc_qp_opts* opts, const sdfnmpc_qp_args* args);
/* The same SQP-RTI step split the way acados splits it (rti_phase 1 / 2, ocp.py:110): everything that
 * does not depend on x0 -- the linearisation and the QP's stage records (H, g, dynamics, constraint
 * rows) -- in the preparation phase, the IPM alone in the feedback phase.  sdfnmpc_rti_prepare =
 * sdfnmpc_linearize + the record pack (qp_args must name lin_args' iterate and outputs; the pack runs
 * beside the SDF kernel); sdfnmpc_qp_feedback = the IPM on those records, once per preparation
 * (SDFNMPC_E_ARG without a matching sdfnmpc_rti_prepare).  Results are bitwise those of
 * sdfnmpc_linearize + sdfnmpc_qp_solve. */
int sdfnmpc_rti_prepare(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* model,
                        const sdfnmpc_lin_args* lin_args, const sdfnmpc_qp_opts* opts, const sdfnmpc_qp_args* qp_args);
int sdfnmpc_qp_feedback(sdfnmpc_ctx* ctx, const sdfnmpc_qp_opts* opts, const sdfnmpc_qp_args* args);
/* x[B][N+1][10] += dx, u[B][N][4] += du, u0[B][4] = u[:, 0] (u0 may be NULL).  status [B] (may be NULL):
 * instances with status >= 2 (QP failure) keep x and u; their u0 is the unchanged u[:, 0]. */
int sdfnmpc_rti_apply(sdfnmpc_ctx* ctx, int B, int N, double* x, double* u, const double* dx, const double* du,
                      double* u0, const int* status);

/* One whole SQP-RTI control step -- sdfnmpc_rti_prepare + sdfnmpc_qp_feedback + sdfnmpc_rti_apply on
 * fixed buffers -- captured once into a HIP graph and replayed by sdfnmpc_step_launch with one host call
 * (the latency path: the per-call form spends its host time in ≈10 runtime calls per step).  create runs the
 * step once eagerly (workspaces allocated, arguments checked), then captures it on a private stream; launch
 * enqueues the graph on the context stream.  The buffers named in the arguments must stay allocated at the
 * same addresses; results are bitwise those of the three calls.  The graph also addresses the context's own
 * workspaces: a later call on the context that grows them (a larger B or N) reallocates them, and launch then
 * fails with SDFNMPC_E_ARG instead of running on freed memory (destroy and create the step again).  Timing (sdfnmpc_ctx_enable_timing) does not
 * see graph launches.  (Not a reference interface: the acados solver object's solve() is one call too.) */
typedef struct sdfnmpc_step sdfnmpc_step;
int sdfnmpc_step_create(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_quad_model* model,
                        const sdfnmpc_lin_args* lin_args, const sdfnmpc_qp_opts* opts, const sdfnmpc_qp_args* qp_args,
                        double* u0, const int* status, sdfnmpc_step** out);
int sdfnmpc_step_launch(sdfnmpc_ctx* ctx, sdfnmpc_step* step);
void sdfnmpc_step_destroy(sdfnmpc_step* step);

/* ---- batched reference / parameter packing into the OCP device buffers (sdfnmpc_ref_args) ---- */
int sdfnmpc_pack_refs(sdfnmpc_ctx* ctx, const sdfnmpc_ref_opts* opts, const sdfnmpc_ref_args* args);

/* ---- in-loop VAE encoder ----
 * Replaces VaeWrapper.set_img + VaeWrapper.encode (sdf_nmpc/vae.py:29-40): preprocessing
 * (vae.py:15-24: float32 cast, Reshape's bilinear resize, ClipDistance, Depth2Range) and
 * Encoder.forward (network/vae.py:39-43, eval mode) for B images in one call on the context stream.
 * The encoder is the reference architecture (1 channel, conv7x7/2 + ELU + maxpool, ResBlocks
 * 64/128/256/512, avgpool 2x2, mean Linear); weights come as a `.vaew` blob (sdf-nmpc_amd/vae.py:pack)
 * with every BatchNorm folded into its convolution. */
typedef struct sdfnmpc_vae sdfnmpc_vae;

typedef struct {
    int B;                 /* images */
    int in_h, in_w;        /* raw image size; resized bilinearly to the encoder's H x W when different */
    int dtype;             /* 0 float32, 1 uint16 (ToDevice casts to float32) */
    float clip;            /* ClipDistance.dmax = sensor.dmax / sensor.mm_resolution * 1000 */
    const float* yz;       /* device [H][W] Depth2Range.yz_sqrt (sdf-nmpc_amd/vae.py:depth2range_table),
                              NULL when sensor.is_depth is false */
} sdfnmpc_vae_opts;

int sdfnmpc_vae_load(sdfnmpc_ctx* ctx, const void* vaew_blob, size_t bytes, sdfnmpc_vae** out);
void sdfnmpc_vae_free(sdfnmpc_vae* vae);
int sdfnmpc_vae_size_latent(const sdfnmpc_vae* vae);
/* img: device [B][in_h][in_w]; latent: device [B][L] float32; latent64: optional device [B][L] float64
 * (the precision Nmpc.set_latent stores into p).  The activation workspace (~5.7 MB per 270x480 image)
 * is owned by the encoder object and grows with B. */
int sdfnmpc_vae_encode(sdfnmpc_ctx* ctx, sdfnmpc_vae* vae, const sdfnmpc_vae_opts* opts, const void* img,
                       float* latent, double* latent64);

/* ---- device memory on a context (inputs of the device-side setters without a tensor library) ----
 * memcpy kind: 1 host -> device, 2 device -> host, 3 device -> device; ordered on the context stream,
 * synchronous (returns when the copy has completed). */
int sdfnmpc_dev_alloc(sdfnmpc_ctx* ctx, size_t bytes, void** out);
void sdfnmpc_dev_free(sdfnmpc_ctx* ctx, void* ptr);
int sdfnmpc_memcpy(sdfnmpc_ctx* ctx, void* dst, const void* src, size_t bytes, int kind);

/* ---- the batched SQP-RTI solver object (owns its device workspace) ----
 * Fields (name: [B][nodes][width] fp64 unless noted): x [N+1][10], u [N][4], p [N+1][np], x0 [1][10],
 * yref / W [N][ny], yNref / WN [1][nyN], u0 [1][4], dx [N+1][10], du [N][4], the sdfnmpc_lin_args outputs
 * xn, AB, y, Jy, yN [1][nyN], JyN [1][10 nyN], h, Jh, hE [1][6], JhE [1][60], res [1][2], slack [N+1][6]
 * ((sl, su) per soft row), status / iters [1][1] int32.  A field's device pointer may be handed to the
 * lower-level entry points (e.g. sdfnmpc_pack_refs or sdfnmpc_vae_encode writing p).  The network may be
 * NULL when the constraint set (qp.nh / h_col, qp.hN_col) and the cost (ny == 11) never read the SDF. */
typedef struct sdfnmpc_solver sdfnmpc_solver;

typedef struct {
    int B, N, np, ny;          /* instances, horizon, parameters per node, stage residuals (11 / 12) */
    int latent_mode;           /* as sdfnmpc_lin_args.latent_mode */
    const double* dt;          /* [N] shooting-grid steps (host; copied) */
    sdfnmpc_quad_model model;
    sdfnmpc_qp_opts qp;        /* qp.ny == ny */
} sdfnmpc_solver_opts;

int sdfnmpc_solver_create(sdfnmpc_ctx* ctx, const sdfnmpc_net* net, const sdfnmpc_solver_opts* opts,
                          sdfnmpc_solver** out);
void sdfnmpc_solver_destroy(sdfnmpc_solver* s);
int sdfnmpc_solver_field(sdfnmpc_solver* s, const char* name, void** dev, int* nodes, int* width);
/* host [B][nodes][width] (the caller's full mirror of the field): columns [col0, col0 + ncol) of the rows
 * r = b * nodes + k with row_mask[r] != 0 (row_mask NULL: every row) -> device.  Asynchronous: the data
 * is staged in pinned memory before the call returns, so host may be reused at once. */
int sdfnmpc_solver_upload(sdfnmpc_solver* s, const char* name, int col0, int ncol, const unsigned char* row_mask,
                          const double* host);
/* the whole field -> host [B][nodes][width] (synchronous) */
int sdfnmpc_solver_download(sdfnmpc_solver* s, const char* name, void* host);
/* reset + init (ocp.py:144-153): x0 = x_k = x0[b] for k = 0..N, u_k = u_init[4], dx = du = 0 */
int sdfnmpc_solver_init(sdfnmpc_solver* s, const double* x0, const double* u_init);
/* shift (ocp.py:152-156): x_{i-k} = x_i, u_{i-k} = u_i for i = k..N-1 (k <= 0 or k >= N: no-op) */
int sdfnmpc_solver_shift(sdfnmpc_solver* s, int k);
/* enqueue one SQP-RTI iteration: x_0 = x0, preparation phase, QP, full step (failed instances keep their
 * iterate), then u_0 / status / iterations into pinned host memory.  Asynchronous. */
int sdfnmpc_solver_step(sdfnmpc_solver* s);
/* wait for the stream; copy the last step's u0 [B][4], status [B], iters [B] (each may be NULL) */
int sdfnmpc_solver_wait(sdfnmpc_solver* s, double* u0, int* status, int* iters);

/* ---- shooting grid (host, bit-exact numpy.linspace/diff semantics of ocp.py:21-27) ---- */
int sdfnmpc_shooting_grid(int N, double T, int uniform, int nb_short_nodes, double dt_short, double* nodes,
                          double* dt);

#ifdef __cplusplus
}
#endif
#endif /* SDFNMPC_H */
