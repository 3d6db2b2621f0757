/*
 * cmpc.h -- C-ABI of the MI355X batched convex-MPC contact-force QP solver.
 *
 * Drop-in boundary for the QP solve of ltinphan/convex-mpc-unitree-go2:
 *   convex_mpc/centroidal_mpc.py:212-213  ca.conic('S', 'osqp', {h, a}, OPTS)   -> cmpc_plan_create
 *   convex_mpc/centroidal_mpc.py:76-98    _update_sparse_matrix + _compute_bounds
 *                                         + self.solver(h, g, a, lba, uba, lbx, ubx)
 *                                                                                -> cmpc_solve
 *   convex_mpc/centroidal_mpc.py:113-119  self.solver.stats()['return_status']  -> status[]
 *
 * One call solves B independent instances of the reference QP (centroidal_mpc.py:122-359):
 *   min  sum_k (x_{k+1}-xref_k)' Q (x_{k+1}-xref_k) + u_k' R u_k
 *   s.t. x_{k+1} = Ad x_k + Bd_k u_k + gd           (k = 0..N-1, x_0 given)
 *        swing leg:  f = 0                           (centroidal_mpc.py:150-161)
 *        stance leg: fz >= fz_min, |fx| <= mu fz, |fy| <= mu fz
 *                                                    (centroidal_mpc.py:163-170, 264-283, 324-359)
 * which is exactly ½w'Hw + g'w of the reference with H = diag(2Q.., 2R..), g = [-2Q xref; 0]
 * (up to the constant sum xref'Q xref).
 *
 * Layouts (row-major, all device pointers, caller-owned):
 *   Ad      [B][12][12]        fp32   (traj.Ad)
 *   Bd      [B][N][12][12]     fp32   (traj.Bd)
 *   gd      [B][12]            fp32   (traj.gd)
 *   x0      [B][12]            fp32   (traj.initial_x_vec)
 *   xref    [B][N][12]         fp32   (traj.compute_x_ref_vec() transposed: xref[b][k] is the
 *                                      reference's column k = target for x_{k+1})
 *   contact [B][4][N]          uint8  (traj.contact_table, legs FL FR RL RR; nonzero = stance)
 *   w_out   [B][24N]           fp32   reference decision layout (centroidal_mpc.py:44,
 *                                      test_MPC.py:190-192): w = [x_1..x_N | u_0..u_{N-1}],
 *                                      each 12 contiguous, i.e. vec(X (12,N),'F') then vec(U,'F')
 *   status  [B]                int32  1 solved: an active-set polish passed the KKT check --
 *                                       primal violations <= polish_tol x the force scale us
 *                                       (<= 5 x for a loose acceptance; the returned forces are
 *                                       then projected onto the pyramid), a refinement step
 *                                       <= polish_tol x us that was still contracting (never
 *                                       one stalled on a face-downdated factorization), and, for
 *                                       the reference's nilpotent step matrix (float64 rollout),
 *                                       a CERTIFIED bound on the force error of the held faces:
 *                                       with c = sum_f min(lambda_f, 0) a_f over the faces held,
 *                                       |u - u*|_2 <= |c|_2 / min(2R) <= 5e-5 x us (strong
 *                                       convexity).  Together: within ~1e-4 of the optimum
 *                                       except along directions weighed only by R, which the
 *                                       fp32 refinement resolves poorly (fresh-seed surveys:
 *                                       2 of 196,606 status-1 answers at 1.1e-4 / 2.1e-4 at
 *                                       polish_refine 2, none above 5.6e-5 at polish_refine 4,
 *                                       DESIGN.md 8).
 *                                     2 solved inaccurate: ADMM residuals within eps, or a polished
 *                                       point that misses the certified bound (returned, but not
 *                                       verified to 1e-4),
 *                                     -2 max iterations, -10 numerical failure
 *   iters   [B]                int32  ADMM iterations taken
 *
 * Threading: one plan per host thread / stream.  cmpc_solve is asynchronous on `stream`
 * (a hipStream_t, NULL = default stream); it performs no allocation, no host synchronisation
 * and is graph-capturable.  Return codes are 0 or a negative CMPC_E* value; the message is
 * available from cmpc_last_error() (thread-local).
 */
#ifndef CMPC_H_
#define CMPC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 6: status 1 carries a certified force-error bound (see status above); cmpc_plan_stats.
 * 5: the interior-point variant and its cmpc_plan_set_ipm / cmpc_plan_ipm_batch are gone
 *    (cmpc_params.reserved0 must be 0).  4: three solve-kernel timing slots. */
#define CMPC_ABI_VERSION 6

#define CMPC_OK 0
#define CMPC_E_INVALID (-22)   /* bad argument / parameter (EINVAL) */
#define CMPC_E_NOMEM (-12)     /* device allocation failed (ENOMEM) */
#define CMPC_E_HIP (-5)        /* HIP runtime error (EIO) */
#define CMPC_E_RANGE (-34)     /* batch larger than the plan's max_batch (ERANGE) */

/* Solver parameters.  cmpc_params_default() fills the reference's values
 * (centroidal_mpc.py:12-38, fz_min from :127) and this solver's ADMM settings. */
typedef struct cmpc_params {
  int32_t abi_version;    /* must be CMPC_ABI_VERSION */
  int32_t N;              /* horizon, 1..16 (reference: 16, com_trajectory.py:66) */
  float Q[12];            /* state weight diagonal (centroidal_mpc.py:12) */
  float R[12];            /* input weight diagonal (centroidal_mpc.py:13) */
  float mu;               /* friction coefficient (centroidal_mpc.py:15) */
  float fz_min;           /* stance normal-force lower bound (centroidal_mpc.py:127) */
  float eps_abs;          /* ADMM residual tolerances for status 2 (OPTS eps_abs/eps_rel) */
  float eps_rel;
  int32_t max_iter;       /* ADMM iteration cap (OPTS max_iter) */
  float rho;              /* initial ADMM penalty (the NC = 128 bin starts at rho / 2 and returns
                             to rho after a failed polish session) */
  float sigma;            /* ADMM proximal regularisation (OSQP sigma) */
  float alpha;            /* over-relaxation (OSQP alpha) */
  int32_t adaptive_rho_interval; /* iterations between rho updates (0 = off) */
  int32_t polish_stable;  /* polish after the active set is unchanged this many iterations */
  int32_t polish_refine;  /* refinement steps inside the polish before its convergence test may
                             stop them (up to 4 more while the step still halves); default 2
                             (4: ~5 % slower, tighter along R-weighted directions) */
  float polish_tol;       /* relative KKT tolerance for accepting the polished point */
  int32_t polish_repairs; /* active-set repairs (add violated / drop negative-multiplier faces
                             and re-polish) before resuming ADMM */
  int32_t reserved0;      /* must be 0 (ABI 4's ipm_facts: the interior-point fallback was
                             removed in ABI 5) */
  int32_t check_termination; /* ADMM iterations between termination tests (OPTS check_termination,
                             centroidal_mpc.py:31): the polish trigger (face set stable for
                             polish_stable iterations -> active-set polish + KKT check, the only
                             way an instance ends solved) is evaluated only at iterations that
                             are multiples of it.  Default 1: here the test is one wave ballot
                             of the face codes, so checking every iteration costs nothing, while
                             OSQP's 10 amortises a residual evaluation (two sparse matvecs) this
                             solver does not need.  The reference's 10 is accepted (the drop-in
                             CentroidalMPC passes it): same solutions, iterations rounded up to
                             multiples of 10. */
  int64_t max_batch;      /* largest B passed to cmpc_solve (sizes plan workspace) */
} cmpc_params;

typedef struct cmpc_plan cmpc_plan;

/* Fill *p with defaults.  Replaces the OPTS dict (centroidal_mpc.py:20-36). */
void cmpc_params_default(cmpc_params* p);

/* Validate params, allocate workspace for max_batch instances on the current device.  Every
 * later call with this plan must run with that device current (else CMPC_E_INVALID).
 * Replaces CentroidalMPC.__init__/_build_sparse_matrix (centroidal_mpc.py:41-67,178-230). */
int cmpc_plan_create(const cmpc_params* p, cmpc_plan** out);

/* Solve B instances (see layouts above).  Replaces CentroidalMPC.solve_QP's update + solve
 * (centroidal_mpc.py:69-120) for a whole batch.  `stream` is a hipStream_t or NULL. */
int cmpc_solve(cmpc_plan* plan, int64_t B, const float* Ad, const float* Bd, const float* gd,
               const float* x0, const float* xref, const uint8_t* contact, float* w_out,
               int32_t* status, int32_t* iters, void* stream);

/* Warm-started solve: the reference's x0 / lam_x0 / lam_a0 warm start
 * (centroidal_mpc.py:91-95, kept from the previous solve at :108-110; OPTS warm_start_primal /
 * warm_start_dual, :33-34).  As cmpc_solve, plus:
 *   w_init  [B][24N]  fp32  nullable; a previous w_out (optionally shifted by the caller).
 *                           Only the force part (w_init[b][12N + 12k + 3l + a]) is used: each
 *                           stance force starts at its projection onto the friction pyramid.
 *   y_init  [B][12N]  fp32  nullable; a previous y_out (force layout, swing entries ignored).
 *   y_out   [B][12N]  fp32  nullable; this solver's dual at the returned forces: -grad of the
 *                           condensed objective at u* (zero on swing legs).  It is cmpc's own
 *                           multiplier, not OSQP's lam_a (there are no constraint rows here).
 * With w_init, the faces of the friction pyramid the warm point holds (its forces on a face to
 * fp32 rounding, or pushed outward by y_init) go straight to the active-set polish: when that
 * face set (after up to polish_repairs repairs) passes the KKT check, the solve takes one
 * reduced factorization and no ADMM iteration (iters = 0).  Otherwise ADMM starts from
 * x = z = the projected warm forces, y = y_init (or 0).
 * NaN/Inf warm entries start at zero.  w_init may alias w_out and y_init may alias y_out (every
 * instance reads its warm data before it writes its outputs).  Both NULL == cmpc_solve. */
int cmpc_solve_warm(cmpc_plan* plan, int64_t B, const float* Ad, const float* Bd,
                    const float* gd, const float* x0, const float* xref,
                    const uint8_t* contact, const float* w_init, const float* y_init,
                    float* w_out, float* y_out, int32_t* status, int32_t* iters, void* stream);

/* Solve with the REFERENCE's multipliers (SURVEY.md 8(b) y_inout; centroidal_mpc.py:91-95
 * warm start lam_x0 / lam_a0, :108-110 sol["lam_x"] / sol["lam_a"]).  As cmpc_solve, plus:
 *   w_init    [B][24N]  fp32  nullable; primal warm start, as for cmpc_solve_warm.
 *   lam_init  [B][52N]  fp32  nullable; warm duals in the reference layout
 *                             [lam_x (24N: states, then forces) | lam_a (28N: 12N dynamics rows,
 *                             then 16N friction rows fx-mu fz, -fx-mu fz, fy-mu fz, -fy-mu fz per
 *                             (step, leg))], CasADi's sign convention.  Mapped on the device to
 *                             this solver's force dual y = F' lam_fric + lam_x[u].
 *   lam_out   [B][52N]  fp32  nullable; the multipliers of the returned point in the same layout:
 *                             H w + g + A' lam_a + lam_x = 0 with lam > 0 on active upper and
 *                             lam < 0 on active lower bounds (lam_a dynamics rows = minus the
 *                             adjoint of the rollout; friction / fz-bound multipliers from the
 *                             accepted face set; swing forces lam_x = -(2R u - Bd' lam_eq)).
 * lam_init may alias lam_out and w_init may alias w_out. */
int cmpc_solve_ref(cmpc_plan* plan, int64_t B, const float* Ad, const float* Bd, const float* gd,
                   const float* x0, const float* xref, const uint8_t* contact,
                   const float* w_init, const float* lam_init, float* w_out, float* lam_out,
                   int32_t* status, int32_t* iters, void* stream);

void cmpc_plan_destroy(cmpc_plan* plan);

/* QP data on the device: the reference's discrete dynamics
 * (com_trajectory.py:221-286, _continuousDynamics + _discreteDynamics) for B robots, in closed
 * form.  Ac is nilpotent (Ac^2 = 0), so the ZOH of com_trajectory.py:278 is exactly
 * Ad = I + Ac dt, Bd_k = (I dt + Ac dt^2/2) Bc_k, and the 50-sample trapezoid of :281-284 is
 * exact for its linear integrand: gd = (I dt + Ac dt^2/2) gc.  Computed in fp64, stored fp32.
 *   mass    [B]            fp32   go2.data.Ig.mass (com_trajectory.py:39)
 *   inertia [B][3][3]      fp32   I_com_world (com_trajectory.py:40); inverted on the device
 *   r_feet  [B][N][4][3]   fp32   lever arms COM -> foot in the world frame, legs FL FR RL RR
 *                                 (r_*_foot_world[:, k], com_trajectory.py:108-207, 242-245)
 *   xref    [B][N][12]     fp32   as for cmpc_solve; yaw_avg = mean_k xref[b][k][5]
 *                                 (np.average(rpy_traj_world[2, :]), com_trajectory.py:226)
 *   Ad, Bd, gd                    outputs, in cmpc_solve's input layouts
 * N is the plan's horizon; dt > 0 (com_trajectory.py:210, time_step).  Asynchronous on
 * `stream`; the outputs can be passed straight to cmpc_solve on the same stream. */
int cmpc_build_dynamics(cmpc_plan* plan, int64_t B, float dt, const float* mass,
                        const float* inertia, const float* r_feet, const float* xref,
                        float* Ad, float* Bd, float* gd, void* stream);

/* Reference trajectory, contact table and foot levers on the device: the
 * reference's ComTraj.generate_traj (com_trajectory.py:27-207) up to the dynamics, for B robots,
 * with the Pinocchio quantities it reads passed in (see oracle/traj_ref.py):
 *   x0         [B][12]    fp32   go2.compute_com_x_vec() (com_trajectory.py:37): p, rpy, v, w.
 *                                R_z(x0[5]) is go2.R_z; (R_z R_y R_x)(x0[3:6])' is
 *                                go2.R_world_to_body (go2_robot_data.py:211-222)
 *   pos_des    [B][3]     fp64   in/out: ComTraj.pos_des_world, the per-robot desired position
 *                                (initialise to x0[0:3], com_trajectory.py:12-13); clamped to
 *                                0.1 m of x0 in x/y and set to the commanded z (:47-60)
 *   cmd        [B][4]     fp32   x_vel_des_body, y_vel_des_body, z_pos_des_body,
 *                                yaw_rate_des_body (generate_traj's arguments, :27-35)
 *   t_now      [B]        fp64   time_now (:30)
 *   gait       [B][6]     fp64   gait_period (= 1/frequency_hz), duty, phase offsets FL FR RL RR
 *                                (gait.py:8, 13-19)
 *   foot_lever [B][4][3]  fp32   go2.get_foot_lever_world() (:113, go2_robot_data.py:261-269)
 *   hip        [4][3]     fp32   go2.get_hip_offset(leg), body frame (gait.py:46), all robots
 *   xref       [B][N][12] fp32   out: compute_x_ref_vec() transposed (cmpc_solve's layout)
 *   contact    [B][4][N]  uint8  out: contact_table (:106, gait.py:26-37), bit-identical
 *   r_feet     [B][N][4][3] fp32 out: r_{fl,fr,rl,rr}_foot_world (:108-207), the levers
 *                                cmpc_build_dynamics takes
 * N is the plan's horizon (the reference's int(gait_period / time_step)); dt = time_step > 0.
 * Asynchronous on `stream`; the outputs chain into cmpc_build_dynamics and cmpc_solve. */
int cmpc_generate_traj(cmpc_plan* plan, int64_t B, double dt, const float* x0, double* pos_des,
                       const float* cmd, const double* t_now, const double* gait,
                       const float* foot_lever, const float* hip, float* xref, uint8_t* contact,
                       float* r_feet, void* stream);

/* The reference's 1 kHz leg controller for B robots (the consumer of the
 * QP's first forces): LegController.compute_leg_torque for legs FL FR RL RR
 * (leg_controller.py:43-112; test_MPC.py:199-225) -- stance tau = J_foot' (-f) (:100-101),
 * swing tau = J_foot' (KP e_p + KD e_v + Lambda (a_des - Jdot dq)) + (C dq + g)[leg] with
 * Lambda = (J_full M^-1 J_full')^-1 (:75-98) and the swing trajectory planned at take-off
 * (gait.py:77-174) -- then clipped to +-tau_max (test_MPC.py:227-228; tau_max <= 0: no clip).
 * Pinocchio's quantities are inputs (fp64, as the reference computes them):
 *   t        [B]           time_now;  gait [B][6] as for cmpc_generate_traj
 *   force    fp32 rows of 12, row stride force_stride (>= 12) floats: U[:, 0] of each robot,
 *            e.g. w_out + 12 N with stride 24 N (test_MPC.py:196)
 *   J_foot   [B][4][3][3]  compute_3x3_foot_Jacobian_world(leg) (go2_robot_data.py:286-301)
 *   J_full   [B][4][3][18] compute_full_foot_Jacobian_world(leg) (:347-353)
 *   M, C     [B][18][18]   compute_dynamcis_terms() (:355-360);  g, dq [B][18]
 *   Jdot_dq, foot_pos, foot_vel [B][4][3]  compute_Jdot_dq_world, get_single_foot_state_in_world
 *   body     [B][16]  base_pos(3), pos_com_world(3), vel_com_world(3), yaw (R_z),
 *                     yaw_rate_des_world, x/y_pos_des_world, x/y_vel_des_world, 0
 *                     (what gait.py:80-96 reads; the des values generate_traj stored)
 *   hip      [4][3]   get_hip_offset(leg)
 *   state    [B][4][8] in/out, the controller's memory: last mask (initialise to 2), take-off
 *                     time, swing start (3), touchdown (3)  (leg_controller.py:41, 67-72, 104)
 *   tau      [B][12]  out, fp64. */
int cmpc_leg_torque(cmpc_plan* plan, int64_t B, const double* t, const double* gait,
                    const float* force, int64_t force_stride, const double* J_foot,
                    const double* J_full, const double* M, const double* C, const double* g,
                    const double* dq, const double* Jdot_dq, const double* foot_pos,
                    const double* foot_vel, const double* body, const double* hip,
                    double* state, double tau_max, double* tau, void* stream);

/* Closed-loop stand-in for the simulator (MuJoCo is absent from this image):
 * advance B single-rigid-body robots by nsub substeps of dt under the held ground forces U[:, 0]
 * (rows of 12 fp32, row stride force_stride), with the gait deciding contact at each substep.
 *   t_now [B] fp64 (start time, not advanced), gait [B][6] as above, mass [B],
 *   inertia_body [B][3][3] (body-frame I_com), hip [4][3];
 *   x [B][12] in/out (p, rpy, v, w_world: the MPC state), feet [B][4][3] in/out (world foot
 *   positions, used while in stance), contact_state [B] in/out (bit l: leg l in stance).
 * Not a reference interface: it exists to exercise the on-device tick in closed loop. */
int cmpc_srb_step(cmpc_plan* plan, int64_t B, int nsub, double dt, const double* t_now,
                  const double* gait, const float* mass, const float* inertia_body,
                  const float* force, int64_t force_stride, const float* hip, float* x,
                  float* feet, uint8_t* contact_state, void* stream);

/* Measurement hooks (not on the reference's interface; used by bench.py).  A solve launches at
 * most CMPC_NUM_SOLVE_KERNELS persistent solve kernels; cmpc_plan_solve_kernel names solve
 * kernel k (0, 1 or 2) of a batch of B instances, or returns NULL if that slot is not launched:
 *   B <= cmpc_plan_team_batch:  "solve_team_kernel<4, 1>" (B <= CUs: one workgroup per CU)
 *                               or "solve_team_kernel<4, 2>" (k = 0 only);
 *   larger batches:             "solve_group_kernel<128, 96>" (k = 0, the NC <= 128
 *                               class), "solve_group_kernel<160, 144>" (k = 1, the
 *                               NC 144 / 160 class; NULL if N is too short to need it) and
 *                               "solve_group_kernel<192, 0>" (k = 2, the NC 192 bin, more
 *                               than 160 free forces; NULL if N is too short).  Slots are
 *                               per kernel, whichever class is submitted first
 *                               (cmpc_plan_set_heavy_first).
 * While enabled, cmpc_solve records a hipEvent pair around each solve-kernel launch on the
 * stream it is launched on -- for slot 2 only the NC 192 kernel's early launch (a few waves on
 * the highest-priority plan stream, submitted before the classes); its overflow launch, which
 * drains what those waves left after both classes are done, is not timed.  An event pair spans
 * the launch's queueing too: with an empty bin the early launch's waves exit at once, but they
 * are dispatched only when the class kernels free a SIMD, so that span can read milliseconds
 * while holding nothing.  cmpc_plan_timing_read waits for the recorded events, returns the
 * summed milliseconds per kernel slot (ms_per_kernel[CMPC_NUM_SOLVE_KERNELS]) and the launch
 * counts since the last read, and resets them.  At most 4096 x CMPC_NUM_SOLVE_KERNELS launches
 * are recorded between reads (later ones are not timed). */
#define CMPC_NUM_SOLVE_KERNELS 3
int cmpc_plan_set_timing(cmpc_plan* plan, int enable);
int cmpc_plan_timing_read(cmpc_plan* plan, float* ms_per_kernel, int32_t* calls_per_kernel);
const char* cmpc_plan_solve_kernel(const cmpc_plan* plan, int64_t B, int k);

/* Small-batch mode.  A solve of B <= max_batch instances runs each QP on a workgroup of four
 * waves (one per SIMD of a CU) that split the condensation, the inversion and the matrix-vector
 * products, instead of one wave per QP: B = 256 on 256 CUs otherwise leaves 3 of every 4 SIMDs
 * idle.  All five bins then run in one kernel on `stream` (timed as solve kernel 0).  Results
 * are the same algorithm's (parity-tested in both modes).  max_batch = -1 (the default) selects
 * it for B <= 4 x CUs; 0 disables it.  cmpc_plan_team_batch returns the effective bound. */
int cmpc_plan_set_team(cmpc_plan* plan, int64_t max_batch);
int cmpc_plan_team_batch(const cmpc_plan* plan, int64_t* max_batch);

/* Launch order of the two register classes.  A batch above the small-batch bound launches one
 * persistent kernel per register class (NC <= 128: two waves per SIMD; NC 144 / 160: one; plus
 * the NC 192 bin's kernel, submitted before both on its own stream); the
 * class submitted first fills the device and the other takes SIMDs as they free up, so the
 * step ends with the tail of the class that runs second.  Batches of B >= min_batch submit the
 * NC 144 / 160 class first (its tail is then filled by NC <= 128 waves: config 3 at 65,536 and
 * 16,384 faster), smaller ones the NC <= 128 class (config 2 at 4,096 faster).  Results do not
 * depend on the order (each instance is solved by one wave, deterministically).
 * min_batch = -1 (the default) selects B > 16 x CUs; 0 never.  cmpc_plan_heavy_first_batch
 * returns the effective bound (0: never). */
int cmpc_plan_set_heavy_first(cmpc_plan* plan, int64_t min_batch);
int cmpc_plan_heavy_first_batch(const cmpc_plan* plan, int64_t* min_batch);

/* Acceptance statistics (not on the reference's interface; bench.py reports them): cumulative
 * counts over every solve with this plan since creation or the last reset, read after a device
 * synchronisation:
 *   out[0]  loose acceptances (a polish session that ended on a face set within 5 x polish_tol);
 *   out[1]  answers returned as status 2 because the certified face bound was missed;
 *   out[2]  KKT checks that ran on a refinement that had stopped contracting on a face-downdated
 *           factorization (its step no longer bounds the error): each time the face set was
 *           refactored and the check redone on a fresh refinement;
 *   out[3]  reserved (0).
 * reset != 0 zeroes the counters after reading.  The copy and the reset run on the plan's own
 * stream, never on the null stream (a null-stream operation from the library slowed the
 * caller's later HIP-graph replays). */
#define CMPC_NUM_STATS 4
int cmpc_plan_stats(cmpc_plan* plan, uint64_t* out, int reset);

/* Thread-local description of the last error returned on this thread ("" if none). */
const char* cmpc_last_error(void);

/* Build / ABI identification, e.g. "cmpc 1 gfx950". */
const char* cmpc_version(void);

#ifdef __cplusplus
}
#endif

#endif /* CMPC_H_ */
