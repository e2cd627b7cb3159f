/*
 * kf.h — C ABI of libkfmi.so, the MI355X (gfx950) batched Kalman-filter engine.
 *
 * One handle holds B independent filters of one model on one GPU.  State lives in HBM
 * in structure-of-arrays form (filter index fastest):
 *     x  [n][B]                 state estimate
 *     P  [n(n+1)/2][B]          covariance, upper triangle packed row-major (i <= j)
 *     status [B] int32          KF_OK, or KF_ENOTSPD once a filter lost positive-definiteness
 * Per-step streams handed to the engine are device pointers in the same layout,
 * with the time index slowest:  u [T][c][B], z [U][m][B], traj [T][n][B], logdet [T][B].
 * Scalars are the handle's dtype (KF_F32 / KF_F64); time steps dt are always double
 * (absolute epoch stamps ~1.7e9 s are differenced on the host in fp64).
 *
 * The reference (IseanB/SensorFusion-KalmanFilter) has no native boundary: its hot path
 * is a per-event sequence of NumPy calls on KF_SensorFusion (kf_workers.py:493-621)
 * driven by Python time loops (kf_workers.py:623-728, 22-97).  Each entry point below
 * names the reference code it replaces.  The per-step math is
 *     x = F x + G u;  P = F P F^T + Q;  K = P H^T (H P H^T + R)^-1;
 *     x += K (z - H x);  then the covariance update, whose form depends on the model:
 *   - KF_MODEL_CV2 / CV3 (both dtypes): Joseph's form
 *         P = (I - K H) P (I - K H)^T + K R K^T   (north_star);
 *   - KF_MODEL_REF15 / REF8, fp64: the reference's own P = (I - K H) P (kf_workers.py:711,
 *     hw5_2.py:358, 376); a build with -DKF_REF_JOSEPH_F64=1 takes Joseph's form instead;
 *   - KF_MODEL_REF15 / REF8, fp32: Joseph's form (the simple form drifts in fp32);
 *   - the IMU pseudo-measurement's H = I chain updates of REF15 / REF8, both dtypes: P = K R,
 *     which equals (I - K H) P exactly when H = I and R is diagonal; a build
 *     with -DKF_REF_GAIN_R=0 takes the dtype's form above instead.
 * S^-1 comes from an in-lane LDL^T factorisation and logdet(P) from an LDL^T of P (block
 * determinants for the reference models).
 *
 * All functions return KF_OK (0) or a negative KF_E* code; kf_last_error() then
 * describes the failure (thread-local).  Launching entry points are asynchronous on
 * the given hipStream_t (NULL = the null stream) and never synchronise, so they can be
 * captured into a hipGraph.  Workspaces: kf_search_combos, kf_run_stream and
 * kf_run_scheduled(_rec) keep a device workspace in the handle, allocated by the first call
 * that needs it and grown (hipMalloc; hipFree synchronises the device) only by a call that
 * needs more than every earlier one; every other launch allocates nothing.  Run such a call
 * once eagerly before capturing it: inside a capture nothing is allocated (kf_run_scheduled
 * then takes its fused kernel, kf_run_stream returns KF_EINVAL; kf_search_combos synchronises
 * and is never captured).  A workspace a capture used
 * is never freed before kf_free, so a graph stays valid after a later, larger eager call: each
 * such growth keeps the smaller buffer (retired) until kf_free or kf_release_retired, so a
 * handle that alternates captures with ever-larger eager calls holds all of them.
 *
 * Threading: distinct handles may be used from different threads at once; one handle is used
 * by one thread at a time.  That includes the calls that only read it (kf_get_state,
 * kf_get_status, which therefore take a non-const handle): they run a held-back kf_predict
 * first (see kf_predict).
 */
#ifndef KFMI_KF_H
#define KFMI_KF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KF_OK        0
#define KF_EINVAL   (-1)  /* bad argument (shape, pointer, model, dtype)                      */
#define KF_EHIP     (-2)  /* HIP runtime error                                                */
#define KF_ENOTSPD  (-3)  /* per filter: S or P not positive definite; outputs become NaN.
                             Mirrors the reference skipping a failing combo (kf_workers.py:88-91) */
#define KF_ENODEV   (-4)  /* no usable gfx950 device                                          */
#define KF_ENOMEM   (-5)  /* device allocation failed                                         */

#define KF_F32 0
#define KF_F64 1

/* Models.  Both are restrictions of the reference models to [position, velocity] per axis,
 * with the IMU acceleration moved from state to control input u:
 *   KF_MODEL_CV2  n=4 m=2 c=2  [x, y, vx, vy]            hw5_2.py:219-304
 *   KF_MODEL_CV3  n=6 m=3 c=3  [x, y, z, vx, vy, vz]     kf_workers.py:493-614
 * F = [[I, dt I], [0, I]], G = [[dt^2/2 I], [dt I]], H = [I 0] (GPS position fix).       */
#define KF_MODEL_CV2 2
#define KF_MODEL_CV3 3

/* The reference's own 15-state GPS+IMU model (kf_workers.py:493-614): state
 * [pos(3), att(3), vel(3), rate(3), acc(3)], GPS fix m=3, IMU pseudo-measurement m=15, the
 * reference's constants (kf_params NULL) or a caller's diagonal ones (kf_params.ref_*).  Every
 * covariance reachable from a diagonal P0 is exactly block-diagonal over the axis chains (pos,vel,acc) and
 * (att,rate), so the handle stores P as 27 block-packed rows ([27][B]):
 *   rows 6i..6i+5   axis i (pos_i, vel_i, acc_i) upper triangle (pp pv pa vv va aa)
 *   rows 18+3i..+2  axis i (att_i, rate_i) upper triangle (tt tw ww)
 * Driven by per-filter event streams (kf_run_events) or the combination search (kf_eval_combos). */
#define KF_MODEL_REF15 15

/* The reference's 8-state planar model (hw5_2.py:219-311): state [x, y, theta, vx, vy,
 * theta_dot, ax, ay], GPS fix m=2 (easting, northing), IMU pseudo-measurement m=8 with theta =
 * yaw and theta_dot = wz (hw5_2.py:352-366), P0 = diag(1000, 1000, 100, 100, 100, 100, 1000,
 * 1000).  Same chain structure, 15 block-packed rows ([15][B]):
 *   rows 6i..6i+5   axis i in {x, y}: (pos_i, vel_i, acc_i) upper triangle
 *   rows 12..14     (theta, theta_dot) upper triangle
 * kf_run_events only; its trajectory records (x, y, theta) as hw5_2.py:369 does. */
#define KF_MODEL_REF8 8

/* Event codes for kf_run_events / kf_eval_combos. */
#define KF_EVENT_GPS     0    /* payload = (easting, northing, altitude, ...)              */
#define KF_EVENT_IMU     1    /* payload = (roll, pitch, yaw, wx, wy, wz, ax, ay, az)     */
#define KF_EVENT_PREDICT 2    /* predict only (the worker's final propagation)            */
#define KF_EVENT_NONE    255  /* no event: state unchanged (padding of ragged streams)    */

/* Model constants; kf_default_params() fills the reference's values.
 * KF_MODEL_CV2 / CV3 read q_pos .. p0_vel; KF_MODEL_REF15 / REF8 read the ref_* arrays: diagonal
 * Q rates, R_imu, R_gps and P0 per state, in the model's state order (REF8: the first 8 / 2
 * entries).  Diagonal constants keep every covariance block-diagonal over the axis chains, which
 * the handle's block-packed P requires.  The reference's getters hard-code them
 * (kf_workers.py:519-614, P0 :651; hw5_2.py:233-304, P0 :317-326) and its class_args dict of
 * callables lets a caller replace them (kf_workers.py:1242-1251).  A handle whose constants
 * equal the reference's runs the kernels compiled with the reference's literals. */
typedef struct kf_params {
    double q_pos;   /* Q = diag(q_pos*dt I, q_vel*dt I): 5, 1   (kf_workers.py:521,523)        */
    double q_vel;
    double r[9];    /* R, m x m row-major, symmetric: 3 I       (kf_workers.py:581-585)        */
    double p0_pos;  /* initial P = diag(p0_pos I, p0_vel I): CV3 1e4/1e3 (kf_workers.py:651), */
    double p0_vel;  /*                                         CV2 1000/100 (hw5_2.py:317-326) */
    double ref_q[15];      /* Q = diag(ref_q * dt), >= 0                                         */
    double ref_r_imu[15];  /* R_imu = diag(ref_r_imu), > 0                                       */
    double ref_r_gps[3];   /* R_gps = diag(ref_r_gps), > 0                                       */
    double ref_p0[15];     /* P0 = diag(ref_p0), > 0 (kf_reset / kf_alloc)                      */
} kf_params;

typedef struct kf_batch kf_batch;

/* Library version string: "kfmi <version> (gfx950) src:<hash>", where <hash> is the first 16 hex
 * digits of the SHA-256 of the sources the library was built from (the .cpp, .h and .hip files of
 * csrc in name order, then include/kf.h).  The Python binding refuses a library whose hash
 * differs from the tree it is loaded from (a stale or foreign build). */
const char* kf_version(void);

/* Per-handle options: the variant choices the library otherwise makes by itself, for A/B runs
 * and tests.  0 is the library's choice for every option, and a new handle starts with all 0.
 * Nothing is read from the environment.
 *   KF_OPT_PREDICT        0 = hold a scalar-dt kf_predict back and fuse it into the next
 *                         kf_update; 1 = eager (one kernel per call)
 *   KF_OPT_CV_KERNEL      kf_run on the BASELINE models: 0 = auto (cv_block_kernel when P is
 *                         block-diagonal and R diagonal), 1 = the general kernel,
 *                         2 / 4 / 8 = the block kernel with that input-ring depth (where legal)
 *   KF_OPT_BLOCKS_PER_CU  kf_run: cap resident workgroups per CU at 2..8 (reserving unused LDS);
 *                         0 = no cap
 *   KF_OPT_EVENTS_KERNEL  kf_run_events: 0 = auto, 1 = one lane per filter (inputs in registers),
 *                         2 = one lane per axis chain, 3 = LDS-staged inputs (where legal),
 *                         4 = one gated f64 filter (B = 1, gate) with closed-form look-ahead
 *                         over runs of predict-only events (8 events per wave step: 2.3x
 *                         the chain kernel at 3 % updated, slower from about 20 %; the
 *                         gated stream fallback picks it by itself, see kf_run_stream)
 *   KF_OPT_STREAM         kf_run_events: 0 = route one long filter through kf_run_stream,
 *                         1 = never (every filter in sequence)
 *   KF_OPT_STREAM_CHUNKS  kf_run_stream: target chunk count (>= 2); 0 = 8192
 *   KF_OPT_STREAM_FINAL   kf_run_stream: 0 = records from the map pass, 1 = a final pass from the
 *                         true chunk starts
 *   KF_OPT_START_THREADS  kf_run_stream: threads per block of the start kernel; 0 = 256
 *   KF_OPT_SEARCH_KERNEL  kf_search_combos: 0 = per level, 1 = child-major, 2 = parent-major
 *   KF_OPT_SEARCH_PM      kf_search_combos' parent-major kernel: 0 = parent in LDS, 1 = registers
 *   KF_OPT_SEARCH_HEAD    kf_search_combos: 0 = the first levels (sizes whose subsets need few event
 *                         steps in all) in one launch, one lane per subset; 1 = level by level
 *   KF_OPT_SEARCH_END     kf_search_combos: 0 = the last levels (sizes whose subsets need few event
 *                         steps from a stored prefix) in one launch, one lane per subset from its
 *                         stored prefix; 1 = level by level
 *   KF_OPT_SEARCH_PAIR    kf_search_combos, axis-symmetric: 0 = a parent-major level with at least
 *                         2^22 stored parents and the next level in one launch (the first level's
 *                         nodes kept in LDS, never stored: half the level traffic); 1 = one level
 *                         per launch; 2 = pair every parent-major level; 3 = pair every level
 *                         child-major, a wave per parent block and child event (measured slower;
 *                         A/B only); >= 1024 = pair the parent-major levels with at least that
 *                         many stored parents
 *   KF_OPT_AXIS_SYM       0 = where the handle's noise constants are the same on every axis
 *                         (the reference's), work that depends on the constants alone is done
 *                         once for the axes' identical chains: kf_run_stream's covariance maps
 *                         (one pva and one aw chain's maps stand for all: the same numbers, bit
 *                         for bit); kf_search_combos when the init covariance's axis blocks are
 *                         also equal bit for bit (one pva and one aw chain computed and stored:
 *                         the every-chain search's results to rounding, its three compiled
 *                         copies of a chain's arithmetic rounding alike in ~98 % of subsets, one
 *                         ulp apart in the rest); 1 = every chain
 *   KF_OPT_SCHED_KERNEL   kf_run_scheduled: 0 = auto (the two passes where legal, as 3), 1 = the
 *                         fused register-input kernel, 2 = the fused LDS-input kernel, 3 = the
 *                         pick and apply passes as two launches, 4 = as the two phases of one
 *                         launch
 *   KF_OPT_SCHED_GROUP    kf_run_scheduled's two passes: waves per workgroup, 0 = 4, 1 or 4
 *                         (one-wave groups free their slot when their wave's pick list ends;
 *                         measured slower; kf_run_scheduled_rec's apply pass: 4)
 *   KF_OPT_SCHED_ORDER    kf_run_scheduled's two launches: 0 = the apply pass runs the waves
 *                         heaviest first (their longest pick lists, sorted on the device),
 *                         1 = in batch order
 *   KF_OPT_SCHED_REC_TIME kf_run_scheduled_rec / _random over f64 records of rec_len >= 10:
 *                         0 = rec[9..] unread; 1 = rec[9] holds the event's time (t[i][f]) and
 *                         the apply pass takes each pick's time from the record it gathers
 *                         anyway (the pick pass then writes no sel_time row of its own: the apply
 *                         pass writes it, coalesced)
 * KF_EINVAL for an unknown option or an out-of-range value. */
#define KF_OPT_PREDICT        1
#define KF_OPT_CV_KERNEL      2
#define KF_OPT_BLOCKS_PER_CU  3
#define KF_OPT_EVENTS_KERNEL  4
#define KF_OPT_STREAM         5
#define KF_OPT_STREAM_CHUNKS  6
#define KF_OPT_STREAM_FINAL   7
#define KF_OPT_START_THREADS  8
#define KF_OPT_SEARCH_KERNEL  9
#define KF_OPT_SEARCH_PM      10
#define KF_OPT_SCHED_KERNEL   11
#define KF_OPT_SCHED_GROUP    12
#define KF_OPT_SCHED_ORDER    13
#define KF_OPT_SCHED_REC_TIME 14
#define KF_OPT_SEARCH_HEAD    15
#define KF_OPT_AXIS_SYM       16
#define KF_OPT_SEARCH_END     17
#define KF_OPT_SEARCH_PAIR    18
#define KF_OPT_COUNT          19
int kf_set_option(kf_batch* handle, int option, int64_t value);
int kf_get_option(const kf_batch* handle, int option, int64_t* value);

/* Thread-local description of the last failure on this thread ("" if none). */
const char* kf_last_error(void);

/* Reference constants for a model (every model; the ref_* arrays for REF15 / REF8).  Replaces the
 * hard-coded getters get_process_noise_covariance_matrix / get_*_measurement_noise_covariance_matrix
 * (kf_workers.py:519-614, hw5_2.py:233-304) and the P0 literals (kf_workers.py:651, hw5_2.py:317-326). */
int kf_default_params(int model, kf_params* out);

/* Number of visible HIP devices (0 on a host without a GPU). */
int kf_device_count(int* count);

/* Select device `device` for the calling thread and check that it is gfx950.
 * Idempotent.  No reference counterpart (the reference never leaves the CPU). */
int kf_init(int device);

/* Create a handle for `batch` filters of `model` in `dtype` on the current device, with
 * x = 0, P = P0, status = KF_OK.  params may be NULL (reference constants); KF_EINVAL for a
 * negative or non-finite Q rate or a non-positive R or P0 entry of a reference model.
 * Replaces KF_SensorFusion.__init__ + the per-run initial state (kf_workers.py:641-651). */
int kf_alloc(kf_batch** handle, int model, int64_t batch, int dtype, const kf_params* params);
int kf_free(kf_batch* handle);

/* Free the workspaces a graph capture used that larger eager calls have since replaced (see
 * "Workspaces" above); *bytes_freed (nullable) = their size.  Call it only once every graph
 * captured from this handle's calls is destroyed: their replays would write freed memory.
 * The workspaces in use stay.  Synchronises the device (hipFree). */
int kf_release_retired(kf_batch* handle, int64_t* bytes_freed);

/* Dimensions of a handle (any pointer may be NULL).  For KF_MODEL_REF15: n = 15, m = 3 (GPS),
 * c = 0, and the covariance has 27 block-packed rows instead of n(n+1)/2 (KF_MODEL_REF8: n = 8,
 * m = 2, c = 0, 15 rows). */
int kf_dims(const kf_batch* handle, int* n, int* m, int* c, int64_t* batch, int* dtype);

/* Re-initialise every filter: x = x0 (device [n][B]; NULL = zeros), P = P0, status = OK.
 * The reference's cold start sets the position to the first GPS fix and everything else to
 * zero (kf_workers.py:651-666). */
int kf_reset(kf_batch* handle, const void* x0, void* stream);

/* Copy state in/out.  on_device != 0: x/P are device pointers (async on stream);
 * on_device == 0: host pointers (synchronous).  The warm start of the reference
 * (initial_pt / initial_state, kf_workers.py:643-649) maps to kf_set_state. */
int kf_set_state(kf_batch* handle, const void* x, const void* P, int on_device, void* stream);
int kf_get_state(kf_batch* handle, void* x, void* P, int on_device, void* stream);
int kf_get_status(kf_batch* handle, int32_t* status, int on_device, void* stream);

/* One predict step for every filter: x = F(dt) x + G(dt) u, P = F P F^T + Q(dt).
 * dt_per_filter: device [B] double (NULL = scalar dt for all filters; the brute-force caller
 * has a different dt per combo, kf_workers.py:37).  u: device [c][B] (NULL = zero control).
 * logdet_out: device [B] (NULL = skip), logdet of the predicted P, as the adaptive-threshold
 * driver uses it (kf_workers.py:1023).
 * Replaces get_state_transition_matrix + get_process_noise_covariance_matrix +
 * x = np.dot(F, x) + predict_covariance (kf_workers.py:493-549, 688-691).
 * With a scalar dt and no logdet_out the step is held back and runs fused with the next
 * kf_update (one kernel, the state read and written once); a copy of u into the handle is
 * queued on `stream`, so the caller may overwrite u with work ordered after this call on
 * `stream`; a host write to u (pinned or managed memory) or a write on another stream must
 * first synchronise with `stream`.  Any other call that reads or replaces the state
 * (kf_get_state, kf_get_status, kf_set_state, kf_run, another kf_predict) runs a held-back
 * predict first, on its own stream; kf_reset discards it.  Results are those of the two
 * separate kernels (KF_OPT_PREDICT = 1).  The control buffer is allocated by kf_alloc, so a
 * predict/update loop allocates nothing and can be captured into a graph (capture whole
 * predict + update pairs: a predict left pending at the end of a capture runs outside it).
 * Warm-up on one stream and capture on another (the torch.cuda.graph pattern) works: a predict
 * whose control copy would have to wait for a kernel recorded outside the capture runs eagerly
 * instead (the same results). */
int kf_predict(kf_batch* handle, double dt, const double* dt_per_filter, const void* u,
               void* logdet_out, void* stream);

/* One GPS update for every filter: z device [m][B]; mask device [B] uint8 (NULL = all;
 * 0 = skip this filter); logdet_out device [B] (NULL = skip).
 * Replaces get_gps_observation_matrix + get_gps_measurement_noise_covariance_matrix +
 * calculate_kalman_gain + the state/covariance update + slogdet
 * (kf_workers.py:551-558, 581-585, 616-621, 694-717). */
int kf_update(kf_batch* handle, const void* z, const uint8_t* mask, void* logdet_out, void* stream);

/* The fused hot path: T steps for every filter in ONE launch, state held in registers.
 * Step t predicts with dt_t (dt_steps device [T] double, or the scalar dt when NULL) and
 * control u[t] (device [T][c][B]), then, when (t+1) % update_every == 0, updates with
 * z[(t+1)/update_every - 1] (device [U][m][B], U = T / update_every) unless
 * mask[(t+1)/update_every - 1][f] == 0 (mask device [U][B] uint8, NULL = all).
 * traj (device [T][n][B]) and logdet (device [T][B]) receive x and logdet(P) after every
 * step; either may be NULL.
 * Replaces the time loop of run_kalman_filter_full (kf_workers.py:681-721) and the per-combo
 * loop of evaluate_combo_chunk_worker (kf_workers.py:36-71), batched over filters. */
int kf_run(kf_batch* handle, int T, double dt, const double* dt_steps, const void* u,
           const void* z, const uint8_t* mask, int update_every, void* traj, void* logdet,
           void* stream);

/* Deterministic synthetic GPS+IMU streams for filters
 * [filter_offset, filter_offset + B) of a global population: counter-based Philox4x32-10
 * keyed by seed and the GLOBAL filter index, so any shard regenerates its own slice.
 * Truth: p0 ~ U(-1000,1000) m, v0 ~ N(0,10^2) m/s, a_t ~ N(0,0.3^2); u_t = a_t + N(0,0.1^2);
 * z = p_true + N(0,3).  x0_out [n][B] = (first fix, 0 velocity).  Outputs in the handle's
 * dtype, computed in fp64 and rounded once.  Not a reference entry point: it replaces the
 * missing imu_data.csv (.MISSING_LARGE_BLOBS) with a synthetic stream of the same shape. */
int kf_synth(kf_batch* handle, uint64_t seed, int64_t filter_offset, int T, double dt,
             int update_every, void* x0_out, void* u_out, void* z_out, void* stream);

/* KF_MODEL_REF15 / KF_MODEL_REF8: T events per filter in one launch.  etype device [T][B]
 * uint8 (KF_EVENT_*), dt device [T][B] double (time since the filter's previous event), payload
 * device [T][9][B] (handle dtype).  Per event: predict over dt, then the GPS update
 * (kf_workers.py:694-697) or the IMU pseudo-measurement update built from the predicted state
 * (:698-706); with gate != 0 the update is applied only when logdet(P_pred) > threshold
 * (:1023-1025).  Per-event records, each of which may be NULL: traj device [T][6][B] (REF8:
 * [T][3][B]) receives x[0:6] after each event (:714; hw5_2.py:369), cov device [T][27][B]
 * (REF8: [T][15][B]) the block-packed covariance (the sf_KF_covariance list of :739-824),
 * logdet [T][B] the log-determinant (:716-717), updated [T][B] uint8 whether the update was
 * applied.  Replaces the loops of run_kalman_filter_full (:681-721), run_kalman_filter
 * (:763-824), run_adaptive_threshold_kalman_filter (:1010-1053), run_no_update_kalman_filter
 * (:1110-1155, as KF_EVENT_PREDICT streams) and hw5_2.run_kalman_filter (hw5_2.py:328-380),
 * batched over filters. */
int kf_run_events(kf_batch* handle, int T, const uint8_t* etype, const double* dt, const void* payload,
                  void* traj, void* cov, void* logdet, uint8_t* updated, int gate, double threshold,
                  void* stream);

/* kf_run_events without its one-filter route through kf_run_stream: every filter runs its
 * events in sequence, whatever B and T are (same arguments and outputs).  For callers that want
 * the sequential single-filter run for one call (A/B, the reference's own op order over a whole
 * log) without the handle-wide KF_OPT_STREAM = 1. */
int kf_run_events_seq(kf_batch* handle, int T, const uint8_t* etype, const double* dt, const void* payload,
                      void* traj, void* cov, void* logdet, uint8_t* updated, int gate, double threshold,
                      void* stream);

/* One filter over a long event stream, parallel over time: kf_run_events for a handle of ONE
 * filter (B = 1, here without a gate), with the same arguments, outputs and final state, computed as
 * chunks of `chunk` events run as filters of one launch (chunk <= 0: max(128, T / 2048)).
 * Each chunk's start covariance comes from the covariance recursion's linear-fractional maps
 * (per chain and piece of <= 160 events), iterated over all chunks at once from the handle's
 * covariance (warmup = -1, the default; -2 - k adds k chunks of event warm-up), or from a
 * warm-up over the `warmup` events before the chunk (warmup >= 0).  The state recursion given
 * the gains is affine: each chunk runs from a guess and three perturbed guesses, whose ends
 * give its map start -> end; the maps are composed into the true chunk starts, and the records
 * are the map pass's (covariance, logdet, updated from the guess; the trajectory as the maps'
 * value at the true starts).  KF_OPT_STREAM_FINAL = 1 (or a stream too long for the four
 * trajectory variants' 32-bit offsets) runs a final pass from the true starts instead, with
 * its own state seam check.  Checked on the device: the start covariances must meet their
 * predecessors' end covariances (relative 1e-12 in f64, 1e-5 in f32), the chunk starts and end
 * state must be finite (final pass: every chunk's end state its successor's start, 1e-9 /
 * 1e-4), and no chunk filter may fail; otherwise the sequential kernel runs the stream as one
 * filter from the handle's state and rewrites every record.  Asynchronous on `stream` either
 * way.  kf_run_events takes this route by itself for B = 1 and T >= 65536 (KF_OPT_STREAM = 1
 * disables it); with its gate (the adaptive threshold, kf_workers.py:959-1058) the chunk starts
 * come from 2048 events of warm-up that apply the gate (the maps cannot carry it) and every
 * pass and the fallback apply it too, the seam check deciding as above; in f64 with update
 * flags requested, a fallback whose chunked pass updated at most 1 event in 8 runs the
 * look-ahead kernel (KF_OPT_EVENTS_KERNEL = 4: same flags, records to rounding, 1.8e-12
 * relative measured), chosen on the device (KF_OPT_EVENTS_KERNEL = 2 keeps the chain
 * kernel).  The run of
 * run_kalman_filter_full (kf_workers.py:623-728) over a whole drive log. */
int kf_run_stream(kf_batch* handle, int T, const uint8_t* etype, const double* dt, const void* payload,
                  void* traj, void* cov, void* logdet, uint8_t* updated, int chunk, int warmup,
                  void* stream);

/* The checks of the handle's last kf_run_stream (synchronises `stream`): out[0] = 1 if the
 * chunked run's records stood (0: the sequential fallback ran), out[1] = 1 if a chunk filter
 * failed, out[2] = covariance seam gap, out[3] = state seam gap (final pass only; records from
 * the map pass: NaN = not measured, the chunk starts being the composed maps' values, or inf for
 * a non-finite chunk start), out[4] = chunks (1: the stream was too short to split
 * and ran sequentially), out[5] = chunk length, out[6] = events of event warm-up, out[7] = the
 * sequential fallback's kernel (0 = none, the chunked records stood; 2 = the chain kernel; 4 =
 * the look-ahead kernel, which a gated f64 run takes when its chunked pass updated at most 1
 * event in 8).  out: 8 doubles. */
int kf_stream_check(kf_batch* handle, double* out, void* stream);

/* KF_MODEL_REF15 brute-force search: filter f of the handle evaluates combination number
 * combo_offset + f (itertools.combinations order) of k out of n_events candidate events, from the
 * common initial state init (host [15 + 27] doubles: x, block-packed P), exactly as
 * evaluate_combo_chunk_worker does (kf_workers.py:22-97): events in combination order, an event
 * with negative dt skipped, then a predict to target_end.  events: host [n_events][11] doubles
 * (t, KF_EVENT_GPS|KF_EVENT_IMU, payload[9]), n_events <= 64.  Outputs per filter: the final
 * state in the handle, logdets device [k+2][B] (records, NaN-padded) and max_logdet device [B]
 * (the brute-force acceptance test max(log_det) < R_threshold, :1353), n_records device [B];
 * status 1 marks lanes past the last combination.  With logdets non-NULL, (k + 2) * B * w must
 * stay below 4 GiB (KF_EINVAL otherwise; w = 8 for f64, 4 for f32).  Replaces the Pool(30) fan-out of
 * run_brute_force_kalman_filter_no_sampling_min_usage (:1320-1346). */
int kf_eval_combos(kf_batch* handle, int n_events, const double* events, const double* init,
                   double prev_time, double target_end, int k, uint64_t combo_offset, void* logdets,
                   void* max_logdet, int32_t* n_records, void* stream);

/* KF_MODEL_REF15 brute-force search with shared prefixes: the search of
 * run_brute_force_kalman_filter_no_sampling_min_usage (kf_workers.py:1218-1392) over the
 * subsets of the n_events candidates, for subset sizes k = 1 .. k_max.  The filter of a subset
 * is its prefix's filter (stored in device level buffers owned by the handle) advanced by one
 * event, so each subset costs one event step plus the worker's final predict instead of a
 * whole filter run; the arithmetic per subset is kf_eval_combos's.  A subset is accepted when
 * its max log-determinant (records as kf_eval_combos) is < threshold (:1353).  The search
 * stops after the first size with an accepted subset unless `exhaustive`.  Host outputs:
 * *k_found = that size (0 = none), *winner = bit mask (bit i = candidate i) of its first
 * accepted subset in itertools.combinations order (the reference's pick, :1349-1356),
 * n_fixed / fixed_mask: search only the subsets whose intersection with candidates
 * 0 .. n_fixed - 1 is fixed_mask (0 / 0 = every subset; one class per GPU shards the search
 * evenly, kfmi.dist), k_max counting the fixed candidates,
 * n_accepted host [k_max + 1] (nullable) accepted subsets per size (0 past *k_found when not
 * `exhaustive`).  subset_max: device [2^n] of the handle's dtype (n_events <= 30, nullable)
 * receives every evaluated subset's max log-determinant (NaN for a failed filter), indexed by
 * mask; not `exhaustive`, the sizes past *k_found that the one-launch head scored are written
 * too (KF_OPT_SEARCH_HEAD; the level-by-level search leaves them untouched).  Level k stores the C(n - 2, k)
 * subsets whose largest free candidate is <= n - 3 (a subset holding n - 1 has no extensions,
 * one holding n - 2 only the one adding n - 1, which is scored from registers); C(n - 2, k)
 * must stay below 2^28, and the handle's level buffers take 2 * C(n - 2, k) * (28 w + 20)
 * bytes at the widest stored level (w = 8 for f64, 4 for f32; n = free candidates; 10 w + 20
 * for an axis-symmetric search, KF_OPT_AXIS_SYM).  The call synchronises `stream` (its results
 * return to the host through a mapped host buffer of the handle), so it cannot be captured into
 * a hipGraph: inside a capture it returns KF_EINVAL. */
int kf_search_combos(kf_batch* handle, int n_events, const double* events, const double* init,
                     double prev_time, double target_end, double threshold, int k_max, int exhaustive,
                     int n_fixed, uint64_t fixed_mask, uint64_t* winner, int* k_found,
                     uint64_t* n_accepted, void* subset_max, void* stream);

/* How kf_search_combos would run with these arguments, without running it (no device work):
 * out[0] = 1 if axis-symmetric (KF_OPT_AXIS_SYM and init's axis blocks equal bit for bit),
 * out[1] = the workspace bytes it needs (two buffers of the widest stored level plus 4 KiB),
 * out[2] = the widest stored level's nodes, out[3] = the most stored parents of a level,
 * out[4] = the first size over the 2^28-parent cap (0 = none; kf_search_combos refuses it).
 * The host uses it to split a search too large for one call into classes (n_fixed /
 * fixed_mask) run one after another (kfmi.ref15.search_combos_classed). */
int kf_search_plan(const kf_batch* handle, int n_events, const double* init, int n_fixed, uint64_t fixed_mask,
                   int k_max, int64_t* out);

/* The last kf_search_combos on this handle: out[0] = 1 if it ran axis-symmetric
 * (KF_OPT_AXIS_SYM: one pva and one aw chain for the three of each), out[1] = the sizes its
 * head launch covered (KF_OPT_SEARCH_HEAD; 0 = none), out[2] = its level launches after the
 * head, out[3] = the bytes of one of its two level buffers.  All 0 before the first search. */
int kf_search_info(const kf_batch* handle, int64_t* out);

/* KF_MODEL_REF15 scheduler scoring: gain device [n_types][B] = trace of the posterior
 * covariance each candidate sensor type (types: host [n_types] KF_EVENT_GPS|KF_EVENT_IMU,
 * n_types <= 16) would give every filter's current covariance.  full = 0: the reference's
 * Scheduler.gain, an update with the first measurement row only (cov_matrix(S=[1]),
 * kf_workers.py:112-147, 174-185); full = 1: every measurement row of the sensor.  post:
 * device [n_types][27][B] block-packed posterior covariances (Scheduler.cov_matrix), or NULL. */
int kf_score_candidates(kf_batch* handle, int n_types, const int32_t* types, int full, void* gain,
                        void* post, void* stream);

/* KF_MODEL_REF15 Scheduler.cov_matrix for any measurement rows S (kf_workers.py:112-147: H_hat =
 * H[S], R_hat = R[S, S]): candidate c is sensor types[c] (KF_EVENT_GPS | KF_EVENT_IMU) with the rows
 * of row_masks[c] (host, bit i = 1-based row i + 1 of that sensor's H: GPS rows 1..3 = pos x, y, z;
 * IMU rows 1..15 = the 15 states; non-zero).  gain device [n_cand][B] = trace of the posterior,
 * post device [n_cand][27][B] the block-packed posterior (nullable).  R is the handle's (diagonal)
 * R_gps / R_imu, so the rows are independent and each chain takes its own.  n_cand <= 16. */
int kf_score_rows(kf_batch* handle, int n_cand, const int32_t* types, const uint32_t* row_masks, void* gain,
                  void* post, void* stream);

/* KF_MODEL_REF15 rate-decimated greedy filter (run_kalman_filter_scheduled with
 * selection_method='greedy', kf_workers.py:826-957), per filter.  By default two passes: the
 * windows and picks from the event times and types (the greedy pick's gains differ only in R,
 * so the constants decide it), then the picked events, with the gains checked on the covariance
 * wherever both sensor classes were queued; a filter where they disagree (a NaN covariance, a
 * rounding tie) is rerun by the fused kernel.  The handle keeps a [T][B] pick workspace, grown
 * on demand; inside a graph capture it is never allocated, so a capture before any eager call of
 * that T runs the fused kernel (same outputs to rounding).  The apply pass runs the waves with
 * the longest pick lists first (KF_OPT_SCHED_ORDER).  Streams:
 * t device [T][B] absolute event times (double), etype device [T][B] (KF_EVENT_GPS|IMU, NONE =
 * padding at the end), payload device [T][9][B].  prev_time device [B]: time of the state in the
 * handle.  Events within 1/f of the last processed one are queued; the first event past the
 * window triggers the greedy pick from the queue (first candidate with the largest Scheduler.gain
 * on the current covariance; the trigger itself is dropped unless the queue was empty, as in the
 * reference), then one predict over the accumulated dt and one update.  f per filter: freq
 * device [B] (a sampling sweep in one launch), or freq_all when freq is NULL.  Outputs per
 * selection s (compacted): traj [s][6][B], logdet [s][B], sel_time [s][B]; n_sel [B]. */
int kf_run_scheduled(kf_batch* handle, int T, const double* t, const uint8_t* etype, const void* payload,
                     const double* prev_time, const double* freq, double freq_all, void* traj, void* logdet,
                     double* sel_time, int32_t* n_sel, void* stream);

/* kf_run_scheduled with the payload as one record per event: records device [T][B][rec_len], the
 * 9 values of kf_run_scheduled's payload at rec[0..8] (rec[9..] unread: the reference keeps each
 * event's sensor values together, sdata of its (index, type, time, sdata) tuples,
 * kf_workers.py:870, 910).  rec_len >= 9 with rec_len * element size a multiple of 16 bytes
 * (f64: 10, f32: 12) and records 16-byte aligned, else KF_EINVAL.  The picked events' values are
 * then one contiguous span per filter instead of nine rows B elements apart, which is what the
 * apply pass gathers.  The memory moves whole 128-byte lines (every read request
 * of the apply pass measures 128 B), so the shortest record packs a wave's picks of one event
 * into the fewest lines: f64 rec_len 10 with the event's time at rec[9] (KF_OPT_SCHED_REC_TIME),
 * 80 B per pick where a wave's lanes pick the same event.  Same outputs as kf_run_scheduled, bit
 * for bit. */
int kf_run_scheduled_rec(kf_batch* handle, int T, const double* t, const uint8_t* etype, const void* records,
                         int rec_len, const double* prev_time, const double* freq, double freq_all, void* traj,
                         void* logdet, double* sel_time, int32_t* n_sel, void* stream);

/* The random arm (run_kalman_filter_scheduled with selection_method='random', kf_workers.py:
 * 826-957, Scheduler.random_schedule :188-193): the same windows and outputs as kf_run_scheduled,
 * the pick drawn as np.random.choice(len(queue)) draws it from NumPy's global legacy RandomState —
 * randint(0, n): no draw for n = 1, else 32-bit generator outputs masked to the smallest
 * 2^k - 1 >= n - 1 until one is <= n - 1.  The windows follow the picks (each one opens at the
 * picked event's time), so the draws happen on the device, in the reference's order, from
 * words device [n_words][B] u32: column f holds the raw 32-bit outputs filter f consumes in
 * order (for the reference's one filter, the next n_words outputs of np.random's MT19937:
 * RandomState.randint(0, 2**32, n, dtype=uint32) on a copy of its state).  words_used device
 * [B] int32: the outputs each filter took (the caller advances its generator by that many), or
 * -1 if its column ran out (its outputs stop at the last completed pick; retry with more).
 * payload: [T][9][B] rows (rec_len 0) or [T][B][rec_len] records as kf_run_scheduled_rec. */
int kf_run_scheduled_random(kf_batch* handle, int T, const double* t, const uint8_t* etype, const void* payload,
                            int rec_len, const double* prev_time, const double* freq, double freq_all,
                            const uint32_t* words, int n_words, int32_t* words_used, void* traj, void* logdet,
                            double* sel_time, int32_t* n_sel, void* stream);

/* The random arm's picks alone: the same windows and draws as kf_run_scheduled_random (they need
 * no filter state), no filter run.  pick device [T][B] int32: the picked events' indices (the
 * first n_sel[f] rows of filter f), sel_time [T][B] their times, words_used as above.  Run the
 * picked events through kf_run_events (dt = sel_time[s] - sel_time[s - 1], the first from
 * prev_time): for ONE filter over a long log that is kf_run_events' time-parallel route, which
 * is what kfmi.ref15.run_kalman_filter_scheduled does for the reference's one filter.  Any
 * model's handle (only its batch size is used). */
int kf_sched_random_picks(kf_batch* handle, int T, const double* t, const uint8_t* etype, const double* prev_time,
                          const double* freq, double freq_all, const uint32_t* words, int n_words, int32_t* words_used,
                          int32_t* pick, double* sel_time, int32_t* n_sel, void* stream);

/* ---------------------------------------------------------------------------------------
 * Ingest: CSV logs -> one merged event stream in HBM (the reference's load_data,
 * gps_to_modified_utm, compute_imu_biases, unbias_imu_data, combine_sensor_data;
 * kf_workers.py:290-385, hw5_2.py:15-119).
 * --------------------------------------------------------------------------------------- */

/* Data rows and the field count of the first data row of a CSV file (header skipped when
 * has_header; trailing blank lines are not rows).  Host-only, no GPU needed. */
int kf_csv_shape(const char* path, int has_header, int64_t* rows, int* cols);

/* Parse the first ncols fields of each of `rows` data rows into host out[col * ld + row]
 * (column-major doubles).  A field containing "nan" in any case becomes NaN (the reference's
 * 'nan' in s.lower() test, kf_workers.py:310, 336); any other field must parse as Python's
 * float() would, else KF_EINVAL naming the row and column.  Multithreaded, host-only.
 * Replaces load_data_from_csv (kf_workers.py:290-298) + the float() calls at each use. */
int kf_csv_read(const char* path, int has_header, int ncols, double* out, int64_t ld, int64_t rows);

#define KF_INGEST_GPS_ALTITUDE 1  /* kf_workers.py:310: drop a fix whose altitude is 'nan' too;
                                     0 = hw5_2.py:35 (latitude/longitude only)              */

typedef struct kf_ingest_info {
    int64_t n_events;           /* fixes kept + IMU rows                                    */
    int64_t n_fixes;            /* len(utm_data)                                            */
    int64_t n_imu;
    int64_t first_valid_index;  /* compute_imu_biases: first GPS row with a latitude        */
    int64_t origin_row;         /* GPS row of the first kept fix (UTM origin), -1 if none   */
    double gyro_bias[3];        /* angular_velocity_bias                                    */
    double accel_bias[3];       /* linear_acceleration_bias                                 */
    double utm_origin[2];       /* easting/northing subtracted from every fix               */
} kf_ingest_info;

/* Build the merged event stream.  gps device [4][ld_gps] (time, latitude, longitude,
 * altitude), imu device [11][ld_imu] (time, orientation x y z w, angular velocity x y z,
 * linear acceleration x y z) — the column layouts hw5_1.py:14-38 writes.  bias: host [6]
 * (angular velocity, linear acceleration) to subtract instead of the compute_imu_biases means,
 * or NULL.  Outputs (device,
 * capacity >= n_gps + n_imu; info->n_events rows written): etype [N] (KF_EVENT_GPS/IMU),
 * t [N], payload [N][9] — fix: (easting - e0, northing - n0, altitude, 0...), the UTM
 * projection of the `utm` package; IMU: (roll, pitch, yaw, w - bias_w, a - bias_a) —
 * src [N] (position in utm_data for a fix, IMU row index), zone_number [N], zone_letter [N]
 * (0 for IMU rows); src/zone_* may be NULL.  Events are ordered by time, fixes first on ties
 * (Python's stable sort, kf_workers.py:384).  Synchronous (the event count is returned).
 * KF_EINVAL when no GPS row has a latitude (the reference's biases are undefined then). */
int kf_ingest(const double* gps, int64_t n_gps, int64_t ld_gps, const double* imu, int64_t n_imu, int64_t ld_imu,
              int flags, const double* bias, uint8_t* etype, double* t, double* payload, int32_t* src,
              int8_t* zone_number, char* zone_letter, kf_ingest_info* info, void* stream);

/* quaternion_to_euler (kf_workers.py:399-425) for n quaternions: q device [4][ld] (x, y, z, w),
 * out device [3][n] (roll, pitch, yaw). */
int kf_quat_to_euler(int64_t n, const double* q, int64_t ld, double* out, void* stream);

/* Time since the previous event for a driver over a merged stream, computed on the device.
 *   KF_DT_FULL      run_kalman_filter_full (kf_workers.py:682-686): previous = the previous
 *                   event's time; a negative dt marks the event KF_EVENT_NONE (skipped)
 *   KF_DT_MONOTONE  adaptive / no-update drivers and the combination worker (:1012-1016,
 *                   :1113-1116, :38-40): a skipped event does not move the previous time
 *   KF_DT_RAW       run_kalman_filter / hw5_2 (:763-767, hw5_2.py:331-336): no guard
 * t/etype_in/dt/etype_out device [n]; prev0 = the time of the state the run starts from, or
 * NaN for a driver with no previous time yet, whose first event gets dt 0 (hw5_2.py:401, 407;
 * FULL and RAW only); etype_in NULL = all KF_EVENT_IMU; etype_out may be NULL. */
#define KF_DT_FULL     0
#define KF_DT_MONOTONE 1
#define KF_DT_RAW      2
int kf_events_dt(int64_t n, const double* t, const uint8_t* etype_in, double prev0, int rule, double* dt,
                 uint8_t* etype_out, void* stream);

/* The events of one type out of a merged stream, in stream order: hw5_2.run_dead_reckoning_for_IMU
 * walks the IMU events alone, skipping every fix (hw5_2.py:402-404).  etype device [n], t device
 * [n], payload device [n][9] (kf_ingest's layout); writes the K kept events' t_out [K],
 * payload_out [K][9] and src_out [K] (their stream positions), each of which may be NULL, with
 * capacity n, and *n_kept = K (host).  Synchronous (the count is returned): inside a hipGraph
 * capture it returns KF_EINVAL before queuing anything.  Its scratch (block counts, a mapped host
 * int) is per device, allocated by the first call, so later calls allocate nothing; `stream` must
 * belong to the current device (KF_EINVAL otherwise). */
int kf_events_select(int64_t n, const uint8_t* etype, const double* t, const double* payload, int keep_type,
                     double* t_out, double* payload_out, int32_t* src_out, int64_t* n_kept, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* KFMI_KF_H */
