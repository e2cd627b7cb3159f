// Internal interface between the C ABI (kf_capi.cpp) and the gfx950 kernels (kf_cv.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kfmi {

// Everything one launch of a constant-velocity kernel needs.  Passed by value (kernarg
// segment), so wave-uniform values land in SGPRs.
struct CvArgs {
    int64_t B;               // filters in this handle
    int T;                   // time steps in this launch (kf_run), 1 for predict/update
    int update_every;        // k: update after step t when (t+1) % k == 0
    double dt;               // scalar dt (used when dt_steps == nullptr)
    const double* dt_steps;  // [T] per-step dt or nullptr
    const double* dt_filter; // [B] per-filter dt (kf_predict only) or nullptr
    void* x;                 // [n][B]
    void* P;                 // [n(n+1)/2][B]
    int32_t* status;         // [B]
    const void* u;           // [T][c][B] or nullptr (zero control)
    const void* x0;          // [n][B] reset state (Op::Reset) or nullptr (zeros)
    const void* z;           // [U][m][B]
    const uint8_t* mask;     // [U][B] or nullptr
    void* traj;              // [T][n][B] or nullptr
    void* logdet;            // [T][B] or nullptr
    double q_pos, q_vel;     // Q = diag(q_pos dt, q_vel dt)
    double r[6];             // R upper triangle, packed row-major (m <= 3)
    double p0_pos, p0_vel;   // reset covariance
    int block_p;             // P is block-diagonal over the axes (kf_run may use cv_block_kernel)
    int prefetch_depth;      // cv_block_kernel's input ring: 2, 4 or 8 steps
    int blocks_per_cu;       // 2..8: cap resident workgroups per CU (KF_OPT_BLOCKS_PER_CU); 0 = none
};

struct SynthArgs {
    int64_t B;
    int64_t filter_offset;
    uint64_t seed;
    int T;
    int update_every;
    double dt;
    void* x0;                // [n][B]
    void* u;                 // [T][c][B]
    void* z;                 // [U][m][B]
};

struct StreamCheck;

// A reference-model handle's noise constants when the caller set its own (kf_params): diagonal,
// per state in the model's state order (REF8 uses the first 8 / 2 entries).  Q = diag(q dt)
// (kf_workers.py:519-544), R_imu = diag(r_imu) (:587-614), R_gps = diag(r_gps) (:581-585),
// P0 = diag(p0) (:651).  Kernels read them through a device pointer (kc below); kc = nullptr
// selects the kernels compiled with the reference's constants.
struct RefConsts {
    double q[15];
    double r_imu[15];
    double r_gps[3];
    double p0[15];
};

// Reference chain models on per-filter event streams: KF_MODEL_REF15 (kf_workers.py:493-614,
// N = 15, NBLK = 27, NTRAJ = 6) and KF_MODEL_REF8 (hw5_2.py:219-311, N = 8, NBLK = 15, NTRAJ = 3).
// Event codes in etype: 0 GPS fix, 1 IMU sample, 2 predict only, 255 no event (padding).
struct RefArgs {
    int64_t B;
    int T;
    const uint8_t* etype;    // [T][B]
    const double* dt;        // [T][B] time since the filter's previous event
    const void* payload;     // [T][9][B]: GPS (easting, northing, altitude, -), IMU (roll, pitch,
                             // yaw, wx, wy, wz, ax, ay, az) as in kf_workers.py:367
    void* x;                 // [N][B]
    void* P;                 // [NBLK][B] block-packed covariance (see kf_ref.hip)
    int32_t* status;         // [B]
    const void* x0;          // reset: [N][B] or nullptr
    void* traj;              // [T][NTRAJ][B] x[0:NTRAJ] after each event, or nullptr
    void* cov;               // [T][NBLK][B] covariance after each event, or nullptr
    void* logdet;            // [T][B] or nullptr
    uint8_t* updated;        // [T][B] 1 if the event's update was applied, or nullptr
    int gate;                // adaptive threshold (kf_workers.py:1023-1025): update only if
    double threshold;        //   logdet(P_pred) > threshold
    // Stream mode (kf_run_stream, chain kernel only): ONE event stream of s_len events, laid
    // out as a single filter's [S] / [S][9] / records [S][W] ...; filter f runs the events
    // (f % s_nchunks) * s_chunk + s_shift + t, t < T; events outside [0, S) are skipped and
    // record nothing.  s_len = 0: the per-filter [T][B] layout above.
    int64_t s_len;
    int64_t s_chunk;
    int64_t s_shift;
    int64_t s_nchunks;
    int s_nvar;              // > 1: trajectory records per variant (filter / s_nchunks), s_vstride rows apart
    int64_t s_vstride;
    const int32_t* skip;     // if non-null and *skip != 0, the launch does nothing
    const RefConsts* kc;     // the handle's own noise constants (device), or nullptr: the reference's
    // the map pass of kf_run_stream (4 state variants per filter): its epilogue writes each
    // chunk's affine state map per chain, [C][chains][12] = A (3x3 row-major), b, from the
    // variants' end states (their starts differ by s_delta on one chain component), and checks
    // the covariance seam against the next chunk's start covariance s_wnext ([NBLK][C])
    double* s_maps;
    double s_delta;
    const void* s_wnext;
    StreamCheck* s_check;
};

// Time-parallel run of one filter over a long event stream (kf_run_stream): the state banks of
// the three chunk passes and the check.  Bank layouts are the handle's ([N][B], [NBLK][B]).
struct StreamCheck {
    int32_t ok;              // 1: the chunked run passed every check, its records stand
    int32_t bad;             // a chunk filter failed (non-SPD)
    double cov_gap;          // max over chunk seams of the warm-up covariance's relative gap
    double state_gap;        // max over chunk seams of |end state - next start| / max(|start|, 1)
    int32_t done;            // chain blocks of the scan phase that have finished (the last decides)
    int32_t pad;
    // the sequential fallback's kernel of a gated f64 run (launch_stream_choose): each kernel
    // returns at once when its flag is set.  The start phases zero skip_chain only (no choice:
    // the chain kernel runs on ok alone)
    int32_t skip_chain;      // ok, or the look-ahead kernel takes the fallback
    int32_t skip_gated;      // ok, or the chain kernel takes the fallback
};
struct StreamArgs {
    int64_t C;               // chunks
    double delta;            // state perturbation of the map pass (a power of two)
    double rdelta;           // 1 / delta (exact)
    double tol_state, tol_cov;
    void* hx;                // handle state (one filter): [N], [NBLK], status
    void* hP;
    int32_t* hstatus;
    void* wx;                // warm-up bank [.][C]: each chunk's start covariance and a state guess
    void* wP;
    int32_t* wst;
    void* mx;                // map bank [.][4C]: guess + 0 / delta e_q (q = chain component)
    void* mP;
    int32_t* mst;
    void* fx;                // final bank [.][C]: the true chunk starts, run with the records
    void* fP;
    int32_t* fst;
    double* maps;            // [C][chains][12]: per chunk and chain, A (3x3) and b of x_end = A x_start + b
    double* pref;            // [C][chains][12]: the product of the chunk maps before c in c's tile
    double* tiles;           // [C / kScanTile][chains][12]: each tile's product
    double* tstart;          // [C / kScanTile][chains][3]: each tile's start (phase 3), or nullptr
                             // (one scan round of tiles: the starts kernel composes its prefix)
    double* starts;          // [N][C] the chunk starts (fp64)
    double* dtab;            // [C][chains][4] (records from the map pass): start - guess per chain component
    StreamCheck* check;
    // covariance start by linear-fractional maps (kf_run_stream's default warm-up)
    const uint8_t* etype;    // the stream [S], dt [S]
    const double* dt;
    int64_t S, L;            // stream length, chunk length
    int kp;                  // polish chunks: the warm-up bank starts chunk c from P(c - kp)
    int np;                  // pieces per chunk (of lp events) with a covariance map each
    int64_t lp;
    double* phi;             // [C][np][chains][36]: per piece and chain, the 6x6 covariance map [[A B] [C D]]
    int iters;               // chunk maps (at least) behind every chunk start
    int64_t G;               // chunks per block of the start kernel (their windows' maps staged in LDS)
    int64_t g;               // chunks per thread of the start kernel; 0: no LDS, one chunk per thread
    int start_threads;       // threads per block of the start kernel (KF_OPT_START_THREADS); 0 = kBlock
    int sym;                 // KF_OPT_AXIS_SYM: the constants are the same on every axis, so the
                             // covariance maps of one pva and one aw chain (chains 0 and NP) stand
                             // for every chain (lft_maps computes only those; lft_start reads them)
    const RefConsts* kc;     // the handle's noise constants, or nullptr (the reference's)
    // records from the map pass (no final pass): the map bank's trajectories per variant
    const void* traj4;       // [4][vstride][NTRAJ]
    int64_t vstride;
    void* traj;              // [S][NTRAJ] the records: variant 0 + sum_q A_q (start - guess)_q
    double* xend;            // [N] the last chunk's end state (fp64)
};
// phase 0: warm-up bank from the handle, check zeroed; 1: map bank from the warm-up bank;
// 2-4: the chunk maps (written by the map pass) composed into every chunk start by a parallel
// scan (tiles, tile starts, chunk starts; then the final bank's starts, or with records from
// the map pass the verdict); 5: state seam check, verdict, and (if it passed) the handle's
// final state after a final pass
hipError_t launch_stream_phase(int model, bool f64, int phase, const StreamArgs& a, hipStream_t stream);
// after the verdict of a gated f64 stream run: the sequential fallback goes to the look-ahead
// kernel (ref_chain_gated_kernel) when at most 1 in `share_den` of the chunked run's update flags
// is set (a sample of up to 64K of them), else to the chain kernel (check->skip_chain / skip_gated)
hipError_t launch_stream_choose(StreamCheck* check, const uint8_t* updated, int64_t T, int share_den,
                                hipStream_t stream);
// the linear-fractional covariance warm-up: phase 6 = every chunk's covariance map, phase 7 =
// every chunk's start covariance from the maps (and the warm-up / map banks, the zeroed check)
constexpr int kStreamPhaseLftMaps = 6, kStreamPhaseLftStart = 7;
// check->bad bits: a chunk filter failed / a chunk start or the end state is not finite
constexpr int kStreamBadFilter = 1, kStreamBadStart = 2;
// records from the map pass: phase 8 = trajectories from the variants and the chunk starts
constexpr int kStreamPhaseScanTiles = 2, kStreamPhaseTop = 3, kStreamPhaseStarts = 4, kStreamPhaseFinish = 5,
              kStreamPhaseRecords = 8;
constexpr int64_t kStreamScanTile = 256;  // chunks per scan tile (kScanTile in kf_ref.hip)

// Brute-force search over k-subsets of n candidate events (kf_workers.py:22-97, 1218-1392):
// lane f evaluates combination number combo_offset + f in itertools.combinations order.
struct Ref15ComboArgs {
    int64_t B;
    int n_events;
    int k;
    uint64_t combo_offset;
    uint64_t n_combos;       // C(n, k)
    const double* ev;        // device [n][11]: t, type, payload[9]
    const uint64_t* binom;   // device [65][65] binomial coefficients
    double prev_time;
    double target_end;
    const double* init;      // device [15 + 27]: x0, P0 blocks
    void* x;                 // [15][B] final state per combination
    void* P;                 // [27][B]
    int32_t* status;         // [B]: 0, KF_ENOTSPD, or 1 = padding lane (no combination)
    void* logdets;           // [k+2][B] record list (NaN-padded) or nullptr
    void* max_logdet;        // [B] or nullptr
    int32_t* n_records;      // [B] or nullptr
    const RefConsts* kc;     // the handle's noise constants, or nullptr (the reference's)
};

// Brute-force search with shared prefixes (kf_search_combos): the filter of a k-subset S is its
// parent's (S minus its largest event) advanced by one event, so level k is built from level
// k - 1's stored states.  Levels are in colex order: the subsets whose largest event is j hold
// ranks [C(j, k), C(j + 1, k)) and child rank = parent rank + C(j, k).  One lane per parent
// evaluates all of its children.  Level buffer: node blocks of 64 nodes, block b =
//   [28][64] T       block-packed P (27), the running max log-det's determinant: its mantissa
//                    (NaN = failed filter); no state: the max log-det depends on the covariance
//                    alone (sym: [10][64], one pva block, one aw block, the mantissa)
//   [64] int32       the running max's binary exponent
//   [64] double      time of the last applied event
//   [64] uint64      subset bit mask
struct Ref15SearchArgs {
    int n_events;            // free candidates (events shift .. shift + n_events - 1 of ev_all)
    int k;                   // child level: k free events (k >= 1; k = 1 builds the root)
    int shift;               // fixed candidates below the free ones
    int k_base;              // popcount(root_mask): level k holds subsets of size k_base + k
    uint64_t root_mask;      // the fixed candidates every subset of this search contains
    const double* ev_all;    // device [shift + n_events][11]
    uint64_t n_par;          // C(n - 2, k - 1) stored parents (largest event <= n - 3), one lane each
    uint64_t n_child;        // C(n, k)
    const double* ev;        // device [n_events][11]: the free candidates (t, type, payload[9])
    const uint64_t* binom;   // device [65][65]
    const uint64_t* binom_host;  // host copy (launch geometry)
    const double* init;      // device [15 + 27]: root state (level 0)
    double prev_time;        // root time
    double target_end;
    double threshold;        // acceptance: max log-det < threshold (kf_workers.py:1353)
    // the same test on the max's determinant (set_search_band): accepted below 2^lo_e lo_m,
    // rejected above 2^hi_e hi_m, the log decides in between; mode 1 / 2 / 3: accept all / a
    // zero determinant only / none
    double band_lo_m, band_hi_m;
    int band_lo_e, band_hi_e, band_mode;
    const void* par;         // level k - 1 buffer (unused for k = 1)
    void* child;             // level k buffer, or nullptr when level k is not stored
    uint64_t* best;          // device [65]: per subset size, max over accepted subsets of bitrev(mask)
    uint64_t* n_acc;         // device [65]: per subset size, number of accepted subsets
    void* subset_max;        // device [2^n] T: every subset's max log-det by mask, or nullptr
    int tail;                // level k + 1 is searched: a child holding event n - 2 is not stored, its
                             // only child (plus event n - 1) is scored by this launch (size k + 1)
    // child-major work items (k >= 2; filled by launch_ref15_search): group i holds the parent
    // blocks whose first parent's largest event is v = v_lo + i, blocks [gblk[i], gblk[i + 1]),
    // each with n - 1 - v items (child events v + 1 .. n - 1); its first item is gitem[i]
    int v_lo, n_groups;
    uint64_t gitem[66];
    uint64_t gblk[66];
    bool pm_regs;            // parent-major: the parent's covariance in registers, not LDS (KF_OPT_SEARCH_PM)
    bool sym;                // axis-symmetric: the noise constants and the root's blocks are the same on
                             // the three axes, so the three pva chains (and the three aw chains) carry
                             // the same covariance; one of each is computed and stored
                             // (KF_OPT_AXIS_SYM)
    const RefConsts* kc;     // the handle's noise constants, or nullptr (the reference's)
    // a non-exhaustive search queues several levels between its result peeks: a level launch
    // does nothing when an earlier launch accepted a subset of a size it completed
    // (stop_best[stop_lo .. stop_hi] not all zero; stop_hi - stop_lo < 64; nullptr: no test)
    const uint64_t* stop_best;
    int stop_lo, stop_hi;
    int k_end;               // the end launch (launch_ref15_search_end): sizes k .. k_end
};

// T rows of a search node: the block-packed P (27) and the running max's mantissa; an
// axis-symmetric search (Ref15SearchArgs::sym) keeps one pva block and one aw block (6 + 3) and
// the mantissa; then 4 B of exponent, 8 B of time and 8 B of mask per node
__host__ __device__ constexpr int search_rows(bool sym) { return sym ? 10 : 28; }
__host__ __device__ constexpr uint64_t search_block_bytes(uint64_t elem, bool sym = false) {
    return 64 * (search_rows(sym) * elem + 20);
}
__host__ __device__ inline uint64_t search_level_bytes(uint64_t nodes, uint64_t elem, bool sym = false) {
    return (nodes + 63) / 64 * search_block_bytes(elem, sym);
}

// Scheduler scoring (kf_workers.py:112-185): trace of the posterior covariance each candidate
// sensor would give, per filter.  full = 0: the reference's S = [1] (first measurement row
// only); full = 1: every row of the sensor.
struct Ref15ScoreArgs {
    int64_t B;
    int n_types;
    int full;
    int8_t types[16];        // KF_EVENT_GPS / KF_EVENT_IMU per candidate
    const void* x;
    const void* P;
    void* gain;              // [n_types][B]
    void* post;              // [n_types][27][B] posterior covariance blocks, or nullptr
    const RefConsts* kc;     // the handle's noise constants, or nullptr (the reference's)
    int rows;                // 1: candidate c updates with the measurement rows masks[c] (kf_score_rows)
    uint32_t masks[16];      //    bit i = row i + 1 of the sensor's H (Scheduler.cov_matrix's S)
};

// Rate-decimated greedy driver (run_kalman_filter_scheduled, kf_workers.py:826-957), per filter.
struct Ref15SchedArgs {
    int64_t B;
    int T;
    const double* t;         // [T][B] absolute event times (fp64)
    const uint8_t* etype;    // [T][B]
    const void* payload;     // [T][9][B], or [T][B][pay_rec] records
    int pay_rec;             // 0: payload rows [T][9][B]; else elements per record (kf_run_scheduled_rec)
    const double* prev_time; // [B] time of the state in the handle
    const double* freq;      // [B] processing frequency per filter, or nullptr
    double freq_all;         // used when freq == nullptr
    void* x;
    void* P;
    int32_t* status;
    void* traj;              // [T][6][B] per selection (compacted)
    void* logdet;            // [T][B]
    double* sel_time;        // [T][B]
    int32_t* n_sel;          // [B]
    bool regs;               // the register-input kernel even where the LDS one is legal (KF_OPT_SCHED_KERNEL)
    const RefConsts* kc;     // the handle's noise constants, or nullptr (the reference's)
    // two-pass run (launch_ref15_scheduled): a pick pass (windows, queue, greedy rule from the
    // constants; no covariance) writes picks[s][f] = code << 24 | event index and sel_time, an
    // apply pass runs the picked events (checking the greedy rule on the covariance wherever
    // both sensor classes were queued), and the fused kernel reruns any filter flagged there
    uint32_t* picks;         // [T][B] workspace
    int32_t* flags;          // [B] workspace: 1 = rerun this filter (the rule and the gains disagreed)
    const int32_t* only;     // fused kernel: only the filters with only[f] != 0 (nullptr = all)
    int gps_wins;            // both classes queued: 1 the GPS fix wins, 0 the other event, -1 a tie
    bool fused;              // the fused kernels (KF_OPT_SCHED_KERNEL 1 / 2) instead of the two passes
    int group_waves;         // the two passes' waves per workgroup (KF_OPT_SCHED_GROUP: 1 or 4)
    bool one_launch;         // the two passes as the phases of one kernel (KF_OPT_SCHED_KERNEL 4)
    // heaviest waves first (KF_OPT_SCHED_ORDER 0): the pick pass writes each wave's longest pick
    // list (wave_key) and its index (wave_id); a descending radix sort gives `order`, the apply
    // pass's wave sequence.  All nullptr: batch order.
    uint32_t* wave_key;      // [B / 64]
    uint32_t* wave_id;       // [B / 64]
    uint32_t* wave_key_sorted;
    uint32_t* order;         // [B / 64]
    void* sort_tmp;
    size_t sort_tmp_bytes;
    // random selection (Scheduler.random_schedule, kf_workers.py:188-193; kf_run_scheduled_random):
    // filter f draws np.random.choice(len(queue)) from its column of raw 32-bit generator outputs
    // words[n_words][B] (NumPy's legacy masked rejection) and records how many it consumed in
    // words_used[f] (-1: the column ran out).  nullptr: the greedy pick.
    const uint32_t* words;
    int n_words;
    int32_t* words_used;
    // f64 records whose element 9 is the event's time (KF_OPT_SCHED_REC_TIME): the two passes
    // take each pick's time from its gathered record (the pick pass writes no sel_time)
    bool rec_time;
};

enum class Op { Run, Predict, Update, Step, Reset };  // Step: predict + update (kf_capi's deferral)

// Launchers (kf_cv.hip, kf_ref.hip).  Return hipSuccess or the launch error.
hipError_t launch_cv(int axes, bool f64, Op op, const CvArgs& a, hipStream_t stream);
// *flag |= 1 if any filter's P couples different axes (flag: device int, zeroed by the caller).
hipError_t launch_cv_offblock(int axes, bool f64, const CvArgs& a, int* flag, hipStream_t stream);
hipError_t launch_synth(int axes, bool f64, const SynthArgs& a, hipStream_t stream);
// bytes (a multiple of 4) from src to dst on the stream, by a kernel
hipError_t launch_copy(void* dst, const void* src, size_t bytes, hipStream_t stream);
// chain = true: the chain-parallel kernel (kGroup lanes per filter), for few filters.
// kf_run_events kernel variants: one lane per filter (inputs loaded to registers), one lane
// per axis chain (few filters), one lane per filter with inputs staged through LDS by DMA
constexpr int kEventsLane = 0, kEventsChain = 1, kEventsLds = 2, kEventsGated = 3;  // gated: B = 1 look-ahead
hipError_t launch_ref_events(int model, bool f64, const RefArgs& a, hipStream_t stream, int variant);
// the chain kernel in stream mode (a.s_len > 0); nv = 4: the map pass, four state variants per
// filter sharing its covariance (state bank of 4 B columns)
hipError_t launch_ref_stream(int model, bool f64, const RefArgs& a, hipStream_t stream, int nv = 1);
hipError_t launch_ref_reset(int model, bool f64, const RefArgs& a, hipStream_t stream);
hipError_t launch_ref15_combos(bool f64, const Ref15ComboArgs& a, hipStream_t stream);
// child_major: one wave per (parent block, child event) instead of one lane per parent
hipError_t launch_ref15_search(bool f64, const Ref15SearchArgs& a, bool child_major, hipStream_t stream);
// levels a.k and a.k + 1 in one launch (axis-symmetric search): level a.k - 1's stored parents,
// their children computed into LDS and never stored, the children's children stored in a.child;
// child_major: one wave per (parent block, child event) item, else one lane per parent
hipError_t launch_ref15_search_pair(bool f64, const Ref15SearchArgs& a, bool child_major, hipStream_t stream);
// the acceptance band of a search's threshold (Ref15SearchArgs::band_*), for its dtype
void set_search_band(Ref15SearchArgs& a, bool f64);
// levels 1 .. a.k of a search in one launch (one lane per subset of at most a.k free events)
hipError_t launch_ref15_search_head(bool f64, const Ref15SearchArgs& a, hipStream_t stream);
// levels a.k .. a.k_end of a search in one launch, each subset from its stored (a.k - 1)-prefix
hipError_t launch_ref15_search_end(bool f64, const Ref15SearchArgs& a, hipStream_t stream);
// a search's counters[0 .. n) (n <= 256) copied to `host` (the device address of mapped host
// memory), and zeroed with `zero` (the end of the search)
hipError_t launch_search_finish(uint64_t* counters, uint64_t* host, int n, bool zero, hipStream_t stream);
hipError_t launch_ref15_score(bool f64, const Ref15ScoreArgs& a, hipStream_t stream);
hipError_t launch_ref15_scheduled(bool f64, const Ref15SchedArgs& a, hipStream_t stream);
// random_schedule's picks only (a.words): pick [T][B] event indices, a.sel_time, a.n_sel, a.words_used
hipError_t launch_ref15_random_picks(const Ref15SchedArgs& a, int32_t* pick, hipStream_t stream);
// descending stable radix sort of n (key, value) pairs on the key's low `bits` bits (kf_ingest.hip,
// hipCUB); tmp == nullptr: *tmp_bytes = the scratch it needs
hipError_t sort_pairs_desc_u32(void* tmp, size_t* tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                               const uint32_t* vals_in, uint32_t* vals_out, int n, int bits, hipStream_t stream);

constexpr int kBlock = 256;  // 4 wave64 per workgroup

// Record the thread-local message kf_last_error returns; returns `code` (kf_capi.cpp).
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace kfmi
