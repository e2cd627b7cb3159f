// C ABI of libkfmi.so (declared in include/kf.h): handle management, argument checking,
// and dispatch to the gfx950 kernels in kf_cv.hip.  No compute happens here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <climits>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kf.h"
#include "kf_internal.h"

struct kf_batch {
    int model;
    int axes;   // d: state n = 2d, measurement m = d, control c = d
    int n, m, c;
    int np;     // covariance rows: n(n+1)/2, or the block-packed rows of KF_MODEL_REF15 (27) / REF8 (15)
    int dtype;
    int64_t B;
    int device;
    kf_params params;
    void* x;          // [n][B]
    void* P;          // [n(n+1)/2][B]
    int32_t* status;  // [B]
    void* ws;         // KF_MODEL_REF15: device workspace for kf_eval_combos (events, binomials, init)
    // what ws holds (the binomials from kf_alloc on; the events and init of the last upload, whose
    // copy ws_evt marks on ws_stream): a search or evaluation over the same inputs uploads nothing
    std::vector<double> ws_events, ws_init;
    int ws_n;
    bool ws_captured;  // an upload was captured into a graph: its replays rewrite ws, so never skip
    hipEvent_t ws_evt;
    hipStream_t ws_stream;
    void* search_ws;  // KF_MODEL_REF15: kf_search_combos level buffers (grown on demand)
    size_t search_ws_bytes;
    bool r_diag;      // BASELINE models: R has no off-diagonal entry
    bool block_p;     // BASELINE models: every filter's P is block-diagonal over the axes
    int* flag;        // device int for the kf_set_state block check (allocated on first use)
    void* stream_ws;  // kf_run_stream: chunk banks, maps, check (grown on demand)
    size_t stream_ws_bytes;
    int64_t s_chunks, s_len, s_warm;  // the last kf_run_stream's split (s_chunks = 1: sequential)
    // BASELINE models: a kf_predict held back so the next kf_update runs predict + update as one
    // fused step (the state crosses HBM once instead of twice).  The control is copied into
    // pend_u on the predict's stream, so the caller may reuse its u buffer at once.
    bool pend;
    bool pend_has_u;
    double pend_dt;
    void* pend_u;          // [c][B] (allocated by kf_alloc)
    hipEvent_t pend_done;    // recorded right after each kernel that reads pend_u (outside a capture)
    hipStream_t pend_reader; // the stream of the last such kernel (compared, never used in a call)
    bool pend_read;          // a kernel has read pend_u
    bool pend_evt;           // pend_done marks that read (false: it was captured into a graph)
    bool last_predict;       // the handle's last state call was kf_predict
    int64_t opt[KF_OPT_COUNT];  // kf_set_option values (0 = the library's choice)
    // reference models: the caller's noise constants on the device when they differ from the
    // reference's (kf_params.ref_*), else nullptr and the kernels built on the reference's literals
    kfmi::RefConsts* kc;
    double gps_r0, imu_r0;   // R_gps[0], R_imu[0]: which sensor the greedy scheduler picks
    void* sched_ws;          // kf_run_scheduled's two passes: picks [T][B] u32, flags [B] (grown on demand)
    size_t sched_ws_bytes;
    // a graph capture baked the address of this workspace in: its replays write it, so it is
    // never freed before kf_free (a larger one replaces it and it moves to `retired`)
    bool search_ws_graph, stream_ws_graph, sched_ws_graph;
    std::vector<std::pair<void*, size_t>> retired;
    int64_t search_info[4];  // the last kf_search_combos: sym, head sizes, level launches, level bytes
    // kf_search_combos' results: the finish kernel copies the device counters (best[], n_acc[])
    // into this mapped, coherent host buffer and zeroes them, so the next search on the same
    // stream starts without a clear and no result copy is staged through pageable memory
    uint64_t* search_host;
    uint64_t* search_host_dev;
    bool search_ctr_zero;            // the counters are zero for a search queued on search_ctr_stream
    hipStream_t search_ctr_stream;
};

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(KF_EHIP, "%s: %s (%d)", what, hipGetErrorString(e), static_cast<int>(e));
}

size_t elem(const kf_batch* h) { return h->dtype == KF_F64 ? 8 : 4; }
int64_t ntri(const kf_batch* h) { return h->np; }

constexpr int kMaxComboEvents = 64;
// below this many filters kf_run_events runs the chain-parallel kernel (B * 8 lanes): at 16384
// filters one lane each is 256 waves, a quarter of the chip's SIMDs
constexpr int64_t kChainMaxFilters = 16384;
constexpr size_t kWsEvents = sizeof(double) * kMaxComboEvents * 11;
constexpr size_t kWsBinom = sizeof(uint64_t) * (kMaxComboEvents + 1) * (kMaxComboEvents + 1);
constexpr size_t kWsInit = sizeof(double) * 42;
// levels with at most this many parents run child-major (see search_child_major)
constexpr uint64_t kSearchChildMajorParents = 200000;
// the search's head launch covers the sizes whose subsets' event steps from the root add up to at
// most this many (n = 25: sizes 1 .. 5, 323,775 steps for 68,405 subsets)
constexpr uint64_t kSearchHeadSteps = 400000;
// the end launch covers the last sizes whose subsets' event steps from their stored prefixes add
// up to at most this many (n = 25: sizes 20 .. 25 from level 19, 86,712 steps for 68,406 subsets)
constexpr uint64_t kSearchEndSteps = 200000;
// KF_OPT_SEARCH_PAIR = 0: levels with at least this many stored parents pair with the next level
// parent-major (each parent's lane walks its children and their children in sequence, so such a
// launch needs many more lanes than a level launch to fill the chip), narrower ones child-major
// 
constexpr uint64_t kSearchPairParents = uint64_t(1) << 22;

int64_t opt(const kf_batch* h, int o) { return h->opt[o]; }

bool is_ref15(const kf_batch* h) { return h->model == KF_MODEL_REF15; }

// binomial table C(a, b), a, b <= 64 (exact in uint64; C(64, 32) < 2^63)
const uint64_t* binom_table() {
    static uint64_t binom[(kMaxComboEvents + 1) * (kMaxComboEvents + 1)];
    static std::once_flag once;
    std::call_once(once, [] {
        for (int a = 0; a <= kMaxComboEvents; ++a)
            for (int b = 0; b <= kMaxComboEvents; ++b) {
                uint64_t v = 0;
                if (b == 0) v = 1;
                else if (a > 0 && b <= a) v = binom[(a - 1) * (kMaxComboEvents + 1) + b - 1] + binom[(a - 1) * (kMaxComboEvents + 1) + b];
                binom[a * (kMaxComboEvents + 1) + b] = v;
            }
    });
    return binom;
}

bool capturing(hipStream_t st);

// Grow a per-handle device workspace to at least `need` bytes (the grown-on-demand buffers
// search_ws / stream_ws / sched_ws).  Growing allocates, and hipFree synchronises the device, so
// it happens only on the first call of a kind and on a call that needs more than any before it
// (kf.h: "Workspaces").  A buffer that a graph capture used stays alive until kf_free, since the
// graph's replays still write it; inside a capture nothing is allocated (returns false).
bool grow_ws(kf_batch* h, void** buf, size_t* bytes, bool* graph, size_t need, hipStream_t st) {
    if (*bytes >= need) return true;
    if (capturing(st)) return false;
    if (*buf) {
        if (*graph) h->retired.emplace_back(*buf, *bytes);
        else (void)hipFree(*buf);
    }
    *buf = nullptr;
    *bytes = 0;
    *graph = false;
    if (hipMalloc(buf, need) != hipSuccess) {
        (void)hipGetLastError();
        *buf = nullptr;
        return false;
    }
    *bytes = need;
    return true;
}

// Upload the combination search's inputs (events, root state) to the handle's workspace (the
// binomials went there at kf_alloc).  Inputs equal, bit for bit, to the last upload are already
// there: nothing is copied, and a call on another stream waits for that upload's copy.  A call
// inside a graph capture copies (HIP refuses to capture a copy from pageable host memory, so
// such a capture fails today; were it to succeed, its replays would rewrite the workspace
// behind the cache, so from then on every call copies).
int upload_combo_inputs(kf_batch* h, int n_events, const double* events, const double* init, hipStream_t st,
                        const char* what) {
    char* ws = static_cast<char*>(h->ws);
    const size_t ne = size_t(11) * size_t(n_events);
    const bool cap = capturing(st);
    if (cap) h->ws_captured = true;
    if (!h->ws_captured && h->ws_n == n_events && std::memcmp(h->ws_events.data(), events, sizeof(double) * ne) == 0 &&
        std::memcmp(h->ws_init.data(), init, kWsInit) == 0) {
        const hipError_t e = h->ws_stream == st ? hipSuccess : hipStreamWaitEvent(st, h->ws_evt, 0);
        return e == hipSuccess ? KF_OK : hip_fail(e, what);
    }
    h->ws_n = -1;  // until this upload is queued
    hipError_t e = hipMemcpyAsync(ws, events, sizeof(double) * ne, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(ws + kWsEvents + kWsBinom, init, kWsInit, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return hip_fail(e, what);
    if (!cap && hipEventRecord(h->ws_evt, st) == hipSuccess) {
        h->ws_events.assign(events, events + ne);
        h->ws_init.assign(init, init + kWsInit / sizeof(double));
        h->ws_n = n_events;
        h->ws_stream = st;
    }
    return KF_OK;
}

// kf_search_combos kernel per level: child-major (one wave per parent block and child event)
// for the narrow levels, where one lane per parent would walk up to n - 1 children in sequence;
// parent-major (one lane per parent, its children in a wave-uniform loop) for the wide ones,
// where it reads each parent once and keeps it in registers (interleaved A/B:
// profiles/r01_ab/search_kernels_ab.txt).  KF_OPT_SEARCH_KERNEL = 1 | 2 forces one.
bool search_child_major(const kf_batch* h, uint64_t n_par) {
    if (opt(h, KF_OPT_SEARCH_KERNEL) == 1) return true;
    if (opt(h, KF_OPT_SEARCH_KERNEL) == 2) return false;
    return n_par <= kSearchChildMajorParents;
}

int check_combo_inputs(const kf_batch* h, int n_events, const double* events, const double* init, const char* what) {
    if (!is_ref15(h)) return fail(KF_EINVAL, "%s: needs a KF_MODEL_REF15 handle", what);
    if (n_events < 1 || n_events > kMaxComboEvents)
        return fail(KF_EINVAL, "%s: n_events = %d outside [1, %d]", what, n_events, kMaxComboEvents);
    if (!events || !init) return fail(KF_EINVAL, "%s: null events/init", what);
    for (int i = 0; i < n_events; ++i) {
        const double ty = events[i * 11 + 1];
        if (ty != KF_EVENT_GPS && ty != KF_EVENT_IMU)
            return fail(KF_EINVAL, "%s: event %d has type %g (GPS=0 or IMU=1)", what, i, ty);
    }
    return KF_OK;
}
bool is_ref(int model) { return model == KF_MODEL_REF15 || model == KF_MODEL_REF8; }
bool is_ref(const kf_batch* h) { return is_ref(h->model); }

int need_cv(const kf_batch* h, const char* what) {
    if (is_ref(h)) return fail(KF_EINVAL, "%s: not available for the reference models (use kf_run_events)", what);
    return KF_OK;
}

kfmi::CvArgs base_args(const kf_batch* h) {
    kfmi::CvArgs a{};
    a.B = h->B;
    a.T = 1;
    a.update_every = 1;
    a.x = h->x;
    a.P = h->P;
    a.status = h->status;
    a.q_pos = h->params.q_pos;
    a.q_vel = h->params.q_vel;
    int k = 0;
    for (int i = 0; i < h->m; ++i)
        for (int j = i; j < h->m; ++j) a.r[k++] = h->params.r[i * h->m + j];
    a.p0_pos = h->params.p0_pos;
    a.p0_vel = h->params.p0_vel;
    // the block kernel needs a block-diagonal P (kept so by a diagonal R);
    // KF_OPT_CV_KERNEL = 1 forces the general kernel (tests, A/B)
    const int64_t v = opt(h, KF_OPT_CV_KERNEL);
    a.block_p = (h->block_p && h->r_diag && v != 1) ? 1 : 0;
    // the block kernel keeps 7 steps of inputs in flight per lane: with one filter per lane a
    // small batch is one or two waves per SIMD, too few to cover HBM latency with 1-step
    // prefetch, and at 2^20 filters depth 8 still measured ~1.5% ahead of depth 2
    // (profiles/r01_ab/prefetch_depth_ab.txt); KF_OPT_CV_KERNEL = 2 | 4 forces the depth
    a.prefetch_depth = (v == 2 || v == 4) ? int(v) : 8;
    a.blocks_per_cu = int(opt(h, KF_OPT_BLOCKS_PER_CU));
    return a;
}

int launch(const kf_batch* h, kfmi::Op op, const kfmi::CvArgs& a, void* stream, const char* what) {
    if (h->B == 0) return KF_OK;
    hipError_t e = kfmi::launch_cv(h->axes, h->dtype == KF_F64, op, a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, what);
    return KF_OK;
}

int check_handle(const kf_batch* h) {
    if (!h) return fail(KF_EINVAL, "null kf_batch handle");
    return KF_OK;
}

int model_axes(int model) {
    switch (model) {
        case KF_MODEL_CV2: return 2;
        case KF_MODEL_CV3: return 3;
        case KF_MODEL_REF15: return 3;
        case KF_MODEL_REF8: return 2;
        default: return 0;
    }
}

kfmi::RefArgs ref_args(const kf_batch* h) {
    kfmi::RefArgs a{};
    a.B = h->B;
    a.x = h->x;
    a.P = h->P;
    a.status = h->status;
    a.kc = h->kc;
    return a;
}

// The reference's diagonal noise constants per state (kf_workers.py:519-614, P0 :651;
// hw5_2.py:233-304, P0 :317-326), by state group: pos, att, vel, rate, acc.
void ref_default_consts(int model, kf_params* p) {
    static const double q[5] = {5.0, 0.05, 1.0, 0.1, 2.0};
    static const double r[5] = {50.0, 0.05, 10.0, 0.1, 100.0};
    static const int g15[15] = {0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4};
    static const int g8[8] = {0, 0, 1, 2, 2, 3, 4, 4};  // x, y, theta, vx, vy, theta_dot, ax, ay
    const bool m15 = model == KF_MODEL_REF15;
    const int n = m15 ? 15 : 8;
    static const double p15[5] = {10000.0, 1000.0, 1000.0, 1000.0, 10000.0};
    static const double p8[5] = {1000.0, 100.0, 100.0, 100.0, 1000.0};
    for (int i = 0; i < n; ++i) {
        const int g = m15 ? g15[i] : g8[i];
        p->ref_q[i] = q[g];
        p->ref_r_imu[i] = r[g];
        p->ref_p0[i] = m15 ? p15[g] : p8[g];
    }
    for (int i = 0; i < (m15 ? 3 : 2); ++i) p->ref_r_gps[i] = 3.0;
}

// KF_OPT_PREDICT = 1 turns the deferral off (tests, A/B)
bool defer_predicts(const kf_batch* h) { return opt(h, KF_OPT_PREDICT) == 0; }

bool capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// After a kernel on `stream` read pend_u: record pend_done there at once, so a later control
// copy on another stream can wait for the read without this call keeping the stream for later
// (the caller may destroy it).  Inside a graph capture nothing is recorded: a later deferral on
// another stream then runs its predict eagerly instead (kf_predict).
int note_pend_reader(kf_batch* h, void* stream, const char* what) {
    if (!h->pend_has_u) return KF_OK;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    h->pend_reader = st;
    h->pend_read = true;
    h->pend_evt = !capturing(st);
    if (h->pend_evt) {
        hipError_t e = hipEventRecord(h->pend_done, st);
        if (e != hipSuccess) return hip_fail(e, what);
    }
    return KF_OK;
}

// Runs a held-back kf_predict on `stream` (the stream of the call that needs the state: a caller
// that orders that call after its kf_predict has also ordered it after the control copy).
int flush_predict(kf_batch* h, void* stream, const char* what) {
    if (!h->pend) return KF_OK;
    h->pend = false;
    kfmi::CvArgs a = base_args(h);
    a.dt = h->pend_dt;
    a.u = h->pend_has_u ? h->pend_u : nullptr;
    if (int rc = launch(h, kfmi::Op::Predict, a, stream, what)) return rc;
    return note_pend_reader(h, stream, what);
}

// KF_OPT_AXIS_SYM: the handle's noise constants are the same on every axis, bit for bit — REF15:
// pos / vel / acc and att / rate of axes 1 and 2 those of axis 0, and R_gps; REF8: x's and y's
// (pos, vel, acc) chains (its heading chain is the only aw chain) — so work that depends on the
// constants alone is the same for the axes' chains
bool same_bits(double a, double b) { return std::memcmp(&a, &b, sizeof a) == 0; }

bool axis_sym_consts(const kf_batch* h) {
    if (opt(h, KF_OPT_AXIS_SYM) == 1) return false;
    const kf_params& p = h->params;
    auto same_state = [&](int s, int t) {
        return same_bits(p.ref_q[s], p.ref_q[t]) && same_bits(p.ref_r_imu[s], p.ref_r_imu[t]);
    };
    if (h->model == KF_MODEL_REF15) {
        for (int c = 1; c < 3; ++c) {
            for (int s : {0, 6, 12, 3, 9})
                if (!same_state(s + c, s)) return false;
            if (!same_bits(p.ref_r_gps[c], p.ref_r_gps[0])) return false;
        }
        return true;
    }
    if (h->model == KF_MODEL_REF8) {
        for (int s : {0, 3, 6})
            if (!same_state(s + 1, s)) return false;
        return same_bits(p.ref_r_gps[1], p.ref_r_gps[0]);
    }
    return false;
}

// kf_search_combos' axis-symmetric variant (Ref15SearchArgs::sym): axis-symmetric constants and
// the root covariance's blocks init[15 ..] equal on the three axes (bit for bit), so every
// covariance the search reaches has three equal pva blocks and three equal aw blocks
bool search_sym(const kf_batch* h, const double* init) {
    if (!axis_sym_consts(h)) return false;
    const double* blk = init + 15;
    for (int c = 1; c < 3; ++c) {
        for (int i = 0; i < 6; ++i)
            if (!same_bits(blk[6 * c + i], blk[i])) return false;
        for (int i = 0; i < 3; ++i)
            if (!same_bits(blk[18 + 3 * c + i], blk[18 + i])) return false;
    }
    return true;
}

}  // namespace

namespace kfmi {
int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
}  // namespace kfmi

extern "C" {

#ifndef KFMI_SRC_HASH
#define KFMI_SRC_HASH "unknown"
#endif
const char* kf_version(void) { return "kfmi 0.3.0 (gfx950) src:" KFMI_SRC_HASH; }

int kf_set_option(kf_batch* h, int option, int64_t value) {
    if (int rc = check_handle(h)) return rc;
    bool ok = false;
    switch (option) {
        case KF_OPT_PREDICT:
        case KF_OPT_STREAM:
        case KF_OPT_STREAM_FINAL:
        case KF_OPT_SEARCH_PM:
        case KF_OPT_SEARCH_HEAD:
        case KF_OPT_SEARCH_END: ok = value == 0 || value == 1; break;
        case KF_OPT_SEARCH_PAIR: ok = (value >= 0 && value <= 3) || value >= 1024; break;
        case KF_OPT_AXIS_SYM: ok = value == 0 || value == 1; break;
        case KF_OPT_SCHED_KERNEL: ok = value >= 0 && value <= 4; break;
        case KF_OPT_SCHED_GROUP: ok = value == 0 || value == 1 || value == 4; break;
        case KF_OPT_SCHED_ORDER:
        case KF_OPT_SCHED_REC_TIME: ok = value == 0 || value == 1; break;
        case KF_OPT_CV_KERNEL: ok = value == 0 || value == 1 || value == 2 || value == 4 || value == 8; break;
        case KF_OPT_BLOCKS_PER_CU: ok = value == 0 || (value >= 2 && value <= 8); break;
        case KF_OPT_EVENTS_KERNEL: ok = value >= 0 && value <= 4; break;
        case KF_OPT_STREAM_CHUNKS: ok = value == 0 || (value >= 2 && value <= (int64_t(1) << 24)); break;
        case KF_OPT_START_THREADS: ok = value == 0 || (value >= 1 && value <= kfmi::kBlock); break;
        case KF_OPT_SEARCH_KERNEL: ok = value >= 0 && value <= 2; break;
        default: return fail(KF_EINVAL, "kf_set_option: unknown option %d", option);
    }
    if (!ok) return fail(KF_EINVAL, "kf_set_option: value %lld out of range for option %d", (long long)value, option);
    // (a predict already held back stays so: the next call that needs the state runs it, as
    // before; the option governs the predicts that follow)
    h->opt[option] = value;
    return KF_OK;
}

int kf_get_option(const kf_batch* h, int option, int64_t* value) {
    if (int rc = check_handle(h)) return rc;
    if (option < 1 || option >= KF_OPT_COUNT) return fail(KF_EINVAL, "kf_get_option: unknown option %d", option);
    if (!value) return fail(KF_EINVAL, "kf_get_option: null output");
    *value = h->opt[option];
    return KF_OK;
}

const char* kf_last_error(void) { return g_err.c_str(); }

int kf_default_params(int model, kf_params* out) {
    const int d = model_axes(model);
    if (!d) return fail(KF_EINVAL, "unknown model %d", model);
    if (!out) return fail(KF_EINVAL, "null params");
    std::memset(out, 0, sizeof *out);
    if (is_ref(model)) {
        ref_default_consts(model, out);
        return KF_OK;
    }
    out->q_pos = 5.0;  // position_noise = 5 * dt   (kf_workers.py:521)
    out->q_vel = 1.0;  // velocity_noise = 1 * dt   (kf_workers.py:523)
    for (int i = 0; i < d; ++i) out->r[i * d + i] = 3.0;  // gps variance 3 (kf_workers.py:583)
    if (d == 3) {
        out->p0_pos = 10000.0;  // kf_workers.py:651
        out->p0_vel = 1000.0;
    } else {
        out->p0_pos = 1000.0;   // hw5_2.py:318-319
        out->p0_vel = 100.0;    // hw5_2.py:321-322
    }
    return KF_OK;
}

int kf_device_count(int* count) {
    if (!count) return fail(KF_EINVAL, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = (e == hipSuccess) ? n : 0;
    return KF_OK;
}

int kf_init(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(KF_ENODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(KF_ENODEV, "device %d out of range [0,%d)", device, n);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(KF_ENODEV, "device %d is %s; libkfmi is built for gfx950 only", device, prop.gcnArchName);
    return KF_OK;
}

int kf_alloc(kf_batch** handle, int model, int64_t batch, int dtype, const kf_params* params) {
    if (!handle) return fail(KF_EINVAL, "null handle out-pointer");
    *handle = nullptr;
    const int d = model_axes(model);
    if (!d) return fail(KF_EINVAL, "unknown model %d", model);
    if (dtype != KF_F32 && dtype != KF_F64) return fail(KF_EINVAL, "unknown dtype %d", dtype);
    if (batch < 0) return fail(KF_EINVAL, "negative batch %lld", static_cast<long long>(batch));
    if (batch * 8 >= (int64_t(1) << 31))
        return fail(KF_EINVAL, "batch %lld too large (one [B] row must stay below 2 GiB)", static_cast<long long>(batch));
    const int nref = model == KF_MODEL_REF15 ? 15 : 8, ngps = model == KF_MODEL_REF15 ? 3 : 2;
    bool custom = false;
    if (is_ref(model) && params) {
        kf_params ref{};
        ref_default_consts(model, &ref);
        for (int i = 0; i < nref; ++i) {
            if (!(params->ref_q[i] >= 0.0) || !std::isfinite(params->ref_q[i]))
                return fail(KF_EINVAL, "kf_alloc: ref_q[%d] = %g (need a finite rate >= 0)", i, params->ref_q[i]);
            if (!(params->ref_r_imu[i] > 0.0) || !std::isfinite(params->ref_r_imu[i]))
                return fail(KF_EINVAL, "kf_alloc: ref_r_imu[%d] = %g (need a finite variance > 0)", i, params->ref_r_imu[i]);
            if (!(params->ref_p0[i] > 0.0) || !std::isfinite(params->ref_p0[i]))
                return fail(KF_EINVAL, "kf_alloc: ref_p0[%d] = %g (need a finite variance > 0)", i, params->ref_p0[i]);
            custom = custom || params->ref_q[i] != ref.ref_q[i] || params->ref_r_imu[i] != ref.ref_r_imu[i] ||
                     params->ref_p0[i] != ref.ref_p0[i];
        }
        for (int i = 0; i < ngps; ++i) {
            if (!(params->ref_r_gps[i] > 0.0) || !std::isfinite(params->ref_r_gps[i]))
                return fail(KF_EINVAL, "kf_alloc: ref_r_gps[%d] = %g (need a finite variance > 0)", i, params->ref_r_gps[i]);
            custom = custom || params->ref_r_gps[i] != ref.ref_r_gps[i];
        }
    }
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail(KF_ENODEV, "no current HIP device: %s", hipGetErrorString(e));
    kf_batch* h = new kf_batch{};
    h->model = model;
    h->axes = d;
    h->n = model == KF_MODEL_REF15 ? 15 : model == KF_MODEL_REF8 ? 8 : 2 * d;
    h->m = d;
    h->c = is_ref(model) ? 0 : d;
    h->np = model == KF_MODEL_REF15 ? 27 : model == KF_MODEL_REF8 ? 15 : h->n * (h->n + 1) / 2;
    h->dtype = dtype;
    h->B = batch;
    h->device = dev;
    if (params) h->params = *params;
    else kf_default_params(model, &h->params);
    h->gps_r0 = h->params.ref_r_gps[0];
    h->imu_r0 = h->params.ref_r_imu[0];
    h->r_diag = true;
    for (int i = 0; i < h->m; ++i)
        for (int j = 0; j < h->m; ++j)
            if (i != j && h->params.r[i * h->m + j] != 0.0) h->r_diag = false;
    const size_t w = elem(h);
    const size_t nb = static_cast<size_t>(batch);
    if (nb) {
        if (hipMalloc(&h->x, w * h->n * nb) != hipSuccess ||
            hipMalloc(&h->P, w * ntri(h) * nb) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&h->status), sizeof(int32_t) * nb) != hipSuccess) {
            (void)hipGetLastError();
            kf_free(h);
            return fail(KF_ENOMEM, "hipMalloc of %zu filters failed", nb);
        }
    }
    // the held-back predict's control copy (kf_predict), allocated here so that a per-step loop
    // never allocates (and can be captured into a graph)
    if (!is_ref(model) && nb &&
        (hipMalloc(&h->pend_u, w * h->c * nb) != hipSuccess ||
         hipEventCreateWithFlags(&h->pend_done, hipEventDisableTiming) != hipSuccess)) {
        (void)hipGetLastError();
        kf_free(h);
        return fail(KF_ENOMEM, "hipMalloc of the control copy of %zu filters failed", nb);
    }
    h->ws_n = -1;
    if (model == KF_MODEL_REF15 &&
        (hipMalloc(&h->ws, kWsEvents + kWsBinom + kWsInit) != hipSuccess ||
         hipMemcpy(static_cast<char*>(h->ws) + kWsEvents, binom_table(), kWsBinom, hipMemcpyHostToDevice) != hipSuccess ||
         hipEventCreateWithFlags(&h->ws_evt, hipEventDisableTiming) != hipSuccess)) {
        (void)hipGetLastError();
        kf_free(h);
        return fail(KF_ENOMEM, "hipMalloc of the combination workspace failed");
    }
    if (custom) {  // the caller's constants, read by the kernels compiled for them
        kfmi::RefConsts k{};
        for (int i = 0; i < nref; ++i) {
            k.q[i] = params->ref_q[i];
            k.r_imu[i] = params->ref_r_imu[i];
            k.p0[i] = params->ref_p0[i];
        }
        for (int i = 0; i < ngps; ++i) k.r_gps[i] = params->ref_r_gps[i];
        if (hipMalloc(reinterpret_cast<void**>(&h->kc), sizeof k) != hipSuccess ||
            hipMemcpy(h->kc, &k, sizeof k, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipGetLastError();
            kf_free(h);
            return fail(KF_ENOMEM, "kf_alloc: device copy of the noise constants failed");
        }
    }
    int rc = kf_reset(h, nullptr, nullptr);
    if (rc == KF_OK && nb) {
        e = hipStreamSynchronize(nullptr);
        if (e != hipSuccess) rc = hip_fail(e, "kf_alloc reset");
    }
    if (rc != KF_OK) {
        kf_free(h);
        return rc;
    }
    *handle = h;
    return KF_OK;
}

int kf_free(kf_batch* h) {
    if (!h) return KF_OK;
    if (h->x) (void)hipFree(h->x);
    if (h->P) (void)hipFree(h->P);
    if (h->status) (void)hipFree(h->status);
    if (h->ws) (void)hipFree(h->ws);
    if (h->ws_evt) (void)hipEventDestroy(h->ws_evt);
    if (h->search_ws) (void)hipFree(h->search_ws);
    if (h->search_host) (void)hipHostFree(h->search_host);
    if (h->flag) (void)hipFree(h->flag);
    if (h->stream_ws) (void)hipFree(h->stream_ws);
    if (h->pend_u) (void)hipFree(h->pend_u);
    if (h->pend_done) (void)hipEventDestroy(h->pend_done);
    if (h->kc) (void)hipFree(h->kc);
    if (h->sched_ws) (void)hipFree(h->sched_ws);
    for (auto& r : h->retired) (void)hipFree(r.first);
    delete h;
    return KF_OK;
}

int kf_release_retired(kf_batch* h, int64_t* bytes_freed) {
    if (int rc = check_handle(h)) return rc;
    int64_t freed = 0;
    for (auto& r : h->retired) {
        (void)hipFree(r.first);
        freed += static_cast<int64_t>(r.second);
    }
    h->retired.clear();
    if (bytes_freed) *bytes_freed = freed;
    return KF_OK;
}

int kf_dims(const kf_batch* h, int* n, int* m, int* c, int64_t* batch, int* dtype) {
    if (int rc = check_handle(h)) return rc;
    if (n) *n = h->n;
    if (m) *m = h->m;
    if (c) *c = h->c;
    if (batch) *batch = h->B;
    if (dtype) *dtype = h->dtype;
    return KF_OK;
}

int kf_reset(kf_batch* h, const void* x0, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (is_ref(h)) {
        if (h->B == 0) return KF_OK;
        kfmi::RefArgs a = ref_args(h);
        a.x0 = x0;
        hipError_t e = kfmi::launch_ref_reset(h->model, h->dtype == KF_F64, a, static_cast<hipStream_t>(stream));
        return e == hipSuccess ? KF_OK : hip_fail(e, "kf_reset");
    }
    h->pend = false;  // a predict followed by a reset leaves the reset state
    h->last_predict = false;
    // (pend_read stays: a kernel that read pend_u may still be running on another stream, and
    // pend_done, recorded right after it, is what the next control copy waits for)
    kfmi::CvArgs a = base_args(h);
    a.x0 = x0;
    h->block_p = true;  // P = P0 is diagonal
    return launch(h, kfmi::Op::Reset, a, stream, "kf_reset");
}

int kf_set_state(kf_batch* h, const void* x, const void* P, int on_device, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (!x && !P) return fail(KF_EINVAL, "kf_set_state: x and P both null");
    if (x && P) h->pend = false;  // both overwritten: a held-back predict has no effect
    else if (int rc = flush_predict(h, stream, "kf_set_state")) return rc;
    h->last_predict = false;
    const hipMemcpyKind kind = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const size_t w = elem(h), nb = static_cast<size_t>(h->B);
    hipError_t e = hipSuccess;
    if (x && nb) e = hipMemcpyAsync(h->x, x, w * h->n * nb, kind, static_cast<hipStream_t>(stream));
    if (e == hipSuccess && P && nb)
        e = hipMemcpyAsync(h->P, P, w * ntri(h) * nb, kind, static_cast<hipStream_t>(stream));
    if (e == hipSuccess && nb)
        e = hipMemsetAsync(h->status, 0, sizeof(int32_t) * nb, static_cast<hipStream_t>(stream));
    if (e == hipSuccess && !on_device) e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "kf_set_state");
    if (P && nb && !is_ref(h)) {
        // does the new P keep every filter block-diagonal over the axes (cv_block_kernel)?
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (!h->flag && hipMalloc(reinterpret_cast<void**>(&h->flag), sizeof(int)) != hipSuccess) {
            (void)hipGetLastError();
            h->flag = nullptr;
            h->block_p = false;
            return KF_OK;
        }
        int any = 1;
        e = hipMemsetAsync(h->flag, 0, sizeof(int), st);
        if (e == hipSuccess) e = kfmi::launch_cv_offblock(h->axes, h->dtype == KF_F64, base_args(h), h->flag, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&any, h->flag, sizeof(int), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(e, "kf_set_state block check");
        h->block_p = any == 0;
    }
    return KF_OK;
}

int kf_get_state(kf_batch* h, void* x, void* P, int on_device, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (int rc = flush_predict(h, stream, "kf_get_state")) return rc;
    const hipMemcpyKind kind = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    const size_t w = elem(h), nb = static_cast<size_t>(h->B);
    hipError_t e = hipSuccess;
    if (x && nb) e = hipMemcpyAsync(x, h->x, w * h->n * nb, kind, static_cast<hipStream_t>(stream));
    if (e == hipSuccess && P && nb)
        e = hipMemcpyAsync(P, h->P, w * ntri(h) * nb, kind, static_cast<hipStream_t>(stream));
    if (e == hipSuccess && !on_device) e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "kf_get_state");
    return KF_OK;
}

int kf_get_status(kf_batch* h, int32_t* status, int on_device, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (!status) return fail(KF_EINVAL, "kf_get_status: null output");
    if (int rc = flush_predict(h, stream, "kf_get_status")) return rc;
    const size_t nb = static_cast<size_t>(h->B);
    if (!nb) return KF_OK;
    hipError_t e = hipMemcpyAsync(status, h->status, sizeof(int32_t) * nb,
                                  on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                  static_cast<hipStream_t>(stream));
    if (e == hipSuccess && !on_device) e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "kf_get_status");
    return KF_OK;
}

int kf_predict(kf_batch* h, double dt, const double* dt_per_filter, const void* u, void* logdet_out,
               void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (int rc = need_cv(h, "kf_predict")) return rc;
    if (!dt_per_filter && !(dt >= 0.0)) return fail(KF_EINVAL, "kf_predict: dt must be >= 0 (got %g)", dt);
    if (int rc = flush_predict(h, stream, "kf_predict")) return rc;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    // a predict right after a predict runs at once: in a predict-only stretch (the async
    // config's 100 Hz predicts between 10 Hz fixes) a held-back predict would only add its
    // control copy, since the next call is another predict
    const bool after_predict = h->last_predict;
    h->last_predict = true;
    // the control copy overwrites pend_u (kf_alloc), so it must follow the last kernel that read
    // it: on the same stream that is stream order; on another stream a wait for pend_done, which
    // a capture cannot take when that read was recorded outside it (or captured itself) — then
    // this predict runs eagerly and pend_u is not written
    const bool cross = u && h->pend_read && h->pend_reader != st;
    const bool can_defer = !cross || (h->pend_evt && !capturing(st));
    if (h->B && !dt_per_filter && !logdet_out && !after_predict && defer_predicts(h) && can_defer) {
        // hold it back for a fused step with the next kf_update (the reference's loop calls
        // predict then update every step, kf_workers.py:688-711)
        if (u) {
            hipError_t e = hipSuccess;
            if (cross) e = hipStreamWaitEvent(st, h->pend_done, 0);
            if (e == hipSuccess) e = kfmi::launch_copy(h->pend_u, u, elem(h) * h->c * static_cast<size_t>(h->B), st);
            if (e != hipSuccess) return hip_fail(e, "kf_predict control copy");
        }
        h->pend = true;
        h->pend_has_u = u != nullptr;
        h->pend_dt = dt;
        return KF_OK;
    }
    kfmi::CvArgs a = base_args(h);
    a.dt = dt;
    a.dt_filter = dt_per_filter;
    a.u = u;
    a.logdet = logdet_out;
    return launch(h, kfmi::Op::Predict, a, stream, "kf_predict");
}

int kf_update(kf_batch* h, const void* z, const uint8_t* mask, void* logdet_out, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (int rc = need_cv(h, "kf_update")) return rc;
    if (!z && h->B) return fail(KF_EINVAL, "kf_update: null measurement stream z");
    h->last_predict = false;
    kfmi::CvArgs a = base_args(h);
    a.z = z;
    a.mask = mask;
    a.logdet = logdet_out;
    if (h->pend) {
        // the held-back predict and this update as one kernel (cv_step_kernel)
        h->pend = false;
        a.dt = h->pend_dt;
        a.u = h->pend_has_u ? h->pend_u : nullptr;
        if (int rc = launch(h, kfmi::Op::Step, a, stream, "kf_update (fused with the predict)")) return rc;
        return note_pend_reader(h, stream, "kf_update");
    }
    return launch(h, kfmi::Op::Update, a, stream, "kf_update");
}

int kf_run(kf_batch* h, int T, double dt, const double* dt_steps, const void* u, const void* z,
           const uint8_t* mask, int update_every, void* traj, void* logdet, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (int rc = need_cv(h, "kf_run")) return rc;
    if (T < 0) return fail(KF_EINVAL, "kf_run: T = %d < 0", T);
    if (update_every < 1) return fail(KF_EINVAL, "kf_run: update_every = %d < 1", update_every);
    if (!dt_steps && !(dt >= 0.0)) return fail(KF_EINVAL, "kf_run: dt must be >= 0 (got %g)", dt);
    const int U = T / update_every;
    if (U > 0 && !z && h->B) return fail(KF_EINVAL, "kf_run: %d updates need a z stream", U);
    if (int rc = flush_predict(h, stream, "kf_run")) return rc;
    h->last_predict = false;
    if (T == 0) return KF_OK;
    kfmi::CvArgs a = base_args(h);
    a.T = T;
    a.update_every = update_every;
    a.dt = dt;
    a.dt_steps = dt_steps;
    a.u = u;
    a.z = z;
    a.mask = mask;
    a.traj = traj;
    a.logdet = logdet;
    return launch(h, kfmi::Op::Run, a, stream, "kf_run");
}

int kf_synth(kf_batch* h, uint64_t seed, int64_t filter_offset, int T, double dt, int update_every,
             void* x0_out, void* u_out, void* z_out, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (int rc = need_cv(h, "kf_synth")) return rc;
    if (T < 0 || update_every < 1 || filter_offset < 0)
        return fail(KF_EINVAL, "kf_synth: bad T/update_every/filter_offset");
    if (h->B && (!x0_out || (T > 0 && !u_out) || (T / update_every > 0 && !z_out)))
        return fail(KF_EINVAL, "kf_synth: null output stream");
    if (h->B == 0) return KF_OK;
    kfmi::SynthArgs a{};
    a.B = h->B;
    a.filter_offset = filter_offset;
    a.seed = seed;
    a.T = T;
    a.update_every = update_every;
    a.dt = dt;
    a.x0 = x0_out;
    a.u = u_out;
    a.z = z_out;
    hipError_t e = kfmi::launch_synth(h->axes, h->dtype == KF_F64, a, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "kf_synth");
    return KF_OK;
}

namespace {

// kf_run_events' kernel choice and launch (skip: device flag, see RefArgs::skip; variant >= 0:
// that kernel, for the stream fallback's device-side choice)
int run_events_launch(kf_batch* h, int T, const uint8_t* etype, const double* dt, const void* payload, void* traj,
                      void* cov, void* logdet, uint8_t* updated, int gate, double threshold, const int32_t* skip,
                      void* stream, int forced = -1) {
    kfmi::RefArgs a = ref_args(h);
    a.T = T;
    a.etype = etype;
    a.dt = dt;
    a.payload = payload;
    a.traj = traj;
    a.cov = cov;
    a.logdet = logdet;
    a.updated = updated;
    a.gate = gate;
    a.threshold = threshold;
    a.skip = skip;
    // Few filters cannot fill the chip one lane each: give every axis chain its own lane
    // (8 lanes per filter).  Otherwise one lane per filter, with the inputs staged through LDS
    // by DMA where its layout conditions hold.  KF_OPT_EVENTS_KERNEL = 1 | 2 | 3 (lane, chain,
    // lds) forces a variant (tests, A/B) where it is legal; 4 picks the look-ahead kernel for one
    // gated f64 filter (in f32 its closed-form predicts round differently enough to move gate
    // decisions: 8 of 70,000 flags at r_value = -10, profiles/r06_lookahead)
    const uint64_t span = static_cast<uint64_t>(h->B) * elem(h);
    // the chain kernel addresses up to 27 [B] rows through one descriptor (32-bit byte count);
    // the LDS kernel moves 16-B chunks (B % 16 == 0: none straddles B) of a 9-row payload span
    const bool chain_ok = span * 27u < (uint64_t(1) << 32);
    const bool lds_ok = h->B % 16 == 0 && span * 9u < (uint64_t(1) << 32);
    int variant = h->B < kChainMaxFilters && chain_ok ? kfmi::kEventsChain
                  : lds_ok                            ? kfmi::kEventsLds
                                                      : kfmi::kEventsLane;
    const int64_t v = opt(h, KF_OPT_EVENTS_KERNEL);
    if (v == 2 && chain_ok) variant = kfmi::kEventsChain;
    else if (v == 1) variant = kfmi::kEventsLane;
    else if (v == 3 && lds_ok) variant = kfmi::kEventsLds;
    else if (v == 4 && h->B == 1 && gate && h->dtype == KF_F64) variant = kfmi::kEventsGated;
    if (forced >= 0) variant = forced;
    if (skip && variant != kfmi::kEventsChain && variant != kfmi::kEventsGated)
        return fail(KF_EINVAL, "kf_run_stream: fallback needs the chain kernel");
    hipError_t e = kfmi::launch_ref_events(h->model, h->dtype == KF_F64, a, static_cast<hipStream_t>(stream), variant);
    return e == hipSuccess ? KF_OK : hip_fail(e, "kf_run_events");
}

// kf_run_events routes one-filter runs of at least this many events through kf_run_stream
constexpr int kStreamMinEvents = 65536;
// a gated run (the adaptive threshold) takes its chunk starts from this many events of warm-up:
// the gate makes the covariance recursion's map depend on the covariance, so the
// linear-fractional maps cannot carry it; the seam check decides whether the warm-up converged
constexpr int kStreamGateWarmup = 2048;
// the gated fallback takes the look-ahead kernel when at most 1 in this many events updated in
// the chunked pass (70,000 events: 1.4x the chain kernel at 11 %, 0.74x at 22 %;
// profiles/r06_lookahead/ab_f64.log)
constexpr int kStreamLookaheadShare = 8;
// default (warmup < 0): covariance maps iterated to cover this many events, then kStreamPolish
// chunks of event warm-up
constexpr int64_t kStreamLftEvents = 2048;
constexpr int kStreamPolish = 0;
// events per covariance map: the roundoff of a map's evaluation grows with the events it spans
// (config 1 log: seam gap 4.8e-15 with 285-event maps, 1.5e-11 with 777-event maps)
constexpr int64_t kStreamLftPiece = 160;
// default split: T / kStreamTargetChunks events per chunk, at least kStreamMinChunk.  The map
// pass runs a chunk's four variants in one 8-lane group: 8192 chunks are 1024 waves, one per
// SIMD, and the pass's time is its chunk length in sequence (KF_OPT_STREAM_CHUNKS overrides the
// target, for sweeps: KF_OPT_STREAM_CHUNKS)
constexpr int64_t kStreamTargetChunks = 8192;
constexpr int64_t kStreamMinChunk = 32;
// piece maps (36 doubles) the start kernel stages in LDS per block: 64 KB
constexpr int64_t kStreamStartLdsMaps = 65536 / (36 * 8);
// chunks per start thread, at most: 2 of the 3 that fit measured 0.1937 vs 0.1951 ms per log
// (config 1 in-process, profiles/r04_pmc/cfg1_diag/ab_start_g_chunks.log; 1: 0.1948)
#ifndef KF_START_MAX_G
#define KF_START_MAX_G 2
#endif

size_t align256(size_t n) { return (n + 255) & ~size_t(255); }

}  // namespace

namespace {
// kf_run_events / kf_run_events_seq arguments; 1 = valid and there is work, 0 = nothing to do
int check_events_args(const kf_batch* h, int T, const uint8_t* etype, const double* dt, const void* payload,
                      const char* what, int* rc) {
    *rc = check_handle(h);
    if (*rc) return 0;
    if (!is_ref(h)) *rc = fail(KF_EINVAL, "%s: needs a KF_MODEL_REF15 or KF_MODEL_REF8 handle", what);
    else if (T < 0) *rc = fail(KF_EINVAL, "%s: T = %d < 0", what, T);
    else if (T == 0 || h->B == 0) return 0;
    else if (!etype || !dt || !payload) *rc = fail(KF_EINVAL, "%s: null etype/dt/payload stream", what);
    return *rc == KF_OK;
}
}  // namespace

namespace {
int run_stream_impl(kf_batch* h, int T, const uint8_t* etype, const double* dt, const void* payload, void* traj,
                    void* cov, void* logdet, uint8_t* updated, int chunk, int warmup, int gate, double threshold,
                    void* stream);
}  // namespace

int kf_run_events(kf_batch* h, int T, const uint8_t* etype, const double* dt, const void* payload,
                  void* traj, void* cov, void* logdet, uint8_t* updated, int gate, double threshold,
                  void* stream) {
    int rc = KF_OK;
    if (!check_events_args(h, T, etype, dt, payload, "kf_run_events", &rc)) return rc;
    // one filter over a long stream: parallel over time (checked, with a sequential fallback);
    // gated (the adaptive threshold) from an event warm-up; KF_OPT_STREAM = 1 turns the route
    // off for the handle, kf_run_events_seq for one call
    if (h->B == 1 && T >= kStreamMinEvents && opt(h, KF_OPT_STREAM) == 0)
        return run_stream_impl(h, T, etype, dt, payload, traj, cov, logdet, updated, 0, gate ? kStreamGateWarmup : -1,
                               gate, threshold, stream);
    return run_events_launch(h, T, etype, dt, payload, traj, cov, logdet, updated, gate, threshold, nullptr, stream);
}

int kf_run_events_seq(kf_batch* h, int T, const uint8_t* etype, const double* dt, const void* payload,
                      void* traj, void* cov, void* logdet, uint8_t* updated, int gate, double threshold,
                      void* stream) {
    int rc = KF_OK;
    if (!check_events_args(h, T, etype, dt, payload, "kf_run_events_seq", &rc)) return rc;
    return run_events_launch(h, T, etype, dt, payload, traj, cov, logdet, updated, gate, threshold, nullptr, stream);
}

int kf_run_stream(kf_batch* h, int T, const uint8_t* etype, const double* dt, const void* payload, void* traj,
                  void* cov, void* logdet, uint8_t* updated, int chunk, int warmup, void* stream) {
    return run_stream_impl(h, T, etype, dt, payload, traj, cov, logdet, updated, chunk, warmup, 0, 0.0, stream);
}

namespace {
// kf_run_stream, and with gate != 0 kf_run_events' gated one-filter route: every chain pass and
// the fallback apply the gate, and the chunk starts come from an event warm-up (warmup < 0
// becomes kStreamGateWarmup)
int run_stream_impl(kf_batch* h, int T, const uint8_t* etype, const double* dt, const void* payload, void* traj,
                    void* cov, void* logdet, uint8_t* updated, int chunk, int warmup, int gate, double threshold,
                    void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (gate && warmup < 0) warmup = kStreamGateWarmup;
    if (!is_ref(h)) return fail(KF_EINVAL, "kf_run_stream: needs a KF_MODEL_REF15 or KF_MODEL_REF8 handle");
    if (h->B != 1) return fail(KF_EINVAL, "kf_run_stream: needs a handle of one filter (B = %lld)", (long long)h->B);
    if (T < 0) return fail(KF_EINVAL, "kf_run_stream: T = %d < 0", T);
    if (T == 0) return KF_OK;
    if (!etype || !dt || !payload) return fail(KF_EINVAL, "kf_run_stream: null etype/dt/payload stream");
    const hipStream_t st = static_cast<hipStream_t>(stream);
    int64_t target = kStreamTargetChunks;
    if (opt(h, KF_OPT_STREAM_CHUNKS) > 0) target = std::max<int64_t>(2, opt(h, KF_OPT_STREAM_CHUNKS));
    const int64_t L = chunk > 0 ? chunk : std::max<int64_t>(kStreamMinChunk, (int64_t(T) + target - 1) / target);
    const int64_t C = (int64_t(T) + L - 1) / L;
    // warmup >= 0: W events of warm-up before each chunk from the handle's covariance;
    // -1: linear-fractional covariance maps + kStreamPolish chunks of warm-up; -2 - k: maps + k chunks
    const bool lft = warmup < 0;
    const int kp = !lft ? 0 : warmup == -1 ? kStreamPolish : -(warmup + 2);
    const int64_t W = lft ? int64_t(kp) * L : warmup;
    const size_t w = elem(h);
    const int nblk = h->np, n = h->n;
    const int nch = h->model == KF_MODEL_REF15 ? 6 : 3;
    // stream offsets are 32-bit products (events before the start wrap past every length, and
    // bit 31 marks dropped records): (T + W) rows of the widest record below 2^31 bytes
    const bool fits = uint64_t(T + std::max<int64_t>(W, 0)) * uint64_t(std::max(nblk, 9)) * 8u < (uint64_t(1) << 31);
    h->s_len = L;
    h->s_warm = W;
    if (C < 2 || !fits || L > INT32_MAX || W > INT32_MAX) {
        h->s_chunks = 1;
        return run_events_launch(h, T, etype, dt, payload, traj, cov, logdet, updated, gate, threshold, nullptr,
                                 stream);
    }
    h->s_chunks = C;
    // workspace: check | banks W (C), M (4C), F (C) | maps | starts
    const size_t bank1 = align256(size_t(n + nblk) * C * w) + align256(sizeof(int32_t) * C);
    const size_t bank4 = align256(size_t(n + nblk) * 4 * C * w) + align256(sizeof(int32_t) * 4 * C);
    const int np = int((L + kStreamLftPiece - 1) / kStreamLftPiece);
    const size_t lft_bytes = lft ? align256(sizeof(double) * 36 * nch * C * np) : 0;
    // records straight from the map pass (no final pass) unless the four variants' trajectory
    // rows exceed the 32-bit offsets or KF_OPT_STREAM_FINAL = 1 asks for the final pass
    const int ntraj = h->model == KF_MODEL_REF15 ? 6 : 3;
    const int64_t vstride = T + L;
    const bool map_records = opt(h, KF_OPT_STREAM_FINAL) == 0 && uint64_t(4 * vstride) * ntraj * w < (uint64_t(1) << 31);
    const size_t rec_bytes = map_records ? align256(size_t(4 * vstride) * ntraj * w) + align256(sizeof(double) * n) +
                                               align256(sizeof(double) * 4 * nch * C)
                                         : 0;
    const int64_t ntiles = (C + kfmi::kStreamScanTile - 1) / kfmi::kStreamScanTile;
    // more tiles than one scan round: the top kernel writes the tile starts (kf_ref.hip phase 3)
    const bool top = ntiles > kfmi::kStreamScanTile;
    const size_t top_bytes = top ? align256(sizeof(double) * 3 * nch * ntiles) : 0;
    const size_t need = 256 + 2 * bank1 + bank4 + 2 * align256(sizeof(double) * 12 * nch * C) +
                        align256(sizeof(double) * 12 * nch * ntiles) + align256(sizeof(double) * n * C) + lft_bytes +
                        rec_bytes + top_bytes;
    if (!grow_ws(h, &h->stream_ws, &h->stream_ws_bytes, &h->stream_ws_graph, need, static_cast<hipStream_t>(stream)))
        return capturing(static_cast<hipStream_t>(stream))
                   ? fail(KF_EINVAL, "kf_run_stream: the chunk banks (%zu bytes) must be sized by an eager call "
                                     "before a graph capture", need)
                   : fail(KF_EHIP, "kf_run_stream: cannot allocate %zu bytes of chunk banks", need);
    if (capturing(static_cast<hipStream_t>(stream))) h->stream_ws_graph = true;
    char* p = static_cast<char*>(h->stream_ws);
    kfmi::StreamArgs sa{};
    sa.C = C;
    sa.delta = 1024.0;  // the maps are affine: a large step only shrinks the roundoff of the differences
    sa.rdelta = 1.0 / sa.delta;  // exact: delta is a power of two
    sa.tol_state = h->dtype == KF_F64 ? 1e-9 : 1e-4;
    sa.tol_cov = h->dtype == KF_F64 ? 1e-12 : 1e-5;
    sa.start_threads = int(opt(h, KF_OPT_START_THREADS));
    sa.kc = h->kc;
    sa.sym = axis_sym_consts(h);
    sa.hx = h->x;
    sa.hP = h->P;
    sa.hstatus = h->status;
    sa.check = reinterpret_cast<kfmi::StreamCheck*>(p);
    p += 256;
    auto bank = [&](int64_t B, void*& x, void*& P, int32_t*& status) {
        x = p;
        P = p + size_t(n) * B * w;
        p += align256(size_t(n + nblk) * B * w);
        status = reinterpret_cast<int32_t*>(p);
        p += align256(sizeof(int32_t) * B);
    };
    bank(C, sa.wx, sa.wP, sa.wst);
    bank(4 * C, sa.mx, sa.mP, sa.mst);
    bank(C, sa.fx, sa.fP, sa.fst);
    sa.maps = reinterpret_cast<double*>(p);
    p += align256(sizeof(double) * 12 * nch * C);
    sa.pref = reinterpret_cast<double*>(p);
    p += align256(sizeof(double) * 12 * nch * C);
    sa.tiles = reinterpret_cast<double*>(p);
    p += align256(sizeof(double) * 12 * nch * ntiles);
    sa.starts = reinterpret_cast<double*>(p);
    p += align256(sizeof(double) * n * C);
    if (top) {
        sa.tstart = reinterpret_cast<double*>(p);
        p += top_bytes;
    }
    if (lft) {
        sa.phi = reinterpret_cast<double*>(p);
        p += align256(sizeof(double) * 36 * nch * C * np);
    }
    void* traj4 = nullptr;
    if (map_records) {
        traj4 = p;
        p += align256(size_t(4 * vstride) * ntraj * w);
        sa.xend = reinterpret_cast<double*>(p);
        p += align256(sizeof(double) * n);
        sa.dtab = reinterpret_cast<double*>(p);  // the records' start offsets, [C][chains][4]
        sa.traj4 = traj4;
        sa.vstride = vstride;
        sa.traj = traj;
    }
    sa.etype = etype;
    sa.dt = dt;
    sa.S = T;
    sa.L = L;
    sa.kp = kp;
    sa.np = np;
    sa.lp = (L + np - 1) / np;

    const bool f64 = h->dtype == KF_F64;
    // nv = 4: the map pass, B = C filters of four state variants each (banks of 4C columns)
    auto chain = [&](int64_t B, void* x, void* P, int32_t* status, int64_t Tc, int64_t shift, bool records,
                     void* traj_rec = nullptr, int nvar = 1, int nv = 1) {
        kfmi::RefArgs a{};
        a.B = B;
        a.kc = h->kc;
        a.T = int(Tc);
        a.etype = etype;
        a.dt = dt;
        a.payload = payload;
        a.x = x;
        a.P = P;
        a.status = status;
        if (records) {
            a.traj = traj_rec ? traj_rec : traj;
            a.s_nvar = nvar;
            a.s_vstride = nvar > 1 ? vstride : 0;
            a.cov = cov;
            a.logdet = logdet;
            a.updated = updated;
        }
        a.gate = gate;
        a.threshold = threshold;
        a.s_len = T;
        a.s_chunk = L;
        a.s_shift = shift;
        a.s_nchunks = C;
        if (nv == 4) {  // the map pass: its epilogue writes the chunk maps and checks the seams
            a.s_maps = sa.maps;
            a.s_delta = sa.delta;
            a.s_wnext = sa.wP;
            a.s_check = sa.check;
        }
        return kfmi::launch_ref_stream(h->model, f64, a, st, nv);
    };
    hipError_t e = hipSuccess;
    if (lft) {
        // every chunk start from at least `iters` chunks of maps: kStreamLftEvents events of
        // forgetting; one start thread walks iters + G chunks
        sa.iters = int((kStreamLftEvents + L - 1) / L) + 1;
        // the start kernel: a block of 64 threads, g chunks each, stages the piece maps of its
        // windows, (64 g + iters) * np of them, in 64 KB of LDS; g = 0: no LDS (one chunk per
        // thread, maps from global memory)
        const int64_t fit = kStreamStartLdsMaps / np - sa.iters;
        sa.g = fit >= 64 ? std::min<int64_t>(fit / 64, KF_START_MAX_G) : 0;  // <= kStartMaxG
        sa.G = 64 * sa.g;
        e = kfmi::launch_stream_phase(h->model, f64, kfmi::kStreamPhaseLftMaps, sa, st);
        // the start kernel also zeroes the check and fills the warm-up bank (and, without event
        // warm-up, the map bank)
        if (e == hipSuccess) e = kfmi::launch_stream_phase(h->model, f64, kfmi::kStreamPhaseLftStart, sa, st);
    } else {
        e = kfmi::launch_stream_phase(h->model, f64, 0, sa, st);
    }
    if (e == hipSuccess && W > 0) e = chain(C, sa.wx, sa.wP, sa.wst, W, -W, false);
    if (e == hipSuccess && (!lft || W > 0)) e = kfmi::launch_stream_phase(h->model, f64, 1, sa, st);
    if (map_records) {
        // the map pass writes the records (variant 0's covariance, logdet, updated flags, and
        // every variant's trajectory); the trajectories are then the affine maps' values at the
        // true chunk starts
        if (e == hipSuccess) e = chain(C, sa.mx, sa.mP, sa.mst, L, 0, true, traj ? traj4 : nullptr, 4, 4);
        // the maps composed into the chunk starts (the tile scan, then the starts kernel, which
        // composes the tile products itself), and the verdict
        for (int ph : {kfmi::kStreamPhaseScanTiles, kfmi::kStreamPhaseTop, kfmi::kStreamPhaseStarts})
            if (e == hipSuccess && (ph != kfmi::kStreamPhaseTop || top))
                e = kfmi::launch_stream_phase(h->model, f64, ph, sa, st);
        if (e == hipSuccess && traj) e = kfmi::launch_stream_phase(h->model, f64, kfmi::kStreamPhaseRecords, sa, st);
    } else {
        if (e == hipSuccess) e = chain(C, sa.mx, sa.mP, sa.mst, L, 0, false, nullptr, 1, 4);
        for (int ph : {kfmi::kStreamPhaseScanTiles, kfmi::kStreamPhaseTop, kfmi::kStreamPhaseStarts})
            if (e == hipSuccess && (ph != kfmi::kStreamPhaseTop || top))
                e = kfmi::launch_stream_phase(h->model, f64, ph, sa, st);
        if (e == hipSuccess) e = chain(C, sa.fx, sa.fP, sa.fst, L, 0, true);
        if (e == hipSuccess) e = kfmi::launch_stream_phase(h->model, f64, kfmi::kStreamPhaseFinish, sa, st);
    }
    if (e != hipSuccess) return hip_fail(e, "kf_run_stream");
    // the sequential run, which does nothing unless a check failed.  A gated f64 run whose
    // chunked pass updated at most 1 event in kStreamLookaheadShare runs it with the look-ahead
    // kernel (2.3x the chain kernel at 3 % updated, slower from about 20 %), chosen
    // on the device: both launches are queued and each returns on its flag
    if (gate && f64 && updated && opt(h, KF_OPT_EVENTS_KERNEL) == 0) {
        e = kfmi::launch_stream_choose(sa.check, updated, T, kStreamLookaheadShare, st);
        if (e != hipSuccess) return hip_fail(e, "kf_run_stream");
        int rc = run_events_launch(h, T, etype, dt, payload, traj, cov, logdet, updated, gate, threshold,
                                   &sa.check->skip_gated, stream, kfmi::kEventsGated);
        if (rc != KF_OK) return rc;
        return run_events_launch(h, T, etype, dt, payload, traj, cov, logdet, updated, gate, threshold,
                                 &sa.check->skip_chain, stream, kfmi::kEventsChain);
    }
    return run_events_launch(h, T, etype, dt, payload, traj, cov, logdet, updated, gate, threshold, &sa.check->ok,
                             stream);
}
}  // namespace

int kf_stream_check(kf_batch* h, double* out, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (!out) return fail(KF_EINVAL, "kf_stream_check: null output");
    if (!h->stream_ws && h->s_chunks != 1) return fail(KF_EINVAL, "kf_stream_check: no kf_run_stream on this handle");
    kfmi::StreamCheck k{};
    if (h->s_chunks > 1) {
        hipError_t e = hipMemcpyAsync(&k, h->stream_ws, sizeof k, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream));
        if (e == hipSuccess) e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
        if (e != hipSuccess) return hip_fail(e, "kf_stream_check");
    }
    out[0] = k.ok;
    out[1] = (k.bad & ~kfmi::kStreamBadStart) ? 1.0 : 0.0;
    out[2] = k.cov_gap;
    out[3] = k.state_gap;
    out[4] = double(h->s_chunks);
    out[5] = double(h->s_len);
    out[6] = double(h->s_warm);
    // the sequential fallback's kernel: 0 none (the chunked records stood), 2 chain, 4 look-ahead
    out[7] = h->s_chunks > 1 && k.ok ? 0.0 : k.skip_chain ? 4.0 : 2.0;
    return KF_OK;
}

int kf_eval_combos(kf_batch* h, int n_events, const double* events, const double* init, double prev_time,
                   double target_end, int k, uint64_t combo_offset, void* logdets, void* max_logdet,
                   int32_t* n_records, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (int rc = check_combo_inputs(h, n_events, events, init, "kf_eval_combos")) return rc;
    if (k < 1 || k > n_events) return fail(KF_EINVAL, "kf_eval_combos: k = %d outside [1, %d]", k, n_events);
    // the k + 2 logdet record rows are addressed through one buffer descriptor with a 32-bit
    // byte range and 32-bit lane offsets (ref15_combo_kernel)
    if (logdets && uint64_t(k + 2) * uint64_t(h->B) * elem(h) >= (uint64_t(1) << 32))
        return fail(KF_EINVAL, "kf_eval_combos: logdet records of %d rows x %lld filters exceed 4 GiB; "
                               "use fewer filters per launch or logdets = NULL", k + 2, (long long)h->B);
    if (h->B == 0) return KF_OK;
    const uint64_t n_combos = binom_table()[n_events * (kMaxComboEvents + 1) + k];
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (int rc = upload_combo_inputs(h, n_events, events, init, st, "kf_eval_combos: upload")) return rc;
    char* ws = static_cast<char*>(h->ws);
    kfmi::Ref15ComboArgs a{};
    a.B = h->B;
    a.kc = h->kc;
    a.n_events = n_events;
    a.k = k;
    a.combo_offset = combo_offset;
    a.n_combos = n_combos;
    a.ev = reinterpret_cast<const double*>(ws);
    a.binom = reinterpret_cast<const uint64_t*>(ws + kWsEvents);
    a.init = reinterpret_cast<const double*>(ws + kWsEvents + kWsBinom);
    a.prev_time = prev_time;
    a.target_end = target_end;
    a.x = h->x;
    a.P = h->P;
    a.status = h->status;
    a.logdets = logdets;
    a.max_logdet = max_logdet;
    a.n_records = n_records;
    hipError_t e = kfmi::launch_ref15_combos(h->dtype == KF_F64, a, st);
    return e == hipSuccess ? KF_OK : hip_fail(e, "kf_eval_combos");
}

namespace {
// kf_search_combos' shape for (n_events, n_fixed, fixed_mask, k_max): the free levels it
// searches, whether it runs axis-symmetric, its widest stored level, the first level over the
// parent cap (0 = none) and its workspace bytes.  Free levels 1 .. kf_max - 1 are stored, and
// of each only the subsets whose largest free candidate is <= n - 3 (the colex ranks below
// C(n - 2, k)): a subset holding candidate n - 1 has no children, and one holding n - 2 (but not
// n - 1) has the single child that adds n - 1, which the launch creating it scores from
// registers (Ref15SearchArgs::tail).
struct SearchShape {
    int n = 0, k_base = 0, kf_max = 0, over_cap = 0;
    bool sym = false;
    uint64_t widest = 0, max_par = 0;
    size_t level = 0, need = 0;
};
constexpr size_t kSearchHeadBytes = 4096;  // best[65], n_acc[65]

int search_shape(const kf_batch* h, int n_events, const double* init, int n_fixed, uint64_t fixed_mask, int k_max,
                 const char* who, SearchShape* s) {
    if (n_fixed < 0 || n_fixed >= n_events)
        return fail(KF_EINVAL, "%s: n_fixed = %d outside [0, %d)", who, n_fixed, n_events);
    if (n_fixed < 64 && (fixed_mask >> n_fixed) != 0)
        return fail(KF_EINVAL, "%s: fixed_mask has bits at or above n_fixed = %d", who, n_fixed);
    s->k_base = __builtin_popcountll(fixed_mask);
    s->n = n_events - n_fixed;  // free candidates
    if (k_max <= s->k_base || k_max > n_events)
        return fail(KF_EINVAL, "%s: k_max = %d outside [%d, %d]", who, k_max, s->k_base + 1, n_events);
    const int n = s->n;
    s->kf_max = k_max - s->k_base < n ? k_max - s->k_base : n;  // free levels searched
    const uint64_t* binom = binom_table();
    auto C = [&](int a, int b) { return binom[a * (kMaxComboEvents + 1) + b]; };
    for (int k = 1; k < s->kf_max; ++k) s->widest = n >= 2 && C(n - 2, k) > s->widest ? C(n - 2, k) : s->widest;
    for (int k = 2; k <= s->kf_max && n >= 2; ++k) {
        const uint64_t par = C(n - 2, k - 1);
        s->max_par = par > s->max_par ? par : s->max_par;
        if (!s->over_cap && par >= (1ull << 28)) s->over_cap = k;
    }
    s->sym = search_sym(h, init);
    s->level = s->widest ? static_cast<size_t>(kfmi::search_level_bytes(s->widest, elem(h), s->sym)) : 0;
    s->need = kSearchHeadBytes + 2 * s->level;
    return KF_OK;
}
}  // namespace

int kf_search_plan(const kf_batch* h, int n_events, const double* init, int n_fixed, uint64_t fixed_mask, int k_max,
                   int64_t* out) {
    if (int rc = check_handle(h)) return rc;
    if (h->model != KF_MODEL_REF15) return fail(KF_EINVAL, "kf_search_plan: needs a KF_MODEL_REF15 handle");
    if (n_events < 1 || n_events > kMaxComboEvents)
        return fail(KF_EINVAL, "kf_search_plan: n_events = %d outside [1, %d]", n_events, kMaxComboEvents);
    if (!init || !out) return fail(KF_EINVAL, "kf_search_plan: null init/out");
    SearchShape s;
    if (int rc = search_shape(h, n_events, init, n_fixed, fixed_mask, k_max, "kf_search_plan", &s)) return rc;
    out[0] = s.sym;
    out[1] = static_cast<int64_t>(s.need);
    out[2] = static_cast<int64_t>(s.widest);
    out[3] = static_cast<int64_t>(s.max_par);
    out[4] = s.over_cap;
    return KF_OK;
}

int kf_search_combos(kf_batch* h, int n_events, const double* events, const double* init, double prev_time,
                     double target_end, double threshold, int k_max, int exhaustive, int n_fixed,
                     uint64_t fixed_mask, uint64_t* winner, int* k_found, uint64_t* n_accepted, void* subset_max,
                     void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (int rc = check_combo_inputs(h, n_events, events, init, "kf_search_combos")) return rc;
    SearchShape shape;
    if (int rc = search_shape(h, n_events, init, n_fixed, fixed_mask, k_max, "kf_search_combos", &shape)) return rc;
    const int k_base = shape.k_base, n = shape.n, kf_max = shape.kf_max;
    if (!winner || !k_found) return fail(KF_EINVAL, "kf_search_combos: null winner/k_found");
    if (subset_max && n_events > 30)
        return fail(KF_EINVAL, "kf_search_combos: subset_max needs n_events <= 30 (2^n entries)");
    const uint64_t* binom = binom_table();
    auto C = [&](int a, int b) { return binom[a * (kMaxComboEvents + 1) + b]; };
    if (shape.over_cap) {
        const int k = shape.over_cap;
        return fail(KF_EINVAL, "kf_search_combos: level %d has C(%d, %d) = %llu parents (limit 2^28); lower k_max",
                    k, n - 2, k - 1, static_cast<unsigned long long>(C(n - 2, k - 1)));
    }
    const size_t head = kSearchHeadBytes;
    const bool sym = shape.sym;
    const size_t level = shape.level;
    int64_t launches = 0;
    const size_t need = shape.need;
    hipStream_t st = static_cast<hipStream_t>(stream);
    void* const ws_before = h->search_ws;
    if (!grow_ws(h, &h->search_ws, &h->search_ws_bytes, &h->search_ws_graph, need, st))
        return capturing(st) ? fail(KF_EINVAL, "kf_search_combos: the level buffers (%zu bytes) must be sized by an "
                                               "eager call before a graph capture", need)
                             : fail(KF_ENOMEM, "kf_search_combos: hipMalloc of %zu bytes of level buffers failed", need);
    if (capturing(st))
        return fail(KF_EINVAL, "kf_search_combos: not capturable (its results return to the host in the call)");
    if (!h->search_host) {
        void* p = nullptr;
        if (hipHostMalloc(&p, sizeof(uint64_t) * 2 * (kMaxComboEvents + 1), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess) {
            (void)hipGetLastError();
            return fail(KF_ENOMEM, "kf_search_combos: hipHostMalloc of the result buffer failed");
        }
        void* pd = nullptr;
        if (hipHostGetDevicePointer(&pd, p, 0) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipHostFree(p);
            return fail(KF_EHIP, "kf_search_combos: no device address for the result buffer");
        }
        h->search_host = static_cast<uint64_t*>(p);
        h->search_host_dev = static_cast<uint64_t*>(pd);
    }
    if (int rc = upload_combo_inputs(h, n_events, events, init, st, "kf_search_combos: upload")) return rc;
    char* ws = static_cast<char*>(h->ws);
    char* sw = static_cast<char*>(h->search_ws);
    uint64_t* d_best = reinterpret_cast<uint64_t*>(sw);
    uint64_t* d_acc = d_best + (kMaxComboEvents + 1);
    // the counters: zeroed by the previous search's finish kernel when it ran on this stream in
    // this workspace, otherwise cleared here; until this search's finish they are not known zero
    const bool ctr_zero = h->search_ctr_zero && h->search_ctr_stream == st && h->search_ws == ws_before;
    h->search_ctr_zero = false;
    hipError_t e = ctr_zero ? hipSuccess : hipMemsetAsync(sw, 0, head, st);
    if (e != hipSuccess) return hip_fail(e, "kf_search_combos: clear");
    char* lv[2] = {sw + head, sw + head + level};
    int cur = 0;  // the buffer holding the last stored level (its children go to the other one)
    uint64_t best[kMaxComboEvents + 1] = {}, acc[kMaxComboEvents + 1] = {};
    int found = 0, last = 0;
    // the head: levels 1 .. K in one launch, one lane per subset (launch_ref15_search_head), K the
    // largest size whose subsets' event steps from the root (sum_k k C(n, k)) stay within
    // kSearchHeadSteps, at least 2 and below kf_max (level K + 1 reads its stored nodes)
    int K = 0;
    if (opt(h, KF_OPT_SEARCH_HEAD) == 0 && n >= 5) {
        uint64_t steps = 0;
        for (int k = 1; k <= n - 2 && k < kf_max; ++k) {
            steps += uint64_t(k) * C(n, k);
            if (steps > kSearchHeadSteps) break;
            K = k;
        }
        if (K < 2) K = 0;
    }
    int k_first = 1;
    if (K) {
        kfmi::Ref15SearchArgs a{};
        a.kc = h->kc;
        a.n_events = n;
        a.k = K;
        a.shift = n_fixed;
        a.k_base = k_base;
        a.root_mask = fixed_mask;
        a.ev_all = reinterpret_cast<const double*>(ws);
        for (int k = 1; k <= K; ++k) a.n_child += C(n, k);
        a.ev = reinterpret_cast<const double*>(ws) + 11 * n_fixed;
        a.binom = reinterpret_cast<const uint64_t*>(ws + kWsEvents);
        a.binom_host = binom;
        a.init = reinterpret_cast<const double*>(ws + kWsEvents + kWsBinom);
        a.prev_time = prev_time;
        a.target_end = target_end;
        a.threshold = threshold;
        kfmi::set_search_band(a, h->dtype == KF_F64);
        a.child = lv[cur = K & 1];
        a.best = d_best;
        a.n_acc = d_acc;
        a.subset_max = subset_max;
        a.tail = 1;
        a.sym = sym;
        e = kfmi::launch_ref15_search_head(h->dtype == KF_F64, a, st);
        if (e != hipSuccess) return hip_fail(e, "kf_search_combos: head launch");
        last = k_base + K;
        k_first = K + 1;
        if (!exhaustive) {  // any acceptable subset of sizes k_base .. k_base + K ends the search
            e = kfmi::launch_search_finish(d_best, h->search_host_dev, kMaxComboEvents + 1, false, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return hip_fail(e, "kf_search_combos: head result");
            for (int k = k_base; k <= last; ++k)
                if (h->search_host[k]) k_first = kf_max + 1;
        }
    }
    // the end launch: sizes k_end0 .. kf_max in one launch, each subset from its stored
    // (k_end0 - 1)-prefix (launch_ref15_search_end), k_end0 the smallest size whose subsets' steps
    // from their prefixes (sum_{k >= k_end0} (k - k_end0 + 1) C(n, k)) stay within
    // kSearchEndSteps, above level 1 and above the head (level k_end0 - 1 is stored by a launch
    // before it), and replacing at least two level launches (levels k_end0 and k_end0 + 1 have
    // stored parents: k_end0 <= n - 2)
    // The end launch takes one wave per (extension, 64 prefixes), its extensions (the subsets of
    // k_end0 - 1 .. n - 1 of at most kf_max - k_end0 + 1 members) listed in the kernel
    // arguments: at most 63 of them (n - k_end0 + 1 <= 6).
    int k_end0 = kf_max + 1;
    if (opt(h, KF_OPT_SEARCH_END) == 0)
        for (int k0 = std::min(kf_max - 1, n - 2); k0 >= 2 && k0 > k_first && n - k0 + 1 <= 6; --k0) {
            uint64_t steps = 0;
            for (int k = k0; k <= kf_max; ++k) steps += uint64_t(k - k0 + 1) * C(n, k);
            if (steps > kSearchEndSteps) break;
            k_end0 = k0;
        }
    // not exhaustive: the results are peeked after groups of 1, 1, 2, 4, ... level launches, and
    // a launch queued past the first accepted size does nothing (Ref15SearchArgs::stop_best)
    int peek_at = k_first, peek_step = 1;
    // KF_OPT_SEARCH_PAIR: in the axis-symmetric search, level k and level k + 1 (below the end
    // launch's sizes) in one launch (launch_ref15_search_pair), level k never stored: parent-major
    // (a lane per parent) for a level of at least pm_min stored parents; with 3, every level
    // child-major instead (a wave per parent block and child event; measured slower: A/B only)
    const int64_t pair_opt = opt(h, KF_OPT_SEARCH_PAIR);
    const bool pairs = pair_opt != 1 && sym && opt(h, KF_OPT_SEARCH_PM) == 0 && opt(h, KF_OPT_SEARCH_KERNEL) == 0;
    const uint64_t pm_min = pair_opt == 0 ? kSearchPairParents : pair_opt == 2 ? 0 : pair_opt == 3 ? ~uint64_t(0)
                                                                                                   : uint64_t(pair_opt);
    const bool cm_pairs = pair_opt == 3;
    for (int k = k_first; k <= kf_max; ++k) {
        kfmi::Ref15SearchArgs a{};
        a.kc = h->kc;
        a.n_events = n;
        a.k = k;
        a.shift = n_fixed;
        a.k_base = k_base;
        a.root_mask = fixed_mask;
        a.ev_all = reinterpret_cast<const double*>(ws);
        a.n_par = k == 1 ? 1 : C(n - 2, k - 1);  // the stored parents (n >= 2 when k >= 2)
        a.n_child = C(n, k);
        a.ev = reinterpret_cast<const double*>(ws) + 11 * n_fixed;
        a.binom = reinterpret_cast<const uint64_t*>(ws + kWsEvents);
        a.binom_host = binom;
        a.init = reinterpret_cast<const double*>(ws + kWsEvents + kWsBinom);
        a.prev_time = prev_time;
        a.target_end = target_end;
        a.threshold = threshold;
        kfmi::set_search_band(a, h->dtype == KF_F64);
        a.par = k > 1 ? lv[cur] : nullptr;
        a.child = k < kf_max ? lv[1 - cur] : nullptr;
        a.best = d_best;
        a.n_acc = d_acc;
        a.subset_max = subset_max;
        a.tail = k < kf_max;
        a.sym = sym;
        if (!exhaustive && k > 1) {  // sizes k_base .. k_base + k - 1 are complete
            a.stop_best = d_best;
            a.stop_lo = k_base;
            a.stop_hi = k_base + k - 1;
        }
        if (k == k_end0) {  // the rest of the search in one launch
            a.k_end = kf_max;
            a.n_par = 0;
            a.child = nullptr;
            a.tail = 0;
            // extensions E of k_end0 - 1 .. n - 1, by size, then colex; each with the stored
            // prefixes below its smallest member (C(e, k - 1); C(n - 2, k - 1) for E = {n - 1})
            const int lo_c = k - 1, span = n - lo_c;
            a.n_groups = 0;
            a.n_child = 0;
            uint64_t waves = 0;
            for (int m = 1; m <= kf_max - k + 1; ++m)
                for (uint32_t bits = 1; bits < (1u << span); ++bits) {
                    if (__builtin_popcount(bits) != m) continue;
                    const uint64_t ext = uint64_t(bits) << lo_c;
                    const int e = __builtin_ctzll(ext);
                    const uint64_t pre = C(e == n - 1 ? n - 2 : e, k - 1);
                    if (!pre) continue;
                    a.gblk[a.n_groups] = ext;
                    a.gitem[a.n_groups] = waves;
                    ++a.n_groups;
                    waves += (pre + 63) / 64;
                    a.n_child += pre;
                }
            a.gitem[a.n_groups] = waves;
            e = kfmi::launch_ref15_search_end(h->dtype == KF_F64, a, st);
            if (e != hipSuccess) return hip_fail(e, "kf_search_combos: end launch");
            ++launches;
            last = k_base + kf_max;
            break;
        }
        // a level without stored parents was scored whole by the previous launch's tail
        const bool pm_pair = !search_child_major(h, a.n_par) && a.n_par >= pm_min;
        if (a.n_par && pairs && k >= 2 && k + 1 <= kf_max && k + 1 < k_end0 && (pm_pair || cm_pairs)) {
            // levels k and k + 1: level k + 1 stored (in the other buffer) when it has children
            a.child = k + 1 < kf_max ? lv[1 - cur] : nullptr;
            a.tail = k + 1 < kf_max;
            e = kfmi::launch_ref15_search_pair(h->dtype == KF_F64, a, !pm_pair, st);
            if (e != hipSuccess) return hip_fail(e, "kf_search_combos: pair launch");
            ++launches;
            ++k;
        } else if (a.n_par) {
            a.pm_regs = opt(h, KF_OPT_SEARCH_PM) == 1;
            e = kfmi::launch_ref15_search(h->dtype == KF_F64, a, search_child_major(h, a.n_par), st);
            if (e != hipSuccess) return hip_fail(e, "kf_search_combos: level launch");
            ++launches;
        }
        if (a.n_par && a.child) cur = 1 - cur;
        last = k_base + k;
        if (!exhaustive && k >= peek_at && k < kf_max) {
            // the reference stops at the first size with an acceptable subset (the first launch
            // also scores the fixed root itself, size k_base)
            e = kfmi::launch_search_finish(d_best, h->search_host_dev, kMaxComboEvents + 1, false, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return hip_fail(e, "kf_search_combos: level result");
            bool any = false;
            for (int s2 = k_base; s2 <= last; ++s2) any = any || h->search_host[s2] != 0;
            if (any) break;
            peek_at = k + peek_step;
            peek_step *= 2;
        }
    }
    // best[] and n_acc[] are adjacent on the device: one kernel writes both to the host buffer
    // and zeroes them for the next search
    e = kfmi::launch_search_finish(d_best, h->search_host_dev, 2 * (kMaxComboEvents + 1), true, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "kf_search_combos: results");
    h->search_ctr_zero = true;
    h->search_ctr_stream = st;
    std::memcpy(best, h->search_host, sizeof best);
    std::memcpy(acc, h->search_host + (kMaxComboEvents + 1), sizeof acc);
    for (int k = k_base > 0 ? k_base : 1; k <= last && !found; ++k)
        if (best[k]) found = k;
    h->search_info[0] = sym;
    h->search_info[1] = K;
    h->search_info[2] = launches;
    h->search_info[3] = static_cast<int64_t>(level);
    *k_found = found;
    *winner = found ? __builtin_bitreverse64(best[found]) : 0;
    // without `exhaustive` the search ends at the first accepted size: the one-launch head may
    // have counted larger sizes too, which the level-by-level search never reaches
    const int reported = !exhaustive && found ? found : last;
    if (n_accepted)
        for (int k = 0; k <= k_max; ++k) n_accepted[k] = k <= reported ? acc[k] : 0;
    return KF_OK;
}

int kf_search_info(const kf_batch* h, int64_t* out) {
    if (int rc = check_handle(h)) return rc;
    if (!out) return fail(KF_EINVAL, "kf_search_info: null output");
    for (int i = 0; i < 4; ++i) out[i] = h->search_info[i];
    return KF_OK;
}

int kf_score_candidates(kf_batch* h, int n_types, const int32_t* types, int full, void* gain, void* post,
                        void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (!is_ref15(h)) return fail(KF_EINVAL, "kf_score_candidates: needs a KF_MODEL_REF15 handle");
    if (n_types < 1 || n_types > 16) return fail(KF_EINVAL, "kf_score_candidates: n_types = %d outside [1, 16]", n_types);
    if (!types || !gain) return fail(KF_EINVAL, "kf_score_candidates: null types/gain");
    if (h->B == 0) return KF_OK;
    kfmi::Ref15ScoreArgs a{};
    a.B = h->B;
    a.kc = h->kc;
    a.n_types = n_types;
    a.full = full;
    for (int i = 0; i < n_types; ++i) {
        if (types[i] != KF_EVENT_GPS && types[i] != KF_EVENT_IMU)
            return fail(KF_EINVAL, "kf_score_candidates: candidate %d has type %d (GPS=0 or IMU=1)", i, types[i]);
        a.types[i] = static_cast<int8_t>(types[i]);
    }
    a.x = h->x;
    a.P = h->P;
    a.gain = gain;
    a.post = post;
    hipError_t e = kfmi::launch_ref15_score(h->dtype == KF_F64, a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? KF_OK : hip_fail(e, "kf_score_candidates");
}

int kf_score_rows(kf_batch* h, int n_cand, const int32_t* types, const uint32_t* row_masks, void* gain, void* post,
                  void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (!is_ref15(h)) return fail(KF_EINVAL, "kf_score_rows: needs a KF_MODEL_REF15 handle");
    if (n_cand < 1 || n_cand > 16) return fail(KF_EINVAL, "kf_score_rows: n_cand = %d outside [1, 16]", n_cand);
    if (!types || !row_masks || !gain) return fail(KF_EINVAL, "kf_score_rows: null types/row_masks/gain");
    kfmi::Ref15ScoreArgs a{};
    a.B = h->B;
    a.kc = h->kc;
    a.n_types = n_cand;
    a.rows = 1;
    for (int i = 0; i < n_cand; ++i) {
        const bool gps = types[i] == KF_EVENT_GPS;
        if (!gps && types[i] != KF_EVENT_IMU)
            return fail(KF_EINVAL, "kf_score_rows: candidate %d has type %d (GPS=0 or IMU=1)", i, types[i]);
        const uint32_t rows = gps ? 3u : 15u;
        if (row_masks[i] == 0 || (row_masks[i] >> rows) != 0)
            return fail(KF_EINVAL, "kf_score_rows: candidate %d row mask 0x%x is empty or names a row beyond %u", i,
                        row_masks[i], rows);
        a.types[i] = static_cast<int8_t>(types[i]);
        a.masks[i] = row_masks[i];
    }
    if (h->B == 0) return KF_OK;
    a.x = h->x;
    a.P = h->P;
    a.gain = gain;
    a.post = post;
    hipError_t e = kfmi::launch_ref15_score(h->dtype == KF_F64, a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? KF_OK : hip_fail(e, "kf_score_rows");
}

}  // extern "C"

namespace {
// kf_run_scheduled (rec = 0: payload rows [T][9][B]) and kf_run_scheduled_rec (rec elements per
// record, [T][B][rec])
int run_scheduled(const char* fn, kf_batch* h, int T, const double* t, const uint8_t* etype, const void* payload,
                  int rec, const double* prev_time, const double* freq, double freq_all, void* traj, void* logdet,
                  double* sel_time, int32_t* n_sel, void* stream, const uint32_t* words = nullptr, int n_words = 0,
                  int32_t* words_used = nullptr) {
    if (int rc = check_handle(h)) return rc;
    if (!is_ref15(h)) return fail(KF_EINVAL, "%s: needs a KF_MODEL_REF15 handle", fn);
    if (T < 0) return fail(KF_EINVAL, "%s: T = %d < 0", fn, T);
    if (!freq && !(freq_all > 0.0)) return fail(KF_EINVAL, "%s: processing frequency must be > 0", fn);
    const int esz = h->dtype == KF_F64 ? 8 : 4;
    if (rec && (rec < 9 || (int64_t(rec) * esz) % 16 != 0))
        return fail(KF_EINVAL, "%s: rec_len = %d: need >= 9 elements and a multiple of 16 bytes (%d-byte elements)",
                    fn, rec, esz);
    if (rec && reinterpret_cast<uintptr_t>(payload) % 16 != 0)
        return fail(KF_EINVAL, "%s: the records must be 16-byte aligned", fn);
    if (h->B == 0) return KF_OK;
    if (!t || !etype || !payload || !prev_time) return fail(KF_EINVAL, "%s: null input stream", fn);
    if (words && (n_words < 0 || !words_used))
        return fail(KF_EINVAL, "%s: n_words = %d, words_used %s", fn, n_words, words_used ? "set" : "null");
    kfmi::Ref15SchedArgs a{};
    a.words = words;
    a.n_words = words ? n_words : 0;
    a.words_used = words_used;
    a.B = h->B;
    a.kc = h->kc;
    a.T = T;
    a.t = t;
    a.etype = etype;
    a.payload = payload;
    a.pay_rec = rec;
    a.prev_time = prev_time;
    a.freq = freq;
    a.freq_all = freq_all;
    a.x = h->x;
    a.P = h->P;
    a.status = h->status;
    a.traj = traj;
    a.logdet = logdet;
    a.sel_time = sel_time;
    a.n_sel = n_sel;
    // KF_OPT_SCHED_KERNEL: 1 / 2 the fused register / LDS kernels, 3 the two passes as two
    // launches, 4 as the phases of one launch; 0 the library's choice
    const int64_t sk = opt(h, KF_OPT_SCHED_KERNEL);
    a.regs = sk == 1;
    a.fused = sk == 1 || sk == 2;
    a.one_launch = sk == 4 && !words;
    // the event's time at rec[9] of f64 records (KF_OPT_SCHED_REC_TIME): the apply pass reads it
    // from the record it gathers, and writes sel_time itself
    a.rec_time = opt(h, KF_OPT_SCHED_REC_TIME) == 1 && rec >= 10 && h->dtype == KF_F64;
    a.group_waves = opt(h, KF_OPT_SCHED_GROUP) == 1 ? 1 : 4;
    // the greedy pick when both sensor classes are queued: the larger R gives the larger
    // posterior trace (launch_ref15_scheduled; checked on the covariance by the apply pass)
    a.gps_wins = h->gps_r0 > h->imu_r0 ? 1 : h->gps_r0 < h->imu_r0 ? 0 : -1;
    if (!a.fused && T > 0 && n_sel && sel_time) {
        // picks [T][B] | flags [B] | with B % 64 == 0 and KF_OPT_SCHED_ORDER 0: the waves' keys, ids,
        // sorted keys, order [B / 64] and the sort's scratch
        const size_t picks_b = align256(sizeof(uint32_t) * size_t(T) * size_t(h->B));
        const size_t flags_b = align256(sizeof(int32_t) * size_t(h->B));
        const int nw = h->B % 64 == 0 && opt(h, KF_OPT_SCHED_ORDER) == 0 ? int(h->B / 64) : 0;
        size_t sort_b = 0;
        if (nw && kfmi::sort_pairs_desc_u32(nullptr, &sort_b, nullptr, nullptr, nullptr, nullptr, nw, 32, nullptr) !=
                      hipSuccess) {
            (void)hipGetLastError();
            sort_b = 0;
        }
        const size_t wave_b = nw && sort_b ? 4 * align256(sizeof(uint32_t) * size_t(nw)) + align256(sort_b) : 0;
        const size_t need = picks_b + flags_b + wave_b;
        // no allocation inside a graph capture (hipMalloc / hipFree are not capturable): a
        // workspace too small for this T (or none at all) leaves the fused kernel to run
        if (grow_ws(h, &h->sched_ws, &h->sched_ws_bytes, &h->sched_ws_graph, need, static_cast<hipStream_t>(stream))) {
            if (capturing(static_cast<hipStream_t>(stream))) h->sched_ws_graph = true;
            char* w = static_cast<char*>(h->sched_ws);
            a.picks = reinterpret_cast<uint32_t*>(w);
            a.flags = reinterpret_cast<int32_t*>(w + picks_b);
            if (wave_b) {
                const size_t wb = align256(sizeof(uint32_t) * size_t(nw));
                char* k = w + picks_b + flags_b;
                a.wave_key = reinterpret_cast<uint32_t*>(k);
                a.wave_id = reinterpret_cast<uint32_t*>(k + wb);
                a.wave_key_sorted = reinterpret_cast<uint32_t*>(k + 2 * wb);
                a.order = reinterpret_cast<uint32_t*>(k + 3 * wb);
                a.sort_tmp = k + 4 * wb;
                a.sort_tmp_bytes = sort_b;
            }
        }
    }
    hipError_t e = kfmi::launch_ref15_scheduled(h->dtype == KF_F64, a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? KF_OK : hip_fail(e, fn);
}
}  // namespace

extern "C" {

int kf_run_scheduled(kf_batch* h, int T, const double* t, const uint8_t* etype, const void* payload,
                     const double* prev_time, const double* freq, double freq_all, void* traj, void* logdet,
                     double* sel_time, int32_t* n_sel, void* stream) {
    return run_scheduled("kf_run_scheduled", h, T, t, etype, payload, 0, prev_time, freq, freq_all, traj, logdet,
                         sel_time, n_sel, stream);
}

int kf_run_scheduled_rec(kf_batch* h, int T, const double* t, const uint8_t* etype, const void* records,
                         int rec_len, const double* prev_time, const double* freq, double freq_all, void* traj,
                         void* logdet, double* sel_time, int32_t* n_sel, void* stream) {
    if (rec_len <= 0) return fail(KF_EINVAL, "kf_run_scheduled_rec: rec_len = %d", rec_len);
    return run_scheduled("kf_run_scheduled_rec", h, T, t, etype, records, rec_len, prev_time, freq, freq_all, traj,
                         logdet, sel_time, n_sel, stream);
}

int kf_sched_random_picks(kf_batch* h, int T, const double* t, const uint8_t* etype, const double* prev_time,
                          const double* freq, double freq_all, const uint32_t* words, int n_words, int32_t* words_used,
                          int32_t* pick, double* sel_time, int32_t* n_sel, void* stream) {
    if (int rc = check_handle(h)) return rc;
    if (T < 0) return fail(KF_EINVAL, "kf_sched_random_picks: T = %d < 0", T);
    if (!freq && !(freq_all > 0.0)) return fail(KF_EINVAL, "kf_sched_random_picks: processing frequency must be > 0");
    if (h->B == 0) return KF_OK;
    if (!t || !etype || !prev_time || !words || n_words < 0 || !words_used || !pick || !sel_time || !n_sel)
        return fail(KF_EINVAL, "kf_sched_random_picks: null stream or output");
    kfmi::Ref15SchedArgs a{};
    a.B = h->B;
    a.T = T;
    a.t = t;
    a.etype = etype;
    a.prev_time = prev_time;
    a.freq = freq;
    a.freq_all = freq_all;
    a.sel_time = sel_time;
    a.n_sel = n_sel;
    a.words = words;
    a.n_words = n_words;
    a.words_used = words_used;
    hipError_t e = kfmi::launch_ref15_random_picks(a, pick, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? KF_OK : hip_fail(e, "kf_sched_random_picks");
}

int kf_run_scheduled_random(kf_batch* h, int T, const double* t, const uint8_t* etype, const void* payload,
                            int rec_len, const double* prev_time, const double* freq, double freq_all,
                            const uint32_t* words, int n_words, int32_t* words_used, void* traj, void* logdet,
                            double* sel_time, int32_t* n_sel, void* stream) {
    if (rec_len < 0) return fail(KF_EINVAL, "kf_run_scheduled_random: rec_len = %d", rec_len);
    if (!words) return fail(KF_EINVAL, "kf_run_scheduled_random: null words");
    return run_scheduled("kf_run_scheduled_random", h, T, t, etype, payload, rec_len, prev_time, freq, freq_all, traj,
                         logdet, sel_time, n_sel, stream, words, n_words, words_used);
}

}  // extern "C"
