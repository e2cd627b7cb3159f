// gfx950 ingest: parsed GPS/IMU columns -> one merged, time-sorted event stream in HBM
// (kf_ingest), and the per-event dt of the reference drivers (kf_events_dt).
//
// Replaces the per-row Python of KF_SensorFusion (kf_workers.py:304-385):
//   gps_to_modified_utm (304-331)  -> fix_kernel: keep/drop test, UTM projection per fix
//   compute_imu_biases (333-347)   -> bias_kernel: mean of the first first_valid_index IMU rows
//   unbias_imu_data (349-373) with quaternion_to_euler (399-425)
//                                  -> fused into gather_kernel, computed once per IMU event
//   combine_sensor_data (375-385)  -> stable radix sort on time of [fixes..., IMU rows...]
//                                     (hipCUB), so ties keep GPS first as Python's stable sort
//                                     does, then gather_kernel writes the SoA stream
// Everything is fp64, as in the reference.  Expressions are evaluated in the reference's order
// with FMA contraction off, so the only differences left are the last-ulp behaviour of the
// transcendental functions (sin/cos/atan2/asin vs the host libm).
//
// Output stream layout (one row per event, the [T][9] payload layout kf_run_events reads for a
// single filter): etype [N] uint8, t [N] f64, payload [N][9] f64, src [N] int32 (position in
// the reference's utm_data list for a fix, IMU row index for an IMU sample).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <hipcub/hipcub.hpp>
#include <mutex>
#include <vector>

#include "../../include/kf.h"
#include "kf_internal.h"

namespace kfmi {
hipError_t sort_pairs_desc_u32(void* tmp, size_t* tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                               const uint32_t* vals_in, uint32_t* vals_out, int n, int bits, hipStream_t stream) {
    return hipcub::DeviceRadixSort::SortPairsDescending(tmp, *tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0,
                                                        bits, stream);
}

namespace {

constexpr int kIngBlock = 256;

// --- utm.from_latlon (published algorithm of the `utm` package; oracle/ref_ingest.py) --------
constexpr double kK0 = 0.9996;
constexpr double kE = 0.00669438;
constexpr double kE2 = kE * kE;
constexpr double kE3 = kE2 * kE;
constexpr double kEP2 = kE / (1 - kE);
constexpr double kM1 = (1 - kE / 4 - 3 * kE2 / 64 - 5 * kE3 / 256);
constexpr double kM2 = (3 * kE / 8 + 3 * kE2 / 32 + 45 * kE3 / 1024);
constexpr double kM3 = (15 * kE2 / 256 + 45 * kE3 / 1024);
constexpr double kM4 = (35 * kE3 / 3072);
constexpr double kR = 6378137.0;
constexpr double kPi = 3.141592653589793;

__device__ __forceinline__ double radians(double d) {
#pragma clang fp contract(off)
    return d * (kPi / 180.0);  // math.radians: x * (pi / 180)
}

__device__ __forceinline__ int zone_number(double lat, double lon) {
    if (56 <= lat && lat < 64 && 3 <= lon && lon < 12) return 32;
    if (72 <= lat && lat <= 84 && lon >= 0) {
        if (lon < 9) return 31;
        if (lon < 21) return 33;
        if (lon < 33) return 35;
        if (lon < 42) return 37;
    }
    return static_cast<int>((lon + 180) / 6) + 1;  // int() truncates toward zero
}

__device__ __forceinline__ char zone_letter(double lat) {
    const char letters[] = "CDEFGHJKLMNPQRSTUVWXX";
    if (!(-80 <= lat && lat <= 84)) return 0;
    return letters[static_cast<int>(lat + 80) >> 3];
}

__device__ void utm_from_latlon(double lat, double lon, double& easting, double& northing, int& zn, char& zl) {
#pragma clang fp contract(off)
    const double lat_rad = radians(lat);
    const double lat_sin = sin(lat_rad);
    const double lat_cos = cos(lat_rad);
    const double lat_tan = lat_sin / lat_cos;
    const double lat_tan2 = lat_tan * lat_tan;
    const double lat_tan4 = lat_tan2 * lat_tan2;
    zn = zone_number(lat, lon);
    zl = zone_letter(lat);
    const double lon_rad = radians(lon);
    const double central_lon_rad = radians(static_cast<double>((zn - 1) * 6 - 180 + 3));
    const double n = kR / sqrt(1 - kE * (lat_sin * lat_sin));
    const double c = kEP2 * (lat_cos * lat_cos);
    const double a = lat_cos * (lon_rad - central_lon_rad);
    const double a2 = a * a, a3 = pow(a, 3.0), a4 = pow(a, 4.0), a5 = pow(a, 5.0), a6 = pow(a, 6.0);
    const double m = kR * (kM1 * lat_rad - kM2 * sin(2 * lat_rad) + kM3 * sin(4 * lat_rad) - kM4 * sin(6 * lat_rad));
    easting = kK0 * n * (a + a3 / 6 * (1 - lat_tan2 + c) + a5 / 120 * (5 - 18 * lat_tan2 + lat_tan4 + 72 * c - 58 * kEP2)) +
              500000;
    northing = kK0 * (m + n * lat_tan * (a2 / 2 + a4 / 24 * (5 - lat_tan2 + 9 * c + 4 * (c * c)) +
                                         a6 / 720 * (61 - 58 * lat_tan2 + lat_tan4 + 600 * c - 330 * kEP2)));
    if (lat < 0) northing += 10000000;
}

// quaternion_to_euler (kf_workers.py:399-425)
__device__ void quat_to_euler(double x, double y, double z, double w, double& roll, double& pitch, double& yaw) {
#pragma clang fp contract(off)
    const double sinr_cosp = 2 * (w * x + y * z);
    const double cosr_cosp = 1 - 2 * (x * x + y * y);
    roll = atan2(sinr_cosp, cosr_cosp);
    const double sinp = 2 * (w * y - z * x);
    if (fabs(sinp) >= 1)
        pitch = kPi / 2 * (sinp > 0 ? 1.0 : -1.0);  // np.pi / 2 * np.sign(sinp)
    else
        pitch = asin(sinp);
    const double siny_cosp = 2 * (w * z + x * y);
    const double cosy_cosp = 1 - 2 * (y * y + z * z);
    yaw = atan2(siny_cosp, cosy_cosp);
}

struct IngestArgs {
    int64_t n_gps, n_imu;
    int64_t ld_gps, ld_imu;
    const double* gps;          // [4][ld_gps]: time, latitude, longitude, altitude
    const double* imu;          // [11][ld_imu]: time, qx, qy, qz, qw, wx, wy, wz, ax, ay, az
    int check_alt;
    double* east;               // [n_gps] workspace
    double* north;
    int8_t* zone;               // [n_gps] zone number (0: not kept)
    char* letter;
    int32_t* keep;              // [n_gps] 0/1
    unsigned long long* first;  // [2]: first row with a latitude, first kept row
    double* bias;               // [6]: angular velocity, linear acceleration
    double* keys;               // [n_gps + n_imu]
    int32_t* vals;
};

__global__ __launch_bounds__(kIngBlock) void fix_kernel(const IngestArgs a) {
    const int64_t i = int64_t(blockIdx.x) * kIngBlock + threadIdx.x;
    if (i >= a.n_gps) return;
    const double t = a.gps[i];
    const double lat = a.gps[a.ld_gps + i];
    const double lon = a.gps[2 * a.ld_gps + i];
    const double alt = a.gps[3 * a.ld_gps + i];
    const bool lat_ok = !isnan(lat);
    const bool kept = lat_ok && !isnan(lon) && !(a.check_alt && isnan(alt));  // kf_workers.py:310 / hw5_2.py:35
    if (lat_ok) atomicMin(&a.first[0], static_cast<unsigned long long>(i));
    double e = 0, n = 0;
    int zn = 0;
    char zl = 0;
    if (kept) {
        atomicMin(&a.first[1], static_cast<unsigned long long>(i));
        utm_from_latlon(lat, lon, e, n, zn, zl);
    }
    a.east[i] = e;
    a.north[i] = n;
    a.zone[i] = static_cast<int8_t>(zn);
    a.letter[i] = zl;
    a.keep[i] = kept ? 1 : 0;
    a.keys[i] = kept ? t : __builtin_inf();  // dropped fixes sort past every event
    a.vals[i] = static_cast<int32_t>(i);
}

__global__ __launch_bounds__(kIngBlock) void imu_keys_kernel(const IngestArgs a) {
    const int64_t j = int64_t(blockIdx.x) * kIngBlock + threadIdx.x;
    if (j >= a.n_imu) return;
    a.keys[a.n_gps + j] = a.imu[j];
    a.vals[a.n_gps + j] = static_cast<int32_t>(a.n_gps + j);
}

// compute_imu_biases: np.mean over axis 0 of the first first_valid_index rows, i.e. a sequential
// row-by-row sum per component divided by the count (NaN for an empty slice, as NumPy gives).
__global__ void bias_kernel(const IngestArgs a) {
    const int k = threadIdx.x;
    if (k >= 6) return;
    const unsigned long long f = a.first[0];
    const int64_t cnt = static_cast<int64_t>(f < static_cast<unsigned long long>(a.n_imu) ? f : a.n_imu);
    const double* col = a.imu + (5 + k) * a.ld_imu;
    // rows added one after another (NumPy's axis-0 order), their loads issued 32 at a time (a
    // load-add loop waited one memory latency per row: 0.5 ms for the config 1 log)
    double s = 0.0;
    int64_t r = 0;
    for (; r + 32 <= cnt; r += 32) {
        double v[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = col[r + j];
#pragma unroll
        for (int j = 0; j < 32; ++j) s += v[j];
    }
    for (; r < cnt; ++r) s += col[r];
    a.bias[k] = s / static_cast<double>(cnt);
}

struct GatherArgs {
    int64_t n_events, n_gps, ld_gps, ld_imu;
    const double* gps;
    const double* imu;
    const int32_t* vals;   // sorted source ids
    const int32_t* pos;    // exclusive scan of keep: fix id -> utm_data position
    const double* east;
    const double* north;
    const int8_t* zone;
    const char* letter;
    const unsigned long long* first;
    const double* bias;
    uint8_t* etype;
    double* t;
    double* payload;       // [N][9]
    int32_t* src;
    int8_t* zone_out;
    char* letter_out;
};

__global__ __launch_bounds__(kIngBlock) void gather_kernel(const GatherArgs a) {
#pragma clang fp contract(off)
    const int64_t p = int64_t(blockIdx.x) * kIngBlock + threadIdx.x;
    if (p >= a.n_events) return;
    const int64_t v = a.vals[p];
    double pay[9];
    if (v < a.n_gps) {
        const int64_t o = static_cast<int64_t>(a.first[1]);
        a.etype[p] = KF_EVENT_GPS;
        a.t[p] = a.gps[v];
        pay[0] = a.east[v] - a.east[o];    // kf_workers.py:325-328
        pay[1] = a.north[v] - a.north[o];
        pay[2] = a.gps[3 * a.ld_gps + v];  // altitude
#pragma unroll
        for (int k = 3; k < 9; ++k) pay[k] = 0.0;
        if (a.src) a.src[p] = a.pos[v];
        if (a.zone_out) a.zone_out[p] = a.zone[v];
        if (a.letter_out) a.letter_out[p] = a.letter[v];
    } else {
        const int64_t j = v - a.n_gps;
        const double* q = a.imu + j;
        a.etype[p] = KF_EVENT_IMU;
        a.t[p] = q[0];
        quat_to_euler(q[1 * a.ld_imu], q[2 * a.ld_imu], q[3 * a.ld_imu], q[4 * a.ld_imu], pay[0], pay[1], pay[2]);
#pragma unroll
        for (int k = 0; k < 6; ++k) pay[3 + k] = q[(5 + k) * a.ld_imu] - a.bias[k];  // kf_workers.py:358-359
        if (a.src) a.src[p] = static_cast<int32_t>(j);
        if (a.zone_out) a.zone_out[p] = 0;
        if (a.letter_out) a.letter_out[p] = 0;
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) a.payload[p * 9 + k] = pay[k];
}

// kf_events_dt.  rule 0 (run_kalman_filter_full, kf_workers.py:682-686): the previous time is
// the previous event's time whether or not that event was skipped; rule 1 (adaptive / no-update
// drivers and the combination worker, :1012-1016, :38-40): a skipped event leaves the previous
// time alone, so it is the running maximum of the times before; rule 2 (run_kalman_filter,
// :763-767, hw5_2.py:331-336): no guard, negative dt is predicted over.
__global__ __launch_bounds__(kIngBlock) void dt_kernel(int64_t n, const double* t, const double* prev,
                                                        const uint8_t* et_in, double prev0, int rule, double* dt,
                                                        uint8_t* et_out) {
    const int64_t i = int64_t(blockIdx.x) * kIngBlock + threadIdx.x;
    if (i >= n) return;
    double p;
    if (rule == 1)
        p = prev[i];
    else if (i == 0)
        p = prev0 != prev0 ? t[0] : prev0;  // NaN: no previous time yet, dt 0 (hw5_2.py:401, 407)
    else
        p = t[i - 1];
    const double d = t[i] - p;
    const uint8_t e = et_in ? et_in[i] : uint8_t(KF_EVENT_IMU);
    dt[i] = d;
    if (et_out) et_out[i] = (rule != 2 && d < 0) ? uint8_t(KF_EVENT_NONE) : e;
}

__global__ __launch_bounds__(kIngBlock) void euler_kernel(int64_t n, const double* q, int64_t ld, double* out) {
    const int64_t i = int64_t(blockIdx.x) * kIngBlock + threadIdx.x;
    if (i >= n) return;
    quat_to_euler(q[i], q[ld + i], q[2 * ld + i], q[3 * ld + i], out[i], out[n + i], out[2 * n + i]);
}

// kf_events_select in two passes over blocks of consecutive events (at most kSelBlocks blocks;
// a block walks its range in tiles of kIngBlock x kSelItems events):
//   select_count_kernel   each block's number of kept events -> counts[b];
//   select_gather_kernel  each block sums the counts of the blocks before it (its output
//                         offset), ranks its tiles' kept events with a block scan and writes their
//                         time and position; the payload rows of a tile are then copied one
//                         output double per thread (contiguous stores, loads along the kept rows).
// The last block writes the total.  Keeps stream order, so the output is DeviceSelect's.
constexpr int kSelItems = 2;
constexpr int kSelTile = kIngBlock * kSelItems;
constexpr int kSelBlocks = 2048;

__global__ __launch_bounds__(kIngBlock) void select_count_kernel(int64_t n, int64_t per_block, const uint8_t* etype,
                                                                  uint8_t type, int32_t* counts) {
    using Reduce = hipcub::BlockReduce<int, kIngBlock>;
    __shared__ typename Reduce::TempStorage tmp;
    const int64_t lo = int64_t(blockIdx.x) * per_block;
    const int64_t hi = lo + per_block < n ? lo + per_block : n;
    int c = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kIngBlock) c += etype[i] == type;
    c = Reduce(tmp).Sum(c);
    if (threadIdx.x == 0) counts[blockIdx.x] = c;
}

__global__ __launch_bounds__(kIngBlock) void select_gather_kernel(int64_t n, int64_t per_block, const uint8_t* etype,
                                                                   uint8_t type, const int32_t* counts, const double* t,
                                                                   const double* payload, double* t_out,
                                                                   double* payload_out, int32_t* src_out,
                                                                   int32_t* n_kept) {
    using Reduce = hipcub::BlockReduce<int, kIngBlock>;
    using Scan = hipcub::BlockScan<int, kIngBlock>;
    __shared__ union {
        typename Reduce::TempStorage red;
        typename Scan::TempStorage scan;
    } tmp;
    __shared__ int32_t rows[kSelTile];
    __shared__ int tile_kept;
    const int tid = int(threadIdx.x);
    int before = 0;
    for (int b = tid; b < int(blockIdx.x); b += kIngBlock) before += counts[b];
    int64_t base = Reduce(tmp.red).Sum(before);
    __shared__ int64_t base_sh;
    if (tid == 0) base_sh = base;
    __syncthreads();
    base = base_sh;
    const int64_t lo = int64_t(blockIdx.x) * per_block;
    const int64_t hi = lo + per_block < n ? lo + per_block : n;
    for (int64_t t0 = lo; t0 < hi; t0 += kSelTile) {
        // thread tid ranks events t0 + tid * kSelItems + 0 .. kSelItems - 1
        const int64_t e0 = t0 + int64_t(tid) * kSelItems;
        bool keep[kSelItems];
        int mine = 0;
#pragma unroll
        for (int k = 0; k < kSelItems; ++k) {
            keep[k] = e0 + k < hi && etype[e0 + k] == type;
            mine += keep[k];
        }
        int off, total;
        __syncthreads();  // tmp and rows are free again
        Scan(tmp.scan).ExclusiveSum(mine, off, total);
#pragma unroll
        for (int k = 0; k < kSelItems; ++k)
            if (keep[k]) {
                const int64_t o = base + off;
                rows[off] = int32_t(e0 + k);
                if (t_out) t_out[o] = t[e0 + k];
                if (src_out) src_out[o] = int32_t(e0 + k);
                ++off;
            }
        if (tid == 0) tile_kept = total;
        __syncthreads();
        const int kept = tile_kept;
        if (payload_out)
            for (int q0 = tid; q0 < 9 * kept; q0 += 4 * kIngBlock) {  // four loads in flight
                double v[4];
                int64_t dst[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int q = q0 + u * kIngBlock;
                    const int qc = q < 9 * kept ? q : 9 * kept - 1;  // past the tile: reload its last value
                    const int j = qc / 9;
                    v[u] = payload[int64_t(rows[j]) * 9 + (qc - 9 * j)];
                    dst[u] = q < 9 * kept ? (base + j) * 9 + (qc - 9 * j) : -1;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (dst[u] >= 0) payload_out[dst[u]] = v[u];
            }
        base += kept;
    }
    if (blockIdx.x == gridDim.x - 1 && tid == 0) {
        *n_kept = int32_t(base);  // mapped host memory
        __threadfence_system();
    }
}

struct MaxOp {
    __device__ __forceinline__ double operator()(double a, double b) const { return b > a ? b : a; }
};

unsigned grid(int64_t n) { return static_cast<unsigned>((n + kIngBlock - 1) / kIngBlock); }

}  // namespace
}  // namespace kfmi

using namespace kfmi;

namespace {
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

int hip_err(hipError_t e, const char* what) {
    return set_error(KF_EHIP, "%s: %s (%d)", what, hipGetErrorString(e), static_cast<int>(e));
}

// kf_events_select's scratch, one slot per device (each with its own lock, held through the
// call: the next call on that device reuses the buffers; hipMalloc / hipFree per call would
// synchronise the device)
constexpr int kSelMaxDevices = 64;
struct SelectSlot {
    std::mutex mu;
    int32_t* counts = nullptr;    // the count pass's [kSelBlocks] block counts
    int32_t* kept = nullptr;      // mapped, coherent host int the gather pass fills
    int32_t* kept_dev = nullptr;  // its device address
};
SelectSlot& select_slot(int dev) {
    static SelectSlot slots[kSelMaxDevices];
    return slots[dev];
}
}  // namespace

#define KF_TRY(expr, what)                          \
    do {                                            \
        hipError_t e_ = (expr);                     \
        if (e_ != hipSuccess) return hip_err(e_, what); \
    } while (0)

extern "C" {

int kf_ingest(const double* gps, int64_t n_gps, int64_t ld_gps, const double* imu, int64_t n_imu, int64_t ld_imu,
              int flags, const double* bias, uint8_t* etype, double* t, double* payload, int32_t* src,
              int8_t* zone_number, char* zone_letter, kf_ingest_info* info, void* stream) {
    if (n_gps < 0 || n_imu < 0) return set_error(KF_EINVAL, "kf_ingest: negative row count");
    if ((n_gps && (!gps || ld_gps < n_gps)) || (n_imu && (!imu || ld_imu < n_imu)))
        return set_error(KF_EINVAL, "kf_ingest: null column array or leading dimension below the row count");
    if (n_gps + n_imu >= (int64_t(1) << 31)) return set_error(KF_EINVAL, "kf_ingest: more than 2^31 rows");
    if (!etype || !t || !payload || !info) return set_error(KF_EINVAL, "kf_ingest: null output");
    if (flags & ~KF_INGEST_GPS_ALTITUDE) return set_error(KF_EINVAL, "kf_ingest: unknown flags 0x%x", flags);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t nk = n_gps + n_imu;

    // one workspace: east, north, keys, keys_sorted (8 B); keep, pos, vals, vals_sorted (4 B);
    // zone, letter (1 B); first[2], bias[6]; then hipCUB temporaries
    size_t sort_tmp = 0, scan_tmp = 0;
    KF_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (double*)nullptr, (double*)nullptr, (int32_t*)nullptr,
                                              (int32_t*)nullptr, static_cast<int>(nk), 0, 64, st),
           "kf_ingest sort sizing");
    KF_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (int32_t*)nullptr, (int32_t*)nullptr,
                                            static_cast<int>(n_gps), st),
           "kf_ingest scan sizing");
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t g8 = al(8 * std::max<int64_t>(n_gps, 1)), k8 = al(8 * std::max<int64_t>(nk, 1));
    const size_t g4 = al(4 * std::max<int64_t>(n_gps, 1)), k4 = al(4 * std::max<int64_t>(nk, 1));
    const size_t g1 = al(std::max<int64_t>(n_gps, 1));
    const size_t bytes = 2 * g8 + 2 * k8 + 2 * g4 + 2 * k4 + 2 * g1 + al(8 * 8) + al(std::max(sort_tmp, scan_tmp));
    DevBuf ws;
    KF_TRY(hipMalloc(&ws.p, bytes), "kf_ingest workspace");
    char* w = static_cast<char*>(ws.p);
    IngestArgs a{};
    a.n_gps = n_gps;
    a.n_imu = n_imu;
    a.ld_gps = ld_gps;
    a.ld_imu = ld_imu;
    a.gps = gps;
    a.imu = imu;
    a.check_alt = (flags & KF_INGEST_GPS_ALTITUDE) ? 1 : 0;
    a.east = reinterpret_cast<double*>(w); w += g8;
    a.north = reinterpret_cast<double*>(w); w += g8;
    a.keys = reinterpret_cast<double*>(w); w += k8;
    double* keys_sorted = reinterpret_cast<double*>(w); w += k8;
    a.keep = reinterpret_cast<int32_t*>(w); w += g4;
    int32_t* pos = reinterpret_cast<int32_t*>(w); w += g4;
    a.vals = reinterpret_cast<int32_t*>(w); w += k4;
    int32_t* vals_sorted = reinterpret_cast<int32_t*>(w); w += k4;
    a.zone = reinterpret_cast<int8_t*>(w); w += g1;
    a.letter = w; w += g1;
    a.first = reinterpret_cast<unsigned long long*>(w);
    a.bias = reinterpret_cast<double*>(w + 16);
    w += al(8 * 8);
    void* tmp = w;

    const unsigned long long none[2] = {~0ull, ~0ull};
    KF_TRY(hipMemcpyAsync(a.first, none, sizeof none, hipMemcpyHostToDevice, st), "kf_ingest init");
    if (n_gps) {
        fix_kernel<<<grid(n_gps), kIngBlock, 0, st>>>(a);
        KF_TRY(hipGetLastError(), "kf_ingest fix_kernel");
    }
    if (n_imu) {
        imu_keys_kernel<<<grid(n_imu), kIngBlock, 0, st>>>(a);
        KF_TRY(hipGetLastError(), "kf_ingest imu_keys_kernel");
    }
    if (bias) {  // caller's biases (unbias_imu_data takes them as arguments, kf_workers.py:349)
        KF_TRY(hipMemcpyAsync(a.bias, bias, 6 * sizeof(double), hipMemcpyHostToDevice, st), "kf_ingest bias");
    } else {
        bias_kernel<<<1, 64, 0, st>>>(a);
        KF_TRY(hipGetLastError(), "kf_ingest bias_kernel");
    }
    if (n_gps) {
        size_t tb = scan_tmp;
        KF_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, a.keep, pos, static_cast<int>(n_gps), st), "kf_ingest scan");
    }
    if (nk) {
        size_t tb = sort_tmp;
        KF_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, a.keys, keys_sorted, a.vals, vals_sorted,
                                                  static_cast<int>(nk), 0, 64, st),
               "kf_ingest sort");
    }
    unsigned long long first[2];
    double bias_out[6];
    int32_t last_pos = 0, last_keep = 0;
    KF_TRY(hipMemcpyAsync(first, a.first, sizeof first, hipMemcpyDeviceToHost, st), "kf_ingest readback");
    KF_TRY(hipMemcpyAsync(bias_out, a.bias, sizeof bias_out, hipMemcpyDeviceToHost, st), "kf_ingest readback");
    if (n_gps) {
        KF_TRY(hipMemcpyAsync(&last_pos, pos + n_gps - 1, 4, hipMemcpyDeviceToHost, st), "kf_ingest readback");
        KF_TRY(hipMemcpyAsync(&last_keep, a.keep + n_gps - 1, 4, hipMemcpyDeviceToHost, st), "kf_ingest readback");
    }
    KF_TRY(hipStreamSynchronize(st), "kf_ingest sync");
    if (first[0] == ~0ull)
        return set_error(KF_EINVAL, "kf_ingest: no GPS row has a latitude (compute_imu_biases finds no "
                                    "first valid index, kf_workers.py:336-338)");
    const int64_t n_fix = last_pos + last_keep;
    GatherArgs g{};
    g.n_events = n_fix + n_imu;
    g.n_gps = n_gps;
    g.ld_gps = ld_gps;
    g.ld_imu = ld_imu;
    g.gps = gps;
    g.imu = imu;
    g.vals = vals_sorted;
    g.pos = pos;
    g.east = a.east;
    g.north = a.north;
    g.zone = a.zone;
    g.letter = a.letter;
    g.first = a.first;
    g.bias = a.bias;
    g.etype = etype;
    g.t = t;
    g.payload = payload;
    g.src = src;
    g.zone_out = zone_number;
    g.letter_out = zone_letter;
    if (g.n_events) {
        gather_kernel<<<grid(g.n_events), kIngBlock, 0, st>>>(g);
        KF_TRY(hipGetLastError(), "kf_ingest gather_kernel");
    }
    double origin[2] = {0.0, 0.0};
    if (n_fix) {
        KF_TRY(hipMemcpyAsync(&origin[0], a.east + first[1], 8, hipMemcpyDeviceToHost, st), "kf_ingest readback");
        KF_TRY(hipMemcpyAsync(&origin[1], a.north + first[1], 8, hipMemcpyDeviceToHost, st), "kf_ingest readback");
    }
    KF_TRY(hipStreamSynchronize(st), "kf_ingest sync");
    info->n_events = g.n_events;
    info->n_fixes = n_fix;
    info->n_imu = n_imu;
    info->first_valid_index = static_cast<int64_t>(first[0]);
    info->origin_row = n_fix ? static_cast<int64_t>(first[1]) : -1;
    for (int k = 0; k < 3; ++k) {
        info->gyro_bias[k] = bias_out[k];
        info->accel_bias[k] = bias_out[3 + k];
    }
    info->utm_origin[0] = origin[0];
    info->utm_origin[1] = origin[1];
    return KF_OK;
}

int kf_quat_to_euler(int64_t n, const double* q, int64_t ld, double* out, void* stream) {
    if (n < 0 || (n && (!q || !out || ld < n))) return set_error(KF_EINVAL, "kf_quat_to_euler: bad arguments");
    if (n == 0) return KF_OK;
    euler_kernel<<<grid(n), kIngBlock, 0, static_cast<hipStream_t>(stream)>>>(n, q, ld, out);
    KF_TRY(hipGetLastError(), "kf_quat_to_euler");
    return KF_OK;
}

int kf_events_dt(int64_t n, const double* t, const uint8_t* etype_in, double prev0, int rule, double* dt,
                 uint8_t* etype_out, void* stream) {
    if (n < 0) return set_error(KF_EINVAL, "kf_events_dt: n = %lld", (long long)n);
    if (rule < KF_DT_FULL || rule > KF_DT_RAW) return set_error(KF_EINVAL, "kf_events_dt: unknown rule %d", rule);
    if (rule == KF_DT_MONOTONE && prev0 != prev0)
        return set_error(KF_EINVAL, "kf_events_dt: KF_DT_MONOTONE needs a previous time (prev0 is NaN)");
    if (n == 0) return KF_OK;
    if (!t || !dt) return set_error(KF_EINVAL, "kf_events_dt: null t/dt");
    if (n >= (int64_t(1) << 31)) return set_error(KF_EINVAL, "kf_events_dt: more than 2^31 events");
    hipStream_t st = static_cast<hipStream_t>(stream);
    DevBuf ws;
    const double* prev = nullptr;
    if (rule == KF_DT_MONOTONE) {
        size_t tmp = 0;
        KF_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, tmp, t, (double*)nullptr, MaxOp{}, prev0, static_cast<int>(n), st),
               "kf_events_dt scan sizing");
        const size_t pb = (8 * size_t(n) + 255) & ~size_t(255);
        KF_TRY(hipMalloc(&ws.p, pb + tmp), "kf_events_dt workspace");
        double* pm = static_cast<double*>(ws.p);
        KF_TRY(hipcub::DeviceScan::ExclusiveScan(static_cast<char*>(ws.p) + pb, tmp, t, pm, MaxOp{}, prev0,
                                                 static_cast<int>(n), st),
               "kf_events_dt scan");
        prev = pm;
    }
    dt_kernel<<<grid(n), kIngBlock, 0, st>>>(n, t, prev, etype_in, prev0, rule, dt, etype_out);
    KF_TRY(hipGetLastError(), "kf_events_dt");
    if (ws.p) KF_TRY(hipStreamSynchronize(st), "kf_events_dt sync");  // before the workspace goes
    return KF_OK;
}

int kf_events_select(int64_t n, const uint8_t* etype, const double* t, const double* payload, int keep_type,
                     double* t_out, double* payload_out, int32_t* src_out, int64_t* n_kept, void* stream) {
    if (n < 0 || !n_kept) return set_error(KF_EINVAL, "kf_events_select: n = %lld, n_kept %p", (long long)n,
                                           static_cast<void*>(n_kept));
    if (keep_type < 0 || keep_type > 255) return set_error(KF_EINVAL, "kf_events_select: event type %d", keep_type);
    if (n >= (int64_t(1) << 31)) return set_error(KF_EINVAL, "kf_events_select: more than 2^31 events");
    *n_kept = 0;
    if (n == 0) return KF_OK;
    if (!etype || (t_out && !t) || (payload_out && !payload))
        return set_error(KF_EINVAL, "kf_events_select: null etype, or an output without its input");
    hipStream_t st = static_cast<hipStream_t>(stream);
    // the call synchronises the stream to return the count, so it cannot be captured: refuse
    // before anything is queued into the caller's capture (kf_search_combos does the same)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    KF_TRY(hipStreamIsCapturing(st, &cap), "kf_events_select capture status");
    if (cap != hipStreamCaptureStatusNone)
        return set_error(KF_EINVAL, "kf_events_select: not capturable (the kept count returns to the host in the call)");
    // the scratch belongs to the current device: the stream must be one of its streams
    int dev = 0;
    KF_TRY(hipGetDevice(&dev), "kf_events_select device");
    if (st) {
        int sdev = dev;
        KF_TRY(hipStreamGetDevice(st, &sdev), "kf_events_select stream device");
        if (sdev != dev)
            return set_error(KF_EINVAL, "kf_events_select: the stream is on device %d, the current device is %d",
                             sdev, dev);
    }
    if (dev < 0 || dev >= kSelMaxDevices) return set_error(KF_EINVAL, "kf_events_select: device %d", dev);
    SelectSlot& sc = select_slot(dev);
    std::lock_guard<std::mutex> lock(sc.mu);  // held to the end: the scratch is reused by the next call
    if (!sc.counts) {
        void *c = nullptr, *p = nullptr, *pd = nullptr;
        hipError_t e = hipMalloc(&c, sizeof(int32_t) * kSelBlocks);
        if (e == hipSuccess) e = hipHostMalloc(&p, sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer(&pd, p, 0);
        if (e != hipSuccess) {
            if (c) (void)hipFree(c);
            if (p) (void)hipHostFree(p);
            return set_error(KF_EHIP, "kf_events_select workspace: %s", hipGetErrorString(e));
        }
        sc.counts = static_cast<int32_t*>(c);
        sc.kept = static_cast<int32_t*>(p);
        sc.kept_dev = static_cast<int32_t*>(pd);
    }
    // blocks of a multiple of the tile, at most kSelBlocks of them, none empty
    const int64_t tiles = (n + kSelTile - 1) / kSelTile;
    const int64_t per_block = ((tiles + kSelBlocks - 1) / kSelBlocks) * kSelTile;
    const unsigned blocks = static_cast<unsigned>((n + per_block - 1) / per_block);
    const uint8_t ty = static_cast<uint8_t>(keep_type);
    *sc.kept = -1;
    select_count_kernel<<<blocks, kIngBlock, 0, st>>>(n, per_block, etype, ty, sc.counts);
    KF_TRY(hipGetLastError(), "kf_events_select count");
    select_gather_kernel<<<blocks, kIngBlock, 0, st>>>(n, per_block, etype, ty, sc.counts, t, payload, t_out,
                                                       payload_out, src_out, sc.kept_dev);
    KF_TRY(hipGetLastError(), "kf_events_select gather");
    KF_TRY(hipStreamSynchronize(st), "kf_events_select sync");
    const int32_t k = *sc.kept;
    if (k < 0 || k > n) return set_error(KF_EHIP, "kf_events_select: no count came back (%d)", k);
    *n_kept = k;
    return KF_OK;
}

}  // extern "C"
