/* CPU restatement of the reference's filter step in C — TEST INFRASTRUCTURE ONLY.
 *
 * The checker / CPU baseline, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it (via ctypes).  It restates, in the reference's operation
 * order and with dense matrices, what oracle/ref_kf.py restates in NumPy:
 *
 *   x = F x (+ G u)                 kf_workers.py:690
 *   P = (F P) F^T + Q               predict_covariance, kf_workers.py:546-549
 *   K = (P H^T) inv((H P) H^T + R)  calculate_kalman_gain, kf_workers.py:616-621
 *   y = Z - H x ; x = x + K y        kf_workers.py:709-710
 *   P = (I - K H) P                  kf_workers.py:711
 *   slogdet(P)                       kf_workers.py:716-717
 *
 * for the BASELINE 4/2 and 6/3 constant-velocity restrictions and for the
 * 15-state model's GPS / IMU-pseudo-measurement events (kf_workers.py:493-614, 698-706).
 * inv() and slogdet() are LU with partial pivoting, as LAPACK's dgesv/dgetrf do.  OpenMP over
 * filters (the reference itself is one filter per Python process).
 * Pinned against oracle/ref_kf.py in tests/test_oracle.py (<= 1e-10 relative).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define NMAX 15

/* C = A B, A m x k, B k x n, row-major, straightforward dot products */
static void matmul(int m, int k, int n, const double* A, const double* B, double* C) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += A[i * k + l] * B[l * n + j];
            C[i * n + j] = s;
        }
}

/* C = A B^T */
static void matmul_bt(int m, int k, int n, const double* A, const double* B, double* C) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += A[i * k + l] * B[j * k + l];
            C[i * n + j] = s;
        }
}

/* LU with partial pivoting in place (n x n); returns 0 if singular.  piv[i] = row swapped in. */
static int lu(int n, double* A, int* piv, int* nswap) {
    *nswap = 0;
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = fabs(A[k * n + k]);
        for (int i = k + 1; i < n; ++i)
            if (fabs(A[i * n + k]) > best) {
                best = fabs(A[i * n + k]);
                p = i;
            }
        piv[k] = p;
        if (best == 0.0) return 0;
        if (p != k) {
            ++*nswap;
            for (int j = 0; j < n; ++j) {
                double t = A[k * n + j];
                A[k * n + j] = A[p * n + j];
                A[p * n + j] = t;
            }
        }
        for (int i = k + 1; i < n; ++i) {
            A[i * n + k] /= A[k * n + k];
            const double l = A[i * n + k];
            for (int j = k + 1; j < n; ++j) A[i * n + j] -= l * A[k * n + j];
        }
    }
    return 1;
}

/* inverse via LU (columns of the identity solved one by one) */
static int inv(int n, const double* A, double* Ai) {
    double LU[NMAX * NMAX];
    int piv[NMAX], ns;
    memcpy(LU, A, sizeof(double) * n * n);
    if (!lu(n, LU, piv, &ns)) return 0;
    for (int c = 0; c < n; ++c) {
        double b[NMAX];
        for (int i = 0; i < n; ++i) b[i] = (i == c) ? 1.0 : 0.0;
        for (int k = 0; k < n; ++k) {
            const int p = piv[k];
            if (p != k) {
                double t = b[k];
                b[k] = b[p];
                b[p] = t;
            }
        }
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < i; ++k) b[i] -= LU[i * n + k] * b[k];
        for (int i = n - 1; i >= 0; --i) {
            for (int k = i + 1; k < n; ++k) b[i] -= LU[i * n + k] * b[k];
            b[i] /= LU[i * n + i];
        }
        for (int i = 0; i < n; ++i) Ai[i * n + c] = b[i];
    }
    return 1;
}

/* log |det A| (NaN if singular or the sign is negative, i.e. not a covariance) */
static double logdet(int n, const double* A) {
    double LU[NMAX * NMAX];
    int piv[NMAX], ns;
    memcpy(LU, A, sizeof(double) * n * n);
    if (!lu(n, LU, piv, &ns)) return NAN;
    double s = 0.0;
    int neg = ns & 1;
    for (int i = 0; i < n; ++i) {
        const double d = LU[i * n + i];
        if (d < 0) neg ^= 1;
        s += log(fabs(d));
    }
    return neg ? NAN : s;
}

/* predict x = F x + G u, P = (F P) F^T + Q */
static void predict(int n, const double* F, const double* Q, const double* Gu, double* x, double* P) {
    double xn[NMAX], FP[NMAX * NMAX];
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += F[i * n + j] * x[j];
        xn[i] = s + (Gu ? Gu[i] : 0.0);
    }
    memcpy(x, xn, sizeof(double) * n);
    matmul(n, n, n, F, P, FP);
    matmul_bt(n, n, n, FP, F, P);
    for (int i = 0; i < n * n; ++i) P[i] += Q[i];
}

/* update with H (m x n), R (m x m), Z (m): K = (P H^T) inv((H P) H^T + R); x += K (Z - H x);
 * P = (I - K H) P.  Returns 0 if S is singular. */
static int update(int n, int m, const double* H, const double* R, const double* Z, double* x, double* P) {
    double PHt[NMAX * NMAX], HP[NMAX * NMAX], S[NMAX * NMAX], Si[NMAX * NMAX], K[NMAX * NMAX];
    matmul_bt(n, n, m, P, H, PHt);
    matmul(m, n, n, H, P, HP);
    matmul_bt(m, n, m, HP, H, S);
    for (int i = 0; i < m * m; ++i) S[i] += R[i];
    if (!inv(m, S, Si)) return 0;
    matmul(n, m, m, PHt, Si, K);
    double y[NMAX];
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += H[i * n + j] * x[j];
        y[i] = Z[i] - s;
    }
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int j = 0; j < m; ++j) s += K[i * m + j] * y[j];
        x[i] += s;
    }
    double IKH[NMAX * NMAX], Pn[NMAX * NMAX];
    matmul(n, m, n, K, H, IKH);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) IKH[i * n + j] = (i == j ? 1.0 : 0.0) - IKH[i * n + j];
    matmul(n, n, n, IKH, P, Pn);
    memcpy(P, Pn, sizeof(double) * n * n);
    return 1;
}

/* BASELINE constant-velocity filters (d = 2: 4/2, d = 3: 6/3), one per column of the SoA
 * streams: u [T][d][B], z [T/k][d][B], x0 [n][B]; traj [T][n][B] and logdet [T][B] optional.
 * Step t updates when (t+1) % k == 0 (oracle/ref_kf.is_update_step).  Filters [f0, f1). */
static void cv_model(int d, double dt, double q_pos, double q_vel, double* F, double* Q) {
    const int n = 2 * d;
    memset(F, 0, sizeof(double) * n * n);
    memset(Q, 0, sizeof(double) * n * n);
    for (int i = 0; i < n; ++i) F[i * n + i] = 1.0;
    for (int i = 0; i < d; ++i) {
        F[i * n + d + i] = dt;
        Q[i * n + i] = q_pos * dt;
        Q[(d + i) * n + d + i] = q_vel * dt;
    }
}

void cpu_cv_run(int d, int64_t B, int T, double dt0, const double* dt_steps, int k, const double* u, const double* z,
                const double* x0, const double* P0, double q_pos, double q_vel, double r_gps, const double* R_full,
                double* traj, double* logdet_out, double* x_out, double* P_out, int64_t f0, int64_t f1, int nthreads) {
    /* R_full: d x d row-major measurement noise, or NULL for r_gps I (kf_workers.py:581-585) */
    const int n = 2 * d;
    double F0[NMAX * NMAX], Q0[NMAX * NMAX], H[NMAX * NMAX] = {0}, R[NMAX * NMAX] = {0};
    cv_model(d, dt0, q_pos, q_vel, F0, Q0);
    for (int i = 0; i < d; ++i) {
        H[i * n + i] = 1.0;
        R[i * d + i] = r_gps;
    }
    if (R_full) memcpy(R, R_full, sizeof(double) * d * d);
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t f = f0; f < f1; ++f) {
        double x[NMAX], P[NMAX * NMAX], Fs[NMAX * NMAX], Qs[NMAX * NMAX];
        for (int i = 0; i < n; ++i) x[i] = x0[i * B + f];
        memcpy(P, P0, sizeof(double) * n * n);
        for (int t = 0; t < T; ++t) {
            const double dt = dt_steps ? dt_steps[t] : dt0;
            const double* F = F0;
            const double* Q = Q0;
            if (dt_steps) {
                cv_model(d, dt, q_pos, q_vel, Fs, Qs);
                F = Fs;
                Q = Qs;
            }
            double Gu[NMAX];
            for (int i = 0; i < d; ++i) {
                const double a = u[((int64_t)t * d + i) * B + f];
                Gu[i] = 0.5 * dt * dt * a;
                Gu[d + i] = dt * a;
            }
            predict(n, F, Q, Gu, x, P);
            if ((t + 1) % k == 0) {
                double Z[NMAX];
                const int s = (t + 1) / k - 1;
                for (int i = 0; i < d; ++i) Z[i] = z[((int64_t)s * d + i) * B + f];
                update(n, d, H, R, Z, x, P);
            }
            if (traj)
                for (int i = 0; i < n; ++i) traj[((int64_t)t * n + i) * B + f] = x[i];
            if (logdet_out) logdet_out[(int64_t)t * B + f] = logdet(n, P);
        }
        if (x_out)
            for (int i = 0; i < n; ++i) x_out[i * B + f] = x[i];
        if (P_out) memcpy(P_out + f * n * n, P, sizeof(double) * n * n);
    }
}

/* The reference's 15-state model (kf_workers.py:493-614): F(dt), Q(dt), the GPS fix update and
 * the IMU pseudo-measurement update built from the predicted state (kf_workers.py:698-706). */
static void F15(double dt, double* F) {
    memset(F, 0, sizeof(double) * 225);
    for (int i = 0; i < 15; ++i) F[i * 15 + i] = 1.0;
    for (int i = 0; i < 3; ++i) {
        F[i * 15 + 6 + i] = dt;
        F[i * 15 + 12 + i] = 0.5 * dt * dt;
        F[(3 + i) * 15 + 9 + i] = dt;
        F[(6 + i) * 15 + 12 + i] = dt;
    }
}

static void Q15(double dt, double* Q) {
    static const double q[5] = {5.0, 0.05, 1.0, 0.1, 2.0};
    memset(Q, 0, sizeof(double) * 225);
    for (int g = 0; g < 5; ++g)
        for (int i = 0; i < 3; ++i) Q[(3 * g + i) * 15 + 3 * g + i] = q[g] * dt;
}

/* events: etype [T][B] (0 GPS, 1 IMU, 2 predict only, 255 none), dt [T][B], payload [T][9][B];
 * x0 [15][B]; P0 15x15 (shared); traj [T][6][B], logdet [T][B] optional.  Filters [f0, f1). */
void cpu_ref15_events(int64_t B, int T, const uint8_t* etype, const double* dt, const double* payload,
                      const double* x0, const double* P0, double* traj, double* logdet_out, int64_t f0, int64_t f1,
                      int nthreads) {
    static const double rimu[5] = {50.0, 0.05, 10.0, 0.1, 100.0};
    double Hg[3 * 15] = {0}, Rg[9] = {0}, Hi[225] = {0}, Ri[225] = {0};
    for (int i = 0; i < 3; ++i) {
        Hg[i * 15 + i] = 1.0;
        Rg[i * 3 + i] = 3.0;
    }
    for (int i = 0; i < 15; ++i) {
        Hi[i * 15 + i] = 1.0;
        Ri[i * 15 + i] = rimu[i / 3];
    }
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t f = f0; f < f1; ++f) {
        double x[15], P[225], F[225], Q[225];
        for (int i = 0; i < 15; ++i) x[i] = x0[i * B + f];
        memcpy(P, P0, sizeof(P));
        for (int t = 0; t < T; ++t) {
            const int ty = etype[(int64_t)t * B + f];
            const double h = dt[(int64_t)t * B + f];
            const double* p = payload + (int64_t)t * 9 * B + f;
            if (ty != 255) {
                F15(h, F);
                Q15(h, Q);
                predict(15, F, Q, NULL, x, P);
                if (ty == 0) {
                    const double Z[3] = {p[0], p[B], p[2 * B]};
                    update(15, 3, Hg, Rg, Z, x, P);
                } else if (ty == 1) {
                    double Z[15];
                    for (int i = 0; i < 3; ++i) {
                        const double a = p[(6 + i) * B];
                        const double V = x[6 + i] + a * h;
                        Z[i] = x[i] + V * h;
                        Z[3 + i] = p[i * B];
                        Z[6 + i] = V;
                        Z[9 + i] = p[(3 + i) * B];
                        Z[12 + i] = a;
                    }
                    update(15, 15, Hi, Ri, Z, x, P);
                }
            }
            if (traj)
                for (int i = 0; i < 6; ++i) traj[((int64_t)t * 6 + i) * B + f] = x[i];
            if (logdet_out) logdet_out[(int64_t)t * B + f] = logdet(15, P);
        }
    }
}

/* Scheduler.gain (kf_workers.py:174-185) with cov_matrix(S = [1]) (kf_workers.py:112-147, the
 * device='cpu' branch): trace(Sigma - ((Sigma h^T) inv(r + h (Sigma h^T)) h) Sigma) for the
 * first measurement row h of the sensor's H (a unit row: H_gps and H_imu both start with e_0)
 * and its noise r = R[0][0].  The trace is summed in index order (the reference's np.trace may
 * pair terms; the gains only rank candidates, they are not outputs). */
static double sched_gain(const double* P, double r) {
    double h[15] = {0}, Ph[15], hPh, Si, KhP[225];
    h[0] = 1.0;
    matmul_bt(15, 15, 1, P, h, Ph);            /* Sigma h^T */
    matmul(1, 15, 1, h, Ph, &hPh);             /* h (Sigma h^T) */
    const double S = r + hPh;
    if (!inv(1, &S, &Si)) return NAN;
    double K[15], Kh[225];
    for (int i = 0; i < 15; ++i) K[i] = Ph[i] * Si;
    matmul(15, 1, 15, K, h, Kh);
    matmul(15, 15, 15, Kh, P, KhP);
    double tr = 0.0;
    for (int i = 0; i < 15; ++i) tr += P[i * 15 + i] - KhP[i * 15 + i];
    return tr;
}

/* run_kalman_filter_scheduled, greedy arm, warm start (kf_workers.py:826-957): per filter, the
 * events of column f of t [T][B], etype [T][B] (0 GPS, 1 IMU), payload [T][9][B] follow the
 * warm-start event (time prev0[f], state x0[0:6][f] (NULL: zeros), covariance P0).  An event
 * within 1/freq[f] of the last processed time is queued; the next one past the window picks
 * the first queued candidate of largest gain (Scheduler.greedy_schedule :195-213; an empty queue
 * takes the triggering event itself, otherwise it is dropped), then one predict over the
 * accumulated dt and one update on the pick.  Outputs per pick j < n_sel[f]: sel_time [T][B],
 * traj [T][6][B] (x[0:6]), logdet [T][B].  Filters [f0, f1). */
void cpu_ref15_sched(int64_t B, int T, const double* t, const uint8_t* etype, const double* payload,
                     const double* prev0, const double* freq, const double* x0, const double* P0, double* sel_time,
                     double* traj, double* logdet_out, int32_t* n_sel, int64_t f0, int64_t f1, int nthreads) {
    static const double rimu[5] = {50.0, 0.05, 10.0, 0.1, 100.0};
    double Hg[3 * 15] = {0}, Rg[9] = {0}, Hi[225] = {0}, Ri[225] = {0};
    for (int i = 0; i < 3; ++i) {
        Hg[i * 15 + i] = 1.0;
        Rg[i * 3 + i] = 3.0;
    }
    for (int i = 0; i < 15; ++i) {
        Hi[i * 15 + i] = 1.0;
        Ri[i * 15 + i] = rimu[i / 3];
    }
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 16)
    for (int64_t f = f0; f < f1; ++f) {
        double x[15] = {0}, P[225], F[225], Q[225];
        if (x0)
            for (int i = 0; i < 6; ++i) x[i] = x0[i * B + f];
        memcpy(P, P0, sizeof(P));
        double prev = prev0[f];
        const double win = 1.0 / freq[f];
        int q0 = 0, nq = 0, ns = 0;              /* the queue is the events [q0, q0 + nq) */
        for (int i = 0; i < T; ++i) {
            const double ti = t[(int64_t)i * B + f];
            if (ti - prev < win) {
                if (nq == 0) q0 = i;
                ++nq;
                continue;
            }
            if (nq == 0) {
                q0 = i;
                nq = 1;
            }
            int sel = -1;
            double best = -INFINITY;
            for (int q = q0; q < q0 + nq; ++q) {
                const int ty = etype[(int64_t)q * B + f];
                const double g = sched_gain(P, ty == 0 ? Rg[0] : Ri[0]);
                if (g > best) {
                    best = g;
                    sel = q;
                }
            }
            if (sel < 0) sel = q0;
            nq = 0;
            const double st = t[(int64_t)sel * B + f];
            const double h = st - prev;
            const int ty = etype[(int64_t)sel * B + f];
            const double* p = payload + (int64_t)sel * 9 * B + f;
            F15(h, F);
            Q15(h, Q);
            predict(15, F, Q, NULL, x, P);
            if (ty == 0) {
                const double Z[3] = {p[0], p[B], p[2 * B]};
                update(15, 3, Hg, Rg, Z, x, P);
            } else {
                double Z[15];
                for (int c = 0; c < 3; ++c) {
                    const double a = p[(6 + c) * B];
                    const double V = x[6 + c] + a * h;
                    Z[c] = x[c] + V * h;
                    Z[3 + c] = p[c * B];
                    Z[6 + c] = V;
                    Z[9 + c] = p[(3 + c) * B];
                    Z[12 + c] = a;
                }
                update(15, 15, Hi, Ri, Z, x, P);
            }
            if (sel_time) sel_time[(int64_t)ns * B + f] = st;
            if (traj)
                for (int c = 0; c < 6; ++c) traj[((int64_t)ns * 6 + c) * B + f] = x[c];
            if (logdet_out) logdet_out[(int64_t)ns * B + f] = logdet(15, P);
            ++ns;
            prev = st;
        }
        if (n_sel) n_sel[f] = ns;
    }
}

/* hw5_2.py's 8-state planar model [x, y, theta, vx, vy, theta_dot, ax, ay] (hw5_2.py:219-304):
 * F(dt) :219-231, Q(dt) = diag(5, 5, 0.05, 1, 1, 0.1, 2, 2) dt :233-251, a GPS fix updates
 * (x, y) with R = 3 I2 (:258-264, 280-284, 341-349), an IMU sample the whole state with H = I8,
 * R = diag(50, 50, 0.05, 10, 10, 0.1, 100, 100) through the pseudo-measurement built from the
 * predicted state (:352-366). */
static void F8(double dt, double* F) {
    memset(F, 0, sizeof(double) * 64);
    for (int i = 0; i < 8; ++i) F[i * 8 + i] = 1.0;
    F[0 * 8 + 3] = dt;
    F[0 * 8 + 6] = 0.5 * dt * dt;
    F[1 * 8 + 4] = dt;
    F[1 * 8 + 7] = 0.5 * dt * dt;
    F[2 * 8 + 5] = dt;
    F[3 * 8 + 6] = dt;
    F[4 * 8 + 7] = dt;
}

/* events as cpu_ref15_events (payload [T][9][B]: GPS e, n, alt; IMU roll, pitch, yaw, wx, wy,
 * wz, ax, ay, az); x0 [8][B]; P0 8x8; traj [T][3][B] (x, y, theta), logdet [T][B] optional. */
void cpu_ref8_events(int64_t B, int T, const uint8_t* etype, const double* dt, const double* payload,
                     const double* x0, const double* P0, double* traj, double* logdet_out, int64_t f0, int64_t f1,
                     int nthreads) {
    static const double q8[8] = {5.0, 5.0, 0.05, 1.0, 1.0, 0.1, 2.0, 2.0};
    static const double r8[8] = {50.0, 50.0, 0.05, 10.0, 10.0, 0.1, 100.0, 100.0};
    double Hg[2 * 8] = {0}, Rg[4] = {0}, Hi[64] = {0}, Ri[64] = {0};
    for (int i = 0; i < 2; ++i) {
        Hg[i * 8 + i] = 1.0;
        Rg[i * 2 + i] = 3.0;
    }
    for (int i = 0; i < 8; ++i) {
        Hi[i * 8 + i] = 1.0;
        Ri[i * 8 + i] = r8[i];
    }
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t f = f0; f < f1; ++f) {
        double x[8], P[64], F[64], Q[64];
        for (int i = 0; i < 8; ++i) x[i] = x0[i * B + f];
        memcpy(P, P0, sizeof(P));
        for (int t = 0; t < T; ++t) {
            const int ty = etype[(int64_t)t * B + f];
            const double h = dt[(int64_t)t * B + f];
            const double* p = payload + (int64_t)t * 9 * B + f;
            if (ty != 255) {
                F8(h, F);
                memset(Q, 0, sizeof(Q));
                for (int i = 0; i < 8; ++i) Q[i * 8 + i] = q8[i] * h;
                predict(8, F, Q, NULL, x, P);
                if (ty == 0) {
                    const double Z[2] = {p[0], p[B]};
                    update(8, 2, Hg, Rg, Z, x, P);
                } else if (ty == 1) {
                    const double ax = p[6 * B], ay = p[7 * B];
                    const double Vx = x[3] + ax * h, Vy = x[4] + ay * h;
                    const double Z[8] = {x[0] + Vx * h, x[1] + Vy * h, p[2 * B], Vx, Vy, p[5 * B], ax, ay};
                    update(8, 8, Hi, Ri, Z, x, P);
                }
            }
            if (traj)
                for (int i = 0; i < 3; ++i) traj[((int64_t)t * 3 + i) * B + f] = x[i];
            if (logdet_out) logdet_out[(int64_t)t * B + f] = logdet(8, P);
        }
    }
}

/* hw5_2.run_dead_reckoning_for_IMU (hw5_2.py:382-436) over one merged stream as kf_ingest lays
 * it out (etype [N] 0 = GPS / 1 = IMU, t [N], payload [N][9] row-major): only the IMU events
 * are filtered (:403-404), dt runs from the previous IMU event with the first at 0 (:401, 407,
 * no dt < 0 guard), x0 = 0, P0 = diag(1000, 1000, 100, 100, 100, 100, 1000, 1000) (:385-395),
 * and each event predicts then applies the H = I8 pseudo-measurement (:410-431).  Writes one
 * (x, y, theta) row per IMU event into traj [K][3] and its log-det into logdet [K] (either may
 * be NULL) and returns K. */
int64_t cpu_ref8_dead_reckoning(int64_t N, const uint8_t* etype, const double* t, const double* payload,
                                double* traj, double* logdet_out) {
    static const double q8[8] = {5.0, 5.0, 0.05, 1.0, 1.0, 0.1, 2.0, 2.0};
    static const double r8[8] = {50.0, 50.0, 0.05, 10.0, 10.0, 0.1, 100.0, 100.0};
    static const double p08[8] = {1000.0, 1000.0, 100.0, 100.0, 100.0, 100.0, 1000.0, 1000.0};
    double Hi[64] = {0}, Ri[64] = {0}, x[8] = {0}, P[64] = {0}, F[64], Q[64];
    for (int i = 0; i < 8; ++i) {
        Hi[i * 8 + i] = 1.0;
        Ri[i * 8 + i] = r8[i];
        P[i * 8 + i] = p08[i];
    }
    int64_t k = 0;
    int have_prev = 0;
    double prev = 0.0;
    for (int64_t e = 0; e < N; ++e) {
        if (etype[e] != 1) continue;
        const double h = have_prev ? t[e] - prev : 0.0;
        const double* p = payload + e * 9;
        F8(h, F);
        memset(Q, 0, sizeof(Q));
        for (int i = 0; i < 8; ++i) Q[i * 8 + i] = q8[i] * h;
        predict(8, F, Q, NULL, x, P);
        const double ax = p[6], ay = p[7];
        const double Vx = x[3] + ax * h, Vy = x[4] + ay * h;
        const double Z[8] = {x[0] + Vx * h, x[1] + Vy * h, p[2], Vx, Vy, p[5], ax, ay};
        update(8, 8, Hi, Ri, Z, x, P);
        if (traj)
            for (int i = 0; i < 3; ++i) traj[k * 3 + i] = x[i];
        if (logdet_out) logdet_out[k] = logdet(8, P);
        ++k;
        prev = t[e];
        have_prev = 1;
    }
    return k;
}
