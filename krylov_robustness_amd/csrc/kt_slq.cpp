// kt_slq.cpp -- the probe-Lanczos sweep engine and the hot-path entry point.
//
// One sweep = P independent single-vector Lanczos runs (one n x P block),
// m steps of four launches each (K1 spmm_dot, coef, K2 update, norm; see
// kt_kernels.hip).  The per-column recurrence coefficients (alpha, up, low)
// land in a host record; the host then solves the m x m tridiagonal
// eigenproblems (kt_dense.cpp, as the north star prescribes) and forms
//   q_c = ||x_c||^2 e1' f(T_c) e1,   T_c = (H + H')/2   (trace_fun_update.m:78-81)
// and, when the basis is recorded, f(A) x_c ~= ||x_c|| V_c f(T_c) e1.
// Sweeps are seeded either by the device Rademacher generator (kt_slq_trace,
// the Hutchinson hot path) or by a given device block (the Lanczos-f Afun
// of mc_trace, kt_mctrace.cpp).
#include "kt_slq.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <thread>

#include "kt_launch.h"
#include "kt_pool.h"

namespace kt {

int slq_auto_block(int64_t n, int64_t nprobes) {
    // Largest power-of-two P whose gathered n x P block (8nP bytes) stays
    // within ~160 MB, i.e. inside the 256 MiB Infinity Cache next to the CSR
    // stream; measured best on MI355X for n = 1M (P = 16) and n = 100k
    // (P = 128) -- profiles/r01_sweep.txt.
    int P = 128;
    while (P > 8 && (double)n * 8.0 * P > 160.0e6) P >>= 1;
    while (P > 1 && P / 2 >= nprobes) P >>= 1;
    // at least two sweeps, so the two sweep lanes overlap one sweep's small
    // coefficient launches and pass tails with the other's pass: config 2
    // (n = 100k, 128 probes) 150 evals/s at one P = 128 sweep, 168 at two
    // P = 64 sweeps (profiles/r02_er100k_sweep.txt)
    while (P > 16 && nprobes < 2 * P) P >>= 1;
    return P;
}

// Run one sweep.  rec_host receives [alpha | up | low][m][P].
// init: if seeded by RNG, `x` == nullptr; else x (device, n x ldx, ncols
// columns, their squared norms in the DEVICE array dnorms2) is copied into
// the sweep block.  ExplicitSweep enqueues it step by step, so sweeps on
// different lanes can be queued launch by launch (the runtime throttles a
// long enqueue burst to ~58 us per call once the host runs ~1 ms ahead, so
// a second lane queued after a whole first sweep would start ms late).
ExplicitSweep::ExplicitSweep(kt_matrix_s* A_, const DevCSR& M_, int P_, int m_, uint64_t seed_, int64_t probe_base_,
                             const double* x_, int ldx_, int ncols_, const double* dnorms2_, double* rec_host_,
                             DevMat* basis_, std::vector<double>* scale_hist_, int lane_, int bcols_)
    : A(A_), M(M_), P(P_), m(m_), seed(seed_), probe_base(probe_base_), x(x_), ldx(ldx_), ncols(ncols_),
      dnorms2(dnorms2_), rec_host(rec_host_), basis(basis_), scale_hist(scale_hist_), lane(lane_), bcols(bcols_) {
    if (bcols <= 0 || bcols > P) bcols = P;
    kt_context_s* ctx = A->ctx;
    n = (int)A->n;
    if (lane < 0 || lane > 3) fail(KT_ERR_ARG, "sweep lane out of range");
    if (lane && !ctx->aux_stream[lane - 1])
        KT_HIP(hipStreamCreateWithFlags(&ctx->aux_stream[lane - 1], hipStreamNonBlocking));
    st = lane ? ctx->aux_stream[lane - 1] : ctx->stream;
    grid = spmm_grid(n, P, ctx->num_cu * 4);  // K2 / short rows
    lblocks = long_blocks_for(M.n_long, ctx->num_cu * 2);
    grid1 = grid + lblocks;                    // K1 total
    SweepBufs& w = ctx->ws.sweep[lane];
    blk_bytes = sizeof(double) * (size_t)n * P;
    w.X0.ensure(blk_bytes);
    w.X1.ensure(blk_bytes);
    w.Y.ensure(blk_bytes);
    w.partial.ensure(sizeof(double) * (size_t)(grid1 + grid * 3) * P);
    w.k2s.ensure(sizeof(double) * 4 * P);
    w.coef.ensure(sizeof(double) * 2 * P);
    w.scales.ensure(sizeof(double) * 3 * P);
    w.trec.ensure(sizeof(double) * (size_t)3 * m * P);
    part1 = w.partial.as<double>();
    part2 = part1 + (size_t)grid1 * P;
    k2s = w.k2s.as<double>();
    coef = w.coef.as<double>();
    trec = w.trec.as<double>();
    Yb = w.Y.as<double>();
    ucur = w.X1.as<double>();
    uprev = w.X0.as<double>();
    sc = w.scales.as<double>();
    sp = sc + P;
    sn = sc + 2 * P;
}

void ExplicitSweep::start() {
    kt_context_s* ctx = A->ctx;
    if (!x) {
        KT_HIP(launch_rademacher(P, n, seed, probe_base, M.perm, ucur, st));
        KT_HIP(launch_fill(sc, P, 1.0 / std::sqrt((double)n), st));
        KT_HIP(launch_fill(k2s, P, (double)n, st));  // ||z||^2 = n
    } else {
        KT_HIP(hipMemsetAsync(ucur, 0, blk_bytes, st));
        KT_HIP(hipMemcpy2DAsync(ucur, sizeof(double) * P, x, sizeof(double) * ldx, sizeof(double) * ncols, (size_t)n,
                                hipMemcpyDeviceToDevice, st));
        // s_0 = 1/||x_c||, ||x_c||^2 from the device norms: no host round trip
        KT_HIP(launch_sweep_scales(dnorms2, ncols, P, 0, sc, k2s, st));
    }
    if (scale_hist) {
        scale_hist->assign((size_t)m * P, 0.0);
        hist_dev = &ctx->ws.sweep[lane].hist;
        hist_dev->ensure(sizeof(double) * (size_t)m * P);
    }
    // basis slot j (u_j's first bcols columns, n x bcols row-major) at
    // bbase + j n bcols: slot 0 copied from the start block, slot j + 1
    // stored by step j's K2 as it forms u_{j+1} (no copy pass per step)
    bbase = basis ? basis->col(0) : nullptr;
}

void ExplicitSweep::step(int j) {
    kt_context_s* ctx = A->ctx;
    const int first = (j == 0);
    if (basis && first)  // u_0 into slot 0
        KT_HIP(hipMemcpy2DAsync(bbase, sizeof(double) * bcols, ucur, sizeof(double) * P, sizeof(double) * bcols,
                                (size_t)n, hipMemcpyDeviceToDevice, st));
    prof_begin(ctx, PROF_SPMM, st, P);
    KT_HIP(launch_spmm_dot(P, ctx->k1_flags | (A->unit_values ? 2 : 0), grid1, M.rowptr, M.col, M.val, n, ucur, sc, Yb,
                           part1, M.long_rows, M.n_long, A->long_thresh, lblocks, st));
    prof_end(ctx, PROF_SPMM, st);
    // the coefficient launch also records s_j (v_j = s_j u_j) for a basis sweep
    KT_HIP(launch_coef_cgs2(P, part1, grid1, first, k2s, sc, sp, coef, trec + (size_t)(0 * m + j) * P,
                            trec + (size_t)(1 * m + j) * P, hist_dev ? hist_dev->as<double>() + (size_t)j * P : nullptr,
                            st));
    prof_begin(ctx, PROF_UPDATE, st, P);
    double* rec = (basis && j + 1 < m) ? bbase + (size_t)(j + 1) * n * bcols : nullptr;
    KT_HIP(launch_update(P, grid, n, Yb, uprev, ucur, sc, sp, coef, first, part2, st, ctx->k2_nt, rec, bcols));
    prof_end(ctx, PROF_UPDATE, st);
    KT_HIP(launch_norm(P, part2, grid, k2s, sn, trec + (size_t)(2 * m + j) * P, st));
    std::swap(ucur, uprev);  // uprev now holds u_{j+1}
    double* t = sp;
    sp = sc;
    sc = sn;
    sn = t;
}

void ExplicitSweep::finish() {
    KT_HIP(hipMemcpyAsync(rec_host, trec, sizeof(double) * (size_t)3 * m * P, hipMemcpyDeviceToHost, st));
    if (scale_hist)
        KT_HIP(hipMemcpyAsync(scale_hist->data(), hist_dev->ptr, sizeof(double) * (size_t)m * P,
                              hipMemcpyDeviceToHost, st));
}

void lanczos_sweep(kt_matrix_s* A, const DevCSR& M, int P, int m, uint64_t seed, int64_t probe_base,
                   const double* x, int ldx, int ncols, const double* dnorms2, double* rec_host,
                   DevMat* basis, std::vector<double>* scale_hist, int lane, int bcols) {
    ExplicitSweep s(A, M, P, m, seed, probe_base, x, ldx, ncols, dnorms2, rec_host, basis, scale_hist, lane, bcols);
    s.start();
    for (int j = 0; j < m; ++j) s.step(j);
    s.finish();
}

// y-form sweep (RNG-seeded probes only): one fused pass + one coefficient
// launch per Lanczos step (kt_kernels.hip, k_spmm_lanczos / k_ycoef).
// rec_host receives [alpha | up | low][m][P] followed by guard[P].  Enqueued
// step by step (start(), step(j) for j < m - 1, finish()), so sweeps on
// different lanes are queued launch by launch.
YSweep::YSweep(kt_matrix_s* A_, const DevCSR& M_, int P_, int m_, uint64_t seed_, int64_t probe_base_,
               double* rec_host_, int lane_)
    : A(A_), M(M_), P(P_), m(m_), seed(seed_), probe_base(probe_base_), rec_host(rec_host_), lane(lane_) {
    kt_context_s* ctx = A->ctx;
    n = (int)A->n;
    if (lane < 0 || lane > 3) fail(KT_ERR_ARG, "sweep lane out of range");
    if (lane && !ctx->aux_stream[lane - 1])
        KT_HIP(hipStreamCreateWithFlags(&ctx->aux_stream[lane - 1], hipStreamNonBlocking));
    st = lane ? ctx->aux_stream[lane - 1] : ctx->stream;
    grid = spmm_grid(n, P, ctx->num_cu * 4);  // 4 row-group workgroups per CU
    lblocks = long_blocks_for(M.n_long, ctx->num_cu * 2);
    grid1 = grid + lblocks;
    SweepBufs& w = ctx->ws.sweep[lane];
    blk_bytes = sizeof(double) * (size_t)n * P;
    w.X0.ensure(blk_bytes);
    w.X1.ensure(blk_bytes);
    w.Y.ensure(blk_bytes);
    w.partial.ensure(sizeof(double) * (size_t)3 * P * grid1);  // slot-major [3P][grid1]
    w.coef.ensure(sizeof(double) * 9 * P);
    w.trec.ensure(sizeof(double) * ((size_t)3 * m * P + P));
    part = w.partial.as<double>();
    ys = w.coef.as<double>();
    trec = w.trec.as<double>();
    guard = trec + (size_t)3 * m * P;
    flags = ctx->ky_flags | (A->unit_values ? 2 : 0);
    if (blk_bytes >= ((size_t)1 << 31)) flags &= ~16;  // sc1 buffer stores take 32-bit offsets
    Z = w.X1.as<uint32_t>();
    Xc = w.Y.as<double>();   // y_j
    Yo = nullptr;            // y_{j-1} (none at j = 0)
    Ot = w.X0.as<double>();  // y_{j+1}
}

void YSweep::start() {
    kt_context_s* ctx = A->ctx;
    const double s0 = 1.0 / std::sqrt((double)n);  // v_0 = z / ||z||, ||z||^2 = n
    // probes as a packed sign table (n x ceil(P/32) words), gathered by the
    // start pass instead of an 8nP-byte fp64 block
    KT_HIP(launch_rademacher_signs(P, n, seed, probe_base, M.perm, Z, st));
    prof_begin(ctx, PROF_START, st, P);
    KT_HIP(launch_spmm_lanczos_start(P, flags, grid1, M.rowptr, M.col, M.val, n, Z, s0, Xc, part, M.long_rows,
                                     M.n_long, A->long_thresh, lblocks, st));
    prof_end(ctx, PROF_START, st);
    KT_HIP(launch_ycoef(P, part, grid1, 1, m == 1, s0, ys, rec_at(0, 0), rec_at(1, 0), rec_at(2, 0), guard, st));
}

void YSweep::step(int j) {
    kt_context_s* ctx = A->ctx;
    prof_begin(ctx, PROF_SPMM, st, P);
    const bool last = j + 2 == m;  // y_{m} is never used: alpha_{m-1} needs only X.t
    KT_HIP(launch_spmm_lanczos(P, flags, grid1, M.rowptr, M.col, M.val, n, Xc, last ? nullptr : Yo,
                               last ? nullptr : Ot, ys + 6 * P, part, M.long_rows, M.n_long, A->long_thresh,
                               lblocks, st));
    prof_end(ctx, PROF_SPMM, st);
    KT_HIP(launch_ycoef(P, part, grid1, 0, last, 0.0, ys, rec_at(0, j + 1), rec_at(1, j + 1), rec_at(2, j + 1),
                        guard, st));
    Yo = Xc;  // y_{j+1} overwrites y_{j-1} from the next pass on
    Xc = Ot;
    Ot = Yo;
}

void YSweep::finish() {
    KT_HIP(hipMemcpyAsync(rec_host, trec, sizeof(double) * ((size_t)3 * m * P + P), hipMemcpyDeviceToHost, st));
}

// y-form sweep seeded by a given device block (the quadrature-only columns
// of mc_trace's Lanczos Afun, kt_mctrace.cpp): x (n x ldx, ncols columns, in
// M's row order, squared norms in the device array dnorms2) is normalised into the gathered table
// v_0 (zero columns stay zero), the pass in start mode forms y_0 = A v_0 with
// (g, a, b) = (1, 0, 0), then the same passes as the RNG-seeded sweep
// (steps 0 .. m-2).  rec_host (pinned, or the call waits for the copy)
// receives [alpha | up | low][m][P] followed by guard[P].  No basis:
// quadratic forms only.
YBlockSweep::YBlockSweep(kt_matrix_s* A_, const DevCSR& M_, int P_, int m_, const double* x_, int ldx_, int ncols_,
                         const double* dnorms2_, double* rec_host_, int lane_, double* basis_, int bcols_)
    : A(A_), M(M_), P(P_), m(m_), x(x_), ldx(ldx_), ncols(ncols_), dnorms2(dnorms2_), rec_host(rec_host_),
      lane(lane_), basis(basis_), bcols(basis_ ? bcols_ : 0) {
    kt_context_s* ctx = A->ctx;
    n = (int)A->n;
    if (lane < 0 || lane > 3) fail(KT_ERR_ARG, "sweep lane out of range");
    if (ncols < 1 || ncols > P) fail(KT_ERR_ARG, "y-form block sweep: 1 <= ncols <= P");
    if (lane && !ctx->aux_stream[lane - 1])
        KT_HIP(hipStreamCreateWithFlags(&ctx->aux_stream[lane - 1], hipStreamNonBlocking));
    st = lane ? ctx->aux_stream[lane - 1] : ctx->stream;
    grid = spmm_grid(n, P, ctx->num_cu * 4);
    lblocks = long_blocks_for(M.n_long, ctx->num_cu * 2);
    grid1 = grid + lblocks;
    SweepBufs& w = ctx->ws.sweep[lane];
    blk_bytes = sizeof(double) * (size_t)n * P;
    w.X0.ensure(blk_bytes);
    w.X1.ensure(blk_bytes);
    w.Y.ensure(blk_bytes);
    w.partial.ensure(sizeof(double) * (size_t)3 * P * grid1);
    w.coef.ensure(sizeof(double) * 9 * P);
    w.trec.ensure(sizeof(double) * ((size_t)3 * m * P + P));
    part = w.partial.as<double>();
    ys = w.coef.as<double>();
    trec = w.trec.as<double>();
    guard = trec + (size_t)3 * m * P;
    flags = ctx->ky_flags | (A->unit_values ? 2 : 0);
    if (blk_bytes >= ((size_t)1 << 31)) flags &= ~16;  // sc1 buffer stores take 32-bit offsets
    V0 = basis ? slot(0) : w.X1.as<double>();  // the start pass's gathered table v_0 (basis slot 0)
    Xc = w.Y.as<double>();   // y_j
    Yo = nullptr;            // y_{j-1}
    Ot = w.X0.as<double>();  // y_{j+1}
}

void YBlockSweep::start() {
    // ys: [1/||x_c|| (P) | 0 (5P) | start pass (g, a, b) = (1, 0, 0) (3P)], from
    // the device norms (no host round trip)
    KT_HIP(launch_sweep_scales(dnorms2, ncols, P, 1, ys, nullptr, st));
    KT_HIP(hipMemsetAsync(V0, 0, blk_bytes, st));
    KT_HIP(launch_weighted_sum(n, 1, P, ncols, x, ldx, 0, ys, V0, P, st));
    kt_context_s* ctx = A->ctx;
    prof_begin(ctx, PROF_YBLOCK, st, P);
    KT_HIP(launch_spmm_lanczos(P, flags, grid1, M.rowptr, M.col, M.val, n, V0, nullptr, Xc, ys + 6 * P, part,
                               M.long_rows, M.n_long, A->long_thresh, lblocks, st));
    prof_end(ctx, PROF_YBLOCK, st);
    KT_HIP(launch_ycoef(P, part, grid1, 1, m == 1, 1.0, ys, rec_at(0, 0), rec_at(1, 0), rec_at(2, 0), guard, st));
}

void YBlockSweep::step(int j) {
    const bool last = j + 2 == m;
    prof_begin(A->ctx, PROF_YBLOCK, st, P);
    KT_HIP(launch_spmm_lanczos(P, flags, grid1, M.rowptr, M.col, M.val, n, Xc, last ? nullptr : Yo,
                               last ? nullptr : Ot, ys + 6 * P, part, M.long_rows, M.n_long, A->long_thresh, lblocks,
                               st, basis ? slot(j) : nullptr, (basis && j > 0) ? slot(j - 1) : nullptr,
                               basis ? slot(j + 1) : nullptr, bcols));
    prof_end(A->ctx, PROF_YBLOCK, st);
    KT_HIP(launch_ycoef(P, part, grid1, 0, last, 0.0, ys, rec_at(0, j + 1), rec_at(1, j + 1), rec_at(2, j + 1), guard,
                        st));
    Yo = Xc;
    Xc = Ot;
    Ot = Yo;
}

void YBlockSweep::finish() {
    KT_HIP(hipMemcpyAsync(rec_host, trec, sizeof(double) * ((size_t)3 * m * P + P), hipMemcpyDeviceToHost, st));
}

void lanczos_sweep_y_block(kt_matrix_s* A, const DevCSR& M, int P, int m, const double* x, int ldx, int ncols,
                           const double* dnorms2, double* rec_host, int lane) {
    YBlockSweep s(A, M, P, m, x, ldx, ncols, dnorms2, rec_host, lane);
    s.start();
    for (int j = 0; j + 1 < m; ++j) s.step(j);
    s.finish();
}

// A y-form probe is accepted when every used beta_k^2 kept at least this
// fraction of ||y_{k-1}||^2 (its Gram-identity cancellation then costs at most
// ~1e4 ulp); otherwise its sweep is recomputed by the explicit CGS2 sweep.
// Measured minimum on the golden graphs and Chung-Lu up to m = 100: 6.4e-3.
constexpr double kYformGuard = 1e-4;

// Column c of a sweep record -> symmetric tridiagonal (alpha, off); returns
// the number of steps before a lucky breakdown (lanczos_krylov.m:91-93).
int record_tridiag(const double* R, int m, int P, int c, double* al, double* off) {
    int steps = m;
    for (int j = 0; j < m; ++j)
        if (R[(size_t)(2 * m + j) * P + c] < 1e-8) {
            steps = j + 1;
            break;
        }
    for (int j = 0; j < steps; ++j) al[j] = R[(size_t)(0 * m + j) * P + c];
    for (int j = 0; j + 1 < steps; ++j)
        off[j] = 0.5 * (R[(size_t)(2 * m + j) * P + c] + R[(size_t)(1 * m + j + 1) * P + c]);
    return steps;
}

void lanczos_columns(kt_matrix_s* A, const double* X, int ldx, int ncols, int m, int fun,
                     double* quad, double* Y, int ldy) {
    // every column by the explicit sweep (P = pow2 >= ncols, <= 16);
    // KT_LC_YBASIS=1 (tests): the f(A) x columns by basis-forming y-form sweeps
    const char* e = getenv("KT_LC_YBASIS");
    const int yb = (e && e[0] == '1' && Y) ? ncols : 0;
    lanczos_columns_split(A, X, ldx, ncols, Y ? ncols : 0, ncols, m, fun, quad, Y, ldy, 0, 16, yb);
}

// Widths of the y-form sweeps for `cols` quadrature-only columns: sweeps of
// 16, the remainder at the power of two that holds it.  At config 4 the final
// mc_trace round's 20 columns as 16 + 4: 43.2 ms per trace_exp vs 44.8 with
// the remainder zero-padded to 16 (profiles/r05/sweep_plan_ab/; with the
// lanes queued step by step -- the padded form measured faster while the
// second lane was queued only after the whole first sweep).  The explicit
// sweep does not take narrow chunks: 10 + 30 columns as greedy power-of-two
// sweeps (8 + 2, 16 + 8 + 4 + 2) cost 53 ms.
// A smaller `chunk` cuts the columns into sweeps of `chunk` (the last one
// shorter), each at the power of two that holds it: {(columns, width)}.
// KT_LC_YMINP (A/B): the narrowest y-form sweep width (a remainder of 4
// columns padded to 8 or 16 instead of a 4-wide sweep).
static std::vector<std::pair<int, int>> quad_plan(int cols, int chunk = 16) {
    std::vector<std::pair<int, int>> wv;
    chunk = std::max(1, std::min(chunk, 16));
    const char* e = getenv("KT_LC_YMINP");
    const int pmin = e ? std::max(1, std::min(16, atoi(e))) : 1;
    for (int left = cols; left > 0; left -= chunk) {
        const int c = std::min(left, chunk);
        int P = 1;
        while (P < c || P < pmin) P <<= 1;
        wv.push_back({c, P});
    }
    return wv;
}

void lanczos_columns_split(kt_matrix_s* A, const double* X, int ldx, int ncols, int ny, int ne, int m, int fun,
                           double* quad, double* Y, int ldy, int px, int ychunk, int yb) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    if (!Y) ny = 0;
    if (ny < 0 || ny > ne || ne > ncols) fail(KT_ERR_ARG, "lanczos_columns_split: 0 <= ny <= ne <= ncols");
    yb = std::max(0, std::min(yb, ny));
    // squared column norms on the device (the sweeps' start scales are formed
    // from them there); the host reads them with the sweep records
    ctx->ws.colnorm.ensure(sizeof(double) * ncols);
    double* dn2 = ctx->ws.colnorm.as<double>();
    KT_HIP(launch_gram_diag(gram_device(ctx, n, X, ldx, ncols, X, ldx, ncols), ncols, ncols, dn2, ctx->stream));
    // The sweeps run on the hubs-first CSR (equal-length neighbouring rows,
    // adjacent hub segments: the explicit K1 at P = 16 on the bench graph 264
    // -> ~210 us): the block is permuted into that row order on the way in
    // and f(A) x back out; quadratic forms are permutation invariant.
    const DevCSR& M = hub_csr(A);
    const int* perm = M.perm;
    DevMat Xh, Yh;
    const double* Xs = X;
    int ldxs = ldx;
    double* Ys = Y;
    int ldys = ldy;
    if (perm) {
        Xh.alloc(ctx, n, ncols, false);
        KT_HIP(launch_perm_rows((int)n, ncols, perm, 1, X, ldx, Xh.col(0), ncols, ctx->stream));
        Xs = Xh.col(0);
        ldxs = ncols;
        if (ny) {
            Yh.alloc(ctx, n, ny, false);
            Ys = Yh.col(0);
            ldys = ny;
        }
    }
    // Sweeps: columns [0, ne) by the explicit CGS2 sweep (P = px, or pow2 >=
    // ne capped at 16), the basis kept for the ny f(A)x columns among them;
    // columns [ne, ncols) -- quadratic forms only -- by y-form sweeps (no K2,
    // no basis; widths quad_plan).  All queued before the host waits, dealt
    // over the four lanes, so the device runs them side by side.
    struct Sw {
        int c0, nc, P, lane;
        bool yform;
        bool ybasis;  // a y-form sweep that also forms its Lanczos basis (KF_VB)
    };
    std::vector<Sw> sw;
    const char* ye = getenv("KT_LC_YFORM");  // 0: every column by the explicit sweep
    if (ye && ye[0] == '0') {
        ne = ncols;
        yb = 0;
    }
    int Pe = 1;
    while (Pe < ne - yb && Pe < 16) Pe <<= 1;
    if (px > 0) Pe = px;
    if (Pe > 32 || (Pe & (Pe - 1))) fail(KT_ERR_ARG, "lanczos_columns_split: sweep width must be a power of two <= 32");
    // sweeps dealt over the four lanes in order (basis-forming y-form, then
    // explicit, then forms-only y-form), so up to four run side by side; a
    // lane's later sweeps follow its earlier ones
    int k = 0;
    for (int c0 = 0; c0 < yb; c0 += 16) {
        const int c = std::min(16, yb - c0);
        int P = 1;
        while (P < c) P <<= 1;
        sw.push_back({c0, c, P, k++ % 4, true, true});
    }
    for (int c0 = yb; c0 < ne; c0 += Pe) sw.push_back({c0, std::min(Pe, ne - c0), Pe, k++ % 4, false, false});
    {
        int c0 = ne;
        for (const auto& cp : quad_plan(ncols - ne, ychunk)) {
            sw.push_back({c0, cp.first, cp.second, k++ % 4, true, false});
            c0 += cp.first;
        }
    }
    const size_t rec_max = (size_t)3 * m * 32 + 32;
    PinnedBuf& hr = ctx->ws.pin_colrec;
    hr.ensure(sizeof(double) * (rec_max * sw.size() + ncols));
    double* hn2 = hr.as<double>() + rec_max * sw.size();  // the norms, read after the sweeps
    KT_HIP(hipMemcpyAsync(hn2, dn2, sizeof(double) * ncols, hipMemcpyDeviceToHost, ctx->stream));
    // the aux lanes read the permuted block written on ctx->stream
    hipEvent_t ready = ctx->ws.colsplit_ev;
    if (!ready) {
        KT_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
        ctx->ws.colsplit_ev = ready;
    }
    KT_HIP(hipEventRecord(ready, ctx->stream));
    bool used[4] = {true, false, false, false};
    for (size_t i = 0; i < sw.size(); ++i) {
        const Sw& q = sw[i];
        if (used[q.lane]) continue;
        hipStream_t& as = ctx->aux_stream[q.lane - 1];
        if (!as) KT_HIP(hipStreamCreateWithFlags(&as, hipStreamNonBlocking));
        KT_HIP(hipStreamWaitEvent(as, ready, 0));
        used[q.lane] = true;
    }
    // the explicit sweeps keep their bases (slot j: n x nyc); the basis-forming
    // y-form sweeps theirs as m slots of n x P (normalised vectors: no scale
    // history)
    std::vector<DevMat> bases(sw.size());
    std::vector<std::vector<double>> hists(sw.size());
    for (size_t i = 0; i < sw.size(); ++i) {
        const Sw& q = sw[i];
        if (q.ybasis) {
            bases[i].alloc(ctx, (int64_t)m * n, q.P, false);  // slot j = rows [j n, (j + 1) n)
            continue;
        }
        if (q.yform) continue;
        const int nyc = std::max(0, std::min(q.nc, ny - q.c0));
        if (nyc) bases[i].alloc(ctx, n, m * nyc, false);  // every slot is written by the sweep
    }
    // Queue the sweeps launch by launch across lanes (one sweep per lane at a
    // time: a lane's sweeps share its buffers), so every lane starts at once
    std::vector<int> next(4, 0);  // per lane: index into its sweeps
    std::vector<std::vector<int>> by_lane(4);
    for (size_t i = 0; i < sw.size(); ++i) by_lane[sw[i].lane].push_back((int)i);
    for (;;) {
        std::vector<std::unique_ptr<ExplicitSweep>> ex;
        std::vector<std::unique_ptr<YBlockSweep>> ybs;
        for (int l = 0; l < 4; ++l) {
            if (next[l] >= (int)by_lane[l].size()) continue;
            const int i = by_lane[l][next[l]++];
            const Sw& q = sw[i];
            double* R = hr.as<double>() + rec_max * i;
            if (q.yform) {
                ybs.emplace_back(new YBlockSweep(A, M, q.P, m, Xs + q.c0, ldxs, q.nc, dn2 + q.c0, R, q.lane,
                                                 q.ybasis ? bases[i].col(0) : nullptr, q.nc));
            } else {
                const int nyc = std::max(0, std::min(q.nc, ny - q.c0));
                ex.emplace_back(new ExplicitSweep(A, M, q.P, m, 0, 0, Xs + q.c0, ldxs, q.nc, dn2 + q.c0, R,
                                                  nyc ? &bases[i] : nullptr, nyc ? &hists[i] : nullptr, q.lane,
                                                  nyc));
            }
        }
        if (ex.empty() && ybs.empty()) break;
        for (auto& y : ybs) y->start();
        for (auto& e : ex) e->start();
        for (int j = 0; j < m; ++j) {
            for (auto& y : ybs)
                if (j + 1 < m) y->step(j);
            for (auto& e : ex) e->step(j);
        }
        for (auto& y : ybs) y->finish();
        for (auto& e : ex) e->finish();
    }
    KT_HIP(hipStreamSynchronize(ctx->stream));
    for (int l = 1; l < 4; ++l)
        if (used[l]) KT_HIP(hipStreamSynchronize(ctx->aux_stream[l - 1]));
    const std::vector<double> norms2(hn2, hn2 + ncols);
    // a y-form column that tripped the cancellation guard (or broke down) is
    // redone by the explicit CGS2 sweep at the same width; only the tripped
    // columns take the redo's records, so a column's form never depends on
    // which columns share its sweep (mc_trace's world-size bit identity)
    // A basis-forming sweep with a tripped column is redone WHOLE by the
    // explicit sweep with its basis (its columns are f(A) x inputs, not
    // sharded forms): the sweep then takes the explicit path's records,
    // basis and scale history.
    std::vector<double> redo;
    std::vector<char> ex_basis(sw.size(), 0);  // the sweep's basis is the explicit layout
    for (size_t i = 0; i < sw.size(); ++i) ex_basis[i] = !sw[i].yform;
    for (size_t i = 0; i < sw.size(); ++i) {
        const Sw& q = sw[i];
        if (!q.yform) continue;
        double* R = hr.as<double>() + rec_max * i;
        const double* g = R + (size_t)3 * m * q.P;
        std::vector<int> bad;
        for (int c = 0; c < q.nc; ++c)
            if (norms2[q.c0 + c] > 0.0 && !(g[c] >= kYformGuard)) bad.push_back(c);
        if (bad.empty()) continue;
        if (q.ybasis) {
            const int nyc = std::max(0, std::min(q.nc, ny - q.c0));
            DevMat eb;
            if (nyc) eb.alloc(ctx, n, m * nyc, false);
            lanczos_sweep(A, M, q.P, m, 0, 0, Xs + q.c0, ldxs, q.nc, dn2 + q.c0, R, nyc ? &eb : nullptr,
                          nyc ? &hists[i] : nullptr, 0, nyc);
            KT_HIP(hipStreamSynchronize(ctx->stream));
            bases[i] = std::move(eb);
            ex_basis[i] = 1;
            ctx->yform_redone += 1;
            continue;
        }
        redo.assign((size_t)3 * m * q.P, 0.0);
        lanczos_sweep(A, M, q.P, m, 0, 0, Xs + q.c0, ldxs, q.nc, dn2 + q.c0, redo.data(), nullptr, nullptr, 0);
        KT_HIP(hipStreamSynchronize(ctx->stream));
        for (int c : bad)
            for (int row = 0; row < 3 * m; ++row) R[(size_t)row * q.P + c] = redo[(size_t)row * q.P + c];
        ctx->yform_redone += 1;
    }
    // per column (one QL pass each, on the host pool): the quadrature and,
    // for the f(A) x columns, f(T) e1 -> the basis weights
    std::vector<int> nycs(sw.size()), col_sw, col_c;
    std::vector<std::vector<double>> Ws(sw.size());  // Y = sum_j u_j w_j, [j * nyc + c]
    for (size_t i = 0; i < sw.size(); ++i) {
        const Sw& q = sw[i];
        nycs[i] = (q.yform && !q.ybasis) ? 0 : std::max(0, std::min(q.nc, ny - q.c0));
        Ws[i].assign((size_t)m * std::max(nycs[i], 1), 0.0);
        for (int c = 0; c < q.nc; ++c) {
            col_sw.push_back((int)i);
            col_c.push_back(c);
        }
    }
    HostPool::get().run((int)col_sw.size(), [&](int t) {
        const int i = col_sw[t], c = col_c[t], nyc = nycs[i];
        const Sw& q = sw[i];
        const double* R = hr.as<double>() + rec_max * i;
        std::vector<double> al(m), off(m), fe1(m);
        const int steps = record_tridiag(R, m, q.P, c, al.data(), off.data());
        if (norms2[q.c0 + c] == 0.0) {
            if (quad) quad[q.c0 + c] = 0.0;
            return;
        }
        if (c >= nyc) {
            if (quad) quad[q.c0 + c] = norms2[q.c0 + c] * tridiag_quadrature(steps, al.data(), off.data(), fun);
            return;
        }
        const double qd = tridiag_fun_e1(steps, al.data(), off.data(), fun, fe1.data());
        if (quad) quad[q.c0 + c] = norms2[q.c0 + c] * qd;
        const double nx = std::sqrt(norms2[q.c0 + c]);
        if (ex_basis[i]) {
            for (int j = 0; j < steps; ++j)
                Ws[i][(size_t)j * nyc + c] = nx * hists[i][(size_t)j * q.P + c] * fe1[j];  // v_j = s_j u_j
        } else {  // the y-form basis holds the normalised v_j
            for (int j = 0; j < steps; ++j) Ws[i][(size_t)j * nyc + c] = nx * fe1[j];
        }
    }, 4);
    for (size_t i = 0; i < sw.size(); ++i) {
        const Sw& q = sw[i];
        const int nyc = nycs[i];
        const std::vector<double>& W = Ws[i];
        if (nyc) {
            DevBuf& dw = ctx->ws.small2;
            dw.ensure(sizeof(double) * W.size());
            KT_HIP(hipMemcpyAsync(dw.ptr, W.data(), sizeof(double) * W.size(), hipMemcpyHostToDevice, ctx->stream));
            // explicit basis: slot j = n x nyc; y-form basis: slot j = n x P
            const int ldu = ex_basis[i] ? nyc : q.P;
            KT_HIP(launch_weighted_sum((int)n, m, nyc, nyc, bases[i].col(0), ldu, (int64_t)n * ldu, dw.as<double>(),
                                       Ys + q.c0, ldys, ctx->stream));
            KT_HIP(hipStreamSynchronize(ctx->stream));
        }
    }
    if (perm && ny) KT_HIP(launch_perm_rows((int)n, ny, perm, 0, Ys, ldys, Y, ldy, ctx->stream));
}

static bool pow2_le128(int b) { return b >= 1 && b <= 128 && (b & (b - 1)) == 0; }

}  // namespace kt

using namespace kt;

extern "C" int kt_slq_plan(kt_matrix_t A, int64_t nprobes, int* block) {
    if (!A || !block || nprobes < 0) {
        kt::set_error("kt_slq_plan: bad argument");
        return KT_ERR_ARG;
    }
    *block = slq_auto_block(A->n, nprobes);
    return KT_OK;
}

namespace kt {

// The device half of kt_slq_trace: queue the sweeps (their record copies
// land in this call's host slot) and record one event per lane.  Returns the
// ticket; at most two calls may be outstanding per context.
static int slq_submit(kt_matrix_s* A, int fun, int m, uint64_t seed, int64_t probe_offset, int64_t nprobes,
                      int block) {
    if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
    if (m < 1 || m > 256) fail(KT_ERR_ARG, "m must be in [1, 256]");
    if (nprobes < 0 || probe_offset < 0) fail(KT_ERR_ARG, "negative probe range");
    if (block != 0 && !pow2_le128(block)) fail(KT_ERR_ARG, "block must be 0 or a power of two <= 128");
    kt_context_s* ctx = A->ctx;
    Workspace& w = ctx->ws;
    if (w.slq_submitted - w.slq_collected >= 2)
        fail(KT_ERR_ARG, "kt_slq_submit: two calls already outstanding (collect one first)");
    const uint64_t ticket = w.slq_submitted;
    SlqPending& pd = w.slq_pend[ticket & 1];
    const int64_t n = A->n;
    pd.live = false;
    pd.A = A;
    pd.fun = fun;
    pd.m = m;
    pd.seed = seed;
    pd.offset = probe_offset;
    pd.nprobes = (n == 0) ? 0 : nprobes;
    pd.P = block ? block : slq_auto_block(n, std::max<int64_t>(nprobes, 1));
    pd.nsweeps = pd.nprobes ? (pd.nprobes + pd.P - 1) / pd.P : 0;
    // record per sweep: [alpha | up | low][m][P] (+ guard[P] in y-form)
    pd.rec = (size_t)3 * m * pd.P + pd.P;
    // KT_SLQ_LANES=L (<= 4): sweeps round-robin over L streams, so one
    // sweep's small launches (and, in the explicit sweep, its streaming K2)
    // overlap another sweep's gather-bound pass; measured best
    // (profiles/r01_yform_lanes.txt): 2 for the y-form pass, 3 for the
    // explicit K1/K2 sweep
    const char* le = getenv("KT_SLQ_LANES");
    const int lanes_env = le ? std::max(1, std::min(4, atoi(le))) : (ctx->yform ? 2 : 3);
    pd.lanes = (int)std::max<int64_t>(1, std::min<int64_t>(pd.nsweeps, lanes_env));
    if (pd.nsweeps) {
        KT_HIP(hipSetDevice(ctx->device));
        PinnedBuf& hb = w.host_trec[ticket & 1];
        hb.ensure(sizeof(double) * pd.rec * pd.nsweeps);
        double* htrec = hb.as<double>();
        const DevCSR& H = hub_csr(A);
        // profiling: the previous calls' events are folded in while this
        // call's sweeps run on the device
        prof_recycle(ctx);
        size_t prev_events[PROF_NSLOTS];
        for (int k = 0; k < PROF_NSLOTS; ++k) prev_events[k] = ctx->prof[k].used;
        // one sweep per lane at a time, the lanes' sweeps queued step by step
        // (launch by launch across the lanes, so every lane starts at once)
        for (int64_t s0 = 0; s0 < pd.nsweeps; s0 += pd.lanes) {
            const int g = (int)std::min<int64_t>(pd.lanes, pd.nsweeps - s0);
            if (ctx->yform) {
                std::vector<std::unique_ptr<YSweep>> grp;
                for (int l = 0; l < g; ++l)
                    grp.emplace_back(new YSweep(A, H, pd.P, m, seed, probe_offset + (s0 + l) * pd.P,
                                                htrec + pd.rec * (s0 + l), l));
                for (auto& y : grp) y->start();
                for (int j = 0; j + 1 < m; ++j)
                    for (auto& y : grp) y->step(j);
                for (auto& y : grp) y->finish();
            } else {
                std::vector<std::unique_ptr<ExplicitSweep>> grp;
                for (int l = 0; l < g; ++l)
                    grp.emplace_back(new ExplicitSweep(A, H, pd.P, m, seed, probe_offset + (s0 + l) * pd.P, nullptr,
                                                       0, 0, nullptr, htrec + pd.rec * (s0 + l), nullptr, nullptr,
                                                       l, 0));
                for (auto& e : grp) e->start();
                for (int j = 0; j < m; ++j)
                    for (auto& e : grp) e->step(j);
                for (auto& e : grp) e->finish();
            }
        }
        for (int l = 0; l < pd.lanes; ++l) {
            if (!pd.done[l]) KT_HIP(hipEventCreateWithFlags(&pd.done[l], hipEventDisableTiming));
            KT_HIP(hipEventRecord(pd.done[l], l ? ctx->aux_stream[l - 1] : ctx->stream));
        }
        // (those may still be in flight when the previous submission is not
        // collected yet: wait for them -- this call's sweeps are queued already)
        prof_collect(ctx, prev_events, true);
    }
    pd.live = true;
    ++w.slq_submitted;
    return (int)(ticket & 0x7fffffff);
}

// The host half: wait for the call's sweeps (its lane events only, not work
// submitted after it), redo guarded sweeps with the explicit CGS2 sweep,
// host Gauss quadrature, sums.
static void slq_collect(kt_matrix_s* A, int ticket, double* sum_q, double* sum_q2, double* q) {
    kt_context_s* ctx = A->ctx;
    Workspace& w = ctx->ws;
    if (w.slq_collected == w.slq_submitted || (uint64_t)ticket != (w.slq_collected & 0x7fffffff))
        fail(KT_ERR_ARG, "kt_slq_collect: tickets must be collected once each, in submission order");
    SlqPending& pd = w.slq_pend[w.slq_collected & 1];
    const uint64_t slot = w.slq_collected & 1;
    // the record's n, CSR (guard redo) and lanes belong to the submitting
    // matrix: a call with another matrix is refused BEFORE the ticket is
    // consumed, so the caller can collect it with the right one; a ticket
    // whose matrix was destroyed (its sweeps drained) is consumed
    if (pd.live && pd.A && pd.A != A)
        fail(KT_ERR_ARG, "kt_slq_collect: the ticket was submitted with another matrix");
    ++w.slq_collected;
    if (!pd.live) fail(KT_ERR_ARG, "kt_slq_collect: the submission failed");
    pd.live = false;
    if (pd.A != A) fail(KT_ERR_ARG, "kt_slq_collect: the submitting matrix was destroyed");
    if (sum_q) *sum_q = 0.0;
    if (sum_q2) *sum_q2 = 0.0;
    if (pd.nprobes == 0) return;
    const int64_t n = A->n, nprobes = pd.nprobes;
    const int m = pd.m, P = pd.P, fun = pd.fun;
    const size_t rec = pd.rec;
    double* htrec = w.host_trec[slot].as<double>();
    KT_HIP(hipSetDevice(ctx->device));
    for (int l = 0; l < pd.lanes; ++l) KT_HIP(hipEventSynchronize(pd.done[l]));
#if !defined(KT_KY_DIAG) || KT_KY_DIAG == 0  // (diagnostic builds time the pass alone: no redo)
    if (ctx->yform) {  // sweeps with a guarded probe are redone by the explicit CGS2 sweep
        const DevCSR& H = hub_csr(A);
        int64_t redone = 0;
        for (int64_t sw = 0; sw < pd.nsweeps; ++sw) {
            const double* g = htrec + rec * sw + (size_t)3 * m * P;
            const int64_t live = std::min<int64_t>(P, nprobes - sw * P);
            bool bad = false;
            for (int64_t c = 0; c < live; ++c) bad |= !(g[c] >= kYformGuard);
            if (!bad) continue;
            lanczos_sweep(A, H, P, m, pd.seed, pd.offset + sw * P, nullptr, 0, 0, nullptr, htrec + rec * sw,
                          nullptr, nullptr, 0);
            KT_HIP(hipStreamSynchronize(ctx->stream));
            ++redone;
        }
        ctx->yform_redone += redone;
    }
#endif
    // host Gauss quadrature, 16 probes per task on the persistent pool
    // (threads spawned and joined per call cost ~0.1-0.3 ms per call)
    std::vector<double> qv((size_t)nprobes);
    const int64_t chunk = 16;
    HostPool::get().run((int)((nprobes + chunk - 1) / chunk), [&](int t) {
        std::vector<double> al(m), off(m);
        const int64_t pb = t * chunk, pe = std::min<int64_t>(nprobes, pb + chunk);
        for (int64_t p = pb; p < pe; ++p) {
            const int steps = record_tridiag(htrec + rec * (p / P), m, P, (int)(p % P), al.data(), off.data());
            qv[p] = (double)n * tridiag_quadrature(steps, al.data(), off.data(), fun);
        }
    }, 4);
    double s1 = 0.0, s2 = 0.0;
    for (int64_t p = 0; p < nprobes; ++p) {
        s1 += qv[p];
        s2 += qv[p] * qv[p];
        if (q) q[p] = qv[p];
    }
    if (sum_q) *sum_q = s1;
    if (sum_q2) *sum_q2 = s2;
}

}  // namespace kt

#define KT_SLQ_TRY try {
#define KT_SLQ_CATCH                         \
    }                                        \
    catch (const kt::Status& s) {            \
        kt::set_error(s.msg);                \
        return s.code;                       \
    }                                        \
    catch (const std::exception& e) {        \
        kt::set_error(e.what());             \
        return KT_ERR_ARG;                   \
    }                                        \
    return KT_OK;

extern "C" int kt_slq_trace(kt_matrix_t A, int fun, int m, uint64_t seed, int64_t probe_offset,
                            int64_t nprobes, int block, double* sum_q, double* sum_q2, double* q) {
    KT_SLQ_TRY
    if (!A) fail(KT_ERR_ARG, "A is NULL");
    Workspace& w = A->ctx->ws;
    if (w.slq_submitted != w.slq_collected)
        fail(KT_ERR_ARG, "kt_slq_trace: kt_slq_submit calls are outstanding on this context");
    const int t = slq_submit(A, fun, m, seed, probe_offset, nprobes, block);
    slq_collect(A, t, sum_q, sum_q2, q);
    KT_SLQ_CATCH
}

extern "C" int kt_slq_submit(kt_matrix_t A, int fun, int m, uint64_t seed, int64_t probe_offset,
                             int64_t nprobes, int block, int* ticket) {
    KT_SLQ_TRY
    if (!A || !ticket) fail(KT_ERR_ARG, "NULL argument");
    *ticket = slq_submit(A, fun, m, seed, probe_offset, nprobes, block);
    KT_SLQ_CATCH
}

extern "C" int kt_slq_collect(kt_matrix_t A, int ticket, double* sum_q, double* sum_q2, double* q) {
    KT_SLQ_TRY
    if (!A) fail(KT_ERR_ARG, "A is NULL");
    slq_collect(A, ticket, sum_q, sum_q2, q);
    KT_SLQ_CATCH
}
