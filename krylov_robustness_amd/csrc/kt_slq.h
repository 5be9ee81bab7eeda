// kt_slq.h -- probe-Lanczos sweep engine shared by the SLQ hot path and the
// Lanczos-f Afun of mc_trace.
#pragma once
#include "kt_block.h"

namespace kt {

int slq_auto_block(int64_t n, int64_t nprobes);

// One sweep of P independent single-vector Lanczos runs (see kt_slq.cpp).
// lane 0 runs on ctx->stream with ws.sweep[0]; lane l > 0 on
// ctx->aux_stream[l-1] with ws.sweep[l] (independent sweeps overlap).
// basis (optional, >= n m bcols doubles): slot j = u_j's first bcols columns
// as an n x bcols row-major block at basis->col(0) + j n bcols.
void lanczos_sweep(kt_matrix_s* A, const DevCSR& M, int P, int m, uint64_t seed, int64_t probe_base,
                   const double* x, int ldx, int ncols, const double* dnorms2, double* rec_host,
                   DevMat* basis, std::vector<double>* scale_hist, int lane = 0, int bcols = 0);

// lanczos_sweep enqueued step by step: start(), step(j) for j < m, finish().
// Sweeps on different lanes may be interleaved step by step; two sweeps on
// one lane may not (they share the lane's buffers).
class ExplicitSweep {
   public:
    ExplicitSweep(kt_matrix_s* A, const DevCSR& M, int P, int m, uint64_t seed, int64_t probe_base, const double* x,
                  int ldx, int ncols, const double* dnorms2, double* rec_host, DevMat* basis,
                  std::vector<double>* scale_hist, int lane, int bcols);
    void start();
    void step(int j);
    void finish();

   private:
    kt_matrix_s* A;
    const DevCSR& M;
    int P, m;
    uint64_t seed;
    int64_t probe_base;
    const double* x;
    int ldx, ncols;
    const double* dnorms2;
    double* rec_host;
    DevMat* basis;
    std::vector<double>* scale_hist;
    int lane, bcols;
    int n = 0, grid = 0, lblocks = 0, grid1 = 0;
    size_t blk_bytes = 0;
    hipStream_t st = nullptr;
    double *part1 = nullptr, *part2 = nullptr, *k2s = nullptr, *coef = nullptr, *trec = nullptr, *Yb = nullptr;
    double *ucur = nullptr, *uprev = nullptr, *sc = nullptr, *sp = nullptr, *sn = nullptr, *bbase = nullptr;
    DevBuf* hist_dev = nullptr;
};

// lanczos_sweep_y (the RNG-seeded y-form sweep of the Hutchinson hot path)
// enqueued step by step: start(), step(j) for j < m - 1, finish().
class YSweep {
   public:
    YSweep(kt_matrix_s* A, const DevCSR& M, int P, int m, uint64_t seed, int64_t probe_base, double* rec_host,
           int lane);
    void start();
    void step(int j);
    void finish();

   private:
    double* rec_at(int row, int j) { return trec + (size_t)(row * m + j) * P; }
    kt_matrix_s* A;
    const DevCSR& M;
    int P, m;
    uint64_t seed;
    int64_t probe_base;
    double* rec_host;
    int lane;
    int n = 0, grid = 0, lblocks = 0, grid1 = 0, flags = 0;
    size_t blk_bytes = 0;
    hipStream_t st = nullptr;
    double *part = nullptr, *ys = nullptr, *trec = nullptr, *guard = nullptr;
    uint32_t* Z = nullptr;
    double *Xc = nullptr, *Yo = nullptr, *Ot = nullptr;
};

// lanczos_sweep_y_block enqueued step by step: start(), step(j) for j < m - 1,
// finish(); same interleaving rule as ExplicitSweep.
// With `basis` (m slots of n x P, slot j at basis + j n P; bcols > 0) the
// sweep also forms the normalised Lanczos vectors v_0 .. v_{m-1} of its
// first bcols columns there (KF_VB passes; v_0 is the start table itself).
class YBlockSweep {
   public:
    YBlockSweep(kt_matrix_s* A, const DevCSR& M, int P, int m, const double* x, int ldx, int ncols,
                const double* dnorms2, double* rec_host, int lane, double* basis = nullptr, int bcols = 0);
    void start();
    void step(int j);
    void finish();

   private:
    double* rec_at(int row, int j) { return trec + (size_t)(row * m + j) * P; }
    kt_matrix_s* A;
    const DevCSR& M;
    int P, m;
    const double* x;
    int ldx, ncols;
    const double* dnorms2;
    double* rec_host;
    int lane;
    int n = 0, grid = 0, lblocks = 0, grid1 = 0, flags = 0;
    size_t blk_bytes = 0;
    hipStream_t st = nullptr;
    double *part = nullptr, *ys = nullptr, *trec = nullptr, *guard = nullptr;
    double *V0 = nullptr, *Xc = nullptr, *Yo = nullptr, *Ot = nullptr;
    double* basis = nullptr;
    int bcols = 0;
    double* slot(int j) { return basis + (size_t)j * n * P; }
};

int record_tridiag(const double* R, int m, int P, int c, double* al, double* off);

// For the ncols columns of the device block X (n x ldx, natural row order):
// quad[c] = x_c' f(A) x_c by m-step Lanczos quadrature (may be NULL) and, if
// Y != NULL, Y[:, c] = ||x_c|| V_c f(T_c) e1 ~= f(A) x_c.
void lanczos_columns(kt_matrix_s* A, const double* X, int ldx, int ncols, int m, int fun,
                     double* quad, double* Y, int ldy);

// lanczos_columns for a block whose first ny columns need f(A) x (into Y)
// and every column its quadratic form: columns [0, ne) by the explicit CGS2
// sweep (sweeps of px columns, or pow2 >= ne capped at 16 when px = 0), the
// basis kept for the ny f(A)x columns; columns [ne, ncols) -- quadratic
// forms only -- by y-form sweeps (one pass per step, no K2, no basis) on the
// extra sweep lanes, all queued together.  A column's form depends only on
// the widths of the sweeps, which depend only on (ncols, ny, ne, px) -- not
// on the values (zero columns included).  The y-form suits random probes;
// columns that start close to an invariant subspace (mc_trace's Q) trip its
// cancellation guard and belong in [0, ne).
// ychunk: columns per y-form sweep (each sweep at the power of two >= its
// columns, <= 16): 16 packs them; a smaller chunk splits them evenly (mc_trace's
// final round: [Q | pad] and [G | pad] instead of 16 + 4).
// yb (<= ny): the first yb columns run as y-form sweeps that also form their
// Lanczos basis (KF_VB) instead of the explicit sweep: columns [0, yb) y-form
// with basis, [yb, ne) explicit, [ne, ncols) y-form forms only.  A y-form
// basis sweep whose guard trips is redone whole by the explicit sweep.
void lanczos_columns_split(kt_matrix_s* A, const double* X, int ldx, int ncols, int ny, int ne, int m, int fun,
                           double* quad, double* Y, int ldy, int px = 0, int ychunk = 16, int yb = 0);

// y-form sweep seeded by a device block (see kt_slq.cpp)
void lanczos_sweep_y_block(kt_matrix_s* A, const DevCSR& M, int P, int m, const double* x, int ldx, int ncols,
                           const double* dnorms2, double* rec_host, int lane);

}  // namespace kt
