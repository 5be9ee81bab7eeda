// kt_launch.h -- internal launcher declarations (kt_kernels.hip <-> runtime).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kt {

int spmm_grid(int n, int P, int max_blocks);
int long_blocks_for(int n_long, int max_blocks);

hipError_t launch_rademacher(int P, int n, uint64_t seed, int64_t probe_base, const int* perm,
                             double* X, hipStream_t st);
// probes probe_base .. probe_base + ncols - 1 as ncols (<= 64) columns of a
// row-major block with row stride ldx (natural row order)
hipError_t launch_rademacher_cols(int n, int ncols, uint64_t seed, int64_t probe_base, double* X, int ldx,
                                  hipStream_t st);
hipError_t launch_spmm_dot(int P, int flags, int grid, const int* rp, const int* ci,
                           const double* va, int n, const double* ucur, const double* sc,
                           double* y, double* partial, const int* long_rows, int n_long,
                           int long_thresh, int long_blocks, hipStream_t st);
// device CSR + its long-row list and hub-row chunk table (kt_internal.h DevCSR)
struct CsrView {
    const int* rp;
    const int* ci;
    const double* va;
    int n;
    const int* long_rows;
    int n_long, long_thresh, split_thresh;
    const int* ck_beg;
    const int* ck_end;
    int n_chunks;
    const int* sp_rows;
    const int* sp_first;
    int n_split;
    // natural CSR only: rows of degree <= kMedThresh as {row, beg, end, 0},
    // degree-descending (the row-blocked expmv term; nullptr elsewhere)
    const int* short_tasks = nullptr;
    int n_short = 0;
    // natural CSR only: the medium rows (med_rows) as {row, beg, end, 0}
    const int* med_tasks = nullptr;
    // the first n_heavy long rows have degree > kExpmvCoopThresh
    int n_heavy = 0;
};
constexpr int kExpmvCoopThresh = 256;  // expmv terms: a long row this heavy takes a whole workgroup
constexpr int kChunkNnz = 32;      // nonzeros per hub-row chunk
constexpr int kSplitThresh = 64;   // rows longer than this are chunked (block SpMM)
constexpr int kMedThresh = 16;     // expmv terms: rows longer than this get a wave (or a workgroup)
// One workgroup per greedy candidate runs its whole trace_fun_update (kt_pairs.hip
// k_pair_fused); vec: C x 3 x n x 2 doubles; big: C x big_stride doubles of
// eigen scratch, needed only when 2 it > 56 (else may be null); state: C x 8.
size_t pair_fused_lds_bytes(int it);
hipError_t launch_pair_fused(int C, int n, int64_t nnz, const CsrView& A, bool unit, const int* ii,
                             const int* jj, const double* B, int it, int fun, double tol, double* vec,
                             double* big, int64_t big_stride, double* state, hipStream_t st);
// device-resident greedy steps (kt_greedy.cpp): k_pair_reg with the CSR's
// {nnz, n_long} read from dyn (the LDS sized for nnz_max), and one step's
// selection + ranking update + edge deletion into the other CSR buffer
// k_pair_reg: the first kRegLongCap long rows (degree > long_thresh, in the
// CSR's long-row list order) are summed by whole waves, the rest by their
// owning threads -- so the list order is part of the kernel's arithmetic
constexpr int kRegLongCap = 256;
bool pair_reg_applies(int n, int64_t nnz, int it, int n_long, bool unit);
hipError_t launch_pair_reg_dyn(int C, int n, int64_t nnz_max, const CsrView& A, bool unit, const int* ii,
                               const int* jj, const double* B, int it, int fun, double tol, double* state,
                               const int* dyn, hipStream_t st);
hipError_t launch_greedy_edit(int C, const double* state, int* Ti, int* Tj, int nT, int n, int long_thresh,
                              const int* rp, const int* ci, const double* va, const int* lr, const int* dyn,
                              int* rp2, int* ci2, double* va2, int* lr2, int* dyn2, int step, int* sel,
                              double* selv, hipStream_t st);
hipError_t launch_spmm_block(int P, int flags, int grid, const CsrView& M, const double* X, int ldx,
                             double* Y, int ldy, int long_blocks, int chunk_blocks, double* ck_part,
                             hipStream_t st, int slices = 1, const int* skip = nullptr);
// hist (nullable): P doubles receiving the step's scale s_j (sc)
hipError_t launch_coef_cgs2(int P, const double* partial, int nblk, int first, const double* k2s,
                            const double* sc, const double* sp, double* coef, double* t_alpha,
                            double* t_up, double* hist, hipStream_t st);
// rec (optional): u_next's first bcols columns also to rec[row * bcols + c]
hipError_t launch_update(int P, int grid, int n, const double* y, double* uprev,
                         const double* ucur, const double* sc, const double* sp,
                         const double* coef, int first, double* partial, hipStream_t st,
                         bool nt = false, double* rec = nullptr, int bcols = 0);
hipError_t launch_norm(int P, const double* partial, int nblk, double* k2s, double* scale_next,
                       double* t_low, hipStream_t st);
// y-form probe Lanczos (one pass per step; slot-major partials [3P][grid]
// for launch_ycoef, the per-probe coefficient step).
// Vn != nullptr: also v_{j+1} = g y_j - a v_j - b v_{j-1} into basis slot Vn
// from slots Vc (v_j) and Vo (v_{j-1}, nullptr at j = 0), columns < bcols
// (every slot n x P, row-major)
hipError_t launch_spmm_lanczos(int P, int flags, int grid, const int* rp, const int* ci,
                               const double* va, int n, const double* X, const double* Yold,
                               double* Out, const double* coef, double* partial,
                               const int* long_rows, int n_long, int long_thresh, int long_blocks,
                               hipStream_t st, const double* Vc = nullptr, const double* Vo = nullptr,
                               double* Vn = nullptr, int bcols = 0);
hipError_t launch_rademacher_signs(int P, int n, uint64_t seed, int64_t probe_base,
                                  const int* perm, uint32_t* S, hipStream_t st);
hipError_t launch_spmm_lanczos_start(int P, int flags, int grid, const int* rp, const int* ci,
                                     const double* va, int n, const uint32_t* S, double s0,
                                     double* Out, double* partial, const int* long_rows, int n_long,
                                     int long_thresh, int long_blocks, hipStream_t st);
hipError_t launch_ycoef(int P, const double* partial, int nblk, int start, int last, double s0,
                        double* ys, double* t_alpha, double* t_up, double* t_low, double* guard,
                        hipStream_t st);
hipError_t launch_fill(double* x, int count, double v, hipStream_t st);
hipError_t launch_delay(double microseconds, hipStream_t st);
// sweep start scales from device column norms (kt_slq.cpp; mode 0 explicit: sc,
// k2s; mode 1 y-form: the 9P coefficient block) and a Gram block's diagonal
hipError_t launch_sweep_scales(const double* n2, int nc, int P, int mode, double* a, double* b, hipStream_t st);
hipError_t launch_gram_diag(const double* G, int ld, int nc, double* n2, hipStream_t st);
// out[i] = D[off[i]], i < count
// tall-skinny Gram / combine (kt_gemm_ts.hip)
int gram_ts_chunks(int64_t n);
hipError_t launch_gram_ts(int64_t n, const double* X, int ldx, int px, const double* Y, int ldy, int py,
                          double* part, double* G, hipStream_t st);
hipError_t launch_combine_ts(int64_t n, const double* X, int ldx, int px, const double* C, int q, double alpha,
                             double beta, double* Y, int ldy, hipStream_t st);
hipError_t launch_fro_colmax_scale(int n, double* M, double* out, double* colsq, hipStream_t st);
// device CholeskyQR factor: G + shift_coef tr(G) I = R' R, Rinv = R^-1 (bs <= 64); ok[0] = 0 on a failed pivot
hipError_t launch_chol_rinv(int bs, const double* G, double shift_coef, double* R, double* Rinv, int* ok,
                            hipStream_t st);
hipError_t launch_scatter_elems(int64_t count, const int64_t* off, const double* val, double* D,
                                hipStream_t st);
hipError_t launch_gather_elems(int64_t count, const double* D, const int64_t* off, double* out,
                               hipStream_t st);
// out (nr x cols, column-major) = rows[r] of the row-major block D (leading dimension ldd)
hipError_t launch_gather_rows(int nr, int cols, const double* D, int ldd, const int64_t* rows, double* out,
                              hipStream_t st);
// Y[r, c] = sum_j U[r * ldu + j * sstride + c] W[j * P + c]
hipError_t launch_weighted_sum(int n, int m, int P, int nc, const double* U, int ldu, int64_t sstride,
                               const double* W, double* Y, int ldy, hipStream_t st);
// dst[r] = src[perm[r]] (gather != 0) or dst[perm[r]] = src[r], rows of `cols` doubles
hipError_t launch_perm_rows(int n, int cols, const int* perm, int gather, const double* src, int lds,
                            double* dst, int ldd, hipStream_t st);
hipError_t launch_axpby(int n, int nc, double a, const double* X, int ldx, double b, double* Y,
                        int ldy, hipStream_t st);
int inf_norm_blocks();
// normest1 (t = 1) reductions, normest1_blocks(n) partials each: sum |Y| in
// partial[0, nb), S_prev . S in partial[nb, 2 nb), S = mysign(Y); per-block
// max |Z| and its smallest index
int normest1_blocks(int n);
hipError_t launch_normest1_y(int n, const double* Y, const double* Sprev, double* S, double* partial,
                             hipStream_t st);
hipError_t launch_absmax_idx(int n, const double* Z, double* pval, int* pidx, hipStream_t st);
// batched greedy candidates (kt_pairs.hip)
hipError_t launch_pair_select(int C, const int* ii, const int* jj, double* X, int ld,
                              hipStream_t st);
// CGS2 of W against [prev cur] (cur == nullptr: none) + Householder thin QR,
// per candidate; hr[c*11 + 0..10] = (h [8], R11, R12, R22)
hipError_t launch_pairs_orth(int C, int n, int num_cu, const double* prev, const double* cur,
                             double* W, int ld, double* coef, double* part, double* hr,
                             hipStream_t st,
                             const int* skip = nullptr);
size_t pairs_part_doubles(int n, int C, int num_cu);
// per-candidate projected eigenproblems + stop logic; state C x 8 doubles
hipError_t launch_pair_eig(int C, int j, int it, int fun, double tol, const double* hist,
                           const double* Cm, double* scratch, int64_t sstride, double* state,
                           int* active, hipStream_t st);
// tall-skinny Householder QR (kt_tsqr.hip)
int ts_nrb(int n, int num_cu);
hipError_t launch_ts_reflectors(int n, int bs, int BP, double* W, int ld, double* V, double* pivot,
                                double* sums, double* part, double* taus, int num_cu,
                                hipStream_t st);
// one launch per column (k_ts_step1): ts_step1_grid > 0 when it applies;
// part: 2 * BP * grid doubles, piv: 2 * BP doubles
int ts_step1_grid(int n, int* rows_per_wg);
hipError_t launch_ts_reflectors1(int n, int bs, int BP, double* W, int ld, double* V, double* part, double* piv,
                                 double* taus, hipStream_t st);
hipError_t launch_ts_formq(int n, int bs, int BP, const double* V, const double* M, double* W,
                           int ld, hipStream_t st);
hipError_t launch_sum_slabs(int count, int S, const double* part, double* G, hipStream_t st);
hipError_t launch_poly4(int n, double beta, const double* in, double c0, double c1, const double* X1,
                        double c2, const double* X2, double c3, const double* X3, double* out,
                        hipStream_t st,
                        int batch = 1);
// column-batched single-vector Arnoldi (kt_colbatch.hip); V blocks at stride vstride
int col_nrb(int n, int num_cu, int rpb_lo = 64);
hipError_t launch_col_dots(int n, int P, int nb, int64_t vstride, const double* V, const double* W,
                           int r_lo, int num_cu, double* part, double* out, hipStream_t st, int rpb_lo = 64);
hipError_t launch_col_update(int n, int P, int nb, int64_t vstride, const double* V,
                             const double* h, double* W, hipStream_t st);
hipError_t launch_col_householder(int n, int P, const double* s, double* W, double* Q, double* r,
                                  hipStream_t st);
hipError_t launch_col_select(int C, int P, const int* idx, double* X, hipStream_t st);
size_t pairs_coef_doubles(int C);
hipError_t launch_inf_norm(int n, int nc, const double* X, int ldx, double* partial,
                           hipStream_t st);
// expmv Taylor stage with the stop test on the device (state: expmv_state_bytes();
// layout {int active; int mv; double c1;}); partial: 2 * inf_norm_blocks() doubles
size_t expmv_state_bytes();
hipError_t launch_expmv_begin(const double* partial, int nb, void* state, hipStream_t st);
hipError_t launch_expmv_term(int n, int nc, double mu, double coef, const double* Ab, double* b,
                             double* F, int ld, double* partial, const void* state, hipStream_t st);
hipError_t launch_expmv_check(int n, const double* partial, double tol, void* state, hipStream_t st);
// one fused launch per Taylor term k (P = pow2 >= nc, P <= 32, ld >= P): the
// check of term k-1, SpMM of the natural-order CSR (M), update, the maxima
// of term k's row sums folded into the state (term_max slot k % 3)
// waves: per block (0: the per-term kernel's)
int expmv_step_blocks(int n, int P, int n_long, int n_med, int waves = 0);
// the default form of launch_expmv_step for this shape (true: SPLIT, grids
// above 1,024 workgroups); with split the host launches
// launch_expmv_slot_check after every term but a stage's last.
// launch_expmv_step form: 0 fused, 1 split (a workgroup per row class unit),
// 2 row-blocked (k_expmv_rows: resident workgroups) with the stop test in
// k_expmv_slot_check, 3 row-blocked with the stop test of term k - 1 at the
// start of term k (no slot-check launch; the default on large grids)
bool expmv_split_check(int n, int P, int n_long, int n_med);
hipError_t launch_expmv_slot_check(void* state, int k, double tol, hipStream_t st, int* hflag, int stage);
hipError_t launch_expmv_step(int P, bool unit, const CsrView& M, const int* med_rows, int n_med, int nc,
                             int ld, double mu, double coef,
                             double tol, int k, const double* bin, double* bout, double* F,
                             void* state, hipStream_t st, int form, int* hflag = nullptr, int stage = 0);

}  // namespace kt
