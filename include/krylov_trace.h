/* krylov_trace.h -- C ABI of libkrylov_hip.so, the MI355X trace(f(A)) evaluator.
 *
 * This is the drop-in boundary of SURVEY.md §8b.  The reference is MATLAB;
 * its callers (Tests/ scripts, greedy_krylov.m, fmincon closures) resolve the
 * functions below by name, so a MEX file of the same name placed in
 * functions/ shadows the .m (krylov_robustness_amd/mex/).
 * The MEX shim forwards mxArray data to these plain-pointer entry points; the
 * ctypes binding in krylov_robustness_amd/_lib.py binds the same symbols for
 * tests.
 *
 * Conventions
 *   - All functions return an int status (KT_OK == 0).  On failure a
 *     thread-local message is available from kt_last_error(); messages
 *     reproduce the reference's error strings where one exists.
 *   - Matrices: MATLAB sparse CSC (mwIndex = int64 jc[n+1], ir[nnz], 0-based;
 *     double pr[nnz]).  A is symmetric on every hot path, so CSC == CSR.
 *   - Dense arrays are column-major fp64 (MATLAB layout); Omega is 1-based.
 *   - Inputs are borrowed (read-only); outputs are caller-allocated.
 *   - A context is externally synchronised: no concurrent calls on one
 *     context (MATLAB calls a MEX on its single interpreter thread).
 *   - fun codes mirror fun_update.m:43-59's handle identities.
 */
#ifndef KRYLOV_TRACE_H
#define KRYLOV_TRACE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KT_ABI_VERSION 3

enum kt_status {
    KT_OK = 0,
    KT_ERR_ARG = 1,           /* bad argument (sizes, null pointers)            */
    KT_ERR_HIP = 2,           /* HIP runtime failure                            */
    KT_ERR_NOT_HERMITIAN = 3, /* fun_and_grad_krylov_exp.m:21-23                */
    KT_ERR_NOT_SQUARE = 4,    /* lanczos_krylov.m:36-38                         */
    KT_ERR_ALLOC = 5,         /* device allocation failed                       */
    KT_ERR_UNSUPPORTED = 6,   /* size / option outside what the build supports  */
    KT_ERR_CALLBACK = 7       /* a caller-supplied callback returned non-zero   */
};

enum kt_fun { /* fun_update.m:43-59 */
    KT_FUN_EXP = 0,
    KT_FUN_SINH = 1,
    KT_FUN_COSH = 2,
    KT_FUN_SIN = 3,
    KT_FUN_COS = 4,
    KT_FUN_LOG = 5,
    KT_FUN_SQRT = 6
};

typedef struct kt_context_s* kt_context_t;
typedef struct kt_matrix_s* kt_matrix_t;

/* ---- runtime ------------------------------------------------------------ */
int kt_abi_version(void);
const char* kt_last_error(void);
int kt_device_count(int* count);
int kt_context_create(int device, kt_context_t* ctx);
int kt_context_destroy(kt_context_t ctx);

/* Device-resident A (SURVEY.md §7 hard part (e): fmincon and greedy call the
 * shim repeatedly with the same A, so the CSR stays in HBM across calls).
 * Replaces the sparse `A` argument of trace_exp.m:1, mc_trace.m:32-34,
 * trace_fun_update.m:1, fun_update.m:1, fun_and_grad_krylov_exp.m:1,
 * fun_and_grad_krylov_fun.m:1.  `check_symmetric` != 0 rejects a
 * non-symmetric A with KT_ERR_NOT_HERMITIAN. */
int kt_matrix_create_csc(kt_context_t ctx, int64_t n, const int64_t* colptr,
                         const int64_t* rowind, const double* vals, int check_symmetric,
                         kt_matrix_t* A);
int kt_matrix_destroy(kt_matrix_t A);
int kt_matrix_info(kt_matrix_t A, int64_t* n, int64_t* nnz);

/* ---- hot path: stochastic Lanczos quadrature ------------------------------
 * For probes p in [probe_offset, probe_offset + nprobes) (Rademacher,
 * splitmix64 stream keyed by the GLOBAL probe index, so any sharding over
 * GPUs gives the same probes), run m steps of the single-vector
 * lanczos_krylov recurrence (lanczos_krylov.m:73-115, bs = 1) and form
 * q_p = ||z||^2 e1' f(T_m) e1.  Returns sum_p q_p and sum_p q_p^2 (for the
 * all-reduce of partial traces and the variance), and optionally q[nprobes].
 * `block` = probes per SpMM sweep (power of two 1..128; 0 = auto).
 * This is the Afun of mc_trace.m:45-49 evaluated as quadratic forms and the
 * plain-Hutchinson estimator of BASELINE.json configs 2-4. */
int kt_slq_trace(kt_matrix_t A, int fun, int m, uint64_t seed, int64_t probe_offset,
                 int64_t nprobes, int block, double* sum_q, double* sum_q2, double* q);

/* kt_slq_trace in two halves, for a pipeline of evaluations: submit queues
 * the probe sweeps on the device and returns at once with a ticket; collect
 * waits for THAT call's sweeps only (not for work submitted after it), runs
 * the guard redo and the host quadrature and returns what kt_slq_trace
 * returns.  So evaluation k + 1's sweeps run on the device while the host
 * finishes evaluation k.  At most two submissions outstanding per context,
 * collected once each in submission order (KT_ERR_ARG otherwise);
 * kt_slq_trace == submit + collect and refuses to run while submissions are
 * outstanding. */
int kt_slq_submit(kt_matrix_t A, int fun, int m, uint64_t seed, int64_t probe_offset, int64_t nprobes,
                  int block, int* ticket);
int kt_slq_collect(kt_matrix_t A, int ticket, double* sum_q, double* sum_q2, double* q);

/* The probes-per-sweep width kt_slq_trace picks when block == 0. */
int kt_slq_plan(kt_matrix_t A, int64_t nprobes, int* block);

/* ---- block-Krylov entry points (bs = number of columns of U, <= 128) ------
 * U: n x rk column-major in ORIGINAL row numbering; B: rk x rk column-major.
 * it <= 0 selects the reference default min(100, n). */

/* MATLAB normest(A, tol): power estimate of ||A||_2 (called with tol 1e-2 at
 * fun_and_grad_krylov_exp.m:26 / fun_and_grad_krylov_fun.m:27). */
int kt_normest(kt_matrix_t A, double tol, double* nrm);

/* [Xm, iter, lucky] = trace_fun_update(A, U, B, tol, it, debug, fun)
 * (trace_fun_update.m:1): tr f(A + U B U') - tr f(A) by block Lanczos seeded
 * with U (lanczos_krylov.m), lag-2 stopping, dense path when n <= 130. */
int kt_trace_fun_update(kt_matrix_t A, int64_t rk, const double* U, const double* B, double tol,
                        int it, int fun, double* Xm, int* iter, int* lucky);

/* Elementwise scalar function for a function handle outside enum kt_fun:
 * y[i] = f(x[i]), i < count; called on the host, on the calling thread.
 * Returns 0 on success; any other value aborts the call, which then returns
 * KT_ERR_CALLBACK (the partial result is discarded, never summed). */
typedef int (*kt_scalar_fn)(const double* x, double* y, int64_t count, void* user);

/* trace_fun_update with an arbitrary elementwise handle (trace_fun_update.m:
 * 85-89 `Xm = sum(fun(d1) - fun(d2))`; the same call as kt_trace_fun_update
 * otherwise): f is applied to the two sorted eigenvalue vectors of each
 * projected pair (tGm, Gm), or of A + UBU' and A on the dense path. */
int kt_trace_fun_update_fn(kt_matrix_t A, int64_t rk, const double* U, const double* B, double tol,
                           int it, kt_scalar_fn f, void* user, double* Xm, int* iter, int* lucky);

/* [Xm, iter, lucky, Um] = fun_update(A, U, B, fun, tol, it, debug) with four
 * outputs (fun_update.m:1, Arnoldi branch :77-91): f(A+UBU') - f(A) ~= Um Xm Um'.
 * Xm is ncols x ncols (column-major, buffer of max_cols^2 doubles); Um (may be
 * NULL) is n x ncols.  When the basis reaches n/2 columns the reference's
 * dense fallback applies (:85-90): Um = eye(n), ncols = n. */
int kt_fun_update(kt_matrix_t A, int64_t rk, const double* U, const double* B, int fun, double tol,
                  int it, int64_t max_cols, double* Xm, int64_t* ncols, int* iter, int* lucky,
                  double* Um);

/* [Xm, iter, lucky] = fun_update(A, U, B, fun, tol, it, debug) with at most
 * three outputs (fun_update.m:69-76: the block-Lanczos branch over
 * lanczos_krylov's 2-block window; Xm = f(tGm) - f(Gm) on the projected
 * block tridiagonal, 2-norm lag-2 stop, no dense fallback).  Xm: ncols x
 * ncols column-major (buffer of max_cols^2).  The reference then evaluates
 * Um(:, 1:size(Xm, 1)) on the n x 2rk window (fun_update.m:137), which errors
 * once ncols > 2 rk; that error is the caller's (the MEX shim raises it). */
int kt_fun_update_lanczos(kt_matrix_t A, int64_t rk, const double* U, const double* B, int fun,
                          double tol, int it, int64_t max_cols, double* Xm, int64_t* ncols, int* iter,
                          int* lucky);

/* [f, gr] = fun_and_grad_krylov_exp(X, A, Omega, eA, tol, it, debug)
 * (fun_and_grad_krylov_exp.m:1).  Omega: nomega x 2 column-major, 1-based
 * (MATLAB doubles); X, eA, gr: nomega.  KT_ERR_NOT_HERMITIAN if A is not
 * symmetric ("FUN_AND_GRAD_KRYLOV:: matrix A is not Hermitian"). */
int kt_fun_and_grad_krylov_exp(kt_matrix_t A, int64_t nomega, const double* X, const double* Omega,
                               const double* eA, double tol, int it, double* f, double* gr);

/* [f, gr] = fun_and_grad_krylov_fun(X, A, Omega, fun, dfun, dfA, tol, it, debug, fun_M)
 * (fun_and_grad_krylov_fun.m:1); fun / dfun are kt_fun codes. */
int kt_fun_and_grad_krylov_fun(kt_matrix_t A, int64_t nomega, const double* X, const double* Omega,
                               int fun, int dfun, const double* dfA, double tol, int it, double* f,
                               double* gr);

/* ---- mc_trace / trace_exp / expmv --------------------------------------- */
enum kt_afun { /* the Afun argument of mc_trace.m:1 */
    KT_AFUN_MATRIX = 0,  /* Afun is the matrix itself (mc_trace.m:32-34)              */
    KT_AFUN_LANCZOS = 1, /* f(A) x by m-step Lanczos (north star)   */
    KT_AFUN_EXPMV = 2    /* @(x) expmv(1, A, x, [], 'double') (trace_exp.m:5)          */
};

/* [tr, res, it] = mc_trace(Afun, n, tol, maxit, isAreal, debug) (mc_trace.m:1):
 * block Hutchinson, m = 10 columns per round, K = ceil(maxit/30) rounds with
 * nested deflation (mc_trace.m:41-58).  Probes of round it are Rademacher
 * columns (it-1)*20 + [0,10) (S) and + [10,20) (G) of the counter RNG. */
int kt_mc_trace(kt_matrix_t A, int afun, int fun, int m, double tol, int maxit, int isAreal,
                uint64_t seed, double* tr, double* res, int* it);

/* All-reduce (sum) of `count` doubles in place across the ranks of a job;
 * supplied by the caller (torch.distributed / RCCL, MPI, ...).  0 = ok. */
typedef int (*kt_reduce_fn)(double* buf, int64_t count, void* user);

/* mc_trace on `world` GPUs (Hutch++ structure): every rank
 * recomputes S, Q and tr(Q' Afun Q) from the shared seed; the 10 G-probe
 * columns of each round are dealt round-robin (column c to rank c % world),
 * their quadratic forms all-reduced with `allreduce` (one call per round,
 * count = 10) and summed in column order, so every rank returns the same
 * tr / res / it.  KT_AFUN_EXPMV is computed replicated (its Taylor degree is
 * chosen per block, expmv.m:41) and never calls `allreduce`.  Replaces
 * mc_trace.m:1-63 on a multi-GPU node; world = 1 equals kt_mc_trace (with a
 * non-NULL `allreduce` the round sums still pass through it, bit-identically;
 * `allreduce` may be NULL only at world = 1). */
int kt_mc_trace_sharded(kt_matrix_t A, int afun, int fun, int m, double tol, int maxit,
                        int isAreal, uint64_t seed, int rank, int world, kt_reduce_fn allreduce,
                        void* user, double* tr, double* res, int* it);

/* tr = trace_exp(A) (trace_exp.m:1-7) = mc_trace(Afun, n, 1e-4, 1000, 1) with
 * Afun = KT_AFUN_EXPMV (the reference composition) or KT_AFUN_LANCZOS (m steps). */
int kt_trace_exp(kt_matrix_t A, int afun, int m, uint64_t seed, double* tr);

/* [F, s, m, mv] = expmv(t, A, B, [], 'double') (expmv.m:1-94; degree selection
 * select_taylor_degree.m, normAm.m for A >= 0).  B, F: n x ncols column-major. */
int kt_expmv(kt_matrix_t A, double t, int64_t ncols, const double* B, double* F, int* s, int* mdeg,
             int* mv);

/* Y = f(A) X by per-column m-step Lanczos: y = ||x|| V f(T) e1 (the Lanczos-f
 * Afun handle).  X, Y: n x ncols column-major, ncols <= 128. */
int kt_lanczos_fmv(kt_matrix_t A, int fun, int m, int64_t ncols, const double* X, double* Y);

/* [Q, R] = qr(W, 0) on the device (MATLAB's economy Householder QR: LAPACK
 * reflector signs, tau = 0 completions of exactly dependent columns), the
 * factorisation lanczos_krylov.m:90, arnoldi_krylov.m:99 and mc_trace.m use.
 * W, Q: n x bs column-major, R: bs x bs column-major, 1 <= bs <= 128. */
int kt_householder_qr(kt_context_t ctx, int64_t n, int64_t bs, const double* W, double* Q,
                      double* R);

/* Host symmetric eigensolver used for the small projected matrices (the
 * m x m / 2j x 2j eig of trace_fun_update.m:83-84, lanczos quadrature):
 * Householder tridiagonalisation + implicit QL.  A: n x n column-major
 * (symmetric), w: n eigenvalues (unsorted), V: n x n eigenvectors or NULL.
 * Pure host code (no device needed). */
int kt_host_sym_eig(int n, const double* A, double* w, double* V);

/* Host Gauss quadrature of one probe's m x m symmetric tridiagonal T
 * (alpha: m diagonal entries, off: m - 1 off-diagonal ones), the per-probe
 * step after every sweep (trace_fun_update.m:78-84 restated for a single
 * vector: e1' f(T) e1 = sum_k tau_k^2 f(theta_k)): one implicit-shift QL pass
 * rotating the first row of the eigenvector matrix.  q: e1' f(T) e1; fe1
 * (m, nullable): f(T) e1, from the same pass by replaying its rotations (the
 * weights of the Lanczos-f Afun, f(A) x = ||x|| V f(T) e1).  fun: KT_FUN_*.
 * Pure host code (no device needed). */
int kt_host_tridiag_quad(int m, const double* alpha, const double* off, int fun, double* q, double* fe1);

/* ---- greedy edge selection (krylov_miobi.m / greedy_krylov.m) ---------- */

/* Batched trace_fun_update over candidate edges, the inner loop of
 * krylov_miobi.m:76-99.  Candidate c (0-based node indices ei[c], ej[c]):
 *   ei != ej : U = [e_ei, e_ej], B (2 x 2 column-major, Hermitian)
 *   ei == ej : U = e_ei,         B = b_self
 * Xm[c] = tr f(A + U B U') - tr f(A) estimated exactly as trace_fun_update.m
 * does (tol, it, lag-2 stop, lucky breakdown, dense shortcut n <= 130);
 * iter, lucky (nullable) as trace_fun_update's outputs.  Replaces ncand
 * calls of trace_fun_update.m:1 from krylov_miobi.m:99. */
int kt_trace_fun_update_pairs(kt_matrix_t A, int64_t ncand, const int64_t* ei, const int64_t* ej,
                              const double* B, double b_self, double tol, int it, int fun,
                              double* Xm, int* iter, int* lucky);

/* krylov_miobi.m:1 with E given as 0-based pairs (E(j,1) >= E(j,2) in the
 * reference's 1-based form).  make = 0 ('break') or 1 ('make'); rescale as
 * krylov_miobi.m:78-84 (B = -+[0 1;1 0]/rescale).  A is edited IN PLACE
 * (A(i,j) = A(j,i) = 0 or 1, krylov_miobi.m:129-135), the returned A_new.
 * sel_i/sel_j (capacity min(k, nE), nullable) receive the chosen edges in
 * order, rob the summed variation, nsel their count.  Errors: the
 * reference's KRYLOV_MIOBI:: messages. */
int kt_krylov_miobi(kt_matrix_t A, int k, int64_t nE, const int64_t* ei, const int64_t* ej,
                    double tol, int it, int make, double rescale, int64_t* sel_i, int64_t* sel_j,
                    double* rob, int64_t* nsel);

/* The step loop of greedy_krylov.m:64-93 once its search space is ranked
 * (find_top_edges / find_top_missing_edges, greedy_krylov.m:82): ntop >= k
 * ranked pairs ti/tj (0-based).  Step s runs krylov_miobi(A, 1, E, tol, it,
 * ...) on E = the first Q remaining pairs (one selection, A edited in place,
 * :89) and drops the selected pair from the ranking (first match, :84-86).
 * sel_i/sel_j (capacity k, nullable) receive the chosen edges, rob the summed
 * variation (:90), nsel their count.  Replaces the per-step host round trips
 * of calling kt_krylov_miobi k times; same results. */
int kt_greedy_krylov_steps(kt_matrix_t A, int k, int64_t Q, int64_t ntop, const int64_t* ti,
                           const int64_t* tj, double tol, int it, int make, double rescale, int64_t* sel_i,
                           int64_t* sel_j, double* rob, int64_t* nsel);

/* A(i,j) = A(j,i) = value for each pair (value 0 removes the entry, as MATLAB
 * sparse assignment does); device copies are refreshed. */
int kt_matrix_set_pairs(kt_matrix_t A, int64_t count, const int64_t* ei, const int64_t* ej,
                        double value);
/* Copy A back out as CSC (colptr n+1, rowind/vals nnz; sizes from
 * kt_matrix_info).  rowind / vals may be NULL. */
int kt_matrix_export_csc(kt_matrix_t A, int64_t* colptr, int64_t* rowind, double* vals);

/* ---- entries of f(A) (function_multiple_entries.m) -------------------- */

/* X[h] ~= f(A)(oi[h], oj[h]) for h < k (0-based indices) by one Arnoldi run
 * per distinct row index (function_multiple_entries.m:1 with poles = inf);
 * tol / it as the reference (lag-3 stop on f(Gm) e1, it <= 0: min(100, n));
 * iter (nullable) = Krylov steps taken.  Replaces
 * function_multiple_entries.m:1 (Tests/test_weighted_*.m:52-77). */
int kt_function_multiple_entries(kt_matrix_t A, int64_t k, const int64_t* oi, const int64_t* oj,
                                 int fun, double tol, int it, double* X, int* iter);

/* ---- Frechet derivatives and Hessians (multiple_frechet_eval.m,
 *      hessianfcn_exp.m, hessianfcn_fun.m) ----------------------------- */

/* out[h + t * k] = Df(A)(e_oi[h] e_oj[h]')(ti[t], tj[t]) for h < k, t < ntarget
 * (0-based), i.e. the reference's Um{row(i)}(ti, :) * Xm{h} * Vm{col(j)}(tj, :)'
 * from multiple_frechet_eval.m:1 (poles = inf, same tol / it / lag-3 stop).
 * A must be symmetric (the Hessians' A + XX + XX' are).  iter nullable. */
int kt_frechet_entries(kt_matrix_t A, int64_t k, const int64_t* oi, const int64_t* oj, int fun,
                       double tol, int it, int64_t ntarget, const int64_t* ti, const int64_t* tj,
                       double* out, int* iter);

/* Hes = hessianfcn_exp(X, A, Omega, tol, it) (fun = KT_FUN_EXP) or
 * hessianfcn_fun(X, A, Omega, f, tol, it): Omega nomega x 2 column-major,
 * 1-based (MATLAB doubles), X nomega, Hes nomega x nomega column-major.
 * Replaces hessianfcn_exp.m:1 / hessianfcn_fun.m:1 (fmincon HessianFcn). */
int kt_hessianfcn(kt_matrix_t A, int64_t nomega, const double* X, const double* Omega, int fun,
                  double tol, int it, double* Hes);

/* Leading eigenpair of symmetric A (compute_centrality.m:15-17: [u, lambda]
 * = eigs(A, 1); centrality = abs(u)): full-reorthogonalisation Arnoldi on
 * the device from the ones vector, restarted from the Ritz vector, residual
 * |h(j+1,j) y(j)| <= tol |lambda| (tol <= 0: machine epsilon); maxit = Krylov
 * steps per restart (<= 0: 300).  v (n, nullable): unit 2-norm, sum(v) >= 0.
 * steps (nullable): total Arnoldi steps.  Largest algebraic eigenvalue (the
 * Perron root of an adjacency matrix). */
int kt_eigs_leading(kt_matrix_t A, double tol, int maxit, double* lambda, double* v, int* steps);

/* Per-kernel timing (HIP events recorded on the library's stream around each
 * launch of the named kernel while enabled).  kernel: 0 = the probe-Lanczos
 * gather pass (k_spmm_lanczos in the y-form sweep, k_spmm_dot = K1 in the
 * explicit sweep), 1 = K2 (k_update, explicit sweep only), 2 = the y-form
 * start pass (k_spmm_lanczos_start), 3 = the y-form pass of a sweep seeded
 * by a given block (k_spmm_lanczos in mc_trace's quadrature-only columns),
 * 4 = the expmv Taylor-term kernel (k_expmv_rows / k_expmv_step, one launch
 * per term; a term queued past its stage's stop is a short no-op launch).
 * Returns launch count and summed milliseconds. */
int kt_profile_enable(kt_context_t ctx, int enable);
int kt_profile_read(kt_context_t ctx, int kernel, int64_t* launches, double* total_ms);
int kt_profile_reset(kt_context_t ctx);
/* The same totals restricted to launches of sweep width `width` (the probe
 * block P of the sweep that launched them). */
int kt_profile_read_width(kt_context_t ctx, int kernel, int width, int64_t* launches, double* total_ms);
/* Wall time during which at least one launch of `kernel` was in flight (the
 * union of the launches' event intervals, on whichever sweep-lane stream
 * each ran): with several lanes overlapping, summed per-launch durations
 * count shared time twice; this does not. */
int kt_profile_busy(kt_context_t ctx, int kernel, double* busy_ms);

/* Test hook: queue a kernel that keeps sweep lane `lane` (0 = the context's
 * stream, 1..3 = the extra sweep-lane streams kt_slq_submit uses) busy for
 * `microseconds` (<= 1e6) and return at once.  Lets a test make one lane's
 * sweeps finish after another's (the profiler's out-of-order completion). */
int kt_debug_delay(kt_context_t ctx, int lane, double microseconds);

/* Hot-path statistics.  stat 0: kt_slq_trace sweeps whose y-form probe
 * Lanczos tripped the cancellation guard (a lucky breakdown, or a beta^2
 * below 1e-4 ||A v||^2) and were recomputed by the explicit CGS2 sweep,
 * counted since context creation.  stat 1: fun_update runs (kt_fun_update,
 * kt_fun_and_grad_krylov_*) that took the dense fallback of fun_update.m:85-90,
 * since context creation.  stat 2: the projected size (basis columns) of the
 * last fun_update run on this context (n when it went dense).  stat 3: expmv
 * calls (kt_expmv and mc_trace's expmv Afun), stat 4: the Taylor terms they
 * executed (one A b product on the block each, expmv.m:75), since context
 * creation. */
int kt_context_stat(kt_context_t ctx, int stat, int64_t* value);

/* Threads of the process-wide host pool (the per-column / per-candidate
 * host work between device steps: Gauss quadratures, the greedy host
 * eigenproblems), the calling thread included: min(16, the CPUs this
 * process may use -- its affinity mask capped by the cgroup CPU quota --
 * divided by LOCAL_WORLD_SIZE, the ranks torchrun started on this node),
 * at least 1; KT_HOST_THREADS overrides.  Fixed at the pool's first use. */
int kt_host_threads(void);

#ifdef __cplusplus
}
#endif
#endif /* KRYLOV_TRACE_H */
