// kt_internal.h -- shared internals of libkrylov_hip.so (not part of the ABI).
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/krylov_trace.h"

struct kt_matrix_s;

// KT_DIAG (compile time, `make EXTRA=-DKT_DIAG=1`): the host-side phase
// clocks of the block-Krylov, eigensolver and greedy drivers print to stderr
// (2: every eigensolve too).  0 in every product build.
#ifndef KT_DIAG
#define KT_DIAG 0
#endif

namespace kt {

void set_error(const std::string& msg);

struct Status {  // exception carrying a kt_status; caught at the ABI edge
    int code;
    std::string msg;
};

[[noreturn]] inline void fail(int code, const std::string& msg) { throw Status{code, msg}; }

#define KT_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            ::kt::fail(KT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

// Growable device buffer (bytes); owns its allocation (move-only).
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : ptr(o.ptr), bytes(o.bytes) { o.ptr = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); ptr = o.ptr; bytes = o.bytes; o.ptr = nullptr; o.bytes = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void ensure(size_t want) {
        if (want <= bytes) return;
        // geometric growth below 64 MB (hipFree synchronises the device)
        if (want < ((size_t)64 << 20)) want = std::max(want, std::max<size_t>(2 * bytes, 64 << 10));
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&ptr, want);
        if (e != hipSuccess) fail(KT_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
        bytes = want;
    }
    template <class T> T* as() { return static_cast<T*>(ptr); }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

// Device scratch blocks recycled per context (behind DevMat, kt_block.h):
// hipFree synchronises the whole device, so block-Krylov calls that allocate
// their bases per call stalled the host at every return (config 1's expmv
// composition: 85 us gaps before each re-allocation's fill, tools/gaps.py).
// Blocks return to the context's free list and are reused by later calls on
// the same stream (stream order makes the reuse safe); freed at context
// destruction.
struct ScratchPool {
    std::vector<std::pair<size_t, void*>> free;  // (bytes, ptr), reusable now
    size_t held = 0;                             // bytes owned (free + in use)
    // a block of >= want bytes (best fit within 4x, else a new allocation)
    void* take(size_t want, size_t* got);
    void give(void* p, size_t bytes);
    void clear();
    ~ScratchPool() { clear(); }
};

struct PinnedBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    ~PinnedBuf() { release(); }
    void ensure(size_t want) {
        if (want <= bytes) return;
        // grow geometrically below 64 MB: a buffer that follows a growing
        // basis (one more block per Krylov step) was freed and re-pinned every
        // step, and hipHostFree costs ~0.25 ms with the device synchronised
        if (want < ((size_t)64 << 20)) want = std::max(want, std::max<size_t>(2 * bytes, 64 << 10));
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
        hipError_t e = hipHostMalloc(&ptr, want, hipHostMallocDefault);
        if (e != hipSuccess) fail(KT_ERR_ALLOC, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        bytes = want;
    }
    template <class T> T* as() { return static_cast<T*>(ptr); }
    void release() {
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
};

struct ProfSlot {
    std::vector<hipEvent_t> ev;  // start/stop pairs
    size_t used = 0;             // events used (2 per launch)
    size_t done = 0;             // events already folded into the totals (prof_collect)
    int64_t launches = 0;
    double total_ms = 0.0;
    // every folded launch's [start, stop] in ms after `anchor` (recorded before
    // the slot's first launch since the last reset): the union is formed over
    // ALL of them when read, so launches of consecutive batches that overlap
    // in time (pipelined calls, several lanes) are counted once
    std::vector<std::pair<double, double>> iv;
    hipEvent_t anchor = nullptr;
    bool anchored = false;
    // a tag per recorded launch not folded in yet (the sweep width P), and
    // the folded launches / milliseconds per tag
    std::vector<int> tags;
    std::vector<std::pair<int, std::pair<int64_t, double>>> by_tag;
};

enum { PROF_SPMM = 0, PROF_UPDATE = 1, PROF_START = 2, PROF_YBLOCK = 3, PROF_EXPMV = 4, PROF_NSLOTS = 5 };

// Buffers of one probe-sweep lane (kt_slq.cpp); two lanes let two sweeps
// run on two streams.
struct SweepBufs {
    DevBuf X0, X1, Y, partial, coef, scales, k2s, trec, hist;  // hist: the explicit sweep's scale history
};

// one host int the device may store to at system scope (fine-grained,
// coherent pinned memory): read by the host without a stream sync
struct HostFlag {
    int* host = nullptr;
    int* dev = nullptr;
    HostFlag() = default;
    HostFlag(const HostFlag&) = delete;
    HostFlag& operator=(const HostFlag&) = delete;
    ~HostFlag() {
        if (host) (void)hipHostFree(host);
    }
    void ensure() {
        if (host) return;
        void* p = nullptr;
        hipError_t e = hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped);
        if (e != hipSuccess) fail(KT_ERR_ALLOC, std::string("hipHostMalloc(coherent): ") + hipGetErrorString(e));
        void* d = nullptr;
        e = hipHostGetDevicePointer(&d, p, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(p);
            fail(KT_ERR_HIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
        }
        host = static_cast<int*>(p);
        dev = static_cast<int*>(d);
    }
};

// One kt_slq_submit call awaiting its host half (kt_slq_collect): the
// parameters, its host record slot and one event per sweep lane recorded
// after the lane's last record copy.
struct SlqPending {
    bool live = false;
    const kt_matrix_s* A = nullptr;  // the submitting matrix (collect must name it)
    int fun = 0, m = 0, P = 1, lanes = 1;
    uint64_t seed = 0;
    int64_t offset = 0, nprobes = 0, nsweeps = 0;
    size_t rec = 0;
    hipEvent_t done[4] = {nullptr, nullptr, nullptr, nullptr};
};

struct Workspace {
    SweepBufs sweep[4];
    HostFlag expmv_stop;  // the stage a k_expmv_step launch found stopped (expmv_device)
    DevBuf small, small2, qrtmp, qrkeep, qrfac, eigA, eigW, eigInfo;  // block-Krylov scratch
    DevBuf expm;                                       // batched device expm (6 x batch x n^2)
    DevBuf ck_part;                                    // block SpMM hub-row chunk partials
    DevBuf norm_part;                                   // inf-norm partials
    DevBuf expmv_state;                                 // expmv stage stop state (device)
    PinnedBuf host_trec[2];  // sweep records of the (at most two) submitted kt_slq calls
    SlqPending slq_pend[2];
    uint64_t slq_submitted = 0, slq_collected = 0;
    PinnedBuf pin_small;  // block-Krylov Gram blocks read back without a sync per pass
    PinnedBuf pin_arn;    // block Arnoldi's Gram read-backs, two step slots (sized once per run)
    // pinned staging for gram() read-backs, combine() uploads and the thin-QR
    // read-backs (pageable transfers are staged synchronously by the runtime)
    PinnedBuf pin_gram, pin_comb, pin_qr, pin_qrfac, pin_colarn, pin_qrm;
    hipEvent_t comb_ev = nullptr;  // last combine() upload out of pin_comb
    hipEvent_t qrfac_ev = nullptr;  // shifted CholeskyQR3's factor read-back (kt_block.cpp)
    hipEvent_t qrm_ev = nullptr;    // last upload of the thin QR's T V1' out of pin_qrm
    bool qrm_pending = false;
    bool comb_pending = false;
    // batched greedy candidates (kt_greedy.cpp): 3 pair blocks, indices,
    // per-candidate coefficients / partials / host records
    DevBuf pair_blk[3], pair_idx, pair_coef, pair_part, pair_hr;
    PinnedBuf pair_host[2];
    DevBuf pair_hist, pair_state, pair_scratch, pair_active;  // device-mode candidate state
    PinnedBuf pair_active_host;
    DevBuf ts_V, ts_part, ts_small;  // tall-skinny Householder QR (kt_tsqr.hip)
    // lanczos_columns_split (kt_slq.cpp): pinned sweep records, the y-form
    // start scales per lane, the permuted block's ready event for the aux lanes
    PinnedBuf pin_colrec;
    DevBuf colnorm;  // the block's squared column norms (device)
    hipEvent_t colsplit_ev = nullptr;
};

}  // namespace kt

struct kt_context_s {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t aux_stream[3] = {nullptr, nullptr, nullptr};  // extra probe-sweep lanes (lazy)
    int num_cu = 256;
    bool profile = false;
    // K1 flags: bit 3 = non-temporal y store (bit 0 non-temporal CSR streams
    // and bit 2 deep gather issue measured no better, profiles/r01_sweep_nt.txt)
    int k1_flags = 8;
    bool k2_nt = true;  // K2 loads y and u_prev non-temporal
    int64_t yform_redone = 0;  // y-form sweeps recomputed by the explicit sweep (guard)
    int64_t fu_dense = 0;      // fun_update calls that took the dense fallback (fun_update.m:85-90)
    int64_t fu_last_cols = 0;  // projected size of the last fun_update (n when dense)
    int64_t expmv_calls = 0;   // expmv_device calls (kt_expmv and the expmv Afun of mc_trace)
    int64_t expmv_terms = 0;   // Taylor terms those calls executed (one A b product each, expmv.m:75)
    int ky_flags = 8;   // y-form pass flags (8 = nontemporal store of y_{j+1}, +0.3 %)
    bool yform = true;  // KT_SLQ_YFORM=0: the hot path runs the explicit K1/K2 sweep
    void* blas = nullptr;  // rocblas_handle, created on first block-Krylov use
    // a second context on the same device (own stream, rocBLAS handle and
    // workspace) for the projected-matrix work that a block-Krylov run hands
    // to a worker thread while its next step runs here (kt_krylov.cpp)
    kt_context_s* helper = nullptr;
    // persistent host worker threads (kt_worker.h StepWorker), kept for the
    // context's lifetime: HIP threads started and joined per call stalled the
    // device's other streams when they exited
    void* workers[3] = {nullptr, nullptr, nullptr};
    void (*workers_free)(void*) = nullptr;
    kt::ProfSlot prof[kt::PROF_NSLOTS];
    kt::Workspace ws;
    kt::ScratchPool pool;  // DevMat scratch (kt_block.h)
};

namespace kt {
// One device copy of A as CSR (int32 indices), rows in some order.
struct DevCSR {
    int* rowptr = nullptr;
    int* col = nullptr;
    double* val = nullptr;
    int* long_rows = nullptr;  // rows with degree > long_thresh, heaviest first
    int n_long = 0;
    int n_heavy = 0;           // the first n_heavy long rows have degree > kExpmvCoopThresh
    int* med_rows = nullptr;   // rows with kMedThresh < degree <= long_thresh (expmv terms)
    int n_med = 0;
    // natural order only (the row-blocked expmv term): rows of degree <=
    // min(kMedThresh, long_thresh) as {row, beg, end, 0}, degree-descending
    // within windows of consecutive rows (kt_runtime.cpp build_csr)
    int* short_tasks = nullptr;
    int n_short = 0;
    int* med_tasks = nullptr;  // natural order only: med_rows as {row, beg, end, 0}
    int* perm = nullptr;       // device row -> original row (nullptr: identity)
    // hub rows (degree > kSplitThresh) cut into kChunkNnz-nonzero chunks for
    // the block SpMM: chunk c = nonzeros [ck_beg[c], ck_end[c]); split row i =
    // device row sp_rows[i], its chunks [sp_first[i], sp_first[i+1])
    int *ck_beg = nullptr, *ck_end = nullptr, *sp_rows = nullptr, *sp_first = nullptr;
    int n_chunks = 0, n_split = 0;
    bool built = false;
    // every array above is a slice of one device allocation; a rebuild after
    // edge edits (greedy) reuses it instead of a hipFree / hipMalloc round trip
    char* blob = nullptr;
    size_t blob_bytes = 0;
    PinnedBuf stage;  // host staging of a (re)build: one async upload, one sync
    void release();
    void invalidate() { built = false; }  // contents stale, buffers kept
};
}  // namespace kt

struct kt_matrix_s {
    kt_context_s* ctx = nullptr;
    int64_t n = 0, nnz = 0;
    int long_thresh = 64;
    bool unit_values = false;  // every stored value == 1.0 (unweighted adjacency)
    int symmetric = -1;        // -1 unknown, 0 no, 1 yes (checked on the host copy)
    // hub: rows relabelled by descending degree (hubs first) for the probe
    // hot path; probes stay keyed by ORIGINAL index via hub.perm, so results
    // do not depend on the relabelling.
    kt::DevCSR hub;
    std::vector<int32_t> new2old, old2new;
    // nat: natural row order, built on first use by the block-Krylov and
    // mc_trace paths so that Householder QR sees the reference's row order
    // (rank-deficient completions qr(w,0) picks depend on it).
    kt::DevCSR nat;
    // host copy (CSR, int64 pointers, original order)
    std::vector<int64_t> h_rowptr;
    std::vector<int32_t> h_col;
    std::vector<double> h_val;
    uint64_t version = 0;  // bumped when the host copy is edited (refresh_device)
    // last normest(A, tol) (kt_krylov.cpp normest_impl), valid for `normest_version`
    bool normest_ok = false;
    uint64_t normest_version = 0;
    double normest_tol = 0.0, normest_val = 0.0;
    // last expmv shift + Taylor degree selection (kt_mctrace.cpp expmv_device):
    // a function of A, t and the block width only (expmv.m:31-68), so calls on
    // the same A (every mc_trace round of trace_exp) reuse it; valid for
    // `expmv_sel_version`
    bool expmv_sel_ok = false;
    uint64_t expmv_sel_version = 0;
    double expmv_sel_t = 0.0, expmv_sel_mu = 0.0;
    int expmv_sel_nc = 0, expmv_sel_s = 1, expmv_sel_m = 0, expmv_sel_mv = 0;
    // twin: a second context (own stream + workspace) holding another device
    // copy of this matrix, built on first use, so that two independent Krylov
    // runs of one call overlap (fun_and_grad_krylov_fun.m:64-65)
    kt_context_s* twin_ctx = nullptr;
    kt_matrix_s* twin = nullptr;
    uint64_t twin_version = 0;
    bool twin_failed = false;  // the last build failed (twin_of falls back to serial)
    uint64_t twin_failed_version = 0;
};

namespace kt {

// build one device CSR of A with rows in the order new2old (identity if empty)
// sync = false: the upload is only stream-ordered (see natural_csr_ordered)
void build_csr(kt_matrix_s* A, const std::vector<int32_t>& new2old, DevCSR& out, bool sync = true);
const DevCSR& natural_csr(kt_matrix_s* A);
const DevCSR& natural_csr_ordered(kt_matrix_s* A);
void refresh_device(kt_matrix_s* A);
const DevCSR& hub_csr(kt_matrix_s* A);

// profiling helpers (no-ops unless ctx->profile)
void prof_begin(kt_context_s* ctx, int slot, hipStream_t st = nullptr, int tag = 0);
void prof_end(kt_context_s* ctx, int slot, hipStream_t st = nullptr);
// fold recorded events into the totals: all of them (every one complete:
// after a stream sync, or waited for here when `wait`), or, with `upto`,
// only the events recorded before upto[slot] (a previous call's, complete)
void prof_collect(kt_context_s* ctx, const size_t* upto = nullptr, bool wait = false);
// at a call's start: recycle the events already folded in, keep the rest
void prof_recycle(kt_context_s* ctx);
void prof_reserve(kt_context_s* ctx, size_t per_slot);
// union of the slot's folded launch intervals (ms)
double prof_busy(const ProfSlot& s);

// dense host helpers (kt_dense.cpp)
double fscalar(int fun, double x);
// Gauss quadrature e1' f(T) e1 for symmetric tridiagonal T (m x m).
double tridiag_quadrature(int m, const double* alpha, const double* off, int fun);
// The same quadrature, and f(T) e1 into fe1[0..m-1], from one QL pass.
double tridiag_fun_e1(int m, const double* alpha, const double* off, int fun, double* fe1);
bool chol_upper(double* G, int n);
void tri_upper_inv(const double* R, int n, double* X);
void sym_eig_host(int n, const double* A, double* w, double* V);
void sym_fun_from_eig(int n, const double* w, const double* V, int fun, double* F);

}  // namespace kt
