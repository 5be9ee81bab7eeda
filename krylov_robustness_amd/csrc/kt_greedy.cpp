// kt_greedy.cpp -- the candidate loop of krylov_miobi.m, batched on the device.
//
// krylov_miobi.m:76-125 scores every candidate edge h with
//   trace_fun_update(A, U_h, B, tol, it)      U_h = [e_i, e_j],  B = -+[0 1;1 0]/rescale
// one call after another.  Here all candidates of a greedy step advance
// together: ONE SpMM over the 2C columns of the pair block per Lanczos step,
// one fused CGS2 + Householder-QR launch (kt_pairs.hip), one small copy of the
// per-candidate coefficients to the host, and per-candidate host work on the
// 2j x 2j projected matrices with per-candidate stopping masks.  Candidate
// h's numbers follow trace_fun_update.m exactly as the single-call path
// (kt_krylov.cpp) does; only the order of independent work changes.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include "kt_krylov.h"
#include "kt_pool.h"
#include "kt_launch.h"

namespace kt {

namespace {

constexpr int kMaxPairs = 256;  // candidates per device batch (512 columns)
constexpr int64_t kFusedMaxN = 16384;  // the fused one-workgroup-per-candidate path up to this n

// Per-candidate Lanczos state: the 2x2 blocks lanczos_krylov.m:88,90 writes
// into H at step b (column-major): D = h(cur), P = h(prev), R = qr's R.
struct PairRun {
    std::vector<double> D, P, R;
    double Cm[4] = {0, 0, 0, 0};
    double Xstop[2] = {0, 0};
    double Xm = 0.0;
    int iter = 0;
    bool lucky = false;
    bool done = false;
};

// trace_fun_update.m:71-89 for one candidate after j Lanczos steps
double pair_xm(const PairRun& s, int j, int fun, std::vector<double>& G, std::vector<double>& T,
               std::vector<double>& w1, std::vector<double>& w2) {
    const int nn = 2 * j;
    G.assign((size_t)nn * nn, 0.0);
    auto put = [&](const std::vector<double>& blk, int b, int row0, int col0) {
        for (int jj = 0; jj < 2; ++jj)
            for (int ii = 0; ii < 2; ++ii)
                G[(row0 + ii) + (size_t)(col0 + jj) * nn] = blk[4 * b + ii + 2 * jj];
    };
    for (int b = 0; b < j; ++b) {
        put(s.D, b, 2 * b, 2 * b);
        if (b >= 1) put(s.P, b, 2 * (b - 1), 2 * b);
        if (b + 1 < j) put(s.R, b, 2 * (b + 1), 2 * b);
    }
    T = G;
    for (int jj = 0; jj < 2; ++jj)
        for (int ii = 0; ii < 2; ++ii) T[ii + (size_t)jj * nn] += s.Cm[ii + 2 * jj];
    for (int b = 0; b < nn; ++b)  // herm: (X + X')/2   :78-81
        for (int a = 0; a < b; ++a) {
            double x = 0.5 * (G[a + (size_t)b * nn] + G[b + (size_t)a * nn]);
            G[a + (size_t)b * nn] = G[b + (size_t)a * nn] = x;
            x = 0.5 * (T[a + (size_t)b * nn] + T[b + (size_t)a * nn]);
            T[a + (size_t)b * nn] = T[b + (size_t)a * nn] = x;
        }
    w1.resize(nn);
    w2.resize(nn);
    sym_eig_host(nn, T.data(), w1.data(), nullptr);
    sym_eig_host(nn, G.data(), w2.data(), nullptr);
    std::sort(w1.begin(), w1.end());
    std::sort(w2.begin(), w2.end());
    return trace_diff(w1, w2, fun);
}

// One device batch of C <= kMaxPairs two-column candidates.
void run_pair_batch(kt_matrix_s* A, int C, const int64_t* ei, const int64_t* ej, const double* B,
                    double tol, int it, int fun, double* Xm, int* iter, int* lucky) {
    kt_context_s* ctx = A->ctx;
    const int64_t n = A->n;
    const int cols = 2 * C;
    using clk = std::chrono::steady_clock;
    constexpr bool timing = KT_DIAG != 0;
    double t_setup = 0, t_gpu = 0, t_host = 0;
    auto t0 = clk::now();
    auto lap = [&](double& acc) {
        auto t = clk::now();
        acc += std::chrono::duration<double, std::milli>(t - t0).count();
        t0 = t;
    };
    Workspace& ws = ctx->ws;
    // Small graphs: one workgroup per candidate runs the whole
    // trace_fun_update in ONE launch (k_pair_fused), no per-step grid-wide
    // hand-offs.  KT_PAIRS_FUSED=0 keeps the batched steps below; larger n
    // keeps them too (one workgroup per candidate would sweep too many rows).
    const char* fz = getenv("KT_PAIRS_FUSED");
    const bool fused = !(fz && fz[0] == '0') && n <= kFusedMaxN && pair_fused_lds_bytes(it) <= 150 * 1024 &&
                       getenv("KT_PAIRS_HOST") == nullptr;
    if (fused) {
        const DevCSR& M = natural_csr_ordered(A);  // every reader below is on ctx->stream
        const CsrView V{M.rowptr, M.col, M.val, (int)n, M.long_rows, M.n_long, A->long_thresh,
                        kSplitThresh, M.ck_beg, M.ck_end, M.n_chunks, M.sp_rows, M.sp_first, M.n_split};
        ws.pair_blk[0].ensure(sizeof(double) * 6 * (size_t)std::max<int64_t>(n, 1) * C);
        ws.pair_idx.ensure(sizeof(int) * 2 * (size_t)C);
        ws.pair_state.ensure(sizeof(double) * 8 * (size_t)C);
        const int nnmax = 2 * it;
        int64_t big_stride = 0;
        double* big = nullptr;
        const char* de = getenv("KT_PAIRS_DENSE_EIG");  // the dense solver needs global scratch past 2j = 56
        if (de && de[0] == '1' && nnmax > 56) {  // G, T, d/e, eigenvalues per candidate
            big_stride = 2 * (int64_t)nnmax * nnmax + 6 * (int64_t)nnmax;
            ws.pair_scratch.ensure(sizeof(double) * (size_t)C * big_stride);
            big = ws.pair_scratch.as<double>();
        }
        // candidate indices up and states down through pinned staging (a
        // pageable copy is staged synchronously by the runtime)
        ws.pair_host[0].ensure(std::max(sizeof(int) * 2 * (size_t)C, sizeof(double) * 8 * (size_t)C));
        int* idx = ws.pair_host[0].as<int>();
        for (int c = 0; c < C; ++c) {
            idx[c] = (int)ei[c];
            idx[C + c] = (int)ej[c];
        }
        KT_HIP(hipMemcpyAsync(ws.pair_idx.ptr, idx, sizeof(int) * 2 * (size_t)C, hipMemcpyHostToDevice,
                              ctx->stream));
        KT_HIP(launch_pair_fused(C, (int)n, (int64_t)A->h_rowptr[n], V, A->unit_values, ws.pair_idx.as<int>(), ws.pair_idx.as<int>() + C,
                                 B, it, fun, tol, ws.pair_blk[0].as<double>(), big, big_stride,
                                 ws.pair_state.as<double>(), ctx->stream));
        ws.pair_host[1].ensure(sizeof(double) * 8 * (size_t)C);
        const double* sv = ws.pair_host[1].as<double>();
        KT_HIP(hipMemcpyAsync(ws.pair_host[1].ptr, ws.pair_state.ptr, sizeof(double) * 8 * (size_t)C,
                              hipMemcpyDeviceToHost, ctx->stream));
        KT_HIP(hipStreamSynchronize(ctx->stream));
        lap(t_gpu);
        for (int c = 0; c < C; ++c) {
            if (sv[(size_t)8 * c + 3] < 0) fail(KT_ERR_HIP, "pair_fused: eigen scratch missing");
            Xm[c] = sv[(size_t)8 * c + 2];
            if (iter) iter[c] = (int)sv[(size_t)8 * c + 3];
            if (lucky) lucky[c] = sv[(size_t)8 * c + 4] != 0.0 ? 1 : 0;
        }
        if (timing) fprintf(stderr, "[kt pairs] fused C=%d n=%lld %.3f ms\n", C, (long long)n, t_gpu);
        return;
    }
    const int CP = cols <= 64 ? pow2_at_least(cols) : (cols + 127) / 128 * 128;
    const size_t blk_bytes = sizeof(double) * (size_t)std::max<int64_t>(n, 1) * CP;
    double* S[3];
    for (int t = 0; t < 3; ++t) {
        ws.pair_blk[t].ensure(blk_bytes);
        S[t] = ws.pair_blk[t].as<double>();
    }
    ws.pair_idx.ensure(sizeof(int) * 2 * (size_t)C);
    ws.pair_hr.ensure(sizeof(double) * 11 * (size_t)C);
    ws.pair_coef.ensure(sizeof(double) * pairs_coef_doubles(C));
    ws.pair_part.ensure(sizeof(double) * pairs_part_doubles((int)n, C, ctx->num_cu));
    for (auto& b : ws.pair_host) b.ensure(sizeof(double) * 11 * (size_t)C);
    double* dhr = ws.pair_hr.as<double>();
    auto orth = [&](const double* p, const double* u, double* W) {
        KT_HIP(launch_pairs_orth(C, (int)n, ctx->num_cu, p, u, W, CP, ws.pair_coef.as<double>(),
                                 ws.pair_part.as<double>(), dhr, ctx->stream));
    };
    std::vector<int> idx(2 * (size_t)C);
    for (int c = 0; c < C; ++c) {
        idx[c] = (int)ei[c];
        idx[C + c] = (int)ej[c];
    }
    // S[0] = 0 (the SpMM then keeps the padding columns of S[1], S[2] at 0)
    KT_HIP(hipMemsetAsync(S[0], 0, blk_bytes, ctx->stream));
    KT_HIP(hipMemcpyAsync(ws.pair_idx.ptr, idx.data(), sizeof(int) * idx.size(), hipMemcpyHostToDevice,
                          ctx->stream));
    double* hr = ws.pair_host[0].as<double>();
    struct Events {
        hipEvent_t e[2] = {nullptr, nullptr};
        Events() {
            for (auto& x : e) KT_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
        }
        ~Events() {
            for (auto& x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } evs, evhs;
    hipEvent_t* ev = evs.e;
    hipEvent_t* evh = evhs.e;
    auto fetch = [&]() {
        KT_HIP(hipMemcpyAsync(hr, dhr, sizeof(double) * 11 * (size_t)C, hipMemcpyDeviceToHost,
                              ctx->stream));
        KT_HIP(hipStreamSynchronize(ctx->stream));
    };
    // [V, ~] = qr(U, 0)  (lanczos_krylov.m:48); V1' U = R exactly for unit
    // selectors, so Cm = R B R'  (trace_fun_update.m:65-66)
    KT_HIP(launch_pair_select(C, ws.pair_idx.as<int>(), ws.pair_idx.as<int>() + C, S[0], CP, ctx->stream));
    orth(nullptr, nullptr, S[0]);
    fetch();
    lap(t_setup);
    std::vector<PairRun> run(C);
    for (int c = 0; c < C; ++c) {
        const double R[4] = {hr[11 * c + 8], 0.0, hr[11 * c + 9], hr[11 * c + 10]};
        double RB[4], Rt[4] = {R[0], R[2], R[1], R[3]};
        matmul(2, 2, 2, R, B, RB);
        matmul(2, 2, 2, RB, Rt, run[c].Cm);
    }
    const bool host_mode = getenv("KT_PAIRS_HOST") != nullptr;
    if (!host_mode) {
        // Device mode: the projected eigenproblems, Xm and the stop masks of
        // every candidate run on the device (k_pair_eig), so the Lanczos
        // steps are queued back to back; the host only polls the active
        // count of the previous step and stops queuing once it reaches 0 (a
        // step queued after that is discarded: done candidates are frozen).
        const int nnmax = 2 * it;
        const int64_t sstride = 2 * (int64_t)nnmax * nnmax + 3 * (int64_t)nnmax;
        ws.pair_hist.ensure(sizeof(double) * (size_t)it * C * 11);
        ws.pair_state.ensure(sizeof(double) * (size_t)C * 8 + sizeof(double) * 4 * (size_t)C);
        const char* dense_eig = getenv("KT_PAIRS_DENSE_EIG");  // only the dense solver uses the scratch
        if (dense_eig && dense_eig[0] == '1') ws.pair_scratch.ensure(sizeof(double) * (size_t)C * sstride);
        ws.pair_active.ensure(sizeof(int) * 2);
        ws.pair_active_host.ensure(sizeof(int) * 2);
        double* hist = ws.pair_hist.as<double>();
        double* state = ws.pair_state.as<double>();
        double* dcm = state + (size_t)C * 8;
        int* act_dev = ws.pair_active.as<int>();
        int* act_host = ws.pair_active_host.as<int>();
        std::vector<double> cm((size_t)4 * C);
        for (int c = 0; c < C; ++c)
            for (int t = 0; t < 4; ++t) cm[(size_t)4 * c + t] = run[c].Cm[t];
        KT_HIP(hipMemsetAsync(state, 0, sizeof(double) * (size_t)C * 8, ctx->stream));
        KT_HIP(hipMemcpyAsync(dcm, cm.data(), sizeof(double) * cm.size(), hipMemcpyHostToDevice, ctx->stream));
        const int act0[2] = {C, C};  // counts only fall: a stale read never skips early
        KT_HIP(hipMemcpyAsync(act_dev, act0, sizeof(act0), hipMemcpyHostToDevice, ctx->stream));
        // The projected eigenproblems of step j (k_pair_eig) only decide when
        // to stop; the recurrence of step j+1 does not need them.  They run
        // on a side stream, gated by an event after step j's coefficients, so
        // they overlap step j+1's SpMM and sweeps.
        if (!ctx->aux_stream[0])
            KT_HIP(hipStreamCreateWithFlags(&ctx->aux_stream[0], hipStreamNonBlocking));
        hipStream_t side = ctx->aux_stream[0];
        int cur = 0, prev = -1, w = 1;
        for (int j = 1; j <= it; ++j) {
            // a step queued after every candidate stopped (the host polls one
            // step behind) exits at once on an earlier step's active count
            const int* skip = j >= 2 ? act_dev + ((j - 1) & 1) : nullptr;
            spmm_slices(A, S[cur], CP, S[w], CP, cols, skip);  // w = A * w   (lanczos_krylov.m:81)
            double* hj = hist + (size_t)(j - 1) * C * 11;
            KT_HIP(launch_pairs_orth(C, (int)n, ctx->num_cu, prev >= 0 ? S[prev] : nullptr, S[cur], S[w], CP,
                                     ws.pair_coef.as<double>(), ws.pair_part.as<double>(), hj, ctx->stream,
                                     skip));
            KT_HIP(hipEventRecord(evh[j & 1], ctx->stream));  // hist[j-1] complete
            KT_HIP(hipStreamWaitEvent(side, evh[j & 1], 0));
            KT_HIP(launch_pair_eig(C, j, it, fun, tol, hist, dcm, ws.pair_scratch.as<double>(), sstride,
                                   state, act_dev + (j & 1), side));
            KT_HIP(hipMemcpyAsync(act_host + (j & 1), act_dev + (j & 1), sizeof(int), hipMemcpyDeviceToHost,
                                  side));
            KT_HIP(hipEventRecord(ev[j & 1], side));
            const int freed = prev >= 0 ? prev : 3 - cur - w;
            prev = cur;
            cur = w;
            w = freed;
            if (j >= 2) {  // poll the previous step while this one runs
                KT_HIP(hipEventSynchronize(ev[(j - 1) & 1]));
                if (act_host[(j - 1) & 1] == 0) break;
            }
        }
        KT_HIP(hipStreamSynchronize(side));
        KT_HIP(hipStreamSynchronize(ctx->stream));
        lap(t_gpu);
        std::vector<double> sv((size_t)C * 8);
        KT_HIP(hipMemcpy(sv.data(), state, sizeof(double) * sv.size(), hipMemcpyDeviceToHost));
        for (int c = 0; c < C; ++c) {
            Xm[c] = sv[(size_t)8 * c + 2];
            if (iter) iter[c] = (int)sv[(size_t)8 * c + 3];
            if (lucky) lucky[c] = sv[(size_t)8 * c + 4] != 0.0 ? 1 : 0;
        }
        if (timing)
            fprintf(stderr, "[kt pairs] device mode C=%d n=%lld setup %.3f ms  loop %.3f ms\n", C,
                    (long long)n, t_setup, t_gpu);
        return;
    }
    // Step j's device work (SpMM + CGS2/QR + copy of its coefficients) is
    // queued before the host processes step j-1, so the host eig work of
    // one step overlaps the device work of the next.  A step launched after
    // every candidate stopped is simply discarded.
    int cur = 0, prev = -1, w = 1;
    PinnedBuf* hbuf = ws.pair_host;
    auto launch_step = [&](int slot) {
        // w = A * w over every candidate (lanczos_krylov.m:81)
        spmm_slices(A, S[cur], CP, S[w], CP, cols);
        orth(prev >= 0 ? S[prev] : nullptr, S[cur], S[w]);
        KT_HIP(hipMemcpyAsync(hbuf[slot].ptr, dhr, sizeof(double) * 11 * (size_t)C,
                              hipMemcpyDeviceToHost, ctx->stream));
        KT_HIP(hipEventRecord(ev[slot], ctx->stream));
        const int freed = prev >= 0 ? prev : 3 - cur - w;
        prev = cur;
        cur = w;
        w = freed;
    };
    int active = C;
    const int d = 2;  // lag (trace_fun_update.m:58)
    std::vector<int> todo;
    launch_step(0);
    for (int j = 1; j <= it && active > 0; ++j) {
        KT_HIP(hipEventSynchronize(ev[(j - 1) & 1]));
        lap(t_gpu);
        if (j < it) launch_step(j & 1);
        const double* hr_j = hbuf[(j - 1) & 1].as<double>();
        todo.clear();
        for (int c = 0; c < C; ++c) {
            if (run[c].done) continue;
            PairRun& s = run[c];
            const double* h = hr_j + 11 * c;
            // h rows (prev0, prev1, cur0, cur1) x cols (w0, w1)
            s.P.insert(s.P.end(), {h[0], h[1], h[4], h[5]});
            s.D.insert(s.D.end(), {h[2], h[3], h[6], h[7]});
            s.R.insert(s.R.end(), {h[8], 0.0, h[9], h[10]});
            s.lucky = std::sqrt(h[8] * h[8] + h[9] * h[9] + h[10] * h[10]) < 1e-8;  // :91-93
            todo.push_back(c);
        }
        HostPool::get().run((int)todo.size(), [&](int t) {
            thread_local std::vector<double> G, T, w1, w2;
            PairRun& s = run[todo[t]];
            s.Xm = pair_xm(s, j, fun, G, T, w1, w2);
        });
        for (int c : todo) {
            PairRun& s = run[c];
            bool stop = false;
            if (j <= d) {  // :104-118
                s.Xstop[j - 1] = s.Xm;
            } else if (std::fabs(s.Xm - s.Xstop[0]) < tol) {
                stop = true;
            } else {
                s.Xstop[0] = s.Xstop[1];
                s.Xstop[1] = s.Xm;
            }
            if (!stop && s.lucky) stop = true;  // :119-124
            if (stop || j == it) {
                s.done = true;
                s.iter = j;
                --active;
            }
        }
        lap(t_host);
    }
    KT_HIP(hipStreamSynchronize(ctx->stream));
    if (timing)
        fprintf(stderr, "[kt pairs] C=%d n=%lld setup %.3f ms  gpu %.3f ms  host %.3f ms\n", C,
                (long long)n, t_setup, t_gpu, t_host);
    for (int c = 0; c < C; ++c) {
        Xm[c] = run[c].Xm;
        if (iter) iter[c] = run[c].iter;
        if (lucky) lucky[c] = run[c].lucky ? 1 : 0;
    }
}

// host CSR edit of one entry (row r, column col); value 0 deletes
void set_entry(kt_matrix_s* A, int64_t r, int32_t col, double value) {
    auto b = A->h_col.begin() + A->h_rowptr[r], e = A->h_col.begin() + A->h_rowptr[r + 1];
    auto f = std::lower_bound(b, e, col);
    const int64_t k = f - A->h_col.begin();
    const bool found = f != e && *f == col;
    if (found && value != 0.0) {
        A->h_val[k] = value;
        return;
    }
    if (!found && value == 0.0) return;
    const int64_t delta = found ? -1 : 1;
    if (found) {
        A->h_col.erase(A->h_col.begin() + k);
        A->h_val.erase(A->h_val.begin() + k);
    } else {
        A->h_col.insert(A->h_col.begin() + k, col);
        A->h_val.insert(A->h_val.begin() + k, value);
    }
    for (int64_t i = r + 1; i <= A->n; ++i) A->h_rowptr[i] += delta;
    A->nnz += delta;
}

}  // namespace

static void run_pairs_range(kt_matrix_s* A, const std::vector<int64_t>& pairs, size_t p0, size_t p1,
                            const int64_t* ei, const int64_t* ej, const double* B, double tol, int it,
                            int fun, double* Xm, int* iter, int* lucky);

void trace_fun_update_pairs(kt_matrix_s* A, int64_t nC, const int64_t* ei, const int64_t* ej,
                            const double* B, double B1, double tol, int it, int fun, double* Xm,
                            int* iter, int* lucky) {
    const int64_t n = A->n;
    if (it <= 0) it = (int)std::min<int64_t>(100, n);  // trace_fun_update.m:25-27
    for (int64_t c = 0; c < nC; ++c)
        if (ei[c] < 0 || ei[c] >= n || ej[c] < 0 || ej[c] >= n)
            fail(KT_ERR_ARG, "candidate edge index out of range");
    std::vector<int64_t> pairs, singles;
    for (int64_t c = 0; c < nC; ++c) (ei[c] != ej[c] && n > 130 ? pairs : singles).push_back(c);
    // self-loop candidates (krylov_miobi.m:88-98) and the dense shortcut of
    // trace_fun_update.m:37-51 (n <= 130) go through the single-call path
    std::vector<double> U;
    for (int64_t c : singles) {
        const bool two = ei[c] != ej[c];
        U.assign((size_t)n * (two ? 2 : 1), 0.0);
        U[ei[c]] = 1.0;
        if (two) U[n + ej[c]] = 1.0;
        int itc = 0, lc = 0;
        Xm[c] = trace_fun_update_impl(A, two ? 2 : 1, U.data(), two ? B : &B1, tol, it, fun, &itc, &lc);
        if (iter) iter[c] = itc;
        if (lucky) lucky[c] = lc;
    }
    if (pairs.empty()) return;
    if (B[1] != B[2]) fail(KT_ERR_UNSUPPORTED, "trace_fun_update: non-Hermitian B (needs a general eig)");
    // One batch sequence on A's own stream.  Splitting the candidates over A
    // and its twin (second stream + host thread) was measured slower: config
    // 5 47 -> 60 ms (profiles/r01_greedy_twin_split.txt) -- each half keeps
    // every launch of a Lanczos step, so the launch count doubles.
    run_pairs_range(A, pairs, 0, pairs.size(), ei, ej, B, tol, it, fun, Xm, iter, lucky);
}

// candidates pairs[p0, p1) in device batches of <= kMaxPairs
static void run_pairs_range(kt_matrix_s* A, const std::vector<int64_t>& pairs, size_t p0, size_t p1,
                            const int64_t* ei, const int64_t* ej, const double* B, double tol, int it,
                            int fun, double* Xm, int* iter, int* lucky) {
    {
        constexpr bool timing = KT_DIAG != 0;
        const auto t0 = std::chrono::steady_clock::now();
        (void)natural_csr_ordered(A);  // candidate kernels run on ctx->stream (side-stream work waits on its events)
        if (timing)
            fprintf(stderr, "[kt pairs] natural CSR %.3f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    for (size_t b0 = p0; b0 < p1; b0 += kMaxPairs) {
        const int C = (int)std::min<size_t>(kMaxPairs, p1 - b0);
        std::vector<int64_t> bi(C), bj(C);
        std::vector<double> xm(C);
        std::vector<int> itv(C), lv(C);
        for (int c = 0; c < C; ++c) {
            bi[c] = ei[pairs[b0 + c]];
            bj[c] = ej[pairs[b0 + c]];
        }
        run_pair_batch(A, C, bi.data(), bj.data(), B, tol, it, fun, xm.data(), itv.data(), lv.data());
        for (int c = 0; c < C; ++c) {
            const int64_t o = pairs[b0 + c];
            Xm[o] = xm[c];
            if (iter) iter[o] = itv[c];
            if (lucky) lucky[o] = lv[c];
        }
    }
}

void set_pairs(kt_matrix_s* A, int64_t count, const int64_t* ei, const int64_t* ej, double value) {
    for (int64_t t = 0; t < count; ++t)
        if (ei[t] < 0 || ei[t] >= A->n || ej[t] < 0 || ej[t] >= A->n)
            fail(KT_ERR_ARG, "edge index out of range");
    KT_HIP(hipStreamSynchronize(A->ctx->stream));
    for (int64_t t = 0; t < count; ++t) {
        set_entry(A, ei[t], (int32_t)ej[t], value);
        if (ei[t] != ej[t]) set_entry(A, ej[t], (int32_t)ei[t], value);
    }
    const bool twin_current = A->twin && A->twin_version == A->version;
    refresh_device(A);
    if (twin_current) {  // the same edit on the twin copy instead of a rebuild
        set_pairs(A->twin, count, ei, ej, value);
        A->twin_version = A->version;
        KT_HIP(hipSetDevice(A->ctx->device));
    }
}

}  // namespace kt

using namespace kt;

#define KT_GUARD_BEGIN try {
#define KT_GUARD_END                                   \
    }                                                  \
    catch (const kt::Status& s) {                      \
        kt::set_error(s.msg);                          \
        return s.code;                                 \
    }                                                  \
    catch (const std::bad_alloc&) {                    \
        kt::set_error("host allocation failed");       \
        return KT_ERR_ALLOC;                           \
    }                                                  \
    catch (const std::exception& e) {                  \
        kt::set_error(e.what());                       \
        return KT_ERR_ARG;                             \
    }                                                  \
    return KT_OK;

extern "C" {

int kt_trace_fun_update_pairs(kt_matrix_t A, int64_t ncand, const int64_t* ei, const int64_t* ej,
                              const double* B, double b_self, double tol, int it, int fun,
                              double* Xm, int* iter, int* lucky) {
    KT_GUARD_BEGIN
    if (!A || !B || !Xm || (ncand > 0 && (!ei || !ej))) fail(KT_ERR_ARG, "NULL argument");
    if (ncand < 0) fail(KT_ERR_ARG, "negative candidate count");
    KT_HIP(hipSetDevice(A->ctx->device));
    trace_fun_update_pairs(A, ncand, ei, ej, B, b_self, tol, it, fun, Xm, iter, lucky);
    KT_GUARD_END
}

int kt_matrix_set_pairs(kt_matrix_t A, int64_t count, const int64_t* ei, const int64_t* ej,
                        double value) {
    KT_GUARD_BEGIN
    if (!A || (count > 0 && (!ei || !ej))) fail(KT_ERR_ARG, "NULL argument");
    KT_HIP(hipSetDevice(A->ctx->device));
    set_pairs(A, count, ei, ej, value);
    KT_GUARD_END
}

int kt_matrix_export_csc(kt_matrix_t A, int64_t* colptr, int64_t* rowind, double* vals) {
    KT_GUARD_BEGIN
    if (!A || !colptr) fail(KT_ERR_ARG, "NULL argument");
    std::copy(A->h_rowptr.begin(), A->h_rowptr.end(), colptr);  // CSR == CSC (symmetric A)
    if (rowind) for (int64_t k = 0; k < A->nnz; ++k) rowind[k] = A->h_col[k];
    if (vals) std::copy(A->h_val.begin(), A->h_val.end(), vals);
    KT_GUARD_END
}

}  // extern "C"

namespace kt {
namespace {

// One selection of krylov_miobi.m:70-135 over the candidates Ei/Ej[0, m):
// score them all (:76-99), take the first extreme (:112-124, strict
// comparison), edit A in place (:129-135).  Returns the chosen index.
int64_t miobi_select(kt_matrix_s* A, std::vector<int64_t>& Ei, std::vector<int64_t>& Ej, int64_t m,
                     const double* B, double sg, double tol, int it, int make, std::vector<double>& xm,
                     double* value) {
    constexpr bool timing = KT_DIAG != 0;
    using clk = std::chrono::steady_clock;
    xm.assign(m, 0.0);
    const auto t0 = clk::now();
    trace_fun_update_pairs(A, m, Ei.data(), Ej.data(), B, sg, tol, it, KT_FUN_EXP, xm.data(), nullptr,
                           nullptr);
    const auto t1 = clk::now();
    int64_t best = -1;
    double bv = make ? -INFINITY : INFINITY;
    for (int64_t h = 0; h < m; ++h)
        if (make ? xm[h] > bv : xm[h] < bv) {
            bv = xm[h];
            best = h;
        }
    if (best < 0) fail(KT_ERR_ARG, "KRYLOV_MIOBI:: no finite candidate score");
    const int64_t ci = Ei[best], cj = Ej[best];
    set_pairs(A, 1, &ci, &cj, make ? 1.0 : 0.0);
    if (timing)
        fprintf(stderr, "[kt miobi] score %.3f ms  select+edit %.3f ms\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(clk::now() - t1).count());
    *value = bv;
    return best;
}

// greedy_krylov's k selection steps with the loop on the device (break
// mode, the register-resident candidate kernel): per step one k_pair_reg
// launch on the first min(Q, |T|) ranked pairs and one k_greedy_edit launch
// (argmin, ranking update, the edge deleted into the other CSR buffer), all
// queued without a host round trip; the host replays the selected edits on
// its copy at the end.  Same candidates, same kernel, same CSR contents as
// the host loop, so the same scores and edges.  false: not applicable (the
// caller runs the host loop).  KT_GREEDY_DEVICE=0 disables it.
bool greedy_steps_device(kt_matrix_s* A, int k, int64_t Q, const std::vector<int64_t>& Ti,
                         const std::vector<int64_t>& Tj, const double* B, double tol, int it, int64_t* sel_i,
                         int64_t* sel_j, double* rob, int64_t* nsel) {
    const char* ge = getenv("KT_GREEDY_DEVICE");
    if (ge && ge[0] == '0') return false;
    const int64_t n = A->n, ntop = (int64_t)Ti.size();
    const char* fz = getenv("KT_PAIRS_FUSED");
    if (k <= 0 || n <= 130 || ntop > 4096 || ntop < k || Q > kMaxPairs || (fz && fz[0] == '0') ||
        getenv("KT_PAIRS_HOST") || n > kFusedMaxN || pair_fused_lds_bytes(it) > 150 * 1024)
        return false;
    for (int64_t h = 0; h < ntop; ++h)
        if (Ti[h] == Tj[h] || Ti[h] < 0 || Ti[h] >= n || Tj[h] < 0 || Tj[h] >= n) return false;
    if (A->nnz - 2 * (int64_t)(k - 1) < 2) return false;  // krylov_miobi.m:63-65 would fire: host loop
    kt_context_s* ctx = A->ctx;
    hipStream_t st = ctx->stream;
    const DevCSR& M0 = natural_csr(A);
    const int64_t nnz0 = A->nnz;
    if (!pair_reg_applies((int)n, nnz0, it, M0.n_long, A->unit_values)) return false;
    // k_greedy_edit keeps the long-row list in its previous order, a host
    // rebuild re-sorts it heaviest first; with more long rows than k_pair_reg
    // hands to whole waves an edit could change which rows those are, and the
    // device loop would no longer form the host loop's sums: host loop
    if (M0.n_long > kRegLongCap) return false;
    const int nl0 = std::max(M0.n_long, 1);
    // device state: two CSR sets {rp, ci, va, lr, dyn}, the ranking, the picks
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t set_bytes = al(sizeof(int) * (n + 1)) + al(sizeof(int) * nnz0) + al(sizeof(double) * nnz0) +
                             al(sizeof(int) * nl0) + al(sizeof(int) * 2);
    const size_t tail = al(sizeof(int) * ntop) * 2 + al(sizeof(int) * 2 * k) + al(sizeof(double) * k);
    Workspace& ws = ctx->ws;
    ws.pair_scratch.ensure(2 * set_bytes + tail);
    char* base = ws.pair_scratch.as<char>();
    struct Set {
        int *rp, *ci, *lr, *dyn;
        double* va;
    } S[2];
    for (int t = 0; t < 2; ++t) {
        char* p = base + t * set_bytes;
        S[t].rp = reinterpret_cast<int*>(p);
        p += al(sizeof(int) * (n + 1));
        S[t].ci = reinterpret_cast<int*>(p);
        p += al(sizeof(int) * nnz0);
        S[t].va = reinterpret_cast<double*>(p);
        p += al(sizeof(double) * nnz0);
        S[t].lr = reinterpret_cast<int*>(p);
        p += al(sizeof(int) * nl0);
        S[t].dyn = reinterpret_cast<int*>(p);
    }
    char* p = base + 2 * set_bytes;
    int* dTi = reinterpret_cast<int*>(p);
    p += al(sizeof(int) * ntop);
    int* dTj = reinterpret_cast<int*>(p);
    p += al(sizeof(int) * ntop);
    int* dsel = reinterpret_cast<int*>(p);
    p += al(sizeof(int) * 2 * k);
    double* dselv = reinterpret_cast<double*>(p);
    ws.pair_state.ensure(sizeof(double) * 8 * (size_t)kMaxPairs);
    // staging: ranking + dyn up, picks down (pinned)
    ws.pair_host[0].ensure(sizeof(int) * (2 * (size_t)ntop + 2));
    int* h = ws.pair_host[0].as<int>();
    for (int64_t t = 0; t < ntop; ++t) {
        h[t] = (int)Ti[t];
        h[ntop + t] = (int)Tj[t];
    }
    h[2 * ntop] = (int)nnz0;
    h[2 * ntop + 1] = M0.n_long;
    KT_HIP(hipMemcpyAsync(dTi, h, sizeof(int) * ntop, hipMemcpyHostToDevice, st));
    KT_HIP(hipMemcpyAsync(dTj, h + ntop, sizeof(int) * ntop, hipMemcpyHostToDevice, st));
    KT_HIP(hipMemcpyAsync(S[0].dyn, h + 2 * ntop, sizeof(int) * 2, hipMemcpyHostToDevice, st));
    KT_HIP(hipMemcpyAsync(S[0].rp, M0.rowptr, sizeof(int) * (n + 1), hipMemcpyDeviceToDevice, st));
    KT_HIP(hipMemcpyAsync(S[0].ci, M0.col, sizeof(int) * nnz0, hipMemcpyDeviceToDevice, st));
    KT_HIP(hipMemcpyAsync(S[0].va, M0.val, sizeof(double) * nnz0, hipMemcpyDeviceToDevice, st));
    if (M0.n_long > 0)
        KT_HIP(hipMemcpyAsync(S[0].lr, M0.long_rows, sizeof(int) * M0.n_long, hipMemcpyDeviceToDevice, st));
    double* state = ws.pair_state.as<double>();
    for (int s = 0; s < k; ++s) {
        const int C = (int)std::min<int64_t>(Q, ntop - s);
        const Set& cur = S[s & 1];
        const Set& nxt = S[(s & 1) ^ 1];
        const CsrView V{cur.rp, cur.ci, cur.va, (int)n, cur.lr, M0.n_long, A->long_thresh, kSplitThresh,
                        nullptr, nullptr, 0, nullptr, nullptr, 0};
        KT_HIP(launch_pair_reg_dyn(C, (int)n, nnz0, V, A->unit_values, dTi, dTj, B, it, KT_FUN_EXP, tol, state,
                                   cur.dyn, st));
        KT_HIP(launch_greedy_edit(C, state, dTi, dTj, (int)(ntop - s), (int)n, A->long_thresh, cur.rp, cur.ci,
                                  cur.va, cur.lr, cur.dyn, nxt.rp, nxt.ci, nxt.va, nxt.lr, nxt.dyn, s, dsel, dselv,
                                  st));
    }
    ws.pair_host[1].ensure(sizeof(int) * 2 * (size_t)k + sizeof(double) * (size_t)k);
    double* hv = ws.pair_host[1].as<double>();
    int* hs = reinterpret_cast<int*>(hv + k);
    KT_HIP(hipMemcpyAsync(hv, dselv, sizeof(double) * k, hipMemcpyDeviceToHost, st));
    KT_HIP(hipMemcpyAsync(hs, dsel, sizeof(int) * 2 * k, hipMemcpyDeviceToHost, st));
    KT_HIP(hipStreamSynchronize(st));
    std::vector<int64_t> ei, ej;
    ei.reserve(k);
    ej.reserve(k);
    double total = 0.0;
    for (int s = 0; s < k; ++s) {
        if (hs[2 * s] < 0) {
            // the host loop (and the reference) had already deleted the edges
            // of steps 0..s-1 when step s found no finite score: leave A so
            if (!ei.empty()) set_pairs(A, (int64_t)ei.size(), ei.data(), ej.data(), 0.0);
            fail(KT_ERR_ARG, "KRYLOV_MIOBI:: no finite candidate score");
        }
        ei.push_back(hs[2 * s]);
        ej.push_back(hs[2 * s + 1]);
        if (sel_i) sel_i[s] = ei[s];
        if (sel_j) sel_j[s] = ej[s];
        total += hv[s];
    }
    set_pairs(A, k, ei.data(), ej.data(), 0.0);  // the host copy (and a current twin) take the same edits
    *rob = total;
    *nsel = k;
    return true;
}

void miobi_checks(kt_matrix_s* A, int k, int make, int& it) {
    require_symmetric(A, "KRYLOV_MIOBI:: Adjacency matrix should be symmetric");  // :26-28
    if (it <= 0) it = (int)std::min<int64_t>(100, A->n);                        // :32-34
    if (!make && A->nnz < 2 * (int64_t)k)                                       // :63-65
        fail(KT_ERR_ARG, "KRYLOV_MIOBI:: edges to be removed are more than edges in the network");
}

}  // namespace
}  // namespace kt

extern "C" {

int kt_krylov_miobi(kt_matrix_t A, int k, int64_t nE, const int64_t* ei, const int64_t* ej,
                    double tol, int it, int make, double rescale, int64_t* sel_i, int64_t* sel_j,
                    double* rob, int64_t* nsel) {
    KT_GUARD_BEGIN
    if (!A || !rob || !nsel || (nE > 0 && (!ei || !ej))) fail(KT_ERR_ARG, "NULL argument");
    if (k < 0 || nE < 0) fail(KT_ERR_ARG, "negative k or candidate count");
    KT_HIP(hipSetDevice(A->ctx->device));
    miobi_checks(A, k, make, it);
    const double sg = make ? 1.0 : -1.0;
    const double B[4] = {0.0, sg / rescale, sg / rescale, 0.0};  // :78-84
    std::vector<int64_t> Ei(ei, ei + nE), Ej(ej, ej + nE);
    std::vector<double> xm;
    double total = 0.0;
    int64_t done = 0;
    const int64_t steps = std::min<int64_t>(k, nE);
    for (int64_t s = 0; s < steps; ++s) {  // :70
        double bv;
        const int64_t best = miobi_select(A, Ei, Ej, (int64_t)Ei.size(), B, sg, tol, it, make, xm, &bv);
        if (sel_i) sel_i[done] = Ei[best];
        if (sel_j) sel_j[done] = Ej[best];
        Ei.erase(Ei.begin() + best);  // :127
        Ej.erase(Ej.begin() + best);
        total += bv;
        ++done;
    }
    *rob = total;
    *nsel = done;
    KT_GUARD_END
}

int kt_greedy_krylov_steps(kt_matrix_t A, int k, int64_t Q, int64_t ntop, const int64_t* ti,
                           const int64_t* tj, double tol, int it, int make, double rescale, int64_t* sel_i,
                           int64_t* sel_j, double* rob, int64_t* nsel) {
    KT_GUARD_BEGIN
    if (!A || !rob || !nsel || (ntop > 0 && (!ti || !tj))) fail(KT_ERR_ARG, "NULL argument");
    if (k < 0 || Q < 1 || ntop < k) fail(KT_ERR_ARG, "greedy steps: need k >= 0, Q >= 1 and ntop >= k");
    KT_HIP(hipSetDevice(A->ctx->device));
    const double sg = make ? 1.0 : -1.0;
    const double B[4] = {0.0, sg / rescale, sg / rescale, 0.0};  // krylov_miobi.m:78-84
    std::vector<int64_t> Ti(ti, ti + ntop), Tj(tj, tj + ntop);
    if (!make && k > 0) {
        int itc = it;
        miobi_checks(A, 1, make, itc);
        if (greedy_steps_device(A, k, Q, Ti, Tj, B, tol, itc, sel_i, sel_j, rob, nsel)) return KT_OK;
    }
    std::vector<double> xm;
    double total = 0.0;
    int64_t done = 0;
    for (int s = 0; s < k; ++s) {  // greedy_krylov.m:80-93
        int itc = it;
        miobi_checks(A, 1, make, itc);  // krylov_miobi(A, 1, E, ...) checks its A each call
        std::vector<int64_t> Ei(Ti.begin(), Ti.begin() + std::min<int64_t>(Q, (int64_t)Ti.size()));
        std::vector<int64_t> Ej(Tj.begin(), Tj.begin() + (int64_t)Ei.size());
        double bv;
        const int64_t best = miobi_select(A, Ei, Ej, (int64_t)Ei.size(), B, sg, tol, itc, make, xm, &bv);
        const int64_t ci = Ei[best], cj = Ej[best];
        if (sel_i) sel_i[done] = ci;
        if (sel_j) sel_j[done] = cj;
        total += bv;
        ++done;
        // drop the selected pair from the ranking (greedy_krylov.m:84-86: first match)
        for (size_t h = 0; h < Ti.size(); ++h)
            if (Ti[h] == ci && Tj[h] == cj) {
                Ti.erase(Ti.begin() + h);
                Tj.erase(Tj.begin() + h);
                break;
            }
    }
    *rob = total;
    *nsel = done;
    KT_GUARD_END
}

}  // extern "C"
