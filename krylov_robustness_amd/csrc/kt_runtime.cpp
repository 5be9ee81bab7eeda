// kt_runtime.cpp -- contexts, device-resident matrices, errors, profiling.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>

#include <rocblas/rocblas.h>

#include "kt_internal.h"
#include "kt_launch.h"
#include "kt_pool.h"

namespace kt {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

// timing-only events: no system-scope fence when recorded, i.e. no L2
// write-back / invalidate between the profiled launches (the stream syncs
// order everything the host reads)
static constexpr unsigned kProfEventFlags = hipEventDisableSystemFence;

void prof_begin(kt_context_s* ctx, int slot, hipStream_t st, int tag) {
    if (!ctx->profile) return;
    ProfSlot& s = ctx->prof[slot];
    if (s.used + 2 > s.ev.size()) {
        for (int i = 0; i < 512; ++i) {
            hipEvent_t e;
            KT_HIP(hipEventCreateWithFlags(&e, kProfEventFlags));
            s.ev.push_back(e);
        }
    }
    if (!s.anchored) {  // the time origin of every interval until the next reset
        if (!s.anchor) KT_HIP(hipEventCreateWithFlags(&s.anchor, kProfEventFlags));
        KT_HIP(hipEventRecord(s.anchor, st ? st : ctx->stream));
        s.anchored = true;
    }
    KT_HIP(hipEventRecord(s.ev[s.used], st ? st : ctx->stream));
    s.tags.push_back(tag);
}

void prof_end(kt_context_s* ctx, int slot, hipStream_t st) {
    if (!ctx->profile) return;
    ProfSlot& s = ctx->prof[slot];
    KT_HIP(hipEventRecord(s.ev[s.used + 1], st ? st : ctx->stream));
    s.used += 2;
}

// The hot path records a start/stop event pair around every launch of the
// profiled kernels.  Folding them in takes ~3 hipEventElapsedTime calls per
// launch (~6 ms per evaluation of the bench workload), so kt_slq_trace folds
// in the PREVIOUS call's events while its own sweeps run on the device, and
// the rest are folded in when the totals are read.
void prof_collect(kt_context_s* ctx, const size_t* upto, bool wait) {
    for (int k = 0; k < PROF_NSLOTS; ++k) {
        ProfSlot& s = ctx->prof[k];
        const size_t end = upto ? std::min(upto[k], s.used) : s.used;
        if (end < s.done + 2) continue;
        // the batch's events come from several sweep lanes (streams): the one
        // recorded last by the host need not complete last, so wait on each
        // (a completed event returns at once)
        if (wait)
            for (size_t i = s.done; i < end; ++i) KT_HIP(hipEventSynchronize(s.ev[i]));
        for (size_t i = s.done; i + 1 < end; i += 2) {
            float ms = 0.f, a = 0.f, b = 0.f;
            KT_HIP(hipEventElapsedTime(&ms, s.ev[i], s.ev[i + 1]));
            KT_HIP(hipEventElapsedTime(&a, s.anchor, s.ev[i]));
            KT_HIP(hipEventElapsedTime(&b, s.anchor, s.ev[i + 1]));
            s.iv.push_back({a, b});
            s.total_ms += ms;
            s.launches += 1;
            const int tag = s.tags[(i - s.done) / 2];
            auto it = std::find_if(s.by_tag.begin(), s.by_tag.end(), [&](const auto& e) { return e.first == tag; });
            if (it == s.by_tag.end()) s.by_tag.push_back({tag, {1, (double)ms}});
            else {
                it->second.first += 1;
                it->second.second += ms;
            }
        }
        s.tags.erase(s.tags.begin(), s.tags.begin() + (std::ptrdiff_t)((end - s.done) / 2));
        s.done = end;
    }
}

double prof_busy(const ProfSlot& s) {
    std::vector<std::pair<double, double>> iv(s.iv);
    std::sort(iv.begin(), iv.end());
    double busy = 0.0, cs = 0.0, ce = -1.0;
    bool open = false;
    for (auto& x : iv) {
        if (!open || x.first > ce) {
            if (open) busy += ce - cs;
            cs = x.first;
            ce = x.second;
            open = true;
        } else if (x.second > ce) {
            ce = x.second;
        }
    }
    if (open) busy += ce - cs;
    return busy;
}

void prof_recycle(kt_context_s* ctx) {
    for (auto& s : ctx->prof) {
        if (s.done == 0) continue;
        // events [done, used) are not folded in yet: move them to the front
        std::rotate(s.ev.begin(), s.ev.begin() + (std::ptrdiff_t)s.done, s.ev.begin() + (std::ptrdiff_t)s.used);
        s.used -= s.done;
        s.done = 0;
    }
}

void prof_reserve(kt_context_s* ctx, size_t per_slot) {
    for (auto& s : ctx->prof)
        while (s.ev.size() < per_slot) {
            hipEvent_t e;
            KT_HIP(hipEventCreateWithFlags(&e, kProfEventFlags));
            s.ev.push_back(e);
        }
}

void DevCSR::release() {
    if (blob) (void)hipFree(blob);
    blob = nullptr;
    blob_bytes = 0;
    rowptr = col = long_rows = perm = med_rows = short_tasks = med_tasks = nullptr;
    ck_beg = ck_end = sp_rows = sp_first = nullptr;
    val = nullptr;
    n_long = n_heavy = n_med = n_short = n_chunks = n_split = 0;
    built = false;
}

void build_csr(kt_matrix_s* A, const std::vector<int32_t>& new2old, DevCSR& out, bool sync) {
    const int64_t n = A->n, nnz = A->nnz;
    const bool ident = new2old.empty();
    const bool tasks = ident;  // the expmv term's task lists: natural order only
    auto orig = [&](int64_t r) -> int64_t { return ident ? r : new2old[r]; };
    std::vector<int32_t> rp32(n + 1), c32(std::max<int64_t>(nnz, 1));
    std::vector<double> v64(std::max<int64_t>(nnz, 1));
    rp32[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t o = orig(r);
        rp32[r + 1] = rp32[r] + (int32_t)(A->h_rowptr[o + 1] - A->h_rowptr[o]);
    }
    std::vector<std::pair<int32_t, double>> tmp;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t o = orig(r);
        const int64_t kb = A->h_rowptr[o], ke = A->h_rowptr[o + 1];
        if (ident) {  // natural order: copy a row that is already sorted (the usual
                      // case -- MATLAB CSC and set_entry keep rows sorted)
            bool sorted = true;
            for (int64_t k = kb + 1; k < ke && sorted; ++k) sorted = A->h_col[k - 1] < A->h_col[k];
            if (sorted) {
                std::copy(A->h_col.begin() + kb, A->h_col.begin() + ke, c32.begin() + rp32[r]);
                std::copy(A->h_val.begin() + kb, A->h_val.begin() + ke, v64.begin() + rp32[r]);
                continue;
            }
        }
        tmp.clear();
        for (int64_t k = kb; k < ke; ++k)
            tmp.push_back({ident ? A->h_col[k] : A->old2new[A->h_col[k]], A->h_val[k]});
        std::sort(tmp.begin(), tmp.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        for (size_t t = 0; t < tmp.size(); ++t) {
            c32[rp32[r] + t] = tmp[t].first;
            v64[rp32[r] + t] = tmp[t].second;
        }
    }
    std::vector<int32_t> lr;
    for (int64_t r = 0; r < n; ++r)
        if (rp32[r + 1] - rp32[r] > A->long_thresh) lr.push_back((int32_t)r);
    std::stable_sort(lr.begin(), lr.end(), [&](int32_t a, int32_t b) {
        return rp32[a + 1] - rp32[a] > rp32[b + 1] - rp32[b];
    });
    std::vector<int32_t> mr;  // medium rows (expmv terms), row order
    for (int64_t r = 0; r < n; ++r) {
        const int32_t d = rp32[r + 1] - rp32[r];
        if (d > kMedThresh && d <= A->long_thresh) mr.push_back((int32_t)r);
    }
    // short-row task list of the row-blocked expmv term (natural order only):
    // rows of degree <= kMedThresh (and not long) as {row, beg, end, 0},
    // counting-sorted by degree (descending; rows in order within a degree)
    // inside each window of consecutive rows
    std::vector<int32_t> st4;
    if (tasks) {
        const int dmax = std::min(kMedThresh, A->long_thresh);
        // sorted within windows of 4,096 consecutive rows: a wave's rows take
        // the same number of gather rounds while the F / b rows a launch
        // touches at one time stay as local as in natural order (config-4
        // expmv trace_exp, same box: natural 1,453 ms, whole-matrix sort
        // 1,432, windows of 4,096 1,401; profiles/r06/expmv_rows_ab).
        // KT_EXPMV_SORTWIN (A/B) sets the window (0: the whole matrix).
        const char* sw = std::getenv("KT_EXPMV_SORTWIN");
        const int64_t win = sw ? std::max<int64_t>(0, std::atoll(sw)) : 4096;
        const int64_t W = win > 0 ? win : n;
        std::vector<int64_t> cnt(dmax + 2);
        size_t ns = 0;
        for (int64_t r = 0; r < n; ++r) ns += (rp32[r + 1] - rp32[r] <= dmax);
        st4.assign(4 * ns, 0);
        int64_t t0 = 0;
        for (int64_t w0 = 0; w0 < n; w0 += W) {
            const int64_t w1 = std::min(n, w0 + W);
            std::fill(cnt.begin(), cnt.end(), 0);
            for (int64_t r = w0; r < w1; ++r) {
                const int32_t d = rp32[r + 1] - rp32[r];
                if (d <= dmax) cnt[dmax - d + 1]++;
            }
            cnt[0] = t0;
            for (int i = 1; i <= dmax + 1; ++i) cnt[i] += cnt[i - 1];
            t0 = cnt[dmax + 1];
            for (int64_t r = w0; r < w1; ++r) {
                const int32_t d = rp32[r + 1] - rp32[r];
                if (d > dmax) continue;
                const int64_t t = cnt[dmax - d]++;
                st4[4 * t] = (int32_t)r;
                st4[4 * t + 1] = rp32[r];
                st4[4 * t + 2] = rp32[r + 1];
            }
        }
    }
    // hub-row chunk table (block SpMM)
    std::vector<int32_t> ckb, cke, spr, spf(1, 0);
    for (int32_t r : lr) {  // heaviest first
        const int32_t b = rp32[r], e = rp32[r + 1];
        if (e - b <= kSplitThresh) continue;
        spr.push_back(r);
        for (int32_t k = b; k < e; k += kChunkNnz) {
            ckb.push_back(k);
            cke.push_back(std::min(e, k + kChunkNnz));
        }
        spf.push_back((int32_t)ckb.size());
    }
    // One device allocation holds every array (256-B aligned slices), filled
    // by ONE async copy out of a pinned staging buffer and one stream sync:
    // greedy rebuilds the natural copy after every edge edit, and a pageable
    // hipMemcpy per array stages and syncs each time.
    struct Seg {
        void** dst;
        const void* src;
        size_t bytes;
    };
    std::vector<Seg> segs;
    auto add = [&](auto*& dst, const void* src, size_t bytes) {
        segs.push_back({reinterpret_cast<void**>(&dst), src, bytes});
    };
    add(out.rowptr, rp32.data(), sizeof(int) * (n + 1));
    add(out.col, c32.data(), sizeof(int) * c32.size());
    add(out.val, v64.data(), sizeof(double) * v64.size());
    add(out.long_rows, lr.data(), sizeof(int) * lr.size());
    add(out.med_rows, mr.data(), sizeof(int) * mr.size());
    add(out.short_tasks, st4.data(), sizeof(int) * st4.size());
    std::vector<int32_t> mt4;
    if (tasks) {
        mt4.assign(4 * mr.size(), 0);
        for (size_t i = 0; i < mr.size(); ++i) {
            mt4[4 * i] = mr[i];
            mt4[4 * i + 1] = rp32[mr[i]];
            mt4[4 * i + 2] = rp32[mr[i] + 1];
        }
    }
    add(out.med_tasks, mt4.data(), sizeof(int) * mt4.size());
    if (!spr.empty()) {
        add(out.ck_beg, ckb.data(), sizeof(int) * ckb.size());
        add(out.ck_end, cke.data(), sizeof(int) * cke.size());
        add(out.sp_rows, spr.data(), sizeof(int) * spr.size());
        add(out.sp_first, spf.data(), sizeof(int) * spf.size());
    }
    if (!ident) add(out.perm, new2old.data(), sizeof(int) * n);
    auto slice = [](size_t b) { return (std::max<size_t>(b, 16) + 255) & ~(size_t)255; };
    size_t total = 0;
    for (const Seg& g : segs) total += slice(g.bytes);
    // buffers may be reused: nothing of this context may still read them, and
    // the previous build's copy out of the staging buffer is done
    KT_HIP(hipStreamSynchronize(A->ctx->stream));
    for (hipStream_t st : A->ctx->aux_stream)
        if (st) KT_HIP(hipStreamSynchronize(st));
    try {
        if (total > out.blob_bytes || !out.blob) {
            if (out.blob) (void)hipFree(out.blob);
            out.blob = nullptr;
            out.blob_bytes = 0;
            KT_HIP(hipMalloc(&out.blob, total));
            out.blob_bytes = total;
        }
        out.stage.ensure(total);
        char* h = out.stage.as<char>();
        size_t off = 0;
        out.ck_beg = out.ck_end = out.sp_rows = out.sp_first = nullptr;
        out.perm = nullptr;
        out.short_tasks = out.med_tasks = nullptr;
        for (const Seg& g : segs) {
            if (g.bytes) std::memcpy(h + off, g.src, g.bytes);
            *g.dst = out.blob + off;
            off += slice(g.bytes);
        }
        KT_HIP(hipMemcpyAsync(out.blob, h, total, hipMemcpyHostToDevice, A->ctx->stream));
        // the copy is ordered before later work on the context's stream; other
        // streams may read the arrays, so the default waits for it (the
        // staging buffer is not rewritten before the next build's sync above)
        if (sync) KT_HIP(hipStreamSynchronize(A->ctx->stream));
        out.n_long = (int)lr.size();
        out.n_heavy = 0;
        while (out.n_heavy < out.n_long &&
               rp32[lr[out.n_heavy] + 1] - rp32[lr[out.n_heavy]] > kExpmvCoopThresh) ++out.n_heavy;
        out.n_med = (int)mr.size();
        out.n_short = (int)(st4.size() / 4);
        if (!tasks) out.short_tasks = out.med_tasks = nullptr;
        out.n_split = (int)spr.size();
        out.n_chunks = (int)ckb.size();
    } catch (...) {
        out.release();
        throw;
    }
    out.built = true;
}

// Drop the device copies after the host CSR changed; hub_csr / natural_csr
// rebuild them on next use.
void refresh_device(kt_matrix_s* A) {
    A->hub.invalidate();
    A->nat.invalidate();
    A->version++;  // a twin copy (kt_krylov.cpp) is now stale
    A->unit_values = std::all_of(A->h_val.begin(), A->h_val.end(), [](double v) { return v == 1.0; });
}

// degree-relabelled CSR of the probe hot path, built on first use
const DevCSR& hub_csr(kt_matrix_s* A) {
    if (A->hub.built) return A->hub;
    const int64_t n = A->n;
    // degree-descending relabelling (stable, so ties keep original order)
    A->new2old.resize(n);
    A->old2new.resize(n);
    for (int64_t i = 0; i < n; ++i) A->new2old[i] = (int32_t)i;
    std::stable_sort(A->new2old.begin(), A->new2old.end(), [&](int32_t a, int32_t b) {
            return A->h_rowptr[a + 1] - A->h_rowptr[a] > A->h_rowptr[b + 1] - A->h_rowptr[b];
        });
    for (int64_t r = 0; r < n; ++r) A->old2new[A->new2old[r]] = (int32_t)r;
    build_csr(A, A->new2old, A->hub);
    return A->hub;
}

const DevCSR& natural_csr(kt_matrix_s* A) {
    if (!A->nat.built) build_csr(A, std::vector<int32_t>(), A->nat);
    return A->nat;
}

// the same, without waiting for the upload: for callers whose every reader of
// the arrays is ordered after the context's stream (the greedy candidate
// paths, which rebuild the copy after every edge edit)
const DevCSR& natural_csr_ordered(kt_matrix_s* A) {
    if (!A->nat.built) build_csr(A, std::vector<int32_t>(), A->nat, false);
    return A->nat;
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

int kt_abi_version(void) { return KT_ABI_VERSION; }

const char* kt_last_error(void) { return kt::g_last_error.c_str(); }

int kt_device_count(int* count) {
    KT_GUARD_BEGIN
    if (!count) fail(KT_ERR_ARG, "count is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *count = c;
    KT_GUARD_END
}

int kt_context_create(int device, kt_context_t* out) {
    KT_GUARD_BEGIN
    if (!out) fail(KT_ERR_ARG, "ctx out is NULL");
    int c = 0;
    KT_HIP(hipGetDeviceCount(&c));
    if (device < 0 || device >= c) fail(KT_ERR_ARG, "device index out of range");
    KT_HIP(hipSetDevice(device));
    auto* ctx = new kt_context_s();
    ctx->device = device;
    hipDeviceProp_t prop;
    KT_HIP(hipGetDeviceProperties(&prop, device));
    ctx->num_cu = prop.multiProcessorCount;
    if (const char* f = getenv("KT_SLQ_YFORM")) ctx->yform = f[0] != '0';
    KT_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    *out = ctx;
    KT_GUARD_END
}

int kt_context_destroy(kt_context_t ctx) {
    KT_GUARD_BEGIN
    if (!ctx) return KT_OK;
    for (auto& w : ctx->workers)  // joined before the helper / twin contexts they drive go away
        if (w) {
            ctx->workers_free(w);
            w = nullptr;
        }
    if (ctx->helper) {
        (void)kt_context_destroy(ctx->helper);
        ctx->helper = nullptr;
    }
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto a : ctx->aux_stream)
        if (a) (void)hipStreamSynchronize(a);
    for (auto& s : ctx->prof) {
        for (auto e : s.ev) (void)hipEventDestroy(e);
        if (s.anchor) (void)hipEventDestroy(s.anchor);
    }
    for (auto a : ctx->aux_stream)
        if (a) (void)hipStreamSynchronize(a);
    Workspace& w = ctx->ws;
    for (auto& b : w.sweep) {
        b.X0.release(); b.X1.release(); b.Y.release(); b.partial.release();
        b.coef.release(); b.scales.release(); b.k2s.release(); b.trec.release(); b.hist.release();
    }
    w.small.release(); w.small2.release(); w.qrtmp.release();
    w.eigA.release(); w.eigW.release(); w.eigInfo.release();
    w.norm_part.release();
    ctx->pool.clear();
    if (ctx->blas) rocblas_destroy_handle(static_cast<rocblas_handle>(ctx->blas));
    if (w.comb_ev) (void)hipEventDestroy(w.comb_ev);
    if (w.qrfac_ev) (void)hipEventDestroy(w.qrfac_ev);
    if (w.qrm_ev) (void)hipEventDestroy(w.qrm_ev);
    if (w.colsplit_ev) (void)hipEventDestroy(w.colsplit_ev);
    for (auto& b : w.host_trec) b.release();
    for (auto& pd : w.slq_pend)
        for (auto& e : pd.done)
            if (e) (void)hipEventDestroy(e);
    for (auto a : ctx->aux_stream)
        if (a) (void)hipStreamDestroy(a);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    KT_GUARD_END
}

int kt_matrix_create_csc(kt_context_t ctx, int64_t n, const int64_t* colptr, const int64_t* rowind,
                         const double* vals, int check_symmetric, kt_matrix_t* out) {
    KT_GUARD_BEGIN
    // the arrays are validated before the context is touched (a malformed
    // CSC never reaches the device, and the checks run without a GPU)
    if (!out || !colptr || (!rowind && n > 0)) fail(KT_ERR_ARG, "NULL argument");
    if (n < 0) fail(KT_ERR_ARG, "negative dimension");
    if (colptr[0] != 0) fail(KT_ERR_ARG, "column pointers must start at 0 (jc[0] == 0)");
    const int64_t nnz = colptr[n];
    if (n >= (int64_t(1) << 31) || nnz >= (int64_t(1) << 31))
        fail(KT_ERR_UNSUPPORTED, "n and nnz must be < 2^31 (int32 device indices)");
    for (int64_t j = 0; j < n; ++j)
        if (colptr[j + 1] < colptr[j]) fail(KT_ERR_ARG, "column pointers not monotone");
    for (int64_t k = 0; k < nnz; ++k)
        if (rowind[k] < 0 || rowind[k] >= n) fail(KT_ERR_ARG, "row index out of range");
    if (!ctx) fail(KT_ERR_ARG, "NULL context");

    auto* A = new kt_matrix_s();
    A->ctx = ctx;
    A->n = n;
    A->nnz = nnz;
    // CSC of a symmetric matrix == CSR; keep the column-sorted host copy.
    A->h_rowptr.assign(colptr, colptr + n + 1);
    A->h_col.resize(nnz);
    A->h_val.resize(nnz);
    for (int64_t k = 0; k < nnz; ++k) {
        A->h_col[k] = (int32_t)rowind[k];
        A->h_val[k] = vals ? vals[k] : 1.0;
    }
    // sort indices within each row (MATLAB keeps them sorted; be defensive)
    for (int64_t i = 0; i < n; ++i) {
        int64_t b = A->h_rowptr[i], e = A->h_rowptr[i + 1];
        bool sorted = true;
        for (int64_t k = b + 1; k < e; ++k)
            if (A->h_col[k] < A->h_col[k - 1]) { sorted = false; break; }
        if (!sorted) {
            std::vector<std::pair<int32_t, double>> t(e - b);
            for (int64_t k = b; k < e; ++k) t[k - b] = {A->h_col[k], A->h_val[k]};
            std::sort(t.begin(), t.end(),
                      [](const auto& x, const auto& y) { return x.first < y.first; });
            for (int64_t k = b; k < e; ++k) { A->h_col[k] = t[k - b].first; A->h_val[k] = t[k - b].second; }
        }
    }
    if (check_symmetric) {
        // transpose by counting sort and compare entry by entry
        std::vector<int64_t> tp(n + 1, 0);
        for (int64_t k = 0; k < nnz; ++k) tp[A->h_col[k] + 1]++;
        for (int64_t i = 0; i < n; ++i) tp[i + 1] += tp[i];
        std::vector<int32_t> tc(nnz);
        std::vector<double> tv(nnz);
        std::vector<int64_t> pos(tp.begin(), tp.end() - 1);
        for (int64_t i = 0; i < n; ++i)
            for (int64_t k = A->h_rowptr[i]; k < A->h_rowptr[i + 1]; ++k) {
                int64_t d = pos[A->h_col[k]]++;
                tc[d] = (int32_t)i;
                tv[d] = A->h_val[k];
            }
        bool sym = std::equal(tp.begin(), tp.end(), A->h_rowptr.begin()) &&
                   std::equal(tc.begin(), tc.end(), A->h_col.begin()) &&
                   std::equal(tv.begin(), tv.end(), A->h_val.begin());
        if (!sym) {
            delete A;
            fail(KT_ERR_NOT_HERMITIAN, "FUN_AND_GRAD_KRYLOV:: matrix A is not Hermitian");
        }
        A->symmetric = 1;
    }
    try {
        KT_HIP(hipSetDevice(ctx->device));
        refresh_device(A);
        (void)hub_csr(A);
    } catch (...) {
        A->hub.release();
        delete A;
        throw;
    }
    *out = A;
    KT_GUARD_END
}

int kt_matrix_destroy(kt_matrix_t A) {
    KT_GUARD_BEGIN
    if (!A) return KT_OK;
    (void)hipSetDevice(A->ctx->device);
    // every lane: kt_slq_submit leaves sweeps queued on the aux streams that
    // read this matrix's CSR until they are collected
    (void)hipStreamSynchronize(A->ctx->stream);
    for (hipStream_t a : A->ctx->aux_stream)
        if (a) (void)hipStreamSynchronize(a);
    for (auto& pd : A->ctx->ws.slq_pend)  // an uncollected ticket of A: collect now fails
        if (pd.A == A) pd.A = nullptr;
    if (A->twin) kt_matrix_destroy(A->twin);
    if (A->twin_ctx) kt_context_destroy(A->twin_ctx);
    (void)hipSetDevice(A->ctx->device);
    A->hub.release();
    A->nat.release();
    delete A;
    KT_GUARD_END
}

int kt_matrix_info(kt_matrix_t A, int64_t* n, int64_t* nnz) {
    KT_GUARD_BEGIN
    if (!A) fail(KT_ERR_ARG, "A is NULL");
    if (n) *n = A->n;
    if (nnz) *nnz = A->nnz;
    KT_GUARD_END
}

int kt_profile_enable(kt_context_t ctx, int enable) {
    KT_GUARD_BEGIN
    if (!ctx) fail(KT_ERR_ARG, "ctx is NULL");
    KT_HIP(hipSetDevice(ctx->device));
    if (enable != 0) prof_reserve(ctx, 8192);  // event pairs for ~2 calls, created here, not in the timed code
    ctx->profile = enable != 0;
    KT_GUARD_END
}

int kt_profile_read(kt_context_t ctx, int kernel, int64_t* launches, double* total_ms) {
    KT_GUARD_BEGIN
    if (!ctx || kernel < 0 || kernel >= PROF_NSLOTS) fail(KT_ERR_ARG, "bad profile query");
    KT_HIP(hipSetDevice(ctx->device));
    prof_collect(ctx, nullptr, true);
    if (launches) *launches = ctx->prof[kernel].launches;
    if (total_ms) *total_ms = ctx->prof[kernel].total_ms;
    KT_GUARD_END
}

int kt_context_stat(kt_context_t ctx, int stat, int64_t* value) {
    KT_GUARD_BEGIN
    if (!ctx || !value || stat < 0 || stat > 4) fail(KT_ERR_ARG, "bad stat query");
    const int64_t v[5] = {ctx->yform_redone, ctx->fu_dense, ctx->fu_last_cols, ctx->expmv_calls,
                          ctx->expmv_terms};
    *value = v[stat];
    KT_GUARD_END
}

int kt_host_threads(void) { return kt::HostPool::get().threads(); }

int kt_profile_reset(kt_context_t ctx) {
    KT_GUARD_BEGIN
    if (!ctx) fail(KT_ERR_ARG, "ctx is NULL");
    KT_HIP(hipSetDevice(ctx->device));
    // events of launches still in flight would be recorded into reused slots
    prof_collect(ctx, nullptr, true);
    for (auto& s : ctx->prof) {
        s.launches = 0;
        s.total_ms = 0.0;
        s.iv.clear();
        s.anchored = false;
        s.tags.clear();
        s.by_tag.clear();
        s.used = 0;
        s.done = 0;
    }
    KT_GUARD_END
}

int kt_debug_delay(kt_context_t ctx, int lane, double microseconds) {
    KT_GUARD_BEGIN
    if (!ctx || lane < 0 || lane > 3) fail(KT_ERR_ARG, "kt_debug_delay: bad context or lane");
    if (!(microseconds >= 0.0 && microseconds <= 1e6)) fail(KT_ERR_ARG, "kt_debug_delay: 0 <= us <= 1e6");
    KT_HIP(hipSetDevice(ctx->device));
    if (lane && !ctx->aux_stream[lane - 1])
        KT_HIP(hipStreamCreateWithFlags(&ctx->aux_stream[lane - 1], hipStreamNonBlocking));
    KT_HIP(launch_delay(microseconds, lane ? ctx->aux_stream[lane - 1] : ctx->stream));
    KT_GUARD_END
}

int kt_profile_read_width(kt_context_t ctx, int kernel, int width, int64_t* launches, double* total_ms) {
    KT_GUARD_BEGIN
    if (!ctx || kernel < 0 || kernel >= PROF_NSLOTS) fail(KT_ERR_ARG, "bad profile query");
    KT_HIP(hipSetDevice(ctx->device));
    prof_collect(ctx, nullptr, true);
    int64_t l = 0;
    double ms = 0.0;
    for (const auto& e : ctx->prof[kernel].by_tag)
        if (e.first == width) {
            l = e.second.first;
            ms = e.second.second;
        }
    if (launches) *launches = l;
    if (total_ms) *total_ms = ms;
    KT_GUARD_END
}

int kt_profile_busy(kt_context_t ctx, int kernel, double* busy_ms) {
    KT_GUARD_BEGIN
    if (!ctx || !busy_ms || kernel < 0 || kernel >= PROF_NSLOTS) fail(KT_ERR_ARG, "bad profile query");
    KT_HIP(hipSetDevice(ctx->device));
    prof_collect(ctx, nullptr, true);
    *busy_ms = prof_busy(ctx->prof[kernel]);
    KT_GUARD_END
}

}  // extern "C"
