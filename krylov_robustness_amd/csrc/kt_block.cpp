// kt_block.cpp -- tall-skinny device block operations (rocBLAS dgemm for the
// plain GEMM shapes, the HIP SpMM kernel for A*X) and CholQR.
#include <cstdlib>
#include <cstring>

#include "kt_block.h"

#include <rocsolver/rocsolver.h>

#include <cfloat>
#include <cmath>

#include "kt_launch.h"

namespace kt {

int pow2_at_least(int b) {
    int p = 1;
    while (p < b) p <<= 1;
    return p;
}

rocblas_handle blas(kt_context_s* ctx) {
    if (!ctx->blas) {
        rocblas_handle h;
        if (rocblas_create_handle(&h) != rocblas_status_success)
            fail(KT_ERR_HIP, "rocblas_create_handle failed");
        rocblas_set_stream(h, ctx->stream);
        rocblas_set_pointer_mode(h, rocblas_pointer_mode_host);
        ctx->blas = h;
    }
    return static_cast<rocblas_handle>(ctx->blas);
}

static void rb(rocblas_status s, const char* what) {
    if (s != rocblas_status_success)
        fail(KT_ERR_HIP, std::string(what) + ": " + rocblas_status_to_string(s));
}

void* ScratchPool::take(size_t want, size_t* got) {
    size_t best = free.size();
    for (size_t i = 0; i < free.size(); ++i)
        if (free[i].first >= want && free[i].first <= 4 * want &&
            (best == free.size() || free[i].first < free[best].first))
            best = i;
    if (best < free.size()) {
        void* p = free[best].second;
        *got = free[best].first;
        free.erase(free.begin() + (std::ptrdiff_t)best);
        return p;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess && !free.empty()) {  // HBM full: give the idle blocks back, retry
        (void)hipGetLastError();
        clear();
        e = hipMalloc(&p, want);
    }
    if (e != hipSuccess) fail(KT_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
    held += want;
    *got = want;
    return p;
}

void ScratchPool::give(void* p, size_t bytes) {
    if (!p) return;
    free.push_back({bytes, p});
    if (free.size() > 64) {  // bound the list: drop the smallest idle block
        size_t s = 0;
        for (size_t i = 1; i < free.size(); ++i)
            if (free[i].first < free[s].first) s = i;
        (void)hipFree(free[s].second);
        held -= free[s].first;
        free.erase(free.begin() + (std::ptrdiff_t)s);
    }
}

void ScratchPool::clear() {
    for (auto& f : free) {
        (void)hipFree(f.second);
        held -= f.first;
    }
    free.clear();
}

void DevMat::alloc(kt_context_s* c, int64_t n_, int ld_, bool zero) {
    n = n_;
    ld = ld_;
    const size_t want = sizeof(double) * (size_t)std::max<int64_t>(n, 1) * (size_t)std::max(ld, 1);
    if (!ptr || ctx != c || bytes < want) {
        release();
        ctx = c;
        ptr = ctx->pool.take(want, &bytes);
    }
    if (zero) KT_HIP(hipMemsetAsync(ptr, 0, want, ctx->stream));
}

void DevMat::release() {
    if (ptr && ctx) ctx->pool.give(ptr, bytes);
    ptr = nullptr;
    bytes = 0;
    ctx = nullptr;
}


void gram(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px, const double* Y,
          int ldy, int py, std::vector<double>& G) {
    G.assign((size_t)px * py, 0.0);
    if (px == 0 || py == 0 || n == 0) return;
    const double* d = gram_device(ctx, n, X, ldx, px, Y, ldy, py);
    PinnedBuf& pb = ctx->ws.pin_gram;
    pb.ensure(sizeof(double) * G.size());
    KT_HIP(hipMemcpyAsync(pb.ptr, d, sizeof(double) * G.size(), hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
    std::memcpy(G.data(), pb.ptr, sizeof(double) * G.size());
}

// gram / combine go through kt_gemm_ts.hip for tall blocks and through
// rocBLAS dgemm below 8,192 rows: on India (n = 3,228) the pipelined
// fun_update with the ts kernels stalled 20-30 ms at the first stream
// operation of every call (profiles/r03_fg_exp_stall.txt), with rocBLAS not
static bool rocblas_gemm_path(int64_t n) {
    return n < 8192;
}

const double* gram_device(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px, const double* Y,
                          int ldy, int py) {
    DevBuf& d = ctx->ws.small;
    if (px == 0 || py == 0 || n == 0) {
        d.ensure(sizeof(double) * (size_t)std::max(px * py, 1));
        KT_HIP(hipMemsetAsync(d.ptr, 0, sizeof(double) * (size_t)std::max(px * py, 1), ctx->stream));
        return d.as<double>();
    }
    const double one = 1.0, zero = 0.0;
    const int64_t count = (int64_t)px * py;
    if (!rocblas_gemm_path(n)) {  // kt_gemm_ts.hip: MFMA row-chunk partials + fixed-order slab sum
        const int S = gram_ts_chunks(n);
        d.ensure(sizeof(double) * (size_t)count * (S + 1));
        KT_HIP(launch_gram_ts(n, X, ldx, px, Y, ldy, py, d.as<double>() + count, d.as<double>(), ctx->stream));
        return d.as<double>();
    }
    // column-major views: X is (ldx x n), Y is (ldy x n);  G = X(0:px,:) Y(0:py,:)'.
    // The reduction dimension n is long and the output tiny, so split it over
    // S row chunks (one strided-batched GEMM) and add the S slabs in a fixed
    // order: enough workgroups to fill the chip.
    int S = (int)std::min<int64_t>(64, std::max<int64_t>(1, n / 1024));
    while (S > 1 && count * S > (int64_t)1 << 24) S /= 2;
    const int64_t chunk = n / S;
    const int64_t rem = n - chunk * S;
    const int slabs = S + (rem > 0 ? 1 : 0);
    d.ensure(sizeof(double) * (size_t)count * (slabs + 1));
    double* part = d.as<double>() + count;
    if (S == 1 && rem == 0) {
        rb(rocblas_dgemm(blas(ctx), rocblas_operation_none, rocblas_operation_transpose, px, py,
                         (rocblas_int)n, &one, X, ldx, Y, ldy, &zero, d.as<double>(), px),
           "rocblas_dgemm(gram)");
    } else {
        rb(rocblas_dgemm_strided_batched(blas(ctx), rocblas_operation_none, rocblas_operation_transpose,
                                         px, py, (rocblas_int)chunk, &one, X, ldx, chunk * ldx, Y, ldy,
                                         chunk * ldy, &zero, part, px, count, S),
           "rocblas_dgemm_strided_batched(gram)");
        if (rem > 0)
            rb(rocblas_dgemm(blas(ctx), rocblas_operation_none, rocblas_operation_transpose, px, py,
                             (rocblas_int)rem, &one, X + chunk * S * ldx, ldx, Y + chunk * S * ldy, ldy,
                             &zero, part + count * S, px),
               "rocblas_dgemm(gram tail)");
        KT_HIP(launch_sum_slabs((int)count, slabs, part, d.as<double>(), ctx->stream));
    }
    return d.as<double>();
}

void combine_device(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px, const double* dC, int q,
                    double alpha, double beta, double* Y, int ldy) {
    if (q == 0 || px == 0) return;
    if (!rocblas_gemm_path(n)) {
        KT_HIP(launch_combine_ts(n, X, ldx, px, dC, q, alpha, beta, Y, ldy, ctx->stream));
        return;
    }
    // Yc (q x n) = beta Yc + alpha C' (q x px) * Xc (px x n), C on the device
    rb(rocblas_dgemm(blas(ctx), rocblas_operation_transpose, rocblas_operation_none, q,
                     (rocblas_int)n, px, &alpha, dC, px, X, ldx, &beta, Y, ldy),
       "rocblas_dgemm(combine_device)");
}

void combine(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px,
             const std::vector<double>& C, int q, double beta, double* Y, int ldy) {
    if (q == 0) return;
    if (px == 0) {
        if (beta != 1.0) fail(KT_ERR_ARG, "combine: empty X with beta != 1");
        return;
    }
    DevBuf& d = ctx->ws.small2;
    const size_t bytes = sizeof(double) * (size_t)px * q;
    // C goes through a pinned staging buffer, so the caller may free C at once
    // and the stream is not drained; the staging buffer is only rewritten once
    // the previous upload out of it has completed (event)
    const double one = 1.0;
    Workspace& ws = ctx->ws;
    if (ws.comb_pending) KT_HIP(hipEventSynchronize(ws.comb_ev));
    ws.comb_pending = false;
    if (!ws.comb_ev) KT_HIP(hipEventCreateWithFlags(&ws.comb_ev, hipEventDisableTiming));
    ws.pin_comb.ensure(bytes);
    std::memcpy(ws.pin_comb.ptr, C.data(), bytes);
    d.ensure(bytes);
    KT_HIP(hipMemcpyAsync(d.ptr, ws.pin_comb.ptr, bytes, hipMemcpyHostToDevice, ctx->stream));
    KT_HIP(hipEventRecord(ws.comb_ev, ctx->stream));
    ws.comb_pending = true;
    // Yc (q x n) = beta Yc + C' (q x px) * Xc (px x n)
    if (!rocblas_gemm_path(n)) {
        KT_HIP(launch_combine_ts(n, X, ldx, px, d.as<double>(), q, 1.0, beta, Y, ldy, ctx->stream));
        return;
    }
    rb(rocblas_dgemm(blas(ctx), rocblas_operation_transpose, rocblas_operation_none, q,
                     (rocblas_int)n, px, &one, d.as<double>(), px, X, ldx, &beta, Y, ldy),
       "rocblas_dgemm(combine)");
}

// Every block SpMM: Y[:, 0:slices P] = A X over `slices` P-wide column slices
// of the natural-order CSR, hub rows through the chunk table + combine.
static void block_spmm(kt_matrix_s* A, int P, const double* X, int ldx, double* Y, int ldy, int slices,
                       const int* skip) {
    kt_context_s* ctx = A->ctx;
    const int n = (int)A->n;
    const DevCSR& M = natural_csr(A);  // block paths run in the reference's row order
    const int grid = spmm_grid(n, P, ctx->num_cu * 4);
    const int lblocks = long_blocks_for(M.n_long, ctx->num_cu * 2);
    const int cblocks = M.n_chunks ? std::min((M.n_chunks + 7) / 8, ctx->num_cu * 2) : 0;
    double* ck_part = nullptr;
    if (M.n_chunks) {
        ctx->ws.ck_part.ensure(sizeof(double) * (size_t)M.n_chunks * P * slices);
        ck_part = ctx->ws.ck_part.as<double>();
    }
    const CsrView V{M.rowptr, M.col, M.val, n, M.long_rows, M.n_long, A->long_thresh, kSplitThresh,
                    M.ck_beg, M.ck_end, M.n_chunks, M.sp_rows, M.sp_first, M.n_split};
    KT_HIP(launch_spmm_block(P, (A->unit_values ? 2 : 0) | (ctx->k1_flags & 4), grid + lblocks + cblocks, V,
                             X, ldx, Y, ldy, lblocks, cblocks, ck_part, ctx->stream, slices, skip));
}

void spmm(kt_matrix_s* A, const double* X, int ldx, double* Y, int ldy, int cols) {
    const int P = pow2_at_least(std::max(cols, 1));
    if (P > 128) fail(KT_ERR_UNSUPPORTED, "block width > 128");
    block_spmm(A, P, X, ldx, Y, ldy, 1, nullptr);
}

// Y[:, 0:cols] = A X[:, 0:cols] for cols > 128 in ONE launch: ceil(cols/128)
// column slices of width 128 on grid.y (ldx, ldy >= slices * 128; columns
// past `cols` are computed too, they must hold finite values).  skip: see
// k_spmm_block.
void spmm_slices(kt_matrix_s* A, const double* X, int ldx, double* Y, int ldy, int cols,
                 const int* skip) {
    if (cols <= 128) {
        block_spmm(A, pow2_at_least(std::max(cols, 1)), X, ldx, Y, ldy, 1, skip);
        return;
    }
    const int slices = (cols + 127) / 128;
    if (ldx < slices * 128 || ldy < slices * 128) fail(KT_ERR_ARG, "spmm_slices: leading dimension");
    block_spmm(A, 128, X, ldx, Y, ldy, slices, skip);
}

void copy_cols(kt_context_s* ctx, int64_t n, const double* X, int ldx, double* Y, int ldy,
               int cols) {
    if (n == 0 || cols == 0) return;
    KT_HIP(hipMemcpy2DAsync(Y, sizeof(double) * ldy, X, sizeof(double) * ldx,
                            sizeof(double) * cols, (size_t)n, hipMemcpyDeviceToDevice,
                            ctx->stream));
}

void zero_cols(kt_context_s* ctx, int64_t n, double* X, int ldx, int cols) {
    if (n == 0 || cols == 0) return;
    KT_HIP(hipMemset2DAsync(X, sizeof(double) * ldx, 0, sizeof(double) * cols, (size_t)n,
                            ctx->stream));
}

void upload_rows(kt_matrix_s* A, const double* H, int cols, double* D, int ldd) {
    const int64_t n = A->n;
    if (n == 0 || cols == 0) return;
    // Mostly-zero blocks (the node selectors U of fun_and_grad_krylov_* and
    // the greedy candidates, e_i columns) travel as their nonzeros: a zeroed
    // device block plus one scatter, instead of a host transpose of n x cols
    // and a pageable copy of it (4.4 MB at n = 21,774, cols = 25).  Column
    // scans are sequential reads; bail out to the dense path past n*cols/16.
    {
        const size_t cap = (size_t)n * cols / 16;
        std::vector<int64_t> off;
        std::vector<double> val;
        bool sparse = true;
        for (int c = 0; c < cols && sparse; ++c) {
            const double* col = H + (size_t)c * n;
            for (int64_t i = 0; i < n; ++i)
                if (col[i] != 0.0) {
                    if (off.size() >= cap) {
                        sparse = false;
                        break;
                    }
                    off.push_back(i * (int64_t)ldd + c);
                    val.push_back(col[i]);
                }
        }
        if (sparse) {
            hipStream_t st = A->ctx->stream;
            KT_HIP(hipMemset2DAsync(D, sizeof(double) * ldd, 0, sizeof(double) * cols, (size_t)n, st));
            const size_t m = off.size();
            if (m) {
                DevBuf& d = A->ctx->ws.qrtmp;
                const size_t ob = (sizeof(int64_t) * m + 255) / 256 * 256;
                d.ensure(ob + sizeof(double) * m);
                PinnedBuf& hp = A->ctx->ws.pin_comb;
                if (A->ctx->ws.comb_pending) {  // combine()'s last upload out of pin_comb
                    KT_HIP(hipEventSynchronize(A->ctx->ws.comb_ev));
                    A->ctx->ws.comb_pending = false;
                }
                hp.ensure(ob + sizeof(double) * m);
                char* h = hp.as<char>();
                std::memcpy(h, off.data(), sizeof(int64_t) * m);
                std::memcpy(h + ob, val.data(), sizeof(double) * m);
                KT_HIP(hipMemcpyAsync(d.ptr, h, ob + sizeof(double) * m, hipMemcpyHostToDevice, st));
                KT_HIP(launch_scatter_elems((int64_t)m, d.as<int64_t>(),
                                            reinterpret_cast<double*>(static_cast<char*>(d.ptr) + ob), D, st));
                // pin_comb is reused by the next upload: wait for this copy
                KT_HIP(hipStreamSynchronize(st));
            }
            return;
        }
    }
    std::vector<double> tmp((size_t)n * cols, 0.0);  // compact row-major, device numbering
    for (int c = 0; c < cols; ++c)
        for (int64_t i = 0; i < n; ++i) tmp[(size_t)i * cols + c] = H[(size_t)c * n + i];
    KT_HIP(hipMemcpy2DAsync(D, sizeof(double) * ldd, tmp.data(), sizeof(double) * cols,
                            sizeof(double) * cols, (size_t)n, hipMemcpyHostToDevice, A->ctx->stream));
    KT_HIP(hipStreamSynchronize(A->ctx->stream));
}

void download_elems(kt_context_s* ctx, const double* D, const std::vector<int64_t>& off,
                    std::vector<double>& out) {
    const size_t m = off.size();
    out.assign(m, 0.0);
    if (m == 0) return;
    DevBuf& d = ctx->ws.qrtmp;
    const size_t idx_bytes = (sizeof(int64_t) * m + 255) / 256 * 256;
    d.ensure(idx_bytes + sizeof(double) * m);
    int64_t* doff = d.as<int64_t>();
    double* dout = reinterpret_cast<double*>(static_cast<char*>(d.ptr) + idx_bytes);
    KT_HIP(hipMemcpyAsync(doff, off.data(), sizeof(int64_t) * m, hipMemcpyHostToDevice, ctx->stream));
    KT_HIP(launch_gather_elems((int64_t)m, D, doff, dout, ctx->stream));
    KT_HIP(hipMemcpyAsync(out.data(), dout, sizeof(double) * m, hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
}

void download_rows(kt_matrix_s* A, const double* D, int ldd, int cols,
                   const std::vector<int64_t>& rows, std::vector<double>& out) {
    const int nr = (int)rows.size();
    out.assign((size_t)nr * cols, 0.0);
    if (nr == 0 || cols == 0) return;
    // one gather kernel + one copy (a copy and a sync per row cost ~40 us each)
    kt_context_s* ctx = A->ctx;
    DevBuf& d = ctx->ws.qrtmp;
    const size_t idx_bytes = (sizeof(int64_t) * nr + 255) / 256 * 256;
    d.ensure(idx_bytes + sizeof(double) * (size_t)nr * cols);
    int64_t* drows = d.as<int64_t>();
    double* dout = reinterpret_cast<double*>(static_cast<char*>(d.ptr) + idx_bytes);
    KT_HIP(hipMemcpyAsync(drows, rows.data(), sizeof(int64_t) * nr, hipMemcpyHostToDevice, ctx->stream));
    KT_HIP(launch_gather_rows(nr, cols, D, ldd, drows, dout, ctx->stream));
    KT_HIP(hipMemcpyAsync(out.data(), dout, sizeof(double) * out.size(), hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
}

void download_block(kt_matrix_s* A, const double* D, int ldd, int cols, double* out) {
    const int64_t n = A->n;
    if (n == 0 || cols == 0) return;
    std::vector<double> tmp((size_t)n * cols);
    KT_HIP(hipMemcpy2DAsync(tmp.data(), sizeof(double) * cols, D, sizeof(double) * ldd,
                            sizeof(double) * cols, (size_t)n, hipMemcpyDeviceToHost, A->ctx->stream));
    KT_HIP(hipStreamSynchronize(A->ctx->stream));
    for (int c = 0; c < cols; ++c)
        for (int64_t i = 0; i < n; ++i) out[i + (size_t)c * n] = tmp[(size_t)i * cols + c];
}

void matmul(int m, int k, int n, const double* A, const double* B, double* C) {
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            for (int l = 0; l < k; ++l) s += A[i + (size_t)l * m] * B[l + (size_t)j * k];
            C[i + (size_t)j * m] = s;
        }
}

double norm_fro(const std::vector<double>& M) {
    double s = 0.0;
    for (double v : M) s += v * v;
    return std::sqrt(s);
}

double norm2_small(int m, int n, const double* M) {
    // sqrt(lambda_max(M'M))
    std::vector<double> G((size_t)n * n), w(n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) {
            double s = 0.0;
            for (int l = 0; l < m; ++l) s += M[l + (size_t)i * m] * M[l + (size_t)j * m];
            G[i + (size_t)j * n] = s;
        }
    sym_eig_host(n, G.data(), w.data(), nullptr);
    return n ? std::sqrt(std::max(0.0, w[n - 1])) : 0.0;
}

// One CholQR pass with optional diagonal shift: W <- W R^{-1}.
static bool cholqr_pass(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, double shift,
                        std::vector<double>& R) {
    std::vector<double> G;
    gram(ctx, n, W, ld, bs, W, ld, bs, G);
    for (int i = 0; i < bs; ++i) G[i + (size_t)i * bs] += shift;
    if (!chol_upper(G.data(), bs)) return false;
    R = G;
    std::vector<double> Ri((size_t)bs * bs);
    tri_upper_inv(R.data(), bs, Ri.data());
    // W <- W Ri via a scratch block (rocBLAS output must not alias its input)
    DevBuf& t = ctx->ws.qrtmp;
    t.ensure(sizeof(double) * (size_t)std::max<int64_t>(n, 1) * bs);
    combine(ctx, n, W, ld, bs, Ri, bs, 0.0, t.as<double>(), bs);
    copy_cols(ctx, n, t.as<double>(), bs, W, ld, bs);
    return true;
}

bool cholqr(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R) {
    std::vector<double> G;
    gram(ctx, n, W, ld, bs, W, ld, bs, G);
    double tr = 0.0;
    for (int i = 0; i < bs; ++i) tr += G[i + (size_t)i * bs];
    R.assign((size_t)bs * bs, 0.0);
    if (!(tr > 0.0) || std::sqrt(tr) < 1e-14) return false;  // numerically zero block
    std::vector<double> R1, R2, R3, T((size_t)bs * bs);
    if (!cholqr_pass(ctx, n, W, ld, bs, 0.0, R1)) {
        // shifted CholQR3 (Fukaya et al.): shift ~ 11 (n bs + bs(bs+1)) eps ||W||^2
        const double s = 11.0 * ((double)n * bs + (double)bs * (bs + 1)) * DBL_EPSILON * tr;
        if (!cholqr_pass(ctx, n, W, ld, bs, s, R1)) return false;
        if (!cholqr_pass(ctx, n, W, ld, bs, 0.0, R2)) return false;
        matmul(bs, bs, bs, R2.data(), R1.data(), T.data());
        R1 = T;
    }
    if (!cholqr_pass(ctx, n, W, ld, bs, 0.0, R3)) return false;
    matmul(bs, bs, bs, R3.data(), R1.data(), R.data());
    return true;
}

}  // namespace kt

namespace kt {

// The thin QR of a block-Krylov step (lanczos_krylov.m:48,90,
// arnoldi_krylov.m:50,99).  When the block is well conditioned the thin QR is
// unique up to the signs of Q's columns, and every quantity the Krylov
// drivers return is invariant under those signs (H, Gm, tGm, Cm change by a
// diagonal +-1 similarity: same eigenvalues, same Um Xm Um', same traces), so
// CholeskyQR2 -- two Gram / Cholesky / W R^-1 passes, 6 launches and 2 host
// round trips -- stands in for the 2 bs + 3 launches of the Householder
// sweep; its Q agrees with Householder's to ~kappa eps.  A block whose first
// Cholesky fails or whose factor's diagonal spans more than 1e4 (kappa >~
// 1e4), or whose scale is at a breakdown, takes householder_qr on the
// untouched W: rank-deficient blocks keep LAPACK's reflectors and tau = 0
// completions, which decide the reference's continuation.

static void apply_rinv(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, const std::vector<double>& R) {
    std::vector<double> Ri((size_t)bs * bs);
    tri_upper_inv(R.data(), bs, Ri.data());
    if (bs <= 32 && !rocblas_gemm_path(n)) {
        // in place: k_combine_ts has ONE workgroup per 64 rows when q <= 32,
        // and it reads all of its rows' X before it writes any Y
        combine(ctx, n, W, ld, bs, Ri, bs, 0.0, W, ld);
        return;
    }
    DevBuf& t = ctx->ws.qrtmp;  // output must not alias the input
    t.ensure(sizeof(double) * (size_t)std::max<int64_t>(n, 1) * bs);
    combine(ctx, n, W, ld, bs, Ri, bs, 0.0, t.as<double>(), bs);
    copy_cols(ctx, n, t.as<double>(), bs, W, ld, bs);
}

// Shifted CholeskyQR3 on W (Fukaya, Kannan, Nakatsukasa, Yamamoto, Yanagisawa
// 2020): one pass with the Gram shifted by 11 (n bs + bs (bs + 1)) eps ||W||_F^2,
// then two plain CholeskyQR passes, all on the device (Gram -> one-workgroup
// Cholesky + inverse -> W R^-1, no host round trip between the passes); the
// three factors and their status come back together.  W is kept aside first;
// false (W restored) when a Cholesky failed or the last pass's factor is not
// the identity to 1e-8 (Q not orthonormal): the caller then takes the
// Householder sweep.
static bool shifted_cholqr3(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R) {
    if (bs > 64) return false;
    const size_t bb = (size_t)bs * bs;
    DevBuf& keep = ctx->ws.qrkeep;
    keep.ensure(sizeof(double) * (size_t)std::max<int64_t>(n, 1) * bs);
    copy_cols(ctx, n, W, ld, keep.as<double>(), bs, bs);
    DevBuf& f = ctx->ws.qrfac;  // R1 R2 R3 | Rinv | ok[3]
    f.ensure(sizeof(double) * 4 * bb + 4 * sizeof(int));
    double* dR = f.as<double>();
    double* dRi = dR + 3 * bb;
    int* dok = reinterpret_cast<int*>(dRi + bb);
    const bool inplace = bs <= 32 && !rocblas_gemm_path(n);  // k_combine_ts reads its rows before writing
    DevBuf& t = ctx->ws.qrtmp;
    if (!inplace) t.ensure(sizeof(double) * (size_t)std::max<int64_t>(n, 1) * bs);
    const double c0 = 11.0 * ((double)n * bs + (double)bs * (bs + 1)) * DBL_EPSILON;
    PinnedBuf& hp = ctx->ws.pin_qrfac;
    hp.ensure(sizeof(double) * 3 * bb + 4 * sizeof(int));
    double* hR = hp.as<double>();
    int* hok = reinterpret_cast<int*>(hR + 3 * bb);
    Workspace& ws = ctx->ws;
    if (!ws.qrfac_ev) KT_HIP(hipEventCreateWithFlags(&ws.qrfac_ev, hipEventDisableTiming));
    for (int p = 0; p < 3; ++p) {
        const double* dG = gram_device(ctx, n, W, ld, bs, W, ld, bs);
        KT_HIP(launch_chol_rinv(bs, dG, p == 0 ? c0 : 0.0, dR + p * bb, dRi, dok + p, ctx->stream));
        if (p == 2) {  // the factors come back while the last W R^-1 runs (the host waits for them only)
            KT_HIP(hipMemcpyAsync(hR, dR, sizeof(double) * 3 * bb, hipMemcpyDeviceToHost, ctx->stream));
            KT_HIP(hipMemcpyAsync(hok, dok, 3 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
            KT_HIP(hipEventRecord(ws.qrfac_ev, ctx->stream));
        }
        if (inplace) {
            combine_device(ctx, n, W, ld, bs, dRi, bs, 1.0, 0.0, W, ld);
        } else {
            combine_device(ctx, n, W, ld, bs, dRi, bs, 1.0, 0.0, t.as<double>(), bs);
            copy_cols(ctx, n, t.as<double>(), bs, W, ld, bs);
        }
    }
    KT_HIP(hipEventSynchronize(ws.qrfac_ev));
    const double* R1 = hR;
    const double* R2 = hR + bb;
    const double* R3 = hR + 2 * bb;
    double dev = 0.0;
    for (int j = 0; j < bs; ++j)
        for (int i = 0; i <= j; ++i) dev = std::max(dev, std::fabs(R3[i + (size_t)j * bs] - (i == j ? 1.0 : 0.0)));
    if (!(hok[0] && hok[1] && hok[2]) || !(dev < 1e-8)) {
        copy_cols(ctx, n, keep.as<double>(), bs, W, ld, bs);
        return false;
    }
    std::vector<double> T(bb);
    matmul(bs, bs, bs, R2, R1, T.data());
    R.assign(bb, 0.0);
    matmul(bs, bs, bs, R3, T.data(), R.data());
    for (int j = 0; j < bs; ++j)
        for (int i = j + 1; i < bs; ++i) R[i + (size_t)j * bs] = 0.0;
    return true;
}

void block_qr(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R, bool allow_shifted) {
    if (n < 4 * (int64_t)bs || bs < 1) {
        householder_qr(ctx, n, W, ld, bs, R);
        return;
    }
    std::vector<double> R1;
    gram(ctx, n, W, ld, bs, W, ld, bs, R1);
    bool ok = chol_upper(R1.data(), bs);
    double dmax = 0.0, dmin = HUGE_VAL;
    for (int k = 0; ok && k < bs; ++k) {
        dmax = std::max(dmax, R1[k + (size_t)k * bs]);
        dmin = std::min(dmin, R1[k + (size_t)k * bs]);
    }
    static const bool qr_log = std::getenv("KT_QR_LOG") != nullptr;  // diagnostics: the QR path per block
    if (qr_log)
        std::fprintf(stderr, "kt_qr n=%lld bs=%d chol=%d dmin=%.3e dmax=%.3e allow_shifted=%d\n", (long long)n, bs,
                     (int)ok, ok ? dmin : -1.0, ok ? dmax : -1.0, (int)allow_shifted);
    if (!ok || !(dmin >= 1e-4 * dmax) || !(dmax > 1e-6)) {
        // block Arnoldi (allow_shifted): an
        // ill-conditioned block that is not at a breakdown takes shifted
        // CholeskyQR3 (Fukaya et al.: Q orthonormal to O(eps) up to kappa ~
        // 1/eps) -- 3 Gram / combine passes instead of 2 bs + 3 Householder
        // launches; its completion of numerically dependent columns is as
        // rounding-dependent as the Householder one, not the
        // same, and fun_update's full-basis reorthogonalisation leaves the
        // gradient on it unchanged to 1e-10 (test_gpu_configs, omega sweep).
        // Exactly dependent columns fail its second Cholesky and keep
        // Householder's tau = 0 completion.  Block Lanczos (trace_fun_update's
        // 2-block window, where the completion direction enters the objective)
        // never takes it.
        // A block whose first plain Cholesky fails is left to Householder: on
        // Hawaii those blocks are exactly dependent, and both the shifted form
        // and a two-shift variant fail there and fall back, at +0.7-1 ms per
        // call (profiles/r03_qr_paths.txt).
        if (allow_shifted && dmax > 1e-6 && shifted_cholqr3(ctx, n, W, ld, bs, R)) return;
        householder_qr(ctx, n, W, ld, bs, R);
        return;
    }
    apply_rinv(ctx, n, W, ld, bs, R1);
    std::vector<double> R2;
    gram(ctx, n, W, ld, bs, W, ld, bs, R2);
    R.assign((size_t)bs * bs, 0.0);
    if (!chol_upper(R2.data(), bs)) {  // not expected after a kappa <= 1e4 first pass
        householder_qr(ctx, n, W, ld, bs, R2);
    } else {
        apply_rinv(ctx, n, W, ld, bs, R2);
    }
    matmul(bs, bs, bs, R2.data(), R1.data(), R.data());
    for (int j = 0; j < bs; ++j)  // R2 R1 is upper triangular; clear rounding below
        for (int i = j + 1; i < bs; ++i) R[i + (size_t)j * bs] = 0.0;
}

// Householder thin QR (the factorisation MATLAB's qr(w, 0) uses: LAPACK
// reflectors, R with dlarfg's signs, Q = H_1 ... H_bs E), on the tall-skinny
// kernels of kt_tsqr.hip.  Exactly rank-deficient W takes dlarfg's tau = 0
// branch, so its completion matches LAPACK's.
void householder_qr(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R) {
    static const bool qr_log = std::getenv("KT_QR_LOG") != nullptr;
    if (qr_log) std::fprintf(stderr, "kt_hh n=%lld bs=%d\n", (long long)n, bs);
    R.assign((size_t)bs * bs, 0.0);
    if (n == 0 || bs == 0) return;
    if (n < bs) fail(KT_ERR_UNSUPPORTED, "thin QR needs n >= block size");
    if (bs > 128) fail(KT_ERR_UNSUPPORTED, "thin QR block size > 128");
    const int BP = pow2_at_least(bs);
    Workspace& ws = ctx->ws;
    const int nrb = ts_nrb((int)n, ctx->num_cu);
    ws.ts_V.ensure(sizeof(double) * (size_t)n * BP);
    ws.ts_part.ensure(sizeof(double) * (size_t)BP * nrb);
    ws.ts_small.ensure(sizeof(double) * ((size_t)3 * BP + (size_t)bs * bs));
    double* V = ws.ts_V.as<double>();
    double* pivot = ws.ts_small.as<double>();
    double* sums = pivot + BP;
    double* taus = sums + BP;
    double* Md = taus + BP;
    KT_HIP(hipMemsetAsync(V, 0, sizeof(double) * (size_t)n * BP, ctx->stream));
    // the reflector sweep: two launches per column (the persistent forms with
    // one or two grid barriers per column measured slower, config 3
    // fun_and_grad 17.9 vs 17.0 ms, profiles/r02_tsqr_persistent.txt, and
    // were dropped in round 5).
    // KT_TSQR_STEP1=1: one launch per column (k_ts_step1) where its grid fits
    // (n <= 49,152) -- measured equal to the two-launch form (config 3: 13.05
    // us per column launch vs 8.43 + 5.01 us, fun_and_grad 9.6-10.0 vs
    // 9.5-10.1 ms, profiles/r03_tsqr_step1.txt): the column's dependent chain
    // (partials -> coefficients -> loads -> update -> partials) costs the same
    // inside one launch, so it stays opt-in
    const char* s1e = std::getenv("KT_TSQR_STEP1");
    int rpw1 = 0;
    const int g1 = (s1e && s1e[0] == '1') ? ts_step1_grid((int)n, &rpw1) : 0;
    if (g1 > 0) {
        ws.ts_part.ensure(sizeof(double) * ((size_t)2 * BP * g1 + 2 * (size_t)BP));
        double* part1 = ws.ts_part.as<double>();
        KT_HIP(launch_ts_reflectors1((int)n, bs, BP, W, ld, V, part1, part1 + (size_t)2 * BP * g1, taus,
                                     ctx->stream));
    } else {
        KT_HIP(launch_ts_reflectors((int)n, bs, BP, W, ld, V, pivot, sums, ws.ts_part.as<double>(), taus,
                                    ctx->num_cu, ctx->stream));
    }
    // R's rows, V's top block and the taus come back through pinned staging
    // (asynchronous); gram's synchronisation covers them
    ws.pin_qr.ensure(sizeof(double) * ((size_t)bs * bs + (size_t)bs * BP + bs));
    double* ptop = ws.pin_qr.as<double>();
    double* pV1 = ptop + (size_t)bs * bs;
    double* ptau = pV1 + (size_t)bs * BP;
    KT_HIP(hipMemcpy2DAsync(ptop, sizeof(double) * bs, W, sizeof(double) * ld, sizeof(double) * bs, (size_t)bs,
                            hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipMemcpyAsync(pV1, V, sizeof(double) * (size_t)bs * BP, hipMemcpyDeviceToHost, ctx->stream));
    KT_HIP(hipMemcpyAsync(ptau, taus, sizeof(double) * bs, hipMemcpyDeviceToHost, ctx->stream));
    std::vector<double> G;  // V' V (bs x bs), gram synchronises the stream
    gram(ctx, n, V, BP, bs, V, BP, bs, G);
    const std::vector<double> top(ptop, ptop + (size_t)bs * bs), V1(pV1, pV1 + (size_t)bs * BP),
        tau(ptau, ptau + bs);
    for (int i = 0; i < bs; ++i)
        for (int j = i; j < bs; ++j) R[i + (size_t)j * bs] = top[(size_t)i * bs + j];
    // dlarft (forward, columnwise): T upper bs x bs, column-major
    std::vector<double> T((size_t)bs * bs, 0.0), tmp(bs);
    for (int i = 0; i < bs; ++i) {
        if (tau[i] != 0.0) {
            for (int l = 0; l < i; ++l) tmp[l] = -tau[i] * G[l + (size_t)i * bs];
            for (int l = 0; l < i; ++l) {
                double s = 0.0;
                for (int q = l; q < i; ++q) s += T[l + (size_t)q * bs] * tmp[q];
                T[l + (size_t)i * bs] = s;
            }
        }
        T[i + (size_t)i * bs] = tau[i];
    }
    // M = T V1'  (row-major for the kernel: M[k * bs + j])
    std::vector<double> M((size_t)bs * bs, 0.0);
    for (int k = 0; k < bs; ++k)
        for (int j = 0; j < bs; ++j) {
            double s = 0.0;
            for (int l = k; l < bs; ++l) s += T[k + (size_t)l * bs] * V1[(size_t)j * BP + l];
            M[(size_t)k * bs + j] = s;
        }
    // M goes up through pinned staging guarded by an event (rewritten only
    // once the previous upload out of it completed), so the formation of Q
    // runs on without a stream sync here
    if (ws.qrm_pending) KT_HIP(hipEventSynchronize(ws.qrm_ev));
    ws.qrm_pending = false;
    if (!ws.qrm_ev) KT_HIP(hipEventCreateWithFlags(&ws.qrm_ev, hipEventDisableTiming));
    ws.pin_qrm.ensure(sizeof(double) * M.size());
    std::memcpy(ws.pin_qrm.ptr, M.data(), sizeof(double) * M.size());
    KT_HIP(hipMemcpyAsync(Md, ws.pin_qrm.ptr, sizeof(double) * M.size(), hipMemcpyHostToDevice, ctx->stream));
    KT_HIP(hipEventRecord(ws.qrm_ev, ctx->stream));
    ws.qrm_pending = true;
    KT_HIP(launch_ts_formq((int)n, bs, BP, V, Md, W, ld, ctx->stream));
}

}  // namespace kt
