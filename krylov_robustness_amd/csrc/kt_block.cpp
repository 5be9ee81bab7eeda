// kt_block.cpp -- tall-skinny device block operations (rocBLAS dgemm for the
// plain GEMM shapes, the HIP SpMM kernel for A*X) and CholQR.
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

void DevMat::alloc(kt_context_s* ctx, int64_t n_, int ld_) {
    n = n_;
    ld = ld_;
    buf.ensure(sizeof(double) * (size_t)std::max<int64_t>(n, 1) * ld);
    KT_HIP(hipMemsetAsync(buf.ptr, 0, sizeof(double) * (size_t)std::max<int64_t>(n, 1) * ld,
                          ctx->stream));
}

void gram(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px, const double* Y,
          int ldy, int py, std::vector<double>& G) {
    G.assign((size_t)px * py, 0.0);
    if (px == 0 || py == 0) return;
    DevBuf& d = ctx->ws.small;
    d.ensure(sizeof(double) * (size_t)px * py);
    const double one = 1.0, zero = 0.0;
    // column-major views: X is (ldx x n), Y is (ldy x n);  G = X(0:px,:) Y(0:py,:)'
    rb(rocblas_dgemm(blas(ctx), rocblas_operation_none, rocblas_operation_transpose, px, py,
                     (rocblas_int)n, &one, X, ldx, Y, ldy, &zero, d.as<double>(), px),
       "rocblas_dgemm(gram)");
    KT_HIP(hipMemcpyAsync(G.data(), d.ptr, sizeof(double) * G.size(), hipMemcpyDeviceToHost,
                          ctx->stream));
    KT_HIP(hipStreamSynchronize(ctx->stream));
}

void combine(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px,
             const std::vector<double>& C, int q, double beta, double* Y, int ldy) {
    if (q == 0) return;
    if (px == 0) {
        if (beta != 1.0) fail(KT_ERR_ARG, "combine: empty X with beta != 1");
        return;
    }
    DevBuf& d = ctx->ws.small2;
    d.ensure(sizeof(double) * (size_t)px * q);
    KT_HIP(hipMemcpyAsync(d.ptr, C.data(), sizeof(double) * (size_t)px * q, hipMemcpyHostToDevice,
                          ctx->stream));
    const double one = 1.0;
    // Yc (q x n) = beta Yc + C' (q x px) * Xc (px x n)
    rb(rocblas_dgemm(blas(ctx), rocblas_operation_transpose, rocblas_operation_none, q,
                     (rocblas_int)n, px, &one, d.as<double>(), px, X, ldx, &beta, Y, ldy),
       "rocblas_dgemm(combine)");
    // the host vector C may be freed by the caller right after: finish the copy
    KT_HIP(hipStreamSynchronize(ctx->stream));
}

void spmm(kt_matrix_s* A, const double* X, int ldx, double* Y, int ldy, int cols) {
    kt_context_s* ctx = A->ctx;
    const int P = pow2_at_least(std::max(cols, 1));
    if (P > 128) fail(KT_ERR_UNSUPPORTED, "block width > 128");
    const int n = (int)A->n;
    const int grid = spmm_grid(n, P, ctx->num_cu * 4);
    const DevCSR& M = natural_csr(A);  // block paths run in the reference's row order
    const int lblocks = long_blocks_for(M.n_long, ctx->num_cu * 2);
    KT_HIP(launch_spmm_block(P, A->unit_values ? 2 : 0, grid + lblocks, M.rowptr, M.col, M.val, n,
                             X, ldx, Y, ldy, M.long_rows, M.n_long, A->long_thresh, lblocks,
                             ctx->stream));
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
    std::vector<double> tmp((size_t)n * cols, 0.0);  // compact row-major, device numbering
    for (int c = 0; c < cols; ++c)
        for (int64_t i = 0; i < n; ++i) tmp[(size_t)i * cols + c] = H[(size_t)c * n + i];
    KT_HIP(hipMemcpy2DAsync(D, sizeof(double) * ldd, tmp.data(), sizeof(double) * cols,
                            sizeof(double) * cols, (size_t)n, hipMemcpyHostToDevice, A->ctx->stream));
    KT_HIP(hipStreamSynchronize(A->ctx->stream));
}

void download_rows(kt_matrix_s* A, const double* D, int ldd, int cols,
                   const std::vector<int64_t>& rows, std::vector<double>& out) {
    const int nr = (int)rows.size();
    out.assign((size_t)nr * cols, 0.0);
    std::vector<double> row(cols);
    for (int r = 0; r < nr; ++r) {
        const int64_t dr = rows[r];
        KT_HIP(hipMemcpyAsync(row.data(), D + (size_t)dr * ldd, sizeof(double) * cols,
                              hipMemcpyDeviceToHost, A->ctx->stream));
        KT_HIP(hipStreamSynchronize(A->ctx->stream));
        for (int c = 0; c < cols; ++c) out[(size_t)c * nr + r] = row[c];
    }
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

// Householder thin QR (the factorisation MATLAB's qr(w, 0) uses).  The
// row-major n x ld block W is the column-major (ld x n) matrix M = W', so an
// LQ factorisation of M's first bs rows (rocsolver_dgelqf) is a Householder QR
// of W: M(0:bs,:) = L Q'  =>  W = Q' ' L'.  R = L' (upper); rocsolver_dorglq
// then overwrites M(0:bs,:) with Q', i.e. W with Q.  Rank-deficient W is
// handled like LAPACK: R gets ~0 diagonal entries and Q stays orthonormal.
void householder_qr(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R) {
    R.assign((size_t)bs * bs, 0.0);
    if (n == 0 || bs == 0) return;
    if (n < bs) fail(KT_ERR_UNSUPPORTED, "thin QR needs n >= block size");
    DevBuf& tau = ctx->ws.small2;
    tau.ensure(sizeof(double) * (size_t)bs);
    rb(rocsolver_dgelqf(blas(ctx), bs, (rocblas_int)n, W, ld, tau.as<double>()), "rocsolver_dgelqf");
    std::vector<double> top((size_t)bs * bs);  // rows 0..bs-1 of W, first bs columns
    KT_HIP(hipMemcpy2DAsync(top.data(), sizeof(double) * bs, W, sizeof(double) * ld,
                            sizeof(double) * bs, (size_t)bs, hipMemcpyDeviceToHost, ctx->stream));
    rb(rocsolver_dorglq(blas(ctx), bs, (rocblas_int)n, bs, W, ld, tau.as<double>()), "rocsolver_dorglq");
    KT_HIP(hipStreamSynchronize(ctx->stream));
    // M(i, j) = top[j * bs + i]; L(i, j) = M(i, j), j <= i;  R(j, i) = L(i, j)
    for (int i = 0; i < bs; ++i)
        for (int j = 0; j <= i; ++j) R[j + (size_t)i * bs] = top[(size_t)j * bs + i];
}

}  // namespace kt
