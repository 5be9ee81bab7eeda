// kt_block.h -- device tall-skinny block operations for the block-Krylov paths
// (lanczos_krylov.m / arnoldi_krylov.m with bs > 1, mc_trace.m's QR and
// deflation).  Blocks are ROW-MAJOR n x ld device arrays in the matrix's
// device row numbering (kt_runtime.cpp relabels rows by degree); a block of
// bs columns occupies PB = pow2 >= bs columns, the padding kept at zero so
// the SpMM kernel (which works on PB columns) multiplies zeros.
#pragma once
#include <rocblas/rocblas.h>

#include <vector>

#include "kt_internal.h"

namespace kt {

int pow2_at_least(int b);

rocblas_handle blas(kt_context_s* ctx);

// Row-major device array n x ld (zero-initialised).
// n x ld row-major device block, zeroed by alloc; the storage comes from and
// returns to the context's ScratchPool (no hipMalloc / hipFree per call).
struct DevMat {
    kt_context_s* ctx = nullptr;
    void* ptr = nullptr;
    size_t bytes = 0;
    int64_t n = 0;
    int ld = 0;
    DevMat() = default;
    DevMat(const DevMat&) = delete;
    DevMat& operator=(const DevMat&) = delete;
    DevMat(DevMat&& o) noexcept { steal(o); }
    DevMat& operator=(DevMat&& o) noexcept {
        if (this != &o) {
            release();
            steal(o);
        }
        return *this;
    }
    ~DevMat() { release(); }
    void alloc(kt_context_s* ctx, int64_t n_, int ld_, bool zero = true);
    void release();
    double* col(int c) { return static_cast<double*>(ptr) + c; }
    const double* col(int c) const { return static_cast<const double*>(ptr) + c; }

  private:
    void steal(DevMat& o) {
        ctx = o.ctx;
        ptr = o.ptr;
        bytes = o.bytes;
        n = o.n;
        ld = o.ld;
        o.ctx = nullptr;
        o.ptr = nullptr;
        o.bytes = 0;
    }
};

// G (host, px x py column-major) = X[:, 0:px]' Y[:, 0:py]   (synchronises)
void gram(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px, const double* Y,
          int ldy, int py, std::vector<double>& G);
// The same Gram matrix left on the device (ctx->ws.small, px x py column-major;
// valid until the next gram on this context): no host round trip
const double* gram_device(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px, const double* Y,
                          int ldy, int py);
// Y[:, 0:q] = beta * Y[:, 0:q] + alpha * X[:, 0:px] * C   (C device px x q column-major)
void combine_device(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px, const double* dC, int q,
                    double alpha, double beta, double* Y, int ldy);
// Y[:, 0:q] = beta * Y[:, 0:q] + X[:, 0:px] * C   (C host px x q column-major)
void combine(kt_context_s* ctx, int64_t n, const double* X, int ldx, int px,
             const std::vector<double>& C, int q, double beta, double* Y, int ldy);
// Y[:, 0:P] = A X[:, 0:P], P = pow2 >= cols (columns cols..P-1 of X must be 0)
void spmm(kt_matrix_s* A, const double* X, int ldx, double* Y, int ldy, int cols);
// cols > 128 in one launch (128-wide column slices); skip: device flag, the
// launch is a no-op when *skip == 0 (nullptr: always run)
void spmm_slices(kt_matrix_s* A, const double* X, int ldx, double* Y, int ldy, int cols,
                 const int* skip = nullptr);
// copy a column slice (n x cols) between device arrays
void copy_cols(kt_context_s* ctx, int64_t n, const double* X, int ldx, double* Y, int ldy, int cols);
void zero_cols(kt_context_s* ctx, int64_t n, double* X, int ldx, int cols);
// host column-major -> device row-major
void upload_rows(kt_matrix_s* A, const double* H, int cols, double* D, int ldd);
// device rows (row indices) -> host nrows x cols column-major
// host out[i] = device D[off[i]] (one upload, one gather launch, one download)
void download_elems(kt_context_s* ctx, const double* D, const std::vector<int64_t>& off,
                    std::vector<double>& out);
void download_rows(kt_matrix_s* A, const double* D, int ldd, int cols,
                   const std::vector<int64_t>& rows, std::vector<double>& out);
// whole device block (n x cols at ldd) -> host column-major n x cols
void download_block(kt_matrix_s* A, const double* D, int ldd, int cols, double* out);
// thin QR of W (n x bs at ld) in place: W <- Q, R upper bs x bs (column-major).
// CholQR2 (shifted CholQR3 if W is ill-conditioned).  Returns false when W
// is numerically zero (R = 0 then, Q unspecified): a lucky breakdown.
bool cholqr(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R);
// Householder thin QR of W in place (rocSOLVER LQ of W'); R upper, signs as LAPACK.
void householder_qr(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R);
// block-Krylov thin QR: CholeskyQR2 where well conditioned, else householder_qr
// allow_shifted: an ill-conditioned block may take shifted CholeskyQR3 instead
// of the Householder sweep (block Arnoldi, kt_block.cpp)
void block_qr(kt_context_s* ctx, int64_t n, double* W, int ld, int bs, std::vector<double>& R,
              bool allow_shifted = false);

// small host helpers (column-major)
void matmul(int m, int k, int n, const double* A, const double* B, double* C);  // C = A B
double norm_fro(const std::vector<double>& M);
double norm2_small(int m, int n, const double* M);  // spectral norm

}  // namespace kt
