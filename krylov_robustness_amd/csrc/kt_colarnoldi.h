// kt_colarnoldi.h -- a batch of independent single-vector Arnoldi runs
// (arnoldi_krylov.m with bs = 1, poles = inf), one per start index e_t, all
// advanced by one SpMM per step.  Shared by function_multiple_entries.m
// (kt_fme.cpp) and multiple_frechet_eval.m / hessianfcn_*.m (kt_frechet.cpp).
#pragma once
#include <vector>

#include "kt_krylov.h"

namespace kt {

class ColArnoldi {
   public:
    // starts: distinct 0-based row indices (<= 128); it: max steps
    ColArnoldi(kt_matrix_s* A, const std::vector<int64_t>& starts, int it);
    // general start block: X host n x C column-major (C <= 128)
    ColArnoldi(kt_matrix_s* A, const double* X, int C, int it);
    int cols() const { return C_; }
    int steps() const { return j_; }
    // one Arnoldi step for every column (arnoldi_krylov.m:78-111)
    void step() {
        step_launch();
        step_finish();
    }
    // the same step split in two: step_launch() queues the step's kernels and
    // the asynchronous read-back of its H column (pinned); step_finish()
    // waits for it and fills H.  Host work on the finished steps' H may run
    // in between (function_multiple_entries: step j's projections while the
    // device runs step j + 1).
    void step_launch();
    void step_finish();
    // Gm = H(1:j, 1:j) of column c (column-major j x j), j = finished steps
    void gm(int c, std::vector<double>& G) const;
    // (V1' e_t)(1) of column c  (function_multiple_entries.m:94-95)
    double uaux(int c) const { return uaux_[c]; }
    // basis entries V_c(r, k) for the given rows, k < nk (nk <= steps() + 1):
    // out[(ri * nk + k) * cols() + c]
    void rows(const std::vector<int64_t>& rr, int nk, std::vector<double>& out) const;
    // H(i, j) of column c (0-based, i <= steps(), j < steps())
    double h(int c, int i, int j) const { return H_[c][i + (size_t)j * (it_ + 1)]; }
    // out (host n x C column-major) = sum_{k < nk} V_k y_k, y[k * C + c]
    void combine(const std::vector<double>& y, int nk, double* out);

   private:
    void init_buffers();
    void start_qr();
    kt_matrix_s* A_;
    kt_context_s* ctx_;
    int64_t n_;
    int C_, P_, it_, j_ = 0, done_ = 0, nrb_;
    int rpb_lo_ = 64;  // rows per k_col_dots workgroup, at least (kt_colbatch.hip)
    bool pending_ = false;
    int64_t vs_;
    DevBuf basis_, W_, part_, red_, idx_;
    std::vector<std::vector<double>> H_;  // (it+1) x it column-major per column
    std::vector<double> uaux_;
};

// symmetric eigendecomposition of (G + G')/2, j x j: w ascending, V columns
void sym_eig_small(int j, const std::vector<double>& G, std::vector<double>& w,
                   std::vector<double>& V);

}  // namespace kt
