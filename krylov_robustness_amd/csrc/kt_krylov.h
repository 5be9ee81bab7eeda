// kt_krylov.h -- block-Krylov entry points shared between translation units.
#pragma once
#include "kt_block.h"

namespace kt {

// fun code of kt_trace_fun_update_fn: the caller's elementwise handle
constexpr int kFunCallback = 100;
// trace_fun_update.m:43-47 / :85-89 with d1, d2 ascending
double trace_diff(const std::vector<double>& d1, const std::vector<double>& d2, int fun);
// fails with KT_ERR_NOT_HERMITIAN and `msg` unless A is symmetric (cached)
void require_symmetric(kt_matrix_s* A, const char* msg);
// trace_fun_update.m on the device (U host n x rk column-major)
double trace_fun_update_impl(kt_matrix_s* A, int rk, const double* U, const double* B, double tol,
                             int it, int fun, int* iter_out, int* lucky_out);

// Batched trace_fun_update over candidate edges (krylov_miobi.m:76-99): for
// each c, U_c = [e_{ei[c]}, e_{ej[c]}] (0-based rows; ei == ej -> U = e_i,
// B = B1) and B (2 x 2 column-major).  Outputs Xm[c], iter[c], lucky[c].
void trace_fun_update_pairs(kt_matrix_s* A, int64_t nC, const int64_t* ei, const int64_t* ej,
                            const double* B, double B1, double tol, int it, int fun, double* Xm,
                            int* iter, int* lucky);

// A's twin: a second device copy on its own context (stream, workspace),
// built on first use and kept current through edits; nullptr when KT_TWIN=0.
// Lets two independent Krylov runs of one call overlap on the GPU.
kt_matrix_s* twin_of(kt_matrix_s* A);

// set A(i,j) = A(j,i) = value for each pair (0 deletes the entry, as MATLAB
// sparse assignment does) on the host copy and refresh the device copies.
void set_pairs(kt_matrix_s* A, int64_t count, const int64_t* ei, const int64_t* ej, double value);

}  // namespace kt
