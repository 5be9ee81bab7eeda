// kt_mex.cpp -- MATLAB MEX shim: drop-in replacements for the reference's
// entry points.  One source, built once per entry point:
//
//   mex -R2018a -DKT_ENTRY_TRACE_EXP        kt_mex.cpp -L<lib> -lkrylov_hip -output trace_exp
//   mex -R2018a -DKT_ENTRY_MC_TRACE         kt_mex.cpp ... -output mc_trace
//   mex -R2018a -DKT_ENTRY_TRACE_FUN_UPDATE kt_mex.cpp ... -output trace_fun_update
//   mex -R2018a -DKT_ENTRY_FUN_UPDATE       kt_mex.cpp ... -output fun_update
//   mex -R2018a -DKT_ENTRY_FG_EXP           kt_mex.cpp ... -output fun_and_grad_krylov_exp
//   mex -R2018a -DKT_ENTRY_FG_FUN           kt_mex.cpp ... -output fun_and_grad_krylov_fun
//   mex -R2018a -DKT_ENTRY_KRYLOV_MIOBI     kt_mex.cpp ... -output krylov_miobi
//   mex -R2018a -DKT_ENTRY_FME              kt_mex.cpp ... -output function_multiple_entries
//   mex -R2018a -DKT_ENTRY_HESS_EXP         kt_mex.cpp ... -output hessianfcn_exp
//   mex -R2018a -DKT_ENTRY_HESS_FUN         kt_mex.cpp ... -output hessianfcn_fun
//
// Placed in the reference's functions/ directory, each MEX shadows the .m of
// the same name (MATLAB's same-folder precedence), so Tests/*.m, greedy_krylov.m
// and the fmincon closures run unchanged.  MATLAB is not installed in the
// build image, so this file is source-only; every call
// forwards to the C ABI in include/krylov_trace.h, which the ctypes tests
// exercise with the same arguments.
//
// Ownership: prhs are borrowed; plhs are created here.  The device context
// and the device copy of the last A live across calls (fmincon and the
// greedy loop pass the same A repeatedly); they are keyed by the sparse
// arrays' contents and released in mexAtExit.  Errors never cross the C ABI:
// a non-zero status becomes mexErrMsgIdAndTxt with the library's message.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <initializer_list>
#include <string>
#include <vector>

#include "mex.h"
#include "../../include/krylov_trace.h"

namespace {

kt_context_t g_ctx = nullptr;
kt_matrix_t g_A = nullptr;
std::vector<int64_t> g_jc, g_ir;  // cache key: pattern + values of the last A
std::vector<double> g_pr;

void release_all() {
    if (g_A) kt_matrix_destroy(g_A);
    if (g_ctx) kt_context_destroy(g_ctx);
    g_A = nullptr;
    g_ctx = nullptr;
}

void check(int st, const char* where) {
    if (st != KT_OK) {
        std::string id = std::string("krylov_hip:") + where;
        mexErrMsgIdAndTxt(id.c_str(), "%s", kt_last_error());
    }
}

kt_context_t context() {
    if (!g_ctx) {
        check(kt_context_create(0, &g_ctx), "context");
        mexAtExit(release_all);
        mexLock();
    }
    return g_ctx;
}

// A: MATLAB sparse (or full) real double, square (lanczos_krylov.m:36-38).
// `nonsquare` is the reference's message for a non-square A on this entry:
// the fun_and_grad_* files test ishermitian(A) first, which a non-square A
// fails (fun_and_grad_krylov_exp.m:21-23, fun_and_grad_krylov_fun.m:22-24).
kt_matrix_t matrix_arg(const mxArray* a, const char* nonsquare = "The matrix A should be square") {
    if (!mxIsDouble(a) || mxIsComplex(a)) mexErrMsgIdAndTxt("krylov_hip:A", "A must be real double");
    const mwSize n = mxGetM(a);
    if (mxGetN(a) != n) mexErrMsgIdAndTxt("krylov_hip:A", "%s", nonsquare);
    std::vector<int64_t> jc(n + 1), ir;
    std::vector<double> pr;
    if (mxIsSparse(a)) {
        const mwIndex* J = mxGetJc(a);
        const mwIndex* I = mxGetIr(a);
        const double* P = mxGetDoubles(a);
        for (mwSize j = 0; j <= n; ++j) jc[j] = (int64_t)J[j];
        ir.assign(I, I + jc[n]);
        pr.assign(P, P + jc[n]);
    } else {  // full matrix: compress
        const double* P = mxGetDoubles(a);
        jc[0] = 0;
        for (mwSize j = 0; j < n; ++j) {
            for (mwSize i = 0; i < n; ++i)
                if (P[i + j * n] != 0.0) {
                    ir.push_back((int64_t)i);
                    pr.push_back(P[i + j * n]);
                }
            jc[j + 1] = (int64_t)ir.size();
        }
    }
    if (g_A && jc == g_jc && ir == g_ir && pr == g_pr) return g_A;  // device-resident reuse
    if (g_A) kt_matrix_destroy(g_A);
    g_A = nullptr;
    check(kt_matrix_create_csc(context(), (int64_t)n, jc.data(), ir.data(), pr.data(), 0, &g_A),
          "matrix");
    g_jc.swap(jc);
    g_ir.swap(ir);
    g_pr.swap(pr);
    return g_A;
}

double scalar_or(int nrhs, const mxArray* prhs[], int k, double dflt) {
    return (nrhs > k && !mxIsEmpty(prhs[k])) ? mxGetScalar(prhs[k]) : dflt;
}

// function_handle -> kt_fun via func2str (fun_update.m:43-59 identities);
// -2 for any other handle when `generic` (callers that take a kt_scalar_fn).
int fun_arg(const mxArray* h, int dflt, bool generic = false) {
    if (!h || mxIsEmpty(h)) return dflt;
    mxArray* out = nullptr;
    mxArray* in = const_cast<mxArray*>(h);
    if (mexCallMATLAB(1, &out, 1, &in, "func2str") != 0) return -1;
    char buf[64] = {0};
    mxGetString(out, buf, sizeof(buf));
    mxDestroyArray(out);
    const char* s = buf[0] == '@' ? buf + 1 : buf;
    static const char* names[] = {"exp", "sinh", "cosh", "sin", "cos", "log", "sqrt"};
    for (int i = 0; i < 7; ++i)
        if (strcmp(s, names[i]) == 0) return i;
    if (generic) return -2;
    mexErrMsgIdAndTxt("krylov_hip:fun", "unsupported function handle %s (exp/sinh/cosh/sin/cos/log/sqrt)", buf);
    return -1;
}

mxArray* scalar(double v) { return mxCreateDoubleScalar(v); }

// kt_scalar_fn over a MATLAB handle: y = feval(h, x) on a count x 1 column.
// Runs inside the library call, so a failure is only recorded and returned
// as a non-zero status (the library then aborts with KT_ERR_CALLBACK); the
// MATLAB error is raised after the call returns, so none unwinds library frames.
bool g_feval_failed = false;
int feval_scalar_fn(const double* x, double* y, int64_t count, void* user) {
    mxArray* h = static_cast<mxArray*>(user);
    mxArray* in = mxCreateDoubleMatrix((mwSize)count, 1, mxREAL);
    memcpy(mxGetDoubles(in), x, sizeof(double) * (size_t)count);
    mxArray* args[2] = {h, in};
    mxArray* out = nullptr;
    const bool ok = mexCallMATLAB(1, &out, 2, args, "feval") == 0 && out && mxIsDouble(out) &&
                    !mxIsComplex(out) && mxGetNumberOfElements(out) == (size_t)count;
    if (ok) {
        memcpy(y, mxGetDoubles(out), sizeof(double) * (size_t)count);
    } else {
        g_feval_failed = true;
        for (int64_t i = 0; i < count; ++i) y[i] = mxGetNaN();
    }
    mxDestroyArray(in);
    if (out) mxDestroyArray(out);
    return ok ? 0 : 1;
}

// ---- mc_trace with a function-handle Afun --------------------------------
// One MATLAB call with owned results (inputs borrowed).
mxArray* call1(const char* fn, std::initializer_list<mxArray*> args) {
    std::vector<mxArray*> in(args);
    mxArray* out = nullptr;
    if (mexCallMATLAB(1, &out, (int)in.size(), in.data(), fn) != 0)
        mexErrMsgIdAndTxt("krylov_hip:mc_trace", "MATLAB call %s failed", fn);
    return out;
}

// The matrix A captured by a handle of the form @(x) expmv(1, A, x, ...)
// (trace_exp.m:5), or nullptr: func2str names the call, functions(h)
// .workspace{1}.A holds the captured matrix.
const mxArray* expmv_handle_matrix(const mxArray* h, mxArray** keep) {
    mxArray* in = const_cast<mxArray*>(h);
    mxArray* str = call1("func2str", {in});
    char buf[128] = {0};
    mxGetString(str, buf, sizeof(buf));
    mxDestroyArray(str);
    std::string f;
    for (const char* c = buf; *c; ++c)
        if (*c != ' ') f.push_back(*c);
    if (f.rfind("@(x)expmv(1,A,x", 0) != 0) return nullptr;
    mxArray* info = call1("functions", {in});
    mxArray* ws = mxGetField(info, 0, "workspace");
    const mxArray* A = nullptr;
    if (ws && mxIsCell(ws) && mxGetNumberOfElements(ws) > 0) {
        const mxArray* w0 = mxGetCell(ws, 0);
        if (w0 && mxIsStruct(w0)) A = mxGetField(w0, 0, "A");
    }
    if (!A || !mxIsDouble(A) || mxIsComplex(A)) {
        mxDestroyArray(info);
        return nullptr;
    }
    *keep = info;  // A lives inside info
    return A;
}

// Afun_k(x) = P_k(Afun_{k-1}(P_k x)), P_k x = x - Q_k (Q_k' x), Afun_0 = h
// (mc_trace.m:47-48 nests one projector per round).  Returns an owned array.
mxArray* apply_deflated(const mxArray* h, const std::vector<mxArray*>& Q, size_t k, mxArray* x) {
    if (k == 0) return call1("feval", {const_cast<mxArray*>(h), x});
    mxArray* Qt = call1("ctranspose", {Q[k - 1]});
    auto proj = [&](mxArray* v) {
        mxArray* c = call1("mtimes", {Qt, v});
        mxArray* qc = call1("mtimes", {Q[k - 1], c});
        mxArray* r = call1("minus", {v, qc});
        mxDestroyArray(c);
        mxDestroyArray(qc);
        return r;
    };
    mxArray* px = proj(x);
    mxArray* y = apply_deflated(h, Q, k - 1, px);
    mxArray* py = proj(y);
    mxDestroyArray(px);
    mxDestroyArray(y);
    mxDestroyArray(Qt);
    return py;
}

// trace(X' * Y)
double trace_xty(mxArray* X, mxArray* Y) {
    mxArray* Xt = call1("ctranspose", {X});
    mxArray* M = call1("mtimes", {Xt, Y});
    mxArray* t = call1("trace", {M});
    const double v = mxGetScalar(t);
    mxDestroyArray(Xt);
    mxDestroyArray(M);
    mxDestroyArray(t);
    return v;
}

// mc_trace.m:33-63 for a handle Afun nothing on the device can evaluate,
// replayed with MATLAB's own built-ins (randn stream, qr, mtimes, trace),
// so the result is the .m file's.  The MEX shadows mc_trace.m, which is why
// the .m cannot simply be called back.
void mc_trace_host(const mxArray* h, double n, double tol, int maxit, int isAreal, int debug,
                   double* tr_out, double* res_out, int* it_out) {
    const int m = 10;
    const int K = (maxit + 3 * m - 1) / (3 * m);  // ceil(maxit / (3 m))
    mxArray* nn = scalar(n);
    mxArray* mm = scalar(m);
    mxArray* zero = scalar(0);
    std::vector<mxArray*> Q;
    double tr = 0.0, tr_old = 0.0, tr_new = 0.0, res = 0.0;
    int it = 0;
    if (debug == 1) mexPrintf("------------- Trace estimation convergence history -------------\n");
    for (it = 1; it <= K; ++it) {
        mxArray* r1 = call1("randn", {nn, mm});
        mxArray* S = call1("sign", {r1});
        mxArray* r2 = call1("randn", {nn, mm});
        mxArray* G = call1("sign", {r2});
        mxArray* Y = apply_deflated(h, Q, Q.size(), S);
        mxArray* qr_out[2] = {nullptr, nullptr};
        mxArray* qr_in[2] = {Y, zero};
        if (mexCallMATLAB(2, qr_out, 2, qr_in, "qr") != 0)
            mexErrMsgIdAndTxt("krylov_hip:mc_trace", "MATLAB call qr failed");
        mxArray* AQ = apply_deflated(h, Q, Q.size(), qr_out[0]);
        tr += trace_xty(qr_out[0], AQ);
        Q.push_back(qr_out[0]);
        mxArray* AG = apply_deflated(h, Q, Q.size(), G);
        tr_new = tr + trace_xty(G, AG) / m;
        res = std::fabs(tr_new - tr_old) / std::max(std::fabs(tr_new), std::fabs(tr_old));
        if (debug == 1)
            mexPrintf("Number of quadrature pts: %d, Trace estimate: %1.4e, Error: %e\n", it * 3 * m, tr_new,
                      res);
        for (mxArray* a : {r1, S, r2, G, Y, qr_out[1], AQ, AG}) mxDestroyArray(a);
        if (res < tol) break;
        tr_old = tr_new;
    }
    if (it > K) it = K;
    for (mxArray* q : Q) mxDestroyArray(q);
    for (mxArray* a : {nn, mm, zero}) mxDestroyArray(a);
    (void)isAreal;  // real arithmetic throughout: real(tr_new) == tr_new
    *tr_out = tr_new;
    *res_out = res;
    *it_out = it;
}

// k x 2 MATLAB index matrix (1-based doubles) -> 0-based columns
void pairs_arg(const mxArray* E, std::vector<int64_t>& a, std::vector<int64_t>& b) {
    const mwSize k = mxGetM(E);
    if (k > 0 && mxGetN(E) != 2) mexErrMsgIdAndTxt("krylov_hip:E", "index list must be k x 2");
    const double* p = mxGetDoubles(E);
    a.resize(k);
    b.resize(k);
    for (mwSize h = 0; h < k; ++h) {
        a[h] = (int64_t)p[h] - 1;
        b[h] = (int64_t)p[h + k] - 1;
    }
}

// the (edited) device matrix back as MATLAB sparse; refreshes the cache key
mxArray* export_sparse(kt_matrix_t A) {
    int64_t n = 0, nnz = 0;
    check(kt_matrix_info(A, &n, &nnz), "export");
    std::vector<int64_t> jc(n + 1), ir(nnz);
    std::vector<double> pr(nnz);
    check(kt_matrix_export_csc(A, jc.data(), ir.data(), pr.data()), "export");
    mxArray* S = mxCreateSparse((mwSize)n, (mwSize)n, (mwSize)(nnz > 0 ? nnz : 1), mxREAL);
    mwIndex* J = mxGetJc(S);
    mwIndex* I = mxGetIr(S);
    double* P = mxGetDoubles(S);
    for (int64_t j = 0; j <= n; ++j) J[j] = (mwIndex)jc[j];
    for (int64_t t = 0; t < nnz; ++t) {
        I[t] = (mwIndex)ir[t];
        P[t] = pr[t];
    }
    if (A == g_A) {
        g_jc.swap(jc);
        g_ir.swap(ir);
        g_pr.swap(pr);
    }
    return S;
}

}  // namespace

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
#if defined(KT_ENTRY_TRACE_EXP)
    // tr = trace_exp(A)                                          trace_exp.m:1
    // trace_exp(A) as the reference's callers write it; an optional second
    // argument names the Afun: 'lanczos' (the north star's Lanczos-quadrature
    // Afun, the default) or 'expmv' (the reference's own handle, trace_exp.m:5)
    if (nrhs < 1 || nrhs > 2) mexErrMsgIdAndTxt("krylov_hip:nargin", "tr = trace_exp(A[, 'lanczos' | 'expmv'])");
    int afun = KT_AFUN_LANCZOS;
    if (nrhs == 2) {
        char af[16] = {0};
        if (!mxIsChar(prhs[1]) || mxGetString(prhs[1], af, sizeof(af)) != 0 ||
            (strcmp(af, "expmv") != 0 && strcmp(af, "lanczos") != 0))
            mexErrMsgIdAndTxt("krylov_hip:afun", "trace_exp: the Afun must be 'lanczos' or 'expmv'");
        if (strcmp(af, "expmv") == 0) afun = KT_AFUN_EXPMV;
    }
    double tr = 0.0;
    check(kt_trace_exp(matrix_arg(prhs[0]), afun, 30, 0, &tr), "trace_exp");
    plhs[0] = scalar(tr);
#elif defined(KT_ENTRY_MC_TRACE)
    // [tr, res, it] = mc_trace(Afun, n, tol, maxit, isAreal, debug)   mc_trace.m:1
    // Afun: a matrix (mc_trace.m:32-34), or a handle @(x) expmv(1, A, x, ...)
    // whose matrix is passed by the caller through the workspace variable A.
    // Afun: a matrix (mc_trace.m:32-34) -> device; the handle trace_exp.m:5
    // builds, @(x) expmv(1, A, x, [], 'double') -> device expmv Afun on its
    // captured A; any other handle -> mc_trace.m replayed with MATLAB's own
    // built-ins (mc_trace_host).  Device paths draw the probes from the
    // build's counter RNG (oracle/krylov_oracle.py:rademacher), the host
    // replay from MATLAB's randn as the .m does.
    if (nrhs < 2) mexErrMsgIdAndTxt("krylov_hip:nargin", "mc_trace(Afun, n, ...)");
    const double tol = scalar_or(nrhs, prhs, 2, 1e-3);
    const int maxit = (int)scalar_or(nrhs, prhs, 3, 10);
    const int isAreal = (int)scalar_or(nrhs, prhs, 4, 0);
    const int debug = (int)scalar_or(nrhs, prhs, 5, 0);
    double tr = 0.0, res = 0.0;
    int it = 0;
    if (mxIsDouble(prhs[0])) {
        check(kt_mc_trace(matrix_arg(prhs[0]), KT_AFUN_MATRIX, KT_FUN_EXP, 0, tol, maxit, isAreal, 0, &tr, &res,
                          &it),
              "mc_trace");
    } else if (mxIsClass(prhs[0], "function_handle")) {
        mxArray* keep = nullptr;
        const mxArray* A = expmv_handle_matrix(prhs[0], &keep);
        if (A) {
            check(kt_mc_trace(matrix_arg(A), KT_AFUN_EXPMV, KT_FUN_EXP, 0, tol, maxit, isAreal, 0, &tr, &res, &it),
                  "mc_trace");
            mxDestroyArray(keep);
        } else {
            mc_trace_host(prhs[0], mxGetScalar(prhs[1]), tol, maxit, isAreal, debug, &tr, &res, &it);
        }
    } else {
        mexErrMsgIdAndTxt("krylov_hip:Afun", "mc_trace: Afun must be a matrix or a function handle");
    }
    plhs[0] = scalar(tr);
    if (nlhs > 1) plhs[1] = scalar(res);
    if (nlhs > 2) plhs[2] = scalar(it);
#elif defined(KT_ENTRY_TRACE_FUN_UPDATE)
    // [Xm, iter, lucky] = trace_fun_update(A, U, B, tol, it, debug, fun)   trace_fun_update.m:1
    if (nrhs < 3) mexErrMsgIdAndTxt("krylov_hip:nargin", "trace_fun_update(A, U, B, ...)");
    kt_matrix_t A = matrix_arg(prhs[0]);
    const mxArray* U = prhs[1];
    const mxArray* B = prhs[2];
    if (mxIsSparse(U) || mxIsSparse(B)) mexErrMsgIdAndTxt("krylov_hip:U", "U and B must be full");
    double xm = 0.0;
    int iter = 0, lucky = 0;
    const mxArray* fh = nrhs > 6 ? prhs[6] : nullptr;
    const int fcode = fun_arg(fh, KT_FUN_EXP, true);
    if (fcode >= 0)
        check(kt_trace_fun_update(A, (int64_t)mxGetN(U), mxGetDoubles(U), mxGetDoubles(B),
                                  scalar_or(nrhs, prhs, 3, 1e-12), (int)scalar_or(nrhs, prhs, 4, 0), fcode,
                                  &xm, &iter, &lucky),
              "trace_fun_update");
    else {  // any elementwise handle: sum(fun(d1) - fun(d2)) with fun evaluated by MATLAB (:88)
        g_feval_failed = false;
        const int st = kt_trace_fun_update_fn(A, (int64_t)mxGetN(U), mxGetDoubles(U), mxGetDoubles(B),
                                              scalar_or(nrhs, prhs, 3, 1e-12), (int)scalar_or(nrhs, prhs, 4, 0),
                                              feval_scalar_fn, const_cast<mxArray*>(fh), &xm, &iter, &lucky);
        if (g_feval_failed)
            mexErrMsgIdAndTxt("krylov_hip:fun", "fun must map a real double vector elementwise");
        check(st, "trace_fun_update");
    }
    {  // warnings stay warnings (trace_fun_update.m:119-130)
        const int it_arg = (int)scalar_or(nrhs, prhs, 4, 0);
        const int it_eff = it_arg > 0 ? it_arg : (int)(mxGetM(prhs[0]) < 100 ? mxGetM(prhs[0]) : 100);
        if (lucky && scalar_or(nrhs, prhs, 5, 0) != 0)
            mexWarnMsgIdAndTxt("TRACE_FUN_UPDATE:lucky", "TRACE_FUN_UPDATE:: Detected lucky breakdown");
        if (iter == it_eff)
            mexWarnMsgIdAndTxt("TRACE_FUN_UPDATE:maxit", "TRACE_FUN_UPDATE:: Reached maximum number of iterations");
    }
    plhs[0] = scalar(xm);
    if (nlhs > 1) plhs[1] = scalar(iter);
    if (nlhs > 2) plhs[2] = scalar(lucky);
#elif defined(KT_ENTRY_FUN_UPDATE)
    // [Xm, iter, lucky, Um] = fun_update(A, U, B, fun, tol, it, debug)   fun_update.m:1
    if (nrhs < 4) mexErrMsgIdAndTxt("krylov_hip:nargin", "fun_update(A, U, B, fun, ...)");
    kt_matrix_t A = matrix_arg(prhs[0]);
    const mwSize n = mxGetM(prhs[0]), rk = mxGetN(prhs[1]);
    const int it = (int)scalar_or(nrhs, prhs, 5, 0);
    const int64_t maxc = (int64_t)(n < (mwSize)((it > 0 ? it : 100) + 1) * rk ? n : ((it > 0 ? it : 100) + 1) * rk);
    std::vector<double> Xm((size_t)maxc * maxc);
    std::vector<double> Um(nlhs > 3 ? (size_t)n * maxc : 0);
    int64_t nc = 0;
    int iter = 0, lucky = 0;
    // nargout <= 3 takes the block-Lanczos branch, 4 the Arnoldi branch (:69-91)
    if (nlhs <= 3)
        check(kt_fun_update_lanczos(A, (int64_t)rk, mxGetDoubles(prhs[1]), mxGetDoubles(prhs[2]),
                                    fun_arg(prhs[3], KT_FUN_EXP), scalar_or(nrhs, prhs, 4, 1e-12), it, maxc,
                                    Xm.data(), &nc, &iter, &lucky),
              "fun_update");
    else
        check(kt_fun_update(A, (int64_t)rk, mxGetDoubles(prhs[1]), mxGetDoubles(prhs[2]),
                            fun_arg(prhs[3], KT_FUN_EXP), scalar_or(nrhs, prhs, 4, 1e-12), it, maxc, Xm.data(),
                            &nc, &iter, &lucky, Um.data()),
              "fun_update");
    if (lucky) mexWarnMsgIdAndTxt("FUN_UPDATE:lucky", "FUN_UPDATE:: Detected lucky breakdown");  // fun_update.m:127-128
    if (iter == (it > 0 ? it : (int)(n < 100 ? n : 100)))
        mexWarnMsgIdAndTxt("FUN_UPDATE:maxit", "FUN_UPDATE:: Reached maximum number of iterations");  // :133-135
    // :137 Um = Um(:, 1:size(Xm, 1)) runs on the Lanczos branch too, where Um
    // is the n x 2rk window: past two steps the reference stops with MATLAB's
    // index error, and so does the shim (never a silently different algorithm)
    if (nlhs <= 3 && nc > (int64_t)(2 * rk))
        mexErrMsgIdAndTxt("MATLAB:badsubscript",
                          "Index in position 2 exceeds array bounds (must not exceed %d). (fun_update.m:137: "
                          "Um(:, 1:size(Xm, 1)) on the 2-block Lanczos window, size(Xm, 1) = %d)",
                          (int)(2 * rk), (int)nc);
    plhs[0] = mxCreateDoubleMatrix(nc, nc, mxREAL);
    memcpy(mxGetDoubles(plhs[0]), Xm.data(), sizeof(double) * nc * nc);
    if (nlhs > 1) plhs[1] = scalar(iter);
    if (nlhs > 2) plhs[2] = scalar(lucky);
    if (nlhs > 3) {
        plhs[3] = mxCreateDoubleMatrix(n, nc, mxREAL);
        memcpy(mxGetDoubles(plhs[3]), Um.data(), sizeof(double) * n * nc);
    }
#elif defined(KT_ENTRY_FG_EXP)
    // [f, gr] = fun_and_grad_krylov_exp(X, A, Omega, eA, tol, it, debug)   fun_and_grad_krylov_exp.m:1
    if (nrhs < 6) mexErrMsgIdAndTxt("krylov_hip:nargin", "fun_and_grad_krylov_exp(X, A, Omega, eA, tol, it, ...)");
    kt_matrix_t A = matrix_arg(prhs[1], "FUN_AND_GRAD_KRYLOV:: matrix A is not Hermitian");
    const mwSize nom = mxGetM(prhs[2]);
    std::vector<double> gr(nom);
    double f = 0.0;
    check(kt_fun_and_grad_krylov_exp(A, (int64_t)nom, mxGetDoubles(prhs[0]), mxGetDoubles(prhs[2]),
                                     mxGetDoubles(prhs[3]), mxGetScalar(prhs[4]), (int)mxGetScalar(prhs[5]), &f,
                                     gr.data()),
          "fun_and_grad_krylov_exp");
    plhs[0] = scalar(f);
    if (nlhs > 1) {
        plhs[1] = mxCreateDoubleMatrix(nom, 1, mxREAL);
        memcpy(mxGetDoubles(plhs[1]), gr.data(), sizeof(double) * nom);
    }
#elif defined(KT_ENTRY_FG_FUN)
    // [f, gr] = fun_and_grad_krylov_fun(X, A, Omega, fun, dfun, dfA, tol, it, debug, fun_M)
    if (nrhs < 8) mexErrMsgIdAndTxt("krylov_hip:nargin", "fun_and_grad_krylov_fun(X, A, Omega, fun, dfun, dfA, tol, it, ...)");
    kt_matrix_t A = matrix_arg(prhs[1], "FUN_AND_GRAD_KRYLOV_FCONNECTIVITY:: matrix A is not Hermitian");
    const int fc = fun_arg(prhs[3], KT_FUN_EXP), dfc = fun_arg(prhs[4], KT_FUN_EXP);
    const mwSize nom = mxGetM(prhs[2]);
    std::vector<double> gr(nom);
    double f = 0.0;
    check(kt_fun_and_grad_krylov_fun(A, (int64_t)nom, mxGetDoubles(prhs[0]), mxGetDoubles(prhs[2]), fc, dfc,
                                     mxGetDoubles(prhs[5]), mxGetScalar(prhs[6]), (int)mxGetScalar(prhs[7]), &f,
                                     gr.data()),
          "fun_and_grad_krylov_fun");
    plhs[0] = scalar(f);
    if (nlhs > 1) {
        plhs[1] = mxCreateDoubleMatrix(nom, 1, mxREAL);
        memcpy(mxGetDoubles(plhs[1]), gr.data(), sizeof(double) * nom);
    }
#elif defined(KT_ENTRY_KRYLOV_MIOBI)
    // [edges, rob, A_new] = krylov_miobi(A, k, E, tol, it, poles, debug, miobi, rescale)
    //                                                                krylov_miobi.m:1
    if (nrhs < 2) mexErrMsgIdAndTxt("krylov_hip:nargin", "krylov_miobi(A, k, E, ...)");
    kt_matrix_t A = matrix_arg(prhs[0]);
    const int k = (int)mxGetScalar(prhs[1]);
    std::vector<int64_t> ei, ej;
    if (nrhs > 2 && !mxIsEmpty(prhs[2])) {
        pairs_arg(prhs[2], ei, ej);
    } else {  // :42-46 all edges with E(:,1) >= E(:,2), in find() order
        int64_t n = 0, nnz = 0;
        check(kt_matrix_info(A, &n, &nnz), "krylov_miobi");
        std::vector<int64_t> jc(n + 1), ir(nnz);
        check(kt_matrix_export_csc(A, jc.data(), ir.data(), nullptr), "krylov_miobi");
        for (int64_t j = 0; j < n; ++j)
            for (int64_t t = jc[j]; t < jc[j + 1]; ++t)
                if (ir[t] >= j) {
                    ei.push_back(ir[t]);
                    ej.push_back(j);
                }
    }
    char mode[16] = "break";
    if (nrhs > 7 && !mxIsEmpty(prhs[7])) mxGetString(prhs[7], mode, sizeof(mode));
    int make = 0;
    if (strcmp(mode, "make") == 0) make = 1;
    else if (strcmp(mode, "break") != 0)
        mexErrMsgIdAndTxt("krylov_hip:miobi", "KRYLOV_MIOBI:: not supported option for miobi");
    const int64_t cap = (int64_t)ei.size() < k ? (int64_t)ei.size() : k;
    std::vector<int64_t> si(cap > 0 ? cap : 1), sj(cap > 0 ? cap : 1);
    double rob = 0.0;
    int64_t ns = 0;
    check(kt_krylov_miobi(A, k, (int64_t)ei.size(), ei.data(), ej.data(), scalar_or(nrhs, prhs, 3, 1e-12),
                          (int)scalar_or(nrhs, prhs, 4, 0), make, scalar_or(nrhs, prhs, 8, 1.0), si.data(),
                          sj.data(), &rob, &ns),
          "krylov_miobi");
    plhs[0] = mxCreateDoubleMatrix((mwSize)ns, 2, mxREAL);
    double* e = mxGetDoubles(plhs[0]);
    for (int64_t h = 0; h < ns; ++h) {
        e[h] = (double)(si[h] + 1);
        e[h + ns] = (double)(sj[h] + 1);
    }
    if (nlhs > 1) plhs[1] = scalar(rob);
    if (nlhs > 2) plhs[2] = export_sparse(A);
#elif defined(KT_ENTRY_FME)
    // [X, iter] = function_multiple_entries(A, omega, f, tol, it, poles, debug)
    //                                                    function_multiple_entries.m:1
    if (nrhs < 3) mexErrMsgIdAndTxt("krylov_hip:nargin", "function_multiple_entries(A, omega, f, ...)");
    if (nrhs > 5 && !mxIsEmpty(prhs[5]) && !(mxGetM(prhs[5]) * mxGetN(prhs[5]) == 1 &&
                                             mxGetScalar(prhs[5]) == mxGetInf()))
        mexErrMsgIdAndTxt("krylov_hip:poles", "FUNCTION_MULTIPLE_ENTRIES::Unsupported rational Krylov yet");
    std::vector<int64_t> oi, oj;
    pairs_arg(prhs[1], oi, oj);
    mxArray* X = mxCreateDoubleMatrix((mwSize)oi.size(), 1, mxREAL);
    int iter = 0;
    check(kt_function_multiple_entries(matrix_arg(prhs[0]), (int64_t)oi.size(), oi.data(), oj.data(),
                                       fun_arg(prhs[2], KT_FUN_EXP), scalar_or(nrhs, prhs, 3, 1e-12),
                                       (int)scalar_or(nrhs, prhs, 4, 0), mxGetDoubles(X), &iter),
          "function_multiple_entries");
    {
        const int it_arg = (int)scalar_or(nrhs, prhs, 4, 0);
        const mwSize na = mxGetM(prhs[0]);
        if (iter == (it_arg > 0 ? it_arg : (int)(na < 100 ? na : 100)))  // :158-161
            mexWarnMsgIdAndTxt("FUNCTION_MULTIPLE_ENTRIES:maxit",
                               "FUNCTION_MULTIPLE_ENTRIES:: Reached maximum number of iterations");
    }
    plhs[0] = X;
    if (nlhs > 1) plhs[1] = scalar(iter);
#elif defined(KT_ENTRY_HESS_EXP) || defined(KT_ENTRY_HESS_FUN)
    // Hes = hessianfcn_exp(X, A, Omega, tol, it)          hessianfcn_exp.m:1
    // Hes = hessianfcn_fun(X, A, Omega, f, tol, it)       hessianfcn_fun.m:1
#if defined(KT_ENTRY_HESS_EXP)
    const int off = 0;
    const int fcode = KT_FUN_EXP;
#else
    const int off = 1;
    if (nrhs < 4) mexErrMsgIdAndTxt("krylov_hip:nargin", "hessianfcn_fun(X, A, Omega, f, tol, it)");
    const int fcode = fun_arg(prhs[3], KT_FUN_EXP);
#endif
    if (nrhs < 3) mexErrMsgIdAndTxt("krylov_hip:nargin", "hessianfcn(X, A, Omega, ...)");
    const mwSize nom = mxGetM(prhs[2]);
    mxArray* H = mxCreateDoubleMatrix(nom, nom, mxREAL);
    check(kt_hessianfcn(matrix_arg(prhs[1]), (int64_t)nom, mxGetDoubles(prhs[0]), mxGetDoubles(prhs[2]),
                        fcode, scalar_or(nrhs, prhs, 3 + off, 1e-12), (int)scalar_or(nrhs, prhs, 4 + off, 0),
                        mxGetDoubles(H)),
          "hessianfcn");
    plhs[0] = H;
#else
#error "define one KT_ENTRY_* (see the header of this file)"
#endif
}
