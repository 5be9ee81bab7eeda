// mex_runtime.cpp -- a stand-in for the pieces of MATLAB's MEX runtime that
// krylov_robustness_amd/mex/kt_mex.cpp uses (TEST INFRASTRUCTURE ONLY).
//
// MATLAB is not installed, so the MEX shim cannot run inside MATLAB.  This
// runtime gives it a host process instead: mxArray values (full and sparse
// real double, char, function handles, the struct/cell that functions()
// returns), the mx/mex API calls the shim makes, and mexCallMATLAB for the
// built-ins the shim calls back into -- func2str, functions, feval (the
// elementwise handles @exp/@sinh/@cosh/@sin/@cos/@log/@sqrt, @(x)x.^2, the
// matrix handle @(x)A*x with its captured A, and a handle that errors),
// randn/sign (deterministic: see below), qr (through the library's own
// kt_householder_qr, the factorisation MATLAB's qr(W, 0) computes), mtimes,
// ctranspose, minus and trace.  tests/test_mex_exec.py builds one shared
// library per KT_ENTRY_* of the shim against this runtime and calls
// mexFunction through the stub_* entry points below with MATLAB-shaped
// arguments (1-based double index lists, omitted defaults).
//
// mexErrMsgIdAndTxt throws (MATLAB longjmps out of the MEX; stub_call catches
// the throw and records the id and message); mexWarnMsgIdAndTxt records the
// warning.  randn(n, m) returns, for its k-th call since stub_set_randn_seed,
// the +-1 Rademacher columns k*m .. k*m+m-1 of the build's counter RNG
// (oracle/krylov_oracle.py rademacher), so sign(randn(n, 10)) in
// mc_trace.m:43-44 draws exactly the probes the oracle's mc_trace uses.
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <cmath>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "mex.h"
#include "../../include/krylov_trace.h"

struct mxArray_tag {
    enum Kind { DOUBLE, SPARSE, CHAR, HANDLE, STRUCT, CELL } kind = DOUBLE;
    size_t m = 0, n = 0;
    std::vector<double> pr;           // DOUBLE: m*n column-major; SPARSE: nzmax values
    std::vector<mwIndex> jc, ir;      // SPARSE
    std::string str;                  // CHAR text; HANDLE: its func2str text
    mxArray* captured = nullptr;      // HANDLE: the workspace variable A (owned)
    std::map<std::string, mxArray*> fields;  // STRUCT (1 x 1, owned)
    std::vector<mxArray*> cells;      // CELL (owned)
};

namespace {

struct MexError {
    std::string id, msg;
};

std::string g_err_id, g_err_msg;
std::vector<std::pair<std::string, std::string>> g_warnings;
std::vector<void (*)(void)> g_atexit;
int g_lock = 0;
uint64_t g_seed = 0;
uint64_t g_randn_calls = 0;
int g_feval_calls = 0;
std::string g_printed;
kt_context_t g_qr_ctx = nullptr;

std::string vfmt(const char* f, va_list ap) {
    char buf[4096];
    vsnprintf(buf, sizeof(buf), f, ap);
    return buf;
}

mxArray* dense(size_t m, size_t n) {
    mxArray* a = new mxArray_tag;
    a->kind = mxArray_tag::DOUBLE;
    a->m = m;
    a->n = n;
    a->pr.assign(m * n, 0.0);
    return a;
}

mxArray* clone(const mxArray* a) {
    if (!a) return nullptr;
    mxArray* c = new mxArray_tag(*a);
    c->captured = clone(a->captured);
    for (auto& f : c->fields) f.second = clone(f.second);
    for (auto& x : c->cells) x = clone(x);
    return c;
}

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

double el(const mxArray* a, size_t i, size_t j) { return a->pr[i + j * a->m]; }

// y = A x for a handle's captured A (full or sparse), x full
mxArray* matmul(const mxArray* A, const mxArray* X) {
    if (A->n != X->m) return nullptr;
    mxArray* Y = dense(A->m, X->n);
    for (size_t c = 0; c < X->n; ++c) {
        if (A->kind == mxArray_tag::SPARSE) {
            for (size_t j = 0; j < A->n; ++j) {
                const double x = el(X, j, c);
                for (mwIndex t = A->jc[j]; t < A->jc[j + 1]; ++t) Y->pr[A->ir[t] + c * A->m] += A->pr[t] * x;
            }
        } else {
            for (size_t j = 0; j < A->n; ++j) {
                const double x = el(X, j, c);
                for (size_t i = 0; i < A->m; ++i) Y->pr[i + c * A->m] += el(A, i, j) * x;
            }
        }
    }
    return Y;
}

bool is_full(const mxArray* a) { return a && a->kind == mxArray_tag::DOUBLE; }

std::string strip(const std::string& s) {
    std::string o;
    for (char c : s)
        if (c != ' ') o.push_back(c);
    return o;
}

int elementwise(const std::string& f, const mxArray* x, mxArray** out) {
    double (*fn)(double) = nullptr;
    if (f == "@exp") fn = std::exp;
    else if (f == "@sinh") fn = std::sinh;
    else if (f == "@cosh") fn = std::cosh;
    else if (f == "@sin") fn = std::sin;
    else if (f == "@cos") fn = std::cos;
    else if (f == "@log") fn = std::log;
    else if (f == "@sqrt") fn = std::sqrt;
    const bool square = f == "@(x)x.^2";
    if (!fn && !square) return 1;
    mxArray* y = dense(x->m, x->n);
    for (size_t i = 0; i < x->pr.size(); ++i) y->pr[i] = square ? x->pr[i] * x->pr[i] : fn(x->pr[i]);
    *out = y;
    return 0;
}

int builtin(const std::string& name, int nlhs, mxArray** plhs, int nrhs, mxArray** prhs) {
    if (name == "func2str") {
        if (nrhs != 1 || prhs[0]->kind != mxArray_tag::HANDLE) return 1;
        plhs[0] = mxCreateDoubleScalar(0);
        plhs[0]->kind = mxArray_tag::CHAR;
        plhs[0]->str = prhs[0]->str;
        return 0;
    }
    if (name == "functions") {  // s.workspace{1}.A (only the captured A is modelled)
        if (nrhs != 1 || prhs[0]->kind != mxArray_tag::HANDLE) return 1;
        mxArray* w0 = new mxArray_tag;
        w0->kind = mxArray_tag::STRUCT;
        if (prhs[0]->captured) w0->fields["A"] = clone(prhs[0]->captured);
        mxArray* ws = new mxArray_tag;
        ws->kind = mxArray_tag::CELL;
        ws->cells.push_back(w0);
        mxArray* s = new mxArray_tag;
        s->kind = mxArray_tag::STRUCT;
        s->fields["workspace"] = ws;
        plhs[0] = s;
        return 0;
    }
    if (name == "feval") {
        if (nrhs != 2 || prhs[0]->kind != mxArray_tag::HANDLE || !is_full(prhs[1])) return 1;
        ++g_feval_calls;
        const std::string f = strip(prhs[0]->str);
        if (f == "@(x)A*x") {
            if (!prhs[0]->captured) return 1;
            plhs[0] = matmul(prhs[0]->captured, prhs[1]);
            return plhs[0] ? 0 : 1;
        }
        return elementwise(f, prhs[1], &plhs[0]);  // @(x)error(...) and the rest: 1
    }
    if (name == "randn") {
        if (nrhs != 2) return 1;
        const size_t m = (size_t)mxGetScalar(prhs[0]), n = (size_t)mxGetScalar(prhs[1]);
        mxArray* r = dense(m, n);
        for (size_t c = 0; c < n; ++c) {
            const uint64_t key = splitmix64(splitmix64(g_seed) + (g_randn_calls * n + c));
            for (size_t i = 0; i < m; ++i) r->pr[i + c * m] = (splitmix64(key + i) >> 63) ? -1.0 : 1.0;
        }
        ++g_randn_calls;
        plhs[0] = r;
        return 0;
    }
    if (name == "sign") {
        if (nrhs != 1 || !is_full(prhs[0])) return 1;
        mxArray* y = dense(prhs[0]->m, prhs[0]->n);
        for (size_t i = 0; i < y->pr.size(); ++i) {
            const double v = prhs[0]->pr[i];
            y->pr[i] = v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0);
        }
        plhs[0] = y;
        return 0;
    }
    if (name == "qr") {  // [Q, R] = qr(W, 0): the library's device Householder QR
        if (nrhs != 2 || !is_full(prhs[0]) || nlhs != 2) return 1;
        const size_t n = prhs[0]->m, bs = prhs[0]->n;
        if (bs < 1 || bs > 128 || n < bs) return 1;
        if (!g_qr_ctx && kt_context_create(0, &g_qr_ctx) != KT_OK) return 1;
        mxArray* Q = dense(n, bs);
        mxArray* R = dense(bs, bs);
        if (kt_householder_qr(g_qr_ctx, (int64_t)n, (int64_t)bs, prhs[0]->pr.data(), Q->pr.data(), R->pr.data()) !=
            KT_OK) {
            mxDestroyArray(Q);
            mxDestroyArray(R);
            return 1;
        }
        plhs[0] = Q;
        plhs[1] = R;
        return 0;
    }
    if (name == "ctranspose") {
        if (nrhs != 1 || !is_full(prhs[0])) return 1;
        const mxArray* a = prhs[0];
        mxArray* t = dense(a->n, a->m);
        for (size_t i = 0; i < a->m; ++i)
            for (size_t j = 0; j < a->n; ++j) t->pr[j + i * a->n] = el(a, i, j);
        plhs[0] = t;
        return 0;
    }
    if (name == "mtimes") {
        if (nrhs != 2 || !is_full(prhs[1])) return 1;
        plhs[0] = matmul(prhs[0], prhs[1]);
        return plhs[0] ? 0 : 1;
    }
    if (name == "minus") {
        if (nrhs != 2 || !is_full(prhs[0]) || !is_full(prhs[1]) || prhs[0]->pr.size() != prhs[1]->pr.size()) return 1;
        mxArray* y = dense(prhs[0]->m, prhs[0]->n);
        for (size_t i = 0; i < y->pr.size(); ++i) y->pr[i] = prhs[0]->pr[i] - prhs[1]->pr[i];
        plhs[0] = y;
        return 0;
    }
    if (name == "trace") {
        if (nrhs != 1 || !is_full(prhs[0])) return 1;
        double s = 0.0;
        for (size_t i = 0; i < std::min(prhs[0]->m, prhs[0]->n); ++i) s += el(prhs[0], i, i);
        plhs[0] = mxCreateDoubleScalar(s);
        return 0;
    }
    return 1;
}

}  // namespace

extern "C" {

// ---- the MEX API subset (tests/mexstub/mex.h) ----------------------------
bool mxIsDouble(const mxArray* a) { return a->kind == mxArray_tag::DOUBLE || a->kind == mxArray_tag::SPARSE; }
bool mxIsComplex(const mxArray*) { return false; }
bool mxIsSparse(const mxArray* a) { return a->kind == mxArray_tag::SPARSE; }
bool mxIsEmpty(const mxArray* a) { return a->m == 0 || a->n == 0; }
bool mxIsChar(const mxArray* a) { return a->kind == mxArray_tag::CHAR; }
mwSize mxGetM(const mxArray* a) { return a->m; }
mwSize mxGetN(const mxArray* a) { return a->n; }
mwIndex* mxGetJc(const mxArray* a) { return const_cast<mwIndex*>(a->jc.data()); }
mwIndex* mxGetIr(const mxArray* a) { return const_cast<mwIndex*>(a->ir.data()); }
double* mxGetDoubles(const mxArray* a) { return const_cast<double*>(a->pr.data()); }
double mxGetScalar(const mxArray* a) { return a->pr.empty() ? 0.0 : a->pr[0]; }
int mxGetString(const mxArray* a, char* buf, mwSize len) {
    if (a->kind != mxArray_tag::CHAR || len == 0) return 1;
    const size_t k = std::min(a->str.size(), (size_t)len - 1);
    memcpy(buf, a->str.data(), k);
    buf[k] = 0;
    return a->str.size() < len ? 0 : 1;
}
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity) { return dense(m, n); }
mxArray* mxCreateDoubleScalar(double v) {
    mxArray* a = dense(1, 1);
    a->pr[0] = v;
    return a;
}
mxArray* mxCreateSparse(mwSize m, mwSize n, mwSize nzmax, mxComplexity) {
    mxArray* a = new mxArray_tag;
    a->kind = mxArray_tag::SPARSE;
    a->m = m;
    a->n = n;
    a->jc.assign(n + 1, 0);
    a->ir.assign(nzmax, 0);
    a->pr.assign(nzmax, 0.0);
    return a;
}
double mxGetInf(void) { return INFINITY; }
double mxGetNaN(void) { return NAN; }
void mxDestroyArray(mxArray* a) {
    if (!a) return;
    mxDestroyArray(a->captured);
    for (auto& f : a->fields) mxDestroyArray(f.second);
    for (auto* c : a->cells) mxDestroyArray(c);
    delete a;
}
int mexCallMATLAB(int nlhs, mxArray** plhs, int nrhs, mxArray** prhs, const char* name) {
    for (int i = 0; i < nlhs; ++i) plhs[i] = nullptr;
    return builtin(name, nlhs, plhs, nrhs, prhs);
}
bool mxIsClass(const mxArray* a, const char* cls) {
    if (strcmp(cls, "function_handle") == 0) return a->kind == mxArray_tag::HANDLE;
    if (strcmp(cls, "double") == 0) return mxIsDouble(a);
    if (strcmp(cls, "char") == 0) return a->kind == mxArray_tag::CHAR;
    return false;
}
bool mxIsCell(const mxArray* a) { return a->kind == mxArray_tag::CELL; }
bool mxIsStruct(const mxArray* a) { return a->kind == mxArray_tag::STRUCT; }
size_t mxGetNumberOfElements(const mxArray* a) {
    if (a->kind == mxArray_tag::CELL) return a->cells.size();
    if (a->kind == mxArray_tag::STRUCT || a->kind == mxArray_tag::HANDLE) return 1;
    if (a->kind == mxArray_tag::CHAR) return a->str.size();
    return a->m * a->n;
}
mxArray* mxGetCell(const mxArray* a, mwIndex i) { return i < a->cells.size() ? a->cells[i] : nullptr; }
mxArray* mxGetField(const mxArray* a, mwIndex i, const char* name) {
    if (a->kind != mxArray_tag::STRUCT || i != 0) return nullptr;
    auto it = a->fields.find(name);
    return it == a->fields.end() ? nullptr : it->second;
}
int mexPrintf(const char* f, ...) {
    va_list ap;
    va_start(ap, f);
    const std::string s = vfmt(f, ap);
    va_end(ap);
    g_printed += s;
    return (int)s.size();
}
void mexErrMsgIdAndTxt(const char* id, const char* f, ...) {
    va_list ap;
    va_start(ap, f);
    MexError e{id, vfmt(f, ap)};
    va_end(ap);
    throw e;
}
void mexWarnMsgIdAndTxt(const char* id, const char* f, ...) {
    va_list ap;
    va_start(ap, f);
    g_warnings.emplace_back(id, vfmt(f, ap));
    va_end(ap);
}
int mexAtExit(void (*fn)(void)) {
    g_atexit.push_back(fn);
    return 0;
}
void mexLock(void) { ++g_lock; }

// ---- test driver API (ctypes) -----------------------------------------------
mxArray* stub_dense(size_t m, size_t n, const double* colmajor) {
    mxArray* a = dense(m, n);
    if (colmajor) memcpy(a->pr.data(), colmajor, sizeof(double) * m * n);
    return a;
}
mxArray* stub_sparse(size_t m, size_t n, const int64_t* jc, const int64_t* ir, const double* pr) {
    const size_t nnz = (size_t)jc[n];
    mxArray* a = mxCreateSparse(m, n, nnz ? nnz : 1, mxREAL);
    for (size_t j = 0; j <= n; ++j) a->jc[j] = (mwIndex)jc[j];
    for (size_t t = 0; t < nnz; ++t) {
        a->ir[t] = (mwIndex)ir[t];
        a->pr[t] = pr[t];
    }
    return a;
}
mxArray* stub_char(const char* s) {
    mxArray* a = new mxArray_tag;
    a->kind = mxArray_tag::CHAR;
    a->m = 1;
    a->n = strlen(s);
    a->str = s;
    return a;
}
// A function handle with func2str text `text`; `captured` (nullable) becomes
// its workspace variable A (copied).
mxArray* stub_handle(const char* text, const mxArray* captured) {
    mxArray* a = new mxArray_tag;
    a->kind = mxArray_tag::HANDLE;
    a->m = a->n = 1;
    a->str = text;
    a->captured = clone(captured);
    return a;
}
void stub_destroy(mxArray* a) { mxDestroyArray(a); }
size_t stub_m(const mxArray* a) { return a->m; }
size_t stub_n(const mxArray* a) { return a->n; }
int stub_is_sparse(const mxArray* a) { return a->kind == mxArray_tag::SPARSE; }
size_t stub_nnz(const mxArray* a) { return a->kind == mxArray_tag::SPARSE ? (size_t)a->jc[a->n] : a->m * a->n; }
const double* stub_data(const mxArray* a) { return a->pr.data(); }
void stub_sparse_export(const mxArray* a, int64_t* jc, int64_t* ir) {
    for (size_t j = 0; j <= a->n; ++j) jc[j] = (int64_t)a->jc[j];
    for (size_t t = 0; t < (size_t)a->jc[a->n]; ++t) ir[t] = (int64_t)a->ir[t];
}

typedef void (*mex_fn)(int, mxArray**, int, const mxArray**);
// Calls an entry's mexFunction.  0: returned normally; 1: it raised an error
// (stub_error_id / stub_error_msg); 2: a C++ exception other than a MEX error
// escaped (a shim defect: nothing may unwind out of the library).
int stub_call(mex_fn fn, int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs) {
    g_err_id.clear();
    g_err_msg.clear();
    for (int i = 0; i < nlhs; ++i) plhs[i] = nullptr;
    try {
        fn(nlhs, plhs, nrhs, prhs);
    } catch (const MexError& e) {
        g_err_id = e.id;
        g_err_msg = e.msg;
        return 1;
    } catch (const std::exception& e) {
        g_err_msg = e.what();
        return 2;
    } catch (...) {
        return 2;
    }
    return 0;
}
const char* stub_error_id(void) { return g_err_id.c_str(); }
const char* stub_error_msg(void) { return g_err_msg.c_str(); }
int stub_warning_count(void) { return (int)g_warnings.size(); }
const char* stub_warning_id(int i) { return g_warnings.at(i).first.c_str(); }
const char* stub_warning_msg(int i) { return g_warnings.at(i).second.c_str(); }
void stub_clear(void) {
    g_warnings.clear();
    g_printed.clear();
    g_feval_calls = 0;
}
const char* stub_printed(void) { return g_printed.c_str(); }
int stub_feval_calls(void) { return g_feval_calls; }
int stub_lock_count(void) { return g_lock; }
int stub_atexit_count(void) { return (int)g_atexit.size(); }
void stub_set_randn_seed(uint64_t seed) {
    g_seed = seed;
    g_randn_calls = 0;
}
// MATLAB's exit (or clear mex): the registered mexAtExit handlers run once.
void stub_run_atexit(void) {
    for (auto fn : g_atexit) fn();
    g_atexit.clear();
    if (g_qr_ctx) kt_context_destroy(g_qr_ctx);
    g_qr_ctx = nullptr;
}

}  // extern "C"
