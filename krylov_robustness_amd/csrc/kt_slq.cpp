// kt_slq.cpp -- driver of the probe-Lanczos quadrature hot path.
//
// For each sweep of P probes (one n x P probe block), m Lanczos steps run as
// four launches each (K1 spmm_dot, coef, K2 update, norm; see
// kt_kernels.hip).  The per-probe recurrence coefficients (alpha, up, low)
// go to a pinned host record; once all sweeps are queued the host solves
// the m x m tridiagonal eigenproblems (kt_dense.cpp) and forms
//   q_p = ||z_p||^2 e1' f(T_p) e1,   T_p = (H + H')/2   (trace_fun_update.m:78-81).
#include <algorithm>
#include <cmath>
#include <thread>

#include "kt_internal.h"
#include "kt_launch.h"

namespace kt {

static int auto_block(int64_t n, int64_t nprobes) {
    // Largest power-of-two P whose gathered n x P block (8nP bytes) stays
    // within ~160 MB, i.e. inside the 256 MiB Infinity Cache next to the CSR
    // stream; measured best on MI355X for n = 1M (P = 16) and n = 100k
    // (P = 128) -- profiles/r01_sweep.txt.
    int P = 128;
    while (P > 8 && (double)n * 8.0 * P > 160.0e6) P >>= 1;
    while (P > 1 && P / 2 >= nprobes) P >>= 1;
    return P;
}

static bool pow2_le128(int b) { return b >= 1 && b <= 128 && (b & (b - 1)) == 0; }

}  // namespace kt

using namespace kt;

extern "C" int kt_slq_plan(kt_matrix_t A, int64_t nprobes, int* block) {
    if (!A || !block || nprobes < 0) {
        kt::set_error("kt_slq_plan: bad argument");
        return KT_ERR_ARG;
    }
    *block = auto_block(A->n, nprobes);
    return KT_OK;
}

extern "C" int kt_slq_trace(kt_matrix_t A, int fun, int m, uint64_t seed, int64_t probe_offset,
                            int64_t nprobes, int block, double* sum_q, double* sum_q2, double* q) {
    try {
        if (!A) fail(KT_ERR_ARG, "A is NULL");
        if (fun < KT_FUN_EXP || fun > KT_FUN_SQRT) fail(KT_ERR_ARG, "unknown fun code");
        if (m < 1 || m > 256) fail(KT_ERR_ARG, "m must be in [1, 256]");
        if (nprobes < 0 || probe_offset < 0) fail(KT_ERR_ARG, "negative probe range");
        if (block != 0 && !pow2_le128(block)) fail(KT_ERR_ARG, "block must be 0 or a power of two <= 128");
        kt_context_s* ctx = A->ctx;
        const int64_t n64 = A->n;
        if (sum_q) *sum_q = 0.0;
        if (sum_q2) *sum_q2 = 0.0;
        if (nprobes == 0 || n64 == 0) return KT_OK;
        const int n = (int)n64;
        const int P = block ? block : auto_block(n64, nprobes);
        const int64_t nsweeps = (nprobes + P - 1) / P;
        const int grid = spmm_grid(n, P, ctx->num_cu * 4);           // K2 / short rows
        const int lblocks = long_blocks_for(A->n_long, ctx->num_cu * 2);
        const int grid1 = grid + lblocks;                             // K1 total
        KT_HIP(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;

        Workspace& w = ctx->ws;
        const size_t blk_bytes = sizeof(double) * (size_t)n * P;
        w.X0.ensure(blk_bytes);
        w.X1.ensure(blk_bytes);
        w.Y.ensure(blk_bytes);
        w.partial.ensure(sizeof(double) * (size_t)(grid1 + grid * 3) * P);
        w.k2s.ensure(sizeof(double) * 4 * P);
        w.coef.ensure(sizeof(double) * 2 * P);
        w.scales.ensure(sizeof(double) * 3 * P);
        const size_t rec = (size_t)3 * m * P;  // [alpha | up | low][m][P]
        w.trec.ensure(sizeof(double) * rec);
        w.host_trec.ensure(sizeof(double) * rec * nsweeps);

        double* part1 = w.partial.as<double>();
        double* part2 = part1 + (size_t)grid1 * P;
        double* k2s = w.k2s.as<double>();
        double* coef = w.coef.as<double>();
        double* trec = w.trec.as<double>();
        double* htrec = w.host_trec.as<double>();

        for (int64_t s = 0; s < nsweeps; ++s) {
            double* ucur = w.X1.as<double>();
            double* uprev = w.X0.as<double>();
            double* sc = w.scales.as<double>();
            double* sp = sc + P;
            double* sn = sc + 2 * P;
            KT_HIP(launch_rademacher(P, n, seed, probe_offset + s * P, A->d_perm, ucur, st));
            KT_HIP(launch_fill(sc, P, 1.0 / std::sqrt((double)n), st));
            KT_HIP(launch_fill(k2s, P, (double)n, st));  // ||z||^2 = n
            for (int j = 0; j < m; ++j) {
                const int first = (j == 0);
                prof_begin(ctx, PROF_SPMM);
                KT_HIP(launch_spmm_dot(P, ctx->k1_flags | (A->unit_values ? 2 : 0), grid1, A->d_rowptr, A->d_col, A->d_val, n,
                                       ucur, sc, w.Y.as<double>(), part1, A->d_long_rows,
                                       A->n_long, A->long_thresh, lblocks, st));
                prof_end(ctx, PROF_SPMM);
                KT_HIP(launch_coef_cgs2(P, part1, grid1, first, k2s, sc, sp, coef,
                                        trec + (size_t)(0 * m + j) * P,
                                        trec + (size_t)(1 * m + j) * P, st));
                prof_begin(ctx, PROF_UPDATE);
                KT_HIP(launch_update(P, grid, n, w.Y.as<double>(), uprev, ucur, sc, sp, coef, first,
                                     part2, st));
                prof_end(ctx, PROF_UPDATE);
                KT_HIP(launch_norm(P, part2, grid, k2s, sn, trec + (size_t)(2 * m + j) * P, st));
                std::swap(ucur, uprev);  // uprev now holds u_{j+1}
                double* t = sp;
                sp = sc;
                sc = sn;
                sn = t;
            }
            KT_HIP(hipMemcpyAsync(htrec + rec * s, trec, sizeof(double) * rec,
                                  hipMemcpyDeviceToHost, st));
        }
        KT_HIP(hipStreamSynchronize(st));
        prof_collect(ctx);

        // host quadrature, parallel over probes
        std::vector<double> qv((size_t)nprobes);
        unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (nprobes < 64) nth = 1;
        auto work = [&](int64_t p_begin, int64_t p_end) {
            std::vector<double> al(m), off(m);
            for (int64_t p = p_begin; p < p_end; ++p) {
                const int64_t s = p / P;
                const int c = (int)(p % P);
                const double* R = htrec + rec * s;
                int steps = m;
                for (int j = 0; j < m; ++j) {
                    if (R[(size_t)(2 * m + j) * P + c] < 1e-8) { steps = j + 1; break; }
                }
                for (int j = 0; j < steps; ++j) al[j] = R[(size_t)(0 * m + j) * P + c];
                for (int j = 0; j + 1 < steps; ++j)
                    off[j] = 0.5 * (R[(size_t)(2 * m + j) * P + c] + R[(size_t)(1 * m + j + 1) * P + c]);
                qv[p] = (double)n * tridiag_quadrature(steps, al.data(), off.data(), fun);
            }
        };
        if (nth == 1) {
            work(0, nprobes);
        } else {
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nth; ++t)
                th.emplace_back(work, nprobes * t / nth, nprobes * (t + 1) / nth);
            for (auto& t : th) t.join();
        }
        double s1 = 0.0, s2 = 0.0;
        for (int64_t p = 0; p < nprobes; ++p) {
            s1 += qv[p];
            s2 += qv[p] * qv[p];
            if (q) q[p] = qv[p];
        }
        if (sum_q) *sum_q = s1;
        if (sum_q2) *sum_q2 = s2;
    } catch (const kt::Status& s) {
        kt::set_error(s.msg);
        return s.code;
    } catch (const std::exception& e) {
        kt::set_error(e.what());
        return KT_ERR_ARG;
    }
    return KT_OK;
}
