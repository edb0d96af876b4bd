// k_lm.hip — lidarFactor residuals + analytic SE(3) Jacobians + Ceres-1.12-equivalent LM on gfx950.
//
// One LM "pass" = one launch over all factor slots at one parameter vector: every workgroup
// reduces its slots' Huber-corrected normal equations (21 upper JtJ + 6 Jtr + cost + count) with
// wave shuffles, publishes them write-through, and the LAST workgroup to arrive (agent-scope
// ticket) sums the per-workgroup partials in workgroup order — deterministic for a fixed grid —
// and runs the trust-region logic of ceres::TrustRegionMinimizer + LevenbergMarquardtStrategy:
//   pass 0:  evaluate at x, Jacobi column scaling, gradient check, first LM step -> candidate
//   pass k:  evaluate cost + JtJ at the candidate (speculatively), parameter / function tolerance,
//            gain-ratio accept (keep the candidate's JtJ) or reject, next LM step
// so the 4 iterations of a Solve (laserOdometry.cpp:573, laserMapping.cpp:715) take 5 launches
// and no host round trip. Semantics: SURVEY Appendix B. The normal equations replace DENSE_QR's
// Householder solve of [J; D] (same minimiser, rounding-level difference).
#include "aloam_device.hpp"
#include "aloam_internal.hpp"

namespace aloam {

constexpr int LB = 256;          // threads per LM workgroup
constexpr int NACC = 29;         // 21 JtJ + 6 Jtr + cost + residual-block count

// residual and 6-column tangent Jacobian of one factor at (q, t). Returns #residuals (0 = invalid).
// One factor type per instantiation: every branch is resolved at compile time, so r/J stay in
// registers (a run-time type switch over shared r/J arrays made the compiler sink their stores into
// dynamically indexed scratch).
template <int TY, bool FAST = false>
__device__ __forceinline__ int eval_factor_t(const aloam_factor& f, const dquat& q, const double* t, double r[3], double J[3][6]) {
    const dvec3 cp{f.cp[0], f.cp[1], f.cp[2]};
    dvec3 pr, lp;
    if constexpr (TY == 0 || TY == 1) {
        dquat ql = qslerp_identity(1.0, q);          // lidarFactor.hpp:29,81 (s = 1)
        pr = qrot(ql, cp);
        lp = {pr.x + 1.0 * t[0], pr.y + 1.0 * t[1], pr.z + 1.0 * t[2]};
    } else {
        pr = qrot(q, cp);                            // lidarFactor.hpp:120,154
        lp = {pr.x + t[0], pr.y + t[1], pr.z + t[2]};
    }
    if constexpr (TY == 0) {                         // LidarEdgeFactor (lidarFactor.hpp:19-43)
        const dvec3 a{f.a[0], f.a[1], f.a[2]}, b{f.b[0], f.b[1], f.b[2]};
        const dvec3 u{lp.x - a.x, lp.y - a.y, lp.z - a.z}, v{lp.x - b.x, lp.y - b.y, lp.z - b.z};
        const dvec3 nu = dcross(u, v);
        const dvec3 w{a.x - b.x, a.y - b.y, a.z - b.z};
        const double n = sqrt(w.x * w.x + w.y * w.y + w.z * w.z);
        // d nu = dlp x w, dlp/dtheta_k = -2 pr x e_k, dlp/dt_k = e_k:
        //   J_rot[i][k] = (2 pr_i w_k - 2 (pr.w) delta_ik) / n ,  J_t[i][k] = (e_k x w)_i / n
        const double inv = 1.0 / n;
        if constexpr (FAST) { r[0] = nu.x * inv; r[1] = nu.y * inv; r[2] = nu.z * inv; }   // one division, not four
        else { r[0] = nu.x / n; r[1] = nu.y / n; r[2] = nu.z / n; }
        const double pw2 = 2.0 * (pr.x * w.x + pr.y * w.y + pr.z * w.z);
        const double prv[3] = {pr.x, pr.y, pr.z}, wv[3] = {w.x, w.y, w.z};
#pragma unroll
        for (int i = 0; i < 3; i++) {
#pragma unroll
            for (int k = 0; k < 3; k++) J[i][k] = (2.0 * prv[i] * wv[k] - (i == k ? pw2 : 0.0)) * inv;
        }
        // e_k x w: e_x x w = (0, -w.z, w.y), e_y x w = (w.z, 0, -w.x), e_z x w = (-w.y, w.x, 0)
        J[0][3] = 0.0;         J[0][4] = w.z * inv;  J[0][5] = -w.y * inv;
        J[1][3] = -w.z * inv;  J[1][4] = 0.0;        J[1][5] = w.x * inv;
        J[2][3] = w.y * inv;   J[2][4] = -w.x * inv; J[2][5] = 0.0;
        return 3;
    }
    if constexpr (TY == 1 || TY == 2) {
        dvec3 nrm;
        if constexpr (TY == 1) {                           // LidarPlaneFactor (lidarFactor.hpp:69-90)
            nrm = {f.b[0], f.b[1], f.b[2]};
            r[0] = (lp.x - f.a[0]) * nrm.x + (lp.y - f.a[1]) * nrm.y + (lp.z - f.a[2]) * nrm.z;
        } else {                                     // LidarPlaneNormFactor (lidarFactor.hpp:113-125)
            nrm = {f.a[0], f.a[1], f.a[2]};
            r[0] = nrm.x * lp.x + nrm.y * lp.y + nrm.z * lp.z + f.b[0];
        }
        dvec3 np = dcross(nrm, pr);                  // dr/dtheta = -2 (n x pr)
        J[0][0] = -2.0 * np.x; J[0][1] = -2.0 * np.y; J[0][2] = -2.0 * np.z;
        J[0][3] = nrm.x; J[0][4] = nrm.y; J[0][5] = nrm.z;
        return 1;
    } else {
        // LidarDistanceFactor (lidarFactor.hpp:147-161): J_rot = -2 [pr]x, J_t = I
        r[0] = lp.x - f.a[0]; r[1] = lp.y - f.a[1]; r[2] = lp.z - f.a[2];
        J[0][0] = 0.0;           J[0][1] = 2.0 * pr.z;   J[0][2] = -2.0 * pr.y;
        J[1][0] = -2.0 * pr.z;   J[1][1] = 0.0;          J[1][2] = 2.0 * pr.x;
        J[2][0] = 2.0 * pr.y;    J[2][1] = -2.0 * pr.x;  J[2][2] = 0.0;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int k = 0; k < 3; k++) J[i][3 + k] = (i == k) ? 1.0 : 0.0;
        return 3;
    }
}

__device__ __forceinline__ int eval_factor(const aloam_factor& f, const dquat& q, const double* t, double r[3], double J[3][6]) {
    switch (f.type) {
        case 0: return eval_factor_t<0>(f, q, t, r, J);
        case 1: return eval_factor_t<1>(f, q, t, r, J);
        case 2: return eval_factor_t<2>(f, q, t, r, J);
        case 3: return eval_factor_t<3>(f, q, t, r, J);
        default: return 0;
    }
}

// ceres::HuberLoss(0.1) + Corrector (rho'' <= 0 => plain sqrt(rho') scaling)
__device__ inline double huber_scale(double s, double* rho0) {
    const double a = 0.1, b = a * a;
    if (s > b) {
        const double r = sqrt(s);
        *rho0 = 2.0 * a * r - b;
        return sqrt(fmax(2.2250738585072014e-308, a / r));
    }
    *rho0 = s;
    return 1.0;
}

// one residual row's normal-equation terms; fused multiply-adds (one rounding per term instead of two:
// the normal equations are a rounding-level restatement of Ceres' QR anyway, and this halves the fp64
// issue of the accumulation, the longest part of a factor's evaluation)
__device__ __forceinline__ void add_row(const double* J, double r, double sc, double* acc) {
    double Ji[6];
#pragma unroll
    for (int c = 0; c < 6; c++) Ji[c] = J[c] * sc;
    const double ri = r * sc;
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
        for (int b = a; b < 6; b++) { acc[k] = fma(Ji[a], Ji[b], acc[k]); k++; }
#pragma unroll
    for (int a = 0; a < 6; a++) acc[21 + a] = fma(Ji[a], ri, acc[21 + a]);
}

template <int TY>
__device__ __forceinline__ void accumulate_t(const aloam_factor& f, const dquat& q, const double* t, double* acc) {
    double r[3], J[3][6];
    constexpr int m = (TY == 1 || TY == 2) ? 1 : 3;
    eval_factor_t<TY, true>(f, q, t, r, J);
    double rho0, sc;
    if constexpr (m == 1) {
        sc = huber_scale(r[0] * r[0], &rho0);
        add_row(J[0], r[0], sc, acc);
    } else {
        double sq = r[0] * r[0];
        sq += r[1] * r[1];
        sq += r[2] * r[2];
        sc = huber_scale(sq, &rho0);
        add_row(J[0], r[0], sc, acc);
        add_row(J[1], r[1], sc, acc);
        add_row(J[2], r[2], sc, acc);
    }
    acc[27] += 0.5 * rho0;
    acc[28] += 1.0;
}
__device__ __forceinline__ void accumulate(const aloam_factor& f, const dquat& q, const double* t, double* acc) {
    switch (f.type) {
        case 0: accumulate_t<0>(f, q, t, acc); break;
        case 1: accumulate_t<1>(f, q, t, acc); break;
        case 2: accumulate_t<2>(f, q, t, acc); break;
        case 3: accumulate_t<3>(f, q, t, acc); break;
        default: break;
    }
}

// ---- host-side-free LM math (thread 0 of the last workgroup) -------------------------------
// Plus of Ceres' EigenQuaternionParameterization: q' = [sin|d|/|d| d, cos|d|] * q, t' = t + d_t.
// Steps are small (|d| < 0.25 rad), where sin(x)/x and cos(x) are evaluated as even Taylor
// polynomials in |d|^2 (truncation < 1e-17; no sqrt, sincos or division on the solver's serial
// tail); larger steps take the libm path.
__device__ __forceinline__ void plus7(const double* x, const double* d, double* out) {
    const double nd2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    dquat q{x[0], x[1], x[2], x[3]};
    if (nd2 > 0.0) {
        double sdd, cs;
        if (nd2 < 0.0625) {
            const double y = nd2;   // Horner in fused multiply-adds: half the dependent fp64 ops
            sdd = fma(y, fma(y, fma(y, fma(y, fma(y, fma(y, 1.0 / 6227020800.0, -1.0 / 39916800), 1.0 / 362880), -1.0 / 5040), 1.0 / 120), -1.0 / 6), 1.0);
            cs = fma(y, fma(y, fma(y, fma(y, fma(y, fma(y, fma(y, -1.0 / 87178291200.0, 1.0 / 479001600.0), -1.0 / 3628800), 1.0 / 40320), -1.0 / 720), 1.0 / 24), -0.5), 1.0);
        } else {
            const double nd = sqrt(nd2);
            double sn;
            sincos(nd, &sn, &cs);
            sdd = sn / nd;
        }
        dquat dq{sdd * d[0], sdd * d[1], sdd * d[2], cs};
        dquat r = qmul(dq, q);
        out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
    } else { out[0] = q.x; out[1] = q.y; out[2] = q.z; out[3] = q.w; }
#pragma unroll
    for (int i = 0; i < 3; i++) out[4 + i] = x[4 + i] + d[3 + i];
}
__device__ __forceinline__ double norm7(const double* a) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) s += a[i] * a[i];
    return sqrt(s);
}
__device__ __forceinline__ double grad_max_norm(const double* x, const double* g) {
    // translation part of x - Plus(x, -g) is g_t up to one rounding of x_t (< 1e-10 for |x_t| < 1e5):
    // when it alone already fails the 1e-10 gradient tolerance, skip the sincos of Plus.
    const double gt = fmax(fabs(g[3]), fmax(fabs(g[4]), fabs(g[5])));
    const double xt = fmax(fabs(x[4]), fmax(fabs(x[5]), fabs(x[6])));
    if (gt > 1e-9 && xt < 1e5) return gt;
    double ng[6], xp[7];
#pragma unroll
    for (int i = 0; i < 6; i++) ng[i] = -g[i];
    plus7(x, ng, xp);
    double m = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) m = fmax(m, fabs(x[i] - xp[i]));
    return m;
}
__device__ __forceinline__ double Aget(const double* A, int a, int b) {   // upper-triangle packed
    if (a > b) { int t = a; a = b; b = t; }
    return A[a * 6 - a * (a - 1) / 2 + (b - a)];
}
// 1/sqrt(s) from the hardware estimate plus three Newton steps (quadratic convergence to full
// precision); the Cholesky pivots take this instead of a sqrt and a division each, which are the
// longest latency chain of the serial solver tail.
// (v_rsq_f64 is good to ~2^-23: two steps reach full precision; NR = 3 keeps the older tails' rounding)
template <int NR = 3>
__device__ __forceinline__ double rsqrt_nr(double s) {
    double r = __builtin_amdgcn_rsq(s);
#pragma unroll
    for (int it = 0; it < NR; it++) {
        const double e = fma(-(s * r), r, 1.0);
        r = fma(0.5 * r, e, r);
    }
    return r;
}
__device__ __forceinline__ bool chol_solve6(double M[6][6], const double* rhs, double* y) {
    double L[6][6], inv[6];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double s = M[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) s -= L[j][k] * L[j][k];
        ok = ok && (s > 0.0);
        inv[j] = rsqrt_nr(s);
        L[j][j] = s * inv[j];
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double v = M[i][j];
#pragma unroll
            for (int k = 0; k < j; k++) v -= L[i][k] * L[j][k];
            L[i][j] = v * inv[j];
        }
    }
    double z[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double v = rhs[i];
#pragma unroll
        for (int k = 0; k < i; k++) v -= L[i][k] * z[k];
        z[i] = v * inv[i];
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double v = z[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) v -= L[k][i] * y[k];
        y[i] = v * inv[i];
    }
#pragma unroll
    for (int i = 0; i < 6; i++) ok = ok && isfinite(y[i]);
    return ok;
}

__device__ __forceinline__ void lm_finish(LMState* st, aloam_lm_summary* out, int term) {
    st->done = 1;
    st->termination = term;
    if (out) {
        out->iterations = st->iteration;
        out->successful_steps = st->successful;
        out->termination = term;
        out->num_residual_blocks = st->nres;
        out->initial_cost = st->initial_cost;
        out->final_cost = st->cost;
    }
}

#ifdef ALOAM_LM_TIMING
__device__ unsigned long long g_ns_ts[4];
#define NS_TS(k) do { if (blockIdx.x == 0) g_ns_ts[k] = wall_clock64(); } while (0)
extern "C" int aloam_dbg_ns_ts(unsigned long long* out) { return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ns_ts), sizeof(g_ns_ts)); }
#else
#define NS_TS(k) do { } while (0)
#endif
// LevenbergMarquardtStrategy::ComputeStep + model cost change; loops over invalid steps.
__device__ __forceinline__ void lm_next_step(LMState* st, aloam_lm_summary* out, int max_iter) {
    while (true) {
        if (st->iteration >= max_iter) { lm_finish(st, out, 0); return; }
        st->iteration++;
        double As[6][6], gs[6];
        #pragma unroll
        for (int a = 0; a < 6; a++) {
            gs[a] = st->scale[a] * st->g[a];
            #pragma unroll
            for (int b = 0; b < 6; b++) As[a][b] = st->scale[a] * Aget(st->A, a, b) * st->scale[b];
        }
        if (!st->reuse_diag)
            #pragma unroll
            for (int a = 0; a < 6; a++) st->diag[a] = fmin(fmax(As[a][a], 1e-6), 1e32);
        double M[6][6];
        const double inv_radius = 1.0 / st->radius;
        #pragma unroll
        for (int a = 0; a < 6; a++) {
            #pragma unroll
            for (int b = 0; b < 6; b++) M[a][b] = As[a][b];
            M[a][a] += st->diag[a] * inv_radius;   // D^2 with D = sqrt(diag / radius)
        }
        double y[6];
        NS_TS(0);
        const bool ok = chol_solve6(M, gs, y);
        NS_TS(1);
        st->reuse_diag = 1;
        double step[6], mcc = -1.0;
        if (ok) {
            #pragma unroll
            for (int a = 0; a < 6; a++) step[a] = -y[a];
            double sg = 0, sAs = 0;
            #pragma unroll
            for (int a = 0; a < 6; a++) {
                sg += step[a] * gs[a];
                double t = 0;
                #pragma unroll
                for (int b = 0; b < 6; b++) t += As[a][b] * step[b];
                sAs += step[a] * t;
            }
            mcc = -(sg + 0.5 * sAs);
        }
        if (!ok || mcc < 0.0) {            // invalid step: StepIsInvalid() == StepRejected(0)
            st->radius = st->radius / st->decrease_factor;
            st->decrease_factor *= 2.0;
            st->reuse_diag = 1;
            continue;
        }
        double delta[6];
        #pragma unroll
        for (int a = 0; a < 6; a++) delta[a] = step[a] * st->scale[a];
        NS_TS(2);
        plus7(st->x, delta, st->cand);
        double dx[7];
        #pragma unroll
        for (int i = 0; i < 7; i++) dx[i] = st->x[i] - st->cand[i];
        st->step_norm = norm7(dx);
        NS_TS(3);
        st->mcc = mcc;
        return;
    }
}

__device__ __forceinline__ void lm_tail(LMState* st, const double* tot, int pass, double* xp, aloam_lm_summary* out, int max_iter) {
    if (pass == 0) {
        #pragma unroll
        for (int i = 0; i < 7; i++) st->x[i] = xp[i];
        st->nres = (int)tot[28];
        st->iteration = 0; st->successful = 0; st->done = 0;
        st->cost = tot[27]; st->initial_cost = tot[27];
        if (st->nres == 0) { st->cost = 0; lm_finish(st, out, 4); return; }
        #pragma unroll
        for (int i = 0; i < 21; i++) st->A[i] = tot[i];
        #pragma unroll
        for (int i = 0; i < 6; i++) st->g[i] = tot[21 + i];
        #pragma unroll
        for (int a = 0; a < 6; a++) st->scale[a] = 1.0 / (1.0 + sqrt(Aget(st->A, a, a)));
        st->x_norm = norm7(st->x);
        st->radius = 1e4; st->decrease_factor = 2.0; st->reuse_diag = 0;
        if (grad_max_norm(st->x, st->g) <= 1e-10) { lm_finish(st, out, 3); return; }
        lm_next_step(st, out, max_iter);
        return;
    }
    const double new_cost = tot[27];
    if (st->step_norm <= 1e-8 * (st->x_norm + 1e-8)) { lm_finish(st, out, 2); return; }
    const double cost_change = st->cost - new_cost;
    if (fabs(cost_change) <= 1e-6 * st->cost) { lm_finish(st, out, 1); return; }
    const double rel = cost_change / st->mcc;
    if (rel > 1e-3) {
        #pragma unroll
        for (int i = 0; i < 7; i++) { st->x[i] = st->cand[i]; xp[i] = st->cand[i]; }
        st->x_norm = norm7(st->x);
        #pragma unroll
        for (int i = 0; i < 21; i++) st->A[i] = tot[i];
        #pragma unroll
        for (int i = 0; i < 6; i++) st->g[i] = tot[21 + i];
        st->cost = new_cost;
        st->successful++;
        const double t = 2.0 * rel - 1.0;
        st->radius = st->radius / fmax(1.0 / 3.0, 1.0 - t * t * t);
        st->radius = fmin(1e16, st->radius);
        st->decrease_factor = 2.0;
        st->reuse_diag = 0;
        if (grad_max_norm(st->x, st->g) <= 1e-10) { lm_finish(st, out, 3); return; }
    } else {
        st->radius = st->radius / st->decrease_factor;
        st->decrease_factor *= 2.0;
        st->reuse_diag = 1;
    }
    lm_next_step(st, out, max_iter);
}

// ---- the persistent solver's tail with a short critical path -------------------------------------
// The tail of k_lm_coop runs on one lane while the grid waits, so only what the next pass needs is
// computed there: the accept / reject decision, the trust radius and the next candidate. The step's
// model cost change (mcc, its validity test) and norm, and the norm of an accepted x, are needed one
// pass later only: lm_post computes them on another wave while the next pass's partials are exchanged.
// A step that lm_post finds invalid (mcc < 0, StepIsInvalid) is then handled by the next tail exactly
// as the immediate check would have (radius / decrease_factor, new step, iteration consumed); only its
// speculative evaluation pass is wasted. Same decisions and state sequence as lm_tail up to rounding.
__device__ __forceinline__ void chol_solve6_packed(double* Ml, const double* rhs, double* y, bool* okp) {
    // Ml: lower triangle packed by rows (i, j <= i) at i(i+1)/2 + j; factored in place (L over M: each
    // entry is read once, before its own L value is written, so the values and their order are unchanged)
    double* L = Ml;
    double inv[6];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double s = Ml[j * (j + 1) / 2 + j];
#pragma unroll
        for (int k = 0; k < j; k++) s = fma(-L[j * (j + 1) / 2 + k], L[j * (j + 1) / 2 + k], s);
        ok = ok && (s > 0.0);
        inv[j] = rsqrt_nr<2>(s);
        L[j * (j + 1) / 2 + j] = s * inv[j];
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double v = Ml[i * (i + 1) / 2 + j];
#pragma unroll
            for (int k = 0; k < j; k++) v = fma(-L[i * (i + 1) / 2 + k], L[j * (j + 1) / 2 + k], v);
            L[i * (i + 1) / 2 + j] = v * inv[j];
        }
    }
    double z[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double v = rhs[i];
#pragma unroll
        for (int k = 0; k < i; k++) v = fma(-L[i * (i + 1) / 2 + k], z[k], v);
        z[i] = v * inv[i];
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double v = z[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) v = fma(-L[k * (k + 1) / 2 + i], y[k], v);
        y[i] = v * inv[i];
    }
#pragma unroll
    for (int i = 0; i < 6; i++) ok = ok && isfinite(y[i]);
    *okp = ok;
}
// The next step from the state in registers (A, g: the current normal equations; the caller passes them
// from where they already are, so an accepted pass's records never round-trip through the LDS state):
// 1 / radius instead of radius (ceres' radius / x and x / radius become products: no fp64 division on
// this serial path; a division is ~200 cycles on one lane, micro/lm_tail_bench.py).
__device__ __forceinline__ void lm_next_step_fast(LMState* st, aloam_lm_summary* out, int max_iter, const double* A, const double* g,
                                                  double inv_radius, double decrease, int reuse, int iteration) {
    double sc[6], x[7], dg[6];
#pragma unroll
    for (int i = 0; i < 6; i++) { sc[i] = st->scale[i]; dg[i] = st->diag[i]; }
#pragma unroll
    for (int i = 0; i < 7; i++) x[i] = st->x[i];
    while (true) {
        if (iteration >= max_iter) {
            st->inv_radius = inv_radius; st->decrease_factor = decrease; st->reuse_diag = reuse; st->iteration = iteration;
            lm_finish(st, out, 0);
            return;
        }
        iteration++;
        double M[21], gs[6];
#pragma unroll
        for (int a = 0; a < 6; a++) {
            gs[a] = sc[a] * g[a];
#pragma unroll
            for (int b = 0; b <= a; b++) M[a * (a + 1) / 2 + b] = sc[b] * Aget(A, b, a) * sc[a];
        }
        if (!reuse)
#pragma unroll
            for (int a = 0; a < 6; a++) dg[a] = fmin(fmax(M[a * (a + 1) / 2 + a], 1e-6), 1e32);
#pragma unroll
        for (int a = 0; a < 6; a++) M[a * (a + 1) / 2 + a] += dg[a] * inv_radius;   // D^2 = diag / radius
        double y[6];
        bool ok;
        chol_solve6_packed(M, gs, y, &ok);
        reuse = 1;
        if (!ok) {                         // invalid step: StepIsInvalid() == StepRejected(0)
            inv_radius *= decrease;        // radius / decrease_factor
            decrease *= 2.0;
            continue;
        }
        double delta[6];
#pragma unroll
        for (int a = 0; a < 6; a++) delta[a] = -y[a] * sc[a];
        double cand[7];
        plus7(x, delta, cand);
#pragma unroll
        for (int i = 0; i < 7; i++) st->cand[i] = cand[i];
#pragma unroll
        for (int a = 0; a < 6; a++) { st->delta[a] = delta[a]; st->diag[a] = dg[a]; }
        st->inv_radius = inv_radius; st->decrease_factor = decrease; st->reuse_diag = reuse; st->iteration = iteration;
        st->pending = 1;
        return;
    }
}
// off the critical path (another wave, during the next pass's exchange): model cost change of the last
// step from the unscaled normal equations (mcc = -(g.d + d'Ad/2), d = the tangent step), its reciprocal
// (the gain ratio is then a product), its norm in the ambient space, and the norm of x
__device__ __forceinline__ void lm_post(LMState* st) {
    if (!st->pending || st->done) return;
    double d[6], x[7], c[7];
#pragma unroll
    for (int a = 0; a < 6; a++) d[a] = st->delta[a];
#pragma unroll
    for (int i = 0; i < 7; i++) { x[i] = st->x[i]; c[i] = st->cand[i]; }
    double sg = 0, sAs = 0;
#pragma unroll
    for (int a = 0; a < 6; a++) {
        sg = fma(d[a], st->g[a], sg);
        double t = 0;
#pragma unroll
        for (int b = 0; b < 6; b++) t = fma(Aget(st->A, a, b), d[b], t);
        sAs = fma(d[a], t, sAs);
    }
    const double mcc = -(sg + 0.5 * sAs);
    double dx[7];
#pragma unroll
    for (int i = 0; i < 7; i++) dx[i] = x[i] - c[i];
    st->mcc = mcc;
    st->inv_mcc = 1.0 / mcc;
    st->invalid = mcc < 0.0;
    st->step_norm = norm7(dx);
    st->x_norm = norm7(x);
    st->pending = 0;
}
__device__ __forceinline__ void lm_tail_fast(LMState* st, const double* tot, int pass, double* xp, aloam_lm_summary* out, int max_iter) {
#ifdef ALOAM_LM_TAIL_REGS
    double A[21], g[6];
#pragma unroll
    for (int i = 0; i < 21; i++) A[i] = tot[i];
#pragma unroll
    for (int i = 0; i < 6; i++) g[i] = tot[21 + i];
#else
    // the normal equations read where they are (LDS) rather than held in 54 registers across the tail: the
    // same values, fewer spills (k_lm_coop runs at the 256-VGPR limit)
    const double* A = tot;
    const double* g = tot + 21;
#endif
    const double new_cost = tot[27];
    if (pass == 0) {
        #pragma unroll
        for (int i = 0; i < 7; i++) st->x[i] = xp[i];
        st->nres = (int)tot[28];
        st->iteration = 0; st->successful = 0; st->done = 0; st->pending = 0; st->invalid = 0;
        st->cost = new_cost; st->initial_cost = new_cost;
        if (st->nres == 0) { st->cost = 0; lm_finish(st, out, 4); return; }
        #pragma unroll
        for (int i = 0; i < 21; i++) st->A[i] = A[i];
        #pragma unroll
        for (int i = 0; i < 6; i++) st->g[i] = g[i];
        #pragma unroll
        for (int a = 0; a < 6; a++) st->scale[a] = 1.0 / (1.0 + sqrt(Aget(A, a, a)));
        st->decrease_factor = 2.0; st->reuse_diag = 0;
        if (grad_max_norm(st->x, g) <= 1e-10) { st->inv_radius = 1e-4; lm_finish(st, out, 3); return; }
        lm_next_step_fast(st, out, max_iter, A, g, 1e-4, 2.0, 0, 0);   // initial radius 1e4
        return;
    }
    // the state this pass needs, loaded together (independent LDS reads)
    const int invalid = st->invalid, iteration = st->iteration;
    const double inv_radius = st->inv_radius, decrease = st->decrease_factor, cost = st->cost;
    const double step_norm = st->step_norm, x_norm = st->x_norm, inv_mcc = st->inv_mcc;
    if (invalid) {                         // the step evaluated in this pass was invalid: not a candidate
        st->invalid = 0;
        lm_next_step_fast(st, out, max_iter, st->A, st->g, inv_radius * decrease, 2.0 * decrease, 1, iteration);
        return;
    }
    if (step_norm <= 1e-8 * (x_norm + 1e-8)) { lm_finish(st, out, 2); return; }
    const double cost_change = cost - new_cost;
    if (fabs(cost_change) <= 1e-6 * cost) { lm_finish(st, out, 1); return; }
    const double rel = cost_change * inv_mcc;
    if (rel > 1e-3) {
        double x[7];
        #pragma unroll
        for (int i = 0; i < 7; i++) { x[i] = st->cand[i]; st->x[i] = x[i]; xp[i] = x[i]; }
        #pragma unroll
        for (int i = 0; i < 21; i++) st->A[i] = A[i];
        #pragma unroll
        for (int i = 0; i < 6; i++) st->g[i] = g[i];
        st->cost = new_cost;
        st->successful++;
        const double t = 2.0 * rel - 1.0;
        // radius = min(1e16, radius / max(1/3, 1 - t^3)) in reciprocal form
        const double ir = fmax(1e-16, inv_radius * fmax(1.0 / 3.0, 1.0 - t * t * t));
        if (grad_max_norm(x, g) <= 1e-10) { st->inv_radius = ir; st->decrease_factor = 2.0; st->reuse_diag = 0; lm_finish(st, out, 3); return; }
        lm_next_step_fast(st, out, max_iter, A, g, ir, 2.0, 0, iteration);
    } else {
        lm_next_step_fast(st, out, max_iter, st->A, st->g, inv_radius * decrease, 2.0 * decrease, 1, iteration);
    }
}

#ifdef ALOAM_LM_TAIL_NOINLINE   // A/B build: the tail with a register allocation of its own
__device__ __noinline__ void lm_tail_call(LMState* st, const double* tot, int pass, double* xp, aloam_lm_summary* out, int max_iter) {
    lm_tail_fast(st, tot, pass, xp, out, max_iter);
}
#else
__device__ __forceinline__ void lm_tail_call(LMState* st, const double* tot, int pass, double* xp, aloam_lm_summary* out, int max_iter) {
    lm_tail_fast(st, tot, pass, xp, out, max_iter);
}
#endif
// The same tail on a register copy of the state (one LDS read/write burst instead of dependent LDS
// round trips inside the step computation).
__device__ __forceinline__ void lm_tail_reg(LMState* st, const double* tot, int pass, double* xp, aloam_lm_summary* out, int max_iter) {
    LMState L = *st;
    lm_tail(&L, tot, pass, xp, out, max_iter);
    *st = L;
}

// Sum of NACC doubles over `nrows` rows of an LDS table rows[r*NACC + i] into tot[] (fixed order =>
// deterministic): 8 x NACC threads each add every 8th row of one column, then NACC threads add the
// 8 partials. Independent LDS loads, no shuffle dependency chains (the 29 chained wave reductions
// this replaces cost ~6 us per pass).
__device__ __forceinline__ void reduce_rows(const double* rows, int nrows, double* part8, double* tot) {
    const int j = threadIdx.x;
    if (j < 8 * NACC) {
        const int i = j % NACC, c = j / NACC;
        double s0 = 0, s1 = 0;
        int r = c;
        for (; r + 8 < nrows; r += 16) { s0 += rows[r * NACC + i]; s1 += rows[(r + 8) * NACC + i]; }
        if (r < nrows) s0 += rows[r * NACC + i];
        part8[c * NACC + i] = s0 + s1;
    }
    __syncthreads();
    if (j < NACC) {
        double s = 0;
#pragma unroll
        for (int c = 0; c < 8; c++) s += part8[c * NACC + j];
        tot[j] = s;
    }
    __syncthreads();
}
// v[l] + v[l ^ 32] + v[l ^ 16] + v[l ^ 48] in every lane l, via the gfx950 cross-row lane swaps
// (no LDS, no dependent shuffles): same summation order in every lane, so the result is deterministic.
__device__ __forceinline__ double quad_row_sum(double v) {
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const double h = __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
    const unsigned lo2 = (unsigned)__double2loint(h), hi2 = (unsigned)__double2hiint(h);
    const auto c = __builtin_amdgcn_permlane16_swap(lo2, lo2, false, false);
    const auto d = __builtin_amdgcn_permlane16_swap(hi2, hi2, false, false);
    return __hiloint2double((int)d[0], (int)c[0]) + __hiloint2double((int)d[1], (int)c[1]);
}
// block-wide sum of NACC doubles per thread (NT >= 8 * NACC threads): each wave first folds its 64
// lanes to 16 with lane swaps, so only NT/4 rows go through LDS (rows = NT/4 * NACC doubles)
template <int NT>
__device__ __forceinline__ void block_reduce_acc(const double* acc, double* rows, double* part8, double* tot) {
    static_assert(NT >= 8 * NACC, "reduce_rows needs 8*NACC threads");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NACC; i++) {
        const double v = quad_row_sum(acc[i]);
        if (lane < 16) rows[(wave * 16 + lane) * NACC + i] = v;
    }
    __syncthreads();
    reduce_rows(rows, NT / 4, part8, tot);
}

constexpr int LM_REC = 32;   // u64 per record of the persistent solver's exchange (NACC partials + check word)

// ---- k_lm_coop's per-pass reduction and exchange ---------------------------------------------------
// Wave sum of NACC (<= 32) doubles by transposition: five halving steps, each exchanging half of the
// lane's remaining values with a partner lane and adding the other half (partners l^32 and l^16 by
// the gfx950 lane swaps, then l^15, l^7, l^2 within rows by DPP), so every step moves half as much as
// the last; a final l^1 add leaves lane l with the wave sum of value (l >> 1) & 31. The masks
// {32, 16, 15, 7, 2, 1} span all 64 lanes, so each lane's result sums all of them, in a fixed order.
__device__ __forceinline__ double dpp_f64(double v, int ctrl_sel) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    int l2, h2;
    switch (ctrl_sel) {   // the DPP control must be a constant
        case 0: l2 = __builtin_amdgcn_mov_dpp(lo, 0x140, 0xf, 0xf, false); h2 = __builtin_amdgcn_mov_dpp(hi, 0x140, 0xf, 0xf, false); break;   // row_mirror: l^15
        case 1: l2 = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xf, 0xf, false); h2 = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xf, 0xf, false); break;   // row_half_mirror: l^7
        case 2: l2 = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xf, 0xf, false); h2 = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xf, 0xf, false); break;    // quad_perm [2,3,0,1]: l^2
        default: l2 = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xf, 0xf, false); h2 = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xf, 0xf, false); break;   // quad_perm [1,0,3,2]: l^1
    }
    return __hiloint2double(h2, l2);
}
// the partner's `v` (partner lane l^32, or l^16 with ROW16): the gfx950 lane swap of a register with
// itself leaves this lane's value and the partner's in its two results; which one is the partner's is
// read from the bits (where the two are equal, either is)
template <bool ROW16>
__device__ __forceinline__ double lane_xchg(double v) {
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto a = ROW16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false) : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = ROW16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false) : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const unsigned pl = (unsigned)a[0] == lo ? (unsigned)a[1] : (unsigned)a[0];
    const unsigned ph = (unsigned)b[0] == hi ? (unsigned)b[1] : (unsigned)b[0];
    return __hiloint2double((int)ph, (int)pl);
}
__device__ __forceinline__ double wave_transpose_sum(const double* acc) {
    double v[32];
#pragma unroll
    for (int j = 0; j < 32; j++) v[j] = j < NACC ? acc[j] : 0.0;
    const int lane = threadIdx.x & 63;
    const bool b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1;
#pragma unroll
    for (int j = 0; j < 16; j++) {                                          // bit 5: partner l^32
        const double send = b5 ? v[j] : v[j + 16], keep = b5 ? v[j + 16] : v[j];
        v[j] = keep + lane_xchg<false>(send);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {                                           // bit 4: partner l^16
        const double send = b4 ? v[j] : v[j + 8], keep = b4 ? v[j + 8] : v[j];
        v[j] = keep + lane_xchg<true>(send);
    }
#pragma unroll
    for (int s = 0; s < 3; s++) {                                           // bits 3, 2, 1: partners l^15, l^7, l^2
        const int half = 4 >> s;
        const bool hi = (lane >> (3 - s)) & 1;
#pragma unroll
        for (int j = 0; j < half; j++) {
            const double send = hi ? v[j] : v[j + half], keep = hi ? v[j + half] : v[j];
            v[j] = keep + dpp_f64(send, s);
        }
    }
    return v[0] + dpp_f64(v[0], 3);
}
// splitmix64 finaliser: record words carry a keyed hash so a reader can tell a complete current record
// from a stale or partly written one without a separate tag (no store ordering to wait for)
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long word_key(unsigned long long w, int i, unsigned long long epoch) {
    return mix64(w ^ (epoch * 0x9e3779b97f4a7c15ull) ^ ((unsigned long long)(i + 1) * 0xd1b54a32d192ed03ull));
}
__device__ __forceinline__ unsigned long long xor32_lanes(unsigned long long v) {   // XOR over each aligned 32-lane half
    auto step = [](unsigned long long x, int sel) {
        const double d = __longlong_as_double((long long)x);
        return x ^ (unsigned long long)__double_as_longlong(dpp_f64(d, sel));
    };
    {
        const unsigned l = (unsigned)v, h = (unsigned)(v >> 32);
        const auto a = __builtin_amdgcn_permlane16_swap(l, l, false, false);
        const auto b = __builtin_amdgcn_permlane16_swap(h, h, false, false);
        v = ((unsigned long long)b[0] << 32 | a[0]) ^ ((unsigned long long)b[1] << 32 | a[1]);   // l ^ (l^16)
    }
    v = step(v, 0);   // l^15
    v = step(v, 1);   // l^7
    v = step(v, 2);   // l^2
    return step(v, 3);   // l^1
}
// Workgroup partial -> record (tot[0..NACC) in wsum[0..NACC) after the wave sums), then the all-gather
// of the G records into rows[b * NACC + i]. Record b = NACC words (the doubles' bits) + one check word
// (XOR of the words' keyed hashes); readers load every record with a 32-lane half each and accept it
// when the hashes of what they read XOR to zero. A stale record (another epoch) or one whose stores
// are still landing fails the check (up to 2^-64). Stores and loads are agent-scope relaxed atomics
// (64-bit single-copy atomic, coherent across XCDs); no fence, no completion wait before a tag.
constexpr int LM_COOP_MAX_RECS = 64;    // records per pass buffer = k_lm_coop's workgroup cap (128 measured slower in round 2)
__device__ __forceinline__ void publish_record(unsigned long long* buf, unsigned long long epoch, double v) {
    const int lane = threadIdx.x & 63;   // wave 0 only; lane i < NACC holds partial i
    const unsigned long long w = lane < NACC ? (unsigned long long)__double_as_longlong(v) : 0ull;
    const unsigned long long chk = xor32_lanes(lane < NACC ? word_key(w, lane, epoch) : 0ull);
    unsigned long long* mine = buf + (size_t)blockIdx.x * LM_REC;
    if (lane < NACC) __hip_atomic_store(&mine[lane], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (lane == NACC) __hip_atomic_store(&mine[lane], chk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int NT>
__device__ __forceinline__ bool gather_records(const unsigned long long* buf, unsigned long long epoch, double* rows, unsigned G, int* err) {
    constexpr int HALVES = NT / 32, MAXK = (LM_COOP_MAX_RECS + HALVES - 1) / HALVES;
    const int lane32 = threadIdx.x & 31, half = threadIdx.x >> 5;
    const int K = ((int)G + HALVES - 1) / HALVES;   // block-uniform
    int spins = 0;
    while (true) {
        unsigned long long w[MAXK];
#pragma unroll
        for (int k = 0; k < MAXK; k++) {
            const int b = half + k * HALVES;
            w[k] = (k < K && b < (int)G && lane32 <= NACC)
                       ? __hip_atomic_load(&buf[(size_t)b * LM_REC + lane32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        }
        bool bad = false;
#pragma unroll
        for (int k = 0; k < MAXK; k++) {
            if (k >= K) continue;   // block-uniform
            const bool rec = half + k * HALVES < (int)G;
            const unsigned long long h = !rec ? 0ull : lane32 < NACC ? word_key(w[k], lane32, epoch) : (lane32 == NACC ? w[k] : 0ull);
            bad |= xor32_lanes(h) != 0ull;
        }
        if (!__syncthreads_or(bad)) {
#pragma unroll
            for (int k = 0; k < MAXK; k++) {
                const int b = half + k * HALVES;
                if (k < K && b < (int)G && lane32 < NACC) rows[b * NACC + lane32] = __longlong_as_double((long long)w[k]);
            }
            __syncthreads();
            return true;
        }
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 20)) {   // uniform: every thread counts the same votes
            if (threadIdx.x == 0) atomicExch(err, 1);
            return false;
        }
    }
}

// Whole Solve as ONE persistent launch over G workgroups: each pass evaluates its slice, publishes
// a 29-double partial, meets the others at a grid barrier, then EVERY workgroup reduces the G
// partials in the same fixed order and runs the identical LM tail on its own LDS copy of the state
// (bitwise-identical on all workgroups, so no broadcast and one barrier per pass).
constexpr int CB = 256;
constexpr int LM_COOP_MAX = LM_COOP_MAX_RECS;      // records per pass buffer
constexpr int LM_CACHE = 1024;                      // factor slots per workgroup kept in LDS (80 KB)
#ifdef ALOAM_LM_TIMING
__device__ unsigned long long g_lm_ts[8][5];   // micro-benchmark only: block-0 phase stamps per pass
// (ALOAM_LM_TIMING = the solve index stamped: lm_run flags that launch in max_iter's bit 16)
#define LM_TS(p, k) do { if (lm_stamp && blockIdx.x == 0 && threadIdx.x == 0 && (p) < 8) g_lm_ts[p][k] = wall_clock64(); } while (0)
__device__ unsigned long long g_lm_ts_edge[2];   // kernel entry / exit of block 0
#define LM_TS_EDGE(k) do { if (lm_stamp && blockIdx.x == 0 && threadIdx.x == 0) g_lm_ts_edge[k] = wall_clock64(); } while (0)
extern "C" int aloam_dbg_lm_ts(unsigned long long* out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lm_ts), sizeof(g_lm_ts));
    if (e == hipSuccess) e = hipMemcpyFromSymbol(out + 40, HIP_SYMBOL(g_lm_ts_edge), sizeof(g_lm_ts_edge));
    return (int)e;
}
#else
#define LM_TS(p, k) do { } while (0)
#define LM_TS_EDGE(k) do { } while (0)
#endif
__global__ void __launch_bounds__(CB) k_lm_coop(const aloam_factor* __restrict__ f, int nslots, double* xp, LMState* st,
                                                unsigned long long* recs, unsigned long long* seq, int* err, aloam_lm_summary* out,
                                                int max_iter, const int* gate, const int* dn, int cache_cap) {
    __shared__ double rows[(CB / 4 > LM_COOP_MAX ? CB / 4 : LM_COOP_MAX) * NACC];   // wave-folded rows, then the G records
    __shared__ double part8[8 * NACC];
    __shared__ double tot[NACC];
    __shared__ double wsum[CB / WAVE * NACC];
    __shared__ double xl[7];
    __shared__ int done;
    __shared__ LMState ls;
    extern __shared__ aloam_factor fcache[];        // this workgroup's contiguous slice of factor slots
#ifdef ALOAM_LM_TIMING
    const bool lm_stamp = (max_iter >> 16) & 1;
    max_iter &= 0xffff;
#endif
    LM_TS_EDGE(0);
    if (gate && *gate == 0) return;                 // mapping skipped (laserMapping.cpp:554)
    if (dn) nslots = min(nslots, dn[0] + dn[1]);    // live slot count known on the device only
    const unsigned G = gridDim.x;
    const int per = (nslots + G - 1) / G;
    const int f0 = blockIdx.x * per, f1 = min(nslots, f0 + per);
    const bool cached = per <= cache_cap;           // slots read from HBM once, then from LDS
    __shared__ unsigned long long ep;
    if (threadIdx.x < 7) xl[threadIdx.x] = xp[threadIdx.x];
    if (threadIdx.x == 0) ep = __hip_atomic_load(seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 256 + 1;
    __syncthreads();
    const unsigned long long epoch0 = ep;
    for (int pass = 0; pass <= max_iter; pass++) {
        const double* xs = pass == 0 ? xl : ls.cand;
        const dquat q{xs[0], xs[1], xs[2], xs[3]};
        const double t[3] = {xs[4], xs[5], xs[6]};
        double acc[NACC];
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = 0;
        if (!cached) {
            for (int i = f0 + threadIdx.x; i < f1; i += CB) accumulate(f[i], q, t, acc);
        } else if (pass == 0) {
            for (int i = f0 + threadIdx.x; i < f1; i += CB) { const aloam_factor fi = f[i]; fcache[i - f0] = fi; accumulate(fi, q, t, acc); }
        } else {
            for (int i = threadIdx.x; i < f1 - f0; i += CB) accumulate(fcache[i], q, t, acc);
        }
        LM_TS(pass, 4);
        {   // wave sums -> LDS; wave 0 adds the waves' sums in wave order and publishes the record
            const double s = wave_transpose_sum(acc);
            const int lane = threadIdx.x & 63;
            if (!(lane & 1) && (lane >> 1) < NACC) wsum[(threadIdx.x >> 6) * NACC + (lane >> 1)] = s;
        }
        __syncthreads();
        unsigned long long* rbuf = recs + (size_t)(pass & 1) * LM_COOP_MAX * LM_REC;
        if (threadIdx.x < WAVE) {
            double v = 0;
            if (threadIdx.x < NACC) {
                v = wsum[threadIdx.x];
#pragma unroll
                for (int w = 1; w < CB / WAVE; w++) v += wsum[w * NACC + threadIdx.x];
            }
            publish_record(rbuf, epoch0 + pass, v);
        }
        LM_TS(pass, 0);
        if (pass > 0 && threadIdx.x == WAVE) lm_post(&ls);   // wave 1, while the records travel
        if (!gather_records<CB>(rbuf, epoch0 + pass, rows, G, err)) return;
        LM_TS(pass, 1);
        reduce_rows(rows, G, part8, tot);
        LM_TS(pass, 2);
        if (threadIdx.x == 0) {
            lm_tail_call(&ls, tot, pass, xl, blockIdx.x == 0 ? out : nullptr, max_iter);
            done = ls.done;
        }
        __syncthreads();
        LM_TS(pass, 3);
        if (done) break;
    }
    if (blockIdx.x == 0) {
        // every workgroup has read seq (it published a pass-0 record before workgroup 0 got here)
        if (threadIdx.x == 0) __hip_atomic_store(seq, epoch0 / 256 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x < 7) xp[threadIdx.x] = xl[threadIdx.x];
        const int nw = sizeof(LMState) / 8;
        for (int i = threadIdx.x; i < nw; i += CB) ((unsigned long long*)st)[i] = ((const unsigned long long*)&ls)[i];
        LM_TS_EDGE(1);
    }
}

void lm_init(Ctx& C) {
    (void)C;   // static rows (59 KB) + up to 80 KB of cached slots: above the default dynamic limit
    HIPCHK(hipFuncSetAttribute((const void*)k_lm_coop, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(aloam_factor) * LM_CACHE)));
}

// one Ceres Solve over nslots factor slots; `gate` (device int, may be null) disables the solve.
void lm_run(Ctx& C, const aloam_factor* d_f, int nslots, double* d_x, int round, const int* gate, const int* d_nslots2,
            int live_hint) {
    aloam_lm_summary* out = C.d_lm_sum + round;
    // Grid size from the expected live slot count (the current scan's count for odometry, last frame's
    // stack sizes for mapping, whose live count is only known on the device; a captured round graph
    // keeps the G of the scan it was captured on, since its key has no size): ~1 slot per thread keeps the
    // evaluation short (fp64 latency-bound), capped so the per-pass grid barrier stays cheap.
    // Correctness never depends on G: the kernel splits the device-side count over the grid.
    const int est = std::max(1, std::min(nslots, live_hint > 0 ? live_hint + live_hint / 4 : nslots));
    static const int spt = getenv("ALOAM_LM_SPT") ? std::max(1, atoi(getenv("ALOAM_LM_SPT"))) : 1;   // tuning knob
    int G = std::max((est + spt * CB - 1) / (spt * CB), (est + LM_CACHE - 1) / LM_CACHE);
    // tuning knob: workgroup cap (C3 pipeline, mapping solves of ~100 workgroups' worth of slots: 64 ->
    // 1393 scans/s, 128 -> 1366; fewer slots per workgroup cost more exchange than they save)
    static const int gmax = getenv("ALOAM_LM_GMAX") ? std::max(1, std::min(LM_COOP_MAX, atoi(getenv("ALOAM_LM_GMAX")))) : 64;
    G = std::max(1, std::min(std::min(gmax, C.n_cus), G));   // every workgroup must be co-resident (<= 1 per CU)
    const int cap = std::min(LM_CACHE, (nslots + G - 1) / G);          // LDS slots per workgroup
    const size_t lds = sizeof(aloam_factor) * (size_t)cap;
    int mi = std::min(C.P.max_solver_iterations, 200);
#ifdef ALOAM_LM_TIMING
    if (round == ALOAM_LM_TIMING) mi |= 1 << 16;
#endif
    k_lm_coop<<<G, CB, lds, C.stream>>>(d_f, nslots, d_x, C.d_lm, C.d_lm_recs, C.d_lm_seq, C.d_bar_err, out, mi, gate, d_nslots2, cap);
    HIPCHK(hipGetLastError());
}

// ---- scan-to-map registration across ranks (aloam_s2m_*) ----------------------------
// A Solve is max_iter + 1 pass launches, each followed by the record exchange, then one final launch.
// The slots are cut into nrec fixed blocks of `per` slots; a rank's pass launch covers its run of
// blocks, one workgroup per block, and writes one S2M_REC-double record per block (the block's 29
// normal-equation sums in the fixed block_reduce_acc order + its corner / surf correspondence
// counts). Pass p > 0 first finishes pass p-1 in EVERY workgroup: it reduces the nrec exchanged
// records in block order (fixed-order reduce_rows) and runs the LM tail on its LDS copy of the state
// (bitwise-identical in every workgroup and on every rank, whatever the world size), workgroup 0
// publishing the new state into the other half of a double-buffered LMState; then it evaluates its
// block at the new candidate. k_s2m_final runs the last tail and writes the parameters.
// A pass after termination is a no-op on every rank.
constexpr int S2M_REC = 32;
static_assert(ALOAM_S2M_RECORDS <= CB, "one record per thread in the record reduction");

// records of the previous pass -> tot (every workgroup, fixed order): thread t loads record t (all 29
// sums in flight at once), then the same fixed-order block reduction as a pass's own partials
__device__ __forceinline__ void s2m_reduce_records(const double* __restrict__ recs, int nrec, double* rows, double* part8, double* tot) {
    double acc[NACC];
    const int t = threadIdx.x;
    if (t < nrec) {
        const double2* r2 = (const double2*)(recs + (size_t)t * S2M_REC);   // records are 256-B aligned
        double2 v[(NACC + 1) / 2];
#pragma unroll
        for (int i = 0; i < (NACC + 1) / 2; i++) v[i] = r2[i];
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = (i & 1) ? v[i / 2].y : v[i / 2].x;
    } else {
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = 0.0;
    }
    block_reduce_acc<CB>(acc, rows, part8, tot);
}

// the same for records handed over inside one launch (k_s2m_solve): every load an agent-scope (sc1) 8-byte load,
// the hand-off form of MI355X_MICROARCH.md's sc1 table (sc1 stores, each storing wave drained before the arrival)
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void s2m_reduce_records_sc1(const double* __restrict__ recs, int nrec, double* rows, double* part8, double* tot) {
    double acc[NACC];
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = t < nrec ? ld_sc1(recs + (size_t)t * S2M_REC + i) : 0.0;
    block_reduce_acc<CB>(acc, rows, part8, tot);
}

__global__ void __launch_bounds__(CB) k_s2m_pass(const aloam_factor* __restrict__ f, int nslots, int per, int rec0, int nrec,
                                                 const double* __restrict__ prev, const LMState* __restrict__ st_in,
                                                 LMState* __restrict__ st_out, const double* __restrict__ x0, int pass,
                                                 aloam_lm_summary* sum, int max_iter, int* round_cnt, double* __restrict__ send) {
    __shared__ double rows[CB / 4 * NACC];
    __shared__ double part8[8 * NACC];
    __shared__ double tot[NACC];
    __shared__ LMState ls;
    __shared__ double xl[7];
    __shared__ int cnt[2];
    double* rec = send + (size_t)blockIdx.x * S2M_REC;
    if (pass > 1 && st_in->done) {               // the Solve ended before the previous pass: nothing to reduce or
        if (threadIdx.x < S2M_REC) rec[threadIdx.x] = 0.0;   // evaluate; the state carried to the next buffer
        if (blockIdx.x == 0 && threadIdx.x == 0) *st_out = *st_in;
        return;
    }
    if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    if (pass > 0) {
        if (threadIdx.x == 0) ls = *st_in;
        s2m_reduce_records(prev, nrec, rows, part8, tot);
        if (pass == 1 && blockIdx.x == 0 && round_cnt) {          // correspondences of this round (pass-0 records)
            int a = 0, b = 0;
            for (int r = threadIdx.x; r < nrec; r += CB) { a += (int)prev[(size_t)r * S2M_REC + NACC]; b += (int)prev[(size_t)r * S2M_REC + NACC + 1]; }
            a = wave_sum_i(a);
            b = wave_sum_i(b);
            if ((threadIdx.x & 63) == 0) { atomicAdd(&cnt[0], a); atomicAdd(&cnt[1], b); }
        }
        if (threadIdx.x == 0) {
            if (pass == 1 || !ls.done) {
                const double* xs = pass == 1 ? x0 : ls.x;
                for (int i = 0; i < 7; i++) xl[i] = xs[i];
                lm_tail_reg(&ls, tot, pass - 1, xl, blockIdx.x == 0 ? sum : nullptr, max_iter);
            }
        }
        __syncthreads();
        if (blockIdx.x == 0) {
            if (threadIdx.x == 0) *st_out = ls;
            if (pass == 1 && round_cnt && threadIdx.x < 2) round_cnt[threadIdx.x] = cnt[threadIdx.x];
        }
        __syncthreads();
        if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    }
    const int g = rec0 + blockIdx.x;
    if ((pass > 0 && ls.done) || g >= nrec) {                    // uniform: the same state everywhere
        if (threadIdx.x < S2M_REC) rec[threadIdx.x] = 0.0;
        return;
    }
    const double* xs = pass == 0 ? x0 : ls.cand;
    const dquat q{xs[0], xs[1], xs[2], xs[3]};
    const double t[3] = {xs[4], xs[5], xs[6]};
    double acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = 0;
    int ne = 0, np = 0;
    const int f0 = g * per, f1 = min(nslots, f0 + per);
    for (int i = f0 + threadIdx.x; i < f1; i += CB) {
        const aloam_factor fi = f[i];
        ne += fi.type == 0;
        np += fi.type == 1 || fi.type == 2;
        accumulate(fi, q, t, acc);
    }
    __syncthreads();
    if (pass == 0) {
        const int se = wave_sum_i(ne), sp = wave_sum_i(np);
        if ((threadIdx.x & 63) == 0 && (se | sp)) { atomicAdd(&cnt[0], se); atomicAdd(&cnt[1], sp); }
    }
    block_reduce_acc<CB>(acc, rows, part8, tot);
    if (threadIdx.x < NACC) rec[threadIdx.x] = tot[threadIdx.x];
    if (threadIdx.x == 0) { rec[NACC] = cnt[0]; rec[NACC + 1] = cnt[1]; rec[NACC + 2] = 0.0; }
}

// the tail of the last pass (one workgroup): parameters -> x
__global__ void __launch_bounds__(CB) k_s2m_final(const double* __restrict__ prev, int nrec, const LMState* __restrict__ st_in,
                                                  double* x, int last_pass, aloam_lm_summary* sum, int max_iter) {
    __shared__ double rows[CB / 4 * NACC];
    __shared__ double part8[8 * NACC];
    __shared__ double tot[NACC];
    __shared__ LMState ls;
    __shared__ double xl[7];
    if (last_pass > 0 && st_in->done) {          // ended earlier: the parameters are the state's
        if (threadIdx.x < 7) x[threadIdx.x] = st_in->x[threadIdx.x];
        return;
    }
    if (threadIdx.x == 0) ls = *st_in;
    s2m_reduce_records(prev, nrec, rows, part8, tot);
    if (threadIdx.x == 0) {
        if (last_pass == 0 || !ls.done) {
            const double* xs = last_pass == 0 ? x : ls.x;
            for (int i = 0; i < 7; i++) xl[i] = xs[i];
            lm_tail_reg(&ls, tot, last_pass, xl, sum, max_iter);
        }
        for (int i = 0; i < 7; i++) x[i] = ls.x[i];
    }
}

// One Solve of the sharded registration as ONE launch per rank: the same records, reductions and tails as
// the max_iter + 1 pass launches and the final launch above, bit for bit (k_s2m_pass's block record code
// and k_s2m_final's tail). G co-resident workgroups compute this rank's block records of a pass (workgroup
// w: blocks rec0 + w, rec0 + w + G, ...) into the double-buffered record array T.recs. At world > 1 each
// record also goes to the rank's exported array T.xrec[rank] (uncached memory other ranks map: IPC over
// xGMI, or direct pointers in group mode), every workgroup then announces the pass on its arrival counter
// (system scope), waits for every peer's arrivals of the same pass and copies its share of the peers'
// blocks into T.recs: the all-gather with no host and no collective library in between. A local barrier
// (agent-scope counters T.gath) closes the pass, then every workgroup reduces the nrec records in block
// order and runs the tail on its LDS copy of the state; a Solve that terminated stops in every workgroup,
// on every rank, at the same pass. All counters are monotonic: pass gp (= *T.base + pass, counted over the
// rank's Solves) is complete when counter c reads (gp + 1) x the workgroups on it, so nothing is zeroed
// between Solves and a straggling peer can never be mistaken for a finished one. Every rank runs the same
// G and the same passes, so the counts agree. A wait longer than ~2 s (a peer that never launched) sets
// *err and ends the Solve (results void).
__device__ __forceinline__ bool s2m_wait(const unsigned* const* ctr, int nranks, int skip, unsigned G, unsigned gp, bool sys, int* err,
                                         int code) {
    const int lane = threadIdx.x;                     // wave 0 only; lanes poll (rank, counter) pairs
    const unsigned long long t0 = wall_clock64();
    while (true) {
        bool late = false;
        for (int i = lane; i < nranks * S2M_BARS; i += WAVE) {
            const int r = i / S2M_BARS, c = i % S2M_BARS;
            if (r == skip) continue;
            const unsigned want = (G / S2M_BARS + ((unsigned)c < G % S2M_BARS ? 1u : 0u)) * (gp + 1u);
            const unsigned v = sys ? __hip_atomic_load(&ctr[r][c * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                   : __hip_atomic_load(&ctr[r][c * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            late |= (int)(v - want) < 0;
        }
        if (!__ballot(late)) break;
        __builtin_amdgcn_s_sleep(2);
        if (wall_clock64() - t0 > 200000000ull) {     // 100 MHz constant clock: 2 s
            if (lane == 0) atomicCAS(err, 0, code);   // the first wait that gave up
            return false;
        }
    }
    if (sys) __threadfence_system();   // the local hand-off needs none: its stores and loads are sc1
    return true;
}

__global__ void __launch_bounds__(CB) k_s2m_solve(const aloam_factor* __restrict__ f, int nslots, int per, int nrec,
                                                  const S2MPeers T, int* err, double* x, LMState* st_out,
                                                  aloam_lm_summary* sum, int max_iter, int* round_cnt) {
    __shared__ double rows[CB / 4 * NACC];
    __shared__ double part8[8 * NACC];
    __shared__ double tot[NACC];
    __shared__ LMState ls;
    __shared__ double xl[7], x0s[7];
    __shared__ int cnt[2];
    __shared__ int done, fail;
    const unsigned G = gridDim.x;
    const unsigned base = *T.base;                   // written by the previous Solve (stream order)
    const int g0 = T.rank * T.rp, g1 = min(nrec, g0 + T.rp);
    const bool xchg = T.world > 1;
    if (threadIdx.x < 7) x0s[threadIdx.x] = x[threadIdx.x];
    if (threadIdx.x == 0) { done = 0; fail = 0; }
    __syncthreads();
    int pass = 0;
    for (; pass <= max_iter; pass++) {
        const unsigned gp = base + (unsigned)pass;
        const double* xs = pass == 0 ? x0s : ls.cand;
        const dquat q{xs[0], xs[1], xs[2], xs[3]};
        const double t[3] = {xs[4], xs[5], xs[6]};
        const size_t half = (size_t)(gp & 1) * nrec * S2M_REC;
        double* rb = T.recs + half;
        for (int g = g0 + blockIdx.x; g < g1; g += G) {               // this workgroup's blocks (k_s2m_pass)
            if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
            __syncthreads();
            double acc[NACC];
#pragma unroll
            for (int i = 0; i < NACC; i++) acc[i] = 0;
            int ne = 0, np = 0;
            const int f0 = g * per, f1 = min(nslots, f0 + per);
            for (int i = f0 + threadIdx.x; i < f1; i += CB) {
                const aloam_factor fi = f[i];
                ne += fi.type == 0;
                np += fi.type == 1 || fi.type == 2;
                accumulate(fi, q, t, acc);
            }
            __syncthreads();
            if (pass == 0) {
                const int se = wave_sum_i(ne), sp = wave_sum_i(np);
                if ((threadIdx.x & 63) == 0 && (se | sp)) { atomicAdd(&cnt[0], se); atomicAdd(&cnt[1], sp); }
            }
            block_reduce_acc<CB>(acc, rows, part8, tot);
            const double v = threadIdx.x < NACC ? tot[threadIdx.x]
                           : threadIdx.x == NACC ? (double)cnt[0] : threadIdx.x == NACC + 1 ? (double)cnt[1] : 0.0;
            if (threadIdx.x < NACC + 3) {
                st_sc1(rb + (size_t)g * S2M_REC + threadIdx.x, v);
                if (xchg) T.xrec[T.rank][half + (size_t)g * S2M_REC + threadIdx.x] = v;
            }
        }
        __syncthreads();
        if (xchg) {
            // announce this workgroup's records of pass gp to the peers, wait for theirs, gather this
            // workgroup's share of the foreign blocks (g = w, w + G, ...; owner g / rp)
            if (threadIdx.x < WAVE) {
                if (threadIdx.x == 0) {
                    __threadfence_system();
                    __hip_atomic_fetch_add(&T.xarr[T.rank][(blockIdx.x % S2M_BARS) * 32], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                if (!s2m_wait(T.xarr, T.world, T.rank, G, gp, true, err, 0x40000000 | (T.rank << 24) | ((pass & 0xff) << 16) | (int)(gp & 0xffff))) fail = 1;
            }
            __syncthreads();
            if (fail) return;
            for (int g = blockIdx.x; g < nrec; g += G) {
                const int owner = g / T.rp;
                if (owner != T.rank && threadIdx.x < NACC + 3)
                    st_sc1(rb + (size_t)g * S2M_REC + threadIdx.x, T.xrec[owner][half + (size_t)g * S2M_REC + threadIdx.x]);
            }
            __syncthreads();
        }
        // local grid barrier: every record of this pass in T.recs. Arrivals spread over S2M_BARS counters
        // (workgroup w on counter w % S2M_BARS, one cache line each), polled by as many lanes of wave 0: one
        // counter for all 256 workgroups serialised their atomics (measured slower than the pass launches)
        if (threadIdx.x < WAVE) {
            if (threadIdx.x == 0) {
                // wave 0 made every record store of this workgroup (sc1): drained, then the arrival
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add(&T.gath[(blockIdx.x % S2M_BARS) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const unsigned* own = T.gath;
            if (!s2m_wait(&own, 1, -1, G, gp, false, err, 0x50000000 | (T.rank << 24) | ((pass & 0xff) << 16) | (int)(gp & 0xffff))) fail = 1;
        }
        __syncthreads();
        if (fail) return;
        s2m_reduce_records_sc1(rb, nrec, rows, part8, tot);
        if (pass == 0 && blockIdx.x == 0 && round_cnt) {              // this round's correspondences (pass-0 records)
            int a = 0, b = 0;
            for (int r = threadIdx.x; r < nrec; r += CB) {
                a += (int)ld_sc1(rb + (size_t)r * S2M_REC + NACC);
                b += (int)ld_sc1(rb + (size_t)r * S2M_REC + NACC + 1);
            }
            a = wave_sum_i(a);
            b = wave_sum_i(b);
            if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
            __syncthreads();
            if ((threadIdx.x & 63) == 0) { atomicAdd(&cnt[0], a); atomicAdd(&cnt[1], b); }
            __syncthreads();
            if (threadIdx.x < 2) round_cnt[threadIdx.x] = cnt[threadIdx.x];
        }
        if (threadIdx.x == 0) {
            const double* xsrc = pass == 0 ? x0s : ls.x;
            for (int i = 0; i < 7; i++) xl[i] = xsrc[i];
            lm_tail_reg(&ls, tot, pass, xl, blockIdx.x == 0 ? sum : nullptr, max_iter);
            done = ls.done;
        }
        __syncthreads();
        if (done) { pass++; break; }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int i = 0; i < 7; i++) x[i] = ls.x[i];
        *st_out = ls;
        *T.base = base + (unsigned)pass;             // passes run (every rank: the same)
    }
}

int s2m_solve_grid(Ctx& C, int world, int rp, bool group) {
    // every workgroup co-resident (<= 1 per CU, like k_lm_coop), each with rp / G blocks (one block each on
    // a full MI355X at world 1: the blocks' evaluations are the Solve's work, 64 workgroups x 4 blocks
    // measured slower). Group mode shares one GPU's CUs among the ranks, and a k_s2m_solve workgroup
    // holds a whole CU (465 VGPRs + AGPRs: one wave per SIMD): every launch's workgroups are dealt from the
    // same first CU over the 8 XCDs and then over each XCD's 4 shader arrays, so a rank gets a multiple of
    // 32 workgroups (the same number on every array). Measured: W x 85 (W = 3) and W x 48 / 40 (W = 5 / 6)
    // left a rank's last workgroups unplaced (30 per XCD, but 9-10 on one 8-CU array) until the timeout;
    // multiples of 32 ran at every W from 2 to 8.
    static const int gcap = getenv("ALOAM_S2M_SOLVE_G") ? std::max(1, atoi(getenv("ALOAM_S2M_SOLVE_G"))) : 256;
    const int share = group ? std::max(32, C.n_cus / std::max(world, 1) / 32 * 32) : C.n_cus;
    return std::max(1, std::min(std::min(gcap, share), rp));
}

void s2m_solve_launch(Ctx& C, int G, const aloam_factor* f, int nslots, int per, int nrec, const S2MPeers& T, double* x,
                      LMState* st_out, aloam_lm_summary* sum, int* round_cnt) {
    if (T.world < 1 || T.world > S2M_PEER_MAX || T.rank < 0 || T.rank >= T.world || T.rp < 1 || !T.recs || !T.gath || !T.base)
        throw ApiError{ALOAM_E_STATE, "s2m solve: bad exchange table"};
    k_s2m_solve<<<G, CB, 0, C.stream>>>(f, nslots, per, nrec, T, C.d_bar_err, x, st_out, sum,
                                        std::min(C.P.max_solver_iterations, 200), round_cnt);
    HIPCHK(hipGetLastError());
}

void s2m_pass_launch(Ctx& C, const aloam_factor* f, int nslots, int per, int rec0, int nrec_local, int nrec, const double* prev,
                     const LMState* st_in, LMState* st_out, const double* x0, int pass, aloam_lm_summary* sum, int* round_cnt,
                     double* send) {
    k_s2m_pass<<<nrec_local, CB, 0, C.stream>>>(f, nslots, per, rec0, nrec, prev, st_in, st_out, x0, pass, sum,
                                                std::min(C.P.max_solver_iterations, 200), round_cnt, send);
    HIPCHK(hipGetLastError());
}
void s2m_final_launch(Ctx& C, const double* prev, int nrec, const LMState* st_in, double* x, int last_pass, aloam_lm_summary* sum) {
    k_s2m_final<<<1, CB, 0, C.stream>>>(prev, nrec, st_in, x, last_pass, sum, std::min(C.P.max_solver_iterations, 200));
    HIPCHK(hipGetLastError());
}

// ---- test entry: per-factor residuals / Jacobians and the normal equations ----
__global__ void k_eval_factors(const aloam_factor* __restrict__ f, int n, const double* x, int robust, double* res,
                               double* jac, double* neq) {
    __shared__ double rows[LB / 4 * NACC];
    __shared__ double part8[8 * NACC];
    __shared__ double tot[NACC];
    const dquat q{x[0], x[1], x[2], x[3]};
    const double t[3] = {x[4], x[5], x[6]};
    double acc[NACC];
    for (int i = 0; i < NACC; i++) acc[i] = 0;
    for (int i = threadIdx.x; i < n; i += LB) {
        double r[3] = {0, 0, 0}, J[3][6] = {};
        const int m = eval_factor(f[i], q, t, r, J);
        double sc = 1.0, rho0 = 0, sq = 0;
        for (int k = 0; k < m; k++) sq += r[k] * r[k];
        if (robust) sc = huber_scale(sq, &rho0); else rho0 = sq;
        double Js[3][6], rs[3];
        for (int k = 0; k < 3; k++) {
            rs[k] = k < m ? r[k] * sc : 0.0;
            res[i * 3 + k] = rs[k];
            for (int c = 0; c < 6; c++) { Js[k][c] = k < m ? J[k][c] * sc : 0.0; jac[(i * 3 + k) * 6 + c] = Js[k][c]; }
        }
        if (!m) continue;
        acc[27] += 0.5 * rho0;
        for (int k = 0; k < m; k++) {
            int kk = 0;
            for (int a = 0; a < 6; a++) for (int b = a; b < 6; b++) acc[kk++] += Js[k][a] * Js[k][b];
            for (int a = 0; a < 6; a++) acc[21 + a] += Js[k][a] * rs[k];
        }
    }
    block_reduce_acc<LB>(acc, rows, part8, tot);
    if (threadIdx.x < 28) neq[threadIdx.x] = tot[threadIdx.x];
}

void lm_eval_only(Ctx& C, const aloam_factor* d_f, int n, const double* d_x, int robust, double* d_res, double* d_jac, double* d_neq) {
    k_eval_factors<<<1, LB, 0, C.stream>>>(d_f, n, d_x, robust, d_res, d_jac, d_neq);
    HIPCHK(hipGetLastError());
}

}  // namespace aloam
