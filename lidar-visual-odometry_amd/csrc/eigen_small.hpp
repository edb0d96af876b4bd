// eigen_small.hpp — the two small Eigen solves of laserMapping, restated for device code.
//
//   eigen_sym3:  Eigen::SelfAdjointEigenSolver<Matrix3d> (vendored Eigen 3.3.7,
//                Eigenvalues/SelfAdjointEigenSolver.h:400-445 compute(), :460-500 3x3
//                tridiagonalisation, computeFromTridiagonal_impl + tridiagonal_qr_step)
//                used at src/laserMapping.cpp:602
//   colpiv_qr_5x3: Eigen::ColPivHouseholderQR<Matrix<double,5,3>>::solve (QR/ColPivHouseholderQR.h
//                computeInPlace + _solve_impl) used at src/laserMapping.cpp:663
// Only +,-,*,/,sqrt: with -ffp-contract=off the device result equals the same code on the host.
// Pinned against the vendored Eigen by tests/golden/eigen_pins.json.
#pragma once
#include <math.h>

#ifndef ALOAM_HD
#if defined(__HIPCC__) || defined(__HIP__)
#define ALOAM_HD __host__ __device__
#else
#define ALOAM_HD
#endif
#endif

namespace aloam {

ALOAM_HD inline double es_fmax(double a, double b) { return a > b ? a : b; }
ALOAM_HD inline double es_fmin(double a, double b) { return a < b ? a : b; }

ALOAM_HD inline double es_hypot(double x, double y) {   // positive_real_hypot
    x = fabs(x); y = fabs(y);
    double p = es_fmax(x, y);
    if (p == 0.0) return 0.0;
    double qp = es_fmin(y, x) / p;
    return p * sqrt(1.0 + qp * qp);
}

// A: 3x3 row-major (only the lower triangle is read). evals ascending; evecs row-major, columns = vectors.
ALOAM_HD inline void eigen_sym3(const double A[9], double evals[3], double evecs[9]) {
    double m[9];
    for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) m[r * 3 + c] = (r >= c) ? A[r * 3 + c] : 0.0;
    double scale = 0;
    for (int i = 0; i < 9; i++) scale = es_fmax(scale, fabs(m[i]));
    if (scale == 0.0) scale = 1.0;
    for (int r = 0; r < 3; r++) for (int c = 0; c <= r; c++) m[r * 3 + c] /= scale;
    double diag[3], sub[2], Q[9];  // Q column-major
    diag[0] = m[0];
    const double dmin = 2.2250738585072014e-308;
    double v1norm2 = m[6] * m[6];
    if (v1norm2 <= dmin) {
        diag[1] = m[4]; diag[2] = m[8]; sub[0] = m[3]; sub[1] = m[7];
        for (int i = 0; i < 9; i++) Q[i] = (i % 4 == 0) ? 1.0 : 0.0;
    } else {
        double beta = sqrt(m[3] * m[3] + v1norm2);
        double invBeta = 1.0 / beta;
        double m01 = m[3] * invBeta, m02 = m[6] * invBeta;
        double q = 2.0 * m01 * m[7] + m02 * (m[8] - m[4]);
        diag[1] = m[4] + m02 * q;
        diag[2] = m[8] - m02 * q;
        sub[0] = beta;
        sub[1] = m[7] - m01 * q;
        double R[9] = {1, 0, 0, 0, m01, m02, 0, m02, -m01};
        for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) Q[c * 3 + r] = R[r * 3 + c];
    }
    // Implicit symmetric QR on the 3x3 tridiagonal (computeFromTridiagonal_impl). Written with
    // compile-time indices only (guards instead of data-dependent subscripts) so device code keeps
    // everything in registers; the arithmetic sequence is unchanged.
    const int n = 3;
    int end = n - 1, start = 0, iter = 0;
    const double precision = 2.0 * 2.220446049250313e-16;
    while (end > 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if (i >= start && i < end)
                if (fabs(sub[i]) <= (fabs(diag[i]) + fabs(diag[i + 1])) * precision || fabs(sub[i]) <= dmin) sub[i] = 0;
        if (end == 2 && sub[1] == 0.0) end = 1;
        if (end == 1 && sub[0] == 0.0) end = 0;
        if (end <= 0) break;
        iter++;
        if (iter > 30 * n) break;
        start = end - 1;
        if (start == 1 && sub[0] != 0) start = 0;
        const double dem1 = end == 2 ? diag[1] : diag[0], dend = end == 2 ? diag[2] : diag[1];
        double td = (dem1 - dend) * 0.5;
        double e = end == 2 ? sub[1] : sub[0];
        double mu = dend;
        if (td == 0.0) mu -= fabs(e);
        else {
            double e2 = e * e;
            double h = es_hypot(td, e);
            if (e2 == 0.0) mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / h);
            else mu -= e2 / (td + (td > 0.0 ? h : -h));
        }
        double x = (start == 0 ? diag[0] : diag[1]) - mu;
        double z = start == 0 ? sub[0] : sub[1];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (k < start || k >= end) continue;
            double c, s;
            if (z == 0.0) { c = x < 0.0 ? -1.0 : 1.0; s = 0.0; }
            else if (x == 0.0) { c = 0.0; s = z < 0.0 ? 1.0 : -1.0; }
            else if (fabs(x) > fabs(z)) {
                double t = z / x; double u = sqrt(1.0 + t * t); if (x < 0.0) u = -u;
                c = 1.0 / u; s = -t * c;
            } else {
                double t = x / z; double u = sqrt(1.0 + t * t); if (z < 0.0) u = -u;
                s = -1.0 / u; c = -t * s;
            }
            double sdk = s * diag[k] + c * sub[k];
            double dkp1 = s * sub[k] + c * diag[k + 1];
            diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
            diag[k + 1] = s * sdk + c * dkp1;
            sub[k] = c * sdk - s * dkp1;
            if (k > start) sub[k - 1 < 0 ? 0 : k - 1] = c * sub[k - 1 < 0 ? 0 : k - 1] - s * z;
            x = sub[k];
            if (k < end - 1) { z = -s * sub[k + 1 > 1 ? 1 : k + 1]; sub[k + 1 > 1 ? 1 : k + 1] = c * sub[k + 1 > 1 ? 1 : k + 1]; }
#pragma unroll
            for (int r = 0; r < 3; r++) {
                double xi = Q[k * 3 + r], yi = Q[(k + 1) * 3 + r];
                Q[k * 3 + r] = c * xi - s * yi;
                Q[(k + 1) * 3 + r] = s * xi + c * yi;
            }
        }
    }
    // ascending sort of the eigenvalues with their vectors (selection, as Eigen does)
#pragma unroll
    for (int i = 0; i < n - 1; ++i) {
        int k = i;
#pragma unroll
        for (int j = i + 1; j < n; j++) if (diag[j] < (k == 0 ? diag[0] : k == 1 ? diag[1] : diag[2])) k = j;
#pragma unroll
        for (int kk = i + 1; kk < n; kk++) {
            if (k != kk) continue;
            double t = diag[i]; diag[i] = diag[kk]; diag[kk] = t;
#pragma unroll
            for (int r = 0; r < 3; r++) { double tq = Q[i * 3 + r]; Q[i * 3 + r] = Q[kk * 3 + r]; Q[kk * 3 + r] = tq; }
        }
    }
    for (int i = 0; i < 3; i++) evals[i] = diag[i] * scale;
    for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) evecs[r * 3 + c] = Q[c * 3 + r];
}

// x = argmin ||A x - b||, A 5x3 row-major, column-pivoted Householder QR (compile-time indices
// only: pivots are applied with guarded static swaps).
ALOAM_HD inline void colpiv_qr_5x3(const double Ain[15], const double bin[5], double xout[3]) {
    const int rows = 5, cols = 3;
    double A[15];
#pragma unroll
    for (int i = 0; i < 15; i++) A[i] = Ain[i];
    double hc[3], nU[3], nD[3];
    int transp[3];
#pragma unroll
    for (int k = 0; k < cols; k++) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < rows; r++) s += A[r * 3 + k] * A[r * 3 + k];
        nD[k] = sqrt(s); nU[k] = nD[k];
    }
    double maxn = es_fmax(nU[0], es_fmax(nU[1], nU[2]));
    const double eps = 2.220446049250313e-16;
    double threshold_helper = (maxn * eps) * (maxn * eps) / (double)rows;
    double norm_downdate_threshold = sqrt(eps);
    int nonzero = cols;
#pragma unroll
    for (int k = 0; k < cols; k++) {
        int big = k; double bv = nU[k];
#pragma unroll
        for (int j = k + 1; j < cols; j++) if (nU[j] > bv) { bv = nU[j]; big = j; }
        if (nonzero == cols && bv * bv < threshold_helper * (double)(rows - k)) nonzero = k;
        transp[k] = big;
#pragma unroll
        for (int j = k + 1; j < cols; j++) {
            if (big != j) continue;
#pragma unroll
            for (int r = 0; r < rows; r++) { double t = A[r * 3 + k]; A[r * 3 + k] = A[r * 3 + j]; A[r * 3 + j] = t; }
            double t = nU[k]; nU[k] = nU[j]; nU[j] = t;
            t = nD[k]; nD[k] = nD[j]; nD[j] = t;
        }
        double tail = 0;
#pragma unroll
        for (int r = k + 1; r < rows; r++) tail += A[r * 3 + k] * A[r * 3 + k];
        double c0 = A[k * 3 + k], tau, beta;
        if (tail <= 2.2250738585072014e-308) {
            tau = 0; beta = c0;
#pragma unroll
            for (int r = k + 1; r < rows; r++) A[r * 3 + k] = 0;
        } else {
            beta = sqrt(c0 * c0 + tail); if (c0 >= 0) beta = -beta;
#pragma unroll
            for (int r = k + 1; r < rows; r++) A[r * 3 + k] /= (c0 - beta);
            tau = (beta - c0) / beta;
        }
        hc[k] = tau; A[k * 3 + k] = beta;
        if (tau != 0.0) {
#pragma unroll
            for (int c = k + 1; c < cols; c++) {
                double w = A[k * 3 + c];
#pragma unroll
                for (int r = k + 1; r < rows; r++) w += A[r * 3 + k] * A[r * 3 + c];
                A[k * 3 + c] -= tau * w;
#pragma unroll
                for (int r = k + 1; r < rows; r++) A[r * 3 + c] -= tau * A[r * 3 + k] * w;
            }
        }
#pragma unroll
        for (int j = k + 1; j < cols; j++) {
            if (nU[j] != 0.0) {
                double temp = fabs(A[k * 3 + j]) / nU[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                double ratio = nU[j] / nD[j];
                double temp2 = temp * ratio * ratio;
                if (temp2 <= norm_downdate_threshold) {
                    double s = 0;
#pragma unroll
                    for (int r = k + 1; r < rows; r++) s += A[r * 3 + j] * A[r * 3 + j];
                    nD[j] = sqrt(s); nU[j] = nD[j];
                } else nU[j] *= sqrt(temp);
            }
        }
    }
    // permutation from the transpositions
    int perm[3] = {0, 1, 2};
#pragma unroll
    for (int k = 0; k < cols; k++) {
#pragma unroll
        for (int j = k + 1; j < cols; j++) {
            if (transp[k] != j) continue;
            int t = perm[k]; perm[k] = perm[j]; perm[j] = t;
        }
    }
    if (nonzero == 0) { xout[0] = xout[1] = xout[2] = 0; return; }
    double c[5];
#pragma unroll
    for (int r = 0; r < rows; r++) c[r] = bin[r];
#pragma unroll
    for (int k = 0; k < cols; k++) {
        if (k >= nonzero || hc[k] == 0.0) continue;
        double w = c[k];
#pragma unroll
        for (int r = k + 1; r < rows; r++) w += A[r * 3 + k] * c[r];
        c[k] -= hc[k] * w;
#pragma unroll
        for (int r = k + 1; r < rows; r++) c[r] -= hc[k] * A[r * 3 + k] * w;
    }
    double y[3] = {0, 0, 0};
#pragma unroll
    for (int i = cols - 1; i >= 0; i--) {
        if (i >= nonzero) continue;
        double s = c[i];
#pragma unroll
        for (int j = i + 1; j < cols; j++) if (j < nonzero) s -= A[i * 3 + j] * y[j];
        y[i] = s / A[i * 3 + i];
    }
#pragma unroll
    for (int o = 0; o < 3; o++) {
        double v = 0;
#pragma unroll
        for (int i = 0; i < cols; i++) if (i < nonzero && perm[i] == o) v = y[i];
        xout[o] = v;
    }
}

}  // namespace aloam
