// oracle/pin_eigen.cpp — golden-vector generator (test infrastructure).
//
// Runs the exact Eigen calls laserMapping makes, using the reference's VENDORED Eigen 3.3.7
// (compiled in place from /root/reference/thirdparty/eigen by oracle/Makefile), on seeded
// synthetic inputs shaped like the mapping's neighbourhoods:
//   * Eigen::SelfAdjointEigenSolver<Eigen::Matrix3d>(covMat)      (src/laserMapping.cpp:602)
//   * matA0.colPivHouseholderQr().solve(matB0), 5x3, b = -1       (src/laserMapping.cpp:663)
// and prints JSON {eig: [...], qr: [...]} with inputs and outputs as hex-exact doubles.
// tests/test_oracle_pins.py checks the oracle's restatements against it.
#include <Eigen/Dense>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static double urand() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * (1.0 / 9007199254740992.0); }

static void pd(double v, bool comma = true) { printf("\"%a\"%s", v, comma ? "," : ""); }

int main() {
    printf("{\"generator\": \"oracle/pin_eigen.cpp\", \"eigen\": \"vendored 3.3.7\",\n \"eig\": [\n");
    const int NE = 400;
    for (int t = 0; t < NE; t++) {
        // 5 points along a noisy line / blob, in float like map points
        double dir[3] = {urand() - 0.5, urand() - 0.5, urand() - 0.5};
        double c0[3] = {urand() * 100 - 50, urand() * 100 - 50, urand() * 10 - 5};
        double noise = (t % 3 == 0) ? 0.3 : 0.02;
        std::vector<Eigen::Vector3d> pts;
        Eigen::Vector3d center(0, 0, 0);
        for (int j = 0; j < 5; j++) {
            double l = urand() * 2 - 1;
            Eigen::Vector3d p((float)(c0[0] + l * dir[0] + noise * (urand() - 0.5)),
                              (float)(c0[1] + l * dir[1] + noise * (urand() - 0.5)),
                              (float)(c0[2] + l * dir[2] + noise * (urand() - 0.5)));
            pts.push_back(p);
            center = center + p;
        }
        center = center / 5.0;
        Eigen::Matrix3d cov = Eigen::Matrix3d::Zero();
        for (int j = 0; j < 5; j++) { Eigen::Vector3d z = pts[j] - center; cov = cov + z * z.transpose(); }
        Eigen::SelfAdjointEigenSolver<Eigen::Matrix3d> saes(cov);
        printf("  {\"A\": [");
        for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) pd(cov(r, c), !(r == 2 && c == 2));
        printf("], \"evals\": [");
        for (int i = 0; i < 3; i++) pd(saes.eigenvalues()[i], i < 2);
        printf("], \"evecs\": [");
        for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) pd(saes.eigenvectors()(r, c), !(r == 2 && c == 2));
        printf("]}%s\n", t + 1 < NE ? "," : "");
    }
    printf(" ],\n \"qr\": [\n");
    const int NQ = 400;
    for (int t = 0; t < NQ; t++) {
        // 5 points near a plane n.p + d = 0, float-rounded
        Eigen::Vector3d n(urand() - 0.5, urand() - 0.5, urand() * 2 - 1);
        n.normalize();
        double d = urand() * 20 - 10;
        Eigen::Vector3d u = n.unitOrthogonal(), v = n.cross(u);
        Eigen::Vector3d o = -d * n + Eigen::Vector3d(urand() * 60 - 30, urand() * 60 - 30, urand() * 4 - 2);
        Eigen::Matrix<double, 5, 3> A;
        Eigen::Matrix<double, 5, 1> b = -1 * Eigen::Matrix<double, 5, 1>::Ones();
        double noise = (t % 4 == 0) ? 0.2 : 0.01;
        for (int j = 0; j < 5; j++) {
            Eigen::Vector3d p = o + (urand() - 0.5) * u + (urand() - 0.5) * v + noise * (urand() - 0.5) * n;
            A(j, 0) = (float)p.x(); A(j, 1) = (float)p.y(); A(j, 2) = (float)p.z();
        }
        Eigen::Vector3d x = A.colPivHouseholderQr().solve(b);
        printf("  {\"A\": [");
        for (int r = 0; r < 5; r++) for (int c = 0; c < 3; c++) pd(A(r, c), !(r == 4 && c == 2));
        printf("], \"x\": [");
        for (int i = 0; i < 3; i++) pd(x[i], i < 2);
        printf("]}%s\n", t + 1 < NQ ? "," : "");
    }
    printf(" ]\n}\n");
    return 0;
}
