/*
 * aloam_lidar_factor.hpp — the lidarFactor.hpp cost-functor API of the reference
 * (src/lidarFactor.hpp:12-172), kept source-compatible for host code, plus packing into the
 * device factor record (aloam_factor, include/aloam_hip.h) that the HIP solver evaluates.
 *
 * Same struct names, constructor signatures, public members and functor signature:
 *   LidarEdgeFactor(curr_point, last_point_a, last_point_b, s)             lidarFactor.hpp:12-55
 *   LidarPlaneFactor(curr_point, last_point_j, last_point_l, last_point_m, s)       :57-104
 *   LidarPlaneNormFactor(curr_point, plane_unit_norm, negative_OA_dot_norm)         :106-138
 *   LidarDistanceFactor(curr_point, closed_point)                                   :141-172
 *   template <typename T> bool operator()(const T* q, const T* t, T* residual) const
 * with q in Eigen (x, y, z, w) order and t = (x, y, z). Any vector type with operator[]
 * (Eigen::Vector3d included) is accepted by the constructors. `Create(...)` returns the
 * ceres::AutoDiffCostFunction exactly like the reference when HAVE_CERES is defined.
 *
 * The functors are generic in T (double, ceres::Jet, ...): sqrt/acos/sin/abs resolve by ADL.
 * On the device the same residuals and their analytic SE(3) Jacobians are evaluated by
 * csrc/k_lm.hip; to_device() packs a functor into that record. The device path implements the
 * reference's configuration s = 1 (DISTORTION 0, laserOdometry.cpp:67,158-161); to_device()
 * refuses other s.
 */
#ifndef ALOAM_LIDAR_FACTOR_HPP
#define ALOAM_LIDAR_FACTOR_HPP

#include <cmath>

#include "aloam_hip.h"

#ifdef HAVE_CERES
#include <ceres/ceres.h>
#endif

namespace aloam_api {

// Eigen-like 3-vector of doubles for the public members (x()/y()/z() and operator[])
struct Vec3d {
    double v[3] = {0, 0, 0};
    Vec3d() = default;
    Vec3d(double x, double y, double z) : v{x, y, z} {}
    template <class V>
    static Vec3d from(const V& a) { return Vec3d(double(a[0]), double(a[1]), double(a[2])); }
    double x() const { return v[0]; }
    double y() const { return v[1]; }
    double z() const { return v[2]; }
    double operator[](int i) const { return v[i]; }
    double& operator[](int i) { return v[i]; }
};

namespace detail {
// p' = q * p for a unit quaternion q = (x, y, z, w), Eigen's _transformVector order:
// uv = 2 (q.vec x p); p' = p + w uv + q.vec x uv
template <typename T>
inline void rotate(const T q[4], const T p[3], T out[3]) {
    T uv[3] = {q[1] * p[2] - q[2] * p[1], q[2] * p[0] - q[0] * p[2], q[0] * p[1] - q[1] * p[0]};
    for (int i = 0; i < 3; i++) uv[i] = uv[i] + uv[i];
    const T c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    for (int i = 0; i < 3; i++) out[i] = p[i] + q[3] * uv[i] + c[i];
}
// slerp(identity, q, s) as Eigen::QuaternionBase::slerp computes it (dot = q.w)
template <typename T>
inline void slerp_identity(const T& s, const T q[4], T out[4]) {
    using std::abs;
    using std::acos;
    using std::sin;
    const T one(1.0);
    const T d = q[3];
    const T absd = abs(d);
    T s0, s1;
    if (absd >= one - T(2.220446049250313e-16)) {   // Eigen: 1 - NumTraits<Scalar>::epsilon()
        s0 = one - s;
        s1 = s;
    } else {
        const T theta = acos(absd);
        const T st = sin(theta);
        s0 = sin((one - s) * theta) / st;
        s1 = sin(s * theta) / st;
    }
    if (d < T(0.0)) s1 = -s1;
    out[0] = s1 * q[0];
    out[1] = s1 * q[1];
    out[2] = s1 * q[2];
    out[3] = s0 + s1 * q[3];
}
}  // namespace detail

struct LidarEdgeFactor {
    template <class V>
    LidarEdgeFactor(const V& curr_point_, const V& last_point_a_, const V& last_point_b_, double s_)
        : curr_point(Vec3d::from(curr_point_)), last_point_a(Vec3d::from(last_point_a_)),
          last_point_b(Vec3d::from(last_point_b_)), s(s_) {}

    template <typename T>
    bool operator()(const T* q, const T* t, T* residual) const {
        using std::sqrt;
        const T cp[3] = {T(curr_point[0]), T(curr_point[1]), T(curr_point[2])};
        const T ss(s);
        T qs[4], lp[3];
        detail::slerp_identity(ss, q, qs);
        detail::rotate(qs, cp, lp);
        for (int i = 0; i < 3; i++) lp[i] = lp[i] + ss * t[i];
        const T u[3] = {lp[0] - T(last_point_a[0]), lp[1] - T(last_point_a[1]), lp[2] - T(last_point_a[2])};
        const T w[3] = {lp[0] - T(last_point_b[0]), lp[1] - T(last_point_b[1]), lp[2] - T(last_point_b[2])};
        const T nu[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
        const T de[3] = {T(last_point_a[0] - last_point_b[0]), T(last_point_a[1] - last_point_b[1]),
                         T(last_point_a[2] - last_point_b[2])};
        const T n = sqrt(de[0] * de[0] + de[1] * de[1] + de[2] * de[2]);
        for (int i = 0; i < 3; i++) residual[i] = nu[i] / n;
        return true;
    }

#ifdef HAVE_CERES
    template <class V>
    static ceres::CostFunction* Create(const V& curr_point_, const V& last_point_a_, const V& last_point_b_, const double s_) {
        return new ceres::AutoDiffCostFunction<LidarEdgeFactor, 3, 4, 3>(
            new LidarEdgeFactor(curr_point_, last_point_a_, last_point_b_, s_));
    }
#endif

    bool to_device(aloam_factor* f) const {
        if (s != 1.0) return false;
        *f = aloam_factor{};
        f->type = 0;
        for (int i = 0; i < 3; i++) { f->cp[i] = curr_point[i]; f->a[i] = last_point_a[i]; f->b[i] = last_point_b[i]; }
        return true;
    }

    Vec3d curr_point, last_point_a, last_point_b;
    double s;
};

struct LidarPlaneFactor {
    template <class V>
    LidarPlaneFactor(const V& curr_point_, const V& last_point_j_, const V& last_point_l_, const V& last_point_m_, double s_)
        : curr_point(Vec3d::from(curr_point_)), last_point_j(Vec3d::from(last_point_j_)),
          last_point_l(Vec3d::from(last_point_l_)), last_point_m(Vec3d::from(last_point_m_)), s(s_) {
        // ljm_norm = normalize((j - l) x (j - m)) as in the reference constructor
        const double a[3] = {last_point_j[0] - last_point_l[0], last_point_j[1] - last_point_l[1], last_point_j[2] - last_point_l[2]};
        const double b[3] = {last_point_j[0] - last_point_m[0], last_point_j[1] - last_point_m[1], last_point_j[2] - last_point_m[2]};
        double c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
        const double nn = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        if (nn > 0) for (int i = 0; i < 3; i++) c[i] /= nn;
        ljm_norm = Vec3d(c[0], c[1], c[2]);
    }

    template <typename T>
    bool operator()(const T* q, const T* t, T* residual) const {
        const T cp[3] = {T(curr_point[0]), T(curr_point[1]), T(curr_point[2])};
        const T ss(s);
        T qs[4], lp[3];
        detail::slerp_identity(ss, q, qs);
        detail::rotate(qs, cp, lp);
        for (int i = 0; i < 3; i++) lp[i] = lp[i] + ss * t[i];
        residual[0] = (lp[0] - T(last_point_j[0])) * T(ljm_norm[0]) + (lp[1] - T(last_point_j[1])) * T(ljm_norm[1]) +
                      (lp[2] - T(last_point_j[2])) * T(ljm_norm[2]);
        return true;
    }

#ifdef HAVE_CERES
    template <class V>
    static ceres::CostFunction* Create(const V& curr_point_, const V& last_point_j_, const V& last_point_l_,
                                       const V& last_point_m_, const double s_) {
        return new ceres::AutoDiffCostFunction<LidarPlaneFactor, 1, 4, 3>(
            new LidarPlaneFactor(curr_point_, last_point_j_, last_point_l_, last_point_m_, s_));
    }
#endif

    bool to_device(aloam_factor* f) const {
        if (s != 1.0) return false;
        *f = aloam_factor{};
        f->type = 1;
        for (int i = 0; i < 3; i++) { f->cp[i] = curr_point[i]; f->a[i] = last_point_j[i]; f->b[i] = ljm_norm[i]; }
        return true;
    }

    Vec3d curr_point, last_point_j, last_point_l, last_point_m;
    Vec3d ljm_norm;
    double s;
};

struct LidarPlaneNormFactor {
    template <class V>
    LidarPlaneNormFactor(const V& curr_point_, const V& plane_unit_norm_, double negative_OA_dot_norm_)
        : curr_point(Vec3d::from(curr_point_)), plane_unit_norm(Vec3d::from(plane_unit_norm_)),
          negative_OA_dot_norm(negative_OA_dot_norm_) {}

    template <typename T>
    bool operator()(const T* q, const T* t, T* residual) const {
        const T cp[3] = {T(curr_point[0]), T(curr_point[1]), T(curr_point[2])};
        T pw[3];
        detail::rotate(q, cp, pw);
        for (int i = 0; i < 3; i++) pw[i] = pw[i] + t[i];
        residual[0] = T(plane_unit_norm[0]) * pw[0] + T(plane_unit_norm[1]) * pw[1] + T(plane_unit_norm[2]) * pw[2] +
                      T(negative_OA_dot_norm);
        return true;
    }

#ifdef HAVE_CERES
    template <class V>
    static ceres::CostFunction* Create(const V& curr_point_, const V& plane_unit_norm_, const double negative_OA_dot_norm_) {
        return new ceres::AutoDiffCostFunction<LidarPlaneNormFactor, 1, 4, 3>(
            new LidarPlaneNormFactor(curr_point_, plane_unit_norm_, negative_OA_dot_norm_));
    }
#endif

    bool to_device(aloam_factor* f) const {
        *f = aloam_factor{};
        f->type = 2;
        for (int i = 0; i < 3; i++) { f->cp[i] = curr_point[i]; f->a[i] = plane_unit_norm[i]; }
        f->b[0] = negative_OA_dot_norm;
        return true;
    }

    Vec3d curr_point, plane_unit_norm;
    double negative_OA_dot_norm;
};

struct LidarDistanceFactor {
    template <class V>
    LidarDistanceFactor(const V& curr_point_, const V& closed_point_)
        : curr_point(Vec3d::from(curr_point_)), closed_point(Vec3d::from(closed_point_)) {}

    template <typename T>
    bool operator()(const T* q, const T* t, T* residual) const {
        const T cp[3] = {T(curr_point[0]), T(curr_point[1]), T(curr_point[2])};
        T pw[3];
        detail::rotate(q, cp, pw);
        for (int i = 0; i < 3; i++) residual[i] = pw[i] + t[i] - T(closed_point[i]);
        return true;
    }

#ifdef HAVE_CERES
    template <class V>
    static ceres::CostFunction* Create(const V& curr_point_, const V& closed_point_) {
        return new ceres::AutoDiffCostFunction<LidarDistanceFactor, 3, 4, 3>(new LidarDistanceFactor(curr_point_, closed_point_));
    }
#endif

    bool to_device(aloam_factor* f) const {
        *f = aloam_factor{};
        f->type = 3;
        for (int i = 0; i < 3; i++) { f->cp[i] = curr_point[i]; f->a[i] = closed_point[i]; }
        return true;
    }

    Vec3d curr_point, closed_point;
};

}  // namespace aloam_api

#ifndef ALOAM_NO_GLOBAL_FACTOR_NAMES
// the reference's names live in the global namespace
using aloam_api::LidarDistanceFactor;
using aloam_api::LidarEdgeFactor;
using aloam_api::LidarPlaneFactor;
using aloam_api::LidarPlaneNormFactor;
#endif

#endif  // ALOAM_LIDAR_FACTOR_HPP
