// aloam_device.hpp — shared device helpers of the HIP hot path (gfx950, wave64).
//
// All parity-critical arithmetic is written in the reference's operation order and the whole
// library is compiled with -ffp-contract=off, so fp32 / fp64 results round exactly like the
// reference's x86-64 SSE2 build (CMakeLists.txt:6, no -march => no FMA).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/aloam_hip.h"

#define WAVE 64

namespace aloam {

struct dquat { double x, y, z, w; };
struct dvec3 { double x, y, z; };

__host__ __device__ inline dvec3 dcross(const dvec3& a, const dvec3& b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// Eigen QuaternionBase::_transformVector (Quaternion.h:476-485)
__host__ __device__ inline dvec3 qrot(const dquat& q, const dvec3& v) {
    dvec3 qv{q.x, q.y, q.z};
    dvec3 uv = dcross(qv, v);
    uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    dvec3 c = dcross(qv, uv);
    return {v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z};
}
// Eigen quat_product<SSE,...,double> (arch/Geometry_SSE.h) operation order: a * b
__host__ __device__ inline dquat qmul(const dquat& a, const dquat& b) {
    dquat r;
    r.x = (a.w * b.x + a.y * b.z) - (a.z * b.y - a.x * b.w);
    r.y = (a.w * b.y + a.y * b.w) + (a.z * b.x - a.x * b.z);
    r.z = (a.w * b.z - a.y * b.x) + (a.z * b.w + a.x * b.y);
    r.w = (a.w * b.w - a.y * b.y) - (a.z * b.z + a.x * b.x);
    return r;
}
// QuaternionBase::inverse: conjugate / squaredNorm (SSE2 packet-redux order)
__host__ __device__ inline dquat qinv(const dquat& q) {
    double n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
    if (n2 > 0) return {-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
    return {0, 0, 0, 0};
}
// Identity().slerp(t, q) (Quaternion.h:726-754)
__device__ inline dquat qslerp_identity(double t, const dquat& q) {
    const double one = 1.0 - 2.220446049250313e-16;
    double d = q.w;
    double absD = fabs(d);
    double s0, s1;
    if (absD >= one) { s0 = 1.0 - t; s1 = t; }
    else {
        double theta = acos(absD);
        double sinTheta = sin(theta);
        s0 = sin((1.0 - t) * theta) / sinTheta;
        s1 = sin(t * theta) / sinTheta;
    }
    if (d < 0) s1 = -s1;
    return {s0 * 0.0 + s1 * q.x, s0 * 0.0 + s1 * q.y, s0 * 0.0 + s1 * q.z, s0 * 1.0 + s1 * q.w};
}

// ---- wave64 helpers ------------------------------------------------------------------
__device__ inline int lane_id() { return threadIdx.x & (WAVE - 1); }

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long t = __shfl_xor(v, o, WAVE);
        v = t < v ? t : v;
    }
    return v;
}
__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long t = __shfl_xor(v, o, WAVE);
        v = t > v ? t : v;
    }
    return v;
}
__device__ inline double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ inline int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ inline unsigned long long lanemask_lt64() {
    int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// float >= 0 (or +inf) ordered as unsigned: key = (bits << 32) | index
__device__ inline unsigned long long dist_key(float d2, int idx) {
    return ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)idx;
}

// ordered-int encoding of floats for atomic min/max
__device__ inline unsigned f2ord(float f) {
    unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float ord2f(unsigned u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__host__ __device__ inline unsigned f2ord_h(float f) {
    unsigned u; memcpy(&u, &f, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// float L2^2 in the reference's order: ((dx*dx + dy*dy) + dz*dz)  (FLANN L2_Simple, laserOdometry.cpp:404-409)
__device__ inline float sqdist(float ax, float ay, float az, float bx, float by, float bz) {
    float dx = ax - bx, dy = ay - by, dz = az - bz;
    return dx * dx + dy * dy + dz * dz;
}

}  // namespace aloam
