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
// Identity().slerp(t, q) (Quaternion.h:726-754) at t = 1, the only value on the hot path
// (DISTORTION 0 => s = 1, laserOdometry.cpp:67,158-161; lidarFactor.hpp:29,81 get s = 1).
// With t = 1 Eigen computes scale0 = sin(0*theta)/sin(theta) = +0 and scale1 = sin(theta)/sin(theta)
// = 1 exactly (same bits divided by themselves; the |d| >= 1-eps branch gives 0 and 1 directly), so
// the result is exactly sign(w) * q: the acos/sin evaluations are skipped without changing a bit
// (up to the sign of a zero component, which no later operation can observe).
__device__ inline dquat qslerp_identity(double t, const dquat& q) {
    (void)t;
    if (q.w < 0) return {-q.x, -q.y, -q.z, -q.w};
    return q;
}

// ---- wave64 helpers ------------------------------------------------------------------
__device__ inline int lane_id() { return threadIdx.x & (WAVE - 1); }

// Cross-lane exchange without LDS: DPP for partners inside a 16-lane row (quad_perm swaps, then
// half-row and row mirrors — after the quad steps a mirror reaches exactly the other half), the
// gfx950 row-pair and half-wave swaps for 16 and 32. A __shfl_xor is a ds_bpermute round trip
// through the LDS unit per step; these are plain VALU ops.
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ unsigned swap16_u32(unsigned v) {      // value of lane l ^ 16
    const auto s = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return ((threadIdx.x >> 4) & 1) ? s[0] : s[1];
}
__device__ __forceinline__ unsigned swap32_u32(unsigned v) {      // value of lane l ^ 32
    const auto s = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return ((threadIdx.x >> 5) & 1) ? s[0] : s[1];
}
// partner value at step k of a wave all-reduce (k = 0..5: quad xor 1, quad xor 2, half-row mirror,
// row mirror, row pair, half wave)
template <int K>
__device__ __forceinline__ unsigned xstep_u32(unsigned v) {
    if constexpr (K == 0) return dpp_u32<0xB1>(v);        // quad_perm [1,0,3,2]
    else if constexpr (K == 1) return dpp_u32<0x4E>(v);   // quad_perm [2,3,0,1]
    else if constexpr (K == 2) return dpp_u32<0x141>(v);  // row_half_mirror
    else if constexpr (K == 3) return dpp_u32<0x140>(v);  // row_mirror
    else if constexpr (K == 4) return swap16_u32(v);
    else return swap32_u32(v);
}
template <int K>
__device__ __forceinline__ unsigned long long xstep_u64(unsigned long long v) {
    return ((unsigned long long)xstep_u32<K>((unsigned)(v >> 32)) << 32) | xstep_u32<K>((unsigned)v);
}
// all-reduce over the first 2^NS steps' lanes (NS = 6: whole wave; NS = 3: aligned groups of 8)
template <int NS, typename F>
__device__ __forceinline__ unsigned long long allreduce_u64(unsigned long long v, F op) {
    if constexpr (NS > 0) v = op(v, xstep_u64<0>(v));
    if constexpr (NS > 1) v = op(v, xstep_u64<1>(v));
    if constexpr (NS > 2) v = op(v, xstep_u64<2>(v));
    if constexpr (NS > 3) v = op(v, xstep_u64<3>(v));
    if constexpr (NS > 4) v = op(v, xstep_u64<4>(v));
    if constexpr (NS > 5) v = op(v, xstep_u64<5>(v));
    return v;
}
template <int NS, typename F>
__device__ __forceinline__ unsigned allreduce_u32(unsigned v, F op) {
    if constexpr (NS > 0) v = op(v, xstep_u32<0>(v));
    if constexpr (NS > 1) v = op(v, xstep_u32<1>(v));
    if constexpr (NS > 2) v = op(v, xstep_u32<2>(v));
    if constexpr (NS > 3) v = op(v, xstep_u32<3>(v));
    if constexpr (NS > 4) v = op(v, xstep_u32<4>(v));
    if constexpr (NS > 5) v = op(v, xstep_u32<5>(v));
    return v;
}
// Inclusive prefix sum over the wave with DPP (row shifts 1/2/4/8, then row broadcasts of lanes 15
// and 31), no LDS round trips. Lanes a shift does not reach keep the 0 of the update's old value.
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return v;
}
// value of a wave-uniform lane (SGPR result, no LDS)
__device__ __forceinline__ int readlane_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ float readlane_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
    return allreduce_u64<6>(v, [](unsigned long long a, unsigned long long b) { return b < a ? b : a; });
}
__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
    return allreduce_u64<6>(v, [](unsigned long long a, unsigned long long b) { return b > a ? b : a; });
}
__device__ inline double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ inline int wave_sum_i(int v) {
    return (int)allreduce_u32<6>((unsigned)v, [](unsigned a, unsigned b) { return a + b; });
}
__device__ inline unsigned long long lanemask_lt64() {
    int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// float >= 0 (or +inf) ordered as unsigned: key = (bits << 32) | index
__device__ inline unsigned long long dist_key(float d2, int idx) {
    return ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)idx;
}

// Guarded load without control flow: the address is clamped to element 0 (valid in every buffer
// this is used on) and the value replaced afterwards. A branch around each load of an unrolled
// batch makes the compiler wait for the load inside the branch — one memory round trip per load
// instead of one per batch.
template <typename T>
__device__ __forceinline__ T load_or(const T* __restrict__ a, int i, bool ok, T dflt) {
    const T v = a[ok ? i : 0];
    return ok ? v : dflt;
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

// Per-wave phase stamps for profiling builds only (-DALOAM_WSTAMP_<KERNEL>): lane 0 of each wave
// writes wall_clock64() (100 MHz) into slot k of its wave's row; aloam_dbg_wstamps() copies the table
// of the kernel's last launch out. In the product build WSTAMP(k) is empty.
constexpr int WSTAMP_WAVES = 8192, WSTAMP_SLOTS = 8;
#define WSTAMP_DEFINE_TABLE                                                                                 \
    __device__ unsigned long long g_wstamp[WSTAMP_WAVES * WSTAMP_SLOTS];                                   \
    extern "C" int aloam_dbg_wstamps(unsigned long long* out) {                                            \
        return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wstamp), sizeof(g_wstamp));                      \
    }
#define WSTAMP_ON(k)                                                                                       \
    do {                                                                                                   \
        const unsigned w_ = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;                                \
        if ((threadIdx.x & (WAVE - 1)) == 0 && w_ < WSTAMP_WAVES) g_wstamp[w_ * WSTAMP_SLOTS + (k)] = wall_clock64(); \
    } while (0)

// float L2^2 in the reference's order: ((dx*dx + dy*dy) + dz*dz)  (FLANN L2_Simple, laserOdometry.cpp:404-409)
__device__ inline float sqdist(float ax, float ay, float az, float bx, float by, float bz) {
    float dx = ax - bx, dy = ay - by, dz = az - bz;
    return dx * dx + dy * dy + dz * dz;
}

}  // namespace aloam

namespace aloam {
// ---- grid neighbourhood as contiguous x-rows --------------------------------------------------
// Points are sorted by cell id c = (z*dy + y)*dx + x, so the cells [x0, x1] of one (y, z) row are one
// contiguous point range. A (2m+1)^3 neighbourhood of the query's cell is (2m+1)^2 ranges, flattened
// so all 64 lanes of a wave stream candidates regardless of how the points spread over the rows.
template <int MAXR>
struct RowSet {
    int b[MAXR];
    int pre[MAXR + 1];
    int nr;
};
// rs lives in LDS, one per wave. Lane r < (2m+1)^2 owns row r: its two cell_start loads are issued
// by all lanes at once (one round trip), a wave prefix sum turns the row lengths into offsets.
// Empty rows stay in the set with zero length.
template <int MAXR>
__device__ __forceinline__ int build_rows(const float ox, const float oy, const float oz, const float inv_cell,
                                          const int gdx, const int gdy, const int gdz, const int* __restrict__ start,
                                          float qx, float qy, float qz, int m, RowSet<MAXR>& rs) {
    static_assert(MAXR <= WAVE, "one row per lane");
    const int lane = lane_id();
    const int cx = (int)floorf((qx - ox) * inv_cell), cy = (int)floorf((qy - oy) * inv_cell), cz = (int)floorf((qz - oz) * inv_cell);
    const int x0 = max(cx - m, 0), x1 = min(cx + m, gdx - 1);
    const int w = 2 * m + 1;
    const int nrow = w * w;
    const int y = cy - m + lane % w, z = cz - m + lane / w;
    const bool ok = lane < nrow && lane < MAXR && x0 <= x1 && y >= 0 && y < gdy && z >= 0 && z < gdz;
    const int c = (z * gdy + y) * gdx;
    const int b = load_or(start, c + x0, ok, 0);
    const int len = load_or(start, c + x1 + 1, ok, 0) - b;
    int incl = len;
    incl = wave_incl_scan(incl);
    const int nr = min(nrow, MAXR);
    __builtin_amdgcn_wave_barrier();
    if (lane < nr) { rs.b[lane] = b; rs.pre[lane + 1] = incl; }
    if (lane == 0) { rs.pre[0] = 0; rs.nr = nr; }
    const int total = readlane_i(incl, nr - 1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return total;
}
// flattened candidate t -> point position (binary search over the row offsets)
constexpr int pow2_floor(int v) { int p = 1; while (p * 2 <= v) p *= 2; return p; }
// Fixed-step binary search (last row r with pre[r] <= t): uniform trip count, so the searches of a
// lane's several candidates interleave instead of running one data-dependent loop after another.
template <int MAXR>
__device__ __forceinline__ int row_pos(const RowSet<MAXR>& rs, int t) {
    const int last = rs.nr - 1;
    int r = 0;
#pragma unroll
    for (int step = pow2_floor(MAXR > 1 ? MAXR - 1 : 1); step >= 1; step >>= 1) {
        const int c = min(r + step, last);
        r = rs.pre[c] <= t ? c : r;
    }
    return rs.b[r] + (t - rs.pre[r]);
}
}  // namespace aloam

namespace aloam {
// Exact radius k-NN of one query by one wave over the (2m+1)^3 cell neighbourhood: every lane keeps a
// sorted top-K of the candidates it streams (4 loads in flight), then K rounds of a 64-bit wave-min
// over the lanes' heads merge them. Keys (d2 bits, index) order equal distances by point index.
// Returns the number found (<= K); out_pos = positions in the grid's sorted arrays.
template <int K, int MAXR>
__device__ __forceinline__ int wave_knn_rows(const float ox, const float oy, const float oz, const float inv_cell,
                                             const int gdx, const int gdy, const int gdz,
                                             const int* __restrict__ start, const float4* __restrict__ spts,
                                             const int* __restrict__ sidx, float qx, float qy, float qz, float r2, int m,
                                             int* out_pos, float* out_d2, int* out_idx, int* ncand, RowSet<MAXR>& rs) {
    const int lane = lane_id();
    const int total = build_rows<MAXR>(ox, oy, oz, inv_cell, gdx, gdy, gdz, start, qx, qy, qz, m, rs);
    if (ncand) *ncand = total;
    float bd[K];
    int bi[K], bp[K];
#pragma unroll
    for (int k = 0; k < K; k++) { bd[k] = INFINITY; bi[k] = 0x7fffffff; bp[k] = -1; }
    for (int t0 = 0; t0 < total; t0 += 4 * WAVE) {
        int pp[4];
        float4 vv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int t = t0 + u * WAVE + lane;
            const int pos = row_pos<MAXR>(rs, min(t, total - 1));
            pp[u] = t < total ? pos : -1;
            vv[u] = load_or(spts, pp[u], pp[u] >= 0, make_float4(0, 0, 0, 0));
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (pp[u] < 0) continue;
            const float d2 = sqdist(vv[u].x, vv[u].y, vv[u].z, qx, qy, qz);
            if (!(d2 < r2)) continue;
            const int id = sidx[pp[u]];
            if (d2 < bd[K - 1] || (d2 == bd[K - 1] && id < bi[K - 1])) {
                float nd = d2; int ni = id, np = pp[u];
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const bool lt = nd < bd[k] || (nd == bd[k] && ni < bi[k]);
                    if (lt) { float td = bd[k]; int ti = bi[k], tp = bp[k]; bd[k] = nd; bi[k] = ni; bp[k] = np; nd = td; ni = ti; np = tp; }
                }
            }
        }
    }
    int head = 0, found = 0;
    for (int k = 0; k < K; k++) {
        float hd = INFINITY; int hi = 0x7fffffff, hp = -1;
#pragma unroll
        for (int j = 0; j < K; j++) if (j == head) { hd = bd[j]; hi = bi[j]; hp = bp[j]; }
        const unsigned long long key = hp < 0 ? ~0ull : dist_key(hd, hi);
        const unsigned long long mn = wave_min_u64(key);
        if (mn == ~0ull) break;
        const unsigned long long won = __ballot(key == mn);
        if (key == mn) head++;
        out_pos[k] = readlane_i(hp, __ffsll((long long)won) - 1);
        out_d2[k] = __uint_as_float((unsigned)(mn >> 32));
        out_idx[k] = (int)(mn & 0xffffffffu);
        found++;
    }
    return found;
}
// Exact radius k-NN of one query by ONE THREAD over the 3x3x3 cell block (m = 1): the 9 (y, z)
// rows of 3 cells are 9 contiguous point ranges, their bounds loaded together; candidates stream
// 4 at a time (point + index loads in flight) into a sorted top-K keyed by (d2, index) — the same
// total order as the wave version, hence the same neighbours in the same order. For sparse
// neighbourhoods (the mapping stacks see ~10-60 candidates) this beats a wave per query.
template <int K>
__device__ __forceinline__ int thread_knn27(const float ox, const float oy, const float oz, const float inv_cell,
                                            const int gdx, const int gdy, const int gdz,
                                            const int* __restrict__ start, const float4* __restrict__ spts,
                                            const int* __restrict__ sidx, float qx, float qy, float qz, float r2,
                                            int* out_pos, float* out_d2, int* out_idx, int* ncand) {
    const int cx = (int)floorf((qx - ox) * inv_cell), cy = (int)floorf((qy - oy) * inv_cell), cz = (int)floorf((qz - oz) * inv_cell);
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, gdx - 1);
    int rb[9], re[9];
#pragma unroll
    for (int r = 0; r < 9; r++) {
        const int y = cy + (r % 3) - 1, z = cz + (r / 3) - 1;
        const bool ok = x0 <= x1 && y >= 0 && y < gdy && z >= 0 && z < gdz;
        const int c = (z * gdy + y) * gdx;
        rb[r] = load_or(start, c + x0, ok, 0);
        re[r] = load_or(start, c + x1 + 1, ok, 0);
    }
    float bd[K];
    int bi[K], bp[K];
#pragma unroll
    for (int k = 0; k < K; k++) { bd[k] = INFINITY; bi[k] = 0x7fffffff; bp[k] = -1; }
    int total = 0;
#pragma unroll
    for (int r = 0; r < 9; r++) {
        const int e = re[r];
        total += e - rb[r];
        for (int p = rb[r]; p < e; p += 4) {
            float4 v[4];
            int id[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const bool in = p + u < e;
                v[u] = load_or(spts, p + u, in, make_float4(INFINITY, INFINITY, INFINITY, 0.f));
                id[u] = load_or(sidx, p + u, in, 0x7fffffff);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const float d2 = sqdist(v[u].x, v[u].y, v[u].z, qx, qy, qz);
                if (!(d2 < r2)) continue;
                if (d2 < bd[K - 1] || (d2 == bd[K - 1] && id[u] < bi[K - 1])) {
                    float nd = d2; int ni = id[u], np = p + u;
#pragma unroll
                    for (int k = 0; k < K; k++) {
                        const bool lt = nd < bd[k] || (nd == bd[k] && ni < bi[k]);
                        if (lt) { float td = bd[k]; int ti = bi[k], tp = bp[k]; bd[k] = nd; bi[k] = ni; bp[k] = np; nd = td; ni = ti; np = tp; }
                    }
                }
            }
        }
    }
    if (ncand) *ncand = total;
    int found = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
        out_pos[k] = bp[k]; out_d2[k] = bd[k]; out_idx[k] = bi[k];
        found += bp[k] >= 0;
    }
    return found;
}
// merge of a GS-lane group's per-lane sorted top-K lists (bd, bi, bp): K rounds of a group min over
// 64-bit (d2, index) keys; every lane returns the same result
template <int K, int GS>
__device__ __forceinline__ int group_merge_topk(const float* bd, const int* bi, const int* bp, int* out_pos, float* out_d2,
                                                int* out_idx) {
    int head = 0, found = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
        float hd = INFINITY; int hi = 0x7fffffff, hp = -1;
#pragma unroll
        for (int j = 0; j < K; j++) if (j == head) { hd = bd[j]; hi = bi[j]; hp = bp[j]; }
        const unsigned long long key = hp < 0 ? ~0ull : dist_key(hd, hi);
        constexpr int NS = GS >= 64 ? 6 : GS >= 32 ? 5 : GS >= 16 ? 4 : GS >= 8 ? 3 : GS >= 4 ? 2 : GS >= 2 ? 1 : 0;
        const unsigned long long mn = allreduce_u64<NS>(key, [](unsigned long long a, unsigned long long b) { return b < a ? b : a; });
        // the owner of the minimum (unique: indices are unique) publishes its position
        const bool mine = key == mn && mn != ~0ull;
        int pos = mine ? hp : -1;
        pos = (int)allreduce_u32<NS>((unsigned)(pos + 1), [](unsigned a, unsigned b) { return a > b ? a : b; }) - 1;
        if (mine) head++;
        out_pos[k] = pos;
        out_d2[k] = mn == ~0ull ? INFINITY : __uint_as_float((unsigned)(mn >> 32));
        out_idx[k] = mn == ~0ull ? -1 : (int)(mn & 0xffffffffu);
        found += mn != ~0ull;
    }
    return found;
}
// Candidate collection riding on a group search (the mapping rounds' per-query cache): every block
// point within sqrt(r2) of the query is appended (point, grid position) at pts / pos[0, cap), group
// lanes compacting by ballot; *n ends as the number within, which may exceed cap (then the list is
// incomplete and must not be used).
struct KnnCollect { float r2; float4* pts; int* pos; int cap; };
// Exact radius k-NN of one query by a GROUP of GS aligned lanes (GS | 64) over the 3x3x3 cell
// block. The 9 row bounds are loaded together (same addresses across the group: one coalesced
// round trip) into a per-group LDS table tab[20] (row base - prefix, prefix); the rows are
// flattened, lane l streams candidates l, l+GS, ... tracking its row incrementally (candidates
// only move forward), U loads in flight, and keeps a sorted top-K by (d2, index); K rounds of a
// group min over 64-bit keys merge the lanes' lists. IDXW: the grid stores each point's original
// index in w (no second load per candidate). Same total order as the wave / thread versions;
// every lane returns the same result. COL: also collect the block points within col.r2 (above).
template <int K, int GS, bool IDXW, int U = 4, bool COL = false, int XP = 0>
__device__ __forceinline__ int group_knn27(const float ox, const float oy, const float oz, const float inv_cell,
                                           const int gdx, const int gdy, const int gdz,
                                           const int* __restrict__ start, const float4* __restrict__ spts,
                                           const int* __restrict__ sidx, float qx, float qy, float qz, float r2, bool active,
                                           int* out_pos, float* out_d2, int* out_idx, int* ncand, int* tab, int npts,
                                           const KnnCollect col = KnnCollect{0.f, nullptr, nullptr, 0}, int* ncol = nullptr,
                                           float prune = INFINITY) {
    const int gl = lane_id() & (GS - 1);
    int total;
    {
        const int cx = (int)floorf((qx - ox) * inv_cell), cy = (int)floorf((qy - oy) * inv_cell), cz = (int)floorf((qz - oz) * inv_cell);
        const int x0 = max(cx - 1, 0), x1 = min(cx + 1, gdx - 1);
        int rb[9], pre[10];
        pre[0] = 0;
#pragma unroll
        for (int r = 0; r < 9; r++) {
            const int y = cy + (r % 3) - 1, z = cz + (r / 3) - 1;
            const bool ok = active && x0 <= x1 && y >= 0 && y < gdy && z >= 0 && z < gdz;
            const int c = (z * gdy + y) * gdx;
            rb[r] = load_or(start, c + x0, ok, 0);
            pre[r + 1] = pre[r] + (load_or(start, c + x1 + 1, ok, 0) - rb[r]);
        }
        total = pre[9];
        if constexpr ((XP & 2) != 0) total = pre[9] > 1000000000 ? 1 : 0;   // (experiment: no candidate loop)
        if constexpr ((XP & 8) != 0) {
            // row bounds kept in registers: every candidate slot's position by 8 compare / select pairs on
            // them, so the U loads of a batch issue back to back (no LDS round trip between them)
#pragma unroll
            for (int r = 0; r < 9; r++) rb[r] -= pre[r];
            if (ncand) *ncand = total;
            float bd[K];
            int bi[K], bp[K];
#pragma unroll
            for (int k = 0; k < K; k++) { bd[k] = INFINITY; bi[k] = 0x7fffffff; bp[k] = -1; }
            for (int t0 = gl; t0 < total; t0 += U * GS) {
                float4 v[U];
                int ps[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int t = t0 + u * GS;
                    int o = rb[0];
#pragma unroll
                    for (int r = 1; r < 9; r++) o = t >= pre[r] ? rb[r] : o;
                    int p = t < total ? o + t : -1;
                    if ((unsigned)p >= (unsigned)npts) p = -1;                 // defensive: inconsistent index
                    ps[u] = p;
                    v[u] = load_or(spts, p, p >= 0, make_float4(INFINITY, INFINITY, INFINITY, 0.f));
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const float d2 = sqdist(v[u].x, v[u].y, v[u].z, qx, qy, qz);
                    if (!(d2 < r2) || d2 > fminf(bd[K - 1], prune)) continue;
                    const int iu = __float_as_int(v[u].w);
                    if (d2 < bd[K - 1] || iu < bi[K - 1]) {
                        float nd = d2; int ni = iu, np = ps[u];
#pragma unroll
                        for (int k = 0; k < K; k++) {
                            const bool lt = nd < bd[k] || (nd == bd[k] && ni < bi[k]);
                            if (lt) { float td = bd[k]; int ti = bi[k], tp = bp[k]; bd[k] = nd; bi[k] = ni; bp[k] = np; nd = td; ni = ti; np = tp; }
                        }
                    }
                }
            }
            return group_merge_topk<K, GS>(bd, bi, bp, out_pos, out_d2, out_idx);
        }
        __builtin_amdgcn_wave_barrier();
        if (gl == 0) {
#pragma unroll
            for (int r = 0; r < 9; r++) { tab[r] = rb[r] - pre[r]; tab[10 + r] = pre[r + 1]; }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (ncand) *ncand = total;
    float bd[K];
    int bi[K], bp[K];
#pragma unroll
    for (int k = 0; k < K; k++) { bd[k] = INFINITY; bi[k] = 0x7fffffff; bp[k] = -1; }
    int row = 0, base = tab[0], nxt = tab[10];
    int nc = 0;
    for (int t0 = gl; t0 < total; t0 += U * GS) {
        float4 v[U];
        int id[U], ps[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + u * GS;
            int p = -1;
            if (t < total) {
                while (t >= nxt && row < 8) { row++; base = tab[row]; nxt = tab[10 + row]; }
                p = base + t;
                if ((unsigned)p >= (unsigned)npts) p = -1;                   // defensive: inconsistent index
            }
            ps[u] = p;
            v[u] = load_or(spts, p, p >= 0, make_float4(INFINITY, INFINITY, INFINITY, 0.f));
            if (!IDXW) id[u] = load_or(sidx, p, p >= 0, 0x7fffffff);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const float d2 = sqdist(v[u].x, v[u].y, v[u].z, qx, qy, qz);
            if constexpr (COL) {
                // lanes still in the loop are exactly the group lanes with candidates left (the group's
                // lane 0 stays longest, so its count is complete)
                const bool take = ps[u] >= 0 && d2 < col.r2;
                const unsigned long long m = __ballot(take);
                const int gb = lane_id() & ~(GS - 1);
                const unsigned long long gm = GS == 64 ? m : (m >> gb) & ((1ull << (GS & 63)) - 1);
                const int slot = nc + __popcll(gm & ((1ull << gl) - 1));
                if (take && slot < col.cap) { col.pts[slot] = v[u]; col.pos[slot] = ps[u]; }
                nc += __popcll(gm);
            }
            // prune: an upper bound of the group's k-th distance known before the search (a candidate
            // strictly beyond it cannot enter the top k; one AT it still can, by index)
            if (!(d2 < r2) || d2 > fminf(bd[K - 1], prune)) continue;
            const int iu = IDXW ? __float_as_int(v[u].w) : id[u];
            if (d2 < bd[K - 1] || iu < bi[K - 1]) {
                float nd = d2; int ni = iu, np = ps[u];
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const bool lt = nd < bd[k] || (nd == bd[k] && ni < bi[k]);
                    if (lt) { float td = bd[k]; int ti = bi[k], tp = bp[k]; bd[k] = nd; bi[k] = ni; bp[k] = np; nd = td; ni = ti; np = tp; }
                }
            }
        }
    }
    if constexpr (COL) { if (ncol) *ncol = nc; }
    if constexpr ((XP & 4) != 0) {            // (experiment: no merge — each lane returns its own list)
        int found = 0;
#pragma unroll
        for (int k = 0; k < K; k++) { out_pos[k] = bp[k]; out_d2[k] = bd[k]; out_idx[k] = bi[k]; found += bp[k] >= 0; }
        return found;
    }
    return group_merge_topk<K, GS>(bd, bi, bp, out_pos, out_d2, out_idx);
}
// The same k-NN over an explicit candidate list (a query's collected block points, w = original
// index): lane l takes entries l, l + GS, ... (U in flight), same (d2, index) order and radius test,
// so over any list holding every point within sqrt(r2) of the query it returns group_knn27's result.
template <int K, int GS, int U>
__device__ __forceinline__ int group_knn_list(const float4* __restrict__ lpts, const int* __restrict__ lpos, int n, float qx,
                                              float qy, float qz, float r2, int* out_pos, float* out_d2, int* out_idx) {
    const int gl = lane_id() & (GS - 1);
    float bd[K];
    int bi[K], bp[K];
#pragma unroll
    for (int k = 0; k < K; k++) { bd[k] = INFINITY; bi[k] = 0x7fffffff; bp[k] = -1; }
    for (int t0 = gl; t0 < n; t0 += U * GS) {
        float4 v[U];
        int ps[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + u * GS;
            v[u] = load_or(lpts, t, t < n, make_float4(INFINITY, INFINITY, INFINITY, 0.f));
            ps[u] = load_or(lpos, t, t < n, -1);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (ps[u] < 0) continue;
            const float d2 = sqdist(v[u].x, v[u].y, v[u].z, qx, qy, qz);
            if (!(d2 < r2) || d2 > bd[K - 1]) continue;
            const int iu = __float_as_int(v[u].w);
            if (d2 < bd[K - 1] || iu < bi[K - 1]) {
                float nd = d2; int ni = iu, np = ps[u];
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const bool lt = nd < bd[k] || (nd == bd[k] && ni < bi[k]);
                    if (lt) { float td = bd[k]; int ti = bi[k], tp = bp[k]; bd[k] = nd; bi[k] = ni; bp[k] = np; nd = td; ni = ti; np = tp; }
                }
            }
        }
    }
    return group_merge_topk<K, GS>(bd, bi, bp, out_pos, out_d2, out_idx);
}
typedef float f32x2 __attribute__((ext_vector_type(2)));   // packed fp32 pair (v_pk_*_f32)
// Large-search variant of group_knn27 (aloam_knn_device, round 6): a candidate is one 64-bit key, (d2 bits
// << 32) | original index (w of the sorted copy); d2 >= 0, so unsigned key order is exactly the (d2, index)
// order of group_knn27. A lane's top K is a sorted key array updated without branches (one 64-bit compare
// and two selects per slot), entered only when some lane of the wave holds a key below its K-th; the nine
// row bounds stay in registers (a slot's position by compare / select on them, no LDS table); invalid slots
// and points outside the radius are ~0 keys. `bound`: a key known to be >= the group's final K-th (keys
// above it are dropped). Returns the group's K smallest keys (~0 = none), the same on every group lane.
// Large-search variant of group_knn27 (aloam_knn_device, round 6): a candidate is one 64-bit key, (d2 bits
// << 32) | original index (w of the sorted copy); d2 >= 0, so unsigned key order is exactly the (d2, index)
// order of group_knn27. A lane's top K is a sorted key array updated without branches (one 64-bit compare
// and two selects per slot), entered only when some lane of the wave holds a key below its K-th; the nine
// row bounds stay in registers (a slot's position by compare / select on them, no LDS table); invalid slots
// and points outside the radius are ~0 keys. `bound`: a key known to be >= the group's final K-th (keys
// above it are dropped). Returns the group's K smallest keys (~0 = none), the same on every group lane.
template <int K, int GS, int U, bool PK = true>
__device__ __forceinline__ int group_knn27_keys(const float ox, const float oy, const float oz, const float inv_cell,
                                                const int gdx, const int gdy, const int gdz, const int* __restrict__ start,
                                                const float4* __restrict__ spts, float qx, float qy, float qz, float r2,
                                                bool active, unsigned long long* out_key, int* ncand, int npts,
                                                unsigned long long bound = ~0ull) {
    const int gl = lane_id() & (GS - 1);
    const int cx = (int)floorf((qx - ox) * inv_cell), cy = (int)floorf((qy - oy) * inv_cell), cz = (int)floorf((qz - oz) * inv_cell);
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, gdx - 1);
    int off[9], pre[10];
    pre[0] = 0;
#pragma unroll
    for (int r = 0; r < 9; r++) {
        const int y = cy + (r % 3) - 1, z = cz + (r / 3) - 1;
        const bool ok = active && x0 <= x1 && y >= 0 && y < gdy && z >= 0 && z < gdz;
        const int c = (z * gdy + y) * gdx;
        const int b = load_or(start, c + x0, ok, 0);
        pre[r + 1] = pre[r] + (load_or(start, c + x1 + 1, ok, 0) - b);
        off[r] = b - pre[r];
    }
    const int total = pre[9];
    if (ncand) *ncand = total;
    unsigned long long bk[K];
#pragma unroll
    for (int k = 0; k < K; k++) bk[k] = ~0ull;
    for (int t0 = gl; t0 < total; t0 += U * GS) {
        float4 v[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = t0 + u * GS;
            int o = off[0];
#pragma unroll
            for (int r = 1; r < 9; r++) o = t >= pre[r] ? off[r] : o;
            const int p = o + t;
            ok[u] = t < total && (unsigned)p < (unsigned)npts;
            v[u] = spts[ok[u] ? p : 0];
        }
        // distances two slots at a time in packed fp32 (v_pk_add_f32 / v_pk_mul_f32: the same IEEE
        // operations in the same order as sqdist, ((dx^2 + dy^2) + dz^2), no contraction)
        float dd[U];
        if constexpr (!PK) {
#pragma unroll
            for (int u = 0; u < U; u++) dd[u] = sqdist(v[u].x, v[u].y, v[u].z, qx, qy, qz);
        } else
#pragma unroll
        for (int u = 0; u + 1 < U; u += 2) {
            const f32x2 ex = f32x2{v[u].x, v[u + 1].x} - f32x2{qx, qx};
            const f32x2 ey = f32x2{v[u].y, v[u + 1].y} - f32x2{qy, qy};
            const f32x2 ez = f32x2{v[u].z, v[u + 1].z} - f32x2{qz, qz};
            const f32x2 s = (ex * ex + ey * ey) + ez * ez;
            dd[u] = s.x;
            dd[u + 1] = s.y;
        }
        if constexpr (PK && U % 2) dd[U - 1] = sqdist(v[U - 1].x, v[U - 1].y, v[U - 1].z, qx, qy, qz);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const float d2 = dd[u];
            unsigned long long key = ((unsigned long long)__float_as_uint(d2) << 32) | (unsigned)__float_as_int(v[u].w);
            if (!(ok[u] && d2 < r2) || key > bound) key = ~0ull;
            if (__any(key < bk[K - 1])) {           // wave-uniform: the branch-free insertion below
#pragma unroll
                for (int k = K - 1; k > 0; k--) bk[k] = key < bk[k - 1] ? bk[k - 1] : (key < bk[k] ? key : bk[k]);
                bk[0] = key < bk[0] ? key : bk[0];
            }
        }
    }
    // merge: K rounds of a group min over the lanes' list heads; the owner of the minimum (unique: one
    // lane per candidate) advances its head
    int head = 0, found = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
        unsigned long long hk = ~0ull;
#pragma unroll
        for (int j = 0; j < K; j++) if (j == head) hk = bk[j];
        constexpr int NS = GS >= 64 ? 6 : GS >= 32 ? 5 : GS >= 16 ? 4 : GS >= 8 ? 3 : GS >= 4 ? 2 : GS >= 2 ? 1 : 0;
        const unsigned long long mn = allreduce_u64<NS>(hk, [](unsigned long long a, unsigned long long b) { return b < a ? b : a; });
        if (hk == mn && mn != ~0ull) head++;
        out_key[k] = mn;
        found += mn != ~0ull;
    }
    return found;
}
// v / k for a point count k in [1, 2^24), correctly rounded like the IEEE division PCL's centroid
// (Eigen "/= num_pts") does. For |x| in [2^-89, 2^90) or x == 0, v_div_scale / v_div_fmas /
// v_div_fixup in the compiler's fp32 division sequence are identities, leaving rcp, one Newton step on
// the reciprocal and two residual corrections of the quotient: that sequence is evaluated here with the
// refined reciprocal shared by the 4 components (~2.5x fewer VALU cycles; the centroid passes are
// VALU-bound on their divisions). Zero numerators are returned as is (sign of zero); anything else
// falls back to the division operator.
__device__ __noinline__ float4 div4_slow(float4 v, float d) { return make_float4(v.x / d, v.y / d, v.z / d, v.w / d); }
__device__ __forceinline__ float4 div4_by_count(float4 v, int k) {
    const float d = (float)k;
    auto in_range = [](float x) {           // biased exponent in [38, 216] (2^-89 .. 2^90), or +-0
        const unsigned b = __float_as_uint(x);
        return (((b >> 23) & 0xffu) - 38u < 179u) | ((b << 1) == 0u);
    };
    if (!(in_range(v.x) & in_range(v.y) & in_range(v.z) & in_range(v.w))) return div4_slow(v, d);
    float rc = __builtin_amdgcn_rcpf(d);
    rc = fmaf(fmaf(-d, rc, 1.0f), rc, rc);
    auto q1 = [&](float x) {
        float q = x * rc;
        q = fmaf(fmaf(-d, q, x), rc, q);
        q = fmaf(fmaf(-d, q, x), rc, q);
        return x == 0.f ? x : q;
    };
    return make_float4(q1(v.x), q1(v.y), q1(v.z), q1(v.w));
}

// Workgroup barrier that orders LDS only: __syncthreads() is also a release fence for global memory,
// so it waits for every outstanding global store (and load) of the wave first; where only LDS is
// shared across the barrier that wait is a full memory round trip for nothing.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Exclusive scan of one int per thread over a whole workgroup of NT threads (NT/64 waves):
// wave shuffle scans + one LDS round for the wave totals. Returns the exclusive prefix; *total =
// the workgroup sum (all threads). Two barriers (LDS-only ones with LDS_ONLY).
template <int NT, bool LDS_ONLY = false>
__device__ __forceinline__ int block_exscan(int v, int* total) {
    __shared__ int wsum[NT / WAVE];
    __shared__ int wtot;
    const int lane = lane_id(), w = threadIdx.x / WAVE;
    int incl = v;
    incl = wave_incl_scan(incl);
    if (lane == WAVE - 1) wsum[w] = incl;
    if (LDS_ONLY) lds_barrier(); else __syncthreads();
    if (w == 0) {
        const int x = lane < NT / WAVE ? wsum[lane] : 0;
        int xi = x;
        xi = wave_incl_scan(xi);
        if (lane < NT / WAVE) wsum[lane] = xi - x;
        if (lane == NT / WAVE - 1) wtot = xi;
    }
    if (LDS_ONLY) lds_barrier(); else __syncthreads();
    *total = wtot;
    return wsum[w] + incl - v;
}
// In-place exclusive scan of a[0, n) by one workgroup of 1024 threads (each owns a contiguous
// chunk); *total = sum. For the small "per-block count" scans.
__device__ __forceinline__ void block_scan_array(int* a, int n, int* total) {
    const int per = (n + 1023) / 1024;
    const int b0 = threadIdx.x * per, b1 = min(n, b0 + per);
    int s = 0;
    for (int i = b0; i < b1; i++) s += a[i];
    int tot;
    int run = block_exscan<1024>(s, &tot);
    for (int i = b0; i < b1; i++) { const int v = a[i]; a[i] = run; run += v; }
    if (threadIdx.x == 0 && total) *total = tot;
}
// Ascending sort of n2 (a multiple of 64) u64 keys held in LDS into out[] (LDS): every 64-key chunk is
// bitonic-sorted inside one wave (lane exchanges only), then each real key's rank is its position in
// its chunk plus, per other chunk, the number of that chunk's keys below it (chunk bounds first, else
// a 6-step binary search). No block-wide compare-exchange stages: the 2048-key bitonic network's ~60
// dependent LDS/permute stages took ~27 us per line, this ~3-5 us. Keys other than the ~0 padding must
// be distinct. Ends with a barrier.
__device__ inline void chunk_rank_sort(unsigned long long* keys, unsigned long long* out, int n2) {
    const int lane = lane_id(), wv = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    const int nch = n2 / WAVE;
    for (int c = wv; c < nch; c += nw) {
        unsigned long long v = keys[c * WAVE + lane];
#pragma unroll
        for (int size = 2; size <= WAVE; size <<= 1) {
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const unsigned long long o = __shfl_xor(v, stride, WAVE);
                const bool asc = (lane & size) == 0, lower = (lane & stride) == 0;
                v = (lower == asc) ? (v < o ? v : o) : (v < o ? o : v);
            }
        }
        keys[c * WAVE + lane] = v;
        out[c * WAVE + lane] = ~0ull;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n2; e += blockDim.x) {
        const unsigned long long x = keys[e];
        if (x == ~0ull) continue;
        const int c = e / WAVE;
        int rank = e % WAVE;
        for (int c2 = 0; c2 < nch; c2++) {
            if (c2 == c) continue;
            const unsigned long long* k = keys + c2 * WAVE;
            if (k[WAVE - 1] < x) { rank += WAVE; continue; }
            if (!(k[0] < x)) continue;
            int lo = 0;
#pragma unroll
            for (int st = WAVE / 2; st >= 1; st >>= 1)
                if (k[lo + st - 1] < x) lo += st;
            rank += lo;
        }
        out[rank] = x;
    }
    __syncthreads();
}

// Block bitonic sort of n2 (power of two, 256 <= n2 <= 4 * blockDim.x, blockDim.x = 1024) u64 keys held in LDS, ascending.
// Thread t keeps positions 4t..4t+3 in registers: strides 1-2 are in-thread, strides 4-128 are
// lane exchanges inside the wave (__shfl_xor), only strides >= 256 go through LDS + barriers
// (10 barrier steps for 4096 keys instead of 78).
__device__ __forceinline__ void cmpx(unsigned long long& a, unsigned long long& b, bool asc) {
    const unsigned long long lo = a < b ? a : b, hi = a < b ? b : a;
    a = asc ? lo : hi;
    b = asc ? hi : lo;
}
__device__ inline void bitonic_sort_reg4(unsigned long long* k, int n2) {
    const int t = threadIdx.x;
    const bool act = 4 * t < n2;
    unsigned long long v[4];
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = act ? k[4 * t + r] : ~0ull;
    for (int size = 2; size <= n2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 256) {
                __syncthreads();
                if (act) {
#pragma unroll
                    for (int r = 0; r < 4; r++) k[4 * t + r] = v[r];
                }
                __syncthreads();
                if (act) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int g = 4 * t + r;
                        const unsigned long long o = k[g ^ stride];
                        const bool asc = (g & size) == 0, lower = (g & stride) == 0;
                        const unsigned long long mn = v[r] < o ? v[r] : o, mx = v[r] < o ? o : v[r];
                        v[r] = (lower == asc) ? mn : mx;
                    }
                }
            } else if (stride >= 4) {
                const int lo = stride >> 2;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int g = 4 * t + r;
                    const unsigned long long o = __shfl_xor(v[r], lo, WAVE);
                    const bool asc = (g & size) == 0, lower = (g & stride) == 0;
                    const unsigned long long mn = v[r] < o ? v[r] : o, mx = v[r] < o ? o : v[r];
                    v[r] = (lower == asc) ? mn : mx;
                }
            } else if (stride == 2) {
                const bool asc = ((4 * t) & size) == 0;
                cmpx(v[0], v[2], asc);
                cmpx(v[1], v[3], asc);
            } else {
                const bool asc0 = ((4 * t) & size) == 0, asc1 = ((4 * t + 2) & size) == 0;
                cmpx(v[0], v[1], asc0);
                cmpx(v[2], v[3], asc1);
            }
        }
    }
    __syncthreads();
    if (act) {
#pragma unroll
        for (int r = 0; r < 4; r++) k[4 * t + r] = v[r];
    }
    __syncthreads();
}

// Ascending sort of n64 (a multiple of 64) distinct keys in LDS (GLOBAL: in global scratch, full
// barriers): every 64-key chunk is bitonic-sorted inside one wave (lane exchanges only), then
// log2(n64 / 64) merge rounds ping-pong between a[] and b[], each thread producing IPT consecutive
// outputs of one pair of runs per step after one binary search along the merge path. Returns the
// buffer holding the result; ends with a barrier. O(n log n): ~4 us for 4096 u64 keys where a rank sort's O(n^2 / 64) took ~26 us.
template <typename T, int IPT, bool GLOBAL = false>
__device__ inline T* block_merge_sort(T* a, T* b, int n64) {
    static_assert(IPT <= 2 * WAVE && (IPT & (IPT - 1)) == 0, "outputs of a thread stay inside one pair of runs");
    const int lane = lane_id(), wv = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    for (int c = wv; c < n64 / WAVE; c += nw) {
        T v = a[c * WAVE + lane];
#pragma unroll
        for (int size = 2; size <= WAVE; size <<= 1) {
#pragma unroll
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                const T o = __shfl_xor(v, stride, WAVE);
                const bool asc = (lane & size) == 0, lower = (lane & stride) == 0;
                v = (lower == asc) ? (v < o ? v : o) : (v < o ? o : v);
            }
        }
        a[c * WAVE + lane] = v;
    }
    if (GLOBAL) __syncthreads(); else lds_barrier();
    T* src = a;
    T* dst = b;
    for (int L = WAVE; L < n64; L <<= 1) {
        for (int t0 = IPT * threadIdx.x; t0 < n64; t0 += IPT * blockDim.x) {
            const int s = t0 / (2 * L) * (2 * L);
            const int la = min(L, n64 - s), lb = max(0, min(L, n64 - s - L));
            const T* A = src + s;
            const T* Bv = src + s + L;
            const int k0 = t0 - s;
            int lo = max(0, k0 - lb), hi = min(k0, la);
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (A[mid] < Bv[k0 - 1 - mid]) lo = mid + 1; else hi = mid;
            }
            int i = lo, j = k0 - lo;
#pragma unroll
            for (int u = 0; u < IPT; u++) {
                const bool ta = i < la && (j >= lb || A[i] < Bv[j]);
                dst[t0 + u] = ta ? A[i] : Bv[j];
                if (ta) i++; else j++;
            }
        }
        if (GLOBAL) __syncthreads(); else lds_barrier();
        T* tmp = src; src = dst; dst = tmp;
    }
    return src;
}
// PCL 1.8 VoxelGrid leaf grid from an ordered-int bbox (voxel_grid.cpp applyFilter)
__device__ inline void voxel_params(const unsigned* bb, float leaf, bool* overflow, int minb[3], int* mul1, int* mul2) {
    const float inv = 1.0f / leaf;
    float mn[3], mx[3];
    for (int a = 0; a < 3; a++) { mn[a] = ord2f(bb[a]); mx[a] = ord2f(bb[3 + a]); }
    long long dx = (long long)((mx[0] - mn[0]) * inv) + 1;
    long long dy = (long long)((mx[1] - mn[1]) * inv) + 1;
    long long dz = (long long)((mx[2] - mn[2]) * inv) + 1;
    *overflow = dx * dy * dz > 2147483647LL;
    int divb[3];
    for (int a = 0; a < 3; a++) {
        minb[a] = (int)floorf(mn[a] * inv);
        int maxb = (int)floorf(mx[a] * inv);
        divb[a] = maxb - minb[a] + 1;
    }
    *mul1 = divb[0];
    *mul2 = divb[0] * divb[1];
}
__device__ inline unsigned voxel_index(float4 p, float inv, const int minb[3], int mul1, int mul2) {
    int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
    int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
    int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
    return (unsigned)(i0 + i1 * mul1 + i2 * mul2);
}
}  // namespace aloam
