// k_odom.hip — laserOdometry correspondence search on gfx950 (src/laserOdometry.cpp:380-561).
//
// One wave per feature point (sharp points, then flat points):
//   1. TransformToStart (:154-172, DISTORTION 0 => s = 1) in double, stored as float
//   2. exact 1-NN in the last less-sharp / less-flat cloud within d^2 < 25 (grid, k_grid.hip)
//   3. the reference's scan-line window search, forward then backward from the closest point,
//      64 candidates per step: break index by ballot, first-occurrence minimum by a 64-bit
//      (d^2, order) wave-min, strict '<' against the running minimum (init 25) exactly like :400-441
//   4. LidarEdgeFactor / LidarPlaneFactor residual block written to the point's factor slot
#include "aloam_device.hpp"
#include "aloam_internal.hpp"

#ifndef ODOM_U
#define ODOM_U 4   // candidate loads in flight per lane in the 1-NN and window searches
#endif
namespace aloam {
#ifdef ALOAM_WSTAMP_ODOM
WSTAMP_DEFINE_TABLE
#define WSTAMP(k) WSTAMP_ON(k)
#else
#define WSTAMP(k) do { } while (0)
#endif

// Exact 1-NN of one query by one wave over the (2m+1)^3 cell block of a grid: every lane keeps the
// (d^2, original index) minimum of the candidates it streams (4 points + 4 indices in flight), one
// 64-bit wave-min merges them, and the winning lane hands out the point itself (its w = intensity,
// i.e. the scan line), so the caller needs no reload of the closest point.
template <int MAXR>
__device__ __forceinline__ bool wave_nn_rows(const GridDesc& gd, const int* __restrict__ start, const float4* __restrict__ spts,
                                             const int* __restrict__ sidx, float qx, float qy, float qz, float r2, int m,
                                             int* out_idx, float* out_d2, float4* out_pt, RowSet<MAXR>& rs) {
    const int lane = lane_id();
    const int total = build_rows<MAXR>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, start, qx, qy, qz, m, rs);
    unsigned long long best = ~0ull;
    float4 bp = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int t0 = 0; t0 < total; t0 += ODOM_U * WAVE) {
        int pp[ODOM_U], id[ODOM_U];
        float4 vv[ODOM_U];
#pragma unroll
        for (int u = 0; u < ODOM_U; u++) {
            const int t = t0 + u * WAVE + lane;
            const int pos = row_pos<MAXR>(rs, min(t, total - 1));
            pp[u] = t < total ? pos : -1;
            vv[u] = load_or(spts, pp[u], pp[u] >= 0, make_float4(0, 0, 0, 0));
            id[u] = load_or(sidx, pp[u], pp[u] >= 0, 0);
        }
#pragma unroll
        for (int u = 0; u < ODOM_U; u++) {
            const float d2 = sqdist(vv[u].x, vv[u].y, vv[u].z, qx, qy, qz);
            const unsigned long long key = dist_key(d2, id[u]);
            if (pp[u] >= 0 && d2 < r2 && key < best) { best = key; bp = vv[u]; }
        }
    }
    const unsigned long long mn = wave_min_u64(best);
    if (mn == ~0ull) return false;
    const int w = __ffsll((long long)__ballot(best == mn)) - 1;
    *out_idx = (int)(mn & 0xffffffffu);
    *out_d2 = __uint_as_float((unsigned)(mn >> 32));
    *out_pt = make_float4(readlane_f(bp.x, w), readlane_f(bp.y, w), readlane_f(bp.z, w), readlane_f(bp.w, w));
    return true;
}

// Exact 1-NN within d^2 < 25 (laserOdometry.cpp:386-389) in up to three phases: the query cell's 3x3x3
// block of a grid with cells of edge g holds every point closer than g, so a best distance < 0.99 g
// found there is final. Phase 1 uses the fine grid (most neighbours lie within a fraction of a metre),
// phase 2 the 2.56 m grid's 3x3x3 block, phase 3 its 5x5x5 block (>= 2g = 5.1 m around the query).
struct OdomGrid { const GridDesc* d; const int* cs; const float4* sp; const int* si; };
__device__ inline int wave_nn1(const OdomGrid& fine, const OdomGrid& coarse, float qx, float qy, float qz, int* out_idx,
                               float* out_d2, float4* out_pt, RowSet<9>& r9, RowSet<25>& r25) {
    const GridDesc gf = *fine.d, gc = *coarse.d;
    if (gf.cell < gc.cell) {
        const float acc = 0.99f * gf.cell;
        if (wave_nn_rows<9>(gf, fine.cs, fine.sp, fine.si, qx, qy, qz, 25.0f, 1, out_idx, out_d2, out_pt, r9) && *out_d2 < acc * acc)
            return 1;
    }
    const float acc = 0.99f * gc.cell;
    if (wave_nn_rows<9>(gc, coarse.cs, coarse.sp, coarse.si, qx, qy, qz, 25.0f, 1, out_idx, out_d2, out_pt, r9) && *out_d2 < acc * acc)
        return 1;
    return wave_nn_rows<25>(gc, coarse.cs, coarse.sp, coarse.si, qx, qy, qz, 25.0f, 2, out_idx, out_d2, out_pt, r25) ? 1 : 0;
}

__device__ inline int line_of(float intensity) { return int(intensity); }

// forward/backward scan-line search of laserOdometry.cpp:400-441 (corner) / :483-532 (surf)
// mode 0 = corner (one candidate set), 1 = surf (two sets).
// Processes 4 chunks of 64 candidates per step (4 coalesced loads in flight per lane); the break
// index is the first flagged position in scan order over the 256, so results equal the serial loop.
template <int MODE>
__device__ inline void window_search(const float4* __restrict__ cl, int n, int closest, int cid, float sx, float sy, float sz,
                                     int* ind2, int* ind3) {
    const int lane = lane_id();
    constexpr int U = 4;
    float best2 = 25.0f, best3 = 25.0f;
    int i2 = -1, i3 = -1;
    // ---- forward (increasing index) ----
    for (int base = closest + 1; base < n; base += U * WAVE) {
        float4 p[U];
        int line[U];
        unsigned long long bm[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int j = base + u * WAVE + lane;
            p[u] = load_or(cl, j, j < n, make_float4(0, 0, 0, 0));
        }
        int first_brk = 0x7fffffff;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int j = base + u * WAVE + lane;
            line[u] = line_of(p[u].w);
            bm[u] = __ballot(j < n && (line[u] > (cid + 2.5)));
            if (bm[u] && first_brk == 0x7fffffff) first_brk = base + u * WAVE + (__ffsll((long long)bm[u]) - 1);
        }
        unsigned long long k2 = ~0ull, k3 = ~0ull;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int j = base + u * WAVE + lane;
            const bool live = j < n && j < first_brk;
            const float d = sqdist(p[u].x, p[u].y, p[u].z, sx, sy, sz);
            const unsigned long long key = dist_key(d, j);
            if (MODE == 0) { if (live && !(line[u] <= cid) && key < k2) k2 = key; }
            else {
                if (live && line[u] <= cid && key < k2) k2 = key;
                if (live && line[u] > cid && key < k3) k3 = key;
            }
        }
        k2 = wave_min_u64(k2);
        if (k2 != ~0ull) { float dm = __uint_as_float((unsigned)(k2 >> 32)); if (dm < best2) { best2 = dm; i2 = (int)(k2 & 0xffffffffu); } }
        if (MODE == 1) {
            k3 = wave_min_u64(k3);
            if (k3 != ~0ull) { float dm = __uint_as_float((unsigned)(k3 >> 32)); if (dm < best3) { best3 = dm; i3 = (int)(k3 & 0xffffffffu); } }
        }
        if (first_brk != 0x7fffffff) break;
    }
    // ---- backward (decreasing index): first occurrence = largest index among equal distances ----
    for (int base = closest - 1; base >= 0; base -= U * WAVE) {
        float4 p[U];
        int line[U];
        unsigned long long bm[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int j = base - u * WAVE - lane;
            p[u] = load_or(cl, j, j >= 0, make_float4(0, 0, 0, 0));
        }
        int first_brk = -1;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int j = base - u * WAVE - lane;
            line[u] = line_of(p[u].w);
            bm[u] = __ballot(j >= 0 && (line[u] < (cid - 2.5)));
            if (bm[u] && first_brk == -1) first_brk = base - u * WAVE - (__ffsll((long long)bm[u]) - 1);
        }
        unsigned long long k2 = ~0ull, k3 = ~0ull;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int j = base - u * WAVE - lane;
            const bool live = j >= 0 && j > first_brk;
            const float d = sqdist(p[u].x, p[u].y, p[u].z, sx, sy, sz);
            const unsigned long long key = dist_key(d, (int)(0x7fffffffu - (unsigned)j));
            if (MODE == 0) { if (live && !(line[u] >= cid) && key < k2) k2 = key; }
            else {
                if (live && line[u] >= cid && key < k2) k2 = key;
                if (live && line[u] < cid && key < k3) k3 = key;
            }
        }
        k2 = wave_min_u64(k2);
        if (k2 != ~0ull) { float dm = __uint_as_float((unsigned)(k2 >> 32)); if (dm < best2) { best2 = dm; i2 = (int)(0x7fffffffu - (unsigned)(k2 & 0xffffffffu)); } }
        if (MODE == 1) {
            k3 = wave_min_u64(k3);
            if (k3 != ~0ull) { float dm = __uint_as_float((unsigned)(k3 >> 32)); if (dm < best3) { best3 = dm; i3 = (int)(0x7fffffffu - (unsigned)(k3 & 0xffffffffu)); } }
        }
        if (first_brk != -1) break;
    }
    *ind2 = i2;
    *ind3 = i3;
}

// The same window search through the grid. When the last cloud is ordered by scan line (it is
// built line by line: laserOdometry.cpp:627-641 takes scanRegistration's per-line output), the
// scan from `closest` visits exactly: forward = {j > closest, line in [c, c+2]}, backward =
// {j < closest, line in [c-2, c]} (the break fires at the first line outside). Only points with
// d^2 < 25 can win (the running minimum starts at 25), and those lie in the 5x5 (x, y) block of
// 2.56 m cells of their line's layer. Per set, the first occurrence of the minimum in scan order is the (d^2, j) minimum going
// forward and the (d^2, -j) minimum going backward; backward replaces forward only when strictly
// closer — the serial loop's result, without walking whole scan lines.
// Rows of the scan-line-layered grid (2-D cells per line: one z cell, a scan line being a thin
// cone) for the lines lo..hi around the query: per line 5 y-rows of the x-cells cx-2..cx+2, so the
// rows hold every point of those lines within the 2 cells (>= 5.1 m) of the query in x and y — a
// superset of the d < 5 m candidates. <= 25 rows, one lane each, one round trip.
__device__ __forceinline__ int build_rows_layers(const GridDesc& gd, const int* __restrict__ start, float qx, float qy,
                                                 int lo, int hi, int skip, RowSet<32>& rs) {
    const int lane = lane_id();
    const int cx = (int)floorf((qx - gd.ox) * gd.inv_cell), cy = (int)floorf((qy - gd.oy) * gd.inv_cell);
    const int x0 = max(cx - 2, 0), x1 = min(cx + 2, gd.dx - 1);
    const int nrow = (hi - lo + 1) * 5;
    const int L = lo + lane / 5, y = cy - 2 + lane % 5;
    const bool ok = lane < nrow && L != skip && L >= 0 && L < gd.nlayers && x0 <= x1 && y >= 0 && y < gd.dy;
    const int c = (L * gd.dz * gd.dy + y) * gd.dx;
    const int bb = load_or(start, c + x0, ok, 0);
    const int len = load_or(start, c + x1 + 1, ok, 0) - bb;
    const int inc = wave_incl_scan(len);
    const int nr = min(nrow, 32);
    __builtin_amdgcn_wave_barrier();
    if (lane < nr) { rs.b[lane] = bb; rs.pre[lane + 1] = inc; }
    if (lane == 0) { rs.pre[0] = 0; rs.nr = nr; }
    const int total = readlane_i(inc, nr - 1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return total;
}

// The same window search through the scan-line-layered grid. When the last cloud is ordered by
// scan line (it is built line by line: laserOdometry.cpp:627-641 takes scanRegistration's
// per-line output), the serial scan from `closest` visits exactly: forward = {j > closest, line
// in [c, c+2]}, backward = {j < closest, line in [c-2, c]} (its break fires at the first line
// outside). Only points with d^2 < 25 can win (the running minimum starts at 25), and those lie in
// the 5x5 (x, y) block of >= 2.56 m cells of their own line's layer. Per set, the first occurrence of
// the minimum in scan order is the (d^2, j) minimum going forward and the (d^2, -j) minimum going
// backward; backward replaces forward only when strictly closer — the serial loop's result.
template <int MODE>
__device__ inline void grid_window(const OdomGrid& wg, int closest, int cid, float sx, float sy, float sz,
                                   int* ind2, int* ind3, float4* p2, float4* p3, RowSet<32>& rs) {
    const int lane = lane_id();
    const GridDesc gd = *wg.d;
    const int total = build_rows_layers(gd, wg.cs, sx, sy, cid - 2, cid + 2, MODE == 0 ? cid : -1000, rs);
    // sets: 0 = fwd ind2, 1 = bwd ind2, 2 = fwd ind3, 3 = bwd ind3 (corner: ind2 sets only); each lane
    // keeps its minimum key per set and that candidate's point
    constexpr int NSET = MODE == 0 ? 2 : 4;
    unsigned long long k[NSET];
    float4 kp[NSET];
#pragma unroll
    for (int s = 0; s < NSET; s++) { k[s] = ~0ull; kp[s] = make_float4(0.f, 0.f, 0.f, 0.f); }
    for (int t0 = 0; t0 < total; t0 += ODOM_U * WAVE) {
        int pp[ODOM_U];
        float4 vv[ODOM_U];
        int jj[ODOM_U];
#pragma unroll
        for (int u = 0; u < ODOM_U; u++) {
            const int t = t0 + u * WAVE + lane;
            const int pos = row_pos<32>(rs, min(t, total - 1));
            pp[u] = t < total ? pos : -1;
            vv[u] = load_or(wg.sp, pp[u], pp[u] >= 0, make_float4(0, 0, 0, 0));
            jj[u] = load_or(wg.si, pp[u], pp[u] >= 0, 0);
        }
#pragma unroll
        for (int u = 0; u < ODOM_U; u++) {
            if (pp[u] < 0) continue;
            const float d = sqdist(vv[u].x, vv[u].y, vv[u].z, sx, sy, sz);
            if (!(d < 25.0f)) continue;
            const int line = line_of(vv[u].w), j = jj[u];
            const bool fwd = j > closest, bwd = j < closest;
            if (!fwd && !bwd) continue;
            const unsigned long long kf = dist_key(d, j), kb = dist_key(d, (int)(0x7fffffffu - (unsigned)j));
            bool t[NSET];
            if (MODE == 0) {
                t[0] = fwd && line > cid && line <= cid + 2 && kf < k[0];
                t[1] = bwd && line < cid && line >= cid - 2 && kb < k[1];
            } else {
                t[0] = fwd && line == cid && kf < k[0];
                t[1] = bwd && line == cid && kb < k[1];
                t[2] = fwd && line > cid && line <= cid + 2 && kf < k[2];
                t[3] = bwd && line < cid && line >= cid - 2 && kb < k[3];
            }
#pragma unroll
            for (int s = 0; s < NSET; s++)
                if (t[s]) { k[s] = (s & 1) ? kb : kf; kp[s] = vv[u]; }
        }
    }
    int res[2] = {-1, -1};
    float4 rp[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
#pragma unroll
    for (int s = 0; s < NSET / 2; s++) {
        const unsigned long long f = wave_min_u64(k[2 * s]), b = wave_min_u64(k[2 * s + 1]);
        float best = 25.0f;
        int idx = -1, from = -1;
        if (f != ~0ull) { best = __uint_as_float((unsigned)(f >> 32)); idx = (int)(f & 0xffffffffu); from = 0; }
        if (b != ~0ull && __uint_as_float((unsigned)(b >> 32)) < best) { idx = (int)(0x7fffffffu - (unsigned)(b & 0xffffffffu)); from = 1; }
        if (from >= 0) {   // the winning lane hands out its point (wave-uniform branch)
            const unsigned long long won = from == 0 ? f : b;
            const float4 mine = from == 0 ? kp[2 * s] : kp[2 * s + 1];
            const int w = __ffsll((long long)__ballot((from == 0 ? k[2 * s] : k[2 * s + 1]) == won)) - 1;
            rp[s] = make_float4(readlane_f(mine.x, w), readlane_f(mine.y, w), readlane_f(mine.z, w), readlane_f(mine.w, w));
        }
        res[s] = idx;
    }
    *ind2 = res[0];
    *ind3 = res[1];
    *p2 = rp[0];
    *p3 = rp[1];
}

// 1 if the cloud's scan line (int(intensity)) never decreases with the index
__global__ void k_line_sorted(const float4* __restrict__ a, const int* na, const float4* __restrict__ b, const int* nb_,
                              int* flag) {
    const float4* cl = blockIdx.y == 0 ? a : b;
    const int n = blockIdx.y == 0 ? *na : *nb_;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j + 1 < n; j += gridDim.x * blockDim.x)
        if (line_of(cl[j + 1].w) < line_of(cl[j].w)) flag[blockIdx.y] = 0;
}

// the six search grids of the last clouds: 1-NN (coarse, fine) and scan-line window, corner and surf
struct OdomGrids { OdomGrid nn_c, nn_s, fine_c, fine_s, win_c, win_s; };

__device__ __forceinline__ void odom_query(int qi, int n_sharp,
    const float4* __restrict__ sharp, const float4* __restrict__ flat,
    const float4* __restrict__ corner_last, int n_cl, const float4* __restrict__ surf_last, int n_sl,
    const OdomGrids& G, const OdomState* __restrict__ odom, aloam_factor* __restrict__ out, int* round_cnt,
    const int* line_sorted, RowSet<9>& r9, RowSet<25>& r25, RowSet<32>& r32, int exp) {
    const int lane = lane_id();
    const bool is_corner = qi < n_sharp;
    const float4 pi = is_corner ? sharp[qi] : flat[qi - n_sharp];
    // TransformToStart (:154-172)
    const dquat q{odom->para[0], odom->para[1], odom->para[2], odom->para[3]};
    const dquat ql = qslerp_identity(1.0, q);
    const dvec3 r = qrot(ql, {pi.x, pi.y, pi.z});
    const float sx = (float)(r.x + 1.0 * odom->para[4]);
    const float sy = (float)(r.y + 1.0 * odom->para[5]);
    const float sz = (float)(r.z + 1.0 * odom->para[6]);
    WSTAMP(2);
    aloam_factor f;
    f.type = -1; f.pad = 0;
    f.cp[0] = pi.x; f.cp[1] = pi.y; f.cp[2] = pi.z;
    const float4* cl = is_corner ? corner_last : surf_last;
    const int n = is_corner ? n_cl : n_sl;
    int closest = -1;
    float d2 = 0.f;
    float4 pc = make_float4(0.f, 0.f, 0.f, 0.f);   // the closest point (cl[closest])
    int found;
    if (exp & 1) { found = n > 0; closest = (qi * 37) % max(n, 1); pc = cl[closest]; }
    else if (is_corner) found = n > 0 ? wave_nn1(G.fine_c, G.nn_c, sx, sy, sz, &closest, &d2, &pc, r9, r25) : 0;
    else found = n > 0 ? wave_nn1(G.fine_s, G.nn_s, sx, sy, sz, &closest, &d2, &pc, r9, r25) : 0;
    if (exp & 2) found = 0;
    WSTAMP(3);
    if (found) {
        const int cid = line_of(pc.w);
        int i2, i3;
        float4 p2, p3;
        const bool by_grid = line_sorted[is_corner ? 0 : 1] != 0;
        if (is_corner) {
            if (by_grid) grid_window<0>(G.win_c, closest, cid, sx, sy, sz, &i2, &i3, &p2, &p3, r32);
            else { window_search<0>(cl, n, closest, cid, sx, sy, sz, &i2, &i3); if (i2 >= 0) p2 = cl[i2]; }
            if (i2 >= 0) {
                f.type = 0;
                f.a[0] = pc.x; f.a[1] = pc.y; f.a[2] = pc.z;
                f.b[0] = p2.x; f.b[1] = p2.y; f.b[2] = p2.z;
            }
        } else {
            if (by_grid) grid_window<1>(G.win_s, closest, cid, sx, sy, sz, &i2, &i3, &p2, &p3, r32);
            else {
                window_search<1>(cl, n, closest, cid, sx, sy, sz, &i2, &i3);
                if (i2 >= 0 && i3 >= 0) { p2 = cl[i2]; p3 = cl[i3]; }
            }
            if (i2 >= 0 && i3 >= 0) {
                // LidarPlaneFactor ctor (lidarFactor.hpp:64-65)
                dvec3 jj{pc.x, pc.y, pc.z}, ll{p2.x, p2.y, p2.z}, mm{p3.x, p3.y, p3.z};
                dvec3 nn = dcross({jj.x - ll.x, jj.y - ll.y, jj.z - ll.z}, {jj.x - mm.x, jj.y - mm.y, jj.z - mm.z});
                double z = nn.x * nn.x + nn.y * nn.y + nn.z * nn.z;
                if (z > 0) { double s = sqrt(z); nn = {nn.x / s, nn.y / s, nn.z / s}; }
                f.type = 1;
                f.a[0] = jj.x; f.a[1] = jj.y; f.a[2] = jj.z;
                f.b[0] = nn.x; f.b[1] = nn.y; f.b[2] = nn.z;
            }
        }
    }
    WSTAMP(4);
    if (lane == 0) {
        out[qi] = f;
        // per-round counters spread over ODOM_CNT_SLOTS cache lines (summed by k_odom_compose): one
        // address taking every wave's atomic cost ~9 us per round (measured)
        if (f.type >= 0) atomicAdd(&round_cnt[(qi & (ODOM_CNT_SLOTS - 1)) * ODOM_CNT_STRIDE + (is_corner ? 0 : 1)], 1);
    }
}

// One wave per feature point, grid-stride over the points: the counts come from the device
// (n_q[0] sharp, n_q[1] flat; n_last[0..1] last-cloud sizes), so the launch configuration is
// fixed and the round loop can be replayed as a graph.
__global__ void __launch_bounds__(256) k_odom_search(
    const float4* __restrict__ sharp, const float4* __restrict__ flat, const int* __restrict__ n_q,
    const float4* __restrict__ corner_last, const float4* __restrict__ surf_last, const int* __restrict__ n_last,
    const OdomGrids G, const OdomState* __restrict__ odom, aloam_factor* __restrict__ out, int* round_cnt,
    const int* line_sorted, int exp) {
    __shared__ RowSet<9> rows9[256 / WAVE];
    __shared__ RowSet<25> rows25[256 / WAVE];
    __shared__ RowSet<32> rows32[256 / WAVE];
    WSTAMP(0);
    const int n_sharp = n_q[0], nq = n_q[0] + n_q[1];
    const int n_cl = n_last[0], n_sl = n_last[1];
    const int w = threadIdx.x / WAVE;
    WSTAMP(1);
    for (int qi = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE; qi < nq; qi += gridDim.x * (blockDim.x / WAVE))
        odom_query(qi, n_sharp, sharp, flat, corner_last, n_cl, surf_last, n_sl, G, odom, out, round_cnt, line_sorted,
                   rows9[w], rows25[w], rows32[w], exp);
    WSTAMP(5);
}

// t_w += q_w * t_lc ; q_w = q_w * q_lc   (laserOdometry.cpp:581-582); threads 0..2R-1 first fold the
// spread correspondence counters of the R rounds into round_cnt. Also writes the next scan's
// last-cloud counts (last_n) and re-arms the line-order flags: the caller must follow it with
// build_last_grids(C, true) (odom_last_sorted with flags_preset), which relies on both.
__global__ void k_odom_compose(OdomState* o, int* __restrict__ spread, int rounds, int* round_cnt, int* last_n, int lc, int ls,
                               const int* dcnt, int* last_sorted) {
    if ((int)threadIdx.x < 2 * rounds) {
        const int r = threadIdx.x >> 1, t = threadIdx.x & 1;
        const int* b = spread + (size_t)r * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE + t;
        int sum = 0;
        for (int k = 0; k < ODOM_CNT_SLOTS; k++) sum += b[k * ODOM_CNT_STRIDE];
        round_cnt[2 * r + t] = sum;
    }
    __syncthreads();   // then re-zero the counters for the next scan (no memset launch on the front)
    for (int i = threadIdx.x; i < rounds * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE; i += blockDim.x) spread[i] = 0;
    if (threadIdx.x != 0) return;
    // the next scan's last-cloud counts and the line-order flags k_line_sorted clears (two k_set2 launches
    // fewer on the front stage; the rounds above already read the previous counts)
    last_n[0] = dcnt ? dcnt[2] : lc; last_n[1] = dcnt ? dcnt[4] : ls;   // scanRegistration's less-sharp / less-flat counts
    last_sorted[0] = 1; last_sorted[1] = 1;
    dquat qw{o->q_w[0], o->q_w[1], o->q_w[2], o->q_w[3]};
    dquat ql{o->para[0], o->para[1], o->para[2], o->para[3]};
    dvec3 r = qrot(qw, {o->para[4], o->para[5], o->para[6]});
    o->t_w[0] = o->t_w[0] + r.x; o->t_w[1] = o->t_w[1] + r.y; o->t_w[2] = o->t_w[2] + r.z;
    dquat n = qmul(qw, ql);
    o->q_w[0] = n.x; o->q_w[1] = n.y; o->q_w[2] = n.z; o->q_w[3] = n.w;
}

static const int g_odom_exp = getenv("ALOAM_ODOM_EXP") ? atoi(getenv("ALOAM_ODOM_EXP")) : 0;   // profiling experiments only
// fixed launch: one wave per possible feature point (caps 12 sharp + 24 flat per line); waves past
// the device-side count exit at once
void odom_round_search(Ctx& C, int round) {
    const int threads = 256;
    // upper bound of the live queries: this context's scan lines x the per-line selection caps (the
    // counts themselves are on the device, so the launch stays graph-replayable)
    const int lines = std::max(1, std::min(MAXL, C.P.scan_line));
    const int nb = (lines * (LINE_SHARP_CAP + LINE_FLAT_CAP) * WAVE + threads - 1) / threads;
    auto og = [](const Grid& g) { return OdomGrid{g.desc, g.cell_start, g.pts, g.idx}; };
    const OdomGrids G{og(C.g_corner_last), og(C.g_surf_last), og(C.g_corner_fine), og(C.g_surf_fine), og(C.g_corner_win),
                      og(C.g_surf_win)};
    k_odom_search<<<nb, threads, 0, C.stream>>>(
        C.d_sharp, C.d_flat, C.d_odom_nq, C.d_corner_last, C.d_surf_last, C.d_last_n, G,
        C.d_odom, C.d_factors, C.d_odom_spread + (size_t)round * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE, C.d_last_sorted, g_odom_exp);
    HIPCHK(hipGetLastError());
}

// after the last clouds change: whether each is ordered by scan line (selects grid_window).
// flags_preset: the flags were re-armed to 1 by k_odom_compose just before (odom_compose and
// build_last_grids(C, true) always come as a pair); otherwise they are re-armed here.
void odom_last_sorted(Ctx& C, bool flags_preset) {
    if (!flags_preset) set_counts2(C, C.d_last_sorted, 1, 1);
    k_line_sorted<<<dim3(64, 2), 256, 0, C.stream>>>(C.d_corner_last, C.d_last_n + 0, C.d_surf_last, C.d_last_n + 1, C.d_last_sorted);
    HIPCHK(hipGetLastError());
}

void odom_compose(Ctx& C, int lc, int ls, const int* dcnt) {
    k_odom_compose<<<1, 64, 0, C.stream>>>(C.d_odom, C.d_odom_spread, std::min(C.P.odom_rounds, ALOAM_MAX_ROUNDS), C.d_round_cnt,
                                           C.d_last_n, lc, ls, dcnt, C.d_last_sorted);
    HIPCHK(hipGetLastError());
}

}  // namespace aloam
