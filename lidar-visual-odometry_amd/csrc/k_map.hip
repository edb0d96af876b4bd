// k_map.hip — laserMapping on gfx950 (src/laserMapping.cpp:305-848).
//
// Map layout in HBM: per feature kind (corner / surf) one float4 array + one cube-id array, kept
// sorted by cube id (21x21x11 cubes of 50 m, laserMapping.cpp:74-82) with each cube's points in the
// reference's per-cube order (filtered points in leaf order, then appended points in stack order).
// A cube recentring (:325-507) is a uniform shift of cube ids, so it never reorders a cube's points.
//
//   map_prepare      transformAssociateToMap, centre cube, recentring shift, 5x5x3 surrounding cubes
//   map_shift        apply the recentring to every map point's cube id (dropping wrapped cubes)
//   grid_build x2    FromMap grids over the points of the surrounding cubes (k_grid.hip)
//   map_gate         the "corner > 10 && surf > 50" test (:554)
//   stacks           VoxelGrid of corner_last (0.4) / surf_last (0.8) (k_voxel.hip)
//   10 rounds of     map_knn5 (wave per stack point) -> map_fit (thread per point: centre /
//                    covariance / SelfAdjointEigenSolver, or 5x3 ColPivHouseholderQR plane) -> LM
//   map_update       transformUpdate (:148-152)
//   insert + rebuild append the stacks to their cubes, counting-sort the map by cube, per-cube
//                    VoxelGrid of the surrounding cubes (:737-801)
#include <cstring>

#include "aloam_device.hpp"
#include "aloam_internal.hpp"
#include "eigen_small.hpp"
#include "ls_sort.hpp"
#include "rvg.hpp"

namespace aloam {
#ifdef ALOAM_WSTAMP_MAP      // k_map_assoc phases of round ALOAM_WSTAMP_MAP (profiling builds only)
WSTAMP_DEFINE_TABLE
#define WSTAMP(k) do { if (wst_round == ALOAM_WSTAMP_MAP) WSTAMP_ON(k); } while (0)
#else
#define WSTAMP(k) do { } while (0)
#endif
#ifdef ALOAM_WSTAMP_RB       // k_rb_cubevox phases, one row per workgroup (profiling builds only)
WSTAMP_DEFINE_TABLE
#define RBSTAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 128) g_wstamp[(blockIdx.x + (leaf > 0.6f ? 128 : 0)) * WSTAMP_SLOTS + (k)] = wall_clock64(); } while (0)
#else
#define RBSTAMP(k) do { } while (0)
#endif

void prof_mark(Ctx& C, int idx);

constexpr int MB = 256;
constexpr int PAD_CUBE = 8191;

__device__ inline int cube_coord(double v, int cen) {   // :314-323, :743-752
    int c = int((v + 25.0) / 50.0) + cen;
    if (v + 25.0 < 0) c--;
    return c;
}
__device__ inline float4 associate_to_map(const double* par, float4 p) {   // :154-163
    const dquat q{par[0], par[1], par[2], par[3]};
    const dvec3 r = qrot(q, {p.x, p.y, p.z});
    return make_float4((float)(r.x + par[4]), (float)(r.y + par[5]), (float)(r.z + par[6]), p.w);
}

// also zeroes this frame's mapping round counters (saves a launch on the host-issue-bound part of the frame)
__global__ void k_map_prepare(MapState* m, unsigned char* cube_valid, int* spread, const double* pose_in) {
    __shared__ int valid_num;
    for (int i = threadIdx.x; i < ALOAM_MAX_ROUNDS * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE; i += blockDim.x) spread[i] = 0;
    if (threadIdx.x == 0) {
        for (int k = 0; k < 4; k++) m->q_wodom[k] = pose_in[k];      // the input set's laser_odom_to_init
        for (int k = 0; k < 3; k++) m->t_wodom[k] = pose_in[4 + k];
        // transformAssociateToMap (:142-146)
        const dquat qm{m->q_wmap_wodom[0], m->q_wmap_wodom[1], m->q_wmap_wodom[2], m->q_wmap_wodom[3]};
        const dquat qo{m->q_wodom[0], m->q_wodom[1], m->q_wodom[2], m->q_wodom[3]};
        const dquat qw = qmul(qm, qo);
        const dvec3 r = qrot(qm, {m->t_wodom[0], m->t_wodom[1], m->t_wodom[2]});
        m->parameters[0] = qw.x; m->parameters[1] = qw.y; m->parameters[2] = qw.z; m->parameters[3] = qw.w;
        m->parameters[4] = r.x + m->t_wmap_wodom[0];
        m->parameters[5] = r.y + m->t_wmap_wodom[1];
        m->parameters[6] = r.z + m->t_wmap_wodom[2];
        int cI = cube_coord(m->parameters[4], m->cenW), cJ = cube_coord(m->parameters[5], m->cenH), cK = cube_coord(m->parameters[6], m->cenD);
        int si = 0, sj = 0, sk = 0;
        while (cI < 3) { cI++; m->cenW++; si++; }
        while (cI >= CUBE_W - 3) { cI--; m->cenW--; si--; }
        while (cJ < 3) { cJ++; m->cenH++; sj++; }
        while (cJ >= CUBE_H - 3) { cJ--; m->cenH--; sj--; }
        while (cK < 3) { cK++; m->cenD++; sk++; }
        while (cK >= CUBE_D - 3) { cK--; m->cenD--; sk--; }
        m->shift[0] = si; m->shift[1] = sj; m->shift[2] = sk;
        m->cI = cI; m->cJ = cJ; m->cK = cK;
        int nv = 0;
        for (int i = cI - 2; i <= cI + 2; i++)
            for (int j = cJ - 2; j <= cJ + 2; j++)
                for (int k = cK - 1; k <= cK + 1; k++)
                    if (i >= 0 && i < CUBE_W && j >= 0 && j < CUBE_H && k >= 0 && k < CUBE_D)
                        m->valid_ind[nv++] = i + CUBE_W * j + CUBE_W * CUBE_H * k;
        m->valid_num = nv;
        m->optimize = 0;
        valid_num = nv;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < CUBE_N; c += blockDim.x) cube_valid[c] = 0;
    __syncthreads();
    for (int t = threadIdx.x; t < valid_num; t += blockDim.x) cube_valid[m->valid_ind[t]] = 1;
}

// recentring: cube (i,j,k) -> (i+si, j+sj, k+sk); cubes pushed off the grid are cleared (:325-507)
__global__ void k_map_shift(int* __restrict__ cube_c, int* __restrict__ cube_s, const int* d_n, const MapState* m) {
    const int si = m->shift[0], sj = m->shift[1], sk = m->shift[2];
    if (si == 0 && sj == 0 && sk == 0) return;
    int* cube = blockIdx.y == 0 ? cube_c : cube_s;     // y = map kind
    const int n = d_n[blockIdx.y];
    for (int p = blockIdx.x * MB + threadIdx.x; p < n; p += gridDim.x * MB) {
        int c = cube[p];
        if (c < 0) continue;
        int k = c / (CUBE_W * CUBE_H), j = (c / CUBE_W) % CUBE_H, i = c % CUBE_W;
        i += si; j += sj; k += sk;
        cube[p] = (i >= 0 && i < CUBE_W && j >= 0 && j < CUBE_H && k >= 0 && k < CUBE_D) ? i + CUBE_W * j + CUBE_W * CUBE_H * k : -1;
    }
}

__global__ void k_map_gate(MapState* m, const GridDesc* gc, const GridDesc* gs) {
    m->n_corner_map = gc->n;
    m->n_surf_map = gs->n;
    m->optimize = (gc->n > 10 && gs->n > 50) ? 1 : 0;
}

// line / plane fit of one stack point's 5 neighbours (kNN order) -> factor (:585-620, :650-686)
__device__ __forceinline__ void fit_factor(bool corner, const float4 po, const float4* __restrict__ sp, const int* nb, aloam_factor& f) {
    f.type = -1; f.pad = 0;
    f.cp[0] = po.x; f.cp[1] = po.y; f.cp[2] = po.z;
    if (corner) {
        double pts[5][3];
        double cx = 0, cy = 0, cz = 0;
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const float4 v = sp[nb[j]];
            pts[j][0] = v.x; pts[j][1] = v.y; pts[j][2] = v.z;
            cx = cx + pts[j][0]; cy = cy + pts[j][1]; cz = cz + pts[j][2];
        }
        cx = cx / 5.0; cy = cy / 5.0; cz = cz / 5.0;
        double cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const double zm[3] = {pts[j][0] - cx, pts[j][1] - cy, pts[j][2] - cz};
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
                for (int c = 0; c < 3; c++) cov[r * 3 + c] = cov[r * 3 + c] + zm[r] * zm[c];
        }
        double ev[3], evec[9];
        eigen_sym3(cov, ev, evec);
        if (ev[2] > 3 * ev[1]) {
            const double u[3] = {evec[2], evec[5], evec[8]};
            f.type = 0;
            f.a[0] = 0.1 * u[0] + cx; f.a[1] = 0.1 * u[1] + cy; f.a[2] = 0.1 * u[2] + cz;
            f.b[0] = -0.1 * u[0] + cx; f.b[1] = -0.1 * u[1] + cy; f.b[2] = -0.1 * u[2] + cz;
        }
    } else {
        double A[15], b[5], P[5][3];
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const float4 v = sp[nb[j]];
            P[j][0] = v.x; P[j][1] = v.y; P[j][2] = v.z;
            A[j * 3] = P[j][0]; A[j * 3 + 1] = P[j][1]; A[j * 3 + 2] = P[j][2];
            b[j] = -1;
        }
        double n[3];
        colpiv_qr_5x3(A, b, n);
        const double negOA = 1 / sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        const double z = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
        if (z > 0) { const double s = sqrt(z); n[0] /= s; n[1] /= s; n[2] /= s; }
        bool valid = true;
#pragma unroll
        for (int j = 0; j < 5; j++)
            if (fabs(n[0] * P[j][0] + n[1] * P[j][1] + n[2] * P[j][2] + negOA) > 0.2) valid = false;
        if (valid) {
            f.type = 2;
            f.a[0] = n[0]; f.a[1] = n[1]; f.a[2] = n[2];
            f.b[0] = negOA; f.b[1] = 0; f.b[2] = 0;
        }
    }
}

// One mapping association round, 8 lanes per stack point (corner stack, then surf stack):
// pointAssociateToMap (:581,647), 5-NN within 1 m (d^2[4] < 1.0, :583-584,649-650) over the
// surround map's 1.025 m grid (group_knn27), then the group's first lane fits the line / plane
// and writes the factor record. Correspondence counts and (profiling) candidate counts are
// aggregated per wave before the atomics.
constexpr int AG = 8;     // lanes per query of the scan-to-map registration (k_s2m_assoc); k_map_assoc: g_map_ag
constexpr int ASSOC_BLOCKS = 512;   // fixed launch (graph-replayable); waves stride over the stacks
constexpr int FIT_BLOCKS = 160;     // k_map_fit: 40960 lanes, one stack point each at C3 sizes

// Per-query candidate cache of the registration rounds. A query's map-frame position moves little
// between rounds (HDL-64 sequence, micro/round_stats.cpp: p99 7 cm after the first round, 2 cm after
// the second, < 1 cm later), so the first round's search (and any later full search) also collects
// the block points within 1 + MC_M of the query: the cache centre c. A later round whose query q has
// |q - c| <= MC_M - eps and whose 1 m ball lies inside c's 3x3x3 block (the points the collection
// saw) finds every point within the 1 m search radius in the cache, so the k-NN over the cached
// list is exactly the grid search's result (same (d2, index) order). Otherwise the query searches
// the grid again and re-centres its cache. A query whose 5 neighbours (in order) equal the previous
// round's keeps its factor: the fit reads nothing but those 5 map points and the stack point.
// Invariant of that reuse: between the rounds of one mapping frame nothing else writes the
// factor slots (C.d_factors). They are shared with the odometry rounds and the eval / solve test entry
// points of the same context, but all of those run on the context's one stream (C.stream), and a frame's
// rounds are issued back to back (one graph); round 0 searches every query and rewrites every slot, so no
// factor of an earlier frame or call is ever reused.
constexpr int MC_CAP = MC_CAP_PTS;  // cached points per query (p99 45, 1e-4 above 64 at MC_M = 0.1; more => full search)
constexpr float MC_M = 0.1f;        // reuse radius (m)
constexpr float MC_EPS = 2e-3f;     // fp32 slack of the distance and cell tests (coordinates << 2^13 m)
struct MapCache {
    float4* ctr;     // [cap_q] centre xyz, w = cached count (int bits; -1 = none)
    float4* pts;     // [cap_q][MC_CAP] cached points (w = original index)
    int* pos;        // [cap_q][MC_CAP] their grid positions
    int* prev;       // [cap_q][5] last round's neighbour positions (-1: no factor)
    int cap_q;       // queries with a cache slot (the rest always search)
    int round;       // 0: search and collect for every query
};
// the 1 m ball (+ eps) around q inside the 3x3x3 cell block of c's cell (cells outside the grid hold no points)
__device__ __forceinline__ bool ball_in_block(const GridDesc& gd, const float4 c, const float4 q) {
    auto axis = [&gd](float cv, float qv, float o, int d) {
        const int cc = (int)floorf((cv - o) * gd.inv_cell);
        const float lo = cc - 1 <= 0 ? -INFINITY : o + (float)(cc - 1) * gd.cell;
        const float hi = cc + 2 >= d ? INFINITY : o + (float)(cc + 2) * gd.cell;
        return qv - (1.0f + MC_EPS) >= lo && qv + (1.0f + MC_EPS) <= hi;
    };
    return axis(c.x, q.x, gd.ox, gd.dx) && axis(c.y, q.y, gd.oy, gd.dy) && axis(c.z, q.z, gd.oz, gd.dz);
}

// slots [s0, s1) of the compact slot space (corner stack at [0, nc), surf stack at [nc, nc + ns) — the
// reference's AddResidualBlock order), pose `par` (laserMapping.cpp:129 parameters)
template <int G, int U>
__device__ __forceinline__ void assoc_slots(
    const float4* __restrict__ cstack, const float4* __restrict__ sstack, const int nc, const int s0, const int s1, const double* par,
    const GridDesc* __restrict__ gdc, const int* __restrict__ cs_c, const float4* __restrict__ sp_c, const int* __restrict__ si_c,
    const GridDesc* __restrict__ gds, const int* __restrict__ cs_s, const float4* __restrict__ sp_s, const int* __restrict__ si_s,
    aloam_factor* __restrict__ out, int* round_cnt, unsigned long long* cand_count, int exp, int (*tabs)[20],
    int* __restrict__ nbr = nullptr, const MapCache mc = MapCache{}) {
    const bool lead = (lane_id() & (G - 1)) == 0;
    const int per_wave = WAVE / G;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE, nwaves = gridDim.x * (blockDim.x / WAVE);
    int cnt_c = 0, cnt_s = 0;
    unsigned long long ncand_sum = 0;
    const bool has_mc = mc.ctr != nullptr;   // by value: no private copy of the struct
    const int round = has_mc ? mc.round : 0, wst_round = round;
    for (int base = s0 + wave * per_wave; base < s1; base += nwaves * per_wave) {   // wave-uniform trip count
        const int qi = base + (lane_id() / G);
        const bool live = qi < s1;
        const bool corner = qi < nc;
        const int li = corner ? qi : qi - nc;
        const float4 po = live ? (corner ? cstack[li] : sstack[li]) : make_float4(0, 0, 0, 0);
        const GridDesc gd = corner ? *gdc : *gds;
        const float4 sel = associate_to_map(par, po);
        const float4* sp = corner ? sp_c : sp_s;
        const bool slot = has_mc && live && qi < mc.cap_q;
        int ncache = -1;
        bool cached = false;
        if (slot && round > 0) {
            const float4 c = mc.ctr[qi];
            ncache = __float_as_int(c.w);
            const float ex = sel.x - c.x, ey = sel.y - c.y, ez = sel.z - c.z;
            cached = ncache >= 0 && ncache <= MC_CAP && ex * ex + ey * ey + ez * ez <= (MC_M - MC_EPS) * (MC_M - MC_EPS) &&
                     ball_in_block(gd, c, sel);
        }
        WSTAMP(2);
        int pos[5], idx[5], ncand = 0;
        float d2[5];
        int found = 5;
        if (exp & 1) { for (int k = 0; k < 5; k++) pos[k] = (li * 7 + k) % 64; }
        else {
            found = 0;
#pragma unroll
            for (int k = 0; k < 5; k++) pos[k] = -1;
            const bool search = live && !cached;
            if (has_mc && round > 0) {
                // the few queries that left their cache: a whole wave per query (its latency bounds the
                // launch: one group's search over a dense block streams hundreds of candidates per lane group)
                unsigned long long todo = __ballot(search && lead);
                while (todo) {
                    const int src = __ffsll((long long)todo) - 1;
                    todo &= todo - 1;
                    const int q = __shfl(qi, src);
                    const bool qc = __shfl((int)corner, src) != 0, qslot = __shfl((int)slot, src) != 0;
                    const float qx = __shfl(sel.x, src), qy = __shfl(sel.y, src), qz = __shfl(sel.z, src);
                    const GridDesc& g = qc ? *gdc : *gds;
                    const KnnCollect col{(1.0f + MC_M) * (1.0f + MC_M), mc.pts + (size_t)q * MC_CAP, mc.pos + (size_t)q * MC_CAP,
                                         qslot ? MC_CAP : 0};
                    int p2[5], i2[5], ncol = 0;
                    float e2[5];
                    const int f2 = group_knn27<5, WAVE, true, 8, true>(g.ox, g.oy, g.oz, g.inv_cell, g.dx, g.dy, g.dz, qc ? cs_c : cs_s,
                                                                       qc ? sp_c : sp_s, qc ? si_c : si_s, qx, qy, qz, 1.0f, true, p2,
                                                                       e2, i2, nullptr, tabs[(threadIdx.x & ~(WAVE - 1)) / G], g.n,
                                                                       col, &ncol);
                    if (lane_id() == 0 && qslot) mc.ctr[q] = make_float4(qx, qy, qz, __int_as_float(ncol <= MC_CAP ? ncol : -1));
                    if (lane_id() / G == src / G) {
#pragma unroll
                        for (int k = 0; k < 5; k++) pos[k] = p2[k];
                        found = f2;
                    }
                }
            } else if (__any(search)) {
                if (has_mc) {   // search + collect: (re)centre the cache at this round's position
                    const KnnCollect col{(1.0f + MC_M) * (1.0f + MC_M), mc.pts + (size_t)qi * MC_CAP, mc.pos + (size_t)qi * MC_CAP,
                                         slot ? MC_CAP : 0};
                    int ncol = 0;
                    found = group_knn27<5, G, true, U, true>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz,
                                                             corner ? cs_c : cs_s, sp, corner ? si_c : si_s, sel.x, sel.y, sel.z,
                                                             1.0f, search, pos, d2, idx, &ncand, tabs[threadIdx.x / G], gd.n,
                                                             col, &ncol);
                    if (search && slot && lead) mc.ctr[qi] = make_float4(sel.x, sel.y, sel.z, __int_as_float(ncol <= MC_CAP ? ncol : -1));
                } else {
                    found = group_knn27<5, G, true, U>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, corner ? cs_c : cs_s, sp,
                                                       corner ? si_c : si_s, sel.x, sel.y, sel.z, 1.0f, search, pos, d2, idx, &ncand,
                                                       tabs[threadIdx.x / G], gd.n);
                }
            }
            WSTAMP(6);
            if (__any(cached)) {
                int p2[5], i2[5];
                float e2[5];
                const size_t cb = cached ? (size_t)qi * MC_CAP : 0;
                const int f2 = group_knn_list<5, G, (MC_CAP + G - 1) / G>(mc.pts + cb, mc.pos + cb, cached ? ncache : 0, sel.x,
                                                                          sel.y, sel.z, 1.0f, p2, e2, i2);
                if (cached) {
#pragma unroll
                    for (int k = 0; k < 5; k++) pos[k] = p2[k];
                    found = f2;
                }
            }
        }
        WSTAMP(3);
        if (live && lead) {
            const bool use = found == 5 && !(exp & 2);
            if (nbr) {   // neighbours only: k_map_fit fits them one query per lane
#pragma unroll
                for (int k = 0; k < 5; k++) nbr[(size_t)qi * 5 + k] = use ? pos[k] : -1;
            } else {
                // unchanged neighbours since the last round: the factor in out[qi] is this round's
                bool same = false;
                if (slot) {
                    int* pv = mc.prev + (size_t)qi * 5;
                    same = round > 0;
#pragma unroll
                    for (int k = 0; k < 5; k++) same = same && pv[k] == (use ? pos[k] : -1);
                    if (!same)
#pragma unroll
                        for (int k = 0; k < 5; k++) pv[k] = use ? pos[k] : -1;
                }
                int type;
                if (same) {
                    type = out[qi].type;
                } else {
                    aloam_factor f;
                    f.type = -1; f.pad = 0;
                    if (use) fit_factor(corner, po, sp, pos, f);
                    WSTAMP(7);
                    out[qi] = f;
                    type = f.type;
                }
                if (type >= 0) { if (corner) cnt_c++; else cnt_s++; }
            }
            ncand_sum += ncand;
        }
        WSTAMP(4);
    }
    // wave-aggregated counters
    if (round_cnt) {
        const int tc = wave_sum_i(cnt_c), ts = wave_sum_i(cnt_s);
        if (lane_id() == 0) {
            // spread over ODOM_CNT_SLOTS cache lines (folded by k_map_update): one address per counter
            // serialises every wave's atomic
            int* rc = round_cnt + ((blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE) & (ODOM_CNT_SLOTS - 1)) * ODOM_CNT_STRIDE;
            if (tc) atomicAdd(&rc[0], tc);
            if (ts) atomicAdd(&rc[1], ts);
        }
    }
    if (cand_count) {
        const int t = wave_sum_i((int)ncand_sum);
        if (lane_id() == 0 && t) atomicAdd(cand_count, (unsigned long long)t);
    }
}

template <int G, int U>
__global__ void __launch_bounds__(256) k_map_assoc(
    const float4* __restrict__ cstack, const float4* __restrict__ sstack, const int* stack_n,
    const GridDesc* __restrict__ gdc, const int* __restrict__ cs_c, const float4* __restrict__ sp_c, const int* __restrict__ si_c,
    const GridDesc* __restrict__ gds, const int* __restrict__ cs_s, const float4* __restrict__ sp_s, const int* __restrict__ si_s,
    const MapState* __restrict__ m, aloam_factor* __restrict__ out, int* round_cnt, int* __restrict__ nbr,
    unsigned long long* cand_count, int exp, const MapCache mc) {
    __shared__ int tabs[256 / G][20];
    const int wst_round = mc.round;
    WSTAMP(0);
    // the solver reads nc + ns from the device
    if (!m->optimize) return;
    const int nc = stack_n[0], ns = stack_n[1];
    double par[7];
#pragma unroll
    for (int i = 0; i < 7; i++) par[i] = m->parameters[i];
    WSTAMP(1);
    assoc_slots<G, U>(cstack, sstack, nc, 0, nc + ns, par, gdc, cs_c, sp_c, si_c, gds, cs_s, sp_s, si_s, out, round_cnt,
                      cand_count, exp, tabs, nbr, mc);
    WSTAMP(5);
}

// The fits of a mapping round, one stack point per lane (the fp64 eigen / QR fits are long serial
// chains: run on the 8-lane groups of the search they kept 7 of 8 lanes idle): line / plane fit of
// the 5 neighbours k_map_assoc found (:585-620, :650-686) -> factor record in slot order, and the
// round's correspondence counts (wave-aggregated, spread over ODOM_CNT_SLOTS cache lines).
__global__ void __launch_bounds__(256) k_map_fit(const float4* __restrict__ cstack, const float4* __restrict__ sstack,
                                                 const int* stack_n, const float4* __restrict__ sp_c, const float4* __restrict__ sp_s,
                                                 const MapState* __restrict__ m, const int* __restrict__ nbr,
                                                 aloam_factor* __restrict__ out, int* round_cnt) {
    if (!m->optimize) return;
    const int nc = stack_n[0], nq = stack_n[0] + stack_n[1];
    int cnt_c = 0, cnt_s = 0;
    const int stride = gridDim.x * blockDim.x;
    for (int i0 = blockIdx.x * blockDim.x + (threadIdx.x & ~(WAVE - 1)); i0 < nq; i0 += stride) {   // whole waves
        const int qi = i0 + lane_id();
        if (qi >= nq) continue;
        const bool corner = qi < nc;
        int pos[5];
#pragma unroll
        for (int k = 0; k < 5; k++) pos[k] = nbr[(size_t)qi * 5 + k];
        aloam_factor f;
        f.type = -1; f.pad = 0;
        const float4 po = corner ? cstack[qi] : sstack[qi - nc];
        f.cp[0] = po.x; f.cp[1] = po.y; f.cp[2] = po.z;
        if (pos[4] >= 0) fit_factor(corner, po, corner ? sp_c : sp_s, pos, f);
        out[qi] = f;
        if (f.type >= 0) { if (corner) cnt_c++; else cnt_s++; }
    }
    const int tc = wave_sum_i(cnt_c), ts = wave_sum_i(cnt_s);
    if (lane_id() == 0) {
        int* rc = round_cnt + ((blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE) & (ODOM_CNT_SLOTS - 1)) * ODOM_CNT_STRIDE;
        if (tc) atomicAdd(&rc[0], tc);
        if (ts) atomicAdd(&rc[1], ts);
    }
}

// Scan-to-map registration association (aloam_s2m_*). Each wave takes 8 NB stack points per pass:
// NB batches of 8 lane groups run the 5-NN and park the neighbour positions in LDS, then 8 NB lanes
// fit one point each (the fp64 line / plane fits on many lanes instead of one per group).
// The 5-NN first searches the 3x3x3 block of a fine grid of the map (edge ~0.3 m): when its 5th
// neighbour is closer than 0.99 fine cells, no point outside the block can be closer, so the result is
// the exact 5-NN (same order, same ties by index). Groups it does not settle search the 1.025 m grid's
// block, which holds the whole 1 m ball (laserMapping.cpp:583-584,649-650). On a dense map (C4: ~1000
// points in the coarse block, the 5 neighbours within ~0.2 m) the fine block streams ~20x fewer points.
struct KindGrids { const GridDesc* gd; const int* cs; const float4* sp; const int* si; };

__device__ __forceinline__ int knn5_fine_coarse(const KindGrids& fc, const KindGrids& fs, const KindGrids& cc, const KindGrids& cs,
                                                bool use_fine, bool corner, const float4 sel, bool live, int* pos,
                                                const float4** sp, int* tab) {
    int idx[5], found = 0;
    float d2[5];
    bool need = live;
    *sp = corner ? cc.sp : cs.sp;
    if (use_fine) {                                    // kernel-uniform
        const KindGrids& f = corner ? fc : fs;
        const GridDesc gd = *f.gd;
        found = group_knn27<5, AG, true>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, f.cs, f.sp, f.si, sel.x, sel.y,
                                         sel.z, 1.0f, live, pos, d2, idx, nullptr, tab, gd.n);
        const float lim = 0.99f * gd.cell;
        need = live && !(found == 5 && d2[4] < lim * lim);
        *sp = f.sp;
    }
    if (__any(need)) {                                 // wave-uniform: every lane takes part in the group search
        const KindGrids& c = corner ? cc : cs;
        const GridDesc gd = *c.gd;
        int p2[5], i2[5];
        float e2[5];
        const int f2 = group_knn27<5, AG, true>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, c.cs, c.sp, c.si, sel.x,
                                                sel.y, sel.z, 1.0f, need, p2, e2, i2, nullptr, tab, gd.n);
        if (need) {
#pragma unroll
            for (int k = 0; k < 5; k++) pos[k] = p2[k];
            found = f2;
            *sp = c.sp;
        }
    }
    return found;
}

template <int NB>
__device__ __forceinline__ void assoc_slots_batched(const float4* __restrict__ cstack, const float4* __restrict__ sstack, const int nc,
                                                    const int s0, const int s1, const double* par, const KindGrids fc,
                                                    const KindGrids fs, const KindGrids cc, const KindGrids cs, bool use_fine,
                                                    aloam_factor* __restrict__ out, int (*tabs)[20], int (*park)[6]) {
    const bool lead = (lane_id() & (AG - 1)) == 0;
    const int per_wave = WAVE / AG;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE, nwaves = gridDim.x * (blockDim.x / WAVE);
    constexpr int PTS = NB * (WAVE / AG);
    int (*my)[6] = park + (threadIdx.x / WAVE) * PTS;    // this wave's parking slots
    for (int base = s0 + wave * PTS; base < s1; base += nwaves * PTS) {   // wave-uniform trip count
#pragma unroll 1
        for (int b = 0; b < NB; b++) {
            const int slot = b * per_wave + lane_id() / AG;
            const int qi = base + slot;
            const bool live = qi < s1;
            const bool corner = qi < nc;
            const int li = corner ? qi : qi - nc;
            const float4 po = live ? (corner ? cstack[li] : sstack[li]) : make_float4(0, 0, 0, 0);
            const float4 sel = associate_to_map(par, po);
            int pos[5];
            const float4* sp;
            const int found = knn5_fine_coarse(fc, fs, cc, cs, use_fine, corner, sel, live, pos, &sp, tabs[threadIdx.x / AG]);
            if (lead) {
#pragma unroll
                for (int k = 0; k < 5; k++) my[slot][k] = pos[k];
                // found | which sorted copy the positions index (1: fine grid) << 8
                my[slot][5] = found | ((use_fine && sp == (corner ? fc.sp : fs.sp)) ? 256 : 0);
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const int qi = base + lane_id();
        if (lane_id() < PTS && qi < s1) {
            const bool corner = qi < nc;
            const float4 po = corner ? cstack[qi] : sstack[qi - nc];
            int pos[5];
#pragma unroll
            for (int k = 0; k < 5; k++) pos[k] = my[lane_id()][k];
            const int fl = my[lane_id()][5];
            const float4* sp = (fl & 256) ? (corner ? fc.sp : fs.sp) : (corner ? cc.sp : cs.sp);
            aloam_factor f;
            f.type = -1; f.pad = 0;
            if ((fl & 255) == 5) fit_factor(corner, po, sp, pos, f);
            out[qi] = f;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// one rank's slots [s0, s1) of the stacks at pose x; NB = 1: latency regime, NB > 1: throughput regime
template <int NB>
__global__ void __launch_bounds__(256) k_s2m_assoc(const float4* __restrict__ cstack, const float4* __restrict__ sstack, int nc,
                                                   int s0, int s1, const double* __restrict__ x, KindGrids fc, KindGrids fs,
                                                   KindGrids cc, KindGrids cs, int use_fine, aloam_factor* __restrict__ out) {
    __shared__ int tabs[256 / AG][20];
    __shared__ int park[4 * NB * (WAVE / AG)][6];
    double par[7];
#pragma unroll
    for (int i = 0; i < 7; i++) par[i] = x[i];
    assoc_slots_batched<NB>(cstack, sstack, nc, s0, s1, par, fc, fs, cc, cs, use_fine != 0, out, tabs, park);
}

// Split association (throughput regime; ALOAM_S2M_SPLIT=0 selects the fused kernel below): the 5-NN by 8-lane groups parks each slot's
// neighbour positions (+ found | fine-copy flag) in global memory, then k_s2m_fit fits one slot per lane
// — the same fit_factor on the same neighbours, so the same factor records as the fused kernel.
constexpr int S2M_NBR = 8;          // ints per parked slot: 5 positions, flags, pad
// The 5-NN of the split path as 64-bit (d2, original index) keys (group_knn27_keys, the C4 search's loop: row bounds
// in registers, branch-free top-5 insertion), fine 3x3x3 block first, the coarse block for the unsettled with phase
// 1's 5th key as the bound. Same neighbours in the same (d2, index) order as knn5_fine_coarse, parked as ORIGINAL
// map indices (the grids carry them in w): k_s2m_fit reads the map arrays themselves.
__global__ void __launch_bounds__(256) k_s2m_knn(const float4* __restrict__ cstack, const float4* __restrict__ sstack, int nc,
                                                 int s0, int s1, const double* __restrict__ x, KindGrids fc, KindGrids fs,
                                                 KindGrids cc, KindGrids cs, int use_fine, int* __restrict__ nbr) {
    double par[7];
#pragma unroll
    for (int i = 0; i < 7; i++) par[i] = x[i];
    const int per_wave = WAVE / AG;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE, nwaves = gridDim.x * (blockDim.x / WAVE);
    for (int base = s0 + wave * per_wave; base < s1; base += nwaves * per_wave) {   // wave-uniform trip count
        const int qi = base + lane_id() / AG;
        const bool live = qi < s1;
        const bool corner = qi < nc;
        const int li = corner ? qi : qi - nc;
        const float4 po = live ? (corner ? cstack[li] : sstack[li]) : make_float4(0, 0, 0, 0);
        const float4 sel = associate_to_map(par, po);
        unsigned long long key[5];
#pragma unroll
        for (int k = 0; k < 5; k++) key[k] = ~0ull;
        int found = 0;
        bool need = live;
        if (use_fine) {                                   // kernel-uniform
            const KindGrids& f = corner ? fc : fs;
            const GridDesc gd = *f.gd;
            found = group_knn27_keys<5, AG, 4, false>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, f.cs, f.sp, sel.x, sel.y,
                                                      sel.z, 1.0f, live, key, nullptr, gd.n);
            const float lim = 0.99f * gd.cell;
            const float d4 = key[4] == ~0ull ? INFINITY : __uint_as_float((unsigned)(key[4] >> 32));
            need = live && !(found == 5 && d4 < lim * lim);
        }
        if (__any(need)) {                                // wave-uniform: every lane takes part in the group search
            const KindGrids& c = corner ? cc : cs;
            const GridDesc gd = *c.gd;
            unsigned long long k2[5];
            const int f2 = group_knn27_keys<5, AG, 4, false>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, c.cs, c.sp, sel.x,
                                                             sel.y, sel.z, 1.0f, need, k2, nullptr, gd.n, key[4]);
            if (need) {
#pragma unroll
                for (int k = 0; k < 5; k++) key[k] = k2[k];
                found = f2;
            }
        }
        if (live && (lane_id() & (AG - 1)) == 0) {
            int* o = nbr + (size_t)(qi - s0) * S2M_NBR;
            int ix[5];
#pragma unroll
            for (int k = 0; k < 5; k++) ix[k] = key[k] == ~0ull ? -1 : (int)(unsigned)key[k];
            *(int4*)o = make_int4(ix[0], ix[1], ix[2], ix[3]);
            *(int4*)(o + 4) = make_int4(ix[4], found, 0, 0);
        }
    }
}
// one slot per lane: the fit on the parked neighbours, read from the map arrays by original index
__global__ void __launch_bounds__(256) k_s2m_fit(const float4* __restrict__ cstack, const float4* __restrict__ sstack, int nc,
                                                 int s0, int s1, const float4* __restrict__ cmap, const float4* __restrict__ smap,
                                                 const int* __restrict__ nbr, aloam_factor* __restrict__ out) {
    for (int qi = s0 + blockIdx.x * blockDim.x + threadIdx.x; qi < s1; qi += gridDim.x * blockDim.x) {
        const int* o = nbr + (size_t)(qi - s0) * S2M_NBR;
        const int4 a = *(const int4*)o, b = *(const int4*)(o + 4);
        const int pos[5] = {a.x, a.y, a.z, a.w, b.x};
        const bool corner = qi < nc;
        const float4 po = corner ? cstack[qi] : sstack[qi - nc];
        aloam_factor f;
        f.type = -1; f.pad = 0;
        if (b.y == 5) fit_factor(corner, po, corner ? cmap : smap, pos, f);
        out[qi] = f;
    }
}

void s2m_assoc_launch(Ctx& C, const float4* cq, const float4* sq, int nc, int s0, int s1, const double* d_x, Grid& gc, Grid& gs,
                      const Grid* gcf, const Grid* gsf, const float4* cmap, const float4* smap, aloam_factor* out) {
    if (s1 <= s0) return;
    // regime threshold (tests force either path). Default 1: the split 5-NN / fit kernels at any slot count —
    // a rank's share at world 4 / 8 (65k / 33k slots) runs 4.65 / 13.55 ms per group registration on one GPU
    // with them against 5.56 / 16.74 ms with the fused latency kernel (micro/s2m_share.py)
    const char* bm = getenv("ALOAM_S2M_BATCH_MIN");
    const int batch_min = bm ? atoi(bm) : 1;
    const bool fine = gcf && gsf;
    const KindGrids cc{gc.desc, gc.cell_start, gc.pts, gc.idx}, cs{gs.desc, gs.cell_start, gs.pts, gs.idx};
    const KindGrids fc = fine ? KindGrids{gcf->desc, gcf->cell_start, gcf->pts, gcf->idx} : cc;
    const KindGrids fs = fine ? KindGrids{gsf->desc, gsf->cell_start, gsf->pts, gsf->idx} : cs;
    // split 5-NN / fit kernels (default; ALOAM_S2M_SPLIT=0: fused): C4 2.74 -> 2.02 ms per registration —
    // the fp64 fits on every lane instead of 16 of 64, the search waves no longer wait on them
    const char* spe = getenv("ALOAM_S2M_SPLIT");
    if (s1 - s0 >= batch_min && !(spe && atoi(spe) == 0)) {
        const int n = s1 - s0;
        if (C.cap_s2m_nbr < n) {         // grown on demand (the old buffer given back)
            dfree(C, C.d_s2m_nbr);
            C.cap_s2m_nbr = std::max(n, 2 * C.cap_s2m_nbr);
            C.d_s2m_nbr = (int*)dalloc(C, sizeof(int) * S2M_NBR * (size_t)C.cap_s2m_nbr);
        }
        const int waves = (n + WAVE / AG - 1) / (WAVE / AG);
        k_s2m_knn<<<std::max(1, std::min(16384, (waves + 3) / 4)), 256, 0, C.stream>>>(cq, sq, nc, s0, s1, d_x, fc, fs, cc, cs,
                                                                                      fine, C.d_s2m_nbr);
        k_s2m_fit<<<std::max(1, std::min(4096, (n + 255) / 256)), 256, 0, C.stream>>>(cq, sq, nc, s0, s1, cmap, smap,
                                                                                      C.d_s2m_nbr, out);
    } else if (s1 - s0 >= batch_min) {   // throughput regime: 8 NB points per wave pass, fits on 8 NB lanes
        const char* nbe = getenv("ALOAM_S2M_NB");                    // tuning knob: 2, 4, 8
        const int nb = nbe ? atoi(nbe) : 2;
        auto go = [&](auto nbc) {
            constexpr int NB = decltype(nbc)::value;
            const int waves = (s1 - s0 + 8 * NB - 1) / (8 * NB);
            const int blocks = std::max(1, std::min(16384, (waves + 3) / 4));
            k_s2m_assoc<NB><<<blocks, 256, 0, C.stream>>>(cq, sq, nc, s0, s1, d_x, fc, fs, cc, cs, fine, out);
        };
        if (nb == 8) go(std::integral_constant<int, 8>{});
        else if (nb == 4) go(std::integral_constant<int, 4>{});
        else go(std::integral_constant<int, 2>{});
    } else {                         // latency regime: 8 points per wave pass
        const int waves = (s1 - s0 + 7) / 8;
        const int blocks = std::max(1, std::min(4096, (waves + 3) / 4));
        k_s2m_assoc<1><<<blocks, 256, 0, C.stream>>>(cq, sq, nc, s0, s1, d_x, fc, fs, cc, cs, fine, out);
    }
    HIPCHK(hipGetLastError());
}

__global__ void k_map_invalidate(aloam_factor* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i].type = -1;
}

// transformUpdate (:148-152)
__global__ void k_map_update(MapState* m, const int* __restrict__ spread, int rounds, int* round_cnt) {
    if ((int)threadIdx.x < 2 * rounds) {      // fold the spread correspondence counters of the rounds
        const int r = threadIdx.x >> 1, t = threadIdx.x & 1;
        const int* b = spread + (size_t)r * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE + t;
        int sum = 0;
        for (int k = 0; k < ODOM_CNT_SLOTS; k++) sum += b[k * ODOM_CNT_STRIDE];
        round_cnt[2 * r + t] = sum;
    }
    if (threadIdx.x != 0) return;
    const dquat qw{m->parameters[0], m->parameters[1], m->parameters[2], m->parameters[3]};
    const dquat qo{m->q_wodom[0], m->q_wodom[1], m->q_wodom[2], m->q_wodom[3]};
    const dquat qm = qmul(qw, qinv(qo));
    m->q_wmap_wodom[0] = qm.x; m->q_wmap_wodom[1] = qm.y; m->q_wmap_wodom[2] = qm.z; m->q_wmap_wodom[3] = qm.w;
    const dvec3 r = qrot(qm, {m->t_wodom[0], m->t_wodom[1], m->t_wodom[2]});
    m->t_wmap_wodom[0] = m->parameters[4] - r.x;
    m->t_wmap_wodom[1] = m->parameters[5] - r.y;
    m->t_wmap_wodom[2] = m->parameters[6] - r.z;
}

// cube bookkeeping arrays: cnt_old, cnt_new, first_old, first_new, off, seg_nout, final_off (each CUBE_N+1)
struct CubeArrays { int *first_old, *last_old, *first_new, *last_new, *off, *seg_nout, *final_off; };
// counts from run boundaries (the old map and the sorted new points are both ordered by cube)
__device__ __forceinline__ int old_count(const CubeArrays& a, int c) { return a.last_old[c] >= a.first_old[c] ? a.last_old[c] - a.first_old[c] + 1 : 0; }
__device__ __forceinline__ int new_count(const CubeArrays& a, int c) { return a.last_new[c] >= a.first_new[c] ? a.last_new[c] - a.first_new[c] + 1 : 0; }

__global__ void k_cube_reset(CubeArrays a) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c <= CUBE_N; c += gridDim.x * blockDim.x) {
        a.last_old[c] = -1; a.last_new[c] = -1; a.first_old[c] = 0x7fffffff; a.first_new[c] = 0x7fffffff; a.seg_nout[c] = 0;
    }
}
// single block: exclusive scan over cubes of v(c); mode 0: cnt_old+cnt_new -> off ; mode 1: final counts -> final_off
__device__ __forceinline__ void cube_scan_body(const CubeArrays& a, const unsigned char* __restrict__ valid, int mode, int* total);
__device__ __forceinline__ void cube_scan_body(const CubeArrays& a, const unsigned char* __restrict__ valid, int mode, int* total) {
    constexpr int PER = (CUBE_N + 1023) / 1024;
    int* dst = mode == 0 ? a.off : a.final_off;
    const int c0 = threadIdx.x * PER;
    int v[PER], s = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int c = c0 + k;
        v[k] = 0;
        if (c < CUBE_N) {
            if (mode == 0) v[k] = old_count(a, c) + new_count(a, c);
            else v[k] = valid[c] ? a.seg_nout[c] : old_count(a, c) + new_count(a, c);
        }
        s += v[k];
    }
    int tot;
    int run = block_exscan<1024>(s, &tot);
#pragma unroll
    for (int k = 0; k < PER; k++) {
        if (c0 + k < CUBE_N) dst[c0 + k] = run;
        run += v[k];
    }
    if (threadIdx.x == 0) { dst[CUBE_N] = tot; if (total) *total = tot; }
}
__global__ void k_map_register(const float4* __restrict__ full, int n, const MapState* __restrict__ m, float4* __restrict__ out) {
    const int i = blockIdx.x * MB + threadIdx.x;
    if (i < n) out[i] = associate_to_map(m->parameters, full[i]);
}


// ------------------------------------------------------------------------------------------
// Per-cube VoxelGrid of the surrounding cubes (:788-801): one 1024-thread workgroup per surrounding cube c,
// over its points in B[off[c], off[c+1]) = the cube's old points, then its appended stack points (the order
// laserCloudCornerArray[ind] has when downSizeFilter.filter runs). PCL sums every leaf from zero in the
// order libstdc++'s std::sort by leaf leaves the (leaf, position) pairs; rvg.hpp: that order only matters
// inside leaves of >= 3 points, so the cube is first sorted order-free (R2: the leaves in key order and the
// points of >= 3-point leaves), and only when such leaves exist is the exact std::sort replayed (R3, heap
// sorts only where two relevant points meet), each relevant leaf then summed in replay order (R4).
// Cubes up to RVG_FIT points sort in LDS; larger ones keep their keys in the cube's global scratch
// (4 u64 per point: E | S | merge buffer | positions + relevance bits), are split by this kernel and their
// segments replayed by k_rb_cubeseg, summed by k_rb_cubered.
constexpr int RBV_T = 1024;
constexpr int RBV_CPW = 10;          // ls_sort: 64-position chunks per wave
constexpr int RBV_CAP = RBV_T * RBV_CPW;   // LDS element region (E | S | positions for cubes <= RVG_FIT)
constexpr int RVG_FIT = 4096;        // cubes sorted in LDS (E, S and positions share the element region)
constexpr int RVG_NEW = 4096;        // big cubes: appended points sorted in LDS for the merge with the old ones
constexpr int RVG_OLD = 16384;       // big cubes: old keys held in LDS for the merge
constexpr size_t RBV_HDR = 64 + 512 + 256;   // RbvShared | relevance bits (RVG_FIT) | reduce scan ints
constexpr size_t RBV_LDS = RBV_HDR + 8 * (size_t)RBV_CAP + ls_global_scratch_bytes(RBV_T, RBV_CAP);
constexpr int RBV_PER = 8;           // points per thread held in registers for the bbox and the keys
static_assert(RBV_LDS <= 160 * 1024, "LDS");
static_assert(2 * (size_t)RVG_FIT + RVG_FIT / 2 <= (size_t)RBV_CAP, "E | S | positions (int) in the element region");
static_assert(4 * (size_t)RVG_OLD + 16 * (size_t)RVG_NEW <= RBV_LDS - RBV_HDR, "merge buffers");
static_assert(8 * (size_t)RVG_FIT <= ls_global_scratch_bytes(RBV_T, RBV_CAP), "merge-sort buffer in the scratch");
struct RbvShared { unsigned bb[6]; int bad; int nrel; };

// whether this thread's pairs (E[t], E[t + 1]), t = tid, tid + NT, ..., have strictly increasing keys: loads 8
// pairs at a time and no short-circuit (a `up && load` loop waits for every load in turn: ~1 us each on global memory)
template <int NT>
__device__ __forceinline__ bool keys_increasing(const unsigned long long* E, int n) {
    bool up = true;
    for (int t0 = threadIdx.x; t0 + 1 < n; t0 += 8 * NT) {
        unsigned a[8], b[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int t = t0 + u * NT;
            a[u] = t + 1 < n ? ps_keyat(E, t) : 0u;
            b[u] = t + 1 < n ? ps_keyat(E, t + 1) : 1u;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) up &= a[u] < b[u];
    }
    return up;
}

// global layout of a split cube's scratch region G = gscr + 4 p0 (4 n u64; split cubes have n > fit >= 512, fit =
// ALOAM_CUBE_FIT, default 2048). rvg_T spans n + 64 u64 = 8 n + 512 bytes: rvg_mark_bytes' n + 31 relevance bytes fit.
__device__ __forceinline__ unsigned long long* rvg_S(unsigned long long* G, int n) { return G + n; }
__device__ __forceinline__ unsigned long long* rvg_T(unsigned long long* G, int n) { return G + 2 * (size_t)n + 64; }
__device__ __forceinline__ int* rvg_fpos(unsigned long long* G, int n) { return (int*)(G + 3 * (size_t)n + 128); }
__device__ __forceinline__ unsigned* rvg_rel(unsigned long long* G, int n) {
    return (unsigned*)(G + 3 * (size_t)n + 128 + (size_t)n / 2 + 1);
}

// R2 of a split cube: S = its (leaf, position) pairs sorted by leaf, in global scratch. The old points are the
// previous filter's output, one per leaf in leaf order: when their keys are strictly increasing the appended
// points are sorted in LDS and merged in by rank (binary searches); otherwise one global merge sort.
__device__ __forceinline__ void rvg_sort_big(unsigned char* smem, unsigned long long* E, int n, int n_old, unsigned long long* S,
                                             unsigned long long* T) {
    RbvShared& SH = *(RbvShared*)smem;
    const int tid = threadIdx.x;
    const int n_new = n - n_old;
    if (tid == 0) SH.bad = !(n_old <= RVG_OLD && n_new <= RVG_NEW);
    __syncthreads();
    if (!SH.bad) {
        const bool up = keys_increasing<RBV_T>(E, n_old);
        if (__ballot(!up) && lane_id() == 0) SH.bad = 1;
    }
    __syncthreads();
    if (SH.bad) {                         // generic: the whole cube by one merge sort in global scratch
        const int n64 = (n + WAVE - 1) / WAVE * WAVE;
        for (int i = tid; i < n64; i += RBV_T) S[i] = i < n ? E[i] : ~0ull;
        __syncthreads();
        const unsigned long long* R = block_merge_sort<unsigned long long, 16, true>(S, T, n64);
        if (R != S) {
            for (int i = tid; i < n; i += RBV_T) S[i] = R[i];
            __syncthreads();
        }
        return;
    }
    unsigned* OK = (unsigned*)(smem + RBV_HDR);
    unsigned long long* X = (unsigned long long*)(smem + RBV_HDR + 4 * (size_t)RVG_OLD);
    unsigned long long* Y = X + RVG_NEW;
    const int m64 = (n_new + WAVE - 1) / WAVE * WAVE;
#pragma unroll 8
    for (int i = tid; i < n_old; i += RBV_T) OK[i] = ps_keyat(E, i);
#pragma unroll 4
    for (int j = tid; j < m64; j += RBV_T) X[j] = j < n_new ? E[n_old + j] : ~0ull;
    lds_barrier();
    const unsigned long long* Xs = m64 ? block_merge_sort<unsigned long long, 16>(X, Y, m64) : X;
    for (int i = tid; i < n_old; i += RBV_T) {          // old point i: after the appended keys below it
        const unsigned k = OK[i];
        int lo = 0, hi = n_new;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (ps_key(Xs[mid]) < k) lo = mid + 1; else hi = mid; }
        S[i + lo] = ((unsigned long long)k << 32) | (unsigned)i;
    }
    for (int j = tid; j < n_new; j += RBV_T) {          // appended point: after the old keys <= it
        const unsigned long long x = Xs[j];
        const unsigned k = ps_key(x);
        int lo = 0, hi = n_old;
        while (lo < hi) { const int mid = (lo + hi) >> 1; if (OK[mid] <= k) lo = mid + 1; else hi = mid; }
        S[j + lo] = x;
    }
    __syncthreads();
}

// FITS: the whole cube in LDS. Else (n <= 65536): keys in the cube's global scratch, split into segments of
// <= seg_limit elements whose list goes to segl (count 0: the cube is finished here) for k_rb_cubeseg and
// k_rb_cubered.
template <bool FITS>
__device__ __forceinline__ void rbv_cube(unsigned char* smem, const float4* __restrict__ B, CubeArrays a, int c, int p0, int n,
                                         float leaf, float4* __restrict__ Cf, unsigned long long* __restrict__ gscr, const int* fb,
                                         int* segl, int seg_limit) {
    RbvShared& SH = *(RbvShared*)smem;
    unsigned* relL = (unsigned*)(smem + 64);
    int* rsc = (int*)(smem + 64 + 512);
    const int tid = threadIdx.x;
    // keys in LDS when the cube fits, else in the cube's global scratch (staged through the same LDS
    // buffer by the sort); the sort's scratch behind the buffer
    unsigned long long* EL = (unsigned long long*)(smem + RBV_HDR);
    unsigned long long* G = gscr + 4 * (size_t)p0;
    unsigned long long* E = FITS ? EL : G;
    int* sc = (int*)(smem + RBV_HDR + 8 * (size_t)RBV_CAP);
    RBSTAMP(0);
#ifdef ALOAM_WSTAMP_RB
    if (threadIdx.x == 0 && blockIdx.x < 128) g_wstamp[(blockIdx.x + (leaf > 0.6f ? 128 : 0)) * WSTAMP_SLOTS + 7] = (unsigned long long)n | ((unsigned long long)FITS << 32) | ((unsigned long long)new_count(a, c) << 40);
#endif
    if (tid < 6) SH.bb[tid] = tid < 3 ? 0xffffffffu : 0u;
    if (tid == 0) { SH.bad = 0; SH.nrel = 0; }
    lds_barrier();
    // the cube's points: up to RBV_PER per thread in registers (bbox, then keys without a reload)
    float4 pt[RBV_PER];
#pragma unroll
    for (int u = 0; u < RBV_PER; u++) {
        const int t = tid + u * RBV_T;
        pt[u] = t < n ? B[p0 + t] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float inv = 1.0f / leaf;
    auto put = [&](int t, unsigned k) { E[t] = ((unsigned long long)k << 32) | (unsigned)t; };
    int minb[3], mul1, mul2;
    // Leaf keys without the bbox (fb != null): the cube's points lie in its 50 m box, so leaf indices
    // taken from a fixed base below the box, 10 bits per axis, order exactly like PCL's (k, j, i)-linear
    // index over the bbox grid and are equal exactly when PCL's are (PCL's int-overflow pass-through
    // cannot occur with under 1024 leaves per axis); std::sort only sees comparisons, so the order it
    // leaves is the same. A key out of range falls back to the bbox path.
    bool slow = fb == nullptr;
    if (!slow) {
        for (int d = 0; d < 3; d++) minb[d] = fb[d];
        mul1 = 1024; mul2 = 1 << 20;
        bool bad = false;
        auto fast_key = [&](float4 p) {
            const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
            const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
            const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
            bad |= (unsigned)i0 >= 1024u || (unsigned)i1 >= 1024u || (unsigned)i2 >= 1024u;
            return (unsigned)(i0 + i1 * mul1 + i2 * mul2);
        };
#pragma unroll
        for (int u = 0; u < RBV_PER; u++) {
            const int t = tid + u * RBV_T;
            if (t < n) put(t, fast_key(pt[u]));
        }
        for (int t = tid + RBV_PER * RBV_T; t < n; t += RBV_T) put(t, fast_key(B[p0 + t]));
        if (__ballot(bad) && lane_id() == 0) SH.bad = 1;
        lds_barrier();
        slow = SH.bad != 0;
    }
    if (slow) {
        {   // bbox (ordered-int encoding)
            unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
#pragma unroll
            for (int u = 0; u < RBV_PER; u++) {
                if (tid + u * RBV_T >= n) continue;
                const unsigned v[3] = {f2ord(pt[u].x), f2ord(pt[u].y), f2ord(pt[u].z)};
#pragma unroll
                for (int d = 0; d < 3; d++) { mn[d] = min(mn[d], v[d]); mx[d] = max(mx[d], v[d]); }
            }
            for (int t = tid + RBV_PER * RBV_T; t < n; t += RBV_T) {   // beyond the register tile
                const float4 p = B[p0 + t];
                const unsigned v[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
#pragma unroll
                for (int d = 0; d < 3; d++) { mn[d] = min(mn[d], v[d]); mx[d] = max(mx[d], v[d]); }
            }
#pragma unroll
            for (int d = 0; d < 3; d++) {
                const unsigned long long lo = wave_min_u64(mn[d]), hi = wave_max_u64(mx[d]);
                if (lane_id() == 0) { atomicMin(&SH.bb[d], (unsigned)lo); atomicMax(&SH.bb[3 + d], (unsigned)hi); }
            }
        }
        lds_barrier();
        bool ovf;
        voxel_params(SH.bb, leaf, &ovf, minb, &mul1, &mul2);    // same bbox -> leaf grid as k_voxel.hip
        if (ovf) {                            // PCL's int overflow: pass-through (every point its own leaf)
            for (int t = tid; t < n; t += RBV_T) Cf[p0 + t] = B[p0 + t];
            if (tid == 0) a.seg_nout[c] = n;
            return;
        }
#pragma unroll
        for (int u = 0; u < RBV_PER; u++) {
            const int t = tid + u * RBV_T;
            if (t < n) put(t, voxel_index(pt[u], inv, minb, mul1, mul2));
        }
        for (int t = tid + RBV_PER * RBV_T; t < n; t += RBV_T) put(t, voxel_index(B[p0 + t], inv, minb, mul1, mul2));
    }
    if (FITS) lds_barrier(); else __syncthreads();
    RBSTAMP(1);
    // A cube that received no points this frame holds the previous filter's output: one point per leaf in
    // leaf order. With its keys strictly increasing every leaf is a single point, and std::sort leaves the
    // order as is, so the filter returns every point summed from zero (0 + x: -0 becomes +0) over 1.
    if (new_count(a, c) == 0) {
        if (tid == 0) SH.bad = 0;
        if (FITS) lds_barrier(); else __syncthreads();
        const bool up = keys_increasing<RBV_T>(E, n);
        if (__ballot(!up) && lane_id() == 0) SH.bad = 1;
        __syncthreads();
        if (SH.bad == 0) {
            for (int t = tid; t < n; t += RBV_T) {
                const float4 v = B[p0 + t];
                Cf[p0 + t] = div4_by_count(make_float4(0.f + v.x, 0.f + v.y, 0.f + v.z, 0.f + v.w), 1);
            }
            if (tid == 0) a.seg_nout[c] = n;
            return;
        }
    }
    auto ptf = [&](int i) { return B[p0 + i]; };
    auto outf = [&](int r, float4 v) { Cf[p0 + r] = v; };
    if (FITS) {
        // R2 in LDS: S = E sorted by one merge sort (buffer: the sort scratch), relevance bits
        unsigned long long* S = EL + RVG_FIT;
        int* fpos = (int*)(EL + 2 * RVG_FIT);
        const int n64 = (n + WAVE - 1) / WAVE * WAVE;
        for (int i = tid; i < n64; i += RBV_T) S[i] = i < n ? E[i] : ~0ull;
        for (int i = tid; i < (n + 31) / 32; i += RBV_T) relL[i] = 0u;
        lds_barrier();
        const unsigned long long* R = block_merge_sort<unsigned long long, 16>(S, (unsigned long long*)sc, n64);
        if (R != S) {
            for (int i = tid; i < n; i += RBV_T) S[i] = R[i];
            lds_barrier();
        }
        RBSTAMP(3);
        rvg_mark<RBV_T>(S, n, relL, &SH.nrel);
        lds_barrier();
#ifdef RVG_EXP_NOREPLAY                         // timing experiment only (results invalid): no exact replay
        if (tid == 0) SH.nrel = 0;
        lds_barrier();
#endif
        RBSTAMP(2);
        if (SH.nrel > 0) {                    // R3: the exact replay, then the relevant points' positions
            ls_sort<RBV_T, RBV_CPW>(E, n, 2 * (31 - __builtin_clz((unsigned)n)), (unsigned char*)sc, RBV_CAP, relL);
            rvg_positions<RBV_T>(E, n, relL, fpos);
            lds_barrier();
        }
        RBSTAMP(4);
        const int tot = rvg_reduce<RBV_T>(S, n, relL, fpos, ptf, outf, rsc);
        if (tid == 0) a.seg_nout[c] = tot;
        RBSTAMP(5);
        return;
    }
    if (n > RBV_T * PS_MAX_CHUNK) {           // beyond the parallel replay's reach: one thread, every heap sort
        if (tid == 0) ps_serial_std_sort(E, n);
        __syncthreads();
        const int tot = rvg_reduce<RBV_T>(E, n, nullptr, nullptr, ptf, outf, rsc);
        if (tid == 0) a.seg_nout[c] = tot;
        return;
    }
    unsigned long long* S = rvg_S(G, n);
    unsigned* rel = rvg_rel(G, n);
    rvg_sort_big(smem, E, n, old_count(a, c), S, rvg_T(G, n));
    RBSTAMP(3);
    // relevance as one byte per point in the (now free) merge buffer, then packed to bits: no global atomics
    unsigned char* relB = (unsigned char*)rvg_T(G, n);
    rvg_mark_bytes<RBV_T>(S, n, relB, &SH.nrel);
    __syncthreads();
    rvg_pack_bits<RBV_T>(relB, n, rel);
    __syncthreads();
#ifdef RVG_EXP_NOREPLAY
    if (tid == 0) SH.nrel = 0;
    __syncthreads();
#endif
    RBSTAMP(2);
    if (SH.nrel == 0) {                       // no leaf of >= 3 points: no replay
        const int tot = rvg_reduce<RBV_T, true>(S, n, rel, rvg_fpos(G, n), ptf, outf, rsc);   // S in global memory: batched
        if (tid == 0) a.seg_nout[c] = tot;
        RBSTAMP(5);
        return;
    }
    ls_split_to_list<RBV_T>(E, n, seg_limit, segl, (unsigned char*)sc, rel);   // -> k_rb_cubeseg, k_rb_cubered
    RBSTAMP(6);
}

// ------------------------------------------------------------------------------------------
// Both map kinds per launch (blockIdx.y / blockIdx.x = kind): insert -> sort + scan -> scatter ->
// per-cube VoxelGrid -> final scan -> copy, 6 launches on one stream for the two kinds.
struct RbKind {
    const float4* stack; const int* d_stack_n; int ub_new; float leaf;
    float4* A; int* Acube; int* d_n; int n_old_ub;        // the kind's map (old points in, rebuilt map out)
    float4* B; int* Bcube;                                // old + appended points grouped by cube
    float4* ins_pts; unsigned* k1; int* v2;               // appended points in the map frame, cube keys, ranks
    float4* Cf; unsigned long long* gscr;                 // per-cube VoxelGrid output / global scratch
    int* segl;                                            // per surrounding cube: its sort's segment list
    CubeArrays a;
    int fast_keys;                                        // leaf keys from the cube box (< 1024 leaves per axis)
};
struct RbKinds { RbKind k[2]; };

// stack point -> map frame -> cube key (k_map_insert), and the old map's per-cube runs (the map is
// ordered by cube); the run tables were reset by the previous rebuild's final copy
__global__ void k_rb_insert(RbKinds P, const MapState* __restrict__ m) {
    const RbKind& K = P.k[blockIdx.y];
    const int n = *K.d_stack_n, n_old = *K.d_n;
    const int stride = gridDim.x * MB;
    for (int i = blockIdx.x * MB + threadIdx.x; i < max(n_old, K.ub_new); i += stride) {
        if (i < K.ub_new) {
            unsigned k = PAD_CUBE;
            if (i < n) {
                const float4 s = associate_to_map(m->parameters, K.stack[i]);
                K.ins_pts[i] = s;
                const int ci = cube_coord(s.x, m->cenW), cj = cube_coord(s.y, m->cenH), ck = cube_coord(s.z, m->cenD);
                if (ci >= 0 && ci < CUBE_W && cj >= 0 && cj < CUBE_H && ck >= 0 && ck < CUBE_D)
                    k = (unsigned)(ci + CUBE_W * cj + CUBE_W * CUBE_H * ck);
            }
            K.k1[i] = k;
        }
        if (i < n_old) {
            const int c = K.Acube[i];
            if (c >= 0) {
                if (i == 0 || K.Acube[i - 1] != c) K.a.first_old[c] = i;
                if (i == n_old - 1 || K.Acube[i + 1] != c) K.a.last_old[c] = i;
            }
        }
    }
}

// one workgroup per kind: stable rank of every appended point among the kind's appended points of its
// cube (its slot after the cube's old points), the per-cube appended counts, then the exclusive scan of
// old + appended counts over the cubes (k_cube_scan mode 0). Counting, not sorting: wave w owns a
// contiguous chunk of the points and a u16 count row per cube in LDS; pass 1 counts (per 64-point batch,
// one ballot per distinct cube — the stacks come in leaf order, so a batch holds few cubes), the rows
// are turned into per-wave bases by a scan over the waves, pass 2 re-walks the chunk handing out ranks
// in order. Same ranks as a stable sort by cube. Over 65535 points: a merge sort in global scratch.
constexpr int RBS_T = 1024, RBS_W = RBS_T / WAVE;
constexpr size_t RBS_LDS = (size_t)RBS_W * CUBE_N * 2;
static_assert(RBS_LDS <= 160 * 1024 - 1024, "LDS");
// the 64 lanes' keys (ok = lane holds a real point): each lane gets its rank among the lanes with the
// same key below it plus cnt[key]; cnt[key] += the key's lanes (one distinct key per step)
__device__ __forceinline__ int wave_rank_by_key(unsigned key, bool ok, unsigned short* cnt) {
    const int lane = lane_id();
    unsigned long long todo = __ballot(ok);
    int rank = 0;
    while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const unsigned kl = (unsigned)__builtin_amdgcn_readlane((int)key, leader);
        const unsigned long long m = __ballot(ok && key == kl) & todo;
        const int base = cnt[kl];                      // uniform address: one LDS read for the wave
        if (ok && key == kl) rank = base + __popcll(m & lanemask_lt64());
        if (lane == leader) cnt[kl] = (unsigned short)(base + __popcll(m));
        todo &= ~m;
    }
    return rank;
}
__global__ void __launch_bounds__(RBS_T) k_rb_sort_scan(RbKinds P, const unsigned char* __restrict__ valid) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RbKind& K = P.k[blockIdx.x];
    const int n = min(*K.d_stack_n, K.ub_new);
    const int lane = lane_id(), w = threadIdx.x / WAVE;
    if (n < 65536) {
        unsigned short* cnt = (unsigned short*)smem;   // [RBS_W][CUBE_N]
        for (int i = threadIdx.x; i < RBS_W * CUBE_N / 2; i += RBS_T) ((unsigned*)cnt)[i] = 0;
        if (threadIdx.x == 0 && (RBS_W * CUBE_N) % 2) cnt[RBS_W * CUBE_N - 1] = 0;
        lds_barrier();
        const int per = ((n + RBS_W - 1) / RBS_W + WAVE - 1) / WAVE * WAVE;
        const int i0 = w * per, i1 = min(n, i0 + per);
        unsigned short* row = cnt + w * CUBE_N;
        constexpr int U = 8;                            // batches whose keys are loaded together
        for (int pass = 0; pass < 2; pass++) {
            for (int b0 = i0; b0 < i1; b0 += U * WAVE) {
                unsigned kk[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int i = b0 + u * WAVE + lane;
                    kk[u] = i < i1 ? K.k1[i] : PAD_CUBE;
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    if (b0 + u * WAVE >= i1) break;
                    const int i = b0 + u * WAVE + lane;
                    const bool ok = kk[u] < (unsigned)CUBE_N;
                    const int r = wave_rank_by_key(kk[u], ok, row);
                    if (pass == 1 && ok) K.v2[i] = r;
                }
            }
            if (pass == 0) {
                __syncthreads();
                for (int c = threadIdx.x; c < CUBE_N; c += RBS_T) {   // counts -> per-wave bases, cube totals
                    int run = 0;
#pragma unroll
                    for (int v = 0; v < RBS_W; v++) { const int t = cnt[v * CUBE_N + c]; cnt[v * CUBE_N + c] = (unsigned short)run; run += t; }
                    if (run > 0) { K.a.first_new[c] = 0; K.a.last_new[c] = run - 1; }
                }
                __syncthreads();
            }
        }
    } else {
        const int n64 = (n + WAVE - 1) / WAVE * WAVE;
        unsigned long long* ga = K.gscr;
        for (int i = threadIdx.x; i < n64; i += RBS_T) ga[i] = i < n ? (((unsigned long long)K.k1[i] << 32) | (unsigned)i) : ~0ull;
        __syncthreads();
        const unsigned long long* sk = block_merge_sort<unsigned long long, 16, true>(ga, ga + n64, n64);
        for (int p = threadIdx.x; p < n; p += RBS_T) {
            const unsigned c = (unsigned)(sk[p] >> 32);
            if (c < (unsigned)CUBE_N) {
                if (p == 0 || (unsigned)(sk[p - 1] >> 32) != c) K.a.first_new[c] = p;
                if (p == n - 1 || (unsigned)(sk[p + 1] >> 32) != c) K.a.last_new[c] = p;
            }
        }
        __syncthreads();
        for (int p = threadIdx.x; p < n; p += RBS_T) {
            const unsigned c = (unsigned)(sk[p] >> 32);
            if (c < (unsigned)CUBE_N) K.v2[(int)(sk[p] & 0xffffffffu)] = p - K.a.first_new[c];
        }
    }
    __syncthreads();                                      // run tables (global) -> the scan below
    cube_scan_body(K.a, valid, 0, nullptr);
}

__global__ void k_rb_scatter(RbKinds P) {
    const RbKind& K = P.k[blockIdx.y];
    const int n_old = *K.d_n, n_new = min(*K.d_stack_n, K.ub_new);
    const int stride = gridDim.x * MB;
    for (int i = blockIdx.x * MB + threadIdx.x; i < n_old; i += stride) {
        const int c = K.Acube[i];
        if (c < 0) continue;
        const int pos = K.a.off[c] + (i - K.a.first_old[c]);
        K.B[pos] = K.A[i];
        K.Bcube[pos] = c;
    }
    for (int i = blockIdx.x * MB + threadIdx.x; i < n_new; i += stride) {   // appended: rank within the cube
        const unsigned c = K.k1[i];
        if (c >= (unsigned)CUBE_N) continue;
        const int pos = K.a.off[c] + old_count(K.a, c) + K.v2[i];
        K.B[pos] = K.ins_pts[i];
        K.Bcube[pos] = (int)c;
    }
}

// part: 0 every cube; 1 the cubes above `fit` (and the empty ones), 2 the others (run concurrently on a second
// stream, so the split cubes' segment sorts need not wait for the longest in-LDS cube)
__global__ void __launch_bounds__(RBV_T) k_rb_cubevox(RbKinds P, const MapState* __restrict__ m, int seg_limit, int fit, int part) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RbKind& K = P.k[blockIdx.y];
    const int r = blockIdx.x;
    if (r >= m->valid_num) return;
    const int c = m->valid_ind[r];
    const CubeArrays& a = K.a;
    const int p0 = a.off[c], n = a.off[c + 1] - p0;
    int* segl = K.segl + (size_t)r * LS_SEGL;
    if (part == 2 && (n == 0 || n > fit)) return;
    // finished here unless split below; reset before any early return, or k_rb_cubeseg / k_rb_cubered would
    // read the list a split cube left in this slot in an earlier frame (part 1 resets every slot: k_rb_cubeseg
    // follows it on its stream)
    if (threadIdx.x == 0 && part != 2) segl[0] = 0;
    if (n == 0) { if (threadIdx.x == 0) a.seg_nout[c] = 0; return; }
    if (part == 1 && n <= fit) return;
    int fbv[3];
    const int* fb = nullptr;
    if (K.fast_keys) {                    // leaf base below the cube's box (cube_coord: x in [50 (ci - cen) - 25, +50])
        const int cc[3] = {c % CUBE_W, (c / CUBE_W) % CUBE_H, c / (CUBE_W * CUBE_H)}, cen[3] = {m->cenW, m->cenH, m->cenD};
        const float inv = 1.0f / K.leaf;
        for (int d = 0; d < 3; d++) fbv[d] = (int)floorf((float)(50.0 * (cc[d] - cen[d]) - 26.0) * inv);
        fb = fbv;
    }
    if (n <= fit) rbv_cube<true>(smem, K.B, a, c, p0, n, K.leaf, K.Cf, K.gscr, fb, segl, seg_limit);
    else rbv_cube<false>(smem, K.B, a, c, p0, n, K.leaf, K.Cf, K.gscr, fb, segl, seg_limit);
}

// the segments of the split cubes, RBV_SEGW workgroups per cube (blockIdx.x = cube slot * RBV_SEGW + w)
constexpr int RBV_SEGW = 16;
__global__ void __launch_bounds__(RBV_T) k_rb_cubeseg(RbKinds P, const MapState* __restrict__ m) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RbKind& K = P.k[blockIdx.y];
    const int r = blockIdx.x / RBV_SEGW, w = blockIdx.x % RBV_SEGW;
    if (r >= m->valid_num) return;
    const int* segl = K.segl + (size_t)r * LS_SEGL;
    if (segl[0] == 0) return;
    const int c = m->valid_ind[r];
    const int p0 = K.a.off[c], n = K.a.off[c + 1] - p0;
    unsigned long long* G = K.gscr + 4 * (size_t)p0;
    unsigned long long* EL = (unsigned long long*)(smem + RBV_HDR);
    ls_sort_list<RBV_T, RBV_CPW>(G, segl, w, RBV_SEGW, EL, RBV_CAP, (unsigned char*)(EL + RBV_CAP), rvg_rel(G, n));
}
// The same for segments of <= RBQ_CAP elements (seg_limit <= RBQ_CAP): 256 threads and ~28 KB of LDS, so
// several workgroups share a CU. One segment's sort is bound by its levels' barriers and dependent LDS
// round trips, not by the CU's lanes, so occupancy is what raises the throughput over many segments.
constexpr int RBQ_T = 256, RBQ_CPW = 8, RBQ_CAP = RBQ_T * RBQ_CPW;
constexpr size_t RBQ_LDS = 8 * (size_t)RBQ_CAP + ls_scratch_bytes(RBQ_T, RBQ_CAP);
constexpr int RBQ_SEGW = 32;
__global__ void __launch_bounds__(RBQ_T) k_rb_cubeseg_s(RbKinds P, const MapState* __restrict__ m) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const RbKind& K = P.k[blockIdx.y];
    const int r = blockIdx.x / RBQ_SEGW, w = blockIdx.x % RBQ_SEGW;
    if (r >= m->valid_num) return;
    const int* segl = K.segl + (size_t)r * LS_SEGL;
    if (segl[0] == 0) return;
    const int c = m->valid_ind[r];
    const int p0 = K.a.off[c], n = K.a.off[c + 1] - p0;
    unsigned long long* G = K.gscr + 4 * (size_t)p0;
    unsigned long long* EL = (unsigned long long*)smem;
    ls_sort_list<RBQ_T, RBQ_CPW>(G, segl, w, RBQ_SEGW, EL, RBQ_CAP, (unsigned char*)(EL + RBQ_CAP), rvg_rel(G, n));
}
// the split cubes' relevant points' positions after the segment replays, then the leaf sums (rvg.hpp R4)
__global__ void __launch_bounds__(RBV_T) k_rb_cubered(RbKinds P, const MapState* __restrict__ m) {
    __shared__ int sc[2 * (RBV_T / WAVE) + 2];
    const RbKind& K = P.k[blockIdx.y];
    const int r = blockIdx.x;
    if (r >= m->valid_num) return;
    if (K.segl[(size_t)r * LS_SEGL] == 0) return;
    const int c = m->valid_ind[r];
    const int p0 = K.a.off[c], n = K.a.off[c + 1] - p0;
    unsigned long long* G = K.gscr + 4 * (size_t)p0;
    rvg_positions<RBV_T>(G, n, rvg_rel(G, n), rvg_fpos(G, n));
    __syncthreads();
    const float4* B = K.B;
    float4* Cf = K.Cf;
    const int tot = rvg_reduce<RBV_T, true>(rvg_S(G, n), n, rvg_rel(G, n), rvg_fpos(G, n), [&](int i) { return B[p0 + i]; },
                                      [&](int q, float4 v) { Cf[p0 + q] = v; }, sc);
    if (threadIdx.x == 0) K.a.seg_nout[c] = tot;
}

__global__ void __launch_bounds__(1024) k_rb_final_scan(RbKinds P, const unsigned char* __restrict__ valid) {
    const RbKind& K = P.k[blockIdx.x];
    cube_scan_body(K.a, valid, 1, K.d_n);
}

// rebuilt map into A (valid cubes: their VoxelGrid output; others: old + appended as grouped), then the
// next rebuild's run tables
__global__ void k_rb_final(RbKinds P, const unsigned char* __restrict__ valid) {
    const RbKind& K = P.k[blockIdx.y];
    const CubeArrays& a = K.a;
    const int total = a.off[CUBE_N];
    for (int p = blockIdx.x * MB + threadIdx.x; p < total; p += gridDim.x * MB) {
        const int c = K.Bcube[p];
        const int local = p - a.off[c];
        if (!valid[c]) { K.A[a.final_off[c] + local] = K.B[p]; K.Acube[a.final_off[c] + local] = c; }
        else if (local < a.seg_nout[c]) { K.A[a.final_off[c] + local] = K.Cf[p]; K.Acube[a.final_off[c] + local] = c; }
    }
    for (int c = blockIdx.x * MB + threadIdx.x; c <= CUBE_N; c += gridDim.x * MB) {
        a.last_old[c] = -1; a.last_new[c] = -1; a.first_old[c] = 0x7fffffff; a.first_new[c] = 0x7fffffff;
    }
}

// ------------------------------------------------------------------------------------------
static int nblk(int n) { return std::max(1, std::min(2048, (n + MB - 1) / MB)); }

static CubeArrays cube_arrays(Ctx& C, int which) {
    CubeArrays a;
    int* base = C.d_cube_cnt + which * 7 * (CUBE_N + 1);
    a.first_old = base; a.last_old = base + (CUBE_N + 1); a.first_new = base + 2 * (CUBE_N + 1);
    a.last_new = base + 3 * (CUBE_N + 1); a.off = base + 4 * (CUBE_N + 1); a.seg_nout = base + 5 * (CUBE_N + 1);
    a.final_off = base + 6 * (CUBE_N + 1);
    return a;
}

// both kinds' map update (:739-797 + the per-cube VoxelGrid :799-820) in 6 launches on the frame's stream
static void rebuild_maps(Ctx& C, const float4* cstack, const float4* sstack, const int* stack_n, int ub_c, int ub_s) {
    hipStream_t st = C.stream;
    if (C.n_mc + C.n_ms + 2 * std::max(ub_c, ub_s) > C.cap_map) throw ApiError{ALOAM_E_CAPACITY, "map capacity exceeded"};
    RbKinds P;
    for (int w = 0; w < 2; w++) {
        RbKind& k = P.k[w];
        KindScratch& K = C.ks[w];
        k.stack = w == 0 ? cstack : sstack;
        k.d_stack_n = stack_n + w;
        k.ub_new = w == 0 ? ub_c : ub_s;
        k.leaf = w == 0 ? C.P.mapping_line_resolution : C.P.mapping_plane_resolution;
        k.A = w == 0 ? C.d_mc : C.d_ms;
        k.Acube = w == 0 ? C.d_mc_cube : C.d_ms_cube;
        k.d_n = C.d_map_n + w;
        k.n_old_ub = w == 0 ? C.n_mc : C.n_ms;
        k.B = w == 0 ? C.d_mc2 : C.d_ms2;
        k.Bcube = w == 0 ? C.d_mc2_cube : C.d_ms2_cube;
        k.ins_pts = K.ins_pts;
        k.k1 = (unsigned*)K.vkeys;
        k.v2 = K.ins_val2;
        k.Cf = K.map_tmp;
        k.gscr = K.seg_keys + 32768;
        k.segl = K.cube_segl;
        k.a = cube_arrays(C, w);
        static const bool bbox_keys = getenv("ALOAM_RB_BBOX") && atoi(getenv("ALOAM_RB_BBOX")) == 1;   // A/B knob
        k.fast_keys = !bbox_keys && k.leaf > 0.f && 53.0 / k.leaf + 2.0 < 1024.0;
    }
    const int n_old = std::max(C.n_mc, C.n_ms), ub = std::max(ub_c, ub_s);
    k_rb_insert<<<dim3(nblk(std::max(n_old, ub)), 2), MB, 0, st>>>(P, C.d_map);
    k_rb_sort_scan<<<2, RBS_T, RBS_LDS, st>>>(P, C.d_cube_valid);
    k_rb_scatter<<<dim3(nblk(n_old + ub), 2), MB, 0, st>>>(P);
    prof_phase(C, Ctx::PM_MAP_ADD);
    // tuning knobs: segment size of the split cubes' parallel sorts; cubes up to `fit` points are sorted
    // whole by their own workgroup, larger ones split. fit 2048 (round 5, was RVG_FIT = 4096): the slowest
    // cubes of a frame were in-LDS cubes of ~3900 points whose heap-sorted segments queued on the workgroup's
    // 4 waves; split, their segments spread over workgroups (profiles/r05_cube_fit_ab.txt: 1024 / 1536 /
    // 2048 / 3072 / 4096 -> 2048 best, C3 50 steps 1025 vs 992 scans/s)
    static const int seg_limit = getenv("ALOAM_CUBE_SEG") ? std::max(2048, std::min(RBV_CAP, atoi(getenv("ALOAM_CUBE_SEG")))) : 4096;
    static const int fit = getenv("ALOAM_CUBE_FIT") ? std::max(512, std::min(RVG_FIT, atoi(getenv("ALOAM_CUBE_FIT")))) : std::min(RVG_FIT, 2048);
    // ALOAM_RB_FORK=1: the cubes sorted in LDS on stream2 beside the split cubes' chain (split, segment sorts,
    // sums) on the frame's stream. Off by default: measured slower (C3 20 steps 867-870 vs 881-882 scans/s,
    // steady state 798-801 vs 819-821, profiles/r05_fork_ab.txt; the mapping rounds of the next frames ran
    // ~25 us longer, and both launches hold one workgroup per CU for their LDS)
    static const bool fork = getenv("ALOAM_RB_FORK") && atoi(getenv("ALOAM_RB_FORK")) == 1;
    if (fork) {
        fork_lane1(C);
        k_rb_cubevox<<<dim3(125, 2), RBV_T, RBV_LDS, C.stream2>>>(P, C.d_map, seg_limit, fit, 2);
    }
    k_rb_cubevox<<<dim3(125, 2), RBV_T, RBV_LDS, st>>>(P, C.d_map, seg_limit, fit, fork ? 1 : 0);
    if (seg_limit <= RBQ_CAP) k_rb_cubeseg_s<<<dim3(125 * RBQ_SEGW, 2), RBQ_T, RBQ_LDS, st>>>(P, C.d_map);
    else k_rb_cubeseg<<<dim3(125 * RBV_SEGW, 2), RBV_T, RBV_LDS, st>>>(P, C.d_map);
    k_rb_cubered<<<dim3(125, 2), RBV_T, 0, st>>>(P, C.d_map);
    if (fork) join_lane1(C);
    k_rb_final_scan<<<2, 1024, 0, st>>>(P, C.d_cube_valid);
    k_rb_final<<<dim3(nblk(n_old + ub), 2), MB, 0, st>>>(P, C.d_cube_valid);
    prof_phase(C, Ctx::PM_MAP_FILTER);
    HIPCHK(hipGetLastError());
}

// one-time state of the rebuild's run tables (afterwards every rebuild leaves them reset)
void rebuild_init(Ctx& C) {
    static bool attr = false;
    if (!attr) {
        HIPCHK(hipFuncSetAttribute((const void*)k_rb_cubevox, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RBV_LDS));
        HIPCHK(hipFuncSetAttribute((const void*)k_rb_cubeseg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RBV_LDS));
        HIPCHK(hipFuncSetAttribute((const void*)k_rb_cubeseg_s, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RBQ_LDS));
        HIPCHK(hipFuncSetAttribute((const void*)k_rb_sort_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RBS_LDS));
        attr = true;
    }
    for (int which = 0; which < 2; which++) {
        CubeArrays a;
        int* base = C.d_cube_cnt + which * 7 * (CUBE_N + 1);
        a.first_old = base; a.last_old = base + (CUBE_N + 1); a.first_new = base + 2 * (CUBE_N + 1);
        a.last_new = base + 3 * (CUBE_N + 1); a.off = base + 4 * (CUBE_N + 1); a.seg_nout = base + 5 * (CUBE_N + 1);
        a.final_off = base + 6 * (CUBE_N + 1);
        k_cube_reset<<<(CUBE_N + 1 + 255) / 256, 256, 0, C.stream>>>(a);
    }
    HIPCHK(hipGetLastError());
}

// The whole laserMapping frame; results are read back by the caller (aloam_api.hip).
static const int g_exp = getenv("ALOAM_EXP") ? atoi(getenv("ALOAM_EXP")) : 0;   // profiling experiments only
static const int g_assoc_blocks = getenv("ALOAM_ASSOC_BLOCKS") ? atoi(getenv("ALOAM_ASSOC_BLOCKS")) : ASSOC_BLOCKS;   // tuning knob
static const int g_fit_split = getenv("ALOAM_FIT_SPLIT") ? atoi(getenv("ALOAM_FIT_SPLIT")) : 0;   // tuning knob
static const int g_map_ag = getenv("ALOAM_MAP_AG") ? atoi(getenv("ALOAM_MAP_AG")) : 8;   // tuning knob: lanes per query (C3, serial on 256 CUs: 8 / 16 / 32 = 25.5 / 19.9 / 29.0 us; pipeline on 128 CUs: 8 / 16 = 22.2 / 24.6 us)
static const int g_map_u = getenv("ALOAM_MAP_U") ? atoi(getenv("ALOAM_MAP_U")) : 4;     // tuning knob: loads in flight
static const bool g_map_cache = getenv("ALOAM_MAP_NOCACHE") == nullptr;   // A/B knob: the rounds' candidate cache
__global__ void k_noop() {}
// ALOAM_MAP_PHASES (profiling aid): GPU time of the frame's phases from events on the frame's stream,
// read back two frames later (that frame is complete by then), means printed every 200 frames
static const bool g_map_phases = getenv("ALOAM_MAP_PHASES") != nullptr;
static void map_phase(Ctx& C, int k) {
    static hipEvent_t ev[2][5];
    static bool made = false, used[2] = {false, false};
    static double acc[5] = {0, 0, 0, 0, 0};
    static long frame = 0, nacc = 0;
    if (!made) { for (auto& r : ev) for (auto& e : r) HIPCHK(hipEventCreate(&e)); made = true; }
    const int s = (int)(frame & 1);
    if (k == 0 && used[s] && used[s ^ 1]) {
        HIPCHK(hipEventSynchronize(ev[s][4]));
        for (int i = 0; i < 4; i++) { float ms = 0; HIPCHK(hipEventElapsedTime(&ms, ev[s][i], ev[s][i + 1])); acc[i] += ms * 1e3; }
        float gap = 0;                   // the next frame's start - this frame's end (stream idle)
        HIPCHK(hipEventSynchronize(ev[s ^ 1][0]));
        HIPCHK(hipEventElapsedTime(&gap, ev[s][4], ev[s ^ 1][0]));
        acc[4] += gap * 1e3;
        if (++nacc % 200 == 0)
            std::fprintf(stderr, "[aloam map phases] us per frame: prepare+grids %.1f, rounds %.1f, rebuild %.1f, register %.1f, idle before %.1f (mean of %ld)\n",
                         acc[0] / nacc, acc[1] / nacc, acc[2] / nacc, acc[3] / nacc, acc[4] / nacc, nacc);
    }
    HIPCHK(hipEventRecord(ev[s][k], C.stream));
    if (k == 4) { used[s] = true; frame++; }
}

void map_frame_launch(Ctx& C, int X) {
    hipStream_t st = C.stream;
    Ctx::MapInSet& in = C.mset[X];
    int* stack_n = C.d_out->stack_n + 2 * X;
    const int ub_c = in.nc, ub_s = in.ns;
    // an input set written on another stream (stream3 hand-off, or this context's stream2 stacks): its
    // clouds, pose and stacks are complete at `ready` — wait before the first kernel that reads the pose
    const bool deferred = in.pstk;   // stacks copied right before the rounds (forward_stacks_pending)
    if (in.stacks || (in.stacks_pub && !deferred)) HIPCHK(hipStreamWaitEvent(st, in.ready, 0));
    if (g_map_phases) map_phase(C, 0);
    k_map_prepare<<<1, 256, 0, st>>>(C.d_map, C.d_cube_valid, C.d_map_spread, in.pose);
    k_map_shift<<<dim3(nblk(std::max(C.n_mc, C.n_ms)), 2), MB, 0, st>>>(C.d_mc_cube, C.d_ms_cube, C.d_map_n, C.d_map);
    prof_phase(C, Ctx::PM_MAP_SHIFT);
    const GridBuild gb[2] = {{&C.g_map_corner, C.d_mc, C.d_map_n + 0, std::max(C.n_mc, 1), C.d_mc_cube, C.d_cube_valid},
                             {&C.g_map_surf, C.d_ms, C.d_map_n + 1, std::max(C.n_ms, 1), C.d_ms_cube, C.d_cube_valid}};
    grid_build_multi(C, gb, 2);
    k_map_gate<<<1, 1, 0, st>>>(C.d_map, C.g_map_corner.desc, C.g_map_surf.desc);
    prof_phase(C, Ctx::PM_MAP_GRIDS);
    // stacks (:542-550): voxelised on stream3 when the input came as a hand-off, else here in two lanes
    if (deferred) {
        forward_stacks_pending(C, X);
    } else if (in.stacks_pub) {
        // present already: voxelised at this context's own publish (stream2), or at the source's and
        // copied in (this stream or stream3); `ready` is recorded behind either
        HIPCHK(hipStreamWaitEvent(st, in.ready, 0));
    } else if (in.stacks) {
        HIPCHK(hipStreamWaitEvent(st, in.ready, 0));
    } else {
        voxel_grid_pair_on(C, st, C.ks[0], in.corner, in.n + 0, ub_c, C.P.mapping_line_resolution, in.cstack, stack_n + 0,
                           in.surf, in.n + 1, ub_s, C.P.mapping_plane_resolution, in.sstack, stack_n + 1);
    }
    in.stacks = false;
    in.stacks_pub = false;
    const int nq = ub_c + ub_s;
    if (g_map_phases) map_phase(C, 1);
    prof_phase(C, Ctx::PM_MAP_ROUNDS_BEGIN);
    C.t_rounds_issued = std::chrono::steady_clock::now();
    if (nq > 0) {
        if (nq > C.cap_factors) throw ApiError{ALOAM_E_CAPACITY, "factor capacity exceeded"};
        const int rounds = std::min(C.P.map_rounds, ALOAM_MAX_ROUNDS);
        // every size comes from the device (stack counts, grids, gate): one fixed launch sequence per set
        auto issue = [&C, st, rounds, &in, stack_n](bool marks, int live_hint) {
            for (int it = 0; it < rounds; it++) {
                if (marks) prof_mark(C, 6 + 2 * (ALOAM_MAX_ROUNDS + it));
                int* cnt = C.d_map_spread + (size_t)it * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE;
                auto kern = g_map_ag == 16 ? (g_map_u == 8 ? k_map_assoc<16, 8> : k_map_assoc<16, 4>)
                          : g_map_ag == 32 ? (g_map_u == 8 ? k_map_assoc<32, 8> : k_map_assoc<32, 4>)
                                           : (g_map_u == 8 ? k_map_assoc<8, 8> : k_map_assoc<8, 4>);
                const MapCache mc{g_map_cache ? C.d_mc_ctr : nullptr, C.d_mc_pts, C.d_mc_pos, C.d_mc_prev, C.cap_mq, it};
                kern<<<g_assoc_blocks, 256, 0, st>>>(
                    in.cstack, in.sstack, stack_n,
                    C.g_map_corner.desc, C.g_map_corner.cell_start, C.g_map_corner.pts, C.g_map_corner.idx,
                    C.g_map_surf.desc, C.g_map_surf.cell_start, C.g_map_surf.pts, C.g_map_surf.idx, C.d_map, C.d_factors, cnt,
                    g_fit_split ? C.d_nbr : nullptr, C.profiling ? C.d_cand : nullptr, g_exp, mc);
                if (g_fit_split)
                    k_map_fit<<<FIT_BLOCKS, 256, 0, st>>>(in.cstack, in.sstack, stack_n, C.g_map_corner.pts, C.g_map_surf.pts, C.d_map,
                                                         C.d_nbr, C.d_factors, cnt);
                if (marks) prof_mark(C, 7 + 2 * (ALOAM_MAX_ROUNDS + it));
                if (g_exp & 16) k_noop<<<1, 64, 0, st>>>();   // (profiling experiment 16: cost of a kernel boundary)
                lm_run(C, C.d_factors, C.cap_factors, C.d_map->parameters, ALOAM_MAX_ROUNDS + it, &C.d_map->optimize,
                       stack_n, live_hint);
            }
        };
        const int hint = C.map_slots_hint > 0 ? C.map_slots_hint : 4096;
        if (C.profiling || !C.use_graphs) issue(true, hint);
        else run_graph(C, 2 + X, in.cstack, in.sstack, rounds, [&] { issue(false, hint); });
    }
    if (g_map_phases) map_phase(C, 2);
    prof_phase(C, Ctx::PM_MAP_ROUNDS_END);
    k_map_update<<<1, 64, 0, st>>>(C.d_map, C.d_map_spread, std::min(C.P.map_rounds, ALOAM_MAX_ROUNDS),
                                   C.d_round_cnt + 2 * ALOAM_MAX_ROUNDS);
    if (g_exp & 4) {                 // (profiling experiment 4: skip the map update — results invalid)
    } else {
        rebuild_maps(C, in.cstack, in.sstack, stack_n, ub_c, ub_s);
    }
    if (g_map_phases) map_phase(C, 3);
    if (in.nf > 0)
        k_map_register<<<(in.nf + MB - 1) / MB, MB, 0, st>>>(in.full, in.nf, C.d_map, C.d_registered);
    if (g_map_phases) map_phase(C, 4);
    HIPCHK(hipGetLastError());
}

// ps_serial_std_sort calls of this translation unit's kernels (aloam_serial_sort_fallbacks)
unsigned long long serial_sort_calls_map() {
    unsigned long long v = 0;
    HIPCHK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ps_serial_calls), sizeof(v)));
    return v;
}

}  // namespace aloam
