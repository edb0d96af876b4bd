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
#include "aloam_device.hpp"
#include "aloam_internal.hpp"
#include "eigen_small.hpp"

namespace aloam {

void prof_mark(Ctx& C, int idx);
void stable_sort_pairs(Ctx& C, unsigned* kin, unsigned* kout, int* vin, int* vout, int n, int end_bit);
void segment_voxel_launch(Ctx& C, const float4* pts, const int* off, const int* seg_list, const int* nseg_p, int max_seg,
                          float leaf, float4* out, int* seg_nout, unsigned long long* gkeys);

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

__global__ void k_map_prepare(MapState* m, unsigned char* cube_valid) {
    __shared__ int valid_num;
    if (threadIdx.x == 0) {
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
__global__ void k_map_shift(int* __restrict__ cube, const int* d_n, const MapState* m) {
    const int si = m->shift[0], sj = m->shift[1], sk = m->shift[2];
    if (si == 0 && sj == 0 && sk == 0) return;
    const int n = *d_n;
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

// one wave per stack point: 5-NN within 1 m (d^2[4] < 1.0, :583-584,649-650)
__global__ void __launch_bounds__(256) k_map_knn5(
    const float4* __restrict__ cstack, const float4* __restrict__ sstack, const int* stack_n, int ub_c, int ub_s,
    const GridDesc* __restrict__ gdc, const int* __restrict__ cs_c, const float4* __restrict__ sp_c, const int* __restrict__ si_c,
    const GridDesc* __restrict__ gds, const int* __restrict__ cs_s, const float4* __restrict__ sp_s, const int* __restrict__ si_s,
    const MapState* __restrict__ m, int* __restrict__ nbr, unsigned long long* cand_count) {
    const int qi = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (qi >= ub_c + ub_s) return;
    if (!m->optimize) return;
    const bool corner = qi < ub_c;
    const int li = corner ? qi : qi - ub_c;
    int* out = nbr + (size_t)qi * 5;
    if (li >= stack_n[corner ? 0 : 1]) { if (lane_id() == 0) out[0] = -1; return; }
    const float4 sel = associate_to_map(m->parameters, corner ? cstack[li] : sstack[li]);
    const GridDesc gd = corner ? *gdc : *gds;
    const int* cs = corner ? cs_c : cs_s;
    const float4* sp = corner ? sp_c : sp_s;
    const int* si = corner ? si_c : si_s;
    // per-lane sorted top-5 then 5 wave-min rounds (ties by point index)
    float bd[5]; int bi[5], bp[5];
#pragma unroll
    for (int k = 0; k < 5; k++) { bd[k] = INFINITY; bi[k] = 0x7fffffff; bp[k] = -1; }
    const float fx = (sel.x - gd.ox) * gd.inv_cell, fy = (sel.y - gd.oy) * gd.inv_cell, fz = (sel.z - gd.oz) * gd.inv_cell;
    const int cx = (int)floorf(fx), cy = (int)floorf(fy), cz = (int)floorf(fz);
    const int x0 = (fx - cx < 0.5f) ? cx - 1 : cx, y0 = (fy - cy < 0.5f) ? cy - 1 : cy, z0 = (fz - cz < 0.5f) ? cz - 1 : cz;
    int ncand = 0;
    for (int c8 = 0; c8 < 8; c8++) {
        const int x = x0 + (c8 & 1), y = y0 + ((c8 >> 1) & 1), z = z0 + (c8 >> 2);
        if (x < 0 || y < 0 || z < 0 || x >= gd.dx || y >= gd.dy || z >= gd.dz) continue;
        const int c = (z * gd.dy + y) * gd.dx + x;
        const int b = cs[c], e = cs[c + 1];
        ncand += e - b;
        for (int p = b + lane_id(); p < e; p += WAVE) {
            const float4 v = sp[p];
            const float d2 = sqdist(v.x, v.y, v.z, sel.x, sel.y, sel.z);
            if (!(d2 < 1.0f)) continue;
            const int id = si[p];
            if (d2 < bd[4] || (d2 == bd[4] && id < bi[4])) {
                float nd = d2; int ni = id, np = p;
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    const bool lt = nd < bd[k] || (nd == bd[k] && ni < bi[k]);
                    if (lt) { float td = bd[k]; int ti = bi[k], tp = bp[k]; bd[k] = nd; bi[k] = ni; bp[k] = np; nd = td; ni = ti; np = tp; }
                }
            }
        }
    }
    int head = 0, res[5];
    int found = 0;
    for (int k = 0; k < 5; k++) {
        float hd = INFINITY; int hi = 0x7fffffff, hp = -1;
#pragma unroll
        for (int j = 0; j < 5; j++) if (j == head) { hd = bd[j]; hi = bi[j]; hp = bp[j]; }
        const unsigned long long key = hp < 0 ? ~0ull : dist_key(hd, hi);
        const unsigned long long mn = wave_min_u64(key);
        if (mn == ~0ull) break;
        const unsigned long long won = __ballot(key == mn);
        if (key == mn) head++;
        res[k] = __shfl(hp, __ffsll((long long)won) - 1, WAVE);
        found++;
    }
    if (lane_id() == 0) {
        if (found == 5) for (int k = 0; k < 5; k++) out[k] = res[k];
        else out[0] = -1;
        if (cand_count) atomicAdd(cand_count, (unsigned long long)ncand);
    }
}

// one thread per stack point: line / plane fit and the factor (:585-620, :650-686)
__global__ void k_map_fit(const float4* __restrict__ cstack, const float4* __restrict__ sstack, int ub_c, int ub_s,
                          const float4* __restrict__ sp_c, const float4* __restrict__ sp_s, const int* __restrict__ nbr,
                          const MapState* __restrict__ m, aloam_factor* __restrict__ out, int* round_cnt) {
    const int qi = blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= ub_c + ub_s) return;
    aloam_factor f;
    f.type = -1; f.pad = 0;
    if (!m->optimize) return;
    const int* nb = nbr + (size_t)qi * 5;
    const bool corner = qi < ub_c;
    if (nb[0] >= 0) {
        const float4 po = corner ? cstack[qi] : sstack[qi - ub_c];
        f.cp[0] = po.x; f.cp[1] = po.y; f.cp[2] = po.z;
        if (corner) {
            double pts[5][3];
            double cx = 0, cy = 0, cz = 0;
            for (int j = 0; j < 5; j++) {
                const float4 v = sp_c[nb[j]];
                pts[j][0] = v.x; pts[j][1] = v.y; pts[j][2] = v.z;
                cx = cx + pts[j][0]; cy = cy + pts[j][1]; cz = cz + pts[j][2];
            }
            cx = cx / 5.0; cy = cy / 5.0; cz = cz / 5.0;
            double cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int j = 0; j < 5; j++) {
                const double zm[3] = {pts[j][0] - cx, pts[j][1] - cy, pts[j][2] - cz};
                for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) cov[r * 3 + c] = cov[r * 3 + c] + zm[r] * zm[c];
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
            for (int j = 0; j < 5; j++) {
                const float4 v = sp_s[nb[j]];
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
            for (int j = 0; j < 5; j++)
                if (fabs(n[0] * P[j][0] + n[1] * P[j][1] + n[2] * P[j][2] + negOA) > 0.2) { valid = false; break; }
            if (valid) {
                f.type = 2;
                f.a[0] = n[0]; f.a[1] = n[1]; f.a[2] = n[2];
                f.b[0] = negOA; f.b[1] = 0; f.b[2] = 0;
            }
        }
    }
    out[qi] = f;
    if (f.type >= 0) atomicAdd(&round_cnt[corner ? 0 : 1], 1);
}

__global__ void k_map_invalidate(aloam_factor* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i].type = -1;
}

// transformUpdate (:148-152)
__global__ void k_map_update(MapState* m) {
    const dquat qw{m->parameters[0], m->parameters[1], m->parameters[2], m->parameters[3]};
    const dquat qo{m->q_wodom[0], m->q_wodom[1], m->q_wodom[2], m->q_wodom[3]};
    const dquat qm = qmul(qw, qinv(qo));
    m->q_wmap_wodom[0] = qm.x; m->q_wmap_wodom[1] = qm.y; m->q_wmap_wodom[2] = qm.z; m->q_wmap_wodom[3] = qm.w;
    const dvec3 r = qrot(qm, {m->t_wodom[0], m->t_wodom[1], m->t_wodom[2]});
    m->t_wmap_wodom[0] = m->parameters[4] - r.x;
    m->t_wmap_wodom[1] = m->parameters[5] - r.y;
    m->t_wmap_wodom[2] = m->parameters[6] - r.z;
}

// stack point -> map frame -> cube (:739-783). key = cube (or PAD_CUBE when outside the grid)
__global__ void k_map_insert(const float4* __restrict__ stack, const int* d_n, int ub, const MapState* __restrict__ m,
                             float4* __restrict__ ins_pts, unsigned* __restrict__ key, int* __restrict__ val) {
    const int n = *d_n;
    for (int i = blockIdx.x * MB + threadIdx.x; i < ub; i += gridDim.x * MB) {
        unsigned k = PAD_CUBE;
        if (i < n) {
            const float4 s = associate_to_map(m->parameters, stack[i]);
            ins_pts[i] = s;
            const int ci = cube_coord(s.x, m->cenW), cj = cube_coord(s.y, m->cenH), ck = cube_coord(s.z, m->cenD);
            if (ci >= 0 && ci < CUBE_W && cj >= 0 && cj < CUBE_H && ck >= 0 && ck < CUBE_D)
                k = (unsigned)(ci + CUBE_W * cj + CUBE_W * CUBE_H * ck);
        }
        key[i] = k;
        val[i] = i;
    }
}

// cube bookkeeping arrays: cnt_old, cnt_new, first_old, first_new, off, seg_nout, final_off (each CUBE_N+1)
struct CubeArrays { int *cnt_old, *cnt_new, *first_old, *first_new, *off, *seg_nout, *final_off; };

__global__ void k_cube_reset(CubeArrays a) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c <= CUBE_N; c += gridDim.x * blockDim.x) {
        a.cnt_old[c] = 0; a.cnt_new[c] = 0; a.first_old[c] = 0x7fffffff; a.first_new[c] = 0x7fffffff; a.seg_nout[c] = 0;
    }
}
__global__ void k_cube_count_old(const int* __restrict__ cube, const int* d_n, CubeArrays a) {
    const int n = *d_n;
    for (int i = blockIdx.x * MB + threadIdx.x; i < n; i += gridDim.x * MB) {
        const int c = cube[i];
        if (c < 0) continue;
        atomicAdd(&a.cnt_old[c], 1);
        atomicMin(&a.first_old[c], i);
    }
}
__global__ void k_cube_count_new(const unsigned* __restrict__ skey, int ub, CubeArrays a) {
    for (int p = blockIdx.x * MB + threadIdx.x; p < ub; p += gridDim.x * MB) {
        const unsigned c = skey[p];
        if (c >= (unsigned)CUBE_N) continue;
        atomicAdd(&a.cnt_new[c], 1);
        atomicMin(&a.first_new[c], p);
    }
}
// single block: exclusive scan over cubes of v(c); mode 0: cnt_old+cnt_new -> off ; mode 1: final counts -> final_off
__global__ void k_cube_scan(CubeArrays a, const unsigned char* __restrict__ valid, int mode, int* total) {
    __shared__ int sh[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    int* dst = mode == 0 ? a.off : a.final_off;
    for (int base = 0; base < CUBE_N; base += 1024) {
        const int c = base + threadIdx.x;
        int v = 0;
        if (c < CUBE_N) {
            if (mode == 0) v = a.cnt_old[c] + a.cnt_new[c];
            else v = valid[c] ? a.seg_nout[c] : a.cnt_old[c] + a.cnt_new[c];
        }
        sh[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            int t = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += t;
            __syncthreads();
        }
        const int incl = sh[threadIdx.x];
        if (c < CUBE_N) dst[c] = carry + incl - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) { dst[CUBE_N] = carry; if (total) *total = carry; }
}
__global__ void k_cube_scatter(const float4* __restrict__ old_pts, const int* __restrict__ old_cube, const int* d_n_old,
                               const float4* __restrict__ ins_pts, const unsigned* __restrict__ skey, const int* __restrict__ sval,
                               int ub_new, CubeArrays a, float4* __restrict__ B, int* __restrict__ Bcube) {
    const int n_old = *d_n_old;
    const int stride = gridDim.x * MB;
    for (int i = blockIdx.x * MB + threadIdx.x; i < n_old; i += stride) {
        const int c = old_cube[i];
        if (c < 0) continue;
        const int pos = a.off[c] + (i - a.first_old[c]);
        B[pos] = old_pts[i];
        Bcube[pos] = c;
    }
    for (int p = blockIdx.x * MB + threadIdx.x; p < ub_new; p += stride) {
        const unsigned c = skey[p];
        if (c >= (unsigned)CUBE_N) continue;
        const int pos = a.off[c] + a.cnt_old[c] + (p - a.first_new[c]);
        B[pos] = ins_pts[sval[p]];
        Bcube[pos] = (int)c;
    }
}
__global__ void k_cube_final(const float4* __restrict__ B, const int* __restrict__ Bcube, const float4* __restrict__ Cf,
                             const unsigned char* __restrict__ valid, CubeArrays a, float4* __restrict__ A, int* __restrict__ Acube) {
    const int total = a.off[CUBE_N];
    for (int p = blockIdx.x * MB + threadIdx.x; p < total; p += gridDim.x * MB) {
        const int c = Bcube[p];
        const int local = p - a.off[c];
        if (!valid[c]) { A[a.final_off[c] + local] = B[p]; Acube[a.final_off[c] + local] = c; }
        else if (local < a.seg_nout[c]) { A[a.final_off[c] + local] = Cf[p]; Acube[a.final_off[c] + local] = c; }
    }
}

__global__ void k_map_register(const float4* __restrict__ full, int n, const MapState* __restrict__ m, float4* __restrict__ out) {
    const int i = blockIdx.x * MB + threadIdx.x;
    if (i < n) out[i] = associate_to_map(m->parameters, full[i]);
}

__global__ void k_copy_int(const int* src, int* dst) { *dst = *src; }

// ------------------------------------------------------------------------------------------
static int nblk(int n) { return std::max(1, std::min(2048, (n + MB - 1) / MB)); }

static void rebuild_map(Ctx& C, int which, int ub_new, const float4* stack, const int* d_stack_n, float leaf) {
    hipStream_t st = C.stream;
    float4* A = which == 0 ? C.d_mc : C.d_ms;
    int* Acube = which == 0 ? C.d_mc_cube : C.d_ms_cube;
    float4* B = which == 0 ? C.d_mc2 : C.d_ms2;
    int* Bcube = which == 0 ? C.d_mc2_cube : C.d_ms2_cube;
    const int n_old_ub = which == 0 ? C.n_mc : C.n_ms;
    int* d_n_old = C.d_map_n + which;
    // scratch carving: cube arrays live in d_cube_cnt ([7][CUBE_N+1])
    CubeArrays a;
    int* base = C.d_cube_cnt + which * 7 * (CUBE_N + 1);
    a.cnt_old = base; a.cnt_new = base + (CUBE_N + 1); a.first_old = base + 2 * (CUBE_N + 1);
    a.first_new = base + 3 * (CUBE_N + 1); a.off = base + 4 * (CUBE_N + 1); a.seg_nout = base + 5 * (CUBE_N + 1);
    a.final_off = base + 6 * (CUBE_N + 1);
    if (C.n_mc + C.n_ms + 2 * ub_new > C.cap_map) throw ApiError{ALOAM_E_CAPACITY, "map capacity exceeded"};
    unsigned* k1 = (unsigned*)C.d_vkeys;
    unsigned* k2 = (unsigned*)C.d_vkeys2;
    k_map_insert<<<nblk(ub_new), MB, 0, st>>>(stack, d_stack_n, ub_new, C.d_map, C.d_ins_pts, k1, C.d_ins_val);
    if (ub_new > 0) stable_sort_pairs(C, k1, k2, C.d_ins_val, C.d_ins_val2, ub_new, 13);
    k_cube_reset<<<(CUBE_N + 1 + 255) / 256, 256, 0, st>>>(a);
    k_cube_count_old<<<nblk(n_old_ub), MB, 0, st>>>(Acube, d_n_old, a);
    k_cube_count_new<<<nblk(ub_new), MB, 0, st>>>(k2, ub_new, a);
    k_cube_scan<<<1, 1024, 0, st>>>(a, C.d_cube_valid, 0, nullptr);
    k_cube_scatter<<<nblk(n_old_ub + ub_new), MB, 0, st>>>(A, Acube, d_n_old, C.d_ins_pts, k2, C.d_ins_val2, ub_new, a, B, Bcube);
    // per-cube VoxelGrid of the surrounding cubes into the insertion scratch at the same offsets
    float4* Cf = C.d_map_tmp;
    segment_voxel_launch(C, B, a.off, C.d_map->valid_ind, &C.d_map->valid_num, 125, leaf, Cf, a.seg_nout, C.d_seg_keys);
    k_cube_scan<<<1, 1024, 0, st>>>(a, C.d_cube_valid, 1, d_n_old);
    k_cube_final<<<nblk(n_old_ub + ub_new), MB, 0, st>>>(B, Bcube, Cf, C.d_cube_valid, a, A, Acube);
    HIPCHK(hipGetLastError());
}

// The whole laserMapping frame; results are read back by the caller (aloam_api.hip).
void map_frame_launch(Ctx& C, aloam_map_result* R) {
    hipStream_t st = C.stream;
    (void)R;
    const int ub_c = C.n_map_corner_in, ub_s = C.n_map_surf_in;
    k_map_prepare<<<1, 256, 0, st>>>(C.d_map, C.d_cube_valid);
    k_map_shift<<<nblk(C.n_mc), MB, 0, st>>>(C.d_mc_cube, C.d_map_n + 0, C.d_map);
    k_map_shift<<<nblk(C.n_ms), MB, 0, st>>>(C.d_ms_cube, C.d_map_n + 1, C.d_map);
    grid_build(C, C.g_map_corner, C.d_mc, C.d_map_n + 0, std::max(C.n_mc, 1), C.d_mc_cube, C.d_cube_valid);
    grid_build(C, C.g_map_surf, C.d_ms, C.d_map_n + 1, std::max(C.n_ms, 1), C.d_ms_cube, C.d_cube_valid);
    k_map_gate<<<1, 1, 0, st>>>(C.d_map, C.g_map_corner.desc, C.g_map_surf.desc);
    // stacks (:542-550)
    voxel_grid_sorted(C, C.d_map_corner_in, C.d_map_in_n + 0, ub_c, C.P.mapping_line_resolution, C.d_cstack, C.d_stack_n + 0);
    voxel_grid_sorted(C, C.d_map_surf_in, C.d_map_in_n + 1, ub_s, C.P.mapping_plane_resolution, C.d_sstack, C.d_stack_n + 1);
    const int nq = ub_c + ub_s;
    HIPCHK(hipMemsetAsync(C.d_round_cnt + 2 * ALOAM_MAX_ROUNDS, 0, sizeof(int) * 2 * ALOAM_MAX_ROUNDS, st));
    if (nq > 0) {
        if (nq > C.cap_factors) throw ApiError{ALOAM_E_CAPACITY, "factor capacity exceeded"};
        k_map_invalidate<<<(nq + 255) / 256, 256, 0, st>>>(C.d_factors, nq);
        const int rounds = std::min(C.P.map_rounds, ALOAM_MAX_ROUNDS);
        for (int it = 0; it < rounds; it++) {
            prof_mark(C, 6 + 2 * (ALOAM_MAX_ROUNDS + it));
            k_map_knn5<<<(nq * WAVE + 255) / 256, 256, 0, st>>>(
                C.d_cstack, C.d_sstack, C.d_stack_n, ub_c, ub_s,
                C.g_map_corner.desc, C.g_map_corner.cell_start, C.g_map_corner.pts, C.g_map_corner.idx,
                C.g_map_surf.desc, C.g_map_surf.cell_start, C.g_map_surf.pts, C.g_map_surf.idx, C.d_map, C.d_nbr, C.profiling ? C.d_cand : nullptr);
            prof_mark(C, 7 + 2 * (ALOAM_MAX_ROUNDS + it));
            k_map_fit<<<(nq + 127) / 128, 128, 0, st>>>(C.d_cstack, C.d_sstack, ub_c, ub_s, C.g_map_corner.pts, C.g_map_surf.pts,
                                                        C.d_nbr, C.d_map, C.d_factors, C.d_round_cnt + 2 * ALOAM_MAX_ROUNDS + 2 * it);
            lm_run(C, C.d_factors, nq, C.d_map->parameters, ALOAM_MAX_ROUNDS + it, &C.d_map->optimize);
        }
    }
    k_map_update<<<1, 1, 0, st>>>(C.d_map);
    rebuild_map(C, 0, ub_c, C.d_cstack, C.d_stack_n + 0, C.P.mapping_line_resolution);
    rebuild_map(C, 1, ub_s, C.d_sstack, C.d_stack_n + 1, C.P.mapping_plane_resolution);
    if (C.n_map_full_in > 0)
        k_map_register<<<(C.n_map_full_in + MB - 1) / MB, MB, 0, st>>>(C.d_map_full_in, C.n_map_full_in, C.d_map, C.d_registered);
    HIPCHK(hipGetLastError());
}

}  // namespace aloam
