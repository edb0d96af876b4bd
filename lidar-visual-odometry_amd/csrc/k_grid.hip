// k_grid.hip — dense uniform grid index + exact radius k-NN (replaces pcl::KdTreeFLANN).
//
// The reference accepts a neighbour only inside a fixed radius: 1-NN with d^2 < 25 in odometry
// (src/laserOdometry.cpp:386-389,470-473) and 5-NN with d^2[4] < 1 in mapping
// (src/laserMapping.cpp:582-584,648-650). So an exact radius-r k-NN over a grid returns FLANN's
// answer as long as the searched cell block contains the r-ball: with cells of edge >= r the query
// cell's 3x3x3 block does (wave_knn_rows in aloam_device.hpp). Distances are fp32
// ((dx^2 + dy^2) + dz^2) like FLANN's L2_Simple<float>; equal distances are ordered by point index.
//
// Build = counting sort by cell: bbox (ordered-int atomics) -> per-cell counts -> exclusive scan ->
// scatter (atomic decrement, which leaves the count array zeroed for the next build).
#include <climits>

#include "aloam_device.hpp"
#include "aloam_internal.hpp"

namespace aloam {

constexpr int GB = 256;

__device__ inline void grid_params(const unsigned bb[6], float min_cell, int nlayers, int flat, int max_cells, GridDesc* d) {
    float mn[3], mx[3];
    for (int a = 0; a < 3; a++) { mn[a] = ord2f(bb[a]); mx[a] = ord2f(bb[3 + a]); }
    float cell = min_cell;
    int dims[3];
    for (int it = 0; it < 64; it++) {
        long long prod = nlayers;
        for (int a = 0; a < 3; a++) {
            float ext = mx[a] - mn[a];
            if (!(ext >= 0.f)) ext = 0.f;
            dims[a] = (a == 2 && flat) ? 1 : (int)(ext / cell) + 2;
            prod *= dims[a];
        }
        if (prod <= max_cells) break;
        cell *= 1.25f;
    }
    d->ox = mn[0]; d->oy = mn[1]; d->oz = mn[2];
    d->cell = cell; d->inv_cell = 1.0f / cell;
    d->dx = dims[0]; d->dy = dims[1]; d->dz = dims[2];
    d->ncells = dims[0] * dims[1] * dims[2] * nlayers;
    d->nlayers = nlayers;
}

__device__ inline int cell_coord(float v, float o, float inv) { return (int)floorf((v - o) * inv); }

__global__ void k_grid_init(GridDesc* d) {
    if (threadIdx.x < 6) d->bb[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    if (threadIdx.x == 0) { d->n = 0; d->n_acc = 0; d->ncells = 0; d->npass = 1; d->ticket = 0; }
}

// Runs of equal cell ids among consecutive lanes (input clouds come line by line, so neighbours
// mostly share a cell): one atomic per run instead of per point — same-address atomics serialise
// at L2. Returns each lane's run length (valid at the head) and its run head lane. c < 0 = none.
__device__ __forceinline__ void cell_runs(int c, int* len, int* head) {
    const int lane = lane_id();
    const int prev = __builtin_amdgcn_update_dpp(-2, c, 0x138, 0xF, 0xF, false);   // wave_shr:1 (lane - 1)
    const bool hd = c >= 0 && (lane == 0 || prev != c);
    const unsigned long long heads = __ballot(hd), brk = __ballot(hd || c < 0);
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int h = 63 - __clzll(heads & upto | 1ull);                 // my run's head (0 if none)
    const unsigned long long above = brk & ~(lane == 63 ? ~0ull : ((2ull << lane) - 1));
    *len = (above ? __ffsll((long long)above) - 1 : WAVE) - lane;   // at a head: distance to next break
    *head = h;
}

__device__ inline bool grid_include(int i, const int* cube_of, const unsigned char* cube_valid) {
    if (!cube_of) return true;
    int c = cube_of[i];
    return c >= 0 && cube_valid[c];
}



// two-launch exclusive scan of cell_count[0, ncells) into cell_start: chunk sums, then per chunk the
// sum of the preceding chunk sums + a local scan. 1024 threads x 16 consecutive cells per chunk (int4
// loads), so an 8M-cell grid is 512 chunks and the chunk-sum prefix is one value per thread.
constexpr int SCAN_T = 1024, SCAN_PER = 16, SCAN_CHUNK = SCAN_T * SCAN_PER;
constexpr int SCAN_CPT = 4;      // chunk sums per thread in the second scan launch
static_assert(GRID_MAX_CELLS_BIG / SCAN_CHUNK <= SCAN_T * SCAN_CPT, "chunk sums: SCAN_CPT per thread");
__device__ __forceinline__ void load16(const int* __restrict__ cnt, int i0, int nc, int v[SCAN_PER]) {
    if (i0 + SCAN_PER <= nc) {
        const int4* q = (const int4*)(cnt + i0);
#pragma unroll
        for (int k = 0; k < SCAN_PER / 4; k++) { const int4 t = q[k]; v[4 * k] = t.x; v[4 * k + 1] = t.y; v[4 * k + 2] = t.z; v[4 * k + 3] = t.w; }
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_PER; k++) v[k] = i0 + k < nc ? cnt[i0 + k] : 0;
    }
}
__device__ __forceinline__ void k_grid_scan1_body(const int* __restrict__ cnt, const int nc, int* blk) {
    const int base = blockIdx.x * SCAN_CHUNK;
    int v[SCAN_PER];
    load16(cnt, base + threadIdx.x * SCAN_PER, nc, v);
    int s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) s += v[k];
    int tot;
    (void)block_exscan<SCAN_T, true>(s, &tot);
    if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}
__device__ __forceinline__ void k_grid_scan3_body(const int* __restrict__ cnt, const int nc, const int* blk, int* start) {
    const int base = blockIdx.x * SCAN_CHUNK;
    const int i0 = base + threadIdx.x * SCAN_PER;
    int v[SCAN_PER];
    load16(cnt, i0, nc, v);
    int pre = 0;                                                             // chunks before this one
#pragma unroll
    for (int c = 0; c < SCAN_CPT; c++) {
        const int ci = threadIdx.x * SCAN_CPT + c;
        if (ci < (int)blockIdx.x) pre += blk[ci];
    }
    int s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) s += v[k];
    int tot, ptot;
    const int ex = block_exscan<SCAN_T, true>(s, &tot);
    (void)block_exscan<SCAN_T, true>(pre, &ptot);
    int run = ptot + ex;
    if (i0 + SCAN_PER <= nc) {
        int4* q = (int4*)(start + i0);
#pragma unroll
        for (int k = 0; k < SCAN_PER / 4; k++) {
            int4 t;
            t.x = run; run += v[4 * k];
            t.y = run; run += v[4 * k + 1];
            t.z = run; run += v[4 * k + 2];
            t.w = run; run += v[4 * k + 3];
            q[k] = t;
        }
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_PER; k++) { if (i0 + k < nc) start[i0 + k] = run; run += v[k]; }
    }
    if (base + SCAN_CHUNK >= nc && threadIdx.x == 0) start[nc] = ptot + tot;
}

void grid_alloc(Ctx& C, Grid& g, int cap, float min_cell, int nlayers, bool w_index, bool flat, int max_cells) {
    if (max_cells > GRID_MAX_CELLS_BIG) throw ApiError{ALOAM_E_ARG, "grid_alloc: cell cap above GRID_MAX_CELLS_BIG"};
    g.cap = cap;
    g.max_cells = max_cells;
    g.flat = flat;
    g.min_cell = min_cell;
    g.nlayers = nlayers;
    g.w_index = w_index;
    g.desc = (GridDesc*)dalloc(C, sizeof(GridDesc));
    g.cell_count = (int*)dalloc(C, sizeof(int) * ((size_t)max_cells + 1));
    g.cell_start = (int*)dalloc(C, sizeof(int) * ((size_t)max_cells + 1));
    g.blk = (int*)dalloc(C, sizeof(int) * (SCAN_T * SCAN_CPT));
    g.pts = (float4*)dalloc(C, sizeof(float4) * cap);
    g.idx = (int*)dalloc(C, sizeof(int) * cap);
    g.pcell = (int*)dalloc(C, sizeof(int) * cap);
    k_grid_init<<<1, 64, 0, C.stream>>>(g.desc);      // bbox armed for the first build
    HIPCHK(hipGetLastError());
}

void grid_free(Ctx& C, Grid& g) {
    for (void* p : {(void*)g.desc, (void*)g.cell_count, (void*)g.cell_start, (void*)g.blk, (void*)g.pts, (void*)g.idx, (void*)g.pcell,
                    (void*)g.rk[0], (void*)g.rk[1], (void*)g.rv[0], (void*)g.rv[1], (void*)g.rH, (void*)g.rHo, (void*)g.rblk,
                    (void*)g.rbb, (void*)g.rcf})
        if (p) dfree(C, p);
    g = Grid{};
}

void grid_build(Ctx& C, Grid& g, const float4* pts, const int* d_n, int cap_n, const int* cube_of,
                const unsigned char* cube_valid) {
    const GridBuild b{&g, pts, d_n, cap_n, cube_of, cube_valid};
    grid_build_multi(C, &b, 1);
}

// ------------------------------------------------------------------------------------------
// Batched builds: up to GRID_MULTI_MAX grids in the same 6 launches (blockIdx.y = grid). The bbox is reset by the
// scatter of the previous build (and once at allocation), so no init launch is needed.
struct GridJob {
    GridDesc* desc; int* cell_count; int* cell_start; int* blk; float4* spts; int* sidx; int* pcell;
    const float4* pts; const int* d_n; const int* cube_of; const unsigned char* cube_valid;
    float min_cell; int nlayers; int w_index; int flat; int max_cells;
};
struct GridJobs { GridJob j[GRID_MULTI_MAX]; };

__global__ void k_gm_bbox(GridJobs J) {
    const GridJob& g = J.j[blockIdx.y];
    __shared__ unsigned sh[6];
    __shared__ int shc;
    if (threadIdx.x < 6) sh[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    if (threadIdx.x == 0) shc = 0;
    __syncthreads();
    const int n = *g.d_n;
    unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    int cnt = 0;
    for (int i = blockIdx.x * GB + threadIdx.x; i < n; i += gridDim.x * GB) {
        if (!grid_include(i, g.cube_of, g.cube_valid)) continue;
        float4 p = g.pts[i];
        unsigned v[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
        for (int a = 0; a < 3; a++) { mn[a] = min(mn[a], v[a]); mx[a] = max(mx[a], v[a]); }
        cnt++;
    }
    for (int a = 0; a < 3; a++) {
        unsigned long long lo = wave_min_u64(mn[a]), hi = wave_max_u64(mx[a]);
        if (lane_id() == 0) { atomicMin(&sh[a], (unsigned)lo); atomicMax(&sh[3 + a], (unsigned)hi); }
    }
    cnt = wave_sum_i(cnt);
    if (lane_id() == 0 && cnt) atomicAdd(&shc, cnt);
    __syncthreads();
    // one global atomic per block and counter (same-address atomics serialise)
    if (threadIdx.x < 3) { atomicMin(&g.desc->bb[threadIdx.x], sh[threadIdx.x]); atomicMax(&g.desc->bb[3 + threadIdx.x], sh[3 + threadIdx.x]); }
    if (threadIdx.x == 3 && shc) atomicAdd(&g.desc->n_acc, shc);
}
__global__ void k_gm_count(GridJobs J) {
    const GridJob& g = J.j[blockIdx.y];
    __shared__ GridDesc gd;
    if (threadIdx.x == 0) {
        unsigned bb[6];
        for (int a = 0; a < 6; a++) bb[a] = g.desc->bb[a];
        grid_params(bb, g.min_cell, g.nlayers, g.flat, g.max_cells, &gd);
        if (blockIdx.x == 0) {
            GridDesc* d = g.desc;
            d->ox = gd.ox; d->oy = gd.oy; d->oz = gd.oz; d->cell = gd.cell; d->inv_cell = gd.inv_cell;
            d->dx = gd.dx; d->dy = gd.dy; d->dz = gd.dz; d->ncells = gd.ncells; d->nlayers = gd.nlayers;
        }
    }
    __syncthreads();
    const int n = *g.d_n;
    // whole waves iterate together (the run aggregation below needs every lane in the ballot)
    for (int i0 = blockIdx.x * GB + (threadIdx.x & ~(WAVE - 1)); i0 < n; i0 += gridDim.x * GB) {
        const int i = i0 + lane_id();
        int c = -1;
        if (i < n && grid_include(i, g.cube_of, g.cube_valid)) {
            const float4 p = g.pts[i];
            const int cx = min(max(cell_coord(p.x, gd.ox, gd.inv_cell), 0), gd.dx - 1);
            const int cy = min(max(cell_coord(p.y, gd.oy, gd.inv_cell), 0), gd.dy - 1);
            const int cz = min(max(cell_coord(p.z, gd.oz, gd.inv_cell), 0), gd.dz - 1);
            const int layer = gd.nlayers > 1 ? min(max((int)p.w, 0), gd.nlayers - 1) : 0;
            c = ((layer * gd.dz + cz) * gd.dy + cy) * gd.dx + cx;
        }
        if (i < n) g.pcell[i] = c;
        int len, h;
        cell_runs(c, &len, &h);
        if (c >= 0 && h == lane_id()) atomicAdd(&g.cell_count[c], len);
    }
}
__global__ void __launch_bounds__(SCAN_T) k_gm_scan1(GridJobs J) {
    const GridJob& g = J.j[blockIdx.y];
    if (blockIdx.x * SCAN_CHUNK >= g.desc->ncells) return;
    k_grid_scan1_body(g.cell_count, g.desc->ncells, g.blk);
}
__global__ void __launch_bounds__(SCAN_T) k_gm_scan3(GridJobs J) {
    const GridJob& g = J.j[blockIdx.y];
    if (blockIdx.x * SCAN_CHUNK >= g.desc->ncells) return;
    k_grid_scan3_body(g.cell_count, g.desc->ncells, g.blk, g.cell_start);
}
__global__ void k_gm_scatter(GridJobs J) {
    const GridJob& g = J.j[blockIdx.y];
    const int n = *g.d_n;
    for (int i0 = blockIdx.x * GB + (threadIdx.x & ~(WAVE - 1)); i0 < n; i0 += gridDim.x * GB) {
        const int i = i0 + lane_id();
        const int c = i < n ? g.pcell[i] : -1;
        int len, h;
        cell_runs(c, &len, &h);
        // the run head claims len slots at the top of the cell's remaining range; members take theirs
        int left = 0;
        if (c >= 0 && h == lane_id()) left = atomicSub(&g.cell_count[c], len);
        left = __shfl(left, h, WAVE) - (lane_id() - h);
        if (c < 0) continue;
        const int pos = g.cell_start[c] + left - 1;
        if (left <= 0 || pos >= g.cell_start[c + 1]) continue;     // defensive: never write outside the cell
        const float4 p = g.pts[i];
        g.spts[pos] = g.w_index ? make_float4(p.x, p.y, p.z, __int_as_float(i)) : p;
        g.sidx[pos] = i;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {            // publish n, re-arm bbox/counter for the next build
        GridDesc* d = g.desc;
        d->n = d->n_acc;
        d->n_acc = 0;
        for (int a = 0; a < 3; a++) { d->bb[a] = 0xffffffffu; d->bb[3 + a] = 0u; }
    }
}

static void grid_build_radix(Ctx& C, const GridBuild* b, int nj);
constexpr int GR_MIN = 1 << 18;   // large-map grids from this many points take the radix build
void grid_build_multi(Ctx& C, const GridBuild* b, int nj) {
    if (nj <= 0) return;
    if (nj > GRID_MULTI_MAX) throw ApiError{ALOAM_E_ARG, "grid_build_multi: too many grids"};
    {
        // large-map search grids (aloam_knn_build, aloam_s2m_set_map) of >= GR_MIN points: radix build
        // (ALOAM_GRID_RADIX=0, read per build: the atomic counting sort below for them too)
        const char* re = getenv("ALOAM_GRID_RADIX");
        bool big = !(re && atoi(re) == 0);
        for (int k = 0; k < nj; k++) big = big && b[k].g->max_cells == GRID_MAX_CELLS_BIG && b[k].cap_n >= GR_MIN;
        if (big) { grid_build_radix(C, b, nj); return; }
    }
    hipStream_t st = C.stream;
    GridJobs J{};
    int cap = 1, maxc = 0;
    for (int k = 0; k < nj; k++) {
        const Grid& g = *b[k].g;
        J.j[k] = GridJob{g.desc, g.cell_count, g.cell_start, g.blk, g.pts, g.idx, g.pcell,
                         b[k].pts, b[k].d_n, b[k].cube_of, b[k].cube_valid, g.min_cell, g.nlayers, g.w_index ? 1 : 0,
                         g.flat ? 1 : 0, g.max_cells};
        cap = std::max(cap, b[k].cap_n);
        maxc = std::max(maxc, g.max_cells);
    }
    const int nb = std::max(1, std::min(1024, (cap + GB - 1) / GB));
    const int nsb = maxc / SCAN_CHUNK;
    k_gm_bbox<<<dim3(nb, nj), GB, 0, st>>>(J);
    k_gm_count<<<dim3(nb, nj), GB, 0, st>>>(J);
    k_gm_scan1<<<dim3(nsb, nj), SCAN_T, 0, st>>>(J);
    k_gm_scan3<<<dim3(nsb, nj), SCAN_T, 0, st>>>(J);
    k_gm_scatter<<<dim3(nb, nj), GB, 0, st>>>(J);
    HIPCHK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// Large grids (>= GR_MIN points: the map index of aloam_knn_build and aloam_s2m_set_map). The counting sort
// above pays two scattered global atomics per point (count, then claim a slot), which on the 2.1M-point C4
// map cost ~280 of the ~340 us build (k_gm_count + k_gm_scatter, profiles/r05_c4_kernel_stats.csv). Here the
// (cell, index) pairs are radix-sorted instead (k_gm_bbox as above counts the included points): 9-bit digits, least significant first, one pass per digit
// the cell ids need (<= 3 below 2^26 cells); per pass a digit histogram of each 4096-point tile, an
// exclusive scan of the (digit, tile) counts, and a stable scatter in which each wave ranks its 64 keys of
// a chunk by 9 ballots (peers with the same digit) and advances its own per-digit run in LDS. No per-point
// global atomic; inside a cell the points end in original index order, so the built grid is deterministic.
// Then the sorted copy (gather) and the cell starts straight from the sorted keys (k_gr_starts: no per-cell
// counts, no scan). Excluded points (cube gating) take key ncells and sort past the last cell.
constexpr int GR_T = 256, GR_PER = 16, GR_TILE = GR_T * GR_PER, GR_BITS = 9, GR_NB = 1 << GR_BITS;
constexpr int GS_T = 256, GS_PER = 8, GS_CH = GS_T * GS_PER;         // k_gr_starts: cells per chunk
constexpr int GS_BLOCKS = 1024;                                       // k_gr_starts workgroups per grid (chunks grid-strided)
constexpr int GS_NCH = GRID_MAX_CELLS_BIG / GS_CH + 2;                // chunks of the largest grid (+ the end cell)
constexpr int GR_WAVES = GR_T / WAVE, GR_WCH = GR_TILE / GR_WAVES / WAVE;   // chunks of 64 per wave and tile
static_assert(GR_NB == 2 * GR_T, "k_gr_scatter: two digits per thread in the tile prefix");
struct GrJob {
    GridDesc* desc; int* cell_count; int* cell_start; int* blk; float4* spts; int* sidx;
    const float4* pts; const int* d_n; const int* cube_of; const unsigned char* cube_valid;
    float min_cell; int nlayers; int w_index; int flat; int max_cells;
    unsigned* k0; unsigned* k1; int* v0; int* v1; int* H; int* Ho; int* Hblk; unsigned* bbp;
    int* cf;          // first run head per chunk of GS_CH cells (INT_MAX: none), for k_gr_starts
};
struct GrJobs { GrJob j[GRID_MULTI_MAX]; };
__device__ __forceinline__ int gr_tiles(int n) { return (n + GR_TILE - 1) / GR_TILE; }

// the lanes of a wave holding the same 9-bit digit (peers), by 9 ballots; invalid lanes are in no set
__device__ __forceinline__ unsigned long long gr_peers(int d, bool valid) {
    unsigned long long m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < GR_BITS; b++) {
        const bool bit = (d >> b) & 1;
        const unsigned long long bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}
// one LDS atomic per distinct digit of the wave (a tile's keys crowd into few digits in the high passes)
__device__ __forceinline__ void gr_count(int* hist, int d, bool valid, bool plain = false) {
    if (plain) {                                   // A/B: one LDS atomic per key
        if (valid) atomicAdd(&hist[d], 1);
        return;
    }
    const unsigned long long m = gr_peers(d, valid);
    if (valid && __popcll(m & lanemask_lt64()) == 0) atomicAdd(&hist[d], __popcll(m));
}

// bbox: per-tile partials (16 points per thread, loads batched); k_gr_keys reduces them
__global__ void __launch_bounds__(GR_T) k_gr_bbox(GrJobs J) {
    const GrJob& g = J.j[blockIdx.y];
    __shared__ unsigned sh[7];
    if (threadIdx.x < 7) sh[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    const int n = *g.d_n;
    unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    int cnt = 0;
    const int i0 = blockIdx.x * GR_TILE + threadIdx.x;
#pragma unroll
    for (int h = 0; h < GR_PER; h += 8) {
        float4 p[8];
        bool in[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = i0 + (h + u) * GR_T;
            in[u] = i < n && grid_include(i, g.cube_of, g.cube_valid);
            p[u] = g.pts[in[u] ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (!in[u]) continue;
            const unsigned v[3] = {f2ord(p[u].x), f2ord(p[u].y), f2ord(p[u].z)};
#pragma unroll
            for (int a = 0; a < 3; a++) { mn[a] = min(mn[a], v[a]); mx[a] = max(mx[a], v[a]); }
            cnt++;
        }
    }
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const unsigned long long lo = wave_min_u64(mn[a]), hi = wave_max_u64(mx[a]);
        if (lane_id() == 0) { atomicMin(&sh[a], (unsigned)lo); atomicMax(&sh[3 + a], (unsigned)hi); }
    }
    cnt = wave_sum_i(cnt);
    if (lane_id() == 0 && cnt) atomicAdd(&sh[6], (unsigned)cnt);
    __syncthreads();
    if (threadIdx.x < 7) g.bbp[blockIdx.x * 8 + threadIdx.x] = sh[threadIdx.x];
}
// every block: the bbox from all tiles' partials (the same order, the same result), the grid parameters
// (block 0 publishes them, the included count and the digit passes); then the cell keys in index order
// and the first digit's histogram per tile
__global__ void __launch_bounds__(GR_T) k_gr_keys(GrJobs J) {
    const GrJob& g = J.j[blockIdx.y];
    __shared__ int hist[GR_NB];
    __shared__ unsigned sh[7];
    __shared__ GridDesc gds;
    if (threadIdx.x < 7) sh[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    for (int i = threadIdx.x; i < GR_NB; i += GR_T) hist[i] = 0;
    __syncthreads();
    {
        unsigned r[7] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0, 0, 0, 0};
        for (int t = threadIdx.x; t < (int)gridDim.x; t += GR_T) {
#pragma unroll
            for (int a = 0; a < 3; a++) { r[a] = min(r[a], g.bbp[t * 8 + a]); r[3 + a] = max(r[3 + a], g.bbp[t * 8 + 3 + a]); }
            r[6] += g.bbp[t * 8 + 6];
        }
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const unsigned long long lo = wave_min_u64(r[a]), hi = wave_max_u64(r[3 + a]);
            if (lane_id() == 0) { atomicMin(&sh[a], (unsigned)lo); atomicMax(&sh[3 + a], (unsigned)hi); }
        }
        const int c = wave_sum_i((int)r[6]);
        if (lane_id() == 0 && c) atomicAdd(&sh[6], (unsigned)c);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned bb[6];
        for (int a = 0; a < 6; a++) bb[a] = sh[a];
        GridDesc gd;
        grid_params(bb, g.min_cell, g.nlayers, g.flat, g.max_cells, &gd);
        const int bits = 32 - __clz((unsigned)gd.ncells);          // keys 0 .. ncells (ncells = excluded)
        gd.npass = max(1, (bits + GR_BITS - 1) / GR_BITS);
        gds = gd;
        if (blockIdx.x == 0) {
            GridDesc* d = g.desc;
            for (int a = 0; a < 6; a++) d->bb[a] = bb[a];
            d->ox = gd.ox; d->oy = gd.oy; d->oz = gd.oz; d->cell = gd.cell; d->inv_cell = gd.inv_cell;
            d->dx = gd.dx; d->dy = gd.dy; d->dz = gd.dz; d->ncells = gd.ncells; d->nlayers = gd.nlayers;
            d->npass = gd.npass;
            d->n_acc = (int)sh[6];
        }
    }
    __syncthreads();
    const GridDesc gd = gds;
    for (int i = blockIdx.x * GR_T + threadIdx.x; i < GS_NCH; i += gridDim.x * GR_T) g.cf[i] = INT_MAX;   // k_gr_finish fills
    const int n = *g.d_n, nt = gr_tiles(n);
    if ((int)blockIdx.x >= nt) return;
    const int i0 = blockIdx.x * GR_TILE + threadIdx.x;
#pragma unroll
    for (int h = 0; h < GR_PER; h += 8) {
        float4 p[8];
        bool in[8], ok[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = i0 + (h + u) * GR_T;
            ok[u] = i < n;
            in[u] = ok[u] && grid_include(i, g.cube_of, g.cube_valid);
            p[u] = g.pts[in[u] ? i : 0];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = i0 + (h + u) * GR_T;
            unsigned key = (unsigned)gd.ncells;                   // excluded: past the last cell
            if (in[u]) {
                const int cx = min(max(cell_coord(p[u].x, gd.ox, gd.inv_cell), 0), gd.dx - 1);
                const int cy = min(max(cell_coord(p[u].y, gd.oy, gd.inv_cell), 0), gd.dy - 1);
                const int cz = min(max(cell_coord(p[u].z, gd.oz, gd.inv_cell), 0), gd.dz - 1);
                const int layer = gd.nlayers > 1 ? min(max((int)p[u].w, 0), gd.nlayers - 1) : 0;
                key = (unsigned)(((layer * gd.dz + cz) * gd.dy + cy) * gd.dx + cx);
            }
            if (ok[u]) { g.k0[i] = key; g.v0[i] = i; }
            gr_count(hist, (int)(key & (GR_NB - 1)), ok[u]);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < GR_NB; d += GR_T) g.H[d * nt + blockIdx.x] = hist[d];
}
// digit histogram of pass `pass` (data in k[pass & 1]), 16 keys per thread loaded at once
__global__ void __launch_bounds__(GR_T) k_gr_hist(GrJobs J, int pass, int plain) {
    const GrJob& g = J.j[blockIdx.y];
    if (pass >= g.desc->npass) return;
    __shared__ int hist[GR_NB];
    const int n = *g.d_n, nt = gr_tiles(n);
    if ((int)blockIdx.x >= nt) return;
    for (int i = threadIdx.x; i < GR_NB; i += GR_T) hist[i] = 0;
    __syncthreads();
    const unsigned* sk = (pass & 1) ? g.k1 : g.k0;
    const int sh = pass * GR_BITS;
    unsigned kk[GR_PER];
#pragma unroll
    for (int k = 0; k < GR_PER; k++) {
        const int i = blockIdx.x * GR_TILE + k * GR_T + threadIdx.x;
        kk[k] = i < n ? sk[i] : 0xffffffffu;
    }
#pragma unroll
    for (int k = 0; k < GR_PER; k++)
        gr_count(hist, (int)((kk[k] >> sh) & (GR_NB - 1)), blockIdx.x * GR_TILE + k * GR_T + (int)threadIdx.x < n, plain & (1 << pass));
    __syncthreads();
    for (int d = threadIdx.x; d < GR_NB; d += GR_T) g.H[d * nt + blockIdx.x] = hist[d];
}
// exclusive scan of the (digit, tile) counts, digit-major: H -> Ho
__global__ void __launch_bounds__(SCAN_T) k_gr_hscan1(GrJobs J, int pass) {
    const GrJob& g = J.j[blockIdx.y];
    if (pass >= g.desc->npass) return;
    const int nc = GR_NB * gr_tiles(*g.d_n);
    if ((int)blockIdx.x * SCAN_CHUNK >= nc) return;
    k_grid_scan1_body(g.H, nc, g.Hblk);
}
__global__ void __launch_bounds__(SCAN_T) k_gr_hscan3(GrJobs J, int pass) {
    const GrJob& g = J.j[blockIdx.y];
    if (pass >= g.desc->npass) return;
    const int nc = GR_NB * gr_tiles(*g.d_n);
    if ((int)blockIdx.x * SCAN_CHUNK >= nc) return;
    k_grid_scan3_body(g.H, nc, g.Hblk, g.Ho);
}
// stable scatter of pass `pass`: k[pass & 1] -> k[(pass + 1) & 1]. Wave w of a tile owns its elements
// [w * 1024, (w + 1) * 1024) (16 per lane, loaded at once) and its own per-digit run (started at the tile's
// digit prefix plus the earlier waves' counts), so positions follow element order within every digit. The
// tile is first laid out by digit in LDS, then written out by consecutive threads: each digit's stretch of
// the tile is one contiguous run of the output (coalesced stores).
__global__ void __launch_bounds__(GR_T) k_gr_scatter(GrJobs J, int pass) {
    const GrJob& g = J.j[blockIdx.y];
    if (pass >= g.desc->npass) return;
    __shared__ int run[GR_WAVES][GR_NB];
    __shared__ int lpre[GR_NB], gofs[GR_NB];
    __shared__ unsigned stk[GR_TILE];
    __shared__ int stv[GR_TILE];
    const int n = *g.d_n, nt = gr_tiles(n);
    if ((int)blockIdx.x >= nt) return;
    const unsigned* sk = (pass & 1) ? g.k1 : g.k0;
    const int* sv = (pass & 1) ? g.v1 : g.v0;
    unsigned* dk = (pass & 1) ? g.k0 : g.k1;
    int* dv = (pass & 1) ? g.v0 : g.v1;
    const int sh = pass * GR_BITS;
    const int w = threadIdx.x / WAVE, lane = lane_id();
    for (int i = threadIdx.x; i < GR_WAVES * GR_NB; i += GR_T) (&run[0][0])[i] = 0;
    const int e0 = blockIdx.x * GR_TILE + w * (GR_TILE / GR_WAVES) + lane;
    unsigned kk[GR_WCH];
    int vv[GR_WCH];
#pragma unroll
    for (int j = 0; j < GR_WCH; j++) {
        const int e = e0 + j * WAVE;
        kk[j] = e < n ? sk[e] : 0u;
        vv[j] = e < n ? sv[e] : 0;
    }
    __syncthreads();
    unsigned long long pm[GR_WCH];
    const unsigned long long lt = lanemask_lt64();
#pragma unroll
    for (int j = 0; j < GR_WCH; j++) {
        const bool valid = e0 + j * WAVE < n;
        const int d = (int)((kk[j] >> sh) & (GR_NB - 1));
        pm[j] = gr_peers(d, valid);
        if (valid && __popcll(pm[j] & lt) == 0) atomicAdd(&run[w][d], __popcll(pm[j]));
    }
    __syncthreads();
    // tile-local digit prefix (LDS layout) and the digit's global offset for this tile
    {
        int tc[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int d = threadIdx.x * 2 + q;
            int c = 0;
#pragma unroll
            for (int ww = 0; ww < GR_WAVES; ww++) c += run[ww][d];
            tc[q] = c;
        }
        int tot;
        const int ex = block_exscan<GR_T>(tc[0] + tc[1], &tot);
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int d = threadIdx.x * 2 + q;
            int r = ex + (q ? tc[0] : 0);
            lpre[d] = r;
            gofs[d] = g.Ho[d * nt + blockIdx.x];
#pragma unroll
            for (int ww = 0; ww < GR_WAVES; ww++) { const int c = run[ww][d]; run[ww][d] = r; r += c; }
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < GR_WCH; j++) {
        const bool valid = e0 + j * WAVE < n;
        const int d = (int)((kk[j] >> sh) & (GR_NB - 1));
        const int rank = __popcll(pm[j] & lt);
        const int base = run[w][d];
        // every lane has read its digit's run before the leader (rank 0) advances it: one wave, LDS in order
        if (valid && rank == 0) run[w][d] = base + __popcll(pm[j]);
        if (valid) { stk[base + rank] = kk[j]; stv[base + rank] = vv[j]; }
    }
    __syncthreads();
    const int cnt = min(GR_TILE, n - (int)blockIdx.x * GR_TILE);
#pragma unroll 4
    for (int t = threadIdx.x; t < cnt; t += GR_T) {
        const unsigned key = stk[t];
        const int d = (int)((key >> sh) & (GR_NB - 1));
        const int pos = gofs[d] + (t - lpre[d]);
        dk[pos] = key;
        dv[pos] = stv[t];
    }
}
// the sorted copy (and the included count published for the searches)
__global__ void __launch_bounds__(GR_T) k_gr_finish(GrJobs J) {
    const GrJob& g = J.j[blockIdx.y];
    GridDesc* d = g.desc;
    const int npass = d->npass, ninc = d->n_acc;
    const unsigned* sk = (npass & 1) ? g.k1 : g.k0;
    const int* sv = (npass & 1) ? g.v1 : g.v0;
    if (blockIdx.x == 0 && threadIdx.x == 0) d->n = ninc;      // published for the searches and the clear
    const int p0 = blockIdx.x * GR_TILE + threadIdx.x;
#pragma unroll
    for (int h = 0; h < GR_PER; h += 8) {
        int val[8];
        unsigned key[8], prv[8];
        float4 pt[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int p = p0 + (h + u) * GR_T;
            const bool ok = p < ninc;
            val[u] = ok ? sv[p] : 0;
            key[u] = ok ? sk[p] : 0u;
            prv[u] = ok && p > 0 ? sk[p - 1] : 0xffffffffu;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) pt[u] = g.pts[val[u]];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int p = p0 + (h + u) * GR_T;
            if (p >= ninc) continue;
            g.spts[p] = g.w_index ? make_float4(pt[u].x, pt[u].y, pt[u].z, __int_as_float(val[u])) : pt[u];
            g.sidx[p] = val[u];
            // a run head: its cell's start + 1 (0: empty, the counts are zero between builds); the first run
            // head of a chunk of cells (its key's chunk differs from the previous key's) also into cf
            if (prv[u] != key[u]) g.cell_count[key[u]] = p + 1;
            if (prv[u] == 0xffffffffu || (int)(key[u] / GS_CH) != (int)(prv[u] / GS_CH)) g.cf[key[u] / GS_CH] = p;
        }
    }
}
// The cell starts from the run heads, with no scan over the dense cell array: cell_start[c] =
// lower_bound(keys, c) for c in [0, ncells] (excluded points carry key ncells, so cell_start[ncells] = the
// included count). k_gr_finish (position-parallel) writes every run head's start + 1 into its cell's count
// slot (zero between builds) and each chunk's first head into cf; k_gr_cfscan turns cf into every chunk's
// lower_bound (a suffix minimum); k_gr_starts fills the chunks: a chunk without points is one constant
// (nothing read), the others read their head slots (clearing them) and take a suffix minimum (an empty cell
// starts where the next occupied one does, the chunk's last ones at the next chunk's lower_bound). The
// dense array is read only where points are, not scanned twice and cleared as in the counting build.
// every chunk's lower_bound: the first recorded head at or after it (ninc if none), by a suffix minimum of
// the chunk heads in place (one workgroup; <= GS_NCH chunks, GS_NCH / GS_T + 1 per thread)
constexpr int GS_CPT = GS_NCH / 1024 + 1;
__global__ void __launch_bounds__(1024) k_gr_cfscan(GrJobs J) {
    const GrJob& g = J.j[blockIdx.y];
    __shared__ int wmin[1024 / WAVE];
    const int nch = g.desc->ncells / GS_CH + 2, ninc = g.desc->n;   // chunk nch - 1: past the end (ninc)
    const int t = threadIdx.x, lane = lane_id(), w = t / WAVE;
    const int cpt = (nch + 1023) / 1024;                  // this grid's chunks per thread (<= GS_CPT)
    int v[GS_CPT];
    int bm = INT_MAX;
#pragma unroll
    for (int i = 0; i < GS_CPT; i++) {
        const int jj = t * cpt + i;
        v[i] = i >= cpt ? INT_MAX : jj < nch - 1 ? g.cf[jj] : (jj == nch - 1 ? ninc : INT_MAX);
        bm = min(bm, v[i]);
    }
    int x = bm;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
        const int y = __shfl_down(x, off);
        if (lane + off < WAVE) x = min(x, y);
    }
    int after = __shfl_down(x, 1);
    if (lane == WAVE - 1) after = INT_MAX;
    if (lane == 0) wmin[w] = x;
    __syncthreads();
    int run = after;
    for (int ww = w + 1; ww < 1024 / WAVE; ww++) run = min(run, wmin[ww]);
#pragma unroll
    for (int i = GS_CPT - 1; i >= 0; i--) {
        run = min(run, v[i]);
        const int jj = t * cpt + i;
        if (i < cpt && jj < nch) g.cf[jj] = run;
    }
}
__global__ void __launch_bounds__(GS_T) k_gr_starts(GrJobs J) {
    const GrJob& g = J.j[blockIdx.y];
    GridDesc* d = g.desc;
    __shared__ int wmin[GS_T / WAVE];
    const int nc = d->ncells;
    const int nch = nc / GS_CH + 1;                       // chunks of cells 0 .. nc
    const int t = threadIdx.x, lane = lane_id(), w = t / WAVE;
    for (int j = blockIdx.x; j < nch; j += gridDim.x) {
        const int c0 = j * GS_CH, c1 = min(c0 + GS_CH, nc + 1);
        const int p0 = g.cf[j], p1 = g.cf[j + 1];         // lower_bound(c0), lower_bound(c0 + GS_CH) (k_gr_cfscan)
        const int cb = c0 + t * GS_PER;
        const bool whole = cb + GS_PER <= c1;
        int v[GS_PER];
        if (p0 == p1) {                                   // no point in the chunk: every cell starts at p0
#pragma unroll
            for (int i = 0; i < GS_PER; i++) v[i] = p0;
        } else {                                          // the heads' starts + 1 (k_gr_finish), read and cleared
            if (whole) {
                int4* q = (int4*)(g.cell_count + cb);
#pragma unroll
                for (int k = 0; k < GS_PER / 4; k++) {
                    const int4 a = q[k];
                    v[4 * k] = a.x; v[4 * k + 1] = a.y; v[4 * k + 2] = a.z; v[4 * k + 3] = a.w;
                    q[k] = make_int4(0, 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int i = 0; i < GS_PER; i++) {
                    v[i] = cb + i < c1 ? g.cell_count[cb + i] : 0;
                    if (cb + i < c1) g.cell_count[cb + i] = 0;
                }
            }
            int bm = INT_MAX;
#pragma unroll
            for (int i = 0; i < GS_PER; i++) { v[i] = v[i] ? v[i] - 1 : INT_MAX; bm = min(bm, v[i]); }
            // min over the threads after t (in the wave, then the later waves), then p1
            int x = bm;
#pragma unroll
            for (int off = 1; off < WAVE; off <<= 1) {
                const int y = __shfl_down(x, off);
                if (lane + off < WAVE) x = min(x, y);
            }
            int after = __shfl_down(x, 1);
            if (lane == WAVE - 1) after = INT_MAX;
            if (lane == 0) wmin[w] = x;
            __syncthreads();
            int carry = p1;
            for (int ww = w + 1; ww < GS_T / WAVE; ww++) carry = min(carry, wmin[ww]);
            int run = min(carry, after);
#pragma unroll
            for (int i = GS_PER - 1; i >= 0; i--) { run = min(run, v[i]); v[i] = run; }
            __syncthreads();                              // wmin is reused by the next chunk
        }
        if (whole) {
            int4* q = (int4*)(g.cell_start + cb);
#pragma unroll
            for (int k = 0; k < GS_PER / 4; k++) q[k] = make_int4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        } else {
#pragma unroll
            for (int i = 0; i < GS_PER; i++) if (cb + i < c1) g.cell_start[cb + i] = v[i];
        }
    }
    if (blockIdx.x == 0 && t == 0) {                      // bbox re-armed for the counting build, count cleared
        d->n_acc = 0;
        for (int a = 0; a < 3; a++) { d->bb[a] = 0xffffffffu; d->bb[3 + a] = 0u; }
    }
}

static void grid_build_radix(Ctx& C, const GridBuild* b, int nj) {
    hipStream_t st = C.stream;
    GrJobs J{};
    int cap = 1, maxc = 0;
    for (int k = 0; k < nj; k++) {
        Grid& g = *b[k].g;
        const int need = std::max(std::max(b[k].cap_n, g.cap), 1);
        if (g.rcap < need) {
            for (void* p : {(void*)g.rk[0], (void*)g.rk[1], (void*)g.rv[0], (void*)g.rv[1], (void*)g.rH, (void*)g.rHo, (void*)g.rblk,
                            (void*)g.rbb, (void*)g.rcf})
                if (p) dfree(C, p);
            const int tcap = (need + GR_TILE - 1) / GR_TILE;
            g.rk[0] = (unsigned*)dalloc(C, sizeof(unsigned) * need);
            g.rk[1] = (unsigned*)dalloc(C, sizeof(unsigned) * need);
            g.rv[0] = (int*)dalloc(C, sizeof(int) * need);
            g.rv[1] = (int*)dalloc(C, sizeof(int) * need);
            g.rH = (int*)dalloc(C, sizeof(int) * ((size_t)GR_NB * tcap + 1));
            g.rHo = (int*)dalloc(C, sizeof(int) * ((size_t)GR_NB * tcap + 1));   // + the scan's total
            g.rblk = (int*)dalloc(C, sizeof(int) * SCAN_T * SCAN_CPT);
            g.rbb = (unsigned*)dalloc(C, sizeof(unsigned) * 8 * (size_t)tcap);
            g.rcf = (int*)dalloc(C, sizeof(int) * GS_NCH);
            g.rcap = need;
        }
        J.j[k] = GrJob{g.desc, g.cell_count, g.cell_start, g.blk, g.pts, g.idx, b[k].pts, b[k].d_n, b[k].cube_of, b[k].cube_valid,
                       g.min_cell, g.nlayers, g.w_index ? 1 : 0, g.flat ? 1 : 0, g.max_cells,
                       g.rk[0], g.rk[1], g.rv[0], g.rv[1], g.rH, g.rHo, g.rblk, g.rbb, g.rcf};
        cap = std::max(cap, b[k].cap_n);
        maxc = std::max(maxc, g.max_cells);
    }
    // every job's grid is sized by the largest cap (tiles beyond a job's live count exit; the bbox ticket
    // counts all launched tiles of a job)
    const int tiles = (cap + GR_TILE - 1) / GR_TILE;
    for (int k = 0; k < nj; k++)
        if ((tiles + 0) > (b[k].g->rcap + GR_TILE - 1) / GR_TILE) throw ApiError{ALOAM_E_ARG, "grid_build_radix: tile scratch"};
    const int nsbH = (GR_NB * tiles + SCAN_CHUNK - 1) / SCAN_CHUNK;
    // knob (read per build): bit p = pass p's histogram with one LDS atomic per key instead of the
    // ballot-aggregated counts (k_gr_hist, passes 1 and 2). Default 2: pass 1 plain (its digits are spread:
    // 20 -> 16 us), pass 2 aggregated (its high digits crowd a tile; plain measured the same),
    // micro/gr_hist_ab.sh
    const char* pe = getenv("ALOAM_GR_PLAIN");
    const int gr_plain = pe ? atoi(pe) : 2;
    k_gr_bbox<<<dim3(tiles, nj), GR_T, 0, st>>>(J);
    k_gr_keys<<<dim3(tiles, nj), GR_T, 0, st>>>(J);
    for (int pass = 0; pass < 3; pass++) {
        if (pass > 0) k_gr_hist<<<dim3(tiles, nj), GR_T, 0, st>>>(J, pass, gr_plain);
        k_gr_hscan1<<<dim3(nsbH, nj), SCAN_T, 0, st>>>(J, pass);
        k_gr_hscan3<<<dim3(nsbH, nj), SCAN_T, 0, st>>>(J, pass);
        k_gr_scatter<<<dim3(tiles, nj), GR_T, 0, st>>>(J, pass);
    }
    k_gr_finish<<<dim3(tiles, nj), GR_T, 0, st>>>(J);
    k_gr_cfscan<<<dim3(1, nj), 1024, 0, st>>>(J);
    k_gr_starts<<<dim3(GS_BLOCKS, nj), GS_T, 0, st>>>(J);
    HIPCHK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// aloam_knn(): exact radius k-NN (k <= 8) over a grid whose cells are >= the radius (27 cells).
__global__ void k_knn(const GridDesc* __restrict__ gdp, const int* __restrict__ start, const float4* __restrict__ spts,
                      const int* __restrict__ sidx, const float4* __restrict__ q, int nq, int k, float r2, int* idx, float* d2) {
    __shared__ RowSet<9> rows9[256 / WAVE];
    const int wq = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (wq >= nq) return;
    const GridDesc gd = *gdp;
    int pos[8], oi[8];
    float od[8];
    const float4 qq = q[wq];
    const int f = wave_knn_rows<8, 9>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, start, spts, sidx,
                                       qq.x, qq.y, qq.z, r2, 1, pos, od, oi, nullptr, rows9[threadIdx.x / WAVE]);
    if (lane_id() == 0)
        for (int j = 0; j < k; j++) {
            idx[wq * k + j] = j < f ? oi[j] : -1;
            d2[wq * k + j] = j < f ? od[j] : INFINITY;
        }
}

// Large searches (aloam_knn_device, C4): a GS-lane group per query (group_knn27 in
// aloam_device.hpp) over the radius-edge grid; candidates counted per wave when profiling.
template <int K, int GS, bool CNT>
__global__ void __launch_bounds__(256) k_knn_group(const GridDesc* __restrict__ gdp, const int* __restrict__ start,
                                                   const float4* __restrict__ spts, const int* __restrict__ sidx,
                                                   const float4* __restrict__ q, int nq, int k, float r2, int* __restrict__ idx,
                                                   float* __restrict__ d2, unsigned long long* cand) {
    __shared__ int tabs[256 / GS][20];
    // natural order (measured: an XCD-contiguous remap of the ring-ordered queries was 20% slower —
    // all XCDs sweeping the same neighbourhood share it through the MALL)
    const int qi = (blockIdx.x * blockDim.x + threadIdx.x) / GS;
    const bool live = qi < nq;
    if (!__ballot(live)) return;
    const GridDesc gd = *gdp;
    const float4 qq = q[live ? qi : 0];
    int pos[K], oi[K], nc = 0;
    float od[K];
    const int f = group_knn27<K, GS, true>(gd.ox, gd.oy, gd.oz, gd.inv_cell, gd.dx, gd.dy, gd.dz, start, spts, sidx,
                                           qq.x, qq.y, qq.z, r2, live, pos, od, oi, &nc, tabs[threadIdx.x / GS], gd.n);
    const int gl = lane_id() & (GS - 1);
    if (live) {
#pragma unroll
        for (int j = 0; j < K; j++)
            if (j < k && j % GS == gl) {
                idx[(size_t)qi * k + j] = j < f ? oi[j] : -1;
                d2[(size_t)qi * k + j] = j < f ? od[j] : INFINITY;
            }
    }
    if (CNT) {
        const int t = wave_sum_i(live && gl == 0 ? nc : 0);
        if (lane_id() == 0 && t) { atomicAdd(&cand[0], (unsigned long long)t); atomicAdd(&cand[1], (unsigned long long)t); }
    }
}

// Points of the 3x3x3 cell block around q (the 9 row ranges' lengths; nothing streamed): C27(q) of the
// roofline's algorithmic bytes when the search itself does not visit that block.
__device__ __forceinline__ int block27_total(const GridDesc& gd, const int* __restrict__ start, float qx, float qy, float qz) {
    const int cx = (int)floorf((qx - gd.ox) * gd.inv_cell), cy = (int)floorf((qy - gd.oy) * gd.inv_cell),
              cz = (int)floorf((qz - gd.oz) * gd.inv_cell);
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, gd.dx - 1);
    int t = 0;
#pragma unroll
    for (int r = 0; r < 9; r++) {
        const int y = cy + (r % 3) - 1, z = cz + (r / 3) - 1;
        const bool ok = x0 <= x1 && y >= 0 && y < gd.dy && z >= 0 && z < gd.dz;
        const int c = (z * gd.dy + y) * gd.dx;
        t += load_or(start, c + x1 + 1, ok, 0) - load_or(start, c + x0, ok, 0);
    }
    return t;
}

// Two-phase exact radius k-NN (aloam_knn_device's default). Phase 1: the 3x3x3 block of a fine grid
// (cell f < r). The block holds every point within f of q (q lies inside its centre cell), so when the
// k-th neighbour found there is closer than 0.99 f, no point outside the block can precede it — the
// result is the exact radius-r k-NN in the same (d2, index) order, ties included. Phase 2 (only groups
// phase 1 did not settle): the radius-edge grid's 27-cell block, which holds the whole r-ball. On a
// dense map (C4: the 5 neighbours within ~0.15 m, ~1000 points in the coarse block) phase 1 streams
// ~10x fewer candidates. cand (profiling): [0] += C27(q) of the coarse block (SURVEY §8(d)'s
// algorithmic count), [1] += candidates actually streamed by both phases.
template <int K, int GS, bool CNT, int U = 4, bool WP2 = true, int XP = 0>
__global__ void __launch_bounds__(256) k_knn_2phase(const GridDesc* __restrict__ fgd, const int* __restrict__ fstart,
                                                    const float4* __restrict__ fpts, const GridDesc* __restrict__ cgd,
                                                    const int* __restrict__ cstart, const float4* __restrict__ cpts,
                                                    const float4* __restrict__ q, int nq, int k, float r2, int* __restrict__ idx,
                                                    float* __restrict__ d2, unsigned long long* cand, int exp) {
    __shared__ int tabs[256 / GS][20];
    const int qi = (blockIdx.x * blockDim.x + threadIdx.x) / GS;
    const bool live = qi < nq;
    if (!__ballot(live)) return;
    const float4 qq = q[live ? qi : 0];
    int pos[K], oi[K], nf = 0, nc = 0;
    float od[K];
    const GridDesc gf = *fgd;
    int f = group_knn27<K, GS, true, U, false, XP>(gf.ox, gf.oy, gf.oz, gf.inv_cell, gf.dx, gf.dy, gf.dz, fstart, fpts, nullptr,
                                                qq.x, qq.y, qq.z, r2, live, pos, od, oi, &nf, tabs[threadIdx.x / GS], gf.n);
    float dk = INFINITY;
#pragma unroll
    for (int j = 0; j < K; j++) if (j == k - 1) dk = od[j];
    const float lim = 0.99f * gf.cell;
    const bool need = live && !(f >= k && dk < lim * lim) && !(exp & 1) && (XP & 6) == 0;
    const GridDesc gc = *cgd;
    const int gl = lane_id() & (GS - 1);
    if constexpr (WP2) {
        // Phase 2 by the whole wave, one unsettled query at a time: the coarse block holds ~10x the fine
        // block's points, so with GS lanes per query a single unsettled query kept its wave ~10x longer than
        // the settled ones; with 64 lanes its block streams in about as many load rounds as phase 1. The
        // phase-1 k-th distance (when k were found) bounds phase 2's (its candidates are a superset), so
        // candidates beyond it skip the insertion.
        unsigned long long todo = __ballot(need && gl == 0);
        int* wtab = tabs[(threadIdx.x & ~(WAVE - 1)) / GS];
        while (todo) {
            const int l = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            const float x = readlane_f(qq.x, l), y = readlane_f(qq.y, l), z = readlane_f(qq.z, l);
            const float pr = f >= k ? dk : INFINITY;
            const float prl = readlane_f(pr, l);
            int p2[K], i2[K], n2 = 0;
            float e2[K];
            const int f2 = group_knn27<K, WAVE, true, U>(gc.ox, gc.oy, gc.oz, gc.inv_cell, gc.dx, gc.dy, gc.dz, cstart, cpts,
                                                         nullptr, x, y, z, r2, true, p2, e2, i2, &n2, wtab, gc.n,
                                                         KnnCollect{0.f, nullptr, nullptr, 0}, nullptr, prl);
            if ((lane_id() & ~(GS - 1)) == (l & ~(GS - 1))) {
#pragma unroll
                for (int j = 0; j < K; j++) { od[j] = e2[j]; oi[j] = i2[j]; }
                f = f2;
                nc = n2;
            }
        }
    } else if (__any(need)) {                  // wave-uniform: every lane takes part in the group search
        int p2[K], i2[K];
        float e2[K];
        const int f2 = group_knn27<K, GS, true, U>(gc.ox, gc.oy, gc.oz, gc.inv_cell, gc.dx, gc.dy, gc.dz, cstart, cpts, nullptr,
                                                   qq.x, qq.y, qq.z, r2, need, p2, e2, i2, &nc, tabs[threadIdx.x / GS], gc.n);
        if (need) {
#pragma unroll
            for (int j = 0; j < K; j++) { od[j] = e2[j]; oi[j] = i2[j]; }
            f = f2;
        }
    }
    if (live) {
#pragma unroll
        for (int j = 0; j < K; j++)
            if (j < k && j % GS == gl) {
                idx[(size_t)qi * k + j] = j < f ? oi[j] : -1;
                d2[(size_t)qi * k + j] = j < f ? od[j] : INFINITY;
            }
    }
    if (CNT) {
        const int c27 = live && gl == 0 ? (need ? nc : block27_total(gc, cstart, qq.x, qq.y, qq.z)) : 0;
        const int a = wave_sum_i(c27), s = wave_sum_i(live && gl == 0 ? nf + (need ? nc : 0) : 0);
        if (lane_id() == 0) {
            if (a) atomicAdd(&cand[0], (unsigned long long)a);
            if (s) atomicAdd(&cand[1], (unsigned long long)s);
        }
    }
}

// k_knn_2phase on 64-bit keys (group_knn27_keys): the same two phases, settle test and results; the
// candidate loop has no data-dependent branches (register row bounds, branch-free top-K insertion), and
// phase 2 starts from the phase-1 K-th key as its bound. Default since round 6 (ALOAM_KNN_KEYS=0: the
// round-5 kernel).
template <int K, int GS, bool CNT, int U, bool PK = true>
__global__ void __launch_bounds__(256) k_knn_keys(const GridDesc* __restrict__ fgd, const int* __restrict__ fstart,
                                                  const float4* __restrict__ fpts, const GridDesc* __restrict__ cgd,
                                                  const int* __restrict__ cstart, const float4* __restrict__ cpts,
                                                  const float4* __restrict__ q, int nq, int k, float r2, int* __restrict__ idx,
                                                  float* __restrict__ d2, unsigned long long* cand) {
    const int qi = (blockIdx.x * blockDim.x + threadIdx.x) / GS;
    const bool live = qi < nq;
    if (!__ballot(live)) return;
    const float4 qq = q[live ? qi : 0];
    unsigned long long key[K];
    int nf = 0, nc = 0;
    const GridDesc gf = *fgd;
    int f = group_knn27_keys<K, GS, U, PK>(gf.ox, gf.oy, gf.oz, gf.inv_cell, gf.dx, gf.dy, gf.dz, fstart, fpts, qq.x, qq.y, qq.z,
                                       r2, live, key, &nf, gf.n);
    unsigned long long kk = ~0ull;
#pragma unroll
    for (int j = 0; j < K; j++) if (j == k - 1) kk = key[j];
    const float dk = kk == ~0ull ? INFINITY : __uint_as_float((unsigned)(kk >> 32));
    const float lim = 0.99f * gf.cell;
    const bool need = live && !(f >= k && dk < lim * lim);
    const GridDesc gc = *cgd;
    if (__any(need)) {                         // wave-uniform: every lane takes part in the group search
        unsigned long long k2[K];
        const int f2 = group_knn27_keys<K, GS, U, PK>(gc.ox, gc.oy, gc.oz, gc.inv_cell, gc.dx, gc.dy, gc.dz, cstart, cpts, qq.x, qq.y,
                                                  qq.z, r2, need, k2, &nc, gc.n, kk);
        if (need) {
#pragma unroll
            for (int j = 0; j < K; j++) key[j] = k2[j];
            f = f2;
        }
    }
    const int gl = lane_id() & (GS - 1);
    if (live) {
#pragma unroll
        for (int j = 0; j < K; j++)
            if (j < k && j % GS == gl) {
                idx[(size_t)qi * k + j] = j < f ? (int)(unsigned)key[j] : -1;
                d2[(size_t)qi * k + j] = j < f ? __uint_as_float((unsigned)(key[j] >> 32)) : INFINITY;
            }
    }
    if (CNT) {
        const int c27 = live && gl == 0 ? (need ? nc : block27_total(gc, cstart, qq.x, qq.y, qq.z)) : 0;
        const int a = wave_sum_i(c27), s = wave_sum_i(live && gl == 0 ? nf + (need ? nc : 0) : 0);
        if (lane_id() == 0) {
            if (a) atomicAdd(&cand[0], (unsigned long long)a);
            if (s) atomicAdd(&cand[1], (unsigned long long)s);
        }
    }
}

// Phase 1 shared by the queries of a wave (the default since round 6). A wave holds 8 consecutive queries
// (8 lanes each); in ring order most of them lie in the same fine cell (C4: 2.8 distinct cells per wave, 8.5
// queries per occupied cell), so their 3x3x3 blocks are the same few blocks. The wave finds its distinct
// cells (ballot loop over the group leaders), loads the 9 row bounds of every distinct block in one
// instruction per 64 values, lays the blocks' rows out as one flattened list (row table in LDS: cumulative
// ends + position bases), and streams the list once, 64 consecutive candidates per load instruction, into
// a per-wave LDS buffer; each query's 8 lanes then scan exactly its own block's stretch of the list from
// LDS. Same candidates per query, same (d2, index) order and settle test as k_knn_2phase, so the result
// is identical; a block's points cross L1 once per wave instead of once per query.
template <int K, bool CNT, int U>
__global__ void __launch_bounds__(256) k_knn_shared(const GridDesc* __restrict__ fgd, const int* __restrict__ fstart,
                                                    const float4* __restrict__ fpts, const GridDesc* __restrict__ cgd,
                                                    const int* __restrict__ cstart, const float4* __restrict__ cpts,
                                                    const float4* __restrict__ q, int nq, int k, float r2, int* __restrict__ idx,
                                                    float* __restrict__ d2, unsigned long long* cand) {
    constexpr int GS = 8, NW = 256 / WAVE, CH = WAVE * U, MAXC = WAVE / GS, MAXR = 9 * MAXC;
    __shared__ float4 cbuf[NW][CH];
    __shared__ int rE[NW][MAXR], rB[NW][MAXR], rtmp[NW][18 * MAXC];
    __shared__ int4 slotc[NW][MAXC];
    __shared__ int tabs[256 / GS][20];
    const int w = threadIdx.x / WAVE, lane = lane_id(), gl = lane & (GS - 1);
    const int qi = (blockIdx.x * blockDim.x + threadIdx.x) / GS;
    const bool live = qi < nq;
    if (!__ballot(live)) return;
    const float4 qq = q[live ? qi : 0];
    const GridDesc gf = *fgd;
    const int cx = (int)floorf((qq.x - gf.ox) * gf.inv_cell), cy = (int)floorf((qq.y - gf.oy) * gf.inv_cell),
              cz = (int)floorf((qq.z - gf.oz) * gf.inv_cell);
    // the block [c-1, c+1]^3 meets the grid (its other rows / cells are clipped below, as in group_knn27)
    const bool blk = live && cx >= -1 && cx <= gf.dx && cy >= -1 && cy <= gf.dy && cz >= -1 && cz <= gf.dz;
    const int key = blk ? ((cz + 1) * (gf.dy + 2) + (cy + 1)) * (gf.dx + 2) + (cx + 1) : -1;
    // distinct cells of the wave, in leader order
    unsigned long long rem = __ballot(gl == 0 && key >= 0);
    int myslot = -1, ncell = 0;
    while (rem) {
        const int l = __ffsll((long long)rem) - 1;
        const int kk = readlane_i(key, l);
        rem &= ~__ballot(gl == 0 && key == kk);
        if (key == kk) myslot = ncell;
        if (lane == l) slotc[w][ncell] = make_int4(cx, cy, cz, 0);
        ncell++;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // row bounds of every distinct block: value i = (cell i / 18, row (i % 18) % 9, end if (i % 18) >= 9)
    for (int b0 = 0; b0 < 18 * ncell; b0 += WAVE) {
        const int i = b0 + lane;
        int v = 0;
        if (i < 18 * ncell) {
            const int4 c = slotc[w][i / 18];
            const int rr = i % 18, r = rr % 9;
            const int x0 = max(c.x - 1, 0), x1 = min(c.x + 1, gf.dx - 1);
            const int y = c.y + (r % 3) - 1, z = c.z + (r / 3) - 1;
            const bool ok = x0 <= x1 && y >= 0 && y < gf.dy && z >= 0 && z < gf.dz;
            v = load_or(fstart, (z * gf.dy + y) * gf.dx + (rr >= 9 ? x1 + 1 : x0), ok, 0);
            rtmp[w][i] = v;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // flattened row table: row R = 9 j + r, E[R] = cumulative end, B[R] = position of flattened item 0 of its run
    const int nr = 9 * ncell;
    int T;
    {
        int rb0 = 0, len0 = 0, rb1 = 0, len1 = 0;
        if (lane < nr) { const int j = lane / 9, r = lane % 9; rb0 = rtmp[w][18 * j + r]; len0 = rtmp[w][18 * j + 9 + r] - rb0; }
        if (WAVE + lane < nr) {
            const int R = WAVE + lane, j = R / 9, r = R % 9;
            rb1 = rtmp[w][18 * j + r];
            len1 = rtmp[w][18 * j + 9 + r] - rb1;
        }
        const int e0 = wave_incl_scan(len0);
        const int t0 = readlane_i(e0, WAVE - 1);
        const int e1 = wave_incl_scan(len1) + t0;
        if (lane < nr) { rE[w][lane] = e0; rB[w][lane] = rb0 - (e0 - len0); }
        if (WAVE + lane < nr) { rE[w][WAVE + lane] = e1; rB[w][WAVE + lane] = rb1 - (e1 - len1); }
        T = nr <= WAVE ? readlane_i(e0, nr > 0 ? nr - 1 : 0) : readlane_i(e1, nr - WAVE - 1);
        if (nr == 0) T = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int off = myslot > 0 ? rE[w][9 * myslot - 1] : 0, end = myslot >= 0 ? rE[w][9 * myslot + 8] : 0;
    float bd[K];
    int bi[K], bp[K];
#pragma unroll
    for (int j = 0; j < K; j++) { bd[j] = INFINITY; bi[j] = 0x7fffffff; bp[j] = -1; }
    for (int c0 = 0; c0 < T; c0 += CH) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int t = c0 + u * WAVE + lane;
            // row of item t: the number of rows whose cumulative end is <= t (branch-free search, 7 steps)
            int R = 0;
#pragma unroll
            for (int st = 64; st >= 1; st >>= 1)
                if (R + st <= nr && rE[w][R + st - 1] <= t) R += st;
            const int p = t < T && R < nr ? rB[w][R] + t : -1;
            v[u] = load_or(fpts, p, p >= 0 && p < gf.n, make_float4(INFINITY, INFINITY, INFINITY, 0.f));
        }
#pragma unroll
        for (int u = 0; u < U; u++) cbuf[w][u * WAVE + lane] = v[u];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int lo = max(off, c0), hi = min(end, c0 + CH);
        for (int tb = lo + gl; tb < hi; tb += 4 * GS) {
            float4 cv[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {              // 4 LDS reads in flight, then the 4 candidates
                const int t = tb + u * GS;
                cv[u] = cbuf[w][min(t, hi - 1) - c0];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int t = tb + u * GS;
                const float4 c = cv[u];
                const float dd = sqdist(c.x, c.y, c.z, qq.x, qq.y, qq.z);
                if (t >= hi || !(dd < r2) || dd > bd[K - 1]) continue;
                const int iu = __float_as_int(c.w);
                if (dd < bd[K - 1] || iu < bi[K - 1]) {
                    float nd = dd; int ni = iu, np = t;
#pragma unroll
                    for (int j = 0; j < K; j++) {
                        const bool lt = nd < bd[j] || (nd == bd[j] && ni < bi[j]);
                        if (lt) { float td = bd[j]; int ti = bi[j], tp = bp[j]; bd[j] = nd; bi[j] = ni; bp[j] = np; nd = td; ni = ti; np = tp; }
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    int pos[K], oi[K];
    float od[K];
    int f = group_merge_topk<K, GS>(bd, bi, bp, pos, od, oi);
    const int nf = end - off;
    float dk = INFINITY;
#pragma unroll
    for (int j = 0; j < K; j++) if (j == k - 1) dk = od[j];
    const float lim = 0.99f * gf.cell;
    const bool need = live && !(f >= k && dk < lim * lim);
    const GridDesc gc = *cgd;
    int nc = 0;
    if (__any(need)) {                         // phase 2 by each unsettled query's own group, bounded by phase 1
        int p2[K], i2[K];
        float e2[K];
        const float pr = f >= k ? dk : INFINITY;
        const int f2 = group_knn27<K, GS, true, 4>(gc.ox, gc.oy, gc.oz, gc.inv_cell, gc.dx, gc.dy, gc.dz, cstart, cpts, nullptr,
                                                   qq.x, qq.y, qq.z, r2, need, p2, e2, i2, &nc, tabs[threadIdx.x / GS], gc.n,
                                                   KnnCollect{0.f, nullptr, nullptr, 0}, nullptr, pr);
        if (need) {
#pragma unroll
            for (int j = 0; j < K; j++) { od[j] = e2[j]; oi[j] = i2[j]; }
            f = f2;
        }
    }
    if (live) {
#pragma unroll
        for (int j = 0; j < K; j++)
            if (j < k && j % GS == gl) {
                idx[(size_t)qi * k + j] = j < f ? oi[j] : -1;
                d2[(size_t)qi * k + j] = j < f ? od[j] : INFINITY;
            }
    }
    if (CNT) {
        const int c27 = live && gl == 0 ? (need ? nc : block27_total(gc, cstart, qq.x, qq.y, qq.z)) : 0;
        const int a = wave_sum_i(c27), s = wave_sum_i(live && gl == 0 ? nf + (need ? nc : 0) : 0);
        if (lane_id() == 0) {
            if (a) atomicAdd(&cand[0], (unsigned long long)a);
            if (s) atomicAdd(&cand[1], (unsigned long long)s);
        }
    }
}

// The same two-phase search with phase 1 read from LDS: a workgroup takes a tile of 256 / GS consecutive
// queries (ring order: neighbours along a scan line, a metre or two of arc), loads the fine-grid cells of
// the union of their 3x3x3 blocks into LDS once — row by row, each (y, z) row of the box one contiguous
// run of the sorted points — and every group searches its block there (the same candidates in the same
// cells, so the same (d2, index) result as from global memory). Neighbouring queries share most of their
// blocks, so the tile reads each cell once instead of once per query, in one burst of coalesced loads
// instead of one dependent gather per query. A tile whose box exceeds the LDS budget searches phase 1 in
// global memory as k_knn_2phase does. Phase 2 (the queries phase 1 leaves unsettled) stays global.
constexpr int KT_MAXC = 768;     // fine cells per tile box
constexpr int KT_MAXP = 2048;    // points per tile (32 KB)
constexpr int KT_MAXR = 64;      // (y, z) rows per tile box (one wave scans their lengths)
struct TileBox { int x0, y0, z0, nx, ny, nz; };
template <int K, int GS>
__device__ __forceinline__ int group_knn27_lds(int cx, int cy, int cz, const GridDesc& gd, const TileBox& b, const int* lstart,
                                               const float4* lpts, float qx, float qy, float qz, float r2, bool active, int* out_pos,
                                               float* out_d2, int* out_idx, int* ncand, int* tab) {
    const int gl = lane_id() & (GS - 1);
    int total;
    {
        const int x0 = max(cx - 1, 0), x1 = min(cx + 1, gd.dx - 1);
        int rb[9], pre[10];
        pre[0] = 0;
#pragma unroll
        for (int r = 0; r < 9; r++) {
            const int y = cy + (r % 3) - 1, z = cz + (r / 3) - 1;
            const bool ok = active && x0 <= x1 && y >= 0 && y < gd.dy && z >= 0 && z < gd.dz;
            const int lc = ok ? ((z - b.z0) * b.ny + (y - b.y0)) * b.nx + (x0 - b.x0) : 0;
            rb[r] = ok ? lstart[lc] : 0;
            pre[r + 1] = pre[r] + (ok ? lstart[lc + (x1 - x0) + 1] - rb[r] : 0);
        }
        total = pre[9];
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
    for (int t = gl; t < total; t += GS) {
        while (t >= nxt && row < 8) { row++; base = tab[row]; nxt = tab[10 + row]; }
        const int p = base + t;
        const float4 v = lpts[p];
        const float d2 = sqdist(v.x, v.y, v.z, qx, qy, qz);
        if (!(d2 < r2) || d2 > bd[K - 1]) continue;
        const int iu = __float_as_int(v.w);
        if (d2 < bd[K - 1] || iu < bi[K - 1]) {
            float nd = d2; int ni = iu, np = p;
#pragma unroll
            for (int k = 0; k < K; k++) {
                const bool lt = nd < bd[k] || (nd == bd[k] && ni < bi[k]);
                if (lt) { float td = bd[k]; int ti = bi[k], tp = bp[k]; bd[k] = nd; bi[k] = ni; bp[k] = np; nd = td; ni = ti; np = tp; }
            }
        }
    }
    return group_merge_topk<K, GS>(bd, bi, bp, out_pos, out_d2, out_idx);
}

template <int K, int GS, bool CNT>
__global__ void __launch_bounds__(256) k_knn_tile(const GridDesc* __restrict__ fgd, const int* __restrict__ fstart,
                                                  const float4* __restrict__ fpts, const GridDesc* __restrict__ cgd,
                                                  const int* __restrict__ cstart, const float4* __restrict__ cpts,
                                                  const float4* __restrict__ q, int nq, int k, float r2, int* __restrict__ idx,
                                                  float* __restrict__ d2, unsigned long long* cand, int max_pts) {
    constexpr int T = 256 / GS;
    __shared__ int tabs[T][20];
    __shared__ int lstart[KT_MAXC + 1];
    __shared__ int rowg[KT_MAXR], rows0[KT_MAXR], rowoff[KT_MAXR + 1];
    __shared__ float4 lpts[KT_MAXP];
    __shared__ int bb[6];
    __shared__ int tile_ok;
    const int tid = threadIdx.x;
    const int qi = blockIdx.x * T + tid / GS;
    const bool live = qi < nq;
    const float4 qq = q[live ? qi : 0];
    const GridDesc gf = *fgd;
    const int cx = (int)floorf((qq.x - gf.ox) * gf.inv_cell), cy = (int)floorf((qq.y - gf.oy) * gf.inv_cell),
              cz = (int)floorf((qq.z - gf.oz) * gf.inv_cell);
    // the tile box: union of the live queries' blocks, clipped to the grid
    if (tid < 6) bb[tid] = (tid & 1) ? -1 : 0x7fffffff;
    __syncthreads();
    {
        const int x0 = max(cx - 1, 0), x1 = min(cx + 1, gf.dx - 1), y0 = max(cy - 1, 0), y1 = min(cy + 1, gf.dy - 1),
                  z0 = max(cz - 1, 0), z1 = min(cz + 1, gf.dz - 1);
        if (live && (tid & (GS - 1)) == 0 && x0 <= x1 && y0 <= y1 && z0 <= z1) {
            atomicMin(&bb[0], x0); atomicMax(&bb[1], x1);
            atomicMin(&bb[2], y0); atomicMax(&bb[3], y1);
            atomicMin(&bb[4], z0); atomicMax(&bb[5], z1);
        }
    }
    __syncthreads();
    TileBox b{bb[0], bb[2], bb[4], bb[1] - bb[0] + 1, bb[3] - bb[2] + 1, bb[5] - bb[4] + 1};
    const bool any = bb[1] >= 0;
    const int nrow = any ? b.ny * b.nz : 0, ncell = nrow * (any ? b.nx : 0);
    bool ok = any && ncell <= KT_MAXC && nrow <= KT_MAXR;
    if (ok) {
        // per-cell global starts (lstart, rebased below) and each row's global start
        for (int j = tid; j < ncell; j += 256) {
            const int x = j % b.nx, r = j / b.nx, y = b.y0 + r % b.ny, z = b.z0 + r / b.ny;
            lstart[j] = fstart[(z * gf.dy + y) * gf.dx + b.x0 + x];
        }
        if (tid < nrow) {
            const int y = b.y0 + tid % b.ny, z = b.z0 + tid / b.ny, c = (z * gf.dy + y) * gf.dx + b.x0;
            rows0[tid] = fstart[c];                     // the row's first point
            rowg[tid] = fstart[c + b.nx];               // its end (start of the cell after the row)
        }
        __syncthreads();
        if (tid < WAVE) {                               // row lengths -> LDS offsets (one wave, nrow <= 64)
            const int len = tid < nrow ? rowg[tid] - rows0[tid] : 0;
            const int inc = wave_incl_scan(len);
            if (tid < nrow) rowoff[tid + 1] = inc;
            if (tid == 0) { rowoff[0] = 0; tile_ok = readlane_i(inc, WAVE - 1) <= max_pts; }
        }
        __syncthreads();
        ok = tile_ok != 0;
        if (ok) {
            const int P = rowoff[nrow];
            for (int p = tid; p < P; p += 256) {        // the box's points, row after row
                int lo = 0, hi = nrow - 1;
                while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (rowoff[mid] <= p) lo = mid; else hi = mid - 1; }
                lpts[p] = fpts[rows0[lo] + (p - rowoff[lo])];
            }
            for (int j = tid; j <= ncell; j += 256) {   // cell starts -> LDS positions (lstart[ncell] = P)
                const int r = j / b.nx;
                lstart[j] = j == ncell ? P : rowoff[r] + (lstart[j] - rows0[r]);
            }
        }
    }
    __syncthreads();
    int pos[K], oi[K], nf = 0, nc = 0;
    float od[K];
    int f;
    if (ok) f = group_knn27_lds<K, GS>(cx, cy, cz, gf, b, lstart, lpts, qq.x, qq.y, qq.z, r2, live, pos, od, oi, &nf, tabs[tid / GS]);
    else f = group_knn27<K, GS, true>(gf.ox, gf.oy, gf.oz, gf.inv_cell, gf.dx, gf.dy, gf.dz, fstart, fpts, nullptr, qq.x, qq.y, qq.z,
                                      r2, live, pos, od, oi, &nf, tabs[tid / GS], gf.n);
    float dk = INFINITY;
#pragma unroll
    for (int j = 0; j < K; j++) if (j == k - 1) dk = od[j];
    const float lim = 0.99f * gf.cell;
    const bool need = live && !(f >= k && dk < lim * lim);
    const GridDesc gc = *cgd;
    if (__any(need)) {
        int p2[K], i2[K];
        float e2[K];
        const int f2 = group_knn27<K, GS, true>(gc.ox, gc.oy, gc.oz, gc.inv_cell, gc.dx, gc.dy, gc.dz, cstart, cpts, nullptr,
                                                qq.x, qq.y, qq.z, r2, need, p2, e2, i2, &nc, tabs[tid / GS], gc.n);
        if (need) {
#pragma unroll
            for (int j = 0; j < K; j++) { od[j] = e2[j]; oi[j] = i2[j]; }
            f = f2;
        }
    }
    const int gl = lane_id() & (GS - 1);
    if (live) {
#pragma unroll
        for (int j = 0; j < K; j++)
            if (j < k && j % GS == gl) {
                idx[(size_t)qi * k + j] = j < f ? oi[j] : -1;
                d2[(size_t)qi * k + j] = j < f ? od[j] : INFINITY;
            }
    }
    if (CNT) {
        const int c27 = live && gl == 0 ? (need ? nc : block27_total(gc, cstart, qq.x, qq.y, qq.z)) : 0;
        const int a = wave_sum_i(c27), s = wave_sum_i(live && gl == 0 ? nf + (need ? nc : 0) : 0);
        if (lane_id() == 0) {
            if (a) atomicAdd(&cand[0], (unsigned long long)a);
            if (s) atomicAdd(&cand[1], (unsigned long long)s);
        }
    }
}

template <int GS>
static void knn_2phase_launch(Ctx& C, Grid& gf, Grid& gc, const float4* q, int nq, int k, float r2, int* idx, float* d2,
                              unsigned long long* cand) {
    const int blocks = (int)(((long long)nq * GS + 255) / 256);
    // A/B knob, read per call (tests run both kernels in one process). Default: phase 1 from global memory —
    // measured on one MI355X (C4, 50 launches): k_knn_2phase 91.5 us vs k_knn_tile 134.1 us per launch
    // (profiles/r05_ab.txt): the tile's serial bbox -> row scan -> copy chain before any distance costs more
    // than the L2 gathers it replaces.
    const char* te = getenv("ALOAM_KNN_TILE");
    const int tmode = te ? atoi(te) : 0;
    const bool tile = tmode != 0;
    // ALOAM_KNN_TILE=2 (tests): every tile takes the over-budget path (phase 1 from global memory in k_knn_tile)
    const int max_pts = tmode == 2 ? -1 : KT_MAXP;
    std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), "%s<%d,%d>", tile ? "k_knn_tile" : "k_knn_2phase", k <= 5 ? 5 : 8, GS);
    if (tile) {
#define KNNT(KK, CN) k_knn_tile<KK, GS, CN><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, max_pts)
        if (k <= 5) { if (cand) KNNT(5, true); else KNNT(5, false); }
        else { if (cand) KNNT(8, true); else KNNT(8, false); }
#undef KNNT
        return;
    }
    // CNT: the candidate-counting instance (profiling), a separate symbol so kernel traces tell it apart.
    // ALOAM_KNN_U (tuning knob, read per call): candidate loads in flight per lane, 4 (default) or 8.
    // ALOAM_KNN_SHARED (read per call): default 1 = k_knn_shared (phase 1 shared by the wave's queries), 0 = the
    // per-query k_knn_2phase; ALOAM_KNN_SU: its loads per lane per staging round (4, or 2).
    // ALOAM_KNN_P2 (A/B knob, read per call, k_knn_2phase): 1 = phase 2 by the whole wave, one unsettled query at a
    // time (measured slower); default = by each query's own group. ALOAM_KNN_EXP (profiling experiments only,
    // results invalid): 1 = no phase 2, 2 / 4 = no phase-1 candidate loop / merge.
    const char* ue = getenv("ALOAM_KNN_U");
    const bool u8 = ue && atoi(ue) == 8;
    const char* pe = getenv("ALOAM_KNN_P2");
    const bool wp2 = pe && atoi(pe) == 1;     // measured slower (114 vs 95 us, r6 c4_exp): opt-in
    const char* xe = getenv("ALOAM_KNN_EXP");
    const int exp = xe ? atoi(xe) : 0;
    std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), "k_knn_2phase<%d,%d%s%s>", k <= 5 ? 5 : 8, GS, u8 ? ",U8" : "",
                  wp2 ? ",P2W" : "");
#define KNN2(KK, CN, UU, WP) k_knn_2phase<KK, GS, CN, UU, WP><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp)
#define KNN2W(KK, CN, UU) do { if (wp2) KNN2(KK, CN, UU, true); else KNN2(KK, CN, UU, false); } while (0)
    const char* ke = getenv("ALOAM_KNN_KEYS");
    const bool keys = GS >= 8 && !(ke && atoi(ke) == 0) && !(exp & 6);
    if constexpr (GS >= 8) if (keys) {
        const int uk = u8 ? 8 : 4;
        // A/B knob: ALOAM_KNN_PK=1 = distances in packed fp32 (measured 59.0 vs 57.0 us: the pair packing moves
        // cost more than the packed ops save), default scalar
        const char* pke = getenv("ALOAM_KNN_PK");
        if (!(pke && atoi(pke) == 1) && !u8) {
            // ALOAM_KNN_U=2 / 3 (tuning knob): candidate slots per lane and batch (default 4)
            const int us = ue ? atoi(ue) : 4;
            std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), us == 2 || us == 3 ? "k_knn_keys<%d,%d,U%d>" : "k_knn_keys<%d,%d>",
                          k <= 5 ? 5 : 8, GS, us);
#define KNNKS(KK, UU) do { if (cand) k_knn_keys<KK, GS, true, UU, false><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand); \
                           else k_knn_keys<KK, GS, false, UU, false><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand); } while (0)
            if (us == 2) { if (k <= 5) KNNKS(5, 2); else KNNKS(8, 2); }
            else if (us == 3) { if (k <= 5) KNNKS(5, 3); else KNNKS(8, 3); }
            else { if (k <= 5) KNNKS(5, 4); else KNNKS(8, 4); }
#undef KNNKS
            return;
        }
        std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), "k_knn_keys<%d,%d,%s>", k <= 5 ? 5 : 8, GS, u8 ? "U8" : "PK");
#define KNNK(KK, CN, UU) k_knn_keys<KK, GS, CN, UU><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand)
        if (uk == 8) {
            if (k <= 5) { if (cand) KNNK(5, true, 8); else KNNK(5, false, 8); }
            else { if (cand) KNNK(8, true, 8); else KNNK(8, false, 8); }
        } else {
            if (k <= 5) { if (cand) KNNK(5, true, 4); else KNNK(5, false, 4); }
            else { if (cand) KNNK(8, true, 4); else KNNK(8, false, 4); }
        }
#undef KNNK
        return;
    }
    const char* she = getenv("ALOAM_KNN_SHARED");
    const bool shared = GS == 8 && she && atoi(she) == 1 && !u8 && !(exp & 6);
    if (shared) {
        const char* sue = getenv("ALOAM_KNN_SU");
        const int su = sue ? atoi(sue) : 4;
        std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), "k_knn_shared<%d,%d>", k <= 5 ? 5 : 8, su == 2 ? 2 : 4);
#define KNNS(KK, CN, UU) k_knn_shared<KK, CN, UU><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand)
        if (su == 2) {
            if (k <= 5) { if (cand) KNNS(5, true, 2); else KNNS(5, false, 2); }
            else { if (cand) KNNS(8, true, 2); else KNNS(8, false, 2); }
        } else {
            if (k <= 5) { if (cand) KNNS(5, true, 4); else KNNS(5, false, 4); }
            else { if (cand) KNNS(8, true, 4); else KNNS(8, false, 4); }
        }
#undef KNNS
        return;
    }
    const char* rre = getenv("ALOAM_KNN_RR");
    const bool rr = rre && atoi(rre) == 1;
    if (rr && !u8 && !(exp & 6)) {
        // row bounds in registers (no LDS row table in the candidate loop)
        std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), "k_knn_2phase<%d,%d,RR>", k <= 5 ? 5 : 8, GS);
        if (k <= 5) { if (cand) k_knn_2phase<5, GS, true, 4, false, 8><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp);
                      else k_knn_2phase<5, GS, false, 4, false, 8><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp); }
        else { if (cand) k_knn_2phase<8, GS, true, 4, false, 8><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp);
               else k_knn_2phase<8, GS, false, 4, false, 8><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp); }
        return;
    }
    const int xp = exp & 6;
    if (xp && k <= 5 && !cand && !u8) {          // (profiling experiments: parts of phase 1 left out)
        std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), "k_knn_2phase<5,%d,XP%d>", GS, xp);
        if (xp == 2) k_knn_2phase<5, GS, false, 4, false, 2><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp);
        else if (xp == 4) k_knn_2phase<5, GS, false, 4, false, 4><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp);
        else k_knn_2phase<5, GS, false, 4, false, 6><<<blocks, 256, 0, C.stream>>>(gf.desc, gf.cell_start, gf.pts, gc.desc, gc.cell_start, gc.pts, q, nq, k, r2, idx, d2, cand, exp);
    } else if (u8) {
        if (k <= 5) { if (cand) KNN2W(5, true, 8); else KNN2W(5, false, 8); }
        else { if (cand) KNN2W(8, true, 8); else KNN2W(8, false, 8); }
    } else {
        if (k <= 5) { if (cand) KNN2W(5, true, 4); else KNN2W(5, false, 4); }
        else { if (cand) KNN2W(8, true, 4); else KNN2W(8, false, 4); }
    }
#undef KNN2W
#undef KNN2
}

void knn_device_2phase_launch(Ctx& C, Grid& gf, Grid& gc, const float4* q, int nq, int k, float radius, int* idx, float* d2,
                              unsigned long long* cand) {
    if (nq <= 0) return;
    const float r2 = radius * radius;
    const int gs = getenv("ALOAM_KNN_GS2") ? atoi(getenv("ALOAM_KNN_GS2")) : 8;   // tuning knob (read per call)
    if (gs == 16) knn_2phase_launch<16>(C, gf, gc, q, nq, k, r2, idx, d2, cand);
    else if (gs == 2) knn_2phase_launch<2>(C, gf, gc, q, nq, k, r2, idx, d2, cand);
    else if (gs == 4) knn_2phase_launch<4>(C, gf, gc, q, nq, k, r2, idx, d2, cand);
    else knn_2phase_launch<8>(C, gf, gc, q, nq, k, r2, idx, d2, cand);
    HIPCHK(hipGetLastError());
}

template <int GS>
static void knn_group_launch(Ctx& C, Grid& g, const float4* q, int nq, int k, float r2, int* idx, float* d2,
                             unsigned long long* cand) {
    const int blocks = (int)(((long long)nq * GS + 255) / 256);
#define KNNG(KK, CN) k_knn_group<KK, GS, CN><<<blocks, 256, 0, C.stream>>>(g.desc, g.cell_start, g.pts, g.idx, q, nq, k, r2, idx, d2, cand)
    if (k <= 5) { if (cand) KNNG(5, true); else KNNG(5, false); }
    else { if (cand) KNNG(8, true); else KNNG(8, false); }
#undef KNNG
}

void knn_device_launch(Ctx& C, Grid& g, const float4* q, int nq, int k, float radius, int* idx, float* d2,
                       unsigned long long* cand) {
    if (nq <= 0) return;
    const float r2 = radius * radius;
    static const int gs = getenv("ALOAM_KNN_GS") ? atoi(getenv("ALOAM_KNN_GS")) : 8;   // tuning knob
    std::snprintf(C.knn_kernel, sizeof(C.knn_kernel), "k_knn_group<%d,%d>", k <= 5 ? 5 : 8, gs);
    if (gs == 64) knn_group_launch<64>(C, g, q, nq, k, r2, idx, d2, cand);
    else if (gs == 32) knn_group_launch<32>(C, g, q, nq, k, r2, idx, d2, cand);
    else if (gs == 16) knn_group_launch<16>(C, g, q, nq, k, r2, idx, d2, cand);
    else if (gs == 4) knn_group_launch<4>(C, g, q, nq, k, r2, idx, d2, cand);
    else if (gs == 2) knn_group_launch<2>(C, g, q, nq, k, r2, idx, d2, cand);
    else if (gs == 1) knn_group_launch<1>(C, g, q, nq, k, r2, idx, d2, cand);
    else knn_group_launch<8>(C, g, q, nq, k, r2, idx, d2, cand);
    HIPCHK(hipGetLastError());
}

void knn_launch(Ctx& C, Grid& g, const float4* q, int nq, int k, float radius, int* idx, float* d2) {
    const int threads = 256, per_block = threads / WAVE;
    const int nbk = (nq + per_block - 1) / per_block;
    const float r2 = radius * radius;
    if (nbk > 0) k_knn<<<nbk, threads, 0, C.stream>>>(g.desc, g.cell_start, g.pts, g.idx, q, nq, k, r2, idx, d2);
    HIPCHK(hipGetLastError());
}

}  // namespace aloam
