// k_scan.hip — scanRegistration on gfx950 (src/scanRegistration.cpp:114-411).
//
// Pipeline (one stream, no host round trip):
//   filter_count/filter_scan/filter_scatter  removeNaN + removeClosedPointCloud, order preserved  (:85-112,136-137)
//   bucket_classify                          elevation -> scanID, azimuth, halfPassed switch index (:141-236)
//   bucket_scan / bucket_scatter             stable counting sort into laserCloud by scanID        (:238-252)
//   curvature                                11-point fp32 stencil, reference summation order       (:256-266)
//   line_features (one workgroup per line)   segment sort, corner / flat greedy selection,
//                                            less-flat candidates, per-line VoxelGrid(0.2)          (:277-408)
//   concat                                   line-major concatenation of the five outputs          (:271-274,407)
// Bit-exactness: libm calls are restated (libm_f32.h atan2f = glibc flt-32; double atan from ocml,
// last-ulp double differences cannot move a float elevation across a scan boundary except with
// probability ~2^-29 per point), and -ffp-contract=off keeps every fp32 op separately rounded.
#include "aloam_device.hpp"
#include "aloam_internal.hpp"
#include "libm_f32.h"
#include "ls_sort.hpp"

namespace aloam {

constexpr int SB = 256;  // threads per block for the per-point kernels

// ------------------------------------------------------------------------------------------
// block-wide exclusive scan of one int per thread (256 threads)
__device__ inline int block_excl_scan_256(int v, int* sh, int* total) {
    const int lane = lane_id(), w = threadIdx.x / WAVE;
    int x = v;
    x = wave_incl_scan(x);
    if (lane == WAVE - 1) sh[w] = x;
    __syncthreads();
    int base = 0;
    for (int i = 0; i < w; i++) base += sh[i];
    int tot = 0;
    for (int i = 0; i < SB / WAVE; i++) tot += sh[i];
    __syncthreads();
    if (total) *total = tot;
    return base + x - v;
}

__device__ inline bool keep_point(const float4 p, int dense, float thres) {
    if (!dense && !(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) return false;
    // removeClosedPointCloud (:99): float arithmetic, strict <
    return !(p.x * p.x + p.y * p.y + p.z * p.z < thres * thres);
}

__global__ void k_filter_count(const float4* __restrict__ in, int n, int dense, float thres, int* blk) {
    __shared__ int sh[SB / WAVE];
    int i = blockIdx.x * SB + threadIdx.x;
    int k = (i < n) && keep_point(in[i], dense, thres);
    int tot;
    block_excl_scan_256(k, sh, &tot);
    if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

// single block of 1024: exclusive scan of nb ints in place, total -> *total
__global__ void k_scan_small(int* a, int nb, int* total) {
    block_scan_array(a, nb, total);
}

__global__ void k_filter_scatter(const float4* __restrict__ in, int n, int dense, float thres, const int* blk,
                                 float4* __restrict__ out) {
    __shared__ int sh[SB / WAVE];
    int i = blockIdx.x * SB + threadIdx.x;
    float4 p = i < n ? in[i] : make_float4(0, 0, 0, 0);
    int k = (i < n) && keep_point(p, dense, thres);
    int r = block_excl_scan_256(k, sh, nullptr);
    if (k) out[blk[blockIdx.x] + r] = p;
}

// ------------------------------------------------------------------------------------------
// start / end azimuth (:141-153), recomputed identically by every thread that needs it
struct Oris { float start, end; };
__device__ inline Oris start_end_ori(const float4* cl, int n) {
    Oris o;
    o.start = -lm_atan2f(cl[0].y, cl[0].x);
    o.end = -lm_atan2f(cl[n - 1].y, cl[n - 1].x) + 2 * M_PI;
    if (o.end - o.start > 3 * M_PI) o.end -= 2 * M_PI;
    else if (o.end - o.start < M_PI) o.end += 2 * M_PI;
    return o;
}

// scanID of one point (:166-205); -1 = dropped
__device__ inline int scan_id(float4 p, int N_SCANS, float gmin, float gmax) {
    float angle = atan((double)p.z / sqrt((double)(p.x * p.x + p.y * p.y))) * 180 / M_PI;
    int scanID;
    if (N_SCANS == 16) {
        scanID = int((angle + 15) / 2 + 0.5);
        if (scanID > (N_SCANS - 1) || scanID < 0) return -1;
    } else if (N_SCANS == 32) {
        scanID = int((angle + 92.0 / 3.0) * 3.0 / 4.0);
        if (scanID > (N_SCANS - 1) || scanID < 0) return -1;
    } else if (N_SCANS == 64) {
        if (angle >= -8.83) scanID = int((2 - angle) * 3.0 + 0.5);
        else scanID = N_SCANS / 2 + int((-8.83 - angle) * 2.0 + 0.5);
        if (angle > 2 || angle < -24.33 || scanID > 50 || scanID < 0) return -1;
    } else {
        double lo = gmin, hi = gmax;
        scanID = int((angle - lo) / (hi - lo) * (N_SCANS - 1) + 0.5);
        if (scanID > (N_SCANS - 1) || scanID < 0) return -1;
    }
    return scanID;
}

// first half of the azimuth unwrap (:209-224): returns adjusted ori, sets *passed
__device__ inline float ori_branch1(float ori, float startOri, bool* passed) {
    if (ori < startOri - M_PI / 2) ori += 2 * M_PI;
    else if (ori > startOri + M_PI * 3 / 2) ori -= 2 * M_PI;
    *passed = (ori - startOri > M_PI);
    return ori;
}
__device__ inline float ori_branch2(float ori, float endOri) {   // (:225-236)
    ori += 2 * M_PI;
    if (ori < endOri - M_PI * 3 / 2) ori += 2 * M_PI;
    else if (ori > endOri + M_PI / 2) ori -= 2 * M_PI;
    return ori;
}

__global__ void k_bucket_classify(const float4* __restrict__ cl, const ScanMeta* meta, int N_SCANS, float gmin, float gmax,
                                  int* __restrict__ sid, float* __restrict__ ori_out, int* hist, int nb, ScanMeta* meta_w) {
    __shared__ int h[MAXL];
    __shared__ int jmin;
    __shared__ Oris sh_o;
    const int n = meta->n_cl;
    for (int i = threadIdx.x; i < N_SCANS; i += SB) h[i] = 0;
    if (threadIdx.x == 0) { jmin = 0x7fffffff; if (n > 0) sh_o = start_end_ori(cl, n); }   // once per block
    __syncthreads();
    int j = blockIdx.x * SB + threadIdx.x;
    if (j < n) {
        float4 p = cl[j];
        int s = scan_id(p, N_SCANS, gmin, gmax);
        sid[j] = s;
        if (s >= 0) {
            float ori = -lm_atan2f(p.y, p.x);
            ori_out[j] = ori;
            bool passed;
            ori_branch1(ori, sh_o.start, &passed);
            if (passed) atomicMin(&jmin, j);
            atomicAdd(&h[s], 1);
        }
    }
    __syncthreads();
    // one global atomic per block (about half the points pass: a per-point atomicMin on one address
    // serialised the kernel)
    if (threadIdx.x == 0 && jmin != 0x7fffffff) atomicMin(&meta_w->jstar, jmin);
    if (blockIdx.x < nb)
        for (int i = threadIdx.x; i < N_SCANS; i += SB) hist[i * nb + blockIdx.x] = h[i];
}

// Line bucket offsets: one workgroup per line L. Its base is the sum of every count of the lines
// before it (hist is line-major [line][block], so that is the prefix hist[0, L nb): read in int4
// pieces, counts only, never rewritten), then the exclusive scan of its own nb block counts. The
// offsets go to hoff (the scatter's table), line_off[L] = base. N_SCANS workgroups instead of one
// serial workgroup over all N_SCANS x nb counts (22 us -> a few us at HDL-64 sizes).
constexpr int BK_T = 512;
__global__ void __launch_bounds__(BK_T) k_bucket_scan(const int* __restrict__ hist, int nb, int N_SCANS, ScanMeta* meta,
                                                      int* __restrict__ hoff) {
    const int L = blockIdx.x, t = threadIdx.x;
    const int pre = L * nb;
    int s = 0;
    const int4* h4 = (const int4*)hist;
    for (int i = t; i < pre / 4; i += BK_T) { const int4 v = h4[i]; s += (v.x + v.y) + (v.z + v.w); }
    for (int i = (pre & ~3) + t; i < pre; i += BK_T) s += hist[i];
    int base;
    (void)block_exscan<BK_T>(s, &base);
    int run = base;
    const int* row = hist + pre;
    for (int c0 = 0; c0 < nb; c0 += BK_T) {
        const int v = c0 + t < nb ? row[c0 + t] : 0;
        int tot;
        const int ex = block_exscan<BK_T>(v, &tot);
        if (c0 + t < nb) hoff[pre + c0 + t] = run + ex;
        run += tot;
    }
    if (t == 0) {
        meta->line_off[L] = base;
        if (L == N_SCANS - 1) {
            meta->line_off[N_SCANS] = run;
            meta->cloud_size = run;
        }
    }
}

__global__ void k_bucket_scatter(const float4* __restrict__ cl, const ScanMeta* meta, const int* __restrict__ sid,
                                 const float* __restrict__ ori_in, const int* __restrict__ hist, int nb, int N_SCANS,
                                 float4* __restrict__ cloud) {
    __shared__ int wcnt[SB / WAVE][MAXL];
    __shared__ Oris sh_o;
    const int n = meta->n_cl;
    const int w = threadIdx.x / WAVE, lane = lane_id();
    for (int i = threadIdx.x; i < (SB / WAVE) * MAXL; i += SB) (&wcnt[0][0])[i] = 0;
    if (threadIdx.x == 0 && n > 0) sh_o = start_end_ori(cl, n);   // once per block
    __syncthreads();
    int j = blockIdx.x * SB + threadIdx.x;
    int s = j < n ? sid[j] : -1;
    // stable rank within the wave among equal scanIDs (match-any emulation)
    int rank = 0;
    unsigned long long active = __ballot(s >= 0);
    while (active) {
        int leader = __ffsll((long long)active) - 1;
        int ls = readlane_i(s, leader);
        unsigned long long m = __ballot(s == ls);
        if (s == ls) rank = __popcll(m & lanemask_lt64());
        if (lane == leader) wcnt[w][ls] = __popcll(m);
        active &= ~m;
    }
    __syncthreads();
    if (s >= 0) {
        int before = 0;
        for (int ww = 0; ww < w; ww++) before += wcnt[ww][s];
        float4 p = cl[j];
        const Oris o = sh_o;
        float ori = ori_in[j];
        if (j <= meta->jstar) { bool passed; ori = ori_branch1(ori, o.start, &passed); }
        else ori = ori_branch2(ori, o.end);
        float relTime = (ori - o.start) / (o.end - o.start);
        p.w = s + 0.1 * relTime;   // scanPeriod * relTime in double, stored as float (:239)
        cloud[hist[s * nb + blockIdx.x] + before + rank] = p;
    }
}

// curvature (:256-266) for i in [5, cloudSize - 5); 0 elsewhere
__global__ void k_curvature(const float4* __restrict__ c, const ScanMeta* meta, float* __restrict__ curv) {
    const int n = meta->cloud_size;
    int i = blockIdx.x * SB + threadIdx.x;
    if (i >= n) return;
    if (i < 5 || i >= n - 5) { curv[i] = 0.f; return; }
    const float4* p = c + i;
    float dX = p[-5].x + p[-4].x + p[-3].x + p[-2].x + p[-1].x - 10 * p[0].x + p[1].x + p[2].x + p[3].x + p[4].x + p[5].x;
    float dY = p[-5].y + p[-4].y + p[-3].y + p[-2].y + p[-1].y - 10 * p[0].y + p[1].y + p[2].y + p[3].y + p[4].y + p[5].y;
    float dZ = p[-5].z + p[-4].z + p[-3].z + p[-2].z + p[-1].z - 10 * p[0].z + p[1].z + p[2].z + p[3].z + p[4].z + p[5].z;
    curv[i] = dX * dX + dY * dY + dZ * dZ;
}

// ------------------------------------------------------------------------------------------
// libstdc++ std::sort (introsort) replica on int indices compared by curvature — only used for
// segments whose curvatures contain exact ties, where the unstable order of the reference's
// std::sort (:288) decides which of the equal points is picked first.
struct CurvLess {
    const float* c;
    int base;
    __device__ bool operator()(int a, int b) const { return c[a - base] < c[b - base]; }
};
__device__ void dev_unguarded_linear_insert(int* last, CurvLess less) {
    int val = *last;
    int* next = last - 1;
    while (less(val, *next)) { *last = *next; last = next; --next; }
    *last = val;
}
__device__ void dev_insertion_sort(int* first, int* last, CurvLess less) {
    if (first == last) return;
    for (int* i = first + 1; i != last; ++i) {
        if (less(*i, *first)) {
            int val = *i;
            for (int* k = i; k != first; --k) *k = *(k - 1);
            *first = val;
        } else dev_unguarded_linear_insert(i, less);
    }
}
__device__ void dev_adjust_heap(int* first, long hole, long len, int value, CurvLess less) {
    const long top = hole;
    long child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (less(first[child], first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    long parent = (hole - 1) / 2;
    while (hole > top && less(first[parent], value)) { first[hole] = first[parent]; hole = parent; parent = (hole - 1) / 2; }
    first[hole] = value;
}
__device__ void dev_heap_sort(int* first, int* last, CurvLess less) {
    long len = last - first;
    if (len >= 2) {
        long parent = (len - 2) / 2;
        while (true) { dev_adjust_heap(first, parent, len, first[parent], less); if (parent == 0) break; parent--; }
    }
    while (last - first > 1) {
        --last;
        int v = *last; *last = *first;
        dev_adjust_heap(first, 0L, (long)(last - first), v, less);
    }
}
__device__ inline void iswap(int* a, int* b) { int t = *a; *a = *b; *b = t; }
__device__ void dev_std_sort(int* first, int* last, CurvLess less) {
    if (first == last) return;
    long n = last - first;
    long depth = (63 - __clzll((long long)n)) * 2;
    // introsort loop with an explicit stack (recursion on the right part)
    int* stk_f[64]; int* stk_l[64]; long stk_d[64]; int sp = 0;
    stk_f[sp] = first; stk_l[sp] = last; stk_d[sp] = depth; sp++;
    while (sp > 0) {
        sp--;
        int* f = stk_f[sp]; int* l = stk_l[sp]; long d = stk_d[sp];
        while (l - f > 16) {
            if (d == 0) { dev_heap_sort(f, l, less); break; }
            --d;
            int* mid = f + (l - f) / 2;
            int *a = f + 1, *b = mid, *c = l - 1;
            if (less(*a, *b)) {
                if (less(*b, *c)) iswap(f, b); else if (less(*a, *c)) iswap(f, c); else iswap(f, a);
            } else if (less(*a, *c)) iswap(f, a); else if (less(*b, *c)) iswap(f, c); else iswap(f, b);
            int *lo = f + 1, *hi = l;
            while (true) {
                while (less(*lo, *f)) ++lo;
                --hi;
                while (less(*f, *hi)) --hi;
                if (!(lo < hi)) break;
                iswap(lo, hi);
                ++lo;
            }
            // recurse on [lo, l) first (pushed), continue with [f, lo)
            // libstdc++ recurses on the right part then loops on the left; order of processing
            // does not change the result because the two ranges are disjoint.
            stk_f[sp] = lo; stk_l[sp] = l; stk_d[sp] = d; sp++;
            l = lo;
        }
    }
    if (n > 16) {
        dev_insertion_sort(first, first + 16, less);
        for (int* i = first + 16; i != last; ++i) dev_unguarded_linear_insert(i, less);
    } else dev_insertion_sort(first, last, less);
}

// ------------------------------------------------------------------------------------------
// One workgroup (1024 threads) per scan line: (:277-408)
constexpr int LT = 1024;
constexpr int LINE_HDR = 256;                          // LDS header (LineShared) ahead of the line arrays
constexpr size_t line_gapw_end() { return LINE_HDR + (size_t)LINE_LDS_CAP * (4 * 4 + 4 + 8 + 2) + (LINE_LDS_CAP / 32 + 2) * 4; }
constexpr size_t line_lds_bytes() { return ((line_gapw_end() + 15) & ~(size_t)15) + (size_t)LINE_LDS_CAP * 8; }   // + sort output

__device__ inline void suppress_neighbours(int ind, const float* X, const float* Y, const float* Z, volatile int8_t* picked) {
    for (int l = 1; l <= 5; l++) {
        float dx = X[ind + l] - X[ind + l - 1], dy = Y[ind + l] - Y[ind + l - 1], dz = Z[ind + l] - Z[ind + l - 1];
        if (dx * dx + dy * dy + dz * dz > 0.05) break;
        picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
        float dx = X[ind + l] - X[ind + l + 1], dy = Y[ind + l] - Y[ind + l + 1], dz = Z[ind + l] - Z[ind + l + 1];
        if (dx * dx + dy * dy + dz * dz > 0.05) break;
        picked[ind + l] = 1;
    }
}

__device__ inline void bitonic_sort_u64(unsigned long long* k, int n2) {
    for (int size = 2; size <= n2; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = threadIdx.x; t < n2 / 2; t += blockDim.x) {
                int i = 2 * t - (t & (stride - 1));
                int j = i + stride;
                bool asc = ((i & size) == 0);
                unsigned long long a = k[i], b = k[j];
                if ((a > b) == asc) { k[i] = b; k[j] = a; }
            }
            __syncthreads();
        }
    }
}

#ifdef ALOAM_LF_TIMING
__device__ unsigned long long g_lf_ts[64][8];      // micro-benchmark only: per-line phase stamps
#define LF_TS(k) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_lf_ts[blockIdx.x][k] = wall_clock64(); } while (0)
__device__ unsigned long long g_lf_ts2[64][16];     // greedy: per-segment stamps (corners, flats)
#define LF_TS2(k) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_lf_ts2[blockIdx.x][k] = wall_clock64(); } while (0)
extern "C" int aloam_dbg_lf_ts2(unsigned long long* out) { return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lf_ts2), sizeof(g_lf_ts2)); }
__device__ unsigned long long g_lf_ts3[64][8];      // sort phase sub-steps
#define LF_TS3(k) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_lf_ts3[blockIdx.x][k] = wall_clock64(); } while (0)
extern "C" int aloam_dbg_lf_ts3(unsigned long long* out) { return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lf_ts3), sizeof(g_lf_ts3)); }
extern "C" int aloam_dbg_lf_ts(unsigned long long* out) { return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lf_ts), sizeof(g_lf_ts)); }
__device__ int g_lf_cnt[64][12];                    // per segment: corner chunks, corner pick-loop trips
#define LF_CNT(j, k) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_lf_cnt[blockIdx.x][2 * (j) + (k)]++; } while (0)
#define LF_CNT0(j) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_lf_cnt[blockIdx.x][2 * (j)] = g_lf_cnt[blockIdx.x][2 * (j) + 1] = 0; } while (0)
extern "C" int aloam_dbg_lf_cnt(int* out) { return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lf_cnt), sizeof(g_lf_cnt)); }
#else
#define LF_CNT(j, k) do { } while (0)
#define LF_CNT0(j) do { } while (0)
#define LF_TS(k) do { } while (0)
#define LF_TS2(k) do { } while (0)
#define LF_TS3(k) do { } while (0)
#endif
// The body, instantiated per storage class of the line's arrays: with LDS lines the pointers are
// provably LDS, so the compiler emits ds_* instructions instead of generic flat accesses.
template <bool BIG>
__device__ __forceinline__ void line_features_body(const float4* __restrict__ cloud, const float* __restrict__ gcurv,
                                                      const ScanMeta* meta, int N_SCANS,
                                                      float4* g_xyz, unsigned long long* g_keys, int* g_i,
                                                      int* line_sharp, int* line_lsharp, int* line_flat, int* line_cnt,
                                                      float4* line_lf, unsigned char* smem_raw) {
    // all LDS is dynamic (Guideline 17: no statics ahead of the dynamic base)
    struct LineShared { int flag, ncand, nrun, cnt[3]; unsigned bb[6]; int wsum[LT / WAVE]; int tlo[6], thi[6]; };
    LineShared& SH = *(LineShared*)smem_raw;
    unsigned char* smem = smem_raw + LINE_HDR;
    static_assert(sizeof(LineShared) <= LINE_HDR, "LineShared");
    int& s_flag = SH.flag; int& s_ncand = SH.ncand; int& s_nrun = SH.nrun;
    int* s_cnt = SH.cnt; unsigned* s_bb = SH.bb; int* s_wsum = SH.wsum; int* s_tlo = SH.tlo; int* s_thi = SH.thi;
    const int line = blockIdx.x;
    const int off0 = meta->line_off[line], off1 = meta->line_off[line + 1];
    const int nl = off1 - off0;
    const int s = off0 + 5, e = off1 - 6;
    int* cnt_out = line_cnt + line * 4;
    if (e - s < 6) {
        if (threadIdx.x < 4) cnt_out[threadIdx.x] = 0;
        return;
    }
    constexpr bool big = BIG;              // lines above the LDS cap keep their arrays in global scratch
    // carve LDS (or global scratch at the line's offset for oversized lines)
    float *X, *Y, *Z, *Cv;
    int* S;                 // sorted global indices per segment position
    int8_t* picked;                   // ordered by the fence at the end of every greedy chunk
    int8_t* label;
    unsigned* gapw;         // bit i of word i/32: pair (i, i+1) is a suppression stop
    unsigned long long* keys;
    unsigned long long* sorted = nullptr;   // LDS lines: chunk_rank_sort output
    if constexpr (!big) {
        X = (float*)smem;
        Y = X + LINE_LDS_CAP;
        Z = Y + LINE_LDS_CAP;
        Cv = Z + LINE_LDS_CAP;
        S = (int*)(Cv + LINE_LDS_CAP);
        keys = (unsigned long long*)(S + LINE_LDS_CAP);
        picked = (int8_t*)(keys + LINE_LDS_CAP);
        label = (int8_t*)(picked + LINE_LDS_CAP);
        gapw = (unsigned*)(label + LINE_LDS_CAP);
        sorted = (unsigned long long*)(smem_raw + ((line_gapw_end() + 15) & ~(size_t)15));
    } else {
        float* gx = (float*)g_xyz;     // 4 floats per cloud point of scratch
        X = gx + off0;
        Y = gx + (size_t)meta->cloud_size + off0;
        Z = gx + 2 * (size_t)meta->cloud_size + off0;
        Cv = gx + 3 * (size_t)meta->cloud_size + off0;
        S = g_i + off0;
        keys = g_keys + 2 * (size_t)off0;   // 2x room for the power-of-two padding
        picked = (int8_t*)(g_i + (size_t)meta->cloud_size + off0);
        label = (int8_t*)(g_i + 2 * (size_t)meta->cloud_size + off0);
        gapw = (unsigned*)((int8_t*)(g_i + (size_t)meta->cloud_size + off0) + ((nl + 3) & ~3));   // rest of picked's int slab
    }
    for (int k = threadIdx.x; k < nl; k += LT) {
        float4 p = cloud[off0 + k];
        X[k] = p.x; Y[k] = p.y; Z[k] = p.z;
        Cv[k] = gcurv[off0 + k];
        picked[k] = 0;
        label[k] = 0;
    }
    if (threadIdx.x < 3) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    LF_TS(0);
    // ---- gap bits: pair (i, i+1) of the line is a suppression stop when its fp32 squared
    // distance > 0.05 (:321-338, :366-383 compute exactly this for every neighbour test) ----
    for (int base = threadIdx.x & ~(WAVE - 1); base < nl; base += LT) {
        const int i = base + lane_id();
        bool gap = false;
        if (i + 1 < nl) {
            const float dx = X[i + 1] - X[i], dy = Y[i + 1] - Y[i], dz = Z[i + 1] - Z[i];
            gap = dx * dx + dy * dy + dz * dz > 0.05;
        }
        const unsigned long long m = __ballot(gap);
        if (lane_id() < 2) gapw[base / 32 + lane_id()] = (unsigned)(m >> (32 * lane_id()));
    }
    // ---- segment sorts (:282-289), all 6 segments at once. LDS lines: one bitonic sort of
    // (segment, curvature bits, position) keys — stable by position, like the rank order; big lines:
    // rank sort. A segment with exact curvature ties is redone by the libstdc++ introsort replica
    // (thread 0), since std::sort's unstable order is what the reference produces. ----
    if (threadIdx.x < 6) { s_tlo[threadIdx.x] = 0x7fffffff; s_thi[threadIdx.x] = -1; }
    __syncthreads();
    LF_TS3(0);
#ifdef ALOAM_LF_RANKSORT
    if (false) {
#else
    if (!big) {
#endif
        const int M = e - s;                                             // positions s .. e-1
        const int n2 = (M + WAVE - 1) / WAVE * WAVE;
        for (int i = threadIdx.x; i < n2; i += LT) {
            unsigned long long key = ~0ull;
            if (i < M) {
                const int a = s + i;
                int j = (int)(((long long)i * 6) / (e - s));
                while (j > 0 && a < s + (e - s) * j / 6) j--;
                while (j < 5 && a >= s + (e - s) * (j + 1) / 6) j++;
                key = ((unsigned long long)j << 44) | ((unsigned long long)__float_as_uint(Cv[a - off0]) << 12) | (unsigned)i;
            }
            keys[i] = key;
        }
        __syncthreads();
        LF_TS3(1);
        const unsigned long long* sorted_k = block_merge_sort<unsigned long long, LINE_LDS_CAP / LT>(keys, sorted, n2);
        LF_TS3(2);
        for (int i = threadIdx.x; i < M; i += LT) {
            const unsigned long long key = sorted_k[i];
            S[s - off0 + i] = s + (int)(key & 0xfffu);
            if (i > 0 && (sorted_k[i - 1] >> 12) == (key >> 12)) {      // exact tie: sorted slots s+i-1, s+i
                atomicMin(&s_tlo[(int)(key >> 44)], s + i - 1);
                atomicMax(&s_thi[(int)(key >> 44)], s + i);
            }
        }
    } else {
        for (int a = s + threadIdx.x; a <= e - 1; a += LT) {
            int j = (int)(((long long)(a - s) * 6) / (e - s));          // segment of a (sp_j <= a)
            while (j > 0 && a < s + (e - s) * j / 6) j--;
            while (j < 5 && a >= s + (e - s) * (j + 1) / 6) j++;
            const int sp = s + (e - s) * j / 6, ep = s + (e - s) * (j + 1) / 6 - 1;
            const int b0 = sp - off0, ai = a - sp, m = ep - sp + 1;
            const float ca = Cv[a - off0];
            int rank = 0, ties = 0;
            for (int bi = 0; bi < m; bi++) {
                const float cb = Cv[b0 + bi];
                rank += (cb < ca) || (cb == ca && bi < ai);
                ties += (cb == ca);
            }
            S[b0 + rank] = a;
            if (ties > 1) { atomicMin(&s_tlo[j], sp + rank); atomicMax(&s_thi[j], sp + rank); }
        }
    }
    __syncthreads();
    LF_TS3(3);
    // exact curvature ties: std::sort's unstable order decides how a tie group is arranged, which
    // matters only if the greedy below reads one of the group's sorted slots; such a segment is redone
    // by the libstdc++ introsort replica and the selection rerun (rare: ties fall mid-order)
    int8_t* posmap = (int8_t*)keys;      // greedy scratch (chunk lane + 1 by line position); keys are rebuilt after
    for (int k = threadIdx.x; k < nl; k += LT) posmap[k] = 0;
    __syncthreads();
    LF_TS(1);
    // ---- greedy selection, one wave, segments in order (:291-390). The sorted candidates go in
    // chunks of 64 (one per lane). Within a chunk the sequential greedy is resolved in parallel:
    // suppression is symmetric (a pick at P marks P+d, |d| <= 5, iff no gap pair lies between them,
    // which is also the test seen from P+d), so lane i can only lose to an earlier-ranked candidate
    // inside its own extents; those are found through a position -> lane map, and the picks follow
    // in rank order by fixed-point rounds over the conflict masks (usually 1-3). Only the first
    // `quota` picks of a chunk count, exactly as the sequential loop stops at its quota. ----
    if (threadIdx.x < WAVE) {
        const int lane = threadIdx.x;
        const unsigned long long lt = lanemask_lt64();
        int n_sharp = 0, n_lsharp = 0, n_flat = 0;
        unsigned redone = 0;                                    // segments in libstdc++ tie order
        // suppression extents of line position p: marks p+1..p+nf and p-1..p-nb (:321-338)
        auto extents = [&](int p, int& nf, int& nbk) {
            const int q0 = p - 5;                                              // pairs p-5 .. p+4
            const int w0 = q0 >> 5, sh = q0 & 31;
            const unsigned long long win = ((unsigned long long)gapw[w0 + 1] << 32 | gapw[w0]) >> sh;
            const unsigned fwd = (unsigned)(win >> 5) & 31u;                 // bit 0 = pair (p, p+1)
            const unsigned bwd = (unsigned)(win & 31u);                        // bit 4 = pair (p-1, p)
            nf = fwd ? __builtin_ctz(fwd) : 5;
            nbk = bwd ? __builtin_clz(bwd << 27) : 5;
        };
        // picks among this chunk's candidates (lane order = rank order), resolved in parallel
        auto resolve = [&](bool cand, int p, int nf, int nbk) -> unsigned long long {
            if (cand) posmap[p] = (int8_t)(lane + 1);
            __threadfence_block();
            __builtin_amdgcn_wave_barrier();
            unsigned long long conf = 0;
            if (cand) {
#pragma unroll
                for (int d = 1; d <= 5; d++) {
                    const int qf = d <= nf ? posmap[p + d] : 0, qb = d <= nbk ? posmap[p - d] : 0;
                    if (qf) conf |= 1ull << (qf - 1);
                    if (qb) conf |= 1ull << (qb - 1);
                }
            }
            const unsigned long long cm = __ballot(cand);
            conf &= cm & lt;                                   // only earlier-ranked candidates suppress
            unsigned long long decided = ~cm, pickm = 0;
            while (~decided) {
                const bool ready = !((decided >> lane) & 1) && (conf & ~decided) == 0;
                pickm |= __ballot(ready && (conf & pickm) == 0);
                decided |= __ballot(ready);
            }
            if (cand) posmap[p] = 0;
            return pickm;
        };
        auto mark = [&](int p, int nf, int nbk) {
            picked[p] = 1;
#pragma unroll
            for (int d = 1; d <= 5; d++) {
                if (d <= nf) picked[p + d] = 1;
                if (d <= nbk) picked[p - d] = 1;
            }
        };
        for (;;) {
        unsigned need = 0;
        n_sharp = n_lsharp = n_flat = 0;
        for (int j = 0; j < 6 && !need; j++) {
            int lo_read, hi_read;                               // sorted slots read: corners [lo, ep], flats [sp, hi]
            const int sp = s + (e - s) * j / 6, ep = s + (e - s) * (j + 1) / 6 - 1;
            // corners: from the largest curvature, at most 20 picks, the first 2 sharp
            int largest = 0;
            lo_read = ep + 1;
            bool stop = false;
            LF_CNT0(j);
            for (int top = ep; top >= sp && !stop; top -= WAVE) {
                LF_CNT(j, 0);
                const int k = top - lane;
                const bool valid = k >= sp;
                const int p = (valid ? S[k - off0] : sp) - off0;
                const bool cv_ok = valid && (double)Cv[p] > 0.1;
                if (!__ballot(cv_ok)) break;                                   // sorted: nothing > 0.1 remains
                lo_read = max(top - (WAVE - 1), sp);
                int nf = 0, nbk = 0;
                if (cv_ok) extents(p, nf, nbk);
                const bool cand = cv_ok && picked[p] == 0;
                const unsigned long long pickm = resolve(cand, p, nf, nbk);
                const int npk = __popcll(pickm), quota = 20 - largest;
                const int rank = __popcll(pickm & lt);
                if ((pickm >> lane) & 1 && rank < quota) {
                    const int g = largest + rank;                              // 0-based pick number
                    label[p] = g < 2 ? 2 : 1;
                    mark(p, nf, nbk);
                    if (g < 2) line_sharp[line * LINE_SHARP_CAP + n_sharp + g] = p + off0;
                    line_lsharp[line * LINE_LSHARP_CAP + n_lsharp + g] = p + off0;
                }
                if (npk > quota) stop = true;
                largest += min(npk, quota);
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
            }
            n_sharp += min(largest, 2);
            n_lsharp += largest;
            LF_TS2(2 * j);
            // flats: from the smallest curvature; the 4th pick is labelled but not marked (:366-388)
            int smallest = 0;
            hi_read = sp - 1;
            stop = false;
            for (int bot = sp; bot <= ep && !stop; bot += WAVE) {
                const int k = bot + lane;
                const bool valid = k <= ep;
                const int p = (valid ? S[k - off0] : sp) - off0;
                const bool cv_ok = valid && (double)Cv[p] < 0.1;
                if (!__ballot(cv_ok)) break;                                   // sorted: nothing < 0.1 remains
                hi_read = min(bot + (WAVE - 1), ep);
                int nf = 0, nbk = 0;
                if (cv_ok) extents(p, nf, nbk);
                const bool cand = cv_ok && picked[p] == 0;
                const unsigned long long pickm = resolve(cand, p, nf, nbk);
                const int npk = __popcll(pickm), quota = 4 - smallest;
                const int rank = __popcll(pickm & lt);
                if ((pickm >> lane) & 1 && rank < quota) {
                    const int g = smallest + rank;
                    label[p] = -1;
                    line_flat[line * LINE_FLAT_CAP + n_flat + g] = p + off0;
                    if (g < 3) mark(p, nf, nbk);
                }
                smallest += min(npk, quota);
                if (smallest >= 4) stop = true;
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
            }
            n_flat += smallest;
            LF_TS2(2 * j + 1);
            // a segment whose tie group overlaps the slots read is redone in libstdc++ order and the
            // selection reruns from the start (later segments see its marks); redone segments are exact
            if (!((redone >> j) & 1) && s_tlo[j] <= s_thi[j] && (s_thi[j] >= lo_read || s_tlo[j] <= hi_read)) need = 1u << j;
        }
        if (!need) break;
        if (lane == 0) {
            for (int j = 0; j < 6; j++) {
                if (!((need >> j) & 1)) continue;
                const int sp = s + (e - s) * j / 6, ep = s + (e - s) * (j + 1) / 6 - 1;
                const int b0 = sp - off0, m = ep - sp + 1;
                for (int a = 0; a < m; a++) S[b0 + a] = sp + a;
                dev_std_sort(S + b0, S + b0 + m, CurvLess{Cv, off0});
            }
            LF_TS3(4);
        }
        for (int k = lane; k < nl; k += WAVE) { picked[k] = 0; label[k] = 0; }
        redone |= need;
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        }
        LF_TS2(12);
        static_assert(LINE_SHARP_CAP >= 12 && LINE_FLAT_CAP >= 24 && LINE_LSHARP_CAP >= 120, "list slots");
        if (lane == 0) { s_cnt[0] = n_sharp; s_cnt[1] = n_lsharp; s_cnt[2] = n_flat; }
    }
    __syncthreads();
    LF_TS(2);
    // ---- less-flat candidates: label <= 0 in [s, e-1], cloud order (:392-398) ----
    // compact into S (reused) by a block-wide scan over chunks of LT
    if (threadIdx.x == 0) s_ncand = 0;
    __syncthreads();
    const int lanei = lane_id(), wi = threadIdx.x / WAVE;
    for (int base = s; base <= e - 1; base += LT) {
        const int k = base + threadIdx.x;
        const int flag = (k <= e - 1) && label[k - off0] <= 0;
        const unsigned long long mk = __ballot(flag);
        if (lanei == 0) s_wsum[wi] = __popcll(mk);
        __syncthreads();
        int before = s_ncand;
        for (int ww = 0; ww < wi; ww++) before += s_wsum[ww];
        if (flag) S[before + __popcll(mk & lanemask_lt64())] = k - off0;
        __syncthreads();
        if (threadIdx.x == 0) { int t = 0; for (int ww = 0; ww < LT / WAVE; ww++) t += s_wsum[ww]; s_ncand += t; }
        __syncthreads();
    }
    const int nc = s_ncand;
    LF_TS(3);
    // ---- the less-flat candidates (line-relative indices, scan order) and their count for k_line_vox,
    // which filters them (VoxelGrid 0.2, PCL order) on its own, possibly on another stream ----
    if constexpr (!big) {
        int* gS = g_i + off0;
        for (int t = threadIdx.x; t < nc; t += LT) gS[t] = S[t];
    }
    if (threadIdx.x == 0) {
        cnt_out[0] = s_cnt[0]; cnt_out[1] = s_cnt[1]; cnt_out[2] = s_cnt[2]; cnt_out[3] = nc;
    }
    LF_TS(4);
}

// oversized lines (rare): not inlined, so their global-scratch body does not load the LDS path's registers
__device__ __noinline__ void line_features_big(const float4* __restrict__ cloud, const float* __restrict__ gcurv, const ScanMeta* meta,
                                               int N_SCANS, float4* g_xyz, unsigned long long* g_keys, int* g_i, int* line_sharp,
                                               int* line_lsharp, int* line_flat, int* line_cnt, float4* line_lf, lds_u8* smem) {
    line_features_body<true>(cloud, gcurv, meta, N_SCANS, g_xyz, g_keys, g_i, line_sharp, line_lsharp, line_flat, line_cnt, line_lf,
                             (unsigned char*)smem);
}
__global__ void __launch_bounds__(LT) k_line_features(const float4* __restrict__ cloud, const float* __restrict__ gcurv,
                                                      const ScanMeta* meta, int N_SCANS,
                                                      float4* g_xyz, unsigned long long* g_keys, int* g_i,
                                                      int* line_sharp, int* line_lsharp, int* line_flat, int* line_cnt,
                                                      float4* line_lf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int nl_ = meta->line_off[blockIdx.x + 1] - meta->line_off[blockIdx.x];
    if (nl_ > LINE_LDS_CAP) line_features_big(cloud, gcurv, meta, N_SCANS, g_xyz, g_keys, g_i, line_sharp, line_lsharp, line_flat, line_cnt, line_lf, (lds_u8*)smem_raw);
    else line_features_body<false>(cloud, gcurv, meta, N_SCANS, g_xyz, g_keys, g_i, line_sharp, line_lsharp, line_flat, line_cnt, line_lf, smem_raw);
}

// ------------------------------------------------------------------------------------------
// Per-line VoxelGrid(0.2) of the less-flat candidates (:401-405, PCL 1.8 applyFilter), points summed in
// PCL's order (ls_sort.hpp), one workgroup per line. Its own kernel so that it can run on the context's
// second stream beside the odometry rounds, which do not read the less-flat cloud (it is needed from the
// last-cloud swap on). Reads the candidates k_line_features left (line-relative indices, scan order, at
// g_i + line offset; their count in line_cnt[4 line + 3]) and writes the leaves' centroids + their count.
constexpr int LV_STAGE_CPW = 10;
constexpr int LV_STAGE = LT * LV_STAGE_CPW;              // big lines: sort segments staged through LDS
constexpr size_t LV_HDR = 256;
constexpr size_t lv_lds_bytes() {
    const size_t lds_line = 8 * (size_t)LINE_LDS_CAP + ls_scratch_bytes(LT, LINE_LDS_CAP) + 4 * (size_t)LINE_LDS_CAP;
    const size_t big_line = 8 * (size_t)LV_STAGE + ls_global_scratch_bytes(LT, LV_STAGE);
    return LV_HDR + (lds_line > big_line ? lds_line : big_line);
}
static_assert(lv_lds_bytes() <= 160 * 1024, "LDS");
template <bool BIG>
__device__ __forceinline__ void line_vox_body(const float4* __restrict__ cloud, const ScanMeta* meta, float4* g_xyz,
                                              unsigned long long* g_keys, int* g_i, int* line_cnt, float4* line_lf,
                                              unsigned char* smem_raw) {
    struct VS { unsigned bb[6]; int nrun; int pad; int wsum[LT / WAVE]; };
    static_assert(sizeof(VS) <= LV_HDR, "VS");
    VS& SH = *(VS*)smem_raw;
    unsigned char* smem = smem_raw + LV_HDR;
    const int line = blockIdx.x;
    const int off0 = meta->line_off[line];
    int* cnt_out = line_cnt + line * 4;
    const int nc = cnt_out[3];
    const int* S = g_i + off0;
    const int lanei = lane_id(), wi = threadIdx.x / WAVE;
    __syncthreads();                      // every thread has read nc before thread 0 overwrites it
    if (nc <= 0) { if (threadIdx.x == 0) cnt_out[3] = 0; return; }
    unsigned long long* keys;
    int* heads;
    if constexpr (!BIG) {
        keys = (unsigned long long*)smem;
        heads = (int*)(smem + 8 * (size_t)LINE_LDS_CAP + ls_scratch_bytes(LT, LINE_LDS_CAP));
    } else {
        keys = g_keys + 2 * (size_t)off0;
        heads = (int*)(g_xyz) + 3 * (size_t)meta->cloud_size + off0;
    }
    if (threadIdx.x < 6) SH.bb[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    {
        unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
        for (int t = threadIdx.x; t < nc; t += LT) {
            const float4 p = cloud[off0 + S[t]];
            const unsigned v[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
            for (int d = 0; d < 3; d++) { mn[d] = min(mn[d], v[d]); mx[d] = max(mx[d], v[d]); }
        }
#pragma unroll
        for (int d = 0; d < 3; d++) {
            mn[d] = allreduce_u32<6>(mn[d], [](unsigned a, unsigned b) { return min(a, b); });
            mx[d] = allreduce_u32<6>(mx[d], [](unsigned a, unsigned b) { return max(a, b); });
        }
        if (lanei == 0)
            for (int d = 0; d < 3; d++) { atomicMin(&SH.bb[d], mn[d]); atomicMax(&SH.bb[3 + d], mx[d]); }
    }
    __syncthreads();
    const float inv = 1.0f / 0.2f;
    float minp[3], maxp[3];
    for (int d = 0; d < 3; d++) { minp[d] = ord2f(SH.bb[d]); maxp[d] = ord2f(SH.bb[3 + d]); }
    const long long ddx = (long long)((maxp[0] - minp[0]) * inv) + 1;
    const long long ddy = (long long)((maxp[1] - minp[1]) * inv) + 1;
    const long long ddz = (long long)((maxp[2] - minp[2]) * inv) + 1;
    const bool overflow = ddx * ddy * ddz > 2147483647LL;
    int minb[3], divb[3];
    for (int d = 0; d < 3; d++) {
        minb[d] = (int)floorf(minp[d] * inv);
        const int maxb = (int)floorf(maxp[d] * inv);
        divb[d] = maxb - minb[d] + 1;
    }
    const int mul1 = divb[0], mul2 = divb[0] * divb[1];
    for (int t = threadIdx.x; t < nc; t += LT) {
        const float4 p = cloud[off0 + S[t]];
        unsigned idx;
        if (overflow) idx = (unsigned)t;   // PCL copies the input through unchanged
        else {
            const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
            const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
            const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
            idx = (unsigned)(i0 + i1 * mul1 + i2 * mul2);
        }
        keys[t] = ((unsigned long long)idx << 32) | (unsigned)t;
    }
    __syncthreads();
    // PCL's order of the (leaf, index) pairs: libstdc++ std::sort by leaf (ls_sort.hpp)
    constexpr int LINE_CPW = LINE_LDS_CAP / LT;
    static_assert(LINE_CPW * LT == LINE_LDS_CAP, "LDS lines: whole chunks per wave");
    if (!BIG) {
        ls_sort<LT, LINE_CPW>(keys, nc, nc > 1 ? 2 * (31 - __builtin_clz((unsigned)nc)) : 0, smem + 8 * (size_t)LINE_LDS_CAP, LINE_LDS_CAP);
    } else if (nc <= LT * PS_MAX_CHUNK) {
        ls_sort_global<LT, LV_STAGE_CPW>(keys, nc, (unsigned long long*)smem, LV_STAGE, smem + 8 * (size_t)LV_STAGE);
    } else {
        if (threadIdx.x == 0) ps_serial_std_sort(keys, nc);
        __syncthreads();
    }
    // run heads -> centroids (CentroidPoint: from zero, in sorted order)
    if (threadIdx.x == 0) SH.nrun = 0;
    __syncthreads();
    for (int base = 0; base < nc; base += LT) {
        const int t = base + threadIdx.x;
        const int flag = t < nc && (t == 0 || (keys[t] >> 32) != (keys[t - 1] >> 32));
        const unsigned long long mk = __ballot(flag);
        if (lanei == 0) SH.wsum[wi] = __popcll(mk);
        __syncthreads();
        int before = SH.nrun;
        for (int ww = 0; ww < wi; ww++) before += SH.wsum[ww];
        if (flag) heads[before + __popcll(mk & lanemask_lt64())] = t;
        __syncthreads();
        if (threadIdx.x == 0) { int tt = 0; for (int ww = 0; ww < LT / WAVE; ww++) tt += SH.wsum[ww]; SH.nrun += tt; }
        __syncthreads();
    }
    const int nrun = SH.nrun;
    for (int r = threadIdx.x; r < nrun; r += LT) {
        const int h0 = heads[r], h1 = (r + 1 < nrun) ? heads[r + 1] : nc;
        int nrs;
        const float4 c = ps_run_sum(keys, nc, h0, ps_key(keys[h0]), [&](int i) { return cloud[off0 + S[i]]; }, nrs);
        const float cnt = (float)(h1 - h0);
        line_lf[off0 + r] = make_float4(c.x / cnt, c.y / cnt, c.z / cnt, c.w / cnt);
    }
    if (threadIdx.x == 0) cnt_out[3] = nrun;
}
__device__ __noinline__ void line_vox_big(const float4* __restrict__ cloud, const ScanMeta* meta, float4* g_xyz,
                                          unsigned long long* g_keys, int* g_i, int* line_cnt, float4* line_lf, lds_u8* smem) {
    line_vox_body<true>(cloud, meta, g_xyz, g_keys, g_i, line_cnt, line_lf, (unsigned char*)smem);
}
__global__ void __launch_bounds__(LT) k_line_vox(const float4* __restrict__ cloud, const ScanMeta* meta, float4* g_xyz,
                                                 unsigned long long* g_keys, int* g_i, int* line_cnt, float4* line_lf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int nc = line_cnt[blockIdx.x * 4 + 3];
    if (nc > LINE_LDS_CAP) line_vox_big(cloud, meta, g_xyz, g_keys, g_i, line_cnt, line_lf, (lds_u8*)smem_raw);
    else line_vox_body<false>(cloud, meta, g_xyz, g_keys, g_i, line_cnt, line_lf, smem_raw);
}

// the less-flat cloud in line order and its count (the other kinds: k_concat)
__global__ void k_concat_lf(const int* line_cnt, const float4* line_lf, int N_SCANS, ScanMeta* meta, float4* lflat) {
    const int line = blockIdx.x;
    __shared__ int sh_o, sh_tot;
    if (threadIdx.x == 0) { sh_o = 0; sh_tot = 0; }
    __syncthreads();
    {
        const int l = threadIdx.x;
        const int v = l < N_SCANS ? line_cnt[l * 4 + 3] : 0;
        if (threadIdx.x < WAVE * ((N_SCANS + WAVE - 1) / WAVE)) {
            const int a = wave_sum_i(l < line ? v : 0), b = wave_sum_i(v);
            if (lane_id() == 0) { if (a) atomicAdd(&sh_o, a); if (b) atomicAdd(&sh_tot, b); }
        }
    }
    __syncthreads();
    const int o = sh_o, n = line_cnt[line * 4 + 3];
    const int off0 = meta->line_off[line];
    for (int t = threadIdx.x; t < n; t += blockDim.x) lflat[o + t] = line_lf[off0 + t];
    if (line == 0 && threadIdx.x == 0) meta->counts[4] = sh_tot;
}

// concatenate per-line outputs in line order (:304-310,356,407)
__global__ void k_concat(const float4* __restrict__ cloud, const int* line_sharp, const int* line_lsharp,
                         const int* line_flat, const int* line_cnt, const float4* line_lf, int N_SCANS, ScanMeta* meta,
                         float4* sharp, int* sharp_idx, float4* lsharp, int* lsharp_idx, float4* flat, int* flat_idx,
                         float4* lflat, int* odom_nq) {
    const int line = blockIdx.x;
    // per kind: the counts of the lines before this one (o) and of all lines (tot), one line per thread
    __shared__ int sh_o[4], sh_tot[4];
    if (threadIdx.x < 4) { sh_o[threadIdx.x] = 0; sh_tot[threadIdx.x] = 0; }
    __syncthreads();
    {
        int v[4] = {0, 0, 0, 0};
        const int l = threadIdx.x;
        if (l < N_SCANS) { const int4 c = ((const int4*)line_cnt)[l]; v[0] = c.x; v[1] = c.y; v[2] = c.z; v[3] = c.w; }
        if (threadIdx.x < WAVE * ((N_SCANS + WAVE - 1) / WAVE)) {
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int a = wave_sum_i(l < line ? v[c] : 0), b = wave_sum_i(v[c]);
                if (lane_id() == 0) { if (a) atomicAdd(&sh_o[c], a); if (b) atomicAdd(&sh_tot[c], b); }
            }
        }
    }
    __syncthreads();
    int o[4], tot[4];
#pragma unroll
    for (int c = 0; c < 4; c++) { o[c] = sh_o[c]; tot[c] = sh_tot[c]; }
    const int* lc = line_cnt + line * 4;
    for (int t = threadIdx.x; t < lc[0]; t += blockDim.x) {
        int i = line_sharp[line * LINE_SHARP_CAP + t];
        sharp[o[0] + t] = cloud[i]; sharp_idx[o[0] + t] = i;
    }
    for (int t = threadIdx.x; t < lc[1]; t += blockDim.x) {
        int i = line_lsharp[line * LINE_LSHARP_CAP + t];
        lsharp[o[1] + t] = cloud[i]; lsharp_idx[o[1] + t] = i;
    }
    for (int t = threadIdx.x; t < lc[2]; t += blockDim.x) {
        int i = line_flat[line * LINE_FLAT_CAP + t];
        flat[o[2] + t] = cloud[i]; flat_idx[o[2] + t] = i;
    }
    if (line == 0 && threadIdx.x == 0) {
        meta->counts[0] = meta->cloud_size;
        meta->counts[1] = tot[0]; meta->counts[2] = tot[1]; meta->counts[3] = tot[2];
        odom_nq[0] = tot[0]; odom_nq[1] = tot[2];   // the odometry's query counts (sharp, flat), no host round trip
    }
}

__global__ void k_meta_init(ScanMeta* m, int n_in, int* odom_nq) {
    m->n_in = n_in;
    m->jstar = 0x7fffffff;
    m->cloud_size = 0;
    for (int i = 0; i < 5; i++) m->counts[i] = 0;
    odom_nq[0] = 0; odom_nq[1] = 0;
}

// ------------------------------------------------------------------------------------------
// side: the per-line VoxelGrid (k_line_vox, k_concat_lf) on stream2 behind an event (ev_lf marks it done)
void scan_registration_launch(Ctx& C, const float4* in, int n, bool side) {
    const aloam_params& P = C.P;
    const int N_SCANS = P.scan_line;
    hipStream_t st = C.stream;
    const int nb = (n + SB - 1) / SB;
    const float thres = (float)P.minimum_range;
    k_meta_init<<<1, 1, 0, st>>>(C.d_meta, n, C.d_odom_nq);
    if (n > 0) {
        k_filter_count<<<nb, SB, 0, st>>>(in, n, P.input_is_dense, thres, C.d_blk);
        k_scan_small<<<1, 1024, 0, st>>>(C.d_blk, nb, &C.d_meta->n_cl);
        k_filter_scatter<<<nb, SB, 0, st>>>(in, n, P.input_is_dense, thres, C.d_blk, C.d_cl);
        k_bucket_classify<<<nb, SB, 0, st>>>(C.d_cl, C.d_meta, N_SCANS, P.generic_min_elev_deg, P.generic_max_elev_deg,
                                             C.d_sid, C.d_ori, C.d_hist, nb, C.d_meta);
        k_bucket_scan<<<N_SCANS, BK_T, 0, st>>>(C.d_hist, nb, N_SCANS, C.d_meta, C.d_hoff);
        k_bucket_scatter<<<nb, SB, 0, st>>>(C.d_cl, C.d_meta, C.d_sid, C.d_ori, C.d_hoff, nb, N_SCANS, C.d_cloud);
        prof_phase(C, Ctx::PM_SCAN_PREP);
        k_curvature<<<nb, SB, 0, st>>>(C.d_cloud, C.d_meta, C.d_curv);
        prof_phase(C, Ctx::PM_SCAN_CURV);
        const size_t lds = line_lds_bytes();
        k_line_features<<<N_SCANS, LT, lds, st>>>(C.d_cloud, C.d_curv, C.d_meta, N_SCANS, C.d_scratch_xyz,
                                                  C.d_scratch_keys, C.d_scratch_i, C.d_line_sharp, C.d_line_lsharp,
                                                  C.d_line_flat, C.d_line_cnt, C.d_line_lf);
        k_concat<<<N_SCANS, 256, 0, st>>>(C.d_cloud, C.d_line_sharp, C.d_line_lsharp, C.d_line_flat, C.d_line_cnt,
                                          C.d_line_lf, N_SCANS, C.d_meta, C.d_sharp, C.d_sharp_idx, C.d_lsharp,
                                          C.d_lsharp_idx, C.d_flat, C.d_flat_idx, C.d_lflat, C.d_odom_nq);
        hipStream_t sv = st;
        if (side) {
            HIPCHK(hipEventRecord(C.ev_scan, st));
            HIPCHK(hipStreamWaitEvent(C.stream2, C.ev_scan, 0));
            sv = C.stream2;
        }
        static bool lv_attr = false;
        if (!lv_attr) {
            HIPCHK(hipFuncSetAttribute((const void*)k_line_vox, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lv_lds_bytes()));
            lv_attr = true;
        }
        k_line_vox<<<N_SCANS, LT, lv_lds_bytes(), sv>>>(C.d_cloud, C.d_meta, C.d_scratch_xyz, C.d_scratch_keys, C.d_scratch_i,
                                                      C.d_line_cnt, C.d_line_lf);
        k_concat_lf<<<N_SCANS, 256, 0, sv>>>(C.d_line_cnt, C.d_line_lf, N_SCANS, C.d_meta, C.d_lflat);
        if (side) HIPCHK(hipEventRecord(C.ev_lf, sv));
    } else {
        prof_phase(C, Ctx::PM_SCAN_PREP);
        prof_phase(C, Ctx::PM_SCAN_CURV);
        if (side) {
            // an empty sweep still orders stream2 after k_meta_init: the early mapping stacks
            // (do_odometry_issue) read this scan's counts and last clouds on stream2, and the
            // counts copy waits on ev_lf, which must mark this registration, not an older one
            HIPCHK(hipEventRecord(C.ev_scan, st));
            HIPCHK(hipStreamWaitEvent(C.stream2, C.ev_scan, 0));
            HIPCHK(hipEventRecord(C.ev_lf, C.stream2));
        }
    }
    HIPCHK(hipGetLastError());
}

// ps_serial_std_sort calls of this translation unit's kernels (aloam_serial_sort_fallbacks)
unsigned long long serial_sort_calls_scan() {
    unsigned long long v = 0;
    HIPCHK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ps_serial_calls), sizeof(v)));
    return v;
}

}  // namespace aloam
