// k_voxel.hip — pcl::VoxelGrid<PointXYZI> (PCL 1.8.0 voxel_grid.hpp applyFilter) on gfx950, one
// workgroup per cloud, one launch per pair of clouds.
//
// Semantics kept: bbox -> leaf index floor(p * (1/leaf)) - min_b (fp32, (k, j, i)-linear), the int64
// leaf-count overflow pass-through (output = input), output in ascending leaf index, every leaf's
// x, y, z, intensity summed in fp32 from zero (CentroidPoint's accumulators) in the order PCL's
// std::sort of the (leaf, index) pairs leaves them (pcl_sort.hpp), divided by the count.
// Call sites: the mapping stacks (src/laserMapping.cpp:542-550: less-sharp at 0.4 m, less-flat at
// 0.8 m) and aloam_voxel_grid(). The per-line filter of scanRegistration (:401-405) runs inside
// k_line_features and the per-cube map filter (:788-801) inside k_rb_cubevox, both on the same sort.
#include <cstring>

#include "aloam_device.hpp"
#include "aloam_internal.hpp"
#ifdef ALOAM_PS_TIMING           // profiling builds only: per-level stamps of the sort of workgroup 0
__device__ unsigned long long g_ps_ts[64][6];
__device__ int g_ps_nseg[64];
#define PS_TS(level, k) do { if (threadIdx.x == 0 && blockIdx.x == 1 && (level) < 64) { g_ps_ts[level][k] = wall_clock64(); if ((k) == 0) g_ps_nseg[level] = hdr[(level) == 60 ? 2 : 0]; } } while (0)
// k_vox_pcl phases per job (blockIdx.x): start, bbox, keys, sort / split, reduce, and n in slot 7
__device__ unsigned long long g_vx_ts[2][8];
#define VX_TS(k) do { if (threadIdx.x == 0) g_vx_ts[blockIdx.x & 1][k] = wall_clock64(); } while (0)
extern "C" int aloam_dbg_vx_ts(unsigned long long* out) { return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vx_ts), sizeof(g_vx_ts)); }
__device__ unsigned long long g_ps_w[16][8];
#define PS_CLK() ((unsigned long long)__builtin_amdgcn_s_memtime())
#define PS_WSTAT(slot, v) do { if (blockIdx.x == 0) { auto& w_ = g_ps_w[threadIdx.x / 64][slot]; w_ = w_ + (unsigned long long)(v); } } while (0)
// per-wave counters of workgroup 0's wave phase (cycles waiting, partitioning, #partitions, elements
// partitioned, cycles in leaves, #leaves), accumulated since the last call; read and cleared
extern "C" int aloam_dbg_ps_w(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ps_w), sizeof(g_ps_w)) != hipSuccess) return -1;
    static unsigned long long zero[16][8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ps_w), zero, sizeof(zero));
}
extern "C" int aloam_dbg_ps_ts(unsigned long long* out, int* nseg) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ps_ts), sizeof(g_ps_ts)) != hipSuccess) return -1;
    return (int)hipMemcpyFromSymbol(nseg, HIP_SYMBOL(g_ps_nseg), sizeof(g_ps_nseg));
}
#else
#define VX_TS(k) do { } while (0)
#endif
#include "ls_sort.hpp"

namespace aloam {

constexpr int VX_T = 1024;
constexpr int VX_CPW = 10;                                  // ls_sort: 64-position chunks per wave
constexpr int VX_LDS_N = VX_T * VX_CPW;                     // clouds up to this size are sorted in LDS
constexpr int VX_NMAX = VX_T * PS_MAX_CHUNK;                // parallel replay up to this size (beyond: one thread)
constexpr size_t VX_HDR = 64;
constexpr size_t VX_LDS = VX_HDR + 8 * (size_t)VX_LDS_N + ls_global_scratch_bytes(VX_T, VX_LDS_N);
static_assert(VX_LDS <= 160 * 1024, "LDS");

struct VoxJob {
    const float4* pts; const int* d_n; int cap; float leaf;
    float4* out; int* d_nout;
    unsigned long long* gE;      // global scratch (cap_voxel keys) for clouds above VX_LDS_N
    int* gseg;                   // their segment list (LS_SEGL ints; count 0: the cloud is done)
};
struct VoxJobs { VoxJob j[2]; };

// Clouds above VX_LDS_N are sorted by several workgroups: k_vox_pcl splits them into segments of at most
// g_vox_seg elements, k_vox_seg sorts the segments in parallel (VX_SEGW workgroups per cloud), k_vox_reduce
// sums the leaves.
constexpr int VX_SEGW = 16;
// tuning knob: split segments of at most this many elements. Round 5, C3 pipeline, 20 steps on one box: with the
// split's levels at ~55 us, 10240 won (846-850 vs 835-837 scans/s for 4096); with the coalesced split (~30 us a
// level) 4096 wins (891-894 vs 880-885, profiles/r05_tune_ab.txt): more, shorter segment sorts in parallel
static const int g_vox_seg = getenv("ALOAM_VOX_SEG") ? std::max(2048, std::min(VX_LDS_N, atoi(getenv("ALOAM_VOX_SEG")))) : 4096;
// tuning knob: clouds up to this size are sorted whole by their own workgroup, larger ones split
static const int g_vox_fit = getenv("ALOAM_VOX_FIT") ? std::max(256, std::min(VX_LDS_N, atoi(getenv("ALOAM_VOX_FIT")))) : VX_LDS_N;
static_assert(ls_split_scratch_bytes(VX_T, VX_LDS_N) <= ls_global_scratch_bytes(VX_T, VX_LDS_N), "split scratch");

// runs of equal leaves in sorted E -> centroids in leaf order; each run summed in sorted order by its head
__device__ void vox_reduce(const VoxJob& J, int n, const unsigned long long* E, int* sc) {
    const int tid = threadIdx.x;
    const int C = (n + VX_T - 1) / VX_T;
    const int p0 = min(n, tid * C), p1 = min(n, p0 + C);
    int nh = 0;
    for (int p = p0; p < p1; p++) nh += (p == 0 || ps_key(E[p]) != ps_key(E[p - 1]));
    int run, dummy = 0, tot, td;
    run = nh;
    ps_exscan2<VX_T>(run, dummy, sc + 16, tot, td);
    for (int p = p0; p < p1; p++) {
        const unsigned k = ps_key(E[p]);
        if (!(p == 0 || k != ps_key(E[p - 1]))) continue;
        int cnt;
        const float4 c = ps_run_sum(E, n, p, k, [&](int i) { return J.pts[i]; }, cnt);
        const float fc = (float)cnt;
        J.out[run] = make_float4(c.x / fc, c.y / fc, c.z / fc, c.w / fc);
        run++;
    }
    if (tid == 0) *J.d_nout = tot;
}

__global__ void __launch_bounds__(VX_T) k_vox_pcl(VoxJobs P, int seg_limit, int fit) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const VoxJob& J = P.j[blockIdx.x];
    unsigned* bb = (unsigned*)smem;
    unsigned long long* EL = (unsigned long long*)(smem + VX_HDR);   // keys, or the staging buffer
    int* sc = (int*)(EL + VX_LDS_N);
    const int tid = threadIdx.x;
    // a hinted launch never reads past its launch size (the exact-size redo replaces the result)
    const int n = min(*J.d_n, J.cap);
    VX_TS(0);
#ifdef ALOAM_PS_TIMING
    if (tid == 0) g_vx_ts[blockIdx.x & 1][7] = (unsigned long long)n;
#endif
    if (n <= fit || n > VX_NMAX) { if (tid == 0) J.gseg[0] = 0; }   // done here (the others: split)
    if (n <= 0) { if (tid == 0) *J.d_nout = 0; return; }
    if (tid < 6) bb[tid] = tid < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    // the cloud's points, 8 per thread and pass with their loads in flight together
    auto pass = [&](auto f) {
        for (int t0 = tid; t0 < n; t0 += 8 * VX_T) {
            float4 q[8];
#pragma unroll
            for (int u = 0; u < 8; u++) q[u] = t0 + u * VX_T < n ? J.pts[t0 + u * VX_T] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (t0 + u * VX_T < n) f(t0 + u * VX_T, q[u]);
        }
    };
    {
        unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
        pass([&](int, float4 p) {
            const unsigned v[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
#pragma unroll
            for (int d = 0; d < 3; d++) { mn[d] = min(mn[d], v[d]); mx[d] = max(mx[d], v[d]); }
        });
#pragma unroll
        for (int d = 0; d < 3; d++) {
            const unsigned long long lo = wave_min_u64(mn[d]), hi = wave_max_u64(mx[d]);
            if (lane_id() == 0) { atomicMin(&bb[d], (unsigned)lo); atomicMax(&bb[3 + d], (unsigned)hi); }
        }
    }
    __syncthreads();
    VX_TS(1);
    bool ovf;
    int minb[3], mul1, mul2;
    voxel_params(bb, J.leaf, &ovf, minb, &mul1, &mul2);
    if (ovf) {                               // PCL: leaf count overflows int32 -> output = input
        for (int t = tid; t < n; t += VX_T) J.out[t] = J.pts[t];
        if (tid == 0) { *J.d_nout = n; J.gseg[0] = 0; }
        return;
    }
    const float inv = 1.0f / J.leaf;
    if (n <= fit) {
        pass([&](int t, float4 p) { EL[t] = ((unsigned long long)voxel_index(p, inv, minb, mul1, mul2) << 32) | (unsigned)t; });
        lds_barrier();
        VX_TS(2);
        ls_sort<VX_T, VX_CPW>(EL, n, 2 * (31 - __builtin_clz((unsigned)n)), (unsigned char*)sc, VX_LDS_N);
        VX_TS(3);
        vox_reduce(J, n, EL, sc);
        VX_TS(4);
        return;
    }
    unsigned long long* E = J.gE;
    pass([&](int t, float4 p) { E[t] = ((unsigned long long)voxel_index(p, inv, minb, mul1, mul2) << 32) | (unsigned)t; });
    __syncthreads();
    VX_TS(2);
    if (n <= VX_NMAX) {
        ls_split_to_list<VX_T>(E, n, seg_limit, J.gseg, (unsigned char*)sc);   // -> k_vox_seg, k_vox_reduce
        VX_TS(3);
        return;
    }
    if (tid == 0) ps_serial_std_sort(E, n);   // beyond the parallel replay's reach: one thread (rare)
    __syncthreads();
    vox_reduce(J, n, E, sc);
}

__global__ void __launch_bounds__(VX_T) k_vox_seg(VoxJobs P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const VoxJob& J = P.j[blockIdx.y];
    if (J.gseg[0] == 0) return;
    unsigned long long* EL = (unsigned long long*)(smem + VX_HDR);
    ls_sort_list<VX_T, VX_CPW>(J.gE, J.gseg, blockIdx.x, gridDim.x, EL, VX_LDS_N, (unsigned char*)(EL + VX_LDS_N));
}
// segments of <= VQ_CAP elements (g_vox_seg <= VQ_CAP): 256 threads, ~28 KB of LDS, several workgroups per CU
// (k_map.hip's k_rb_cubeseg_s, same reasoning)
constexpr int VQ_T = 256, VQ_CPW = 8, VQ_CAP = VQ_T * VQ_CPW, VQ_SEGW = 32;
constexpr size_t VQ_LDS = 8 * (size_t)VQ_CAP + ls_scratch_bytes(VQ_T, VQ_CAP);
__global__ void __launch_bounds__(VQ_T) k_vox_seg_s(VoxJobs P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const VoxJob& J = P.j[blockIdx.y];
    if (J.gseg[0] == 0) return;
    unsigned long long* EL = (unsigned long long*)smem;
    ls_sort_list<VQ_T, VQ_CPW>(J.gE, J.gseg, blockIdx.x, gridDim.x, EL, VQ_CAP, (unsigned char*)(EL + VQ_CAP));
}
static void vox_seg_launch(const VoxJobs& P, int nk, hipStream_t st) {
    if (g_vox_seg <= VQ_CAP) k_vox_seg_s<<<dim3(VQ_SEGW, nk), VQ_T, VQ_LDS, st>>>(P);
    else k_vox_seg<<<dim3(VX_SEGW, nk), VX_T, VX_LDS, st>>>(P);
}

// the leaves of a split cloud, VX_REDW workgroups per cloud: workgroup w owns sorted positions [w R, (w+1) R)
// and counts the run heads before them itself (a pass over the keys) for its output offset
constexpr int VX_REDW = 16;
__global__ void __launch_bounds__(VX_T) k_vox_reduce(VoxJobs P) {
    __shared__ int sc[16 + 2 * (VX_T / WAVE) + 2];
    const VoxJob& J = P.j[blockIdx.y];
    if (J.gseg[0] == 0) return;
    const int n = min(*J.d_n, J.cap), tid = threadIdx.x;
    const int R = (n + gridDim.x - 1) / gridDim.x;
    const int q0 = min(n, (int)blockIdx.x * R), q1 = min(n, q0 + R);
    const unsigned long long* E = J.gE;
    int before = 0;                              // (8 positions per thread in flight)
    for (int p0 = tid; p0 < q0; p0 += 8 * VX_T) {
        unsigned k[8], kp[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int p = p0 + u * VX_T;
            k[u] = p < q0 ? ps_keyat(E, p) : 0u;
            kp[u] = p < q0 && p > 0 ? ps_keyat(E, p - 1) : ~k[u];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) before += p0 + u * VX_T < q0 && k[u] != kp[u];
    }
    const int C = (q1 - q0 + VX_T - 1) / VX_T;
    const int p0 = min(q1, q0 + tid * C), p1 = min(q1, p0 + C);
    int nh = 0;
    for (int p = p0; p < p1; p++) nh += (p == 0 || ps_key(E[p]) != ps_key(E[p - 1]));
    int run = nh, bsum = before, tot, tb;
    ps_exscan2<VX_T>(run, bsum, sc + 16, tot, tb);
    run += tb;                                   // heads before this workgroup's range
    for (int p = p0; p < p1; p++) {
        const unsigned k = ps_key(E[p]);
        if (!(p == 0 || k != ps_key(E[p - 1]))) continue;
        int cnt;
        const float4 c = ps_run_sum(E, n, p, k, [&](int i) { return J.pts[i]; }, cnt);
        const float fc = (float)cnt;
        J.out[run] = make_float4(c.x / fc, c.y / fc, c.z / fc, c.w / fc);
        run++;
    }
    if (blockIdx.x == gridDim.x - 1 && tid == 0) *J.d_nout = tb + tot;
}

static void vox_attr() {
    static bool done = false;
    if (!done) {
        HIPCHK(hipFuncSetAttribute((const void*)k_vox_pcl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)VX_LDS));
        HIPCHK(hipFuncSetAttribute((const void*)k_vox_seg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)VX_LDS));
        HIPCHK(hipFuncSetAttribute((const void*)k_vox_seg_s, hipFuncAttributeMaxDynamicSharedMemorySize, (int)VQ_LDS));
        done = true;
    }
}

// global scratch per cloud: cap_voxel u64 keys
static VoxJob vox_job(Ctx& C, KindScratch& K, int which, const float4* pts, const int* d_n, int cap, float leaf, float4* out,
                      int* d_nout) {
    VoxJob j;
    j.pts = pts; j.d_n = d_n; j.cap = cap; j.leaf = leaf; j.out = out; j.d_nout = d_nout;
    j.gE = which == 0 ? K.vkeys : K.vkeys2;
    j.gseg = which == 0 ? K.vvals : K.vvals2;
    return j;
}

void voxel_grid_pair_on(Ctx& C, hipStream_t st, KindScratch& K, const float4* ptsA, const int* d_nA, int capA, float leafA,
                        float4* outA, int* d_noutA, const float4* ptsB, const int* d_nB, int capB, float leafB, float4* outB,
                        int* d_noutB) {
    if (std::max(capA, capB) > C.cap_voxel) throw ApiError{ALOAM_E_CAPACITY, "voxel grid capacity exceeded"};
    vox_attr();
    VoxJobs P;
    P.j[0] = vox_job(C, K, 0, ptsA, d_nA, std::max(capA, 0), leafA, outA, d_noutA);
    P.j[1] = vox_job(C, K, 1, ptsB, d_nB, std::max(capB, 0), leafB, outB, d_noutB);
    k_vox_pcl<<<2, VX_T, VX_LDS, st>>>(P, g_vox_seg, g_vox_fit);
    if (std::max(capA, capB) > g_vox_fit) {
        vox_seg_launch(P, 2, st);
        k_vox_reduce<<<dim3(VX_REDW, 2), VX_T, 0, st>>>(P);
    }
    HIPCHK(hipGetLastError());
}

void voxel_grid_sorted_on(Ctx& C, hipStream_t st, KindScratch& K, const float4* pts, const int* d_n, int cap_n, float leaf,
                          float4* out, int* d_nout) {
    if (cap_n > C.cap_voxel) throw ApiError{ALOAM_E_CAPACITY, "voxel grid capacity exceeded"};
    vox_attr();
    VoxJobs P;
    P.j[0] = vox_job(C, K, 0, pts, d_n, std::max(cap_n, 0), leaf, out, d_nout);
    P.j[1] = P.j[0];
    k_vox_pcl<<<1, VX_T, VX_LDS, st>>>(P, g_vox_seg, g_vox_fit);
    if (cap_n > g_vox_fit) {
        vox_seg_launch(P, 1, st);
        k_vox_reduce<<<dim3(VX_REDW, 1), VX_T, 0, st>>>(P);
    }
    HIPCHK(hipGetLastError());
}

void voxel_grid_sorted(Ctx& C, const float4* pts, const int* d_n, int cap_n, float leaf, float4* out, int* d_nout, int lane) {
    voxel_grid_sorted_on(C, lane ? C.stream2 : C.stream, C.ks[lane], pts, d_n, cap_n, leaf, out, d_nout);
}

// ps_serial_std_sort calls of this translation unit's kernels (aloam_serial_sort_fallbacks)
unsigned long long serial_sort_calls_voxel() {
    unsigned long long v = 0;
    HIPCHK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ps_serial_calls), sizeof(v)));
    return v;
}

}  // namespace aloam
