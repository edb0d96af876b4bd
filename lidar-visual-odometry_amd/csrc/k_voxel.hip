// k_voxel.hip — pcl::VoxelGrid<PointXYZI> (PCL 1.8.0 voxel_grid.hpp applyFilter) on gfx950.
//
// Semantics kept: bbox -> leaf index floor(p * (1/leaf)) - min_b (fp32), the int64 overflow
// pass-through, output in ascending leaf index, centroid of x,y,z,intensity summed in fp32 and
// divided by the count. One documented difference: PCL orders the points of a leaf by an unstable
// std::sort, we sum them in input order (a stable sort); the oracle runs both orders
// (oracle_set_voxel_order) and the tests bound the difference.
//
//   voxel_grid_sorted  one cloud, device-wide stable radix sort (rocPRIM) — mapping's corner /
//                      surf stacks (laserMapping.cpp:542-550) and aloam_voxel_grid()
//   segment_voxel      one workgroup per segment (map cube), keys bitonic-sorted in LDS —
//                      the per-cube filter of laserMapping.cpp:788-801
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "aloam_device.hpp"
#include "aloam_internal.hpp"

namespace aloam {

constexpr int VB = 256;

struct VoxHdr { unsigned bb[6]; int nrun; int pad; };

__global__ void k_vox_init(VoxHdr* h) {
    if (threadIdx.x < 6) h->bb[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    if (threadIdx.x == 0) h->nrun = 0;
}
__global__ void k_vox_bbox(const float4* __restrict__ pts, const int* d_n, VoxHdr* h) {
    __shared__ unsigned sh[6];
    if (threadIdx.x < 6) sh[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    const int n = *d_n;
    unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    for (int i = blockIdx.x * VB + threadIdx.x; i < n; i += gridDim.x * VB) {
        float4 p = pts[i];
        unsigned v[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
        for (int a = 0; a < 3; a++) { mn[a] = min(mn[a], v[a]); mx[a] = max(mx[a], v[a]); }
    }
    for (int a = 0; a < 3; a++) {
        unsigned long long lo = wave_min_u64(mn[a]), hi = wave_max_u64(mx[a]);
        if (lane_id() == 0) { atomicMin(&sh[a], (unsigned)lo); atomicMax(&sh[3 + a], (unsigned)hi); }
    }
    __syncthreads();
    if (threadIdx.x < 3) { atomicMin(&h->bb[threadIdx.x], sh[threadIdx.x]); atomicMax(&h->bb[3 + threadIdx.x], sh[3 + threadIdx.x]); }
}
__global__ void k_vox_keys(const float4* __restrict__ pts, const int* d_n, int cap, const VoxHdr* h, float leaf,
                           unsigned* __restrict__ keys, int* __restrict__ vals) {
    const int n = *d_n;
    bool ovf; int minb[3], mul1, mul2;
    voxel_params(h->bb, leaf, &ovf, minb, &mul1, &mul2);
    const float inv = 1.0f / leaf;
    for (int i = blockIdx.x * VB + threadIdx.x; i < cap; i += gridDim.x * VB) {
        unsigned k = 0xffffffffu;
        if (i < n) k = ovf ? (unsigned)i : voxel_index(pts[i], inv, minb, mul1, mul2);
        keys[i] = k;
        vals[i] = i;
    }
}
// run heads of the sorted keys -> blk counts
__global__ void k_vox_flags(const unsigned* __restrict__ keys, const int* d_n, int cap, int* blk) {
    __shared__ int sh[VB / WAVE];
    const int n = *d_n;
    const int i = blockIdx.x * VB + threadIdx.x;
    int f = i < n && (i == 0 || keys[i] != keys[i - 1]);
    int s = wave_sum_i(f);
    if (lane_id() == 0) sh[threadIdx.x / WAVE] = s;
    __syncthreads();
    if (threadIdx.x == 0) { int t = 0; for (int w = 0; w < VB / WAVE; w++) t += sh[w]; blk[blockIdx.x] = t; }
}
__global__ void k_vox_heads(const unsigned* __restrict__ keys, const int* d_n, const int* blk, int* heads) {
    __shared__ int sh[VB / WAVE];
    const int n = *d_n;
    const int i = blockIdx.x * VB + threadIdx.x;
    int f = i < n && (i == 0 || keys[i] != keys[i - 1]);
    unsigned long long m = __ballot(f);
    if (lane_id() == 0) sh[threadIdx.x / WAVE] = __popcll(m);
    __syncthreads();
    int before = blk[blockIdx.x];
    for (int w = 0; w < threadIdx.x / WAVE; w++) before += sh[w];
    if (f) heads[before + __popcll(m & lanemask_lt64())] = i;
}
__global__ void k_vox_centroids(const float4* __restrict__ pts, const int* d_n, const int* nrun_p, const int* __restrict__ heads,
                                const int* __restrict__ vals, float4* __restrict__ out, int* d_nout) {
    const int n = *d_n, nrun = *nrun_p;
    const int r = blockIdx.x * VB + threadIdx.x;
    if (r == 0) *d_nout = nrun;
    if (r >= nrun) return;
    const int h0 = heads[r], h1 = r + 1 < nrun ? heads[r + 1] : n;
    // sequential fp32 sum in sorted order (PCL's accumulation order), 8 loads in flight per step
    float4 c = pts[vals[h0]];
    for (int t0 = h0 + 1; t0 < h1; t0 += 8) {
        int vi[8];
        float4 p[8];
#pragma unroll
        for (int u = 0; u < 8; u++) vi[u] = t0 + u < h1 ? vals[t0 + u] : -1;
#pragma unroll
        for (int u = 0; u < 8; u++) p[u] = load_or(pts, vi[u], vi[u] >= 0, make_float4(0, 0, 0, 0));
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (vi[u] >= 0) { c.x += p[u].x; c.y += p[u].y; c.z += p[u].z; c.w += p[u].w; }
    }
    const float cnt = (float)(h1 - h0);
    out[r] = make_float4(c.x / cnt, c.y / cnt, c.z / cnt, c.w / cnt);
}

__global__ void k_scan_small_v(int* a, int nb, int* total) {
    block_scan_array(a, nb, total);
}

unsigned* voxel_hdr(Ctx& C, int lane) {   // the lane's VoxHdr lives behind its value buffer
    return ((VoxHdr*)(C.ks[lane].vvals2 + C.cap_voxel))->bb;
}

void voxel_grid_sorted(Ctx& C, const float4* pts, const int* d_n, int cap_n, float leaf, float4* out, int* d_nout, int lane,
                       bool hdr_armed) {
    voxel_grid_sorted_on(C, lane ? C.stream2 : C.stream, C.ks[lane], pts, d_n, cap_n, leaf, out, d_nout, hdr_armed);
}

void voxel_grid_sorted_on(Ctx& C, hipStream_t st, KindScratch& K, const float4* pts, const int* d_n, int cap_n, float leaf,
                          float4* out, int* d_nout, bool hdr_armed) {
    if (cap_n <= 0) { HIPCHK(hipMemsetAsync(d_nout, 0, sizeof(int), st)); return; }
    if (cap_n > C.cap_voxel) throw ApiError{ALOAM_E_CAPACITY, "voxel grid capacity exceeded"};
    VoxHdr* h = (VoxHdr*)(K.vvals2 + C.cap_voxel);   // header lives behind the value buffer
    unsigned* k1 = (unsigned*)K.vkeys;
    unsigned* k2 = (unsigned*)K.vkeys2;
    int* blk = K.blk;
    int* heads = (int*)(K.vkeys + C.cap_voxel);      // second half of the key scratch
    const int nb = (cap_n + VB - 1) / VB;
    const int nbr = std::min(nb, 1024);
    if (!hdr_armed) k_vox_init<<<1, 64, 0, st>>>(h);   // else armed by an earlier kernel of the stream (k_map_prepare)
    k_vox_bbox<<<nbr, VB, 0, st>>>(pts, d_n, h);
    k_vox_keys<<<nbr, VB, 0, st>>>(pts, d_n, cap_n, h, leaf, k1, K.vvals);
    size_t bytes = C.sort_tmp_bytes;
    HIPCHK(rocprim::radix_sort_pairs(K.sort_tmp, bytes, k1, k2, K.vvals, K.vvals2, (unsigned)cap_n, 0, 32, st));
    k_vox_flags<<<nb, VB, 0, st>>>(k2, d_n, cap_n, blk);
    k_scan_small_v<<<1, 1024, 0, st>>>(blk, nb, &h->nrun);
    k_vox_heads<<<nb, VB, 0, st>>>(k2, d_n, blk, heads);
    k_vox_centroids<<<nb, VB, 0, st>>>(pts, d_n, &h->nrun, heads, K.vvals2, out, d_nout);
    HIPCHK(hipGetLastError());
}

size_t voxel_sort_tmp_bytes(int cap) {
    size_t bytes = 0;
    unsigned* k = nullptr; int* v = nullptr;
    rocprim::radix_sort_pairs(nullptr, bytes, k, k, v, v, (unsigned)cap, 0, 32, (hipStream_t)0);
    return bytes;
}

// stable sort of (unsigned key, int value) pairs — used to order inserted map points by cube
void stable_sort_pairs(Ctx& C, unsigned* kin, unsigned* kout, int* vin, int* vout, int n, int end_bit, int lane) {
    size_t bytes = C.sort_tmp_bytes;
    HIPCHK(rocprim::radix_sort_pairs(C.ks[lane].sort_tmp, bytes, kin, kout, vin, vout, (unsigned)n, 0, end_bit,
                                     lane ? C.stream2 : C.stream));
}

// ------------------------------------------------------------------------------------------
// one workgroup per segment (map cube). Segment c = [off[c], off[c+1]) of pts.
constexpr int SV = 1024;
constexpr int SEG_LDS_KEYS = 16384;

__device__ inline void bitonic_u64(unsigned long long* k, int n2) {
    for (int size = 2; size <= n2; size <<= 1)
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

__global__ void __launch_bounds__(SV) k_segment_voxel(const float4* __restrict__ pts, const int* __restrict__ off,
                                                     const int* __restrict__ seg_list, const int* nseg_p, float leaf,
                                                     float4* __restrict__ out, int* seg_nout, unsigned long long* gkeys) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    struct SegShared { unsigned bb[6]; int nrun; int wsum[SV / WAVE]; };
    SegShared& SH = *(SegShared*)smem_raw;
    unsigned long long* skeys = (unsigned long long*)(smem_raw + 256);
    const int b = blockIdx.x;
    if (b >= *nseg_p) return;
    const int c = seg_list[b];
    const int o0 = off[c], n = off[c + 1] - o0;
    if (n == 0) { if (threadIdx.x == 0) seg_nout[c] = 0; return; }
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    unsigned long long* gseg = gkeys + 4 * (size_t)o0;   // 4 slots per point of global scratch
    unsigned long long* keys = n2 <= SEG_LDS_KEYS ? skeys : gseg;
    if (threadIdx.x < 6) SH.bb[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    if (threadIdx.x == 0) SH.nrun = 0;
    __syncthreads();
    unsigned mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
    for (int t = threadIdx.x; t < n; t += SV) {
        float4 p = pts[o0 + t];
        unsigned v[3] = {f2ord(p.x), f2ord(p.y), f2ord(p.z)};
        for (int a = 0; a < 3; a++) { mn[a] = min(mn[a], v[a]); mx[a] = max(mx[a], v[a]); }
    }
    for (int a = 0; a < 3; a++) { atomicMin(&SH.bb[a], mn[a]); atomicMax(&SH.bb[3 + a], mx[a]); }
    __syncthreads();
    bool ovf; int minb[3], mul1, mul2;
    voxel_params(SH.bb, leaf, &ovf, minb, &mul1, &mul2);
    const float inv = 1.0f / leaf;
    for (int t = threadIdx.x; t < n2; t += SV) {
        unsigned long long k = ~0ull;
        if (t < n) {
            unsigned idx = ovf ? (unsigned)t : voxel_index(pts[o0 + t], inv, minb, mul1, mul2);
            k = ((unsigned long long)idx << 32) | (unsigned)t;
        }
        keys[t] = k;
    }
    __syncthreads();
    bitonic_u64(keys, n2);
    // run heads go behind the keys (LDS tail when it fits, else the segment's global scratch)
    const int lanei = lane_id(), wi = threadIdx.x / WAVE;
    int* hbuf = (n2 <= SEG_LDS_KEYS / 2) ? (int*)(skeys + n2) : (int*)(gseg + n2);
    for (int base = 0; base < n; base += SV) {
        const int t = base + threadIdx.x;
        const int flag = t < n && (t == 0 || (keys[t] >> 32) != (keys[t - 1] >> 32));
        const unsigned long long mk = __ballot(flag);
        if (lanei == 0) SH.wsum[wi] = __popcll(mk);
        __syncthreads();
        int before = SH.nrun;
        for (int ww = 0; ww < wi; ww++) before += SH.wsum[ww];
        if (flag) hbuf[before + __popcll(mk & lanemask_lt64())] = t;
        __syncthreads();
        if (threadIdx.x == 0) { int tt = 0; for (int ww = 0; ww < SV / WAVE; ww++) tt += SH.wsum[ww]; SH.nrun += tt; }
        __syncthreads();
    }
    const int nrun = SH.nrun;
    for (int r = threadIdx.x; r < nrun; r += SV) {
        const int h0 = hbuf[r], h1 = r + 1 < nrun ? hbuf[r + 1] : n;
        float4 cc = pts[o0 + (int)(keys[h0] & 0xffffffffu)];
        for (int t = h0 + 1; t < h1; t++) {
            float4 p = pts[o0 + (int)(keys[t] & 0xffffffffu)];
            cc.x += p.x; cc.y += p.y; cc.z += p.z; cc.w += p.w;
        }
        const float cnt = (float)(h1 - h0);
        out[o0 + r] = make_float4(cc.x / cnt, cc.y / cnt, cc.z / cnt, cc.w / cnt);
    }
    if (threadIdx.x == 0) seg_nout[c] = nrun;
}

void segment_voxel_launch(Ctx& C, const float4* pts, const int* off, const int* seg_list, const int* nseg_p, int max_seg,
                          float leaf, float4* out, int* seg_nout, unsigned long long* gkeys) {
    const size_t lds = 256 + (size_t)SEG_LDS_KEYS * 8;
    k_segment_voxel<<<max_seg, SV, lds, C.stream>>>(pts, off, seg_list, nseg_p, leaf, out, seg_nout, gkeys);
    HIPCHK(hipGetLastError());
}

}  // namespace aloam
