// micro/heap_bench.hip — std::__partial_sort (make_heap + sort_heap) of one segment in LDS: one lane
// (pcl_sort.hpp ps_heap_sort) vs one whole wave (ws_heap_sort: six-level pops, or the child-flag pops
// fh_sort_heap_lds); outputs must be identical. Profiling aid.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include "../lidar-visual-odometry_amd/csrc/pcl_sort.hpp"
using namespace aloam;
constexpr int CAP = 8192;
template <int MODE>
__global__ void __launch_bounds__(64) k_heap(const unsigned long long* in, unsigned long long* out, int n, unsigned long long* cyc) {
    __shared__ unsigned long long E[CAP];
    __shared__ __attribute__((aligned(8))) unsigned char Fs[CAP + 1024];
    for (int t = threadIdx.x; t < n; t += 64) E[t] = in[t];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0) { if (threadIdx.x == 0) ps_heap_sort(E, E + n); }
    else if (MODE == 1) ws_heap_sort(E, 0, n, nullptr);   // E in LDS: the store-wait-free pops
    else ws_heap_sort(E, 0, n, nullptr, Fs);               // the pops on child flags (fh_sort_heap_lds)
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) *cyc = t1 - t0;
    for (int t = threadIdx.x; t < n; t += 64) out[t] = E[t];
}
// clock calibration: n dependent v_fma_f32 (about 4 cycles each for one wave) between two s_memtime reads
__global__ void __launch_bounds__(64) k_calib(float* out, int n, unsigned long long* cyc) {
    float a = out[threadIdx.x], b = 1.0000001f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) a = fmaf(a, b, 0.5f);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
// instruction cost model (one wave alone on the chip), all between two s_memtime reads; n = iterations
//   mode 4: 64 dependent v_fma_f32 per loop iteration (unrolled)
//   mode 5: 64 dependent s_add_u32 per iteration (inline asm, not folded)
//   mode 6: 16 dependent v_readlane -> lane index -> v_readlane per iteration
//   mode 7: 16 dependent ds_read_b32 (pointer chasing in LDS) per iteration
//   mode 8: empty loop (the back-edge: s_add, s_cmp, taken s_cbranch)
template <int M>
__global__ void __launch_bounds__(64) k_cost(float* out, int n, unsigned long long* cyc) {
    __shared__ int chase[64];
    chase[threadIdx.x] = (threadIdx.x * 5 + 1) & 63;
    __syncthreads();
    float a = out[threadIdx.x];
    int vi = (int)threadIdx.x, p = (int)threadIdx.x;
    unsigned sa = (unsigned)n;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        if (M == 4) {
#pragma unroll
            for (int k = 0; k < 64; k++) a = fmaf(a, 1.0000001f, 0.5f);
        } else if (M == 5) {
#pragma unroll
            for (int k = 0; k < 64; k++) asm volatile("s_add_u32 %0, %0, 3" : "+s"(sa));
        } else if (M == 6) {
            int l = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) l = __builtin_amdgcn_readlane(vi, l) ^ 1;
            vi += l;
        } else if (M == 7) {
#pragma unroll
            for (int k = 0; k < 16; k++) p = ((volatile int*)chase)[p];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + (float)vi + (float)p + (float)sa;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
extern "C" int heap_run(const unsigned long long* h_in, unsigned long long* h_out, int n, int mode, unsigned long long* cycles,
                        float* ms) {
    unsigned long long *d_in, *d_out, *d_c;
    hipMalloc(&d_in, 8 * n + 256); hipMalloc(&d_out, 8 * n + 256); hipMalloc(&d_c, 8);
    if (mode < 3) hipMemcpy(d_in, h_in, 8 * n, hipMemcpyHostToDevice);   // mode 3 (calibration): n = chain length
    else hipMemset(d_out, 0, 256);
    double best = 1e30;
    for (int r = 0; r < 3; r++) {
        hipDeviceSynchronize();
        const auto t0 = std::chrono::steady_clock::now();
        if (mode == 0) k_heap<0><<<1, 64>>>(d_in, d_out, n, d_c);
        else if (mode == 1) k_heap<1><<<1, 64>>>(d_in, d_out, n, d_c);
        else if (mode == 2) k_heap<2><<<1, 64>>>(d_in, d_out, n, d_c);
        else if (mode == 3) k_calib<<<1, 64>>>((float*)d_out, n, d_c);
        else if (mode == 4) k_cost<4><<<1, 64>>>((float*)d_out, n, d_c);
        else if (mode == 5) k_cost<5><<<1, 64>>>((float*)d_out, n, d_c);
        else if (mode == 6) k_cost<6><<<1, 64>>>((float*)d_out, n, d_c);
        else if (mode == 7) k_cost<7><<<1, 64>>>((float*)d_out, n, d_c);
        else k_cost<8><<<1, 64>>>((float*)d_out, n, d_c);
        hipDeviceSynchronize();
        best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    *ms = (float)best;   // host wall time of one launch (includes ~10 us of launch overhead)
    if (mode < 3) hipMemcpy(h_out, d_out, 8 * n, hipMemcpyDeviceToHost);
    hipMemcpy(cycles, d_c, 8, hipMemcpyDeviceToHost);
    const int rc = (int)hipGetLastError();
    hipFree(d_in); hipFree(d_out); hipFree(d_c);
    return rc;
}
