// micro/split_bench.hip — the workgroup split alone (ls_split_to_list: pcl_sort.hpp ps_wg_split on global
// memory, one workgroup of 1024 threads) on one key array: kernel time, per-level phase cycles (thread 0,
// s_memtime), the split array and its segment list (compared across builds by split_bench.py). Profiling aid.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_sp_ts[64][6];
__device__ int g_sp_nseg[64];
#define PS_TS(level, k) do { if (threadIdx.x == 0 && (level) < 64) { g_sp_ts[level][k] = __builtin_amdgcn_s_memtime(); \
    if ((k) == 0) g_sp_nseg[level] = hdr[0]; } } while (0)
#include "../lidar-visual-odometry_amd/csrc/ls_sort.hpp"
using namespace aloam;
constexpr int NT = 1024, CAP = NT * 10;
__global__ void __launch_bounds__(NT) k_split(const unsigned long long* in, unsigned long long* E, int n, int limit, int* gseg,
                                              unsigned long long* cyc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    for (int t = threadIdx.x; t < n; t += NT) E[t] = in[t];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    ls_split_to_list<NT>(E, n, limit, gseg, smem);
    __syncthreads();
    if (threadIdx.x == 0) *cyc = __builtin_amdgcn_s_memtime() - t0;
}
extern "C" int split_stamps(unsigned long long* ts, int* nseg) {
    hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_sp_ts), sizeof(g_sp_ts));
    hipMemcpyFromSymbol(nseg, HIP_SYMBOL(g_sp_nseg), sizeof(g_sp_nseg));
    static unsigned long long z[64][6];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sp_ts), z, sizeof(z));
}
// reps timed launches (HIP events) after one warm-up; outputs of the last one
extern "C" int split_run(const unsigned long long* h_in, unsigned long long* h_out, int* h_seg, int n, int limit, int reps, float* ms,
                         unsigned long long* cyc) {
    unsigned long long *d_in, *d_E, *d_cyc;
    int* d_seg;
    hipMalloc(&d_in, 8 * (size_t)n); hipMalloc(&d_E, 8 * (size_t)n); hipMalloc(&d_seg, 4 * LS_SEGL); hipMalloc(&d_cyc, 8);
    hipMemcpy(d_in, h_in, 8 * (size_t)n, hipMemcpyHostToDevice);
    const size_t lds = ls_split_scratch_bytes(NT, CAP);
    hipFuncSetAttribute((const void*)k_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    k_split<<<1, NT, lds>>>(d_in, d_E, n, limit, d_seg, d_cyc);
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) k_split<<<1, NT, lds>>>(d_in, d_E, n, limit, d_seg, d_cyc);
    hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(ms, a, b); *ms /= reps;
    hipMemcpy(h_out, d_E, 8 * (size_t)n, hipMemcpyDeviceToHost);
    hipMemcpy(h_seg, d_seg, 4 * LS_SEGL, hipMemcpyDeviceToHost);
    hipMemcpy(cyc, d_cyc, 8, hipMemcpyDeviceToHost);
    hipFree(d_in); hipFree(d_E); hipFree(d_seg); hipFree(d_cyc);
    return (int)hipGetLastError();
}
