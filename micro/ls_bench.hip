// micro/ls_bench.hip — ls_sort alone: one workgroup sorts a key array in LDS (kernel time + resource use)
#include <hip/hip_runtime.h>
__device__ unsigned long long g_ls_acc[8];   // cycles per phase summed over levels (thread 0), + level count
__device__ unsigned long long g_ls_t0;
#define LS_TS(k) do { if (threadIdx.x == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    if ((k) == 0 || (k) == 6) { if ((k) == 0) g_ls_acc[7]++; } if ((k) > 0) g_ls_acc[(k) - 1] += t_ - g_ls_t0; g_ls_t0 = t_; } } while (0)
__device__ unsigned long long g_ws[16][8];
#define WS_CLK() ((unsigned long long)__builtin_amdgcn_s_memtime())
#define WS_STAT(slot, v) do { if (__lane_id() == 0) { g_ws[threadIdx.x / 64][slot] += (unsigned long long)(v); } } while (0)
#include "../lidar-visual-odometry_amd/csrc/ls_sort.hpp"
using namespace aloam;
constexpr int NT = 1024, CPW = 10, CAP = NT * CPW;
__global__ void __launch_bounds__(NT) k_ls(const unsigned long long* in, unsigned long long* out, int n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* E = (unsigned long long*)smem;
    for (int t = threadIdx.x; t < n; t += NT) E[t] = in[t];
    __syncthreads();
    ls_sort<NT, CPW>(E, n, n > 1 ? 2 * (31 - __builtin_clz((unsigned)n)) : 0, smem + 8 * CAP, CAP);
    for (int t = threadIdx.x; t < n; t += NT) out[t] = E[t];
}
extern "C" int ls_phases(unsigned long long* out) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ls_acc), sizeof(g_ls_acc));
    static unsigned long long z[8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ls_acc), z, sizeof(z));
}
extern "C" int ws_stats(unsigned long long* out) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ws), sizeof(g_ws));
    static unsigned long long z[16][8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ws), z, sizeof(z));
}
extern "C" int ls_run(const unsigned long long* h_in, unsigned long long* h_out, int n, int reps, float* ms) {
    unsigned long long *d_in, *d_out;
    hipMalloc(&d_in, 8 * (size_t)n); hipMalloc(&d_out, 8 * (size_t)n);
    hipMemcpy(d_in, h_in, 8 * (size_t)n, hipMemcpyHostToDevice);
    const size_t lds = 8 * (size_t)CAP + ls_scratch_bytes(NT, CAP);
    hipFuncSetAttribute((const void*)k_ls, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    k_ls<<<1, NT, lds>>>(d_in, d_out, n);
    hipEventRecord(a);
    for (int r = 0; r < reps; r++) k_ls<<<1, NT, lds>>>(d_in, d_out, n);
    hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(ms, a, b); *ms /= reps;
    hipMemcpy(h_out, d_out, 8 * (size_t)n, hipMemcpyDeviceToHost);
    hipFree(d_in); hipFree(d_out);
    return (int)hipGetLastError();
}
