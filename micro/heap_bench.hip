// micro/heap_bench.hip — std::__partial_sort (make_heap + sort_heap) of one segment in LDS: one lane
// (pcl_sort.hpp ps_heap_sort) vs one whole wave (ws_heap_sort); outputs must be identical. Profiling aid.
#include <hip/hip_runtime.h>
#include "../lidar-visual-odometry_amd/csrc/pcl_sort.hpp"
using namespace aloam;
constexpr int CAP = 8192;
template <int MODE>
__global__ void __launch_bounds__(64) k_heap(const unsigned long long* in, unsigned long long* out, int n, unsigned long long* cyc) {
    __shared__ unsigned long long E[CAP];
    for (int t = threadIdx.x; t < n; t += 64) E[t] = in[t];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0) { if (threadIdx.x == 0) ps_heap_sort(E, E + n); }
    else ws_heap_sort(E, 0, n, nullptr);   // E in LDS: the store-wait-free pops
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) *cyc = t1 - t0;
    for (int t = threadIdx.x; t < n; t += 64) out[t] = E[t];
}
extern "C" int heap_run(const unsigned long long* h_in, unsigned long long* h_out, int n, int mode, unsigned long long* cycles) {
    unsigned long long *d_in, *d_out, *d_c;
    hipMalloc(&d_in, 8 * n); hipMalloc(&d_out, 8 * n); hipMalloc(&d_c, 8);
    hipMemcpy(d_in, h_in, 8 * n, hipMemcpyHostToDevice);
    for (int r = 0; r < 3; r++) {
        if (mode == 0) k_heap<0><<<1, 64>>>(d_in, d_out, n, d_c);
        else k_heap<1><<<1, 64>>>(d_in, d_out, n, d_c);
    }
    hipMemcpy(h_out, d_out, 8 * n, hipMemcpyDeviceToHost);
    hipMemcpy(cycles, d_c, 8, hipMemcpyDeviceToHost);
    const int rc = (int)hipGetLastError();
    hipFree(d_in); hipFree(d_out); hipFree(d_c);
    return rc;
}
