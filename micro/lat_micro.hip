// Micro-benchmark (not part of the library): dependent-load latency vs footprint on one wave.
// build: hipcc -O3 --offload-arch=gfx950 micro/lat_micro.hip -o micro/lat_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>
__global__ void chase(const int* __restrict__ nxt, int start, int hops, long long* out, int* sink) {
    int p = start;
    const long long t0 = clock64();
    for (int i = 0; i < hops; i++) p = __builtin_nontemporal_load(&nxt[p]) + (threadIdx.x & 0);
    const long long t1 = clock64();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = p; }
}
__global__ void chase_cached(const int* __restrict__ nxt, int start, int hops, long long* out, int* sink) {
    int p = start;
    const long long t0 = clock64();
    for (int i = 0; i < hops; i++) p = nxt[p];
    const long long t1 = clock64();
    if (threadIdx.x == 0) { out[0] = t1 - t0; sink[0] = p; }
}
__global__ void touch(int* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] += 0;
}
int main() {
    const size_t sizes[] = {1 << 18, 1 << 20, 1 << 22, 1 << 24, 1 << 26, 1 << 28};   // ints
    long long* dout; int* sink; hipMalloc(&dout, 8); hipMalloc(&sink, 4);
    for (size_t n : sizes) {
        // random cycle over n/16 slots spaced 64 B apart
        const size_t m = n / 16;
        std::vector<int> perm(m); for (size_t i = 0; i < m; i++) perm[i] = (int)i;
        std::mt19937 rng(1); std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<int> h(n, 0);
        for (size_t i = 0; i < m; i++) h[(size_t)perm[i] * 16] = perm[(i + 1) % m] * 16;
        int* d; hipMalloc(&d, n * 4); hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
        const int hops = 2000;
        long long c[4];
        chase_cached<<<1, 64>>>(d, perm[0] * 16, hops, dout, sink); hipMemcpy(&c[0], dout, 8, hipMemcpyDeviceToHost);
        chase_cached<<<1, 64>>>(d, perm[0] * 16, hops, dout, sink); hipMemcpy(&c[1], dout, 8, hipMemcpyDeviceToHost);
        touch<<<1024, 256>>>(d, n);    // written by another kernel on all XCDs
        chase_cached<<<1, 64>>>(d, perm[0] * 16, hops, dout, sink); hipMemcpy(&c[2], dout, 8, hipMemcpyDeviceToHost);
        chase<<<1, 64>>>(d, perm[0] * 16, hops, dout, sink); hipMemcpy(&c[3], dout, 8, hipMemcpyDeviceToHost);
        printf("footprint %8.1f MB: cycles/hop first %.0f  again %.0f  after-touch %.0f  nontemporal %.0f\n",
               n * 4 / 1048576.0, c[0] / (double)hops, c[1] / (double)hops, c[2] / (double)hops, c[3] / (double)hops);
        hipFree(d);
    }
    // clock rate calibration: clock64 ticks vs event time
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    {
        const size_t n = 1 << 20; const size_t m = n / 16;
        std::vector<int> h(n, 0); for (size_t i = 0; i < m; i++) h[i * 16] = (int)(((i + 1) % m) * 16);
        int* d; hipMalloc(&d, n * 4); hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
        hipEventRecord(e0); chase_cached<<<1, 64>>>(d, 0, 200000, dout, sink); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); long long c; hipMemcpy(&c, dout, 8, hipMemcpyDeviceToHost);
        printf("clock64: %lld ticks in %.3f ms -> %.1f MHz\n", c, ms, c / (ms * 1e3));
    }
    return 0;
}
