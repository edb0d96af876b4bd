// Micro-benchmark (not part of the library): cost of a dependent kernel boundary on one stream,
// eager vs HIP-graph replay, tiny kernels (1 or 256 workgroups).
// build: hipcc -O3 --offload-arch=gfx950 micro/launch_micro.hip -o micro/launch_micro
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void tiny(int* p) { if (threadIdx.x == 0) atomicAdd(p + blockIdx.x % 64, 1); }
int main() {
    int* d; hipMalloc(&d, 4096); hipMemset(d, 0, 4096);
    hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int blocks : {1, 256}) {
        for (int n : {10, 100}) {
            // eager
            for (int w = 0; w < 3; w++) { for (int i = 0; i < n; i++) tiny<<<blocks, 64, 0, s>>>(d); hipStreamSynchronize(s); }
            auto t0 = std::chrono::steady_clock::now();
            const int reps = 50;
            for (int r = 0; r < reps; r++) { for (int i = 0; i < n; i++) tiny<<<blocks, 64, 0, s>>>(d); }
            hipStreamSynchronize(s);
            auto t1 = std::chrono::steady_clock::now();
            double eager = std::chrono::duration<double, std::micro>(t1 - t0).count() / (reps * n);
            // graph
            hipGraph_t g; hipGraphExec_t ge;
            hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
            for (int i = 0; i < n; i++) tiny<<<blocks, 64, 0, s>>>(d);
            hipStreamEndCapture(s, &g);
            hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            for (int w = 0; w < 3; w++) hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < reps; r++) hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            t1 = std::chrono::steady_clock::now();
            double graph = std::chrono::duration<double, std::micro>(t1 - t0).count() / (reps * n);
            // host-side launch cost alone
            t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; i++) tiny<<<blocks, 64, 0, s>>>(d);
            t1 = std::chrono::steady_clock::now();
            double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
            hipStreamSynchronize(s);
            printf("blocks %3d n %3d : eager %.2f us/kernel, graph %.2f us/kernel, host launch %.2f us\n", blocks, n, eager, graph, host);
            hipGraphExecDestroy(ge); hipGraphDestroy(g);
        }
    }
    return 0;
}
