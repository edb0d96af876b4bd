// Latency probe (profiling aid): dependent chains of fp64 ops on one lane, cycles per op (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ void chain(double* out, long long* cyc, double a, int n) {
    double x = a + threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        if (OP == 0) x = x * 1.0000001 + 1e-9;          // mul + add (no contraction)
        if (OP == 1) x = 1.0000001 / x;                  // correctly rounded division
        if (OP == 2) x = sqrt(x) + 1.0;                  // sqrt + add
        if (OP == 3) x = fma(x, 1.0000001, 1e-9);        // one fma
        if (OP == 4) x = x + 1e-9;                       // one add
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = x; cyc[0] = t1 - t0; }
}
int main() {
    double* d; long long* c; hipMalloc(&d, 8); hipMalloc(&c, 8);
    const char* nm[] = {"mul+add", "div", "sqrt+add", "fma", "add"};
    for (int rep = 0; rep < 2; rep++) {
        long long h; int n = 4096;
        chain<0><<<1, 64>>>(d, c, 1.5, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost); if (rep) printf("%-9s %6.1f cycles/iter\n", nm[0], (double)h / n);
        chain<1><<<1, 64>>>(d, c, 1.5, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost); if (rep) printf("%-9s %6.1f cycles/iter\n", nm[1], (double)h / n);
        chain<2><<<1, 64>>>(d, c, 1.5, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost); if (rep) printf("%-9s %6.1f cycles/iter\n", nm[2], (double)h / n);
        chain<3><<<1, 64>>>(d, c, 1.5, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost); if (rep) printf("%-9s %6.1f cycles/iter\n", nm[3], (double)h / n);
        chain<4><<<1, 64>>>(d, c, 1.5, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost); if (rep) printf("%-9s %6.1f cycles/iter\n", nm[4], (double)h / n);
    }
    return 0;
}
