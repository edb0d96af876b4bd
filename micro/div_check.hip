// Checks div4_by_count (shared-reciprocal division) against the fp32 division operator, bit for bit,
// over random numerators (all exponents of the fast range, both signs, zeros) and counts 1..65535.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "aloam_device.hpp"
using namespace aloam;
__device__ unsigned long long mix(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull; z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull; z = (z ^ (z >> 27)) * 0x94d049bb133111ebull; return z ^ (z >> 31);
}
__global__ void k_check(unsigned long long seed, unsigned long long n, unsigned long long* bad, float* ex) {
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n; i += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long h = mix(seed ^ i);
        int k = (int)(h & 0xffff);
        if ((h >> 16) & 1) k &= 63;
        if (k == 0) k = 1;
        float4 v;
        float* vv = &v.x;
        for (int c = 0; c < 4; c++) {
            const unsigned long long g = mix(h + c);
            unsigned bits = (unsigned)g;
            const unsigned mode = (unsigned)(g >> 40) & 7;
            if (mode == 0) bits &= 0x80000000u;                                   // +-0
            else if (mode < 6) bits = (bits & 0x807fffffu) | ((unsigned)(127 - 89 + (g >> 44) % 178) << 23);   // in range
            vv[c] = __uint_as_float(bits);                                        // mode 6,7: any bits (fallback path)
        }
        const float4 a = div4_by_count(v, k);
        const float d = (float)k;
        const float4 b = make_float4(v.x / d, v.y / d, v.z / d, v.w / d);
        const float* aa = &a.x; const float* bb = &b.x;
        for (int c = 0; c < 4; c++)
            if (__float_as_uint(aa[c]) != __float_as_uint(bb[c]) && !(aa[c] != aa[c] && bb[c] != bb[c])) {
                const unsigned long long o = atomicAdd(bad, 1ull);
                if (o < 8) { ex[3 * o] = vv[c]; ex[3 * o + 1] = d; ex[3 * o + 2] = aa[c]; }
            }
    }
}
int main() {
    unsigned long long* bad; float* ex;
    hipMalloc(&bad, 8); hipMalloc(&ex, 96); hipMemset(bad, 0, 8);
    const unsigned long long n = 1ull << 32;
    for (int s = 0; s < 4; s++) k_check<<<4096, 256>>>(0x1234567ull + s * 0x1000000000ull, n / 4, bad, ex);
    unsigned long long hb; float he[24];
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(he, ex, 96, hipMemcpyDeviceToHost);
    printf("samples %llu x 4 components, mismatches %llu\n", n, hb);
    for (unsigned long long i = 0; i < hb && i < 8; i++) printf("  x=%a d=%g got=%a\n", he[3 * i], he[3 * i + 1], he[3 * i + 2]);
    return hb != 0;
}
