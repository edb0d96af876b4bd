// micro/lm_tail_bench.hip — cycles of the persistent LM solver's tail (k_lm.hip lm_tail_fast, one lane, state in LDS)
// for pass 0 (scaling + first step) and an accepted pass (accept + next step). Profiling aid.
#include "../lidar-visual-odometry_amd/csrc/k_lm.hip"
using namespace aloam;
__global__ void k_tail(const double* tot_in, const double* x_in, unsigned long long* cyc, double* out, int reps) {
    __shared__ LMState ls;
    __shared__ double tot[NACC];
    __shared__ double xl[7];
    if (threadIdx.x < NACC) tot[threadIdx.x] = tot_in[threadIdx.x];
    if (threadIdx.x < 7) xl[threadIdx.x] = x_in[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long acc0 = 0, acc1 = 0;
        for (int r = 0; r < reps; r++) {
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            lm_tail_fast(&ls, tot, 0, xl, nullptr, 4);
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            lm_post(&ls);
            tot[27] = tot[27] * 0.9;           // a decrease: accepted
            const unsigned long long t2 = __builtin_amdgcn_s_memtime();
            lm_tail_fast(&ls, tot, 1, xl, nullptr, 4);
            const unsigned long long t3 = __builtin_amdgcn_s_memtime();
            acc0 += t1 - t0; acc1 += t3 - t2;
            tot[27] = tot_in[27];
            for (int i = 0; i < 7; i++) xl[i] = x_in[i];
        }
        cyc[0] = acc0 / reps; cyc[1] = acc1 / reps;
        for (int i = 0; i < 7; i++) out[i] = ls.cand[i];
    }
}
extern "C" int tail_run(const double* tot, const double* x, unsigned long long* cyc, double* out) {
    double *dt, *dx, *dout; unsigned long long* dc;
    hipMalloc(&dt, 8 * 32); hipMalloc(&dx, 64); hipMalloc(&dout, 64); hipMalloc(&dc, 16);
    hipMemcpy(dt, tot, 8 * 29, hipMemcpyHostToDevice); hipMemcpy(dx, x, 56, hipMemcpyHostToDevice);
    k_tail<<<1, 64>>>(dt, dx, dc, dout, 20);
    hipDeviceSynchronize();
    hipMemcpy(cyc, dc, 16, hipMemcpyDeviceToHost); hipMemcpy(out, dout, 56, hipMemcpyDeviceToHost);
    hipFree(dt); hipFree(dx); hipFree(dout); hipFree(dc);
    return (int)hipGetLastError();
}
// pieces of the tail, each timed alone on one lane (operands from LDS so nothing folds)
__global__ void k_parts(const double* tot_in, unsigned long long* cyc, double* out) {
    __shared__ double s[64];
    if (threadIdx.x < 32) s[threadIdx.x] = tot_in[threadIdx.x];
    __syncthreads();
    if (threadIdx.x != 0) return;
    double M[21], rhs[6], y[6], x[7], d[6], c[7];
    for (int i = 0; i < 21; i++) M[i] = s[i];
    for (int i = 0; i < 6; i++) { rhs[i] = s[21 + i]; d[i] = s[21 + i] * 1e-3; }
    for (int i = 0; i < 7; i++) x[i] = s[i] * 1e-2 + 0.5;
    // A (upper, row-major) -> lower packed for chol_solve6_packed, + a diagonal shift
    double Ml[21];
    for (int a = 0; a < 6; a++) for (int b = 0; b <= a; b++) Ml[a * (a + 1) / 2 + b] = Aget(M, b, a) + (a == b ? 1.0 : 0.0);
    bool ok;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    chol_solve6_packed(Ml, rhs, y, &ok);
    __builtin_amdgcn_s_waitcnt(0);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    plus7(x, d, c);
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    double q = s[5] / s[7];
    q = q / s[9];
    q = 1.0 / q;
    unsigned long long t3 = __builtin_amdgcn_s_memtime();
    double r = rsqrt_nr(s[3] + q);
    unsigned long long t4 = __builtin_amdgcn_s_memtime();
    cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3;
    for (int i = 0; i < 6; i++) out[i] = y[i] + c[i] + (ok ? 0.0 : 1.0) + q + r;
}
extern "C" int parts_run(const double* tot, unsigned long long* cyc, double* out) {
    double *dt, *dout; unsigned long long* dc;
    hipMalloc(&dt, 8 * 32); hipMalloc(&dout, 64); hipMalloc(&dc, 32);
    hipMemcpy(dt, tot, 8 * 29, hipMemcpyHostToDevice);
    for (int r = 0; r < 3; r++) k_parts<<<1, 64>>>(dt, dc, dout);
    hipDeviceSynchronize();
    hipMemcpy(cyc, dc, 32, hipMemcpyDeviceToHost); hipMemcpy(out, dout, 48, hipMemcpyDeviceToHost);
    hipFree(dt); hipFree(dout); hipFree(dc);
    return (int)hipGetLastError();
}

// the same passes with the solver state in registers (thread 0's private copy), tot / x still in LDS
__global__ void k_tail_reg(const double* tot_in, const double* x_in, unsigned long long* cyc, double* out, int reps) {
    __shared__ double tot[NACC];
    __shared__ double xl[7];
    __shared__ LMState sink;
    if (threadIdx.x < NACC) tot[threadIdx.x] = tot_in[threadIdx.x];
    if (threadIdx.x < 7) xl[threadIdx.x] = x_in[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        LMState L;
        unsigned long long acc0 = 0, acc1 = 0;
        for (int r = 0; r < reps; r++) {
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            lm_tail_fast(&L, tot, 0, xl, nullptr, 4);
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            lm_post(&L);
            tot[27] = tot[27] * 0.9;           // a decrease: accepted
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long t2 = __builtin_amdgcn_s_memtime();
            lm_tail_fast(&L, tot, 1, xl, nullptr, 4);
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long t3 = __builtin_amdgcn_s_memtime();
            acc0 += t1 - t0; acc1 += t3 - t2;
            tot[27] = tot_in[27];
            for (int i = 0; i < 7; i++) xl[i] = x_in[i];
        }
        cyc[0] = acc0 / reps; cyc[1] = acc1 / reps;
        for (int i = 0; i < 7; i++) out[i] = L.cand[i];
        sink = L;
    }
}
extern "C" int tail_run_reg(const double* tot, const double* x, unsigned long long* cyc, double* out) {
    double *dt, *dx, *dout; unsigned long long* dc;
    (void)hipMalloc(&dt, 8 * 32); (void)hipMalloc(&dx, 64); (void)hipMalloc(&dout, 64); (void)hipMalloc(&dc, 16);
    (void)hipMemcpy(dt, tot, 8 * 29, hipMemcpyHostToDevice); (void)hipMemcpy(dx, x, 56, hipMemcpyHostToDevice);
    k_tail_reg<<<1, 64>>>(dt, dx, dc, dout, 20);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(cyc, dc, 16, hipMemcpyDeviceToHost); (void)hipMemcpy(out, dout, 56, hipMemcpyDeviceToHost);
    (void)hipFree(dt); (void)hipFree(dx); (void)hipFree(dout); (void)hipFree(dc);
    return (int)hipGetLastError();
}
