// Micro-benchmark of the persistent LM solver (not part of the library): phase timing per pass.
// build: hipcc -DALOAM_LM_TIMING ... micro/lm_micro.hip -o micro/lm_micro
#include "../lidar-visual-odometry_amd/csrc/k_lm.hip"
#include <cstdio>
#include <random>
#include <vector>
using namespace aloam;
__global__ void k_time_eval(const aloam_factor* f, int n, const double* x, double* outv, long long* cyc) {
    const int i = threadIdx.x;
    aloam_factor fi = f[i % n];
    const dquat q{x[0], x[1], x[2], x[3]};
    const double t[3] = {x[4], x[5], x[6]};
    double acc[NACC];
    for (int k = 0; k < NACC; k++) acc[k] = 0;
    __syncthreads();
    long long c0 = clock64();
    accumulate(fi, q, t, acc);
    double s = 0;
    for (int k = 0; k < NACC; k++) s += acc[k];
    long long c1 = clock64();
    outv[i] = s;
    cyc[i] = c1 - c0;
}
template <int V>
__global__ void __launch_bounds__(64) k_tail_bench(const LMState* snap, long long* cyc, int reps) {
    __shared__ LMState ls;
    __shared__ double tot[NACC];
    __shared__ double xl[7];
    if (threadIdx.x != 0) return;
    long long sum = 0;
    for (int r = 0; r < reps; r++) {
        ls = *snap;
        ls.done = 0; ls.iteration = 0;
        for (int i = 0; i < 21; i++) tot[i] = ls.A[i] * (1.0 + 1e-3 * r);
        for (int i = 0; i < 6; i++) tot[21 + i] = ls.g[i];
        tot[27] = ls.cost * 0.5; tot[28] = ls.nres;
        for (int i = 0; i < 7; i++) xl[i] = ls.x[i];
        ls.mcc = ls.cost;  ls.step_norm = 1.0;
        __builtin_amdgcn_s_waitcnt(0);
        const long long c0 = clock64();
        if (V == 0) lm_tail(&ls, tot, 1, xl, nullptr, 4);
        else lm_tail_reg(&ls, tot, 1, xl, nullptr, 4);
        __builtin_amdgcn_s_waitcnt(0);
        const long long c1 = clock64();
        sum += c1 - c0;
    }
    cyc[0] = sum / reps;
    cyc[1] = ls.iteration;
}
// pieces of the fast tail in isolation (one lane, dependent repetitions)
template <int V>
__global__ void __launch_bounds__(64) k_piece_bench(const LMState* snap, long long* cyc, int reps) {
    __shared__ LMState ls;
    if (threadIdx.x != 0) return;
    ls = *snap;
    double M[21], rhs[6], y[6], x[7], d[6], c[7];
    for (int a = 0; a < 6; a++) for (int b = 0; b <= a; b++) M[a * (a + 1) / 2 + b] = ls.A[b * 6 - b * (b - 1) / 2 + (a - b)] + (a == b ? 1.0 : 0.0);
    for (int a = 0; a < 6; a++) { rhs[a] = ls.g[a]; d[a] = 1e-3 * (a + 1); }
    for (int i = 0; i < 7; i++) x[i] = ls.x[i];
    bool ok = true;
    long long sum = 0;
    for (int r = 0; r < reps; r++) {
        __builtin_amdgcn_s_waitcnt(0);
        const long long c0 = clock64();
        if (V == 0) { chol_solve6_packed(M, rhs, y, &ok); rhs[0] += y[0] * 1e-30; }
        if (V == 1) { plus7(x, d, c); x[0] += c[0] * 1e-30; }
        if (V == 2) { ls.done = 0; ls.iteration = 0; lm_next_step_fast(&ls, nullptr, 4); x[0] += ls.cand[0] * 1e-30; }
        if (V == 3) { ls.pending = 1; ls.done = 0; lm_post(&ls); x[0] += ls.mcc * 1e-30; }
        if (V == 4) { y[0] = rsqrt_nr(x[1] + 2.0); x[1] += y[0] * 1e-30; }
        __builtin_amdgcn_s_waitcnt(0);
        const long long c1 = clock64();
        sum += c1 - c0;
    }
    cyc[0] = sum / reps;
    cyc[1] = (long long)(x[0] + y[0] + rhs[0]);
}
int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 20000;
    const int mode = argc > 2 ? atoi(argv[2]) : -1;
    std::mt19937_64 rng(5);
    std::normal_distribution<double> N01(0, 1);
    std::vector<aloam_factor> f(n);
    for (int i = 0; i < n; i++) {
        aloam_factor& a = f[i];
        a = aloam_factor{};
        a.type = mode < 0 ? ((i % 4 == 0) ? 0 : 2) : mode;
        for (int k = 0; k < 3; k++) { a.cp[k] = 5 * N01(rng); a.a[k] = 5 * N01(rng); a.b[k] = 5 * N01(rng); }
        if (a.type == 2) { double nn = sqrt(a.a[0]*a.a[0]+a.a[1]*a.a[1]+a.a[2]*a.a[2]); for (int k=0;k<3;k++) a.a[k]/=nn; a.b[0] = 0.05 * N01(rng) - (a.a[0]*a.cp[0]+a.a[1]*a.cp[1]+a.a[2]*a.cp[2]); }
    }
    Ctx C;
    C.P.max_solver_iterations = 4;
    C.n_cus = 256;
    lm_init(C);
    hipStreamCreate(&C.stream);
    aloam_factor* df; hipMalloc(&df, sizeof(aloam_factor) * n); hipMemcpy(df, f.data(), sizeof(aloam_factor) * n, hipMemcpyHostToDevice);
    hipMalloc(&C.d_lm_sum, sizeof(aloam_lm_summary) * 32); hipMalloc(&C.d_lm, sizeof(LMState));
    hipMalloc(&C.d_lm_recs, 8 * 2 * 64 * 32); hipMemset(C.d_lm_recs, 0, 8 * 2 * 64 * 32); hipMalloc(&C.d_lm_seq, 16); hipMemset(C.d_lm_seq, 0, 16);
    hipMalloc(&C.d_bar_err, 16); hipMemset(C.d_bar_err, 0, 16);
    double x0[7] = {0.01, -0.02, 0.005, 1, 0.1, 0.2, -0.1}; double nq = sqrt(x0[0]*x0[0]+x0[1]*x0[1]+x0[2]*x0[2]+1); for (int i=0;i<4;i++) x0[i]/=nq;
    double* dx; hipMalloc(&dx, 7 * 8);
    {
        double* ov; long long* cy; hipMalloc(&ov, 8 * 256); hipMalloc(&cy, 8 * 256);
        hipMemcpy(dx, x0, 56, hipMemcpyHostToDevice);
        for (int r = 0; r < 2; r++) k_time_eval<<<1, 256>>>(df, n, dx, ov, cy);
        long long hc[256]; hipMemcpy(hc, cy, sizeof(hc), hipMemcpyDeviceToHost);
        printf("accumulate() latency, one factor: %lld cycles (lane 0), %lld (lane 255)\n", hc[0], hc[255]);
    }
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        hipMemcpy(dx, x0, 56, hipMemcpyHostToDevice);
        hipEventRecord(e0, C.stream);
        for (int k = 0; k < 20; k++) lm_run(C, df, n, dx, 0, nullptr, nullptr, n);
        hipEventRecord(e1, C.stream);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("n=%d  %.2f us per solve\n", n, ms * 1000 / 20);
    }
    unsigned long long ts[8][5];
    hipMemcpyFromSymbol(ts, HIP_SYMBOL(aloam::g_lm_ts), sizeof(ts));
    for (int p = 0; p < 5; p++)
        printf("pass %d: eval %.2f blockreduce %.2f us, barrier %.2f us, reduce %.2f us, tail %.2f us\n", p,
               p ? (ts[p][4] - ts[p - 1][3]) / 100.0 : 0.0, (ts[p][0] - ts[p][4]) / 100.0, (ts[p][1] - ts[p][0]) / 100.0, (ts[p][2] - ts[p][1]) / 100.0, (ts[p][3] - ts[p][2]) / 100.0);
    {
        long long* cy; hipMalloc(&cy, 16); long long hc[2];
        k_tail_bench<0><<<1, 64>>>(C.d_lm, cy, 50); hipMemcpy(hc, cy, 16, hipMemcpyDeviceToHost);
        printf("tail (LDS state): %lld cycles, it %lld\n", hc[0], hc[1]);
        k_tail_bench<1><<<1, 64>>>(C.d_lm, cy, 50); hipMemcpy(hc, cy, 16, hipMemcpyDeviceToHost);
        printf("tail (register state): %lld cycles, it %lld\n", hc[0], hc[1]);
        const char* nm[] = {"chol_solve6_packed", "plus7", "lm_next_step_fast", "lm_post", "rsqrt_nr"};
        for (int v = 0; v < 5; v++) {
            if (v == 0) k_piece_bench<0><<<1, 64>>>(C.d_lm, cy, 50);
            if (v == 1) k_piece_bench<1><<<1, 64>>>(C.d_lm, cy, 50);
            if (v == 2) k_piece_bench<2><<<1, 64>>>(C.d_lm, cy, 50);
            if (v == 3) k_piece_bench<3><<<1, 64>>>(C.d_lm, cy, 50);
            if (v == 4) k_piece_bench<4><<<1, 64>>>(C.d_lm, cy, 50);
            hipMemcpy(hc, cy, 16, hipMemcpyDeviceToHost);
            printf("%-20s %lld cycles\n", nm[v], hc[0]);
        }
    }
    aloam_lm_summary s; hipMemcpy(&s, C.d_lm_sum, sizeof(s), hipMemcpyDeviceToHost);
    printf("iters %d succ %d term %d cost %g -> %g\n", s.iterations, s.successful_steps, s.termination, s.initial_cost, s.final_cost);
    return 0;
}
