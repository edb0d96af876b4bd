// aloam_api.hip — the C ABI of include/aloam_hip.h: context, stage orchestration, host I/O.
//
// Host <-> device traffic per scan (pipeline path, aloam_process_scan):
//   H2D  the raw sweep (skipped with ALOAM_INPUT_DEVICE)
//   D2H  ScanMeta counts after scanRegistration (sizes the odometry launches)
//   D2H  OdomState + per-round counters after laserOdometry
//   D2H  MapState + map sizes after laserMapping
// Everything else (clouds, grids, factors, LM state, the map) stays resident in HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <new>

#include "aloam_device.hpp"
#include "aloam_internal.hpp"

namespace aloam {

void* dalloc(Ctx& C, size_t bytes) {
    void* p = nullptr;
    bytes = std::max<size_t>(bytes, 16);
    HIPCHK(hipMalloc(&p, bytes));
    // zeroed on the context's (non-blocking) stream, so every later kernel of the context is ordered
    // after it; a plain hipMemset runs on the null stream, which a non-blocking stream does not wait for
    HIPCHK(hipMemsetAsync(p, 0, bytes, C.stream));
    C.bufs.push_back({p, bytes});
    return p;
}

void dfree(Ctx& C, void* p) {
    if (!p) return;
    HIPCHK(hipStreamSynchronize(C.stream));      // launches queued on the context's stream may still use it
    for (size_t i = 0; i < C.bufs.size(); i++)
        if (C.bufs[i].p == p) {
            C.bufs.erase(C.bufs.begin() + (long)i);
            break;
        }
    HIPCHK(hipFree(p));
}

void prof_mark(Ctx& C, int idx) {
    if (C.profiling && C.ev_ready) HIPCHK(hipEventRecord(C.ev[idx], C.stream));
}
void prof_phase(Ctx& C, int k) {
    if (C.profiling && C.ev_ready) HIPCHK(hipEventRecord(C.evp[k], C.stream));
}

__global__ void k_set2(int* dst, int a, int b) { dst[0] = a; dst[1] = b; }

// Small results block device -> pinned host memory: one workgroup storing straight into the mapped
// buffer (host-coherent, visible at the stream's completion) instead of hipMemcpyAsync, whose copy
// engine / blit launch adds ~10-20 us to the stream for a few KB. ALOAM_D2H_COPY=1: hipMemcpyAsync.
__global__ void k_to_host(const unsigned* __restrict__ src, unsigned* __restrict__ dst, int nwords) {
    const bool al = (((size_t)src | (size_t)dst) & 15) == 0;
    const int n4 = al ? nwords / 4 : 0;
    const uint4* s4 = (const uint4*)src;
    uint4* d4 = (uint4*)dst;
    for (int i = threadIdx.x; i < n4; i += blockDim.x) d4[i] = s4[i];
    for (int i = 4 * n4 + threadIdx.x; i < nwords; i += blockDim.x) dst[i] = src[i];
}
static const bool g_d2h_copy = getenv("ALOAM_D2H_COPY") && atoi(getenv("ALOAM_D2H_COPY")) == 1;
static void d2h_small(void* host_mapped, const void* dev, size_t bytes, hipStream_t st) {
    static_assert(sizeof(DevOut) % 4 == 0 && sizeof(ScanMeta) % 4 == 0 && offsetof(DevOut, map_n) % 4 == 0, "word copies");
    if (g_d2h_copy) { HIPCHK(hipMemcpyAsync(host_mapped, dev, bytes, hipMemcpyDeviceToHost, st)); return; }
    void* dptr = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dptr, host_mapped, 0));
    k_to_host<<<1, 256, 0, st>>>((const unsigned*)dev, (unsigned*)dptr, (int)(bytes / 4));
    HIPCHK(hipGetLastError());
}
void set_counts2(Ctx& C, int* dst, int a, int b) { k_set2<<<1, 1, 0, C.stream>>>(dst, a, b); }
struct Vec7 { double v[7]; };
// clouds 0-2: corner, surf, full (host counts n); 3-4 (optional): the VoxelGrid'ed corner / surf stacks,
// n = upper bound, the live count read from ndev on the device and copied to stack_counts
struct ForwardJob { const float4* src[5] = {}; float4* dst[5] = {}; int n[5] = {}; const int* ndev[5] = {};
                    int* counts = nullptr; int* stack_counts = nullptr; double* pose_dst = nullptr; double pose[7] = {};
                    const double* pose_src = nullptr; };   // pose_src (device) overrides pose
// y = cloud: grid-stride copy; block (0, 0) also writes the counts and the pose
__global__ void k_forward_map_input(ForwardJob j) {
    const int c = blockIdx.y;
    const float4* __restrict__ src = j.src[c];
    float4* __restrict__ dst = j.dst[c];
    const int n = j.ndev[c] ? min(j.n[c], *j.ndev[c]) : j.n[c];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
    if (blockIdx.x == 0 && c == 0) {
        if (threadIdx.x < 2) j.counts[threadIdx.x] = j.ndev[threadIdx.x] ? min(j.n[threadIdx.x], *j.ndev[threadIdx.x]) : j.n[threadIdx.x];
        if (threadIdx.x < 2 && j.stack_counts) j.stack_counts[threadIdx.x] = min(j.n[3 + threadIdx.x], *j.ndev[3 + threadIdx.x]);
        if (threadIdx.x < 7) j.pose_dst[threadIdx.x] = j.pose_src ? j.pose_src[threadIdx.x] : j.pose[threadIdx.x];
    }
}
__global__ void k_set7(double* dst, Vec7 x) { if (threadIdx.x < 7) dst[threadIdx.x] = x.v[threadIdx.x]; }
// the destination's copies are queued on its stream; the source's stream waits for them before it may
// overwrite its buffers (no host round trip on the hand-off)
static void handoff_done(Ctx& S, Ctx& C) {
    HIPCHK(hipEventRecord(C.ev_handoff, C.stream));
    HIPCHK(hipStreamWaitEvent(S.stream, C.ev_handoff, 0));
}

static thread_local std::string g_create_err;

static void init_map_state(MapState& m) {
    std::memset(&m, 0, sizeof(m));
    m.parameters[3] = 1.0;
    m.q_wmap_wodom[3] = 1.0;
    m.q_wodom[3] = 1.0;
    m.cenW = 10; m.cenH = 10; m.cenD = 5;   // laserMapping.cpp:74-76
}

static void allocate(Ctx& C) {
    const aloam_params& P = C.P;
    const int N = std::max(P.max_scan_points, 1024);
    C.cap_in = N;
    const int nb = (N + 255) / 256;
    C.d_in = (float4*)dalloc(C, sizeof(float4) * N);
    C.d_cl = (float4*)dalloc(C, sizeof(float4) * N);
    C.d_sid = (int*)dalloc(C, sizeof(int) * N);
    C.d_ori = (float*)dalloc(C, sizeof(float) * N);
    C.d_blk = (int*)dalloc(C, sizeof(int) * (std::max(nb, std::max(P.max_map_points, 1024) / 256 + 1) + 4096));
    C.d_hist = (int*)dalloc(C, sizeof(int) * (size_t)MAXL * nb);
    C.d_hoff = (int*)dalloc(C, sizeof(int) * (size_t)MAXL * nb);
    C.d_cloud = (float4*)dalloc(C, sizeof(float4) * N);
    C.d_curv = (float*)dalloc(C, sizeof(float) * N);
    C.d_scratch_xyz = (float4*)dalloc(C, sizeof(float4) * N);
    C.d_scratch_keys = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * 2 * (size_t)N);
    C.d_scratch_i = (int*)dalloc(C, sizeof(int) * 3 * (size_t)N);
    C.d_line_sharp = (int*)dalloc(C, sizeof(int) * MAXL * LINE_SHARP_CAP);
    C.d_line_lsharp = (int*)dalloc(C, sizeof(int) * MAXL * LINE_LSHARP_CAP);
    C.d_line_flat = (int*)dalloc(C, sizeof(int) * MAXL * LINE_FLAT_CAP);
    C.d_line_cnt = (int*)dalloc(C, sizeof(int) * MAXL * 4);
    C.d_line_lf = (float4*)dalloc(C, sizeof(float4) * N);
    C.d_meta = (ScanMeta*)dalloc(C, sizeof(ScanMeta));
    const int capS = MAXL * LINE_SHARP_CAP, capLS = MAXL * LINE_LSHARP_CAP, capF = MAXL * LINE_FLAT_CAP;
    C.d_sharp = (float4*)dalloc(C, sizeof(float4) * capS);
    C.d_flat = (float4*)dalloc(C, sizeof(float4) * capF);
    // less-sharp / less-flat ping-pong with the odometry's "last" clouds
    C.d_lsharp = (float4*)dalloc(C, sizeof(float4) * capLS);
    C.d_corner_last = (float4*)dalloc(C, sizeof(float4) * capLS);
    C.d_lflat = (float4*)dalloc(C, sizeof(float4) * N);
    C.d_surf_last = (float4*)dalloc(C, sizeof(float4) * N);
    C.d_sharp_idx = (int*)dalloc(C, sizeof(int) * capS);
    C.d_lsharp_idx = (int*)dalloc(C, sizeof(int) * capLS);
    C.d_flat_idx = (int*)dalloc(C, sizeof(int) * capF);
    // odometry
    C.d_out = (DevOut*)dalloc(C, sizeof(DevOut));
    HIPCHK(hipHostMalloc((void**)&C.h_out, sizeof(DevOut), hipHostMallocMapped));
    std::memset(C.h_out, 0, sizeof(DevOut));
    HIPCHK(hipHostMalloc((void**)&C.h_mout[0], 2 * sizeof(DevOut), hipHostMallocMapped));
    std::memset(C.h_mout[0], 0, 2 * sizeof(DevOut));
    C.h_mout[1] = C.h_mout[0] + 1;
    C.d_odom = &C.d_out->odom;
    std::memset(&C.h_odom, 0, sizeof(C.h_odom));
    C.h_odom.para[3] = 1.0;
    C.h_odom.q_w[3] = 1.0;
    HIPCHK(hipMemcpyAsync(C.d_odom, &C.h_odom, sizeof(OdomState), hipMemcpyHostToDevice, C.stream));
    grid_alloc(C, C.g_corner_last, capLS, 2.5f * 1.025f);   // two-phase 1-NN, k_odom.hip
    grid_alloc(C, C.g_surf_last, N, 2.5f * 1.025f);
    const int layers = std::min(MAXL, std::max(P.scan_line, 1));
    grid_alloc(C, C.g_corner_win, capLS, 2.5f * 1.025f, layers, false, true);   // window search: 2-D cells x scan line
    grid_alloc(C, C.g_surf_win, N, 2.5f * 1.025f, layers, false, true);
    // fine grids for the first 1-NN phase: most nearest neighbours lie well inside one fine cell, whose
    // 3x3x3 block streams a few hundred candidates instead of the coarse block's thousands
    static const float fine = getenv("ALOAM_ODOM_FINE") ? (float)atof(getenv("ALOAM_ODOM_FINE")) : 1.28f;   // tuning knob (0.5-1.28 measured, 1.28 best)
    grid_alloc(C, C.g_corner_fine, capLS, fine > 0.f ? fine : 2.5f * 1.025f);
    grid_alloc(C, C.g_surf_fine, N, fine > 0.f ? fine : 2.5f * 1.025f);
    C.cap_factors = capLS + N;
    C.d_factors = (aloam_factor*)dalloc(C, sizeof(aloam_factor) * C.cap_factors);
    C.d_nbr = (int*)dalloc(C, sizeof(int) * 5 * (size_t)C.cap_factors);
    C.d_lm = (LMState*)dalloc(C, sizeof(LMState));
    C.d_partials = (double*)dalloc(C, sizeof(double) * 512 * 32);
    C.d_lm_recs = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * 2 * 128 * 32);
    C.d_lm_seq = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * 2);
    HIPCHK(hipHostMalloc((void**)&C.h_bar_err, sizeof(int) * 4, hipHostMallocMapped));   // read at every sync, no copy
    std::memset(C.h_bar_err, 0, sizeof(int) * 4);
    HIPCHK(hipHostGetDevicePointer((void**)&C.d_bar_err, C.h_bar_err, 0));
    C.d_lm_sum = C.d_out->lm_sum;
    C.d_round_cnt = C.d_out->round_cnt;
    C.d_odom_spread = (int*)dalloc(C, sizeof(int) * ALOAM_MAX_ROUNDS * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE);
    C.d_map_spread = (int*)dalloc(C, sizeof(int) * ALOAM_MAX_ROUNDS * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE);
    C.d_last_n = (int*)dalloc(C, sizeof(int) * 2);
    C.d_last_sorted = (int*)dalloc(C, sizeof(int) * 2);
    C.d_odom_nq = (int*)dalloc(C, sizeof(int) * 2);
    lm_init(C);
    // round loops issued eagerly by default: replaying them as HIP graphs measured ~1 % slower on the driver's
    // config (graph entry / exit ~10 us per replay, profiles/r05_graph_ab.txt); ALOAM_GRAPHS=1 replays graphs
    C.use_graphs = getenv("ALOAM_GRAPHS") != nullptr && getenv("ALOAM_NO_GRAPHS") == nullptr;
    C.d_cand = C.d_out->cand;
    // mapping
    const int M = std::max(P.max_map_points, 1024);
    C.cap_map = M;
    C.d_map = &C.d_out->map;
    init_map_state(C.h_map);
    HIPCHK(hipMemcpyAsync(C.d_map, &C.h_map, sizeof(MapState), hipMemcpyHostToDevice, C.stream));
    C.d_mc = (float4*)dalloc(C, sizeof(float4) * M);
    C.d_ms = (float4*)dalloc(C, sizeof(float4) * M);
    C.d_mc2 = (float4*)dalloc(C, sizeof(float4) * M);
    C.d_ms2 = (float4*)dalloc(C, sizeof(float4) * M);
    C.d_mc_cube = (int*)dalloc(C, sizeof(int) * M);
    C.d_ms_cube = (int*)dalloc(C, sizeof(int) * M);
    C.d_mc2_cube = (int*)dalloc(C, sizeof(int) * M);
    C.d_ms2_cube = (int*)dalloc(C, sizeof(int) * M);
    C.d_map_tmp = (float4*)dalloc(C, sizeof(float4) * M);
    C.d_seg_keys = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * (4 * (size_t)M + 32768));
    C.d_map_n = C.d_out->map_n;
    C.d_cube_cnt = (int*)dalloc(C, sizeof(int) * 2 * 7 * (CUBE_N + 1));
    C.d_cube_valid = (unsigned char*)dalloc(C, CUBE_N);
    rebuild_init(C);                                              // map rebuild's run tables: reset
    grid_alloc(C, C.g_map_corner, M, 1.0f * 1.025f, 1, true);     // 5-NN within 1 m, 3x3x3 cells
    grid_alloc(C, C.g_map_surf, M, 1.0f * 1.025f, 1, true);
    // candidate cache of the registration rounds: stack points beyond cap_mq always search the grid (exact, but
    // a full 27-cell search per round; reported per frame as aloam_map_result.uncached_queries). 65,536 slots
    // hold every HDL-64 stack (~20k points); 1,280 B per slot
    C.cap_mq = std::min(C.cap_factors, 1 << 16);
    C.d_mc_ctr = (float4*)dalloc(C, sizeof(float4) * (size_t)C.cap_mq);
    C.d_mc_pts = (float4*)dalloc(C, sizeof(float4) * (size_t)C.cap_mq * MC_CAP_PTS);
    C.d_mc_pos = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_mq * MC_CAP_PTS);
    C.d_mc_prev = (int*)dalloc(C, sizeof(int) * 5 * (size_t)C.cap_mq);
    for (auto& m : C.mset) {
        m.corner = (float4*)dalloc(C, sizeof(float4) * capLS);
        m.surf = (float4*)dalloc(C, sizeof(float4) * N);
        m.full = (float4*)dalloc(C, sizeof(float4) * N);
        m.n = (int*)dalloc(C, sizeof(int) * 4);
        m.pose = (double*)dalloc(C, sizeof(double) * 8);
        m.cstack = (float4*)dalloc(C, sizeof(float4) * capLS);
        m.sstack = (float4*)dalloc(C, sizeof(float4) * N);
    }
    use_input_set(C, 0);
    C.d_tmp_n = (int*)dalloc(C, sizeof(int) * 2);
    C.d_registered = (float4*)dalloc(C, sizeof(float4) * N);
    // voxel / sort scratch
    C.cap_voxel = std::max(N, capLS) + 64;
    C.d_vkeys = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * 2 * (size_t)C.cap_voxel);
    C.d_vkeys2 = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * (size_t)C.cap_voxel);
    C.d_vvals = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_voxel);
    C.d_vvals2 = (int*)dalloc(C, sizeof(int) * ((size_t)C.cap_voxel + 64));
    C.d_ins_pts = (float4*)dalloc(C, sizeof(float4) * (size_t)C.cap_voxel);
    C.d_ins_val = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_voxel);
    C.d_ins_val2 = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_voxel);
    // lane scratch: lane 0 aliases the buffers above, lane 1 is a second set for stream2
    KindScratch& k0 = C.ks[0];
    k0.vkeys = C.d_vkeys; k0.vkeys2 = C.d_vkeys2; k0.vvals = C.d_vvals; k0.vvals2 = C.d_vvals2;
    k0.ins_pts = C.d_ins_pts; k0.ins_val = C.d_ins_val; k0.ins_val2 = C.d_ins_val2;
    k0.seg_keys = C.d_seg_keys; k0.blk = C.d_blk; k0.map_tmp = C.d_map_tmp;
    k0.cube_segl = (int*)dalloc(C, sizeof(int) * (size_t)125 * (1 + 3 * 320));
    KindScratch& k1 = C.ks[1];
    k1.vkeys = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * 2 * (size_t)C.cap_voxel);
    k1.vkeys2 = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * (size_t)C.cap_voxel);
    k1.vvals = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_voxel);
    k1.vvals2 = (int*)dalloc(C, sizeof(int) * ((size_t)C.cap_voxel + 64));
    k1.ins_pts = (float4*)dalloc(C, sizeof(float4) * (size_t)C.cap_voxel);
    k1.ins_val = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_voxel);
    k1.ins_val2 = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_voxel);
    k1.seg_keys = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * (4 * (size_t)M + 32768));
    k1.blk = (int*)dalloc(C, sizeof(int) * (std::max(nb, M / 256 + 1) + 4096));
    k1.map_tmp = (float4*)dalloc(C, sizeof(float4) * M);
    k1.cube_segl = (int*)dalloc(C, sizeof(int) * (size_t)125 * (1 + 3 * 320));
    KindScratch& kv = C.ksv;            // stream3: the stacks' VoxelGrid (vkeys, vvals, sort, blk only)
    kv.vkeys = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * 2 * (size_t)C.cap_voxel);
    kv.vkeys2 = (unsigned long long*)dalloc(C, sizeof(unsigned long long) * (size_t)C.cap_voxel);
    kv.vvals = (int*)dalloc(C, sizeof(int) * (size_t)C.cap_voxel);
    kv.vvals2 = (int*)dalloc(C, sizeof(int) * ((size_t)C.cap_voxel + 64));
    kv.blk = (int*)dalloc(C, sizeof(int) * (std::max(nb, M / 256 + 1) + 4096));
    HIPCHK(hipStreamCreateWithFlags(&C.stream2, hipStreamNonBlocking));
    for (auto& m : C.mset) {
        HIPCHK(hipEventCreateWithFlags(&m.ready, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&m.released, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&m.fwd, hipEventDisableTiming));
    }
    HIPCHK(hipEventCreateWithFlags(&C.ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&C.ev_join, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&C.ev_stkn, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&C.ev_handoff, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&C.ev_scan, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&C.ev_lf, hipEventDisableTiming));
    HIPCHK(hipHostMalloc((void**)&C.h_meta_pin, sizeof(ScanMeta), hipHostMallocMapped));
    std::memset(C.h_meta_pin, 0, sizeof(ScanMeta));
    for (auto& e : C.ev_mdone) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int i = 0; i < Ctx::NEV; i++) HIPCHK(hipEventCreate(&C.ev[i]));
    for (int i = 0; i < Ctx::PM_N; i++) HIPCHK(hipEventCreate(&C.evp[i]));
    C.ev_ready = true;
    HIPCHK(hipStreamSynchronize(C.stream));   // all zero-fills and init kernels done
}

void run_graph(Ctx& C, int slot, const void* k0, const void* k1, int n, const std::function<void()>& issue) {
    Ctx::GraphSlot& g = C.graphs[slot];
    if (!g.exec || g.key[0] != k0 || g.key[1] != k1 || g.n != n) {
        if (g.exec) { (void)hipGraphExecDestroy(g.exec); g.exec = nullptr; }
        hipGraph_t graph = nullptr;
        std::lock_guard<std::mutex> lk(C.capture_mu);
        HIPCHK(hipStreamBeginCapture(C.stream, hipStreamCaptureModeThreadLocal));
        try {
            issue();
        } catch (...) {
            (void)hipStreamEndCapture(C.stream, &graph);
            if (graph) (void)hipGraphDestroy(graph);
            throw;
        }
        HIPCHK(hipStreamEndCapture(C.stream, &graph));
        const hipError_t e = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        HIPCHK(e);
        g.key[0] = k0; g.key[1] = k1; g.n = n;
    }
    HIPCHK(hipGraphLaunch(g.exec, C.stream));
}

void fork_lane1(Ctx& C) {
    HIPCHK(hipEventRecord(C.ev_fork, C.stream));
    HIPCHK(hipStreamWaitEvent(C.stream2, C.ev_fork, 0));
}
void join_lane1(Ctx& C) {
    HIPCHK(hipEventRecord(C.ev_join, C.stream2));
    HIPCHK(hipStreamWaitEvent(C.stream, C.ev_join, 0));
}

static void sync(Ctx& C) {
    HIPCHK(hipStreamSynchronize(C.stream));
    if (*(volatile int*)C.h_bar_err) {   // a solver grid barrier timed out: reset it and report (results void)
        HIPCHK(hipMemsetAsync(C.d_lm_recs, 0, sizeof(unsigned long long) * 2 * 128 * 32, C.stream));
        HIPCHK(hipMemsetAsync(C.d_lm_seq, 0, sizeof(unsigned long long) * 2, C.stream));
        HIPCHK(hipStreamSynchronize(C.stream));
        *(volatile int*)C.h_bar_err = 0;
        throw ApiError{ALOAM_E_HIP, "LM cross-workgroup exchange timed out (workgroups not co-resident)"};
    }
}

static float ev_ms(Ctx& C, int a, int b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, C.ev[a], C.ev[b]) != hipSuccess) return 0.f;
    return ms;
}
static float evh_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
    return ms;
}

// scanRegistration's counts reach the host without a sync of their own: the copy is queued behind the
// registration kernels and read at the next sync of the stream (ensure_meta, or the odometry's result sync)
static void queue_meta(Ctx& C) {
    if (C.lf_pending) {                   // counts[4] comes from the per-line VoxelGrid on stream2
        HIPCHK(hipStreamWaitEvent(C.stream, C.ev_lf, 0));
        C.lf_pending = false;
    }
    d2h_small(C.h_meta_pin, C.d_meta, sizeof(ScanMeta), C.stream);
    C.meta_pending = true;
    C.meta_deferred = false;
}
static void apply_meta(Ctx& C) {   // the stream has been synchronised since queue_meta
    C.h_meta = *C.h_meta_pin;
    C.n_full = C.h_meta.counts[0];
    C.n_sharp = C.h_meta.counts[1];
    C.n_lsharp = C.h_meta.counts[2];
    C.n_flat = C.h_meta.counts[3];
    C.n_lflat = C.h_meta.counts[4];
    C.meta_pending = false;
}
static void ensure_meta(Ctx& C) {
    if (!C.meta_pending) return;
    if (C.meta_deferred) queue_meta(C);
    sync(C);
    apply_meta(C);
}

// sensor_msgs/PointCloud2 blob -> float4 (x, y, z, 0): x, y, z float32 at byte offsets 0, 4, 8 of each
// point_step-byte record (the fields pcl::fromROSMsg reads into the PointXYZ laserCloudIn,
// scanRegistration.cpp:131-133; any further fields — intensity, ring, time — are not used by the path)
__global__ void k_pc2_gather(const unsigned char* __restrict__ blob, int n, int step, float4* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* r = (const float*)(blob + (size_t)i * step);
    out[i] = make_float4(r[0], r[1], r[2], 0.f);
}

// ALOAM_FRONT_PHASES (profiling aid): GPU time of the front's phases (scanRegistration, odometry
// rounds, compose + grid builds) from events on the stream, read back at the next scan's start
static const bool g_front_phases = getenv("ALOAM_FRONT_PHASES") != nullptr;
static void front_phase(Ctx& C, int k) {
    static hipEvent_t ev[5];
    static bool made = false, used = false;
    static double acc[4] = {0, 0, 0, 0};
    static long nacc = 0;
    if (!made) { for (auto& e : ev) HIPCHK(hipEventCreate(&e)); made = true; }
    if (k == 0 && used) {
        HIPCHK(hipEventSynchronize(ev[4]));
        for (int i = 0; i < 4; i++) { float ms = 0; HIPCHK(hipEventElapsedTime(&ms, ev[i], ev[i + 1])); acc[i] += ms * 1e3; }
        if (++nacc % 200 == 0)
            std::fprintf(stderr, "[aloam front phases] us per scan: scanRegistration %.1f, gap %.1f, odometry rounds %.1f, compose+grids %.1f (mean of %ld)\n",
                         acc[0] / nacc, acc[1] / nacc, acc[2] / nacc, acc[3] / nacc, nacc);
    }
    HIPCHK(hipEventRecord(ev[k], C.stream));
    if (k == 4) used = true;
}

// defer: the odometry follows in the same call (front_issue, aloam_process_scan): the per-line VoxelGrid
// runs on stream2 beside the odometry rounds and the counts copy is queued behind it (do_odometry_issue)
static void do_scan_registration(Ctx& C, const float* xyzr, int n, int flags, bool defer = false) {
    if (n < 0 || (n > 0 && !xyzr)) throw ApiError{ALOAM_E_ARG, "bad input"};
    if (n > C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "scan larger than max_scan_points"};
    const int L = C.P.scan_line;
    if (!(L == 16 || L == 32 || L == 64) && !C.P.generic_scan_lines)
        throw ApiError{ALOAM_E_SCAN_LINES, "wrong scan number"};
    if (L > MAXL || L <= 0) throw ApiError{ALOAM_E_SCAN_LINES, "scan_line above the device maximum (128)"};
    // a previous scan's per-line VoxelGrid still pending on stream2 (its odometry threw before queue_meta
    // made the stream wait): it reads d_cloud and the line scratch this registration rewrites
    if (C.lf_pending) {
        HIPCHK(hipStreamWaitEvent(C.stream, C.ev_lf, 0));
        C.lf_pending = false;
    }
    const float4* in = (const float4*)xyzr;
    if (!(flags & ALOAM_INPUT_DEVICE) && n > 0) {
        HIPCHK(hipMemcpyAsync(C.d_in, xyzr, sizeof(float4) * n, hipMemcpyHostToDevice, C.stream));
        in = C.d_in;
    }
    prof_mark(C, 0);
    if (g_front_phases) front_phase(C, 0);
    const bool side = defer && !C.profiling;
    scan_registration_launch(C, in, n, side);
    if (side) C.lf_pending = true;
    C.lf_side = side;
    if (g_front_phases) front_phase(C, 1);
    prof_mark(C, 1);
    if (side) {
        C.meta_pending = true;
        C.meta_deferred = true;
    } else {
        queue_meta(C);
    }
    if (C.profiling) {
        ensure_meta(C);
        C.timing.scan_registration_ms = ev_ms(C, 0, 1);
        float* tt = C.timing.tictoc_ms;
        tt[ALOAM_TT_PREPARE] = evh_ms(C.ev[0], C.evp[Ctx::PM_SCAN_PREP]);
        tt[ALOAM_TT_SEPARATE_POINTS] = evh_ms(C.evp[Ctx::PM_SCAN_CURV], C.ev[1]);
        tt[ALOAM_TT_SCAN_REGISTRATION] = C.timing.scan_registration_ms;
    }
    C.have_features = true;
    C.features_from_host = false;
    C.features_swapped = false;
}

// the odometry's kd-tree rebuild (laserOdometry.cpp:640-641): 1-NN grids + scan-line-layered
// window grids of the last clouds, one batched build, and whether the clouds are line-ordered.
// flags_preset = true ONLY right after odom_compose on the same stream: k_odom_compose sets
// d_last_n and re-arms d_last_sorted (= 1, 1) for k_line_sorted to clear; any other caller passes
// false (d_last_n set by the caller, the flags re-armed here).
// cap_c / cap_s: launch-size bounds of the two clouds (the counts themselves are read on the device;
// -1 = the host counts)
static void build_last_grids(Ctx& C, bool flags_preset = false, int cap_c = -1, int cap_s = -1) {
    const int nc = std::max(cap_c >= 0 ? cap_c : C.n_corner_last, 1), ns = std::max(cap_s >= 0 ? cap_s : C.n_surf_last, 1);
    const GridBuild b[6] = {
        {&C.g_corner_last, C.d_corner_last, C.d_last_n + 0, nc, nullptr, nullptr},
        {&C.g_surf_last, C.d_surf_last, C.d_last_n + 1, ns, nullptr, nullptr},
        {&C.g_corner_win, C.d_corner_last, C.d_last_n + 0, nc, nullptr, nullptr},
        {&C.g_surf_win, C.d_surf_last, C.d_last_n + 1, ns, nullptr, nullptr},
        {&C.g_corner_fine, C.d_corner_last, C.d_last_n + 0, nc, nullptr, nullptr},
        {&C.g_surf_fine, C.d_surf_last, C.d_last_n + 1, ns, nullptr, nullptr}};
    grid_build_multi(C, b, 6);
    odom_last_sorted(C, flags_preset);
}

// laserOdometry in two halves: the issue (every launch of the scan, up to the results copy) and the
// completion (the scan's one sync, then the host-side bookkeeping). aloam_odometry runs both; the
// 2-stage pipeline returns between them (front_issue / front_complete), so the caller's round trip
// to the next scan overlaps this scan's GPU work.
// scanRegistration's less-sharp / less-flat counts (ScanMeta::counts[2], [4]) -> the early stacks' own copy
__global__ void k_stack_counts(const int* __restrict__ counts, int* __restrict__ dst) {
    dst[0] = counts[2];
    dst[1] = counts[4];
}

static void do_odometry_issue(Ctx& C) {
    if (!C.have_features) throw ApiError{ALOAM_E_STATE, "odometry before any features"};
    if (C.fp_active) throw ApiError{ALOAM_E_STATE, "an issued odometry scan has not been completed"};
    if (!C.front_failed.empty()) throw ApiError{ALOAM_E_STATE, "context unusable after a failed publish: " + C.front_failed};
    aloam_odom_result r{};
    hipStream_t st = C.stream;
    prof_mark(C, 2);
    const int rounds = std::min(C.P.odom_rounds, ALOAM_MAX_ROUNDS);
    // With scanRegistration's counts still in flight (meta_pending, aloam_process_scan) nothing below
    // waits for them: the rounds, the compose and the grid builds read every count on the device (the
    // host's stale counts only size grid-stride launches), and the one sync of the scan comes after the
    // grid builds, where the counts and the odometry results arrive together.
    const bool pend = C.meta_pending;
    if (!C.odom_inited) {
        C.odom_inited = true;       // laserOdometry.cpp:355-358
        ensure_meta(C);             // first scan: the last-cloud counts are set from the host below
    } else {
        r.optimized = 1;
        r.rounds = rounds;
        // search counters: zero from allocation / re-zeroed by the previous scan's k_odom_compose; a scan
        // that threw between its rounds and its compose left them dirty, so clear them here instead
        if (C.odom_spread_dirty)
            HIPCHK(hipMemsetAsync(C.d_odom_spread, 0, sizeof(int) * ALOAM_MAX_ROUNDS * ODOM_CNT_SLOTS * ODOM_CNT_STRIDE, st));
        int hint;
        if (pend) {                 // d_odom_nq written by k_concat; slot counts bounded by the per-line caps
            hint = C.last_nslots > 0 ? C.last_nslots : MAXL * (LINE_SHARP_CAP + LINE_FLAT_CAP) / 4;
        } else {                    // features from the host / another context
            const int nslots = C.n_sharp + C.n_flat;
            if (nslots > C.cap_factors) throw ApiError{ALOAM_E_CAPACITY, "factor capacity"};
            set_counts2(C, C.d_odom_nq, C.n_sharp, C.n_flat);
            hint = nslots;
        }
        // the rounds read every size from the device, so the same launches serve every scan
        const int cap_slots = MAXL * (LINE_SHARP_CAP + LINE_FLAT_CAP);
        auto issue = [&C, rounds, cap_slots](bool marks, int live_hint) {
            for (int it = 0; it < rounds; it++) {
                if (marks) prof_mark(C, 6 + 2 * it);
                odom_round_search(C, it);
                if (marks) prof_mark(C, 7 + 2 * it);
                lm_run(C, C.d_factors, cap_slots, C.d_odom->para, it, nullptr, C.d_odom_nq, live_hint);
            }
        };
        C.odom_spread_dirty = true;
        if (g_front_phases) front_phase(C, 2);
        if (C.profiling || !C.use_graphs) {
            issue(true, hint);
        } else {   // two cached graphs: the last-cloud buffers alternate between scans
            int slot = (C.graphs[0].key[0] == C.d_corner_last && C.graphs[0].key[1] == C.d_surf_last) ? 0
                     : (C.graphs[1].key[0] == C.d_corner_last && C.graphs[1].key[1] == C.d_surf_last) ? 1
                     : (C.graphs[0].exec ? 1 : 0);
            run_graph(C, slot, C.d_corner_last, C.d_surf_last, rounds, [&] { issue(false, hint); });
        }
        if (g_front_phases) front_phase(C, 3);
        prof_phase(C, Ctx::PM_ODOM_ROUNDS_END);
        // the less-flat cloud (stream2) and the counts copy, then the compose; pairs with
        // build_last_grids(C, true) below; the new last-cloud counts from the device meta
        if (C.meta_deferred) queue_meta(C);
        odom_compose(C, C.n_lsharp, C.n_lflat, pend ? C.d_meta->counts : nullptr);
        C.odom_spread_dirty = false;
    }
    // the current less-sharp / less-flat become the last clouds (:627-641)
    std::swap(C.d_lsharp, C.d_corner_last);
    std::swap(C.d_lflat, C.d_surf_last);
    C.features_swapped = true;
    C.n_corner_last = C.n_lsharp;   // (stale while pend: fixed after the sync below)
    C.n_surf_last = C.n_lflat;
    if (!r.optimized) set_counts2(C, C.d_last_n, C.n_corner_last, C.n_surf_last);   // else set by k_odom_compose
    build_last_grids(C, r.optimized != 0);
    if (g_front_phases && r.optimized) front_phase(C, 4);
    prof_mark(C, 3);
    const int skip = C.P.mapping_skip_frame > 0 ? C.P.mapping_skip_frame : 1;
    r.publish_to_mapping = (C.odom_frame_count % skip == 0);
    if (r.publish_to_mapping) C.odom_frame_count = 0;
    C.odom_frame_count++;
    // the publish (/laser_cloud_corner_last, /laser_cloud_surf_last, /velodyne_cloud_3, pose) is issued
    // ahead of the sync below, sized on the device: the copy reads the clouds' device counts, the stack
    // VoxelGrids run on launch-size hints (the previous publish's sizes + margin) and are redone with the
    // exact sizes after the sync in the rare case a count outgrew its hint
    const int t = C.in_cur ^ 1;
    Ctx::MapInSet& m = C.mset[t];
    int hint_c = 0, hint_s = 0;
    if (r.publish_to_mapping) {
        // publish into the other input set: a hand-off taken by value (MapSnapshot) stays valid until the
        // publish after next, and a mapping frame of this context keeps reading its own set
        const int capLS = MAXL * LINE_LSHARP_CAP;
        const int cap_c = pend ? capLS : C.n_corner_last, cap_s = pend ? C.cap_in : C.n_surf_last;
        const int cap_f = C.features_from_host ? 0 : (pend ? C.cap_in : C.n_full);
        m.stacks = false;
        ForwardJob j;
        j.src[0] = C.d_corner_last; j.src[1] = C.d_surf_last; j.src[2] = C.d_cloud;
        j.dst[0] = m.corner; j.dst[1] = m.surf; j.dst[2] = m.full;
        j.n[0] = cap_c; j.n[1] = cap_s; j.n[2] = cap_f;
        j.ndev[0] = C.d_last_n + 0; j.ndev[1] = C.d_last_n + 1; j.ndev[2] = (pend && cap_f) ? C.d_meta->counts : nullptr;
        j.counts = m.n;
        j.pose_dst = m.pose;
        j.pose_src = C.d_odom->q_w;                    // q_w[4], t_w[3] adjacent (OdomState)
        if (C.pre_publish) {
            // the hand-off wait runs after this scan's rounds and compose were queued: a failure here
            // leaves the front half-advanced, so the context refuses further scans instead of continuing
            auto f = std::move(C.pre_publish);
            C.pre_publish = nullptr;
            try {
                f();
            } catch (const HipError& e) {
                C.front_failed = e.msg;
                throw;
            }
        }
        const int live = std::max(std::max(C.stack_hint[0], C.stack_hint[1]), 1);   // grid-stride copy: any size is correct
        k_forward_map_input<<<dim3(std::max(1, std::min(1024, (std::min(live, std::max(cap_s, cap_c)) + 255) / 256)), 3), 256, 0, st>>>(j);
        HIPCHK(hipGetLastError());
        // the call returns before this copy ends: a hand-off of this set waits on its event
        HIPCHK(hipEventRecord(m.fwd, st));
        m.fwd_rec = true;
        if (C.publish_stacks) {
            // the mapping stacks (laserMapping.cpp:542-550) depend on this publish only: voxelised here on
            // the otherwise idle stream2 (overlapping this context's next scan) and handed over with the
            // clouds, which takes them off the mapping stage's critical path
            hint_c = pend ? std::min(cap_c, C.stack_hint[0] > 0 ? C.stack_hint[0] : cap_c) : cap_c;   // (exact when known)
            hint_s = pend ? std::min(cap_s, C.stack_hint[1] > 0 ? C.stack_hint[1] : cap_s) : cap_s;
            static const bool early = !(getenv("ALOAM_EARLY_STACKS") && atoi(getenv("ALOAM_EARLY_STACKS")) == 0);
            if (pend && early && C.lf_side) {
                // The stacks read the clouds where scanRegistration left them (the last clouds since the swap
                // above) with its device counts, so stream2 needs nothing of this scan's odometry: it follows its
                // own less-flat VoxelGrid (queued there) and the set's hand-off wait (pre_publish), and the stacks
                // are ready ~one odometry earlier (ALOAM_EARLY_STACKS=0: after the publish copy, as before)
                // (their counts copied first: the next registration rewrites the less-sharp count on the stream,
                // which waits for that copy)
                k_stack_counts<<<1, 1, 0, C.stream2>>>(C.d_meta->counts, m.n + 2);
                HIPCHK(hipEventRecord(C.ev_stkn, C.stream2));
                HIPCHK(hipStreamWaitEvent(st, C.ev_stkn, 0));
                voxel_grid_pair_on(C, C.stream2, C.ks[1], C.d_corner_last, m.n + 2, hint_c, C.P.mapping_line_resolution, m.cstack,
                                   C.d_out->stack_n + 2 * t + 0, C.d_surf_last, m.n + 3, hint_s, C.P.mapping_plane_resolution,
                                   m.sstack, C.d_out->stack_n + 2 * t + 1);
            } else {
                fork_lane1(C);
                voxel_grid_pair_on(C, C.stream2, C.ks[1], m.corner, m.n + 0, hint_c, C.P.mapping_line_resolution, m.cstack,
                                   C.d_out->stack_n + 2 * t + 0, m.surf, m.n + 1, hint_s, C.P.mapping_plane_resolution, m.sstack,
                                   C.d_out->stack_n + 2 * t + 1);
            }
            HIPCHK(hipEventRecord(m.ready, C.stream2));
            m.stacks_pub = true;
        } else {
            m.stacks_pub = false;
        }
    }
    // results: odom state, round counts and LM summaries in one copy into the pinned mirror (+ the
    // scan's counts, queued behind scanRegistration): the scan's one sync, in do_odometry_complete
    d2h_small(C.h_out, C.d_out, offsetof(DevOut, map_n), st);
    C.pre_publish = nullptr;                           // (a scan that does not publish drops it)
    C.fp = Ctx::FrontPend{r, pend, t, hint_c, hint_s};
    C.fp_active = true;
}

static void do_odometry_complete(Ctx& C, aloam_odom_result* R) {
    if (!C.fp_active) throw ApiError{ALOAM_E_STATE, "no issued odometry scan"};
    C.fp_active = false;
    aloam_odom_result r = C.fp.r;
    const bool pend = C.fp.pend;
    const int t = C.fp.t, hint_c = C.fp.hint_c, hint_s = C.fp.hint_s;
    Ctx::MapInSet& m = C.mset[t];
    sync(C);
    if (pend) {
        apply_meta(C);
        C.n_corner_last = C.n_lsharp;
        C.n_surf_last = C.n_lflat;
    }
    C.last_nslots = C.n_sharp + C.n_flat;
    C.h_odom = C.h_out->odom;
    const int* cnt = C.h_out->round_cnt;
    std::memcpy(r.lm, C.h_out->lm_sum, sizeof(aloam_lm_summary) * ALOAM_MAX_ROUNDS);
    if (!r.optimized) std::memset(r.lm, 0, sizeof(r.lm));
    for (int i = 0; i < r.rounds; i++) { r.corner_correspondence[i] = cnt[2 * i]; r.plane_correspondence[i] = cnt[2 * i + 1]; }
    for (int k = 0; k < 4; k++) { r.q_w_curr[k] = C.h_odom.q_w[k]; r.q_last_curr[k] = C.h_odom.para[k]; }
    for (int k = 0; k < 3; k++) { r.t_w_curr[k] = C.h_odom.t_w[k]; r.t_last_curr[k] = C.h_odom.para[4 + k]; }
    if (r.publish_to_mapping) {
        for (int k = 0; k < 4; k++) C.h_map.q_wodom[k] = r.q_w_curr[k];
        for (int k = 0; k < 3; k++) C.h_map.t_wodom[k] = r.t_w_curr[k];
        m.nc = C.n_corner_last;
        m.ns = C.n_surf_last;
        m.nf = C.features_from_host ? 0 : C.n_full;
        if (C.publish_stacks && (m.nc > hint_c || m.ns > hint_s)) {
            // a count outgrew its hint: redo both stacks with the exact sizes (stream order overwrites)
            voxel_grid_pair_on(C, C.stream2, C.ks[1], m.corner, m.n + 0, m.nc, C.P.mapping_line_resolution, m.cstack,
                               C.d_out->stack_n + 2 * t + 0, m.surf, m.n + 1, m.ns, C.P.mapping_plane_resolution, m.sstack,
                               C.d_out->stack_n + 2 * t + 1);
            HIPCHK(hipEventRecord(m.ready, C.stream2));
        }
        // next publish's hints: these sizes + 25% + 1024 (capped by the buffers)
        C.stack_hint[0] = std::min(m.nc + m.nc / 4 + 1024, std::min(MAXL * LINE_LSHARP_CAP, C.cap_voxel));
        C.stack_hint[1] = std::min(m.ns + m.ns / 4 + 1024, std::min(C.cap_in, C.cap_voxel));
        use_input_set(C, t);
        C.have_map_input = true;
    }
    if (C.profiling) {
        C.timing.odometry_ms = ev_ms(C, 2, 3);
        float s = 0, sol = 0;
        for (int i = 0; i < r.rounds; i++) {
            s += ev_ms(C, 6 + 2 * i, 7 + 2 * i);
            sol += i + 1 < r.rounds ? ev_ms(C, 7 + 2 * i, 6 + 2 * (i + 1)) : evh_ms(C.ev[7 + 2 * i], C.evp[Ctx::PM_ODOM_ROUNDS_END]);
        }
        C.timing.odom_search_ms = s;
        C.timing.odom_search_launches = r.rounds;
        float* tt = C.timing.tictoc_ms;
        tt[ALOAM_TT_DATA_ASSOCIATION] = s;
        tt[ALOAM_TT_SOLVER] = sol;
        tt[ALOAM_TT_OPTIMIZATION_TWICE] = r.rounds ? evh_ms(C.ev[6], C.evp[Ctx::PM_ODOM_ROUNDS_END]) : 0.f;
        tt[ALOAM_TT_PUBLICATION] = r.rounds ? evh_ms(C.evp[Ctx::PM_ODOM_ROUNDS_END], C.ev[3]) : C.timing.odometry_ms;
        tt[ALOAM_TT_WHOLE_ODOMETRY] = C.timing.odometry_ms;
    }
    if (R) *R = r;
}

static void do_odometry(Ctx& C, aloam_odom_result* R) {
    do_odometry_issue(C);
    do_odometry_complete(C, R);
}

void front_issue(Ctx& C, const float* xyzr, int n, int flags) {
    HIPCHK(hipSetDevice(C.device));
    do_scan_registration(C, xyzr, n, flags, true);
    do_odometry_issue(C);
}
void front_complete(Ctx& C, aloam_odom_result* R) {
    HIPCHK(hipSetDevice(C.device));
    do_odometry_complete(C, R);
}

void mapping_issue(Ctx& C) {
    if (!C.have_map_input) throw ApiError{ALOAM_E_STATE, "mapping before odometry output"};
    if (C.m_issued - C.m_done >= 2) throw ApiError{ALOAM_E_STATE, "two mapping frames already in flight"};
    if (C.profiling && C.m_issued != C.m_done) throw ApiError{ALOAM_E_STATE, "profiling needs one frame at a time"};
    hipStream_t st = C.stream;
    const int slot = (int)(C.m_issued & 1);
    const int X = C.in_cur;
    Ctx::MapInSet& in = C.mset[X];
    if (C.profiling) HIPCHK(hipMemsetAsync(C.d_cand, 0, sizeof(unsigned long long) * 2, st));
    prof_mark(C, 4);
    const auto th0 = std::chrono::steady_clock::now();
    map_frame_launch(C, X);
    C.t_issue_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - th0).count();
    C.t_pre_us = std::chrono::duration<double, std::micro>(C.t_rounds_issued - th0).count();
    prof_mark(C, 5);
    // map state, counts, summaries, sizes: one copy of the results block into this frame's pinned mirror
    d2h_small(C.h_mout[slot], C.d_out, sizeof(DevOut), st);
    HIPCHK(hipEventRecord(C.ev_mdone[slot], st));
    HIPCHK(hipEventRecord(in.released, st));   // the input set may be written again (stream3 waits on this)
    C.m_set[slot] = X;
    C.m_pend[slot][0] = in.nc;
    C.m_pend[slot][1] = in.ns;
    C.m_nfull[slot] = in.nf;
    C.m_frame[slot] = C.map_frame_count;
    C.n_mc += in.nc;                  // the map can grow by at most the frame's stacks until its sizes arrive
    C.n_ms += in.ns;
    C.have_map_input = false;
    C.map_frame_count++;
    C.m_issued++;
}

bool mapping_ready(Ctx& C) {
    if (C.m_done == C.m_issued) return false;
    return hipEventQuery(C.ev_mdone[(int)(C.m_done & 1)]) == hipSuccess;
}

void mapping_complete(Ctx& C, aloam_map_result* R) {
    if (C.m_done == C.m_issued) throw ApiError{ALOAM_E_STATE, "no mapping frame in flight"};
    const int slot = (int)(C.m_done & 1);
    static const bool host_timing = getenv("ALOAM_HOST_TIMING") != nullptr;   // profiling aid
    const auto tw0 = std::chrono::steady_clock::now();
    HIPCHK(hipEventSynchronize(C.ev_mdone[slot]));
    if (*(volatile int*)C.h_bar_err) {   // a solver grid barrier timed out: every frame in flight is void
        C.m_done = C.m_issued;
        sync(C);
    }
    C.m_done++;
    const DevOut* H = C.h_mout[slot];
    aloam_map_result r{};
    double wodom[7];                     // the host's odometry pose of the latest hand-off stays
    std::memcpy(wodom, C.h_map.q_wodom, sizeof(double) * 4);
    std::memcpy(wodom + 4, C.h_map.t_wodom, sizeof(double) * 3);
    C.h_map = H->map;
    std::memcpy(C.h_map.q_wodom, wodom, sizeof(double) * 4);
    std::memcpy(C.h_map.t_wodom, wodom + 4, sizeof(double) * 3);
    if (host_timing) {
        static double acc_issue = 0, acc_wait = 0, acc_pre = 0;
        static int nfr = 0, seen = 0;
        if (++seen > 20) {               // past graph instantiation and allocation
            acc_issue += C.t_issue_us;
            acc_pre += C.t_pre_us;
            acc_wait += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tw0).count();
            if (++nfr % 40 == 0)
                std::fprintf(stderr, "[aloam host] mapping: issue until rounds %.1f us, whole issue %.1f us, completion wait %.1f us (mean of %d)\n",
                             acc_pre / nfr, acc_issue / nfr, acc_wait / nfr, nfr);
        }
    }
    const int* cnt = H->round_cnt + 2 * ALOAM_MAX_ROUNDS;
    std::memcpy(r.lm, H->lm_sum + ALOAM_MAX_ROUNDS, sizeof(aloam_lm_summary) * ALOAM_MAX_ROUNDS);
    const int* mapn = H->map_n;
    const int* stackn = H->stack_n + 2 * C.m_set[slot];
    const unsigned long long* cand = H->cand;
    const bool later = C.m_issued > C.m_done;      // a later frame is still in flight
    C.n_mc = mapn[0] + (later ? C.m_pend[slot ^ 1][0] : 0);
    C.n_ms = mapn[1] + (later ? C.m_pend[slot ^ 1][1] : 0);
    C.n_registered = C.m_nfull[slot];
    r.optimized = C.h_map.optimize;
    r.rounds = r.optimized ? std::min(C.P.map_rounds, ALOAM_MAX_ROUNDS) : 0;
    if (!r.optimized) std::memset(r.lm, 0, sizeof(r.lm));
    for (int i = 0; i < r.rounds; i++) { r.corner_num[i] = cnt[2 * i]; r.surf_num[i] = cnt[2 * i + 1]; }
    r.map_corner_num = C.h_map.n_corner_map;
    r.map_surf_num = C.h_map.n_surf_map;
    r.corner_stack_num = stackn[0];
    r.surf_stack_num = stackn[1];
    C.map_slots_hint = stackn[0] + stackn[1];
    r.map_total_points = mapn[0] + mapn[1];
    for (int k = 0; k < 7; k++) (k < 4 ? r.q_w_curr[k] : r.t_w_curr[k - 4]) = C.h_map.parameters[k];
    std::memcpy(r.q_wmap_wodom, C.h_map.q_wmap_wodom, sizeof(r.q_wmap_wodom));
    std::memcpy(r.t_wmap_wodom, C.h_map.t_wmap_wodom, sizeof(r.t_wmap_wodom));
    r.frame_count = C.m_frame[slot];
    r.pub_surround = r.frame_count % 5 == 0;      // laserMapping.cpp:806
    r.pub_map = r.frame_count % 20 == 0;          // :823
    r.uncached_queries = std::max(0, stackn[0] + stackn[1] - C.cap_mq);   //  no cache slot: full search every round
    {
        std::lock_guard<std::mutex> g(C.hf_mu);
        std::memcpy(C.hf_q, r.q_wmap_wodom, sizeof(C.hf_q));
        std::memcpy(C.hf_t, r.t_wmap_wodom, sizeof(C.hf_t));
    }
    if (C.profiling) {
        C.timing.mapping_ms = ev_ms(C, 4, 5);
        float s = 0, sol = 0;
        const int M = ALOAM_MAX_ROUNDS;
        for (int i = 0; i < r.rounds; i++) {
            s += ev_ms(C, 6 + 2 * (M + i), 7 + 2 * (M + i));
            sol += i + 1 < r.rounds ? ev_ms(C, 7 + 2 * (M + i), 6 + 2 * (M + i + 1))
                                    : evh_ms(C.ev[7 + 2 * (M + i)], C.evp[Ctx::PM_MAP_ROUNDS_END]);
        }
        C.timing.map_search_ms = s;
        float* tt = C.timing.tictoc_ms;
        tt[ALOAM_TT_MAP_PREPARE] = evh_ms(C.ev[4], C.evp[Ctx::PM_MAP_SHIFT]) +
                                   evh_ms(C.evp[Ctx::PM_MAP_GRIDS], C.evp[Ctx::PM_MAP_ROUNDS_BEGIN]);
        tt[ALOAM_TT_BUILD_TREE] = evh_ms(C.evp[Ctx::PM_MAP_SHIFT], C.evp[Ctx::PM_MAP_GRIDS]);
        tt[ALOAM_TT_MAP_ASSOCIATION] = s;
        tt[ALOAM_TT_MAP_SOLVER] = sol;
        tt[ALOAM_TT_MAP_OPTIMIZATION] = evh_ms(C.evp[Ctx::PM_MAP_ROUNDS_BEGIN], C.evp[Ctx::PM_MAP_ROUNDS_END]);
        tt[ALOAM_TT_ADD_POINTS] = evh_ms(C.evp[Ctx::PM_MAP_ROUNDS_END], C.evp[Ctx::PM_MAP_ADD]);
        tt[ALOAM_TT_FILTER] = evh_ms(C.evp[Ctx::PM_MAP_ADD], C.evp[Ctx::PM_MAP_FILTER]);
        tt[ALOAM_TT_MAPPING_PUB] = evh_ms(C.evp[Ctx::PM_MAP_FILTER], C.ev[5]);
        tt[ALOAM_TT_WHOLE_MAPPING] = C.timing.mapping_ms;
        C.timing.map_search_launches = r.rounds;
        // B = sum_q [16 + 16 |C(q)|] + 8 k Q  (k = 5 neighbour slots of 4 B + d2)
        const double Q = (double)(stackn[0] + stackn[1]) * r.rounds;
        C.timing.map_search_bytes = 16.0 * Q + 16.0 * (double)cand[0] + 8.0 * 5.0 * Q;
    }
    if (R) *R = r;
}

static void do_mapping(Ctx& C, aloam_map_result* R) {
    if (C.m_issued != C.m_done) throw ApiError{ALOAM_E_STATE, "a pipelined mapping frame is in flight"};
    mapping_issue(C);
    mapping_complete(C, R);
}

void snapshot_mapping_input(Ctx& S, MapSnapshot* o) {
    if (!S.have_map_input) throw ApiError{ALOAM_E_STATE, "source has no published odometry output"};
    o->src[0] = S.d_map_corner_in; o->src[1] = S.d_map_surf_in; o->src[2] = S.d_map_full_in;
    const Ctx::MapInSet& m = S.mset[S.in_cur];
    o->has_stacks = m.stacks_pub;
    o->stk[0] = m.cstack; o->stk[1] = m.sstack;
    o->stk_n = S.d_out->stack_n + 2 * S.in_cur;
    o->stk_ready = m.ready;
    o->fwd_done = m.fwd_rec ? m.fwd : nullptr;
    o->src_capture_mu = &S.capture_mu;
    o->n[0] = S.n_map_corner_in; o->n[1] = S.n_map_surf_in; o->n[2] = S.n_map_full_in;
    for (int k = 0; k < 4; k++) o->pose[k] = S.h_map.q_wodom[k];
    for (int k = 0; k < 3; k++) o->pose[4 + k] = S.h_map.t_wodom[k];
    S.have_map_input = false;
}

hipStream_t make_stream(Ctx& C, bool side) {
    const std::vector<unsigned>& m = side && !C.cu_mask_side.empty() ? C.cu_mask_side : C.cu_mask;
    hipStream_t st = nullptr;
    if (m.empty()) HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    else HIPCHK(hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data()));
    return st;
}

void set_side_cu_mask(Ctx& C, const unsigned* mask, int nwords) {
    HIPCHK(hipSetDevice(C.device));
    C.cu_mask_side.assign(mask, mask + std::max(nwords, 0));
    if (C.stream3) {
        HIPCHK(hipStreamSynchronize(C.stream3));
        (void)hipStreamDestroy(C.stream3);
        C.stream3 = nullptr;
    }
}

void use_input_set(Ctx& C, int t) {
    C.in_cur = t;
    const Ctx::MapInSet& m = C.mset[t];
    C.d_map_corner_in = m.corner; C.d_map_surf_in = m.surf; C.d_map_full_in = m.full; C.d_map_in_n = m.n;
    C.n_map_corner_in = m.nc; C.n_map_surf_in = m.ns; C.n_map_full_in = m.nf;
}

// The stacks of input set t (VoxelGrid of the corner / surf clouds, laserMapping.cpp:542-550) on stream3:
// they depend on the hand-off only, so they run while the previous frame still occupies the stream.
static void prepare_stacks(Ctx& C, int t) {
    Ctx::MapInSet& m = C.mset[t];
    voxel_grid_pair_on(C, C.stream3, C.ksv, m.corner, m.n + 0, m.nc, C.P.mapping_line_resolution, m.cstack,
                       C.d_out->stack_n + 2 * t + 0, m.surf, m.n + 1, m.ns, C.P.mapping_plane_resolution, m.sstack,
                       C.d_out->stack_n + 2 * t + 1);
    HIPCHK(hipEventRecord(m.ready, C.stream3));
    m.stacks = true;
}

// A hand-off into the other input set, on stream3 (after the frame that last read that set): one copy
// launch for the clouds, counts and pose, `copied` recorded behind it, then the set's stacks.
void forward_snapshot(Ctx& C, const MapSnapshot& s, hipEvent_t copied, bool defer_stacks) {
    HIPCHK(hipSetDevice(C.device));
    if (s.n[0] > MAXL * LINE_LSHARP_CAP || s.n[1] > C.cap_in || s.n[2] > C.cap_in)
        throw ApiError{ALOAM_E_CAPACITY, "mapping input too large"};
    const int t = C.in_cur ^ 1;
    Ctx::MapInSet& m = C.mset[t];
    // ALOAM_SIDE_STACKS=1: copy + stack VoxelGrid on stream3, overlapping the previous frame. Measured on
    // one MI355X (2-stage pipeline): +4% without CU partitions (916 vs 881 scans/s) but -30% with them
    // (715-757 vs 1019-1027, also with stream3 on CUs of its own) — a third busy CU-masked queue per
    // context costs more than the overlap gains. Default: both on the context's stream (stream order
    // then protects the set the previous frame reads).
    static const bool side = getenv("ALOAM_SIDE_STACKS") && atoi(getenv("ALOAM_SIDE_STACKS")) == 1;
    if (side && !C.stream3) C.stream3 = make_stream(C, true);
    hipStream_t fs = side ? C.stream3 : C.stream;
    HIPCHK(hipStreamWaitEvent(fs, m.released, 0));
    if (s.fwd_done) {                                                  // the source's publish copy
        std::unique_lock<std::mutex> lk;
        if (s.src_capture_mu) lk = std::unique_lock<std::mutex>(*s.src_capture_mu);   // not while the source captures
        HIPCHK(hipStreamWaitEvent(fs, s.fwd_done, 0));
    }
    m.nc = s.n[0]; m.ns = s.n[1]; m.nf = s.n[2];
    for (int k = 0; k < 4; k++) C.h_map.q_wodom[k] = s.pose[k];
    for (int k = 0; k < 3; k++) C.h_map.t_wodom[k] = s.pose[4 + k];
    ForwardJob j;
    for (int c = 0; c < 3; c++) j.src[c] = s.src[c], j.n[c] = s.n[c];
    j.dst[0] = m.corner; j.dst[1] = m.surf; j.dst[2] = m.full;
    j.counts = m.n;
    j.pose_dst = m.pose;
    std::memcpy(j.pose, s.pose, sizeof(j.pose));
    int ncl = 3;
    m.pstk = false;
    if (s.has_stacks && !side && defer_stacks) {   // stacks voxelised by the source (its stream2): copied
        m.pstk = true;                // right before the rounds (forward_stacks_pending), the clouds and the
                                      // pose now; `copied` is recorded then (mapping_issue of this set)
        for (int k = 0; k < 2; k++) { m.pstk_src[k] = s.stk[k]; m.pstk_n[k] = s.n[k]; }
        m.pstk_ndev = s.stk_n;
        m.pstk_ready = s.stk_ready;
        m.pstk_mu = s.src_capture_mu;
        m.pstk_copied = copied;
    } else if (s.has_stacks) {        // (copied with the clouds)
        std::unique_lock<std::mutex> lk;
        if (s.src_capture_mu) lk = std::unique_lock<std::mutex>(*s.src_capture_mu);
        HIPCHK(hipStreamWaitEvent(fs, s.stk_ready, 0));
        for (int k = 0; k < 2; k++) {
            j.src[3 + k] = s.stk[k];
            j.dst[3 + k] = k ? m.sstack : m.cstack;
            j.n[3 + k] = s.n[k];
            j.ndev[3 + k] = s.stk_n + k;
        }
        j.stack_counts = C.d_out->stack_n + 2 * t;
        ncl = 5;
    }
    const int nmax = std::max(std::max(j.n[0], j.n[1]), j.n[2]);
    k_forward_map_input<<<dim3(std::max(1, std::min(1024, (nmax + 255) / 256)), ncl), 256, 0, fs>>>(j);
    HIPCHK(hipGetLastError());
    if (copied && !m.pstk) HIPCHK(hipEventRecord(copied, fs));
    m.stacks_pub = s.has_stacks;      // present in this set once `ready` (recorded behind the copy) fires
    if (s.has_stacks && !m.pstk) HIPCHK(hipEventRecord(m.ready, fs));
    if (side && !s.has_stacks) prepare_stacks(C, t);
    else m.stacks = false;
    use_input_set(C, t);
    C.have_map_input = true;
}

__global__ void k_forward_stacks(ForwardJob j) {
    const int c = 3 + blockIdx.y;
    const int n = min(j.n[c], *j.ndev[c]);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) j.dst[c][i] = j.src[c][i];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 2) j.stack_counts[threadIdx.x] = min(j.n[3 + threadIdx.x], *j.ndev[3 + threadIdx.x]);
}
// the deferred stacks copy of input set t on the context's stream (then `copied`: the source may reuse
// its set, and `ready`)
void forward_stacks_pending(Ctx& C, int t) {
    Ctx::MapInSet& m = C.mset[t];
    if (!m.pstk) return;
    hipStream_t st = C.stream;
    {
        std::unique_lock<std::mutex> lk;
        if (m.pstk_mu) lk = std::unique_lock<std::mutex>(*m.pstk_mu);   // not while the source captures
        HIPCHK(hipStreamWaitEvent(st, m.pstk_ready, 0));
    }
    ForwardJob j;
    for (int k = 0; k < 2; k++) {
        j.src[3 + k] = m.pstk_src[k];
        j.dst[3 + k] = k ? m.sstack : m.cstack;
        j.n[3 + k] = m.pstk_n[k];
        j.ndev[3 + k] = m.pstk_ndev + k;
    }
    j.stack_counts = C.d_out->stack_n + 2 * t;
    const int nmax = std::max(m.pstk_n[0], m.pstk_n[1]);
    k_forward_stacks<<<dim3(std::max(1, std::min(1024, (nmax + 255) / 256)), 2), 256, 0, st>>>(j);
    HIPCHK(hipGetLastError());
    if (m.pstk_copied) HIPCHK(hipEventRecord(m.pstk_copied, st));
    HIPCHK(hipEventRecord(m.ready, st));
    m.pstk = false;
}

}  // namespace aloam

using namespace aloam;

#define API_BEGIN(ctx)                                    \
    if (!(ctx)) return ALOAM_E_ARG;                       \
    Ctx& C = *(Ctx*)(ctx);                                \
    try {                                                 \
        HIPCHK(hipSetDevice(C.device));
#define API_END                                           \
        return ALOAM_OK;                                  \
    } catch (const ApiError& e) {                         \
        C.err = e.msg;                                    \
        return e.code;                                    \
    } catch (const HipError& e) {                         \
        C.err = e.msg;                                    \
        return ALOAM_E_HIP;                               \
    } catch (const std::bad_alloc&) {                     \
        C.err = "host allocation failed";                 \
        return ALOAM_E_CAPACITY;                          \
    }

struct aloam_ctx {};   // opaque handle: the pointer is an aloam::Ctx*

extern "C" {

int aloam_abi_version(void) { return ALOAM_ABI_VERSION; }

void aloam_default_params(aloam_params* p, int scan_line) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->scan_line = scan_line;
    p->minimum_range = scan_line == 64 ? 5.0f : 0.3f;
    p->mapping_skip_frame = 1;
    p->mapping_line_resolution = scan_line == 64 ? 0.4f : 0.2f;
    p->mapping_plane_resolution = scan_line == 64 ? 0.8f : 0.4f;
    p->input_is_dense = 1;
    p->generic_scan_lines = (scan_line == 16 || scan_line == 32 || scan_line == 64) ? 0 : 1;
    p->generic_min_elev_deg = -25.f;
    p->generic_max_elev_deg = 15.f;
    p->odom_rounds = 10;
    p->map_rounds = 10;
    p->max_solver_iterations = 4;
    p->max_scan_points = 400000;
    p->max_map_points = 4000000;
}

aloam_ctx* aloam_create(const aloam_params* p, int device) {
    if (!p) { g_create_err = "null params"; return nullptr; }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) { g_create_err = "no HIP device"; return nullptr; }
    if (device < 0 || device >= n) { g_create_err = "bad device index"; return nullptr; }
    Ctx* C = new (std::nothrow) Ctx();
    if (!C) { g_create_err = "host allocation failed"; return nullptr; }
    C->P = *p;
    C->device = device;
    try {
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipStreamCreateWithFlags(&C->stream, hipStreamNonBlocking));
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, device));
        C->n_cus = prop.multiProcessorCount;
        allocate(*C);
    } catch (const HipError& e) {
        g_create_err = e.msg;
        for (auto& b : C->bufs) (void)hipFree(b.p);
        if (C->h_bar_err) (void)hipHostFree(C->h_bar_err);
        if (C->h_out) (void)hipHostFree(C->h_out);
        if (C->h_mout[0]) (void)hipHostFree(C->h_mout[0]);
        if (C->stream2) (void)hipStreamDestroy(C->stream2);
        if (C->stream3) (void)hipStreamDestroy(C->stream3);
        if (C->stream) (void)hipStreamDestroy(C->stream);
        delete C;
        return nullptr;
    }
    g_create_err.clear();
    return (aloam_ctx*)C;
}

void aloam_destroy(aloam_ctx* ctx) {
    if (!ctx) return;
    Ctx* C = (Ctx*)ctx;
    (void)hipSetDevice(C->device);
    if (C->stream) (void)hipStreamSynchronize(C->stream);
    if (C->stream2) (void)hipStreamSynchronize(C->stream2);
    if (C->stream3) (void)hipStreamSynchronize(C->stream3);
    if (C->ev_ready) for (int i = 0; i < Ctx::NEV; i++) (void)hipEventDestroy(C->ev[i]);
    if (C->ev_ready) for (int i = 0; i < Ctx::PM_N; i++) (void)hipEventDestroy(C->evp[i]);
    for (auto& g : C->graphs) if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (C->ev_fork) (void)hipEventDestroy(C->ev_fork);
    if (C->ev_join) (void)hipEventDestroy(C->ev_join);
    if (C->ev_stkn) (void)hipEventDestroy(C->ev_stkn);
    if (C->ev_handoff) (void)hipEventDestroy(C->ev_handoff);
    if (C->ev_scan) (void)hipEventDestroy(C->ev_scan);
    if (C->ev_lf) (void)hipEventDestroy(C->ev_lf);
    if (C->h_meta_pin) (void)hipHostFree(C->h_meta_pin);
    for (auto e : C->ev_mdone) if (e) (void)hipEventDestroy(e);
    for (auto& m : C->mset) {
        if (m.ready) (void)hipEventDestroy(m.ready);
        if (m.released) (void)hipEventDestroy(m.released);
        if (m.fwd) (void)hipEventDestroy(m.fwd);
    }
    s2m_release(*C);
    for (auto& b : C->bufs) (void)hipFree(b.p);
    if (C->h_bar_err) (void)hipHostFree(C->h_bar_err);
    if (C->h_out) (void)hipHostFree(C->h_out);
    if (C->h_mout[0]) (void)hipHostFree(C->h_mout[0]);
    if (C->stream2) (void)hipStreamDestroy(C->stream2);
    if (C->stream3) (void)hipStreamDestroy(C->stream3);
    if (C->stream) (void)hipStreamDestroy(C->stream);
    delete C;
}

const char* aloam_last_error(const aloam_ctx* ctx) {
    if (!ctx) return g_create_err.c_str();
    return ((const Ctx*)ctx)->err.c_str();
}

int aloam_scan_registration(aloam_ctx* ctx, const float* xyzr, int n, int flags) {
    API_BEGIN(ctx)
    do_scan_registration(C, xyzr, n, flags);
    ensure_meta(C);
    API_END
}

int aloam_scan_registration_pc2(aloam_ctx* ctx, const void* data, int n, int point_step, int flags) {
    API_BEGIN(ctx)
    if (n < 0 || (n > 0 && !data) || point_step < 12 || point_step % 4) throw ApiError{ALOAM_E_ARG, "bad PointCloud2 blob"};
    if (n > C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "scan larger than max_scan_points"};
    const unsigned char* blob = (const unsigned char*)data;
    const size_t bytes = (size_t)n * point_step;
    if (!(flags & ALOAM_INPUT_DEVICE) && n > 0) {
        if (bytes > C.cap_pc2) {
            C.cap_pc2 = std::max(bytes, 2 * C.cap_pc2);
            C.d_pc2 = (unsigned char*)dalloc(C, C.cap_pc2);
        }
        HIPCHK(hipMemcpyAsync(C.d_pc2, data, bytes, hipMemcpyHostToDevice, C.stream));
        blob = C.d_pc2;
    }
    if (n > 0) {
        k_pc2_gather<<<(n + 255) / 256, 256, 0, C.stream>>>(blob, n, point_step, C.d_in);
        HIPCHK(hipGetLastError());
    }
    do_scan_registration(C, (const float*)C.d_in, n, ALOAM_INPUT_DEVICE);
    ensure_meta(C);
    API_END
}

int aloam_feature_counts(aloam_ctx* ctx, int counts[5]) {
    API_BEGIN(ctx)
    if (!counts) throw ApiError{ALOAM_E_ARG, "null counts"};
    counts[0] = C.n_full; counts[1] = C.n_sharp; counts[2] = C.n_lsharp; counts[3] = C.n_flat; counts[4] = C.n_lflat;
    API_END
}

static void d2h_cloud(Ctx& C, const float4* src, int n, aloam_cloud* c) {
    if (!c) return;
    c->n = n;
    if (c->pts && n > 0) HIPCHK(hipMemcpyAsync(c->pts, src, sizeof(float4) * std::min(n, c->cap), hipMemcpyDeviceToHost, C.stream));
}

int aloam_get_features(aloam_ctx* ctx, aloam_features* o) {
    API_BEGIN(ctx)
    if (!o) throw ApiError{ALOAM_E_ARG, "null features"};
    if (!C.have_features) throw ApiError{ALOAM_E_STATE, "no features yet"};
    // after aloam_odometry the current less-sharp / less-flat clouds live in the last-cloud slots
    const float4* lsharp = C.features_swapped ? C.d_corner_last : C.d_lsharp;
    const float4* lflat = C.features_swapped ? C.d_surf_last : C.d_lflat;
    d2h_cloud(C, C.d_cloud, C.features_from_host ? 0 : C.n_full, &o->full);
    d2h_cloud(C, C.d_sharp, C.n_sharp, &o->sharp);
    d2h_cloud(C, lsharp, C.n_lsharp, &o->less_sharp);
    d2h_cloud(C, C.d_flat, C.n_flat, &o->flat);
    d2h_cloud(C, lflat, C.n_lflat, &o->less_flat);
    if (o->sharp_idx && C.n_sharp) HIPCHK(hipMemcpyAsync(o->sharp_idx, C.d_sharp_idx, sizeof(int) * C.n_sharp, hipMemcpyDeviceToHost, C.stream));
    if (o->less_sharp_idx && C.n_lsharp) HIPCHK(hipMemcpyAsync(o->less_sharp_idx, C.d_lsharp_idx, sizeof(int) * C.n_lsharp, hipMemcpyDeviceToHost, C.stream));
    if (o->flat_idx && C.n_flat) HIPCHK(hipMemcpyAsync(o->flat_idx, C.d_flat_idx, sizeof(int) * C.n_flat, hipMemcpyDeviceToHost, C.stream));
    if (o->curvature && C.n_full) HIPCHK(hipMemcpyAsync(o->curvature, C.d_curv, sizeof(float) * C.n_full, hipMemcpyDeviceToHost, C.stream));
    sync(C);
    API_END
}

int aloam_set_features(aloam_ctx* ctx, const float* sharp, int ns, const float* less_sharp, int nls,
                       const float* flat, int nf, const float* less_flat, int nlf) {
    API_BEGIN(ctx)
    if (ns < 0 || nls < 0 || nf < 0 || nlf < 0) throw ApiError{ALOAM_E_ARG, "negative size"};
    if (ns > MAXL * LINE_SHARP_CAP || nls > MAXL * LINE_LSHARP_CAP || nf > MAXL * LINE_FLAT_CAP || nlf > C.cap_in)
        throw ApiError{ALOAM_E_CAPACITY, "feature cloud too large"};
    auto up = [&](float4* d, const float* h, int n) {
        if (n > 0) HIPCHK(hipMemcpyAsync(d, h, sizeof(float4) * n, hipMemcpyHostToDevice, C.stream));
    };
    up(C.d_sharp, sharp, ns); up(C.d_lsharp, less_sharp, nls); up(C.d_flat, flat, nf); up(C.d_lflat, less_flat, nlf);
    sync(C);
    C.n_sharp = ns; C.n_lsharp = nls; C.n_flat = nf; C.n_lflat = nlf; C.n_full = 0;
    C.have_features = true;
    C.features_from_host = true;
    C.features_swapped = false;
    API_END
}

int aloam_forward_features(aloam_ctx* src, aloam_ctx* dst) {
    if (!src || src == dst) return ALOAM_E_ARG;
    Ctx& S = *(Ctx*)src;
    API_BEGIN(dst)
    if (S.device != C.device) throw ApiError{ALOAM_E_ARG, "contexts on different devices"};
    if (!S.have_features || S.features_swapped || S.features_from_host)
        throw ApiError{ALOAM_E_STATE, "source has no fresh scanRegistration output"};
    if (S.n_full > C.cap_in || S.n_lflat > C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "feature cloud too large"};
    hipStream_t st = C.stream;   // the source's stream is idle: its API calls return synchronised
    auto cp = [&](float4* d, const float4* s_, int n) {
        if (n > 0) HIPCHK(hipMemcpyAsync(d, s_, sizeof(float4) * n, hipMemcpyDeviceToDevice, st));
    };
    cp(C.d_cloud, S.d_cloud, S.n_full);
    cp(C.d_sharp, S.d_sharp, S.n_sharp);
    cp(C.d_lsharp, S.d_lsharp, S.n_lsharp);
    cp(C.d_flat, S.d_flat, S.n_flat);
    cp(C.d_lflat, S.d_lflat, S.n_lflat);
    C.n_full = S.n_full; C.n_sharp = S.n_sharp; C.n_lsharp = S.n_lsharp; C.n_flat = S.n_flat; C.n_lflat = S.n_lflat;
    C.h_meta = S.h_meta;
    C.have_features = true;
    C.features_from_host = false;
    C.features_swapped = false;
    handoff_done(S, C);
    S.have_features = false;
    API_END
}

int aloam_set_odom_state(aloam_ctx* ctx, const double q[4], const double t[3], const double qw[4], const double tw[3],
                         const float* corner_last, int nc, const float* surf_last, int ns) {
    API_BEGIN(ctx)
    if (!q || !t || !qw || !tw || nc < 0 || ns < 0) throw ApiError{ALOAM_E_ARG, "bad odom state"};
    if (nc > MAXL * LINE_LSHARP_CAP || ns > C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "last cloud too large"};
    for (int k = 0; k < 4; k++) { C.h_odom.para[k] = q[k]; C.h_odom.q_w[k] = qw[k]; }
    for (int k = 0; k < 3; k++) { C.h_odom.para[4 + k] = t[k]; C.h_odom.t_w[k] = tw[k]; }
    HIPCHK(hipMemcpyAsync(C.d_odom, &C.h_odom, sizeof(OdomState), hipMemcpyHostToDevice, C.stream));
    if (nc > 0) HIPCHK(hipMemcpyAsync(C.d_corner_last, corner_last, sizeof(float4) * nc, hipMemcpyHostToDevice, C.stream));
    if (ns > 0) HIPCHK(hipMemcpyAsync(C.d_surf_last, surf_last, sizeof(float4) * ns, hipMemcpyHostToDevice, C.stream));
    C.n_corner_last = nc; C.n_surf_last = ns;
    set_counts2(C, C.d_last_n, nc, ns);
    build_last_grids(C);
    sync(C);
    C.odom_inited = true;
    API_END
}

int aloam_odometry(aloam_ctx* ctx, aloam_odom_result* out) {
    API_BEGIN(ctx)
    do_odometry(C, out);
    API_END
}

int aloam_set_mapping_input(aloam_ctx* ctx, const float* corner, int nc, const float* surf, int ns, const double q[4], const double t[3]) {
    API_BEGIN(ctx)
    if (nc < 0 || ns < 0 || !q || !t) throw ApiError{ALOAM_E_ARG, "bad mapping input"};
    if (nc > MAXL * LINE_LSHARP_CAP || ns > C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "mapping input too large"};
    const int ti = C.in_cur ^ 1;          // the other input set (stream order protects the frame that read it)
    Ctx::MapInSet& m = C.mset[ti];
    if (nc > 0) HIPCHK(hipMemcpyAsync(m.corner, corner, sizeof(float4) * nc, hipMemcpyHostToDevice, C.stream));
    if (ns > 0) HIPCHK(hipMemcpyAsync(m.surf, surf, sizeof(float4) * ns, hipMemcpyHostToDevice, C.stream));
    m.nc = nc; m.ns = ns; m.nf = 0; m.stacks = false; m.stacks_pub = false; m.fwd_rec = false;
    set_counts2(C, m.n, nc, ns);
    for (int k = 0; k < 4; k++) C.h_map.q_wodom[k] = q[k];
    for (int k = 0; k < 3; k++) C.h_map.t_wodom[k] = t[k];
    HIPCHK(hipMemcpyAsync(m.pose, C.h_map.q_wodom, sizeof(double) * 7, hipMemcpyHostToDevice, C.stream));
    use_input_set(C, ti);
    sync(C);
    C.have_map_input = true;
    API_END
}

int aloam_mapping(aloam_ctx* ctx, aloam_map_result* out) {
    API_BEGIN(ctx)
    do_mapping(C, out);
    API_END
}

int aloam_get_map_cloud(aloam_ctx* ctx, int which, aloam_cloud* out) {
    API_BEGIN(ctx)
    if (!out) throw ApiError{ALOAM_E_ARG, "null cloud"};
    if (C.m_issued != C.m_done) throw ApiError{ALOAM_E_STATE, "a pipelined mapping frame is in flight"};
    // map arrays are sorted by cube id; the surround cloud is the surrounding cubes' points
    std::vector<int> cube_c(C.n_mc), cube_s(C.n_ms);
    std::vector<float4> pc(C.n_mc), ps(C.n_ms);
    if (C.n_mc) {
        HIPCHK(hipMemcpyAsync(pc.data(), C.d_mc, sizeof(float4) * C.n_mc, hipMemcpyDeviceToHost, C.stream));
        HIPCHK(hipMemcpyAsync(cube_c.data(), C.d_mc_cube, sizeof(int) * C.n_mc, hipMemcpyDeviceToHost, C.stream));
    }
    if (C.n_ms) {
        HIPCHK(hipMemcpyAsync(ps.data(), C.d_ms, sizeof(float4) * C.n_ms, hipMemcpyDeviceToHost, C.stream));
        HIPCHK(hipMemcpyAsync(cube_s.data(), C.d_ms_cube, sizeof(int) * C.n_ms, hipMemcpyDeviceToHost, C.stream));
    }
    sync(C);
    // reference order: for each cube (surround list order or all cubes in index order): corner then surf
    std::vector<int> cubes;
    if (which == 0) for (int i = 0; i < C.h_map.valid_num; i++) cubes.push_back(C.h_map.valid_ind[i]);
    else for (int i = 0; i < CUBE_N; i++) cubes.push_back(i);
    std::vector<int> oc(CUBE_N + 1, 0), os(CUBE_N + 1, 0);
    for (int c : cube_c) oc[c + 1]++;
    for (int c : cube_s) os[c + 1]++;
    for (int i = 0; i < CUBE_N; i++) { oc[i + 1] += oc[i]; os[i + 1] += os[i]; }
    int n = 0;
    float4* dst = (float4*)out->pts;
    for (int c : cubes) {
        for (int i = oc[c]; i < oc[c + 1]; i++) { if (dst && n < out->cap) dst[n] = pc[i]; n++; }
        for (int i = os[c]; i < os[c + 1]; i++) { if (dst && n < out->cap) dst[n] = ps[i]; n++; }
    }
    out->n = n;
    API_END
}

// profiling aid (not in include/aloam_hip.h): per-cube point counts of one map kind, and whether the
// cube is in the current surrounding set; counts[CUBE_N], valid[CUBE_N]
extern "C" int aloam_dbg_cube_counts(aloam_ctx* ctx, int which, int* counts, int* valid) {
    API_BEGIN(ctx)
    if (C.m_issued != C.m_done) throw ApiError{ALOAM_E_STATE, "a pipelined mapping frame is in flight"};
    const int n = which == 0 ? C.n_mc : C.n_ms;
    std::vector<int> cube(n);
    if (n) HIPCHK(hipMemcpyAsync(cube.data(), which == 0 ? C.d_mc_cube : C.d_ms_cube, sizeof(int) * n, hipMemcpyDeviceToHost, C.stream));
    sync(C);
    for (int c = 0; c < CUBE_N; c++) { counts[c] = 0; valid[c] = 0; }
    for (int c : cube) if (c >= 0 && c < CUBE_N) counts[c]++;
    for (int i = 0; i < C.h_map.valid_num; i++) valid[C.h_map.valid_ind[i]] = 1;
    API_END
}

int aloam_get_registered_cloud(aloam_ctx* ctx, aloam_cloud* out) {
    API_BEGIN(ctx)
    if (C.m_issued != C.m_done) throw ApiError{ALOAM_E_STATE, "a pipelined mapping frame is in flight"};
    d2h_cloud(C, C.d_registered, C.n_registered, out);
    sync(C);
    API_END
}

// laserOdometryHandler's republication (laserMapping.cpp:212-215): host double arithmetic in Eigen's
// order (aloam_device.hpp qmul / qrot are the same __host__ __device__ routines the device's
// transformAssociateToMap uses); no HIP call, so no device is set and no stream is touched
int aloam_map_high_freq_pose(aloam_ctx* ctx, const double q_wodom[4], const double t_wodom[3], double q_out[4], double t_out[3]) {
    if (!ctx || !q_wodom || !t_wodom || !q_out || !t_out) return ALOAM_E_ARG;
    Ctx& C = *(Ctx*)ctx;
    dquat qm;
    double tm[3];
    {
        std::lock_guard<std::mutex> g(C.hf_mu);
        qm = {C.hf_q[0], C.hf_q[1], C.hf_q[2], C.hf_q[3]};
        tm[0] = C.hf_t[0]; tm[1] = C.hf_t[1]; tm[2] = C.hf_t[2];
    }
    const dquat qo{q_wodom[0], q_wodom[1], q_wodom[2], q_wodom[3]};
    const dquat qw = qmul(qm, qo);
    const dvec3 r = qrot(qm, {t_wodom[0], t_wodom[1], t_wodom[2]});
    q_out[0] = qw.x; q_out[1] = qw.y; q_out[2] = qw.z; q_out[3] = qw.w;
    t_out[0] = r.x + tm[0]; t_out[1] = r.y + tm[1]; t_out[2] = r.z + tm[2];
    return ALOAM_OK;
}

int aloam_process_scan(aloam_ctx* ctx, const float* xyzr, int n, int flags, aloam_odom_result* o, aloam_map_result* m) {
    API_BEGIN(ctx)
    do_scan_registration(C, xyzr, n, flags, true);
    aloam_odom_result od{};
    do_odometry(C, &od);
    if (o) *o = od;
    if (od.publish_to_mapping && !(flags & ALOAM_NO_MAPPING)) do_mapping(C, m);
    else if (m) std::memset(m, 0, sizeof(*m));
    API_END
}

int aloam_forward_mapping_input(aloam_ctx* src, aloam_ctx* dst) {
    if (!src || src == dst) return ALOAM_E_ARG;
    Ctx& S = *(Ctx*)src;
    API_BEGIN(dst)
    if (S.device != C.device) throw ApiError{ALOAM_E_ARG, "contexts on different devices"};
    if (!S.have_map_input) throw ApiError{ALOAM_E_STATE, "source has no published odometry output"};
    if (S.n_map_corner_in > MAXL * LINE_LSHARP_CAP || S.n_map_surf_in > C.cap_in || S.n_map_full_in > C.cap_in)
        throw ApiError{ALOAM_E_CAPACITY, "mapping input too large"};
    // the source's stream is idle (its API calls return synchronised); the clouds, their counts and the
    // odometry pose go over in ONE launch (five separate copies / kernels cost ~15 us more)
    MapSnapshot snap;
    snapshot_mapping_input(S, &snap);
    forward_snapshot(C, snap, C.ev_handoff);
    HIPCHK(hipStreamWaitEvent(S.stream, C.ev_handoff, 0));   // the source publishes again only after the copy
    API_END
}

int aloam_eval_factors(aloam_ctx* ctx, const aloam_factor* f, int n, const double x[7], int robust,
                       double* residuals, double* jacobians, double neq[28]) {
    API_BEGIN(ctx)
    if (n < 0 || (n > 0 && !f) || !x) throw ApiError{ALOAM_E_ARG, "bad factors"};
    if (n > C.cap_factors) throw ApiError{ALOAM_E_CAPACITY, "too many factors"};
    double* d_x = (double*)C.d_partials;       // scratch: x[7] + neq[28] + residuals + jac via voxel buffers
    double* d_neq = d_x + 8;
    double* d_res = (double*)C.d_vkeys;        // 3n doubles
    double* d_jac = (double*)C.d_seg_keys;     // 18n doubles
    if ((size_t)3 * n > 2 * (size_t)C.cap_voxel) throw ApiError{ALOAM_E_CAPACITY, "too many factors"};
    if (n) HIPCHK(hipMemcpyAsync(C.d_factors, f, sizeof(aloam_factor) * n, hipMemcpyHostToDevice, C.stream));
    HIPCHK(hipMemcpyAsync(d_x, x, sizeof(double) * 7, hipMemcpyHostToDevice, C.stream));
    lm_eval_only(C, C.d_factors, n, d_x, robust, d_res, d_jac, d_neq);
    if (residuals && n) HIPCHK(hipMemcpyAsync(residuals, d_res, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, C.stream));
    if (jacobians && n) HIPCHK(hipMemcpyAsync(jacobians, d_jac, sizeof(double) * 18 * n, hipMemcpyDeviceToHost, C.stream));
    if (neq) HIPCHK(hipMemcpyAsync(neq, d_neq, sizeof(double) * 28, hipMemcpyDeviceToHost, C.stream));
    sync(C);
    API_END
}

int aloam_lm_solve(aloam_ctx* ctx, const aloam_factor* f, int n, double x[7], aloam_lm_summary* s) {
    API_BEGIN(ctx)
    if (n < 0 || (n > 0 && !f) || !x) throw ApiError{ALOAM_E_ARG, "bad factors"};
    if (n > C.cap_factors) throw ApiError{ALOAM_E_CAPACITY, "too many factors"};
    double* d_x = (double*)C.d_nbr;   // 7 doubles of scratch
    if (n) HIPCHK(hipMemcpyAsync(C.d_factors, f, sizeof(aloam_factor) * n, hipMemcpyHostToDevice, C.stream));
    HIPCHK(hipMemcpyAsync(d_x, x, sizeof(double) * 7, hipMemcpyHostToDevice, C.stream));
    lm_run(C, C.d_factors, n, d_x, 2 * ALOAM_MAX_ROUNDS - 1, nullptr);
    aloam_lm_summary sum{};
    HIPCHK(hipMemcpyAsync(x, d_x, sizeof(double) * 7, hipMemcpyDeviceToHost, C.stream));
    HIPCHK(hipMemcpyAsync(&sum, C.d_lm_sum + 2 * ALOAM_MAX_ROUNDS - 1, sizeof(sum), hipMemcpyDeviceToHost, C.stream));
    sync(C);
    if (s) *s = sum;
    API_END
}

int aloam_voxel_grid(aloam_ctx* ctx, const float* pts, int n, float leaf, aloam_cloud* out) {
    API_BEGIN(ctx)
    if (n < 0 || (n > 0 && !pts) || !out || !(leaf > 0)) throw ApiError{ALOAM_E_ARG, "bad voxel input"};
    if (n > C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "too many points"};
    if (n) HIPCHK(hipMemcpyAsync(C.d_in, pts, sizeof(float4) * n, hipMemcpyHostToDevice, C.stream));
    set_counts2(C, C.d_tmp_n, n, 0);
    voxel_grid_sorted(C, C.d_in, C.d_tmp_n, n, leaf, C.d_cl, C.d_tmp_n + 1);
    int nout = 0;
    HIPCHK(hipMemcpyAsync(&nout, C.d_tmp_n + 1, sizeof(int), hipMemcpyDeviceToHost, C.stream));
    sync(C);
    d2h_cloud(C, C.d_cl, nout, out);
    sync(C);
    C.have_map_input = false;
    API_END
}

int aloam_knn(aloam_ctx* ctx, const float* pts, int n, const float* queries, int nq, int k, float radius, int* idx, float* d2) {
    API_BEGIN(ctx)
    if (n < 0 || nq < 0 || k < 1 || k > 8 || !(radius > 0) || !idx || !d2) throw ApiError{ALOAM_E_ARG, "bad knn args (radius must be > 0, 1 <= k <= 8)"};
    if (n > C.cap_in || nq > C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "too many points"};
    if (n) HIPCHK(hipMemcpyAsync(C.d_in, pts, sizeof(float4) * n, hipMemcpyHostToDevice, C.stream));
    if (nq) HIPCHK(hipMemcpyAsync(C.d_cl, queries, sizeof(float4) * nq, hipMemcpyHostToDevice, C.stream));
    set_counts2(C, C.d_tmp_n, n, 0);
    Grid g = C.g_surf_last;      // borrow the odometry surf grid's storage with the requested radius
    g.min_cell = radius * 1.025f;
    grid_build(C, g, C.d_in, C.d_tmp_n, std::max(n, 1), nullptr, nullptr);
    int* d_idx = (int*)C.d_scratch_i;
    float* d_d2 = (float*)(C.d_scratch_i + (size_t)nq * k);
    if ((size_t)nq * k * 2 > 3 * (size_t)C.cap_in) throw ApiError{ALOAM_E_CAPACITY, "too many queries"};
    knn_launch(C, g, C.d_cl, nq, k, radius, d_idx, d_d2);
    if (nq) {
        HIPCHK(hipMemcpyAsync(idx, d_idx, sizeof(int) * nq * k, hipMemcpyDeviceToHost, C.stream));
        HIPCHK(hipMemcpyAsync(d2, d_d2, sizeof(float) * nq * k, hipMemcpyDeviceToHost, C.stream));
    }
    sync(C);
    // the odometry surf grid was overwritten: rebuild it for the current last cloud
    grid_build(C, C.g_surf_last, C.d_surf_last, C.d_last_n + 1, std::max(C.n_surf_last, 1), nullptr, nullptr);
    sync(C);
    C.have_map_input = false;
    API_END
}

// aloam_knn_build / aloam_knn_query: the map index is built once (both grids of the two-phase search, in
// context memory grown on demand) and then queried any number of times — the split of laserMapping.cpp's
// kdtree*FromMap->setInputCloud (:558-559, once per frame) and nearestKSearch (:582, :648, every round)
static void knn_build(Ctx& C, const float* d_pts, int n, float radius) {
    if (n < 0 || !(radius > 0) || (n > 0 && !d_pts)) throw ApiError{ALOAM_E_ARG, "bad knn build args (device pointer, radius > 0)"};
    C.knn_built = false;
    if (!C.d_knn_n) C.d_knn_n = (int*)dalloc(C, sizeof(int) * 2);
    if (C.g_knn.cap < std::max(n, 1)) {          // grow (old buffers are released with the context)
        Grid g{};
        grid_alloc(C, g, std::max(std::max(n, 1), C.g_knn.cap * 2), radius * 1.025f, 1, true, false, GRID_MAX_CELLS_BIG);
        C.g_knn = g;
    }
    C.g_knn.min_cell = radius * 1.025f;           // cells >= radius: the 27-cell block holds the ball
    const char* fe = getenv("ALOAM_KNN_FINE");    // read per build (tests compare both paths in one process)
    const float fine_frac = fe ? (float)atof(fe) : 0.3f;
    const bool two_phase = fine_frac > 0.f && fine_frac < 1.f;
    if (two_phase && C.g_knn_fine.cap < std::max(n, 1)) {   // grown on demand (the old grid given back)
        const int cap = std::max(std::max(n, 1), C.g_knn_fine.cap * 2);
        if (C.g_knn_fine.cap) grid_free(C, C.g_knn_fine);
        Grid g{};
        grid_alloc(C, g, cap, radius * fine_frac, 1, true, false, GRID_MAX_CELLS_BIG);
        C.g_knn_fine = g;
    }
    set_counts2(C, C.d_knn_n, n, 0);
    if (C.profiling) HIPCHK(hipEventRecord(C.ev[Ctx::NEV - 2], C.stream));
    if (two_phase) {
        C.g_knn_fine.min_cell = radius * fine_frac;
        const GridBuild b[2] = {{&C.g_knn, (const float4*)d_pts, C.d_knn_n, std::max(n, 1), nullptr, nullptr},
                                {&C.g_knn_fine, (const float4*)d_pts, C.d_knn_n, std::max(n, 1), nullptr, nullptr}};
        grid_build_multi(C, b, 2);
    } else {
        grid_build(C, C.g_knn, (const float4*)d_pts, C.d_knn_n, std::max(n, 1), nullptr, nullptr);
    }
    if (C.profiling) HIPCHK(hipEventRecord(C.ev[Ctx::NEV - 1], C.stream));
    sync(C);
    if (C.profiling) C.timing.knn_build_ms = ev_ms(C, Ctx::NEV - 2, Ctx::NEV - 1);
    C.knn_built = true;
    C.knn_two_phase = two_phase;
    C.knn_radius = radius;
    C.knn_n = n;
}

static void knn_query(Ctx& C, const float* d_queries, int nq, int k, int* d_idx, float* d_d2) {
    if (!C.knn_built) throw ApiError{ALOAM_E_STATE, "aloam_knn_query before aloam_knn_build"};
    if (nq < 0 || k < 1 || k > 8 || (nq > 0 && (!d_queries || !d_idx || !d_d2)))
        throw ApiError{ALOAM_E_ARG, "bad knn query args (device pointers, 1 <= k <= 8)"};
    const float radius = C.knn_radius;
    // profiling: the timed launch runs without candidate counters (one same-address atomic per wave
    // would be on the measured path); an untimed second launch (identical results) counts them
    auto launch = [&](unsigned long long* cnt) {
        if (C.knn_two_phase)
            knn_device_2phase_launch(C, C.g_knn_fine, C.g_knn, (const float4*)d_queries, nq, k, radius, d_idx, d_d2, cnt);
        else
            knn_device_launch(C, C.g_knn, (const float4*)d_queries, nq, k, radius, d_idx, d_d2, cnt);
    };
    if (C.profiling) HIPCHK(hipEventRecord(C.ev[Ctx::NEV - 2], C.stream));
    launch(nullptr);
    if (C.profiling) {
        HIPCHK(hipEventRecord(C.ev[Ctx::NEV - 1], C.stream));
        HIPCHK(hipMemsetAsync(C.d_cand, 0, sizeof(unsigned long long) * 2, C.stream));
        launch(C.d_cand);
    }
    unsigned long long cand[2] = {0, 0};
    if (C.profiling) {
        HIPCHK(hipMemcpyAsync(cand, C.d_cand, sizeof(cand), hipMemcpyDeviceToHost, C.stream));
    }
    sync(C);
    if (C.profiling) {
        C.timing.knn_ms = ev_ms(C, Ctx::NEV - 2, Ctx::NEV - 1);
        C.timing.knn_launches = 1;
        // B = sum_q [16 + 16 |C27(q)|] + 8 k Q
        C.timing.knn_bytes = 16.0 * nq + 16.0 * (double)cand[0] + 8.0 * k * (double)nq;
        C.timing.knn_streamed_bytes = 16.0 * nq + 16.0 * (double)cand[1] + 8.0 * k * (double)nq;
    }
}

int aloam_knn_build(aloam_ctx* ctx, const float* d_pts, int n, float radius) {
    API_BEGIN(ctx)
    knn_build(C, d_pts, n, radius);
    API_END
}

int aloam_knn_query(aloam_ctx* ctx, const float* d_queries, int nq, int k, int* d_idx, float* d_d2) {
    API_BEGIN(ctx)
    knn_query(C, d_queries, nq, k, d_idx, d_d2);
    API_END
}

int aloam_knn_device(aloam_ctx* ctx, const float* d_pts, int n, const float* d_queries, int nq, int k, float radius,
                     int* d_idx, float* d_d2) {
    API_BEGIN(ctx)
    if (n < 0 || nq < 0 || k < 1 || k > 8 || !(radius > 0) || (n > 0 && !d_pts) || (nq > 0 && (!d_queries || !d_idx || !d_d2)))
        throw ApiError{ALOAM_E_ARG, "bad knn args (device pointers, radius > 0, 1 <= k <= 8)"};
    knn_build(C, d_pts, n, radius);
    knn_query(C, d_queries, nq, k, d_idx, d_d2);
    API_END
}

const char* aloam_knn_kernel(const aloam_ctx* ctx) {
    if (!ctx) return "";
    return reinterpret_cast<const Ctx*>(ctx)->knn_kernel;
}

int aloam_serial_sort_fallbacks(unsigned long long* count) {
    if (!count) return ALOAM_E_ARG;
    try {
        *count = serial_sort_calls_map() + serial_sort_calls_scan() + serial_sort_calls_voxel();
        return ALOAM_OK;
    } catch (...) {
        return ALOAM_E_HIP;
    }
}

int aloam_set_cu_mask(aloam_ctx* ctx, const unsigned* mask, int nwords) {
    API_BEGIN(ctx)
    if (nwords < 0 || (nwords > 0 && !mask)) throw ApiError{ALOAM_E_ARG, "bad CU mask"};
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, C.device));
    int n = 0;
    for (int w = 0; w < nwords; w++)
        for (int b = 0; b < 32; b++)
            if (w * 32 + b < prop.multiProcessorCount && ((mask[w] >> b) & 1u)) n++;
    if (nwords > 0 && n == 0) throw ApiError{ALOAM_E_ARG, "CU mask selects no CU"};
    HIPCHK(hipStreamSynchronize(C.stream));
    HIPCHK(hipStreamSynchronize(C.stream2));
    if (C.stream3) HIPCHK(hipStreamSynchronize(C.stream3));
    C.cu_mask.assign(mask, mask + nwords);
    hipStream_t s1 = make_stream(C), s2 = make_stream(C), s3 = C.stream3 ? make_stream(C, true) : nullptr;
    (void)hipStreamDestroy(C.stream);
    (void)hipStreamDestroy(C.stream2);
    if (C.stream3) (void)hipStreamDestroy(C.stream3);
    C.stream = s1;
    C.stream2 = s2;
    C.stream3 = s3;
    C.n_cus = nwords > 0 ? n : prop.multiProcessorCount;
    API_END
}

int aloam_set_profiling(aloam_ctx* ctx, int enable) {
    API_BEGIN(ctx)
    C.profiling = enable != 0;
    std::memset(&C.timing, 0, sizeof(C.timing));
    API_END
}

int aloam_get_timing(aloam_ctx* ctx, aloam_timing* t) {
    API_BEGIN(ctx)
    if (!t) throw ApiError{ALOAM_E_ARG, "null timing"};
    *t = C.timing;
    API_END
}

int aloam_s2m_set_map(aloam_ctx* ctx, const float* corner, int nc, const float* surf, int ns, int flags) {
    API_BEGIN(ctx)
    if (nc < 0 || ns < 0 || (nc > 0 && !corner) || (ns > 0 && !surf)) throw ApiError{ALOAM_E_ARG, "bad map"};
    s2m_set_map(C, corner, nc, surf, ns, flags);
    API_END
}

int aloam_s2m_set_queries(aloam_ctx* ctx, const float* corner, int ncq, const float* surf, int nsq, int flags) {
    API_BEGIN(ctx)
    if (ncq < 0 || nsq < 0 || (ncq > 0 && !corner) || (nsq > 0 && !surf)) throw ApiError{ALOAM_E_ARG, "bad query stacks"};
    s2m_set_queries(C, corner, ncq, surf, nsq, flags);
    API_END
}

int aloam_s2m_register(aloam_ctx* ctx, double x[7], aloam_s2m_result* out) {
    API_BEGIN(ctx)
    if (!x) throw ApiError{ALOAM_E_ARG, "null pose"};
    s2m_register(C, x, out);
    API_END
}

int aloam_s2m_register_group(aloam_ctx** ctxs, int world, double x[7], aloam_s2m_result* out) {
    if (!ctxs || world < 1 || world > ALOAM_S2M_RECORDS || !x) return ALOAM_E_ARG;
    for (int r = 0; r < world; r++) if (!ctxs[r]) return ALOAM_E_ARG;
    API_BEGIN(ctxs[0])
    s2m_register_group((Ctx**)ctxs, world, x, out);
    API_END
}

int aloam_shard_unique_id(unsigned char id[128]) {
    if (!id) return ALOAM_E_ARG;
    try {
        shard_unique_id(id);
    } catch (const ApiError& e) {
        g_create_err = e.msg;
        return e.code;
    }
    return ALOAM_OK;
}

int aloam_shard_init(aloam_ctx* ctx, int rank, int world, const unsigned char* id) {
    API_BEGIN(ctx)
    shard_init(C, rank, world, id);
    API_END
}

int aloam_shard_peer_handle(aloam_ctx* ctx, unsigned char handle[ALOAM_PEER_HANDLE_BYTES]) {
    API_BEGIN(ctx)
    if (!handle) throw ApiError{ALOAM_E_ARG, "null handle"};
    shard_peer_handle(C, handle);
    API_END
}

int aloam_shard_peer_open(aloam_ctx* ctx, const unsigned char* handles, int world, int rank) {
    API_BEGIN(ctx)
    shard_peer_open(C, handles, world, rank);
    API_END
}

int aloam_shard_peer_close(aloam_ctx* ctx) {
    API_BEGIN(ctx)
    shard_peer_close(C);
    API_END
}

int aloam_shard_slot_range(int n_slots, int rank, int world, int* begin, int* end) {
    return shard_slot_range(n_slots, rank, world, begin, end);
}

}  // extern "C"
