// aloam_internal.hpp — context layout and kernel-launch entry points shared by the .hip files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <cstdio>
#include <functional>
#include <string>
#include <mutex>
#include <vector>

#include "../../include/aloam_hip.h"

namespace aloam {

constexpr int MAXL = 128;            // scan lines supported on device
constexpr int LINE_SHARP_CAP = 12;   // 2 per segment x 6   (scanRegistration.cpp:301)
constexpr int LINE_LSHARP_CAP = 120; // 20 per segment x 6  (:307)
constexpr int LINE_FLAT_CAP = 24;    // 4 per segment x 6   (:359)
constexpr int ODOM_CNT_SLOTS = 64, ODOM_CNT_STRIDE = 16;   // odometry search counters: 64 lines of 64 B per round
constexpr int LINE_LDS_CAP = 4096;   // points per line kept in LDS (larger lines use global scratch)
constexpr int CUBE_W = 21, CUBE_H = 21, CUBE_D = 11, CUBE_N = 21 * 21 * 11;  // laserMapping.cpp:74-82
constexpr int GRID_MAX_CELLS = 1 << 23;        // default cell cap of a grid (the cell grows x1.25 until it fits)
constexpr int GRID_MAX_CELLS_BIG = 1 << 26;    // cap of the large-map search grids (C4 index, s2m): down to a 0.2 m cell over ~120 x 100 x 25 m

// ---- device-resident bookkeeping of scanRegistration ----
struct ScanMeta {
    int n_in, n_cl, jstar, cloud_size;
    int counts[5];                 // full, sharp, less_sharp, flat, less_flat
    int line_off[MAXL + 1];
};

// ---- dense uniform grid over a point set (kd-tree-free radius search) ----
constexpr int MC_CAP_PTS = 64;   // cached candidates per mapping query (k_map.hip MC_CAP)
struct GridDesc {
    unsigned bb[6];                // ordered-encoded bbox: min xyz, max xyz
    float ox, oy, oz, cell, inv_cell;
    int dx, dy, dz, ncells, n;
    int nlayers;                   // > 1: cells also split by scan line (layer = int(intensity))
    int n_acc;                     // build-time counter (published to n by the scatter)
    int npass;                     // radix build: 9-bit digit passes the cell keys need
    int ticket;                    // radix build: bbox tiles done (the last one reduces the partials)
};
struct Grid {
    GridDesc* desc = nullptr;      // device
    int* cell_count = nullptr;     // GRID_MAX_CELLS (all zero between builds)
    int* cell_start = nullptr;     // GRID_MAX_CELLS + 1
    int* blk = nullptr;            // scan scratch
    float4* pts = nullptr;         // points sorted by cell
    int* idx = nullptr;            // original index of each sorted point
    int* pcell = nullptr;          // cell of each input point
    int nlayers = 1;
    bool w_index = false;          // sorted copy carries the original index in w (search-only grids)
    bool flat = false;             // one z cell (2-D cells per layer: a scan line is a thin cone)
    int cap = 0;
    float min_cell = 1.f;
    int max_cells = GRID_MAX_CELLS;
    // radix build scratch (large grids, grid_build_radix): key / index ping-pong, (digit, tile) counts
    unsigned* rk[2] = {nullptr, nullptr};
    int* rv[2] = {nullptr, nullptr};
    int* rH = nullptr;
    int* rHo = nullptr;
    int* rblk = nullptr;
    unsigned* rbb = nullptr;      // per-tile bbox partials (7 words per tile)
    int* rcf = nullptr;           // per chunk of the cell-start array: its first run head (k_gr_starts)
    int rcap = 0;
};

// ---- Ceres-equivalent LM state (device) ----
struct LMState {
    double x[7], cand[7];
    double A[21], g[6];            // current (unscaled) JtJ upper triangle, gradient Jt r
    double cost, initial_cost;
    double scale[6], diag[6];
    double radius, decrease_factor, x_norm, mcc, step_norm;
    double inv_radius, inv_mcc;    // k_lm_coop's tail: 1 / radius (the step needs only that), 1 / mcc (lm_post)
    double delta[6];               // the last step in tangent space (k_lm_coop: its model cost change and
                                   // norm are computed off the critical path, lm_post)
    int reuse_diag, iteration, done, termination, successful, nres;
    int pending, invalid;          // lm_post owed for `delta`; the step it checked was invalid (mcc < 0)
    unsigned ticket;
};

// ---- the sharded registration's record exchange on the device (k_s2m_solve, k_s2m.hip) ----
constexpr int S2M_PEER_MAX = 8;    // ranks of a device-side exchange (one node)
constexpr int S2M_BARS = 16;       // barrier / arrival counters per rank, 32 unsigned apart
struct S2MPeers {
    double* recs;                  // [2][nrec][32] this rank's gathered records (parity = global pass & 1)
    unsigned* gath;                // [S2M_BARS x 32] local barrier counters, monotonic
    unsigned* base;                // global passes run by this rank's earlier Solves (the same on every rank)
    double* xrec[S2M_PEER_MAX];    // every rank's exported records [2][nrec][32] (uncached memory; peers over xGMI)
    unsigned* xarr[S2M_PEER_MAX];  // every rank's arrival counters [S2M_BARS x 32] (uncached, monotonic)
    int world, rank, rp;           // rp: record blocks per rank (slice_of)
};

struct OdomState {                 // laserOdometry.cpp:123-137
    double para[7];                // q_last_curr (x,y,z,w), t_last_curr
    double q_w[4], t_w[3];
};
struct MapState {                  // laserMapping.cpp:58-120
    double parameters[7];          // q_w_curr, t_w_curr
    double q_wmap_wodom[4], t_wmap_wodom[3];
    double q_wodom[4], t_wodom[3];
    int cenW, cenH, cenD;
    int shift[3];                  // cube shift applied this frame
    int cI, cJ, cK;
    int valid_num;
    int valid_ind[125];
    int optimize;                  // map corner > 10 && surf > 50
    int n_corner_map, n_surf_map;  // FromMap sizes
    int n_corner_stack, n_surf_stack;
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// Per-frame results in ONE device block, so each stage returns them with a single D2H copy into a
// pinned mirror (odometry: [odom .. lm_sum], mapping: the whole block).
struct DevOut {
    OdomState odom;
    int round_cnt[4 * ALOAM_MAX_ROUNDS];
    aloam_lm_summary lm_sum[2 * ALOAM_MAX_ROUNDS];
    int map_n[2];
    int stack_n[4];                  // [set][corner, surf]
    unsigned long long cand[2];
    MapState map;
};
struct KindScratch {               // per-lane scratch for the map kinds' concurrent work
    unsigned long long *vkeys = nullptr, *vkeys2 = nullptr;   // 2 x cap_voxel, cap_voxel
    int *vvals = nullptr, *vvals2 = nullptr;                  // cap_voxel, cap_voxel + 64
    float4* ins_pts = nullptr;
    int *ins_val = nullptr, *ins_val2 = nullptr;
    unsigned long long* seg_keys = nullptr;                   // 4 x cap_map + 32768
    int* cube_segl = nullptr;                                 // per surrounding cube: sort segment list (125 x LS_SEGL)
    int* blk = nullptr;
    float4* map_tmp = nullptr;
};
struct Ctx {
    aloam_params P;
    int device = 0;
    std::string err;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;   // mapping: the surf half of the per-kind work runs here (fork/join)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t ev_stkn = nullptr;    // stream2: the early stacks took their input counts (aloam_api.hip publish)
    hipEvent_t ev_handoff = nullptr; // device-to-device hand-offs: the source stream waits on it
    hipEvent_t ev_scan = nullptr, ev_lf = nullptr;   // per-line VoxelGrid on stream2: after the line kernel / done
    bool profiling = false;
    aloam_timing timing{};
    std::vector<DevBuf> bufs;

    // ---- scanRegistration ----
    int cap_in = 0;
    float4* d_in = nullptr;        // raw points staging
    unsigned char* d_pc2 = nullptr; // PointCloud2 blob staging (grown on demand)
    size_t cap_pc2 = 0;
    float4* d_cl = nullptr;        // after NaN / range filter
    int* d_sid = nullptr;          // scanID per filtered point (-1 = dropped)
    float* d_ori = nullptr;        // raw -atan2f per filtered point
    int* d_blk = nullptr;          // block scratch
    int* d_hist = nullptr;         // line x block histogram
    int* d_hoff = nullptr;         // its exclusive scan: each (line, block)'s first slot in laserCloud
    float4* d_cloud = nullptr;     // laserCloud (line ordered, intensity)
    float* d_curv = nullptr;
    float4* d_scratch_xyz = nullptr;   // per-line scratch for lines above the LDS cap
    unsigned long long* d_scratch_keys = nullptr;
    int* d_scratch_i = nullptr;
    int* d_line_sharp = nullptr;   // [MAXL][12]
    int* d_line_lsharp = nullptr;  // [MAXL][120]
    int* d_line_flat = nullptr;    // [MAXL][24]
    int* d_line_cnt = nullptr;     // [MAXL][4] sharp, lsharp, flat, lessflat
    float4* d_line_lf = nullptr;   // per-line less-flat centroids at line offsets
    ScanMeta* d_meta = nullptr;
    ScanMeta h_meta{};
    ScanMeta* h_meta_pin = nullptr;  // pinned landing slot of the async meta copy
    bool meta_pending = false;       // scanRegistration's counts are in flight to h_meta_pin (no sync yet)
    bool lf_pending = false;         // the per-line VoxelGrid runs on stream2 (stream waits on ev_lf before its results)
    bool lf_side = false;            // the last registration ran its per-line VoxelGrid on stream2
    bool meta_deferred = false;      // the counts copy is queued later (queue_meta, behind the ev_lf wait)
    int last_nslots = 0;             // the previous scan's odometry factor count (LM grid hint)
    int stack_hint[2] = {0, 0};      // launch / sort sizes of the next publish's stack VoxelGrids (0: caps)
    // scanRegistration outputs (the "current" features)
    float4 *d_sharp = nullptr, *d_lsharp = nullptr, *d_flat = nullptr, *d_lflat = nullptr;
    int *d_sharp_idx = nullptr, *d_lsharp_idx = nullptr, *d_flat_idx = nullptr;
    int n_full = 0, n_sharp = 0, n_lsharp = 0, n_flat = 0, n_lflat = 0;
    bool have_features = false;
    bool features_from_host = false;
    bool features_swapped = false;     // odometry moved less_sharp/less_flat into the last-cloud slots

    // ---- laserOdometry ----
    bool odom_inited = false;
    bool odom_spread_dirty = false;  // search counters written since the last k_odom_compose re-zeroed them
    int odom_frame_count = 0;
    OdomState* d_odom = nullptr;
    OdomState h_odom{};
    float4 *d_corner_last = nullptr, *d_surf_last = nullptr;
    int n_corner_last = 0, n_surf_last = 0;
    Grid g_corner_last, g_surf_last;
    Grid g_corner_win, g_surf_win;  // scan-line-layered grids of the last clouds (window search)
    Grid g_corner_fine, g_surf_fine;  // fine grids of the last clouds (first 1-NN phase, k_odom.hip)
    Grid g_knn;                     // aloam_knn_device (grown on demand): radius-edge cells
    Grid g_knn_fine;                // its fine grid (first search phase, k_knn_2phase)
    char knn_kernel[48] = "";        // the search kernel the last aloam_knn_device call launched
    int* d_knn_n = nullptr;
    // aloam_knn_build's index (the map's two grids), queried by aloam_knn_query until the next build
    bool knn_built = false, knn_two_phase = false;
    float knn_radius = 0.f;
    int knn_n = 0;
    aloam_factor* d_factors = nullptr;
    int cap_factors = 0;
    LMState* d_lm = nullptr;
    double* d_partials = nullptr;
    unsigned long long* d_lm_recs = nullptr;  // 2 x 128 x 32 u64: LM pass partial records + tags (double-buffered)
    unsigned long long* d_lm_seq = nullptr;   // LM launch sequence number (record tags = seq*256 + pass + 1)
    int map_slots_hint = 0;          // last mapping frame's stack sizes (LM grid sizing only)
    int* d_last_sorted = nullptr;    // [2]: corner_last / surf_last ordered by scan line
    int* d_bar_err = nullptr;        // set if a grid barrier timed out (device view of h_bar_err)
    int* h_bar_err = nullptr;        // mapped pinned host word
    aloam_lm_summary* d_lm_sum = nullptr;   // [ALOAM_MAX_ROUNDS]
    int* d_round_cnt = nullptr;             // [ALOAM_MAX_ROUNDS][2] correspondences per round
    int* d_odom_spread = nullptr;           // [ALOAM_MAX_ROUNDS][ODOM_CNT_SLOTS][ODOM_CNT_STRIDE] search counters
    int* d_map_spread = nullptr;            // the same for the mapping association

    // ---- laserMapping ----
    MapState* d_map = nullptr;
    MapState h_map{};
    int cap_map = 0;
    float4* d_mc = nullptr; int* d_mc_cube = nullptr;    // corner map, sorted by cube
    float4* d_ms = nullptr; int* d_ms_cube = nullptr;    // surf map
    float4* d_mc2 = nullptr; int* d_mc2_cube = nullptr;  // double buffers
    float4* d_ms2 = nullptr; int* d_ms2_cube = nullptr;
    int n_mc = 0, n_ms = 0;                              // host-known sizes: exact when no mapping frame is in
                                                         // flight, else upper bounds (+ in-flight stack sizes)
    int* d_map_n = nullptr;                              // device sizes [2]
    int* d_cube_cnt = nullptr;                           // [2][CUBE_N + 1]
    int* d_cube_off = nullptr;                           // [2][CUBE_N + 1]
    unsigned char* d_cube_valid = nullptr;               // [CUBE_N]
    Grid g_map_corner, g_map_surf;
    // mapping input, double-buffered (MapInSet): odometry publishes / a hand-off is forwarded into the set
    // frame k does not read; the current set is mset[in_cur], aliased by the d_map_*_in / n_map_*_in fields
    struct MapInSet {
        float4 *corner = nullptr, *surf = nullptr, *full = nullptr;
        int* n = nullptr;                  // device [4]: corner / surf counts; [2..3] the early stacks' input counts
        double* pose = nullptr;            // device [8]: q_wodom[4], t_wodom[3] (laser_odom_to_init)
        float4 *cstack = nullptr, *sstack = nullptr;   // the frame's VoxelGrid'ed stacks (:542-550)
        int nc = 0, ns = 0, nf = 0;        // host counts
        bool stacks = false;               // stacks already voxelised on stream3 (event `ready`)
        bool stacks_pub = false;           // stacks present in cstack / sstack (voxelised at publish, or
                                           // copied in with a hand-off); counts in DevOut::stack_n[2 set]
        hipEvent_t ready = nullptr;        // stream3: stacks of this set done
        hipEvent_t released = nullptr;     // stream: the last frame reading this set done
        hipEvent_t fwd = nullptr;          // stream: the publish copy into this set done (aloam_odometry
                                           // returns before it ends)
        bool fwd_rec = false;              // `fwd` has been recorded for the set's current contents
        // a hand-off's stacks copy deferred to just before the frame's rounds (forward_snapshot): the
        // prepare and grid builds need only the clouds and the pose, so they overlap the source's stacks
        bool pstk = false;
        const float4* pstk_src[2] = {nullptr, nullptr};
        int pstk_n[2] = {0, 0};
        const int* pstk_ndev = nullptr;
        hipEvent_t pstk_ready = nullptr, pstk_copied = nullptr;
        std::mutex* pstk_mu = nullptr;     // the source's capture mutex (MapSnapshot::src_capture_mu)
    };
    MapInSet mset[2];
    int in_cur = 0;
    float4 *d_map_corner_in = nullptr, *d_map_surf_in = nullptr, *d_map_full_in = nullptr;
    int n_map_corner_in = 0, n_map_surf_in = 0, n_map_full_in = 0;
    hipStream_t stream3 = nullptr;       // mapping: forward + stack VoxelGrid of the next hand-off (created on first use)
    bool publish_stacks = false;         // odometry publish also voxelises the mapping stacks (pipeline front)
    std::vector<unsigned> cu_mask;       // aloam_set_cu_mask (empty: all CUs), applied to stream / stream2
    std::vector<unsigned> cu_mask_side;  // stream3's CUs (empty: cu_mask); disjoint from cu_mask keeps the
                                         // cross-workgroup LM kernels of `stream` co-resident
    KindScratch ksv;                     // stack VoxelGrid scratch of stream3
    int* d_tmp_n = nullptr;              // [2] counts scratch of the utility entry points
    int* d_nbr = nullptr;                                // [queries][5] neighbour slots
    // mapping rounds' per-query candidate cache (k_map.hip MapCache): centres, points, positions, last neighbours
    float4* d_mc_ctr = nullptr; float4* d_mc_pts = nullptr; int* d_mc_pos = nullptr; int* d_mc_prev = nullptr;
    int cap_mq = 0;

    int* d_s2m_nbr = nullptr; int cap_s2m_nbr = 0;       // split registration association: parked neighbours
    float4* d_registered = nullptr;
    int n_registered = 0;
    bool have_map_input = false;
    int map_frame_count = 0;
    // voxel-grid scratch
    unsigned long long *d_vkeys = nullptr, *d_vkeys2 = nullptr;
    int *d_vvals = nullptr, *d_vvals2 = nullptr;
    int cap_voxel = 0;
    // insertion scratch
    float4* d_ins_pts = nullptr; int* d_ins_val = nullptr; int* d_ins_val2 = nullptr;
    float4* d_map_tmp = nullptr;                         // per-cube filter output (map capacity)
    unsigned long long* d_seg_keys = nullptr;            // per-cube filter key scratch (4 x map capacity)
    int* d_map_in_n = nullptr;                           // [2] corner / surf input counts of mset[in_cur] (device)
    int* d_last_n = nullptr;                             // [2] corner_last / surf_last counts (device)
    unsigned long long* d_cand = nullptr;                // [2] candidate counters (profiling)

    // profiling events: [0..1] scan, [2..3] odom, [4..5] map, search pairs after that
    static constexpr int NEV = 6 + 4 * ALOAM_MAX_ROUNDS + 2;   // last two: aloam_knn_device
    hipEvent_t ev[NEV];
    // phase boundaries inside a stage (profiling only) for the TicToc stage surface (ALOAM_TT_*)
    enum PhaseMark { PM_SCAN_PREP, PM_SCAN_CURV, PM_ODOM_ROUNDS_END, PM_MAP_SHIFT, PM_MAP_GRIDS, PM_MAP_ROUNDS_BEGIN,
                     PM_MAP_ROUNDS_END, PM_MAP_ADD, PM_MAP_FILTER, PM_N };
    hipEvent_t evp[PM_N];
    KindScratch ks[2];
    DevOut* d_out = nullptr;         // device results block (d_odom, d_round_cnt, ... point into it)
    DevOut* h_out = nullptr;         // pinned host mirror
    // laserMapping frames in flight (mapping_issue / mapping_complete): per parity a pinned results
    // mirror, the event after its copy, and what the host needs back from that frame
    DevOut* h_mout[2] = {nullptr, nullptr};
    hipEvent_t ev_mdone[2] = {nullptr, nullptr};
    long m_issued = 0, m_done = 0;
    int m_pend[2][2] = {{0, 0}, {0, 0}};  // corner / surf stack upper bounds of the frame (map growth)
    int m_nfull[2] = {0, 0};
    int m_set[2] = {0, 0};               // input set of the frame
    int m_frame[2] = {0, 0};             // frameCount of the frame (laserMapping.cpp:806,823,888)
    // the odometry -> map correction of the latest completed frame (/aft_mapped_to_init_high_frec):
    // written by mapping_complete, read by aloam_map_high_freq_pose from any thread
    std::mutex hf_mu;
    double hf_q[4] = {0, 0, 0, 1}, hf_t[3] = {0, 0, 0};
    struct GraphSlot { const void* key[2] = {nullptr, nullptr}; int n = -1; hipGraphExec_t exec = nullptr; };
    GraphSlot graphs[4];             // 0,1: odometry rounds (last-cloud buffer parity), 2,3: mapping rounds (input set)
    bool use_graphs = true;          // round loops replayed as HIP graphs when not profiling
    // held while `stream` is being captured: another thread making its stream wait on an event of this
    // context (the pipeline front on a hand-off's `copied`) must not do so mid-capture, or HIP fails the
    // wait with hipErrorStreamCaptureIsolation
    std::mutex capture_mu;
    // an odometry scan issued but not yet completed (do_odometry_issue -> do_odometry_complete)
    struct FrontPend { aloam_odom_result r; bool pend; int t, hint_c, hint_s; };
    FrontPend fp{};
    bool fp_active = false;
    std::string front_failed;      // a publish's hand-off wait failed mid-scan: the front state is half-advanced
    // run right before the next publish launch (2-stage pipeline: wait until the mapping stage has copied
    // the hand-off that last used the target input set), then cleared; the scan's registration and
    // odometry rounds are queued by then, so the wait holds back the publish only
    std::function<void()> pre_publish;
    int* d_odom_nq = nullptr;        // [2]: sharp / flat counts of the current scan (device copy)
    bool ev_ready = false;
    std::chrono::steady_clock::time_point t_rounds_issued{};   // host-issue profiling (ALOAM_HOST_TIMING)
    double t_issue_us = 0, t_pre_us = 0;

    // ---- scan-to-map registration (k_s2m.hip) and its shard communicator ----
    struct S2M* s2m = nullptr;       // allocated by the first aloam_s2m_* call
    int shard_rank = 0, shard_world = 1;
    int n_cus = 256;                 // CUs this context's streams may use (CU mask popcount; caps co-resident grids)
    void* shard_comm = nullptr;      // ncclComm_t (world > 1)
};

// error helpers
#define HIPCHK(x)                                                                        \
    do {                                                                                 \
        hipError_t _e = (x);                                                             \
        if (_e != hipSuccess) {                                                          \
            throw HipError(std::string(#x) + ": " + hipGetErrorString(_e));              \
        }                                                                                \
    } while (0)
struct HipError {
    std::string msg;
    explicit HipError(std::string m) : msg(std::move(m)) {}
};
struct ApiError {
    int code;
    std::string msg;
};

// ---- launch entry points (defined in the k_*.hip files) ----
void scan_registration_launch(Ctx& C, const float4* in, int n, bool side);
void grid_build(Ctx& C, Grid& g, const float4* pts, const int* d_n, int cap_n, const int* cube_of, const unsigned char* cube_valid);
struct GridBuild { Grid* g; const float4* pts; const int* d_n; int cap_n; const int* cube_of; const unsigned char* cube_valid; };
constexpr int GRID_MULTI_MAX = 6;
void grid_build_multi(Ctx& C, const GridBuild* b, int n);   // up to GRID_MULTI_MAX grids in one set of launches
void knn_device_launch(Ctx& C, Grid& g, const float4* q, int nq, int k, float radius, int* idx, float* d2,
                       unsigned long long* cand);
void knn_device_2phase_launch(Ctx& C, Grid& gf, Grid& gc, const float4* q, int nq, int k, float radius, int* idx, float* d2,
                              unsigned long long* cand);
void grid_alloc(Ctx& C, Grid& g, int cap, float min_cell, int nlayers = 1, bool w_index = false, bool flat = false,
                int max_cells = GRID_MAX_CELLS);
void odom_round_search(Ctx& C, int round);
unsigned long long serial_sort_calls_map();
unsigned long long serial_sort_calls_scan();
unsigned long long serial_sort_calls_voxel();
void rebuild_init(Ctx& C);
void forward_stacks_pending(Ctx& C, int t);
void set_counts2(Ctx& C, int* dst, int a, int b);
// also sets d_last_n (from dcnt[2], dcnt[4] when dcnt = the device ScanMeta counts, else the host values)
// and re-arms d_last_sorted
void odom_compose(Ctx& C, int last_corner_n, int last_surf_n, const int* dcnt = nullptr);
// nslots = host upper bound; d_nslots2 (optional, device int[2]) = live slots as a sum of two counts
void odom_last_sorted(Ctx& C, bool flags_preset = false);
// runs issue() through a cached HIP graph of C.stream keyed by (k0, k1, n) in slot
void run_graph(Ctx& C, int slot, const void* k0, const void* k1, int n, const std::function<void()>& issue);
void lm_init(Ctx& C);   // one-time kernel attributes (before any graph capture)
void lm_run(Ctx& C, const aloam_factor* d_f, int nslots, double* d_x, int round, const int* gate, const int* d_nslots2 = nullptr,
            int live_hint = 0);
void lm_eval_only(Ctx& C, const aloam_factor* d_f, int n, const double* d_x, int robust, double* d_res, double* d_jac, double* d_neq);
void knn_launch(Ctx& C, Grid& g, const float4* q, int nq, int k, float radius, int* idx, float* d2);
// PCL VoxelGrid of one cloud / a pair of clouds (k_voxel.hip, one workgroup per cloud). The count is read
// on the device and clamped to cap (a hinted launch). lane 0: C.stream + the primary scratch; lane 1:
// C.stream2 + the second scratch set
void voxel_grid_sorted_on(Ctx& C, hipStream_t st, KindScratch& K, const float4* pts, const int* d_n, int cap_n, float leaf,
                          float4* out, int* d_nout);
void voxel_grid_pair_on(Ctx& C, hipStream_t st, KindScratch& K, const float4* ptsA, const int* d_nA, int capA, float leafA,
                        float4* outA, int* d_noutA, const float4* ptsB, const int* d_nB, int capB, float leafB, float4* outB,
                        int* d_noutB);
void voxel_grid_sorted(Ctx& C, const float4* pts, const int* d_n, int cap_n, float leaf, float4* out, int* d_nout, int lane = 0);
void fork_lane1(Ctx& C);   // stream2 waits for everything queued on stream so far
void join_lane1(Ctx& C);   // stream waits for everything queued on stream2 so far
void map_frame_launch(Ctx& C, int input_set);
void* dalloc(Ctx& C, size_t bytes);
void dfree(Ctx& C, void* p);           // a dalloc'd buffer given back (after the context's stream drains)
void grid_free(Ctx& C, Grid& g);
void prof_phase(Ctx& C, int k);     // records evp[k] on C.stream when profiling
// the odometry -> mapping hand-off as a value: published buffers (valid until the publish after next),
// counts and pose; the native pipeline forwards it from its mapping thread (aloam_api.hip)
struct MapSnapshot {
    const float4* src[3]; int n[3]; double pose[7];
    bool has_stacks = false;           // the source voxelised the stacks (publish_stacks): copied along
    const float4* stk[2] = {nullptr, nullptr};
    const int* stk_n = nullptr;        // device [2]
    hipEvent_t stk_ready = nullptr;    // source stream2: stacks done
    hipEvent_t fwd_done = nullptr;     // source stream: the publish copy into src[] done
    // the source context's capture mutex: HIP fails a wait on an event whose stream is being captured
    // (hipErrorStreamCaptureIsolation), so waits on the source's events are made under it
    std::mutex* src_capture_mu = nullptr;
};
void snapshot_mapping_input(Ctx& S, MapSnapshot* out);
// scanRegistration + laserOdometry of one scan split at its sync (2-stage pipeline front)
void front_issue(Ctx& C, const float* xyzr, int n, int flags);
void front_complete(Ctx& C, aloam_odom_result* R);
void forward_snapshot(Ctx& C, const MapSnapshot& s, hipEvent_t copied, bool defer_stacks = false);
// laserMapping split in two so the host can issue frame k while the GPU still runs frame k-1 (at most
// two frames in flight; every launch size of frame k is an upper bound known before k-1 completes)
void mapping_issue(Ctx& C);
void use_input_set(Ctx& C, int t);
hipStream_t make_stream(Ctx& C, bool side = false);   // a stream on the context's (side) CU mask
void set_side_cu_mask(Ctx& C, const unsigned* mask, int nwords);   // mset[t] becomes the current mapping input (aliases updated)
void mapping_complete(Ctx& C, aloam_map_result* R);
bool mapping_ready(Ctx& C);          // the oldest frame in flight has finished on the GPU
// scan-to-map registration + shard communicator (k_s2m.hip)
void s2m_set_map(Ctx& C, const float* corner, int nc, const float* surf, int ns, int flags);
void s2m_set_queries(Ctx& C, const float* corner, int ncq, const float* surf, int nsq, int flags);
void s2m_register(Ctx& C, double* x, aloam_s2m_result* out);
void s2m_register_group(Ctx** cs, int world, double* x, aloam_s2m_result* out);
void s2m_release(Ctx& C);
void shard_unique_id(unsigned char* id);
void shard_init(Ctx& C, int rank, int world, const unsigned char* id);
int shard_slot_range(int n_slots, int rank, int world, int* begin, int* end);
void shard_peer_handle(Ctx& C, unsigned char* out);
void shard_peer_open(Ctx& C, const unsigned char* handles, int world, int rank);
void shard_peer_close(Ctx& C);

}  // namespace aloam
