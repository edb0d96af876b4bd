// k_s2m.hip — scan-to-map registration with the query stacks sharded over ranks (host side).
//
// The registration half of laserMapping::process (src/laserMapping.cpp:556-727) against a map the
// caller supplies: per round, k_s2m_assoc (k_map.hip: pointAssociateToMap + 5-NN within 1 m + line /
// plane fit, 8 lanes per query) over this rank's slots, then one Ceres-equivalent Solve as
// max_iter + 1 passes of {k_s2m_pass -> exchange} + k_s2m_final (k_lm.hip; each pass launch first
// finishes the previous pass's LM step in every workgroup). The exchange is the
// only collective of the path: one 32-double record per fixed slot block,
//   * world 1:   none (the tail reads the local records),
//   * RCCL:      ncclAllGather on the context's stream (one process per GPU, xGMI),
//   * group:     peer copies between the streams of contexts driven by one thread
//                (aloam_s2m_register_group: several ranks on one GPU, or one process over several),
//   * device:    no host in the exchange at all (aloam_shard_peer_open, or group mode with
//                ALOAM_S2M_PEER=1): each Solve is ONE persistent launch per rank (k_s2m_solve) whose
//                workgroups export their records into uncached memory the peers map (IPC over xGMI),
//                announce them on monotonic arrival counters and gather the peers' records themselves.
// Because the block decomposition and the reduction order are global, every rank, in every mode and
// world size, runs the bitwise-identical LM tail.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "aloam_internal.hpp"

namespace aloam {

void s2m_assoc_launch(Ctx& C, const float4* cq, const float4* sq, int nc, int s0, int s1, const double* d_x, Grid& gc, Grid& gs,
                      const Grid* gcf, const Grid* gsf, const float4* cmap, const float4* smap, aloam_factor* out);
void s2m_pass_launch(Ctx& C, const aloam_factor* f, int nslots, int per, int rec0, int nrec_local, int nrec, const double* prev,
                     const LMState* st_in, LMState* st_out, const double* x0, int pass, aloam_lm_summary* sum, int* round_cnt,
                     double* send);
void s2m_final_launch(Ctx& C, const double* prev, int nrec, const LMState* st_in, double* x, int last_pass, aloam_lm_summary* sum);
int s2m_solve_grid(Ctx& C, int world, int rp, bool group);
void s2m_solve_launch(Ctx& C, int G, const aloam_factor* f, int nslots, int per, int nrec, const S2MPeers& T, double* x,
                      LMState* st_out, aloam_lm_summary* sum, int* round_cnt);

constexpr int S2M_REC = 32;                     // doubles per record (k_lm.hip)
constexpr int NREC = ALOAM_S2M_RECORDS;
constexpr int RECV_CAP = 2 * NREC;              // world * ceil(NREC / world) <= 2 NREC
constexpr size_t XR_REC_BYTES = sizeof(double) * 2 * NREC * S2M_REC;           // exported records (2 parities)
constexpr size_t XR_BYTES = XR_REC_BYTES + sizeof(unsigned) * S2M_BARS * 32;    // + arrival counters
constexpr size_t GATH_WORDS = S2M_BARS * 32 + 32;                               // local barrier counters + base
static_assert(ALOAM_PEER_HANDLE_BYTES == sizeof(hipIpcMemHandle_t), "IPC handle size");

struct S2MOut {
    aloam_lm_summary lm[ALOAM_MAX_ROUNDS];
    int cnt[ALOAM_MAX_ROUNDS][2];
};

struct S2M {
    int nc = 0, ns = 0, nqc = 0, nqs = 0;
    int cap_mc = 0, cap_ms = 0, cap_qc = 0, cap_qs = 0, cap_f = 0;
    float4 *d_mc = nullptr, *d_ms = nullptr, *d_qc = nullptr, *d_qs = nullptr;
    int* d_n = nullptr;                         // [2] map sizes (grid builds read them on the device)
    Grid gc, gs;                                // 1.025 m cells: the 3x3x3 block holds the 1 m ball
    Grid gcf, gsf;                              // fine cells (~0.3 m): first-phase 5-NN (k_map.hip)
    bool fine = false, shared = false;          // fine grids built; corner map == surf map (one set of grids)
    aloam_factor* d_f = nullptr;
    LMState* d_st = nullptr;                    // [2] LM state, double-buffered across pass launches
    double* d_x = nullptr;                      // [8] parameters (laserMapping.cpp:129)
    double* d_send = nullptr;                   // 2 x NREC records (pass parity: group-mode reuse guard)
    double* d_recv = nullptr;                   // RECV_CAP records
    double* d_lrec = nullptr;                   // one-launch Solves: [2][NREC][32] gathered records
    unsigned* d_gath = nullptr;                 // GATH_WORDS: local barrier counters, then the pass tally (base)
    void* d_xr = nullptr;                       // device exchange: exported records + arrival counters (uncached)
    void* peer_map[S2M_PEER_MAX] = {};          // every rank's d_xr as mapped here (IPC), own at [peer_rank]
    int peer_world = 0, peer_rank = 0;          // > 0: the device exchange is open (aloam_shard_peer_open)
    S2MOut* d_out = nullptr;
    S2MOut* h_out = nullptr;                    // pinned
    hipEvent_t ev[2] = {nullptr, nullptr};      // group mode: records of this rank ready (per parity)
    bool have_map = false, have_q = false;
};

// ---- RCCL, loaded on first use (in a torch process this resolves to the librccl.so.1 torch loaded) ----
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string err;
};
static Rccl* rccl() {
    static Rccl r;
    static bool tried = false;
    if (!tried) {
        tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) { r.err = std::string("cannot load librccl.so.1: ") + dlerror(); return nullptr; }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.error_string) {
            r.err = "librccl.so.1 lacks the nccl* entry points";
            r.get_unique_id = nullptr;
        }
    }
    return r.get_unique_id ? &r : nullptr;
}
static void rcclchk(ncclResult_t e, const char* what) {
    if (e != ncclSuccess) throw ApiError{ALOAM_E_HIP, std::string(what) + ": " + rccl()->error_string(e)};
}

// ---- slot decomposition ----
struct Slice { int per, rp, rec0, rec1, s0, s1; };
static Slice slice_of(int n_slots, int rank, int world) {
    Slice s;
    s.per = std::max(1, (n_slots + NREC - 1) / NREC);       // slots per record block
    s.rp = (NREC + world - 1) / world;                       // record blocks per rank (the last rank may get fewer)
    s.rec0 = std::min(NREC, rank * s.rp);
    s.rec1 = std::min(NREC, s.rec0 + s.rp);
    s.s0 = std::min(n_slots, s.rec0 * s.per);
    s.s1 = std::min(n_slots, s.rec1 * s.per);
    return s;
}

static S2M& s2m_of(Ctx& C) {
    if (!C.s2m) {
        S2M* S = new S2M();
        C.s2m = S;
        S->d_n = (int*)dalloc(C, sizeof(int) * 2);
        S->d_st = (LMState*)dalloc(C, 2 * sizeof(LMState));
        S->d_x = (double*)dalloc(C, sizeof(double) * 8);
        S->d_send = (double*)dalloc(C, sizeof(double) * 2 * NREC * S2M_REC);
        S->d_recv = (double*)dalloc(C, sizeof(double) * RECV_CAP * S2M_REC);
        S->d_out = (S2MOut*)dalloc(C, sizeof(S2MOut));
        S->d_lrec = (double*)dalloc(C, sizeof(double) * 2 * NREC * S2M_REC);
        S->d_gath = (unsigned*)dalloc(C, sizeof(unsigned) * GATH_WORDS);
        HIPCHK(hipHostMalloc((void**)&S->h_out, sizeof(S2MOut), hipHostMallocDefault));
        for (auto& e : S->ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHK(hipMemsetAsync(S->d_recv, 0, sizeof(double) * RECV_CAP * S2M_REC, C.stream));
    }
    return *C.s2m;
}

static void peer_unmap(S2M& S) {
    for (int r = 0; r < S2M_PEER_MAX; r++) {
        if (S.peer_map[r] && S.peer_map[r] != S.d_xr) (void)hipIpcCloseMemHandle(S.peer_map[r]);
        S.peer_map[r] = nullptr;
    }
    S.peer_world = 0;
}

void s2m_release(Ctx& C) {   // device buffers belong to C.bufs; the rest is released here
    if (C.shard_comm && rccl()) (void)rccl()->comm_destroy((ncclComm_t)C.shard_comm);
    C.shard_comm = nullptr;
    if (!C.s2m) return;
    peer_unmap(*C.s2m);
    if (C.s2m->d_xr) (void)hipFree(C.s2m->d_xr);
    for (auto& e : C.s2m->ev) if (e) (void)hipEventDestroy(e);
    if (C.s2m->h_out) (void)hipHostFree(C.s2m->h_out);
    delete C.s2m;
    C.s2m = nullptr;
}

static void copy_in(Ctx& C, float4* dst, const float* src, int n, int flags) {
    if (n > 0)
        HIPCHK(hipMemcpyAsync(dst, src, sizeof(float4) * (size_t)n,
                              (flags & ALOAM_INPUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, C.stream));
}
static float4* grow(Ctx& C, float4* p, int& cap, int n) {   // old buffers stay with the context until destroy
    if (n <= cap) return p;
    cap = std::max(n, 2 * cap);
    return (float4*)dalloc(C, sizeof(float4) * (size_t)cap);
}

void s2m_set_map(Ctx& C, const float* corner, int nc, const float* surf, int ns, int flags) {
    S2M& S = s2m_of(C);
    S.d_mc = grow(C, S.d_mc, S.cap_mc, std::max(nc, 1));
    S.d_ms = grow(C, S.d_ms, S.cap_ms, std::max(ns, 1));
    copy_in(C, S.d_mc, corner, nc, flags);
    copy_in(C, S.d_ms, surf, ns, flags);
    // FromMap indices: 1.025 m cells (5-NN within 1 m: the 27-cell block holds the ball), sorted copies;
    // plus fine grids for the first search phase. One set when the corner and surf maps are one array.
    S.shared = corner == surf && nc == ns;
    const char* fe = getenv("ALOAM_S2M_FINE_CELL");
    const float fine_cell = fe ? (float)atof(fe) : 0.3f;
    S.fine = fine_cell > 0.f;
    auto need = [&](Grid& g, int n, float cell) {
        if (g.cap < std::max(n, 1)) { Grid ng{}; grid_alloc(C, ng, std::max(std::max(n, 1), 2 * g.cap), cell, 1, true, false, GRID_MAX_CELLS_BIG); g = ng; }
        g.min_cell = cell;
    };
    need(S.gc, nc, 1.0f * 1.025f);
    if (!S.shared) need(S.gs, ns, 1.0f * 1.025f);
    if (S.fine) {
        need(S.gcf, nc, fine_cell);
        if (!S.shared) need(S.gsf, ns, fine_cell);
    }
    set_counts2(C, S.d_n, nc, ns);
    GridBuild gb[4];
    int nb = 0;
    gb[nb++] = {&S.gc, S.d_mc, S.d_n + 0, std::max(nc, 1), nullptr, nullptr};
    if (!S.shared) gb[nb++] = {&S.gs, S.d_ms, S.d_n + 1, std::max(ns, 1), nullptr, nullptr};
    if (S.fine) {
        gb[nb++] = {&S.gcf, S.d_mc, S.d_n + 0, std::max(nc, 1), nullptr, nullptr};
        if (!S.shared) gb[nb++] = {&S.gsf, S.d_ms, S.d_n + 1, std::max(ns, 1), nullptr, nullptr};
    }
    grid_build_multi(C, gb, nb);
    S.nc = nc;
    S.ns = ns;
    S.have_map = true;
    HIPCHK(hipStreamSynchronize(C.stream));
}

void s2m_set_queries(Ctx& C, const float* corner, int ncq, const float* surf, int nsq, int flags) {
    S2M& S = s2m_of(C);
    S.d_qc = grow(C, S.d_qc, S.cap_qc, std::max(ncq, 1));
    S.d_qs = grow(C, S.d_qs, S.cap_qs, std::max(nsq, 1));
    copy_in(C, S.d_qc, corner, ncq, flags);
    copy_in(C, S.d_qs, surf, nsq, flags);
    const int q = std::max(ncq + nsq, 1);
    if (S.cap_f < q) {
        S.cap_f = std::max(q, 2 * S.cap_f);
        S.d_f = (aloam_factor*)dalloc(C, sizeof(aloam_factor) * (size_t)S.cap_f);
    }
    S.nqc = ncq;
    S.nqs = nsq;
    S.have_q = true;
    HIPCHK(hipStreamSynchronize(C.stream));
}

static void check_ready(Ctx& C) {
    if (!C.s2m || !C.s2m->have_map || !C.s2m->have_q) throw ApiError{ALOAM_E_STATE, "aloam_s2m_register before set_map / set_queries"};
}

// the map gate of laserMapping.cpp:554
static bool s2m_gate(const S2M& S) { return S.nc > 10 && S.ns > 50; }

// ---- the device exchange (k_s2m_solve) ----
static void ensure_xr(Ctx& C, S2M& S) {
    if (S.d_xr) return;
    HIPCHK(hipSetDevice(C.device));
    // uncached: the peers' polls and record reads go to this GPU's HBM over xGMI, never to a stale line
    HIPCHK(hipExtMallocWithFlags(&S.d_xr, XR_BYTES, hipDeviceMallocUncached));
    HIPCHK(hipMemsetAsync(S.d_xr, 0, XR_BYTES, C.stream));
    HIPCHK(hipStreamSynchronize(C.stream));
}
// counters and pass tally to zero (the stream is idle after this); every rank of an exchange does it
// before any of them launches a Solve (group mode: in the call; IPC: aloam_shard_peer_open + the
// caller's barrier)
static void reset_exchange(Ctx& C, S2M& S) {
    HIPCHK(hipSetDevice(C.device));
    HIPCHK(hipStreamSynchronize(C.stream));
    HIPCHK(hipMemsetAsync(S.d_gath, 0, sizeof(unsigned) * GATH_WORDS, C.stream));
    if (S.d_xr) HIPCHK(hipMemsetAsync((char*)S.d_xr + XR_REC_BYTES, 0, XR_BYTES - XR_REC_BYTES, C.stream));
    HIPCHK(hipStreamSynchronize(C.stream));
}
static S2MPeers table_of(S2M& S, int world, int rank, int rp, void* const* xr) {
    S2MPeers T{};
    T.recs = S.d_lrec;
    T.gath = S.d_gath;
    T.base = S.d_gath + S2M_BARS * 32;
    T.world = world;
    T.rank = rank;
    T.rp = rp;
    for (int r = 0; r < world && xr; r++) {
        T.xrec[r] = (double*)xr[r];
        T.xarr[r] = (unsigned*)((char*)xr[r] + XR_REC_BYTES);
    }
    return T;
}

static void begin(Ctx& C, const double* x) {
    S2M& S = *C.s2m;
    HIPCHK(hipMemsetAsync(S.d_out, 0, sizeof(S2MOut), C.stream));
    HIPCHK(hipMemcpyAsync(S.d_x, x, sizeof(double) * 7, hipMemcpyHostToDevice, C.stream));
}

static void finish(Ctx& C, int rank, int world, double* x, aloam_s2m_result* out, bool copy_x) {
    S2M& S = *C.s2m;
    double xo[7];
    HIPCHK(hipMemcpyAsync(xo, S.d_x, sizeof(double) * 7, hipMemcpyDeviceToHost, C.stream));
    HIPCHK(hipMemcpyAsync(S.h_out, S.d_out, sizeof(S2MOut), hipMemcpyDeviceToHost, C.stream));
    HIPCHK(hipStreamSynchronize(C.stream));
    if (const int code = *(volatile int*)C.h_bar_err) {   // a one-launch Solve's grid barrier timed out (results void)
        *(volatile int*)C.h_bar_err = 0;
        if (getenv("ALOAM_S2M_PEER_DEBUG")) {  // the counters as the Solve left them
            unsigned g[GATH_WORDS], xa[S2M_BARS * 32] = {};
            HIPCHK(hipMemcpy(g, S.d_gath, sizeof(g), hipMemcpyDeviceToHost));
            if (S.d_xr) HIPCHK(hipMemcpy(xa, (char*)S.d_xr + XR_REC_BYTES, sizeof(xa), hipMemcpyDeviceToHost));
            std::fprintf(stderr, "s2m timeout ctx %p: first wait given up %s rank %d pass %d gp %d; base %u gath", (void*)&C,
                         (code >> 28) == 4 ? "peers" : (code >> 28) == 5 ? "local" : "?", (code >> 24) & 15, (code >> 16) & 255,
                         code & 0xffff, g[S2M_BARS * 32]);
            for (int c = 0; c < S2M_BARS; c++) std::fprintf(stderr, " %u", g[c * 32]);
            std::fprintf(stderr, " | arrivals");
            for (int c = 0; c < S2M_BARS; c++) std::fprintf(stderr, " %u", xa[c * 32]);
            std::fprintf(stderr, "\n");
        }
        // the counters no longer agree between the ranks: a device exchange must be opened again
        const bool peer = S.peer_world > 0;
        peer_unmap(S);
        reset_exchange(C, S);
        throw ApiError{ALOAM_E_HIP, peer ? "s2m solve: peer exchange timed out (call aloam_shard_peer_open again on every rank)"
                                         : "s2m solve: grid barrier timed out"};
    }
    if (copy_x) std::memcpy(x, xo, sizeof(xo));
    if (!out) return;
    aloam_s2m_result r{};
    r.optimized = s2m_gate(S) ? 1 : 0;
    r.rounds = r.optimized ? std::min(C.P.map_rounds, ALOAM_MAX_ROUNDS) : 0;
    for (int i = 0; i < r.rounds; i++) {
        r.corner_num[i] = S.h_out->cnt[i][0];
        r.surf_num[i] = S.h_out->cnt[i][1];
        r.lm[i] = S.h_out->lm[i];
    }
    for (int k = 0; k < 4; k++) r.q_w_curr[k] = xo[k];
    for (int k = 0; k < 3; k++) r.t_w_curr[k] = xo[4 + k];
    const Slice sl = slice_of(S.nqc + S.nqs, rank, world);
    r.slot_begin = sl.s0;
    r.slot_end = sl.s1;
    r.world = world;
    *out = r;
}

void s2m_register(Ctx& C, double* x, aloam_s2m_result* out) {
    check_ready(C);
    S2M& S = *C.s2m;
    const bool peer = S.peer_world > 0;                   // the device exchange (aloam_shard_peer_open)
    const int world = peer ? S.peer_world : C.shard_world, rank = peer ? S.peer_rank : C.shard_rank;
    if (world > 1 && !peer && !C.shard_comm) throw ApiError{ALOAM_E_STATE, "shard communicator not initialised"};
    const bool rccl_exchange = !peer && C.shard_comm != nullptr;   // world 1 with a communicator: exercises the RCCL path
    const int Q = S.nqc + S.nqs;
    const Slice sl = slice_of(Q, rank, world);
    begin(C, x);
    // ALOAM_S2M_PERSIST=1, world 1 without a communicator: each Solve is one launch with its exchange on the
    // device (k_s2m_solve). Off by default: measured slower than the stream-ordered pass launches (C4, 2.18-2.21
    // vs 2.04 ms per registration, profiles/r05_s2m_persist.txt): a grid barrier per pass costs ~3 us more
    // than the boundary between two queued launches
    static const bool persist = getenv("ALOAM_S2M_PERSIST") && atoi(getenv("ALOAM_S2M_PERSIST")) == 1;
    const bool one_launch = peer || (persist && world == 1 && !rccl_exchange);
    if (s2m_gate(S)) {
        const int rounds = std::min(C.P.map_rounds, ALOAM_MAX_ROUNDS);
        const int max_iter = std::min(C.P.max_solver_iterations, 200);
        const S2MPeers T = table_of(S, world, rank, sl.rp, peer ? S.peer_map : nullptr);
        const int G = one_launch ? s2m_solve_grid(C, world, sl.rp, false) : 0;
        for (int it = 0; it < rounds; it++) {
            s2m_assoc_launch(C, S.d_qc, S.d_qs, S.nqc, sl.s0, sl.s1, S.d_x, S.gc, S.shared ? S.gc : S.gs, S.fine ? &S.gcf : nullptr,
                             S.fine ? (S.shared ? &S.gcf : &S.gsf) : nullptr, S.d_mc, S.shared ? S.d_mc : S.d_ms, S.d_f);
            if (one_launch) {
                s2m_solve_launch(C, G, S.d_f, Q, sl.per, NREC, T, S.d_x, S.d_st, &S.d_out->lm[it], S.d_out->cnt[it]);
                continue;
            }
            const double* prev = nullptr;   // the exchanged records of the previous pass
            for (int pass = 0; pass <= max_iter; pass++) {
                double* send = S.d_send + (size_t)(pass & 1) * NREC * S2M_REC;
                s2m_pass_launch(C, S.d_f, Q, sl.per, sl.rec0, sl.rp, NREC, prev, S.d_st + ((pass + 1) & 1), S.d_st + (pass & 1), S.d_x,
                                pass, &S.d_out->lm[it], S.d_out->cnt[it], send);
                if (rccl_exchange) {
                    rcclchk(rccl()->all_gather(send, S.d_recv, (size_t)sl.rp * S2M_REC, ncclFloat64, (ncclComm_t)C.shard_comm,
                                               C.stream), "ncclAllGather");
                    prev = S.d_recv;
                } else {
                    prev = send;
                }
            }
            s2m_final_launch(C, prev, NREC, S.d_st + (max_iter & 1), S.d_x, max_iter, &S.d_out->lm[it]);
        }
    }
    finish(C, rank, world, x, out, true);
}

void s2m_register_group(Ctx** cs, int world, double* x, aloam_s2m_result* out) {
    for (int r = 0; r < world; r++) {
        HIPCHK(hipSetDevice(cs[r]->device));
        check_ready(*cs[r]);
    }
    S2M& S0 = *cs[0]->s2m;
    const int Q = S0.nqc + S0.nqs;
    for (int r = 1; r < world; r++) {
        const S2M& S = *cs[r]->s2m;
        if (S.nqc != S0.nqc || S.nqs != S0.nqs || S.nc != S0.nc || S.ns != S0.ns)
            throw ApiError{ALOAM_E_ARG, "group ranks hold different maps / query stacks"};
    }
    for (int r = 0; r < world; r++) { HIPCHK(hipSetDevice(cs[r]->device)); begin(*cs[r], x); }
    const int rp = slice_of(Q, 0, world).rp;
    // ALOAM_S2M_PEER=1: the device exchange between the contexts (direct pointers; one persistent Solve per
    // rank, G = CUs / world each so that every rank's workgroups are co-resident on a shared GPU). The ranks'
    // streams must map to distinct hardware queues (GPU_MAX_HW_QUEUES >= 2 x world + 1): a Solve queued
    // behind a peer's would leave that peer waiting until the exchange times out.
    static const bool dev_x = getenv("ALOAM_S2M_PEER") && atoi(getenv("ALOAM_S2M_PEER")) == 1;
    if (dev_x && world <= S2M_PEER_MAX && s2m_gate(S0)) {
        void* xr[S2M_PEER_MAX] = {};
        bool one_gpu = true;
        for (int r = 0; r < world; r++) {
            Ctx& C = *cs[r];
            ensure_xr(C, *C.s2m);
            xr[r] = C.s2m->d_xr;
            one_gpu &= C.device == cs[0]->device;
            for (int p = 0; p < world; p++)
                if (cs[p]->device != C.device) {
                    const hipError_t e = hipDeviceEnablePeerAccess(cs[p]->device, 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
                    (void)hipGetLastError();
                }
        }
        for (int r = 0; r < world; r++) reset_exchange(*cs[r], *cs[r]->s2m);
        int G = s2m_solve_grid(*cs[0], world, rp, one_gpu);
        const int rounds = std::min(cs[0]->P.map_rounds, ALOAM_MAX_ROUNDS);
        for (int it = 0; it < rounds; it++) {
            for (int r = 0; r < world; r++) {
                Ctx& C = *cs[r];
                S2M& S = *C.s2m;
                const Slice sl = slice_of(Q, r, world);
                HIPCHK(hipSetDevice(C.device));
                s2m_assoc_launch(C, S.d_qc, S.d_qs, S.nqc, sl.s0, sl.s1, S.d_x, S.gc, S.shared ? S.gc : S.gs, S.fine ? &S.gcf : nullptr,
                                 S.fine ? (S.shared ? &S.gcf : &S.gsf) : nullptr, S.d_mc, S.shared ? S.d_mc : S.d_ms, S.d_f);
            }
            for (int r = 0; r < world; r++) {
                Ctx& C = *cs[r];
                S2M& S = *C.s2m;
                HIPCHK(hipSetDevice(C.device));
                s2m_solve_launch(C, G, S.d_f, Q, slice_of(Q, r, world).per, NREC, table_of(S, world, r, rp, xr), S.d_x, S.d_st,
                                 &S.d_out->lm[it], S.d_out->cnt[it]);
            }
        }
    } else if (s2m_gate(S0)) {
        const int rounds = std::min(cs[0]->P.map_rounds, ALOAM_MAX_ROUNDS);
        const int max_iter = std::min(cs[0]->P.max_solver_iterations, 200);
        for (int it = 0; it < rounds; it++) {
            for (int r = 0; r < world; r++) {
                Ctx& C = *cs[r];
                S2M& S = *C.s2m;
                const Slice sl = slice_of(Q, r, world);
                HIPCHK(hipSetDevice(C.device));
                s2m_assoc_launch(C, S.d_qc, S.d_qs, S.nqc, sl.s0, sl.s1, S.d_x, S.gc, S.shared ? S.gc : S.gs, S.fine ? &S.gcf : nullptr,
                             S.fine ? (S.shared ? &S.gcf : &S.gsf) : nullptr, S.d_mc, S.shared ? S.d_mc : S.d_ms, S.d_f);
            }
            for (int pass = 0; pass <= max_iter; pass++) {
                const int parity = pass & 1;
                for (int r = 0; r < world; r++) {      // every rank's records of this pass
                    Ctx& C = *cs[r];
                    S2M& S = *C.s2m;
                    const Slice sl = slice_of(Q, r, world);
                    HIPCHK(hipSetDevice(C.device));
                    s2m_pass_launch(C, S.d_f, Q, sl.per, sl.rec0, rp, NREC, pass ? S.d_recv : nullptr, S.d_st + ((pass + 1) & 1),
                                    S.d_st + parity, S.d_x, pass, &S.d_out->lm[it], S.d_out->cnt[it],
                                    S.d_send + (size_t)parity * NREC * S2M_REC);
                    HIPCHK(hipEventRecord(S.ev[parity], C.stream));
                }
                for (int r = 0; r < world; r++) {      // all-gather as peer copies into every rank's recv (rank order)
                    Ctx& C = *cs[r];
                    HIPCHK(hipSetDevice(C.device));
                    for (int p = 0; p < world; p++) {
                        S2M& P = *cs[p]->s2m;
                        HIPCHK(hipStreamWaitEvent(C.stream, P.ev[parity], 0));
                        HIPCHK(hipMemcpyAsync(C.s2m->d_recv + (size_t)p * rp * S2M_REC, P.d_send + (size_t)parity * NREC * S2M_REC,
                                              sizeof(double) * rp * S2M_REC, hipMemcpyDefault, C.stream));
                    }
                }
                // a rank's send[parity] is rewritten two passes later, after its stream waited for every
                // peer's next-pass records, which those peers recorded after copying this pass's
            }
            for (int r = 0; r < world; r++) {
                Ctx& C = *cs[r];
                S2M& S = *C.s2m;
                HIPCHK(hipSetDevice(C.device));
                s2m_final_launch(C, S.d_recv, NREC, S.d_st + (max_iter & 1), S.d_x, max_iter, &S.d_out->lm[it]);
            }
        }
    }
    if (getenv("ALOAM_S2M_PEER_DEBUG"))
        for (int r = 0; r < world; r++) {
            HIPCHK(hipStreamSynchronize(cs[r]->stream));
            std::fprintf(stderr, "rank %d err %08x\n", r, *(volatile int*)cs[r]->h_bar_err);
        }
    for (int r = 0; r < world; r++) {
        HIPCHK(hipSetDevice(cs[r]->device));
        finish(*cs[r], r, world, x, out ? out + r : nullptr, r == 0);
    }
}

void shard_unique_id(unsigned char* id) {
    Rccl* R = rccl();
    if (!R) throw ApiError{ALOAM_E_NODEVICE, "RCCL unavailable"};
    ncclUniqueId u;
    rcclchk(R->get_unique_id(&u), "ncclGetUniqueId");
    static_assert(sizeof(u) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(id, &u, sizeof(u));
}

void shard_init(Ctx& C, int rank, int world, const unsigned char* id) {
    if (world < 1 || rank < 0 || rank >= world || world > NREC) throw ApiError{ALOAM_E_ARG, "bad rank / world"};
    if (C.shard_comm) { (void)rccl()->comm_destroy((ncclComm_t)C.shard_comm); C.shard_comm = nullptr; }
    C.shard_rank = rank;
    C.shard_world = world;
    if (!id) {
        if (world == 1) return;   // no exchange at all
        throw ApiError{ALOAM_E_ARG, "null unique id"};
    }
    Rccl* R = rccl();
    if (!R) throw ApiError{ALOAM_E_NODEVICE, "RCCL unavailable"};
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    HIPCHK(hipSetDevice(C.device));
    rcclchk(R->comm_init_rank(&comm, world, u, rank), "ncclCommInitRank");
    C.shard_comm = comm;
}

void shard_peer_handle(Ctx& C, unsigned char* out) {
    S2M& S = s2m_of(C);
    ensure_xr(C, S);
    hipIpcMemHandle_t h;
    HIPCHK(hipIpcGetMemHandle(&h, S.d_xr));
    std::memcpy(out, &h, sizeof(h));
}

void shard_peer_open(Ctx& C, const unsigned char* handles, int world, int rank) {
    if (world < 1 || world > S2M_PEER_MAX || rank < 0 || rank >= world || !handles) throw ApiError{ALOAM_E_ARG, "bad rank / world / handles"};
    S2M& S = s2m_of(C);
    ensure_xr(C, S);
    peer_unmap(S);
    HIPCHK(hipSetDevice(C.device));
    for (int r = 0; r < world; r++) {
        if (r == rank) { S.peer_map[r] = S.d_xr; continue; }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)r * sizeof(h), sizeof(h));
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            peer_unmap(S);
            throw ApiError{ALOAM_E_HIP, std::string("hipIpcOpenMemHandle (rank ") + std::to_string(r) + "): " + hipGetErrorString(e)};
        }
        S.peer_map[r] = p;
    }
    reset_exchange(C, S);
    S.peer_world = world;
    S.peer_rank = rank;
}

void shard_peer_close(Ctx& C) {
    if (!C.s2m) return;
    HIPCHK(hipStreamSynchronize(C.stream));
    peer_unmap(*C.s2m);
}

int shard_slot_range(int n_slots, int rank, int world, int* begin, int* end) {
    if (n_slots < 0 || world < 1 || world > NREC || rank < 0 || rank >= world || !begin || !end) return ALOAM_E_ARG;
    const Slice s = slice_of(n_slots, rank, world);
    *begin = s.s0;
    *end = s.s1;
    return ALOAM_OK;
}

}  // namespace aloam
