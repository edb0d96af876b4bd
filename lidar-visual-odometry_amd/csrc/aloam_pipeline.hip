// aloam_pipeline.hip — the reference's node split as a native pipeline on one GPU (host side only).
//
// The reference runs scanRegistration, laserOdometry and laserMapping as three ROS processes, each
// with one thread doing its hot block (src/scanRegistration.cpp:461-503, src/laserOdometry.cpp:311,
// src/laserMapping.cpp:934 `process` thread), connected by topics. Here each stage owns an aloam_ctx
// (own HIP stream) and a native worker thread; the hand-offs are device-to-device copies
// (aloam_forward_features / aloam_forward_mapping_input). push() runs the first stage on the caller's
// thread while the workers run the later stages of earlier scans:
//   stages 2: caller: scanRegistration + laserOdometry (scan k)   || worker M: laserMapping (scan k-1)
//   stages 3: caller: scanRegistration (k) || worker O: laserOdometry (k-1) || worker M: laserMapping (k-2)
// Every scan goes through all stages in order, so results equal aloam_process_scan's.
// The workers spin briefly on an atomic job word before sleeping, so a hand-off costs a cache-line
// transfer instead of a thread wake-up on the critical path.
// With 2 stages the mapping thread is a server over a 2-deep queue of hand-offs taken by value
// (MapSnapshot): it forwards scan k's odometry output and maps it as soon as scan k-1's mapping is done,
// without waiting for the caller's thread; the front publishes into alternating buffer sets, and before a
// publish overwrites a set the front's stream waits (GPU-side) for the copy that read it.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>

#include "aloam_internal.hpp"

namespace {

struct Worker {
    std::thread th;
    std::atomic<int> state{0};            // 0 idle, 1 job posted, 2 job done, 3 quit
    std::mutex m;
    std::condition_variable cv;
    int (*fn)(void*) = nullptr;
    void* arg = nullptr;
    int rc = 0;

    void start() {
        th = std::thread([this] {
            for (;;) {
                int s;
                int spins = 0;
                while ((s = state.load(std::memory_order_acquire)) == 0 || s == 2) {
                    if (++spins < 20000) { std::this_thread::yield(); continue; }
                    std::unique_lock<std::mutex> lk(m);
                    cv.wait(lk, [this] { const int v = state.load(std::memory_order_acquire); return v == 1 || v == 3; });
                    spins = 0;
                }
                if (s == 3) return;
                rc = fn(arg);
                state.store(2, std::memory_order_release);
            }
        });
    }
    void post(int (*f)(void*), void* a) {
        fn = f;
        arg = a;
        {
            std::lock_guard<std::mutex> lk(m);
            state.store(1, std::memory_order_release);
        }
        cv.notify_one();
    }
    bool busy() const { return state.load(std::memory_order_acquire) == 1; }
    // waits for the posted job; returns its rc, or 1 when nothing was posted
    int join() {
        int s;
        while ((s = state.load(std::memory_order_acquire)) == 1) std::this_thread::yield();
        if (s != 2) return 1;
        state.store(0, std::memory_order_release);
        return rc;
    }
    void stop() {
        join();
        {
            std::lock_guard<std::mutex> lk(m);
            state.store(3, std::memory_order_release);
        }
        cv.notify_one();
        if (th.joinable()) th.join();
    }
};

}  // namespace

namespace {
struct MapServer {
    std::thread th;
    std::atomic<long> posted{0}, issued{0}, done{0};
    std::atomic<bool> quit{false};
    std::mutex m;
    std::condition_variable cv;
    aloam::MapSnapshot snap[2];
    static constexpr int NRES = 4;               // result slots (index j % NRES): up to lag + 2 outstanding
    aloam_map_result res[NRES];
    aloam_timing tim[NRES];
    int rc[NRES] = {0, 0, 0, 0};
    std::string err[NRES];
    hipEvent_t copied[2] = {nullptr, nullptr};   // after the copy of hand-off j (index j & 1)
    long returned = 0;                           // results handed to the caller
    // result lag of aloam_pipeline_push: mapping result k-lag is returned at scan k. lag 1 makes the front
    // wait for mapping k-1 before it starts scan k+1, so the two stages alternate their host latencies
    // (hand-off, issue, completion) on one critical path; lag 2 lets the front run one scan further
    // ahead. ALOAM_PIPE_LAG (1 or 2, default 2); profiling runs one frame at a time (lag 1).
    int lag = 2;
    // the front's scan k is issued by push k and completed by push k+1 (or flush): its odometry result
    // is returned one push late, and the caller's round trip overlaps the scan's GPU work
    bool front_pending = false;
    // ALOAM_PIPE_TIMING (profiling aid): host-side stage occupancy, printed at destroy
    double t_fwd = 0, t_issue = 0, t_complete = 0, t_idle = 0, t_front = 0, t_take = 0, t_wiss = 0;
    long n_srv = 0, n_front = 0;
};
static const bool g_pipe_timing = std::getenv("ALOAM_PIPE_TIMING") != nullptr;
static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

struct aloam_pipeline {
    int stages = 2;
    aloam_ctx* front = nullptr;     // scanRegistration (+ laserOdometry when stages == 2)
    aloam_ctx* odom = nullptr;      // laserOdometry (== front when stages == 2)
    aloam_ctx* back = nullptr;      // laserMapping
    Worker wo, wm;
    aloam_odom_result od_job{};     // worker O output
    aloam_map_result mp_job{};      // worker M output
    aloam_timing t_stage[3]{};      // timing snapshots of the last completed job per stage
    int profiling = 0;
    std::string err;
    MapServer ms;                   // stages == 2
};

namespace {

int odom_job(void* a) {
    aloam_pipeline* P = (aloam_pipeline*)a;
    const int rc = aloam_odometry(P->odom, &P->od_job);
    if (rc == 0 && P->profiling) aloam_get_timing(P->odom, &P->t_stage[1]);
    return rc;
}
int map_job(void* a) {
    aloam_pipeline* P = (aloam_pipeline*)a;
    const int rc = aloam_mapping(P->back, &P->mp_job);
    if (rc == 0 && P->profiling) aloam_get_timing(P->back, &P->t_stage[2]);
    return rc;
}
template <class Fn>
int guarded(Fn&& fn, std::string& err) {
    try {
        fn();
        return 0;
    } catch (const aloam::ApiError& e) {
        err = e.msg;
        return e.code;
    } catch (const aloam::HipError& e) {
        err = e.msg;
        return ALOAM_E_HIP;
    } catch (const std::bad_alloc&) {
        err = "host allocation failed";
        return ALOAM_E_CAPACITY;
    }
}
// Hand-off j: forward it, issue its mapping frame, and only then wait for frame j-1 (software pipelining
// on the mapping stream: the host issues frame j while the GPU still runs frame j-1, so the ~0.2-0.4 ms
// of launch issue per frame leaves the critical path). With no next hand-off posted, the frame in
// flight is completed at once. Results are published in order (done = j + 1 after result j).
void map_server(aloam_pipeline* P) {
    MapServer& S = P->ms;
    aloam::Ctx& B = *(aloam::Ctx*)P->back;
    long inflight = -1;
    auto complete = [&](long j) {
        const int i = (int)(j % MapServer::NRES);
        const double t0 = g_pipe_timing ? now_us() : 0;
        const int rc = guarded([&] { aloam::mapping_complete(B, &S.res[i]); }, S.err[i]);
        if (g_pipe_timing) S.t_complete += now_us() - t0;
        if (!rc && P->profiling) aloam_get_timing(P->back, &S.tim[i]);
        S.rc[i] = rc;
        S.done.store(j + 1, std::memory_order_release);
    };
    for (long j = 0;;) {
        int spins = 0;
        const double ti = g_pipe_timing ? now_us() : 0;
        while (S.posted.load(std::memory_order_acquire) <= j) {
            if (inflight >= 0) { complete(inflight); inflight = -1; continue; }
            if (S.quit.load(std::memory_order_acquire)) return;
            if (++spins < 20000) { std::this_thread::yield(); continue; }
            std::unique_lock<std::mutex> lk(S.m);
            S.cv.wait(lk, [&] { return S.posted.load(std::memory_order_acquire) > j || S.quit.load(std::memory_order_acquire); });
            spins = 0;
        }
        const int i = (int)(j % MapServer::NRES);
        std::string e;
        double t1 = 0, t2 = 0;
        if (g_pipe_timing) { t1 = now_us(); S.t_idle += t1 - ti; }
        // the hand-off's stacks are copied inside mapping_issue, right before the rounds (after the
        // prepare and grid builds), and `copied` is recorded there: `issued` follows the issue
        int rc = guarded([&] { aloam::forward_snapshot(B, S.snap[j & 1], S.copied[j & 1], true); }, e);
        if (g_pipe_timing) { t2 = now_us(); S.t_fwd += t2 - t1; }
        // a frame that has already finished is handed back before the ~0.5 ms of launch issue below
        if (inflight >= 0 && aloam::mapping_ready(B)) { complete(inflight); inflight = -1; }
        if (!rc) rc = guarded([&] { aloam::mapping_issue(B); }, e);
        S.issued.store(j + 1, std::memory_order_release);
        if (g_pipe_timing) { S.t_issue += now_us() - t2; S.n_srv++; }
        if (inflight >= 0) { complete(inflight); inflight = -1; }
        if (rc) {
            S.err[i] = e;
            S.rc[i] = rc;
            S.done.store(j + 1, std::memory_order_release);
        } else if (P->profiling) {
            complete(j);                  // profiling events are per context: one frame at a time
        } else {
            inflight = j;
        }
        j++;
    }
}
// hands the caller the oldest unreturned mapping result once done (waits); rc of that job
int take_result(aloam_pipeline* P, aloam_map_result* mp, int* have) {
    MapServer& S = P->ms;
    const long j = S.returned;
    while (S.done.load(std::memory_order_acquire) <= j) std::this_thread::yield();
    const int i = (int)(j % MapServer::NRES);
    S.returned = j + 1;
    if (S.rc[i]) { P->err = S.err[i]; return S.rc[i]; }
    *have = 1;
    if (mp) *mp = S.res[i];
    if (P->profiling) P->t_stage[2] = S.tim[i];
    return 0;
}

int fail(aloam_pipeline* P, aloam_ctx* c, int rc) {
    P->err = aloam_last_error(c);
    return rc;
}
// joins worker M; *have = 1 and *mp filled when a mapping job completed
int join_map(aloam_pipeline* P, aloam_map_result* mp, int* have) {
    const int rc = P->wm.join();
    if (rc == 1) return 0;                      // nothing pending
    if (rc != 0) return fail(P, P->back, rc);
    *have = 1;
    if (mp) *mp = P->mp_job;
    return 0;
}

// completes the front's pending scan: its odometry result, its hand-off to the mapping server, and the
// mapping result due at this point (lag)
int finish_front(aloam_pipeline* P, aloam_odom_result* od, int* have_od, aloam_map_result* mp, int* have_mp) {
    MapServer& S = P->ms;
    aloam::Ctx& F = *(aloam::Ctx*)P->front;
    S.front_pending = false;
    aloam_odom_result o{};
    const double tf0 = g_pipe_timing ? now_us() : 0;
    int rc = guarded([&] { aloam::front_complete(F, &o); }, P->err);
    if (g_pipe_timing) S.t_front += now_us() - tf0;
    if (rc) return rc;
    if (P->profiling) aloam_get_timing(P->front, &P->t_stage[0]), P->t_stage[1] = P->t_stage[0];
    *have_od = 1;
    if (od) *od = o;
    const long seq = S.posted.load(std::memory_order_relaxed);
    bool posted = false;
    if (o.publish_to_mapping) {
        try {
            aloam::snapshot_mapping_input(F, &S.snap[seq & 1]);
        } catch (const aloam::ApiError& e) {
            P->err = e.msg;
            return e.code;
        }
        {
            std::lock_guard<std::mutex> lk(S.m);
            S.posted.store(seq + 1, std::memory_order_release);
        }
        S.cv.notify_one();
        posted = true;
    }
    // mapping result k - lag (the lag-th job before the one just posted); ALOAM_PIPE_POLL=1: returned
    // only once done (no wait) unless NRES - 1 results are outstanding
    const int lag = P->profiling ? 1 : S.lag;
    static const bool poll = std::getenv("ALOAM_PIPE_POLL") && std::atoi(std::getenv("ALOAM_PIPE_POLL")) == 1;
    const long outstanding = S.posted.load(std::memory_order_relaxed) - S.returned;
    const bool due = poll && !P->profiling ? (outstanding >= MapServer::NRES - 1 ||
                                              (outstanding > 0 && S.done.load(std::memory_order_acquire) > S.returned))
                                           : outstanding > (posted ? lag : lag - 1);
    if (due) {
        const double tt0 = g_pipe_timing ? now_us() : 0;
        const int trc = take_result(P, mp, have_mp);
        if (g_pipe_timing) S.t_take += now_us() - tt0;
        return trc;
    }
    return ALOAM_OK;
}

}  // namespace

extern "C" {

aloam_pipeline* aloam_pipeline_create(const aloam_params* p, int device, int stages) {
    if (!p || (stages != 2 && stages != 3)) return nullptr;
    aloam_pipeline* P = new (std::nothrow) aloam_pipeline();
    if (!P) return nullptr;
    P->stages = stages;
    P->front = aloam_create(p, device);
    P->odom = stages == 3 ? aloam_create(p, device) : P->front;
    P->back = aloam_create(p, device);
    if (!P->front || !P->odom || !P->back) {
        if (P->back) aloam_destroy(P->back);
        if (stages == 3 && P->odom) aloam_destroy(P->odom);
        if (P->front) aloam_destroy(P->front);
        delete P;
        return nullptr;
    }
    // Disjoint CUs per stage: the front stage(s) get CUs [0, F), laserMapping [F, ncu); with 3 stages
    // scanRegistration gets [0, F3) and laserOdometry [F3, F). Concurrent latency-bound stages then stop
    // queueing behind each other's workgroups (measured on one MI355X, 2 stages: 822-840 scans/s shared,
    // 968-971 with contiguous halves; alternating runs of 1-32 CUs were in between).
    // ALOAM_PIPE_CU_SPLIT = F (default ncu / 2; 0 shares all CUs), ALOAM_PIPE_CU_SPLIT3 = F3 (default F / 3).
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        const int ncu = prop.multiProcessorCount, nw = (ncu + 31) / 32;
        const char* env = std::getenv("ALOAM_PIPE_CU_SPLIT");
        const int F = env ? std::atoi(env) : ncu / 2;
        const char* env3 = std::getenv("ALOAM_PIPE_CU_SPLIT3");
        const int F3 = env3 ? std::atoi(env3) : F / 3;
        if (F > 0 && F < ncu && (stages == 2 || (F3 > 0 && F3 <= F))) {   // F3 == F: both front stages on [0, F)
            auto range = [&](int a, int b) {
                std::vector<unsigned> m(nw, 0u);
                for (int c = a; c < b; c++) m[c / 32] |= 1u << (c % 32);
                return m;
            };
            // 2 stages with ALOAM_SIDE_STACKS=1 (opt-in, see forward_snapshot): the mapping context's stream3
            // may get the last ALOAM_PIPE_SIDE_CUS CUs of its range to itself (default 0 = shared; measured
            // 715-757 scans/s with 8-32 CUs of its own vs 736 shared: not the cause of the slowdown)
            const char* envs = std::getenv("ALOAM_PIPE_SIDE_CUS");
            const int SIDE = stages == 2 ? std::max(0, std::min(envs ? std::atoi(envs) : 0, (ncu - F) / 2)) : 0;
            const std::vector<unsigned> mf = range(0, stages == 3 ? F3 : F), mo = range(F3 == F ? 0 : F3, F),
                                        mm = range(F, ncu - SIDE), mside = range(ncu - SIDE, ncu);
            if (aloam_set_cu_mask(P->front, mf.data(), nw) || (stages == 3 && aloam_set_cu_mask(P->odom, mo.data(), nw)) ||
                aloam_set_cu_mask(P->back, mm.data(), nw) ||
                (SIDE > 0 && guarded([&] { aloam::set_side_cu_mask(*(aloam::Ctx*)P->back, mside.data(), nw); }, P->err))) {
                aloam_destroy(P->back);
                if (stages == 3) aloam_destroy(P->odom);
                aloam_destroy(P->front);
                delete P;
                return nullptr;
            }
        }
    }
    if (stages == 2) {
        const char* lenv = std::getenv("ALOAM_PIPE_LAG");
        P->ms.lag = lenv && std::atoi(lenv) == 1 ? 1 : 2;
        // the front voxelises the mapping stacks of each publish on its stream2 (ALOAM_PIPE_FRONT_STACKS=0: off)
        const char* fsenv = std::getenv("ALOAM_PIPE_FRONT_STACKS");
        ((aloam::Ctx*)P->front)->publish_stacks = !fsenv || std::atoi(fsenv) != 0;
        for (auto& e : P->ms.copied)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
        P->ms.th = std::thread(map_server, P);
    } else {
        P->wm.start();
        P->wo.start();
    }
    return P;
}

void aloam_pipeline_destroy(aloam_pipeline* P) {
    if (!P) return;
    if (P->stages == 2) {
        {
            std::lock_guard<std::mutex> lk(P->ms.m);
            P->ms.quit.store(true, std::memory_order_release);
        }
        P->ms.cv.notify_one();
        if (P->ms.th.joinable()) P->ms.th.join();
        const MapServer& S = P->ms;
        if (g_pipe_timing && S.n_srv > 0 && S.n_front > 0)
            std::fprintf(stderr, "[aloam pipe] per scan (us): front process %.1f, front wait-for-result %.1f, front wait-for-issue %.1f | server: "
                         "idle %.1f, forward %.1f, issue %.1f, complete(wait+read) %.1f  (%ld / %ld)\n",
                         S.t_front / S.n_front, S.t_take / S.n_front, S.t_wiss / S.n_front, S.t_idle / S.n_srv, S.t_fwd / S.n_srv,
                         S.t_issue / S.n_srv, S.t_complete / S.n_srv, S.n_front, S.n_srv);
        for (auto& e : P->ms.copied) if (e) (void)hipEventDestroy(e);
    } else {
        P->wm.stop();
        P->wo.stop();
    }
    aloam_destroy(P->back);
    if (P->stages == 3) aloam_destroy(P->odom);
    aloam_destroy(P->front);
    delete P;
}

const char* aloam_pipeline_last_error(const aloam_pipeline* P) { return P ? P->err.c_str() : "null pipeline"; }

aloam_ctx* aloam_pipeline_context(aloam_pipeline* P, int stage) {
    if (!P || stage < 0 || stage > 2) return nullptr;
    return stage == 0 ? P->front : stage == 1 ? P->odom : P->back;
}

int aloam_pipeline_set_profiling(aloam_pipeline* P, int enable) {
    if (!P || P->wm.busy() || (P->stages == 3 && P->wo.busy())) return ALOAM_E_STATE;
    if (P->stages == 2 && (P->ms.front_pending || P->ms.done.load() != P->ms.posted.load())) return ALOAM_E_STATE;
    P->profiling = enable != 0;
    int rc = aloam_set_profiling(P->front, enable);
    if (!rc && P->stages == 3) rc = aloam_set_profiling(P->odom, enable);
    if (!rc) rc = aloam_set_profiling(P->back, enable);
    std::memset(P->t_stage, 0, sizeof(P->t_stage));
    return rc;
}

int aloam_pipeline_timing(aloam_pipeline* P, int stage, aloam_timing* t) {
    if (!P || !t || stage < 0 || stage > 2) return ALOAM_E_ARG;
    *t = P->t_stage[stage];
    return ALOAM_OK;
}

int aloam_pipeline_push(aloam_pipeline* P, const float* xyzr, int n, int flags, aloam_odom_result* od, int* have_od,
                        aloam_map_result* mp, int* have_mp) {
    if (!P || !have_od || !have_mp) return ALOAM_E_ARG;
    *have_od = 0;
    *have_mp = 0;
    int rc;
    if (P->stages == 2) {
        MapServer& S = P->ms;
        aloam::Ctx& F = *(aloam::Ctx*)P->front;
        // scan k-1 first: its results, its hand-off (posted before scan k publishes into the other set)
        if (S.front_pending && (rc = finish_front(P, od, have_od, mp, have_mp))) return rc;
        const long seq = S.posted.load(std::memory_order_relaxed);     // index of the next hand-off
        if (seq >= 2) {
            // this scan may publish into the buffer set hand-off seq-2 was taken from: its copy must be
            // issued (host) and finished (GPU) first. Done right before the publish launch (pre_publish),
            // after the scan's registration and odometry rounds are queued: only the publish waits.
            F.pre_publish = [P, &S, &F, seq]() {
                const double tw0 = g_pipe_timing ? now_us() : 0;
                while (S.issued.load(std::memory_order_acquire) < seq - 1) std::this_thread::yield();
                if (g_pipe_timing) S.t_wiss += now_us() - tw0;
                std::lock_guard<std::mutex> lk(((aloam::Ctx*)P->back)->capture_mu);   // not while mapping captures
                hipError_t e = hipStreamWaitEvent(F.stream, S.copied[seq & 1], 0);
                // (the stacks of this publish may run on stream2 ahead of the publish copy: the same wait there)
                if (e == hipSuccess && F.publish_stacks) e = hipStreamWaitEvent(F.stream2, S.copied[seq & 1], 0);
                if (e != hipSuccess)
                    throw aloam::HipError(std::string("hipStreamWaitEvent failed: ") + hipGetErrorName(e) + " (hand-off " +
                                          std::to_string(seq - 2) + ", server rc " + std::to_string(S.rc[(seq - 2) % MapServer::NRES]) +
                                          " " + S.err[(seq - 2) % MapServer::NRES] + ")");
            };
        }
        const double tf0 = g_pipe_timing ? now_us() : 0;
        rc = guarded([&] { aloam::front_issue(F, xyzr, n, flags); }, P->err);
        if (g_pipe_timing) { S.t_front += now_us() - tf0; S.n_front++; }
        if (rc) return rc;
        S.front_pending = true;
        // profiling events are per context and per call: one scan at a time (no lag on the front)
        if (P->profiling) return finish_front(P, od, have_od, mp, have_mp);
        return ALOAM_OK;
    }
    // three stages: scanRegistration here, odometry and mapping of earlier scans in the workers
    rc = aloam_scan_registration(P->front, xyzr, n, flags);
    if (rc) return fail(P, P->front, rc);
    if (P->profiling) aloam_get_timing(P->front, &P->t_stage[0]);
    const int orc = P->wo.join();
    if (orc != 1 && orc != 0) return fail(P, P->odom, orc);
    if ((rc = join_map(P, mp, have_mp))) return rc;
    if (orc == 0) {
        *have_od = 1;
        if (od) *od = P->od_job;
        if (P->od_job.publish_to_mapping) {
            if ((rc = aloam_forward_mapping_input(P->odom, P->back))) return fail(P, P->back, rc);
            P->wm.post(map_job, P);
        }
    }
    if ((rc = aloam_forward_features(P->front, P->odom))) return fail(P, P->odom, rc);
    P->wo.post(odom_job, P);
    return ALOAM_OK;
}

int aloam_pipeline_flush(aloam_pipeline* P, aloam_odom_result* od, int* have_od, aloam_map_result* mp, int* have_mp,
                         aloam_map_result* mp2, int* have_mp2) {
    if (!P || !have_od || !have_mp || !have_mp2) return ALOAM_E_ARG;
    *have_od = *have_mp = *have_mp2 = 0;
    int rc;
    if (P->stages == 2) {             // the pending front scan, then up to two mapping results per call
        if (P->ms.front_pending && (rc = finish_front(P, od, have_od, mp, have_mp))) return rc;
        if (!*have_mp && P->ms.returned < P->ms.posted.load(std::memory_order_relaxed) && (rc = take_result(P, mp, have_mp))) return rc;
        if (P->ms.returned < P->ms.posted.load(std::memory_order_relaxed)) return take_result(P, mp2, have_mp2);
        return ALOAM_OK;
    }
    const int orc = P->wo.join();
    if (orc != 1 && orc != 0) return fail(P, P->odom, orc);
    if ((rc = join_map(P, mp, have_mp))) return rc;
    if (orc == 0) {
        *have_od = 1;
        if (od) *od = P->od_job;
        if (P->od_job.publish_to_mapping) {
            if ((rc = aloam_forward_mapping_input(P->odom, P->back))) return fail(P, P->back, rc);
            if ((rc = aloam_mapping(P->back, mp2))) return fail(P, P->back, rc);
            if (P->profiling) aloam_get_timing(P->back, &P->t_stage[2]);
            *have_mp2 = 1;
        }
    }
    return ALOAM_OK;
}

}  // extern "C"
