// tests/ps_emu.cpp — host emulation of HIP workgroups running csrc/ls_sort.hpp (+ pcl_sort.hpp's pieces).
//
// Every lane is a fiber (ucontext stacks, switched by _setjmp/_longjmp on one OS thread, round robin); the
// wave collectives the sort uses (ballot, shfl, readlane / readfirstlane, DPP scans, all-reduces, the wave
// barrier) are a wave-wide fiber barrier around a shared exchange slot, lds_barrier / __syncthreads a
// workgroup-wide one, the LDS atomics host atomics. The device code is compiled unchanged (PS_HOST_EMU skips
// its HIP include), so its partition arithmetic, work queue and workgroup phase are checked against
// libstdc++'s std::sort on the CPU. (Lanes as OS threads spent most of the run in futex wake-ups.)
// Test infrastructure: built and run by tests/test_pcl_sort_emu.py.
#undef _FORTIFY_SOURCE        // longjmp between fiber stacks: the fortified check rejects a jump to another stack
#include <algorithm>
#include <atomic>
#include <csetjmp>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <random>
#include <ucontext.h>
#include <vector>

#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__
#define WAVE 64

struct Dim3 { unsigned x = 0, y = 0, z = 0; };
static Dim3 threadIdx;
static int t_lane = 0, t_wave = 0;

// ---- fibers: one per emulated lane, all on the calling thread ----
struct Fiber {
    ucontext_t uc;
    jmp_buf jb;
    char* stack = nullptr;
    bool started = false, done = false;
};
static constexpr size_t FIBER_STACK = 1u << 20;
static std::vector<Fiber> g_fib;
static int g_cur = 0, g_live = 0;
static jmp_buf g_main_jb;
static std::function<void(int)> g_body;

static void set_ids(int t) { threadIdx.x = (unsigned)t; t_lane = t % WAVE; t_wave = t / WAVE; }
static void enter(int next) {         // leave the current context for fiber `next` (never returns)
    g_cur = next;
    set_ids(next);
    Fiber& f = g_fib[next];
    if (!f.started) { f.started = true; setcontext(&f.uc); }
    _longjmp(f.jb, 1);
}
__attribute__((noinline)) static void fiber_yield() {
    const int n = (int)g_fib.size();
    int next = g_cur;
    do next = (next + 1) % n; while (g_fib[next].done && next != g_cur);
    if (next == g_cur) return;
    if (_setjmp(g_fib[g_cur].jb)) return;     // resumed by another fiber (ids already set for us)
    enter(next);
}
static void fiber_entry() {
    g_body(g_cur);
    g_fib[g_cur].done = true;
    if (--g_live == 0) _longjmp(g_main_jb, 1);
    fiber_yield();                            // a done fiber is never resumed
    std::abort();
}
// run body(t) for t in [0, nt) as nt lanes; returns when every lane has returned
static void run_group(int nt, std::function<void(int)> body) {
    g_fib = std::vector<Fiber>(nt);
    g_body = std::move(body);
    g_live = nt;
    for (auto& f : g_fib) {
        f.stack = (char*)std::malloc(FIBER_STACK);
        getcontext(&f.uc);
        f.uc.uc_stack.ss_sp = f.stack;
        f.uc.uc_stack.ss_size = FIBER_STACK;
        f.uc.uc_link = nullptr;
        makecontext(&f.uc, fiber_entry, 0);
    }
    if (!_setjmp(g_main_jb)) enter(0);
    for (auto& f : g_fib) std::free(f.stack);
    g_fib.clear();
}
struct FBarrier {
    int n, count = 0;
    volatile unsigned gen = 0;
    explicit FBarrier(int n_) : n(n_) {}
    void arrive_and_wait() {
        const unsigned g = gen;
        if (++count == n) { count = 0; gen = g + 1; return; }
        while (gen == g) fiber_yield();
    }
};

struct WaveCtx {
    std::unique_ptr<FBarrier> bar;
    unsigned long long slot[WAVE];
    unsigned long long out;
};
static std::vector<std::unique_ptr<WaveCtx>> g_waves;
static std::unique_ptr<FBarrier> g_block;

static inline WaveCtx& W() { return *g_waves[t_wave]; }
static inline void wave_sync() { W().bar->arrive_and_wait(); }
// every lane deposits v, all see all
template <typename F>
static inline unsigned long long wave_collect(unsigned long long v, F f) {
    WaveCtx& w = W();
    w.slot[t_lane] = v;
    wave_sync();
    unsigned long long r = f(w.slot);
    wave_sync();
    return r;
}

namespace aloam {
inline int lane_id() { return t_lane; }
inline int wave_incl_scan(int v) {
    return (int)wave_collect((unsigned long long)(unsigned)v, [](const unsigned long long* s) {
        int acc = 0;
        for (int i = 0; i <= t_lane; i++) acc += (int)(unsigned)s[i];
        return (unsigned long long)(unsigned)acc;
    });
}
inline int readlane_i(int v, int lane) {
    return (int)wave_collect((unsigned long long)(unsigned)v, [lane](const unsigned long long* s) { return s[lane]; });
}
template <int NS, typename F>
inline unsigned allreduce_u32(unsigned v, F op) {
    static_assert(NS == 6, "whole-wave reductions only");
    return (unsigned)wave_collect(v, [&op](const unsigned long long* s) {
        unsigned a = (unsigned)s[0];
        for (int i = 1; i < WAVE; i++) a = op(a, (unsigned)s[i]);
        return (unsigned long long)a;
    });
}
inline int wave_sum_i(int v) { return (int)allreduce_u32<6>((unsigned)v, [](unsigned a, unsigned b) { return a + b; }); }
inline void lds_barrier() { g_block->arrive_and_wait(); }
inline unsigned long long lanemask_lt64() { return t_lane == 0 ? 0ull : (~0ull >> (64 - t_lane)); }
}  // namespace aloam

static inline unsigned long long __ballot(bool p) {
    return wave_collect(p ? 1ull : 0ull, [](const unsigned long long* s) {
        unsigned long long m = 0;
        for (int i = 0; i < WAVE; i++) m |= (s[i] ? 1ull : 0ull) << i;
        return m;
    });
}
static inline int __shfl(int v, int src, int) {
    return (int)wave_collect((unsigned long long)(unsigned)v, [src](const unsigned long long* s) { return s[src & 63]; });
}
static inline int __builtin_amdgcn_readfirstlane(int v) { return aloam::readlane_i(v, 0); }
// DPP row_shl:N (ctrl 0x101..0x10f) only: lane l takes lane l + N of its row of 16, else `old`
static inline int __builtin_amdgcn_update_dpp(int old, int src, int ctrl, int, int, bool) {
    const int sh = ctrl - 0x100;
    if (sh < 1 || sh > 15) std::abort();
    return (int)wave_collect((unsigned long long)(unsigned)src, [&](const unsigned long long* s) {
        return (t_lane & 15) + sh < 16 ? s[t_lane + sh] : (unsigned long long)(unsigned)old;
    });
}
static inline void __builtin_amdgcn_wave_barrier() { wave_sync(); }
static inline void __builtin_amdgcn_fence(int, const char*) { std::atomic_thread_fence(std::memory_order_seq_cst); }
static inline void __builtin_amdgcn_s_sleep(int) { fiber_yield(); }
static inline void __syncthreads() { g_block->arrive_and_wait(); }
static inline int __popc(unsigned x) { return __builtin_popcount(x); }
static inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
static inline int __clz(int x) { return __builtin_clz((unsigned)x); }
static inline int atomicAdd(int* p, int v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
static inline int atomicMin(int* p, int v) {
    int o = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (v < o && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {}
    return o;
}
static inline unsigned long long atomicOr(unsigned long long* p, unsigned long long v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
static inline int atomicMax(int* p, int v) {
    int o = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (v > o && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {}
    return o;
}
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
#define __hip_atomic_fetch_add(p, v, o, sc) __atomic_fetch_add((p), (v), __ATOMIC_SEQ_CST)
#define __hip_atomic_load(p, o, sc) __atomic_load_n((p), __ATOMIC_SEQ_CST)
#define __hip_atomic_store(p, v, o, sc) __atomic_store_n((p), (v), __ATOMIC_SEQ_CST)
using std::max;
using std::min;
#define PS_HOST_EMU 1
static std::atomic<long> g_postorder{0};      // ws_heap_postorder hits (coverage of the closed form)
#define PS_POSTORDER_COUNT g_postorder
#include "../lidar-visual-odometry_amd/csrc/pcl_sort.hpp"
#include "../lidar-visual-odometry_amd/csrc/ls_sort.hpp"
struct float4 { float x, y, z, w; };
static inline float4 make_float4(float x, float y, float z, float w) { return {x, y, z, w}; }
static inline unsigned atomicOr(unsigned* p, unsigned v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
namespace aloam {
inline float4 div4_by_count(float4 v, int k) { const float d = (float)k; return {v.x / d, v.y / d, v.z / d, v.w / d}; }
}
#include "../lidar-visual-odometry_amd/csrc/rvg.hpp"

// the level-synchronous sort (csrc/ls_sort.hpp) on one emulated workgroup of NT threads
template <int NT, int CPW>
static void run_ls(std::vector<unsigned long long>& E, const unsigned* rel = nullptr) {
    const int n = (int)E.size(), nmax = NT * CPW;
    std::vector<unsigned long long> scr((aloam::ls_scratch_bytes(NT, nmax) + 7) / 8);
    g_waves.clear();
    for (int w = 0; w < NT / WAVE; w++) {
        auto c = std::make_unique<WaveCtx>();
        c->bar = std::make_unique<FBarrier>(WAVE);
        g_waves.push_back(std::move(c));
    }
    g_block = std::make_unique<FBarrier>(NT);
    const int d0 = n > 1 ? 2 * (31 - __builtin_clz((unsigned)n)) : 0;
    run_group(NT, [&](int) { aloam::ls_sort<NT, CPW>(E.data(), n, d0, (unsigned char*)scr.data(), nmax, rel); });
}
// csrc/ls_sort.hpp's split-to-list + ls_sort_list: one emulated workgroup splits, then nw = 2 workgroups
// (run one after the other) sort their share of the segments
template <int NT, int CPW>
static void run_ls_list(std::vector<unsigned long long>& E, int limit, const unsigned* rel = nullptr) {
    const int n = (int)E.size(), cap = NT * CPW;
    std::vector<unsigned long long> scr((aloam::ls_global_scratch_bytes(NT, cap) + 7) / 8), EL(cap);
    std::vector<int> gseg(aloam::LS_SEGL);
    for (int phase = 0; phase < 3; phase++) {
        g_waves.clear();
        for (int w = 0; w < NT / WAVE; w++) {
            auto c = std::make_unique<WaveCtx>();
            c->bar = std::make_unique<FBarrier>(WAVE);
            g_waves.push_back(std::move(c));
        }
        g_block = std::make_unique<FBarrier>(NT);
        run_group(NT, [&](int) {
                if (phase == 0) aloam::ls_split_to_list<NT>(E.data(), n, limit, gseg.data(), (unsigned char*)scr.data(), rel);
                else aloam::ls_sort_list<NT, CPW>(E.data(), gseg.data(), phase - 1, 2, EL.data(), cap, (unsigned char*)scr.data(), rel);
            });
    }
}
// csrc/ls_sort.hpp's global sort: split in "global" memory by the workgroup phase of pcl_sort.hpp, segments
// staged through an LDS buffer of `cap` elements and sorted there by ls_sort
template <int NT, int CPW>
static void run_ls_global(std::vector<unsigned long long>& E, int cap) {
    const int n = (int)E.size();
    std::vector<unsigned long long> scr((aloam::ls_global_scratch_bytes(NT, cap) + 7) / 8), EL(cap);
    g_waves.clear();
    for (int w = 0; w < NT / WAVE; w++) {
        auto c = std::make_unique<WaveCtx>();
        c->bar = std::make_unique<FBarrier>(WAVE);
        g_waves.push_back(std::move(c));
    }
    g_block = std::make_unique<FBarrier>(NT);
    run_group(NT, [&](int) { aloam::ls_sort_global<NT, CPW>(E.data(), n, EL.data(), cap, (unsigned char*)scr.data()); });
}

// csrc/pcl_sort.hpp's wave heap sort (ws_heap_sort: closed form or six-level pops, early stop) on one
// emulated wave against libstdc++'s heap sort (std::partial_sort(f, l, l) = make_heap + sort_heap): every
// >= 3-point key's points in the same order. Mode 4.
// Mode 6: the same with the child-flag pops (fh_sort_heap_lds, flag bytes passed as fscr) up to FH_MAX points;
// every other trial without rel (all pops: the whole array must equal libstdc++'s).
// Mode 7 (fuzz): inputs aimed at the post-order closed form's edges (ws_heap_postorder, len <= 1024): lengths
// close to 1024, many duplicates, several relevant groups per segment, groups whose keys are the largest (popped
// first), the smallest or in the middle, and group members placed at the input's end (after make_heap they tend
// to sit in the last slots, the danger zone).
static void fuzz_input(std::vector<unsigned long long>& E, std::mt19937_64& rng, int t) {
    const int n = (int)E.size();
    const int style = t % 5;
    const unsigned kinds = style == 0 ? 2 + (unsigned)(n / 8) : 7u * (unsigned)n;
    for (int i = 0; i < n; i++) E[i] = ((unsigned long long)(unsigned)(style == 0 ? rng() % kinds : 7u * (unsigned)i + 3u) << 32);
    if (style != 0) std::shuffle(E.begin(), E.end(), rng);
    const int groups = 1 + (int)(rng() % 5);
    for (int g = 0; g < groups; g++) {
        unsigned kg;
        switch ((style + g) % 4) {
            case 0: kg = 7u * (unsigned)n + 100u + (unsigned)g; break;          // larger than every other key
            case 1: kg = 1u + (unsigned)g; break;                               // smaller than the others
            default: kg = (unsigned)(E[rng() % (unsigned)n] >> 32); break;      // an existing key
        }
        const int sz = 3 + (int)(rng() % 4);
        for (int j = 0; j < sz; j++) {
            // members at the input's end (style 3, 4) or anywhere
            const int p = style >= 3 && j % 2 == 0 ? n - 1 - (int)(rng() % (unsigned)std::max(1, n / 16)) : (int)(rng() % (unsigned)n);
            E[p] = ((unsigned long long)kg << 32);
        }
    }
    for (int i = 0; i < n; i++) E[i] = (E[i] & ~0xffffffffull) | (unsigned)i;
}
static int heap_trials(int trials, std::mt19937_64& rng, bool flags = false, bool fuzz = false) {
    int bad = 0;
    for (int t = 0; t < trials; t++) {
        const int n = fuzz ? 1024 - (int)(rng() % (t % 3 == 0 ? 1000 : 130))
                           : flags ? 2 + (int)(rng() % (t % 3 == 0 ? 200 : aloam::FH_MAX - 1)) : 17 + (int)(rng() % 1000);
        const unsigned kinds = 2 + (unsigned)(rng() % (unsigned)(t % 2 ? n / 3 + 1 : 4 * n));
        std::vector<unsigned long long> E(n);
        for (int i = 0; i < n; i++) E[i] = ((unsigned long long)(unsigned)(rng() % kinds) << 32) | (unsigned)i;
        if (fuzz) fuzz_input(E, rng, t);
        if (!fuzz && t % 4 == 3) {                // distinct keys but one group of 3-5 (few relevant points)
            for (int i = 0; i < n; i++) E[i] = ((unsigned long long)(unsigned)(7 * i + 3) << 32) | (unsigned)i;
            std::shuffle(E.begin(), E.end(), rng);
            const int g = 3 + (int)(rng() % 3);
            const unsigned kg = (unsigned)(E[rng() % n] >> 32);
            for (int j = 0; j < g; j++) { const int p = (int)(rng() % n); E[p] = ((unsigned long long)kg << 32) | (E[p] & 0xffffffffull); }
            for (int i = 0; i < n; i++) E[i] = (E[i] & ~0xffffffffull) | (unsigned)i;
        }
        if (!fuzz && t % 3 == 2) std::sort(E.begin(), E.begin() + n * 3 / 4);     // mostly ascending input
        std::vector<unsigned long long> A = E;
        std::partial_sort(A.begin(), A.end(), A.end(), [](unsigned long long a, unsigned long long b) { return (a >> 32) < (b >> 32); });
        std::map<unsigned, int> cnt;
        for (auto x : E) cnt[(unsigned)(x >> 32)]++;
        std::vector<unsigned> rel(n / 32 + 2, 0u);
        for (auto x : E) if (cnt[(unsigned)(x >> 32)] >= 3) { const unsigned i = (unsigned)x & 0xffffu; rel[i >> 5] |= 1u << (i & 31); }
        g_waves.clear();
        auto c = std::make_unique<WaveCtx>();
        c->bar = std::make_unique<FBarrier>(WAVE);
        g_waves.push_back(std::move(c));
        g_block = std::make_unique<FBarrier>(WAVE);
        std::vector<unsigned char> F(n, 0xee);
        const bool all = flags && !fuzz && t % 2 == 0;
        run_group(WAVE, [&](int) { aloam::ws_heap_sort(E.data(), 0, n, all ? nullptr : rel.data(), flags ? F.data() : nullptr); });
        if (all && E != A) { bad++; std::printf("heap (all pops) mismatch trial %d n %d kinds %u\n", t, n, kinds); continue; }
        auto order = [&](const std::vector<unsigned long long>& X) {
            std::vector<std::pair<unsigned, unsigned>> v;
            for (auto x : X) if (cnt[(unsigned)(x >> 32)] >= 3) v.push_back({(unsigned)(x >> 32), (unsigned)x & 0xffffu});
            std::stable_sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first < b.first; });
            return v;
        };
        std::vector<unsigned long long> B = E, A2 = A;
        std::sort(B.begin(), B.end());
        std::sort(A2.begin(), A2.end());
        if (B != A2 || order(A) != order(E)) { bad++; std::printf("heap mismatch trial %d n %d kinds %u\n", t, n, kinds); }
    }
    return bad;
}

// csrc/rvg.hpp's leaf sums: the batched form (rvg_reduce_batched, the map filter's) against the
// leaf-at-a-time loop on one emulated workgroup: S sorted by key (random tie order), rel = the points of
// >= 3-point leaves, fpos a random position per point; identical centroids (bits) and leaf counts. Mode 5.
static int reduce_trials(int trials, std::mt19937_64& rng) {
    constexpr int NT = 128;
    int bad = 0;
    for (int t = 0; t < trials; t++) {
        const int n = t % 7 == 0 ? (int)(rng() % 40) : 1 + (int)(rng() % 6000);
        const unsigned kinds = 1 + (unsigned)(rng() % (unsigned)(t % 3 == 0 ? n / 4 + 1 : 2 * n + 1));
        std::vector<unsigned long long> S(n);
        for (int i = 0; i < n; i++) S[i] = ((unsigned long long)(unsigned)(rng() % kinds) << 32) | (unsigned)i;
        std::shuffle(S.begin(), S.end(), rng);
        std::stable_sort(S.begin(), S.end(), [](unsigned long long a, unsigned long long b) { return (a >> 32) < (b >> 32); });
        std::vector<unsigned> rel(n / 32 + 2, 0u);
        for (int i = 0; i < n;) {
            int j = i;
            while (j < n && (S[j] >> 32) == (S[i] >> 32)) j++;
            if (j - i >= 3) for (int k = i; k < j; k++) { const unsigned x = (unsigned)S[k] & 0xffffu; rel[x >> 5] |= 1u << (x & 31); }
            i = j;
        }
        std::vector<int> fpos(n + 1);
        for (int i = 0; i < n; i++) fpos[i] = i;
        std::shuffle(fpos.begin(), fpos.begin() + n, rng);
        std::vector<float4> P(n + 1);
        for (int i = 0; i < n; i++) P[i] = {(float)(rng() % 100000) * 0.013f, (float)(rng() % 100000) * -0.007f, (float)(rng() % 1000) * 0.1f, (float)(i % 7)};
        std::vector<float4> out[2];
        int tot[2];
        for (int form = 0; form < 2; form++) {
            out[form].assign(n + 1, float4{-1.f, -1.f, -1.f, -1.f});
            std::vector<int> sc(2 * (NT / WAVE) + 2);
            g_waves.clear();
            for (int w = 0; w < NT / WAVE; w++) {
                auto c = std::make_unique<WaveCtx>();
                c->bar = std::make_unique<FBarrier>(WAVE);
                g_waves.push_back(std::move(c));
            }
            g_block = std::make_unique<FBarrier>(NT);
            std::vector<int> r(NT);
            run_group(NT, [&](int tt) {
                    auto pt = [&](int i) { return P[i]; };
                    auto of = [&](int q, float4 v) { out[form][q] = v; };
                    r[tt] = form == 0 ? aloam::rvg_reduce_loop<NT>(S.data(), n, rel.data(), fpos.data(), pt, of, sc.data())
                                      : aloam::rvg_reduce_batched<NT, 8>(S.data(), n, rel.data(), fpos.data(), pt, of, sc.data());
                });
            tot[form] = r[0];
        }
        if (tot[0] != tot[1] || std::memcmp(out[0].data(), out[1].data(), sizeof(float4) * (size_t)tot[0]) != 0) {
            bad++;
            std::printf("reduce mismatch trial %d n %d kinds %u leaves %d/%d\n", t, n, kinds, tot[0], tot[1]);
        }
    }
    return bad;
}

#ifndef NTHREADS
#define NTHREADS 128
#endif
int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 40;
    std::mt19937_64 rng(argc > 2 ? strtoull(argv[2], nullptr, 10) : 5);
    const int lsm = argc > 3 ? atoi(argv[3]) : 1;        // 1: csrc/ls_sort.hpp (n <= 128 * 16); 2: its global sort; 3: split + list sort
    const bool ls = lsm == 1;
    // 1: every trial a sorted prefix of distinct keys + a short unsorted tail of keys next to them (a map
    // cube's old points + the appended ones): introsort exhausts its depth on much of it (heap sorts)
    const bool cube_pattern = argc > 4 && atoi(argv[4]) == 1;
    // relevance mode (csrc/rvg.hpp): rel = the points of >= 3-point keys; then only those keys' point order
    // must equal std::sort's (heap sorts gated / queued / stopped early, other ties free)
    const bool relmode = argc > 5 && atoi(argv[5]) == 1;
    int bad = 0;
    if (lsm == 5) {
        bad = reduce_trials(trials, rng);
        std::printf("trials %d mismatches %d\n", trials, bad);
        return bad != 0;
    }
    if (lsm == 4 || lsm == 6 || lsm == 7) {
        bad = heap_trials(trials, rng, lsm == 6 || lsm == 7, lsm == 7);
        std::printf("postorder segments %ld\n", (long)g_postorder.load());
        std::printf("trials %d mismatches %d\n", trials, bad);
        return bad != 0;
    }
    for (int t = 0; t < trials; t++) {
        const bool big = t % 2 == 1;
        int n = big ? 4000 + (int)(rng() % 4000) : 1 + (int)(rng() % 4096);
        if (ls) n = 1 + (int)(rng() % 2048);
        if (t % 9 == 0) n = 1 + (int)(rng() % 40);
        const unsigned kinds = 1 + (unsigned)(rng() % (t % 3 == 0 ? 4 : (t % 3 == 1 ? 300 : 100000)));
        std::vector<unsigned long long> E(n);
        for (int i = 0; i < n; i++) {
            unsigned k;
            switch (t % 4) {
                case 0: k = (unsigned)(rng() % kinds); break;
                case 1: k = (unsigned)(i / (1 + (int)(rng() % 4))) % kinds; break;
                case 2: k = (unsigned)((n - i) / 3) % kinds; break;
                default: k = i < n / 2 ? (unsigned)(i / 8) : (unsigned)(rng() % kinds);
            }
            E[i] = ((unsigned long long)k << 32) | (unsigned)i;
        }
        if (cube_pattern) {
            const int tail = std::min(n - 1, 1 + (int)(rng() % (unsigned)(n / 20 + 1)));
            const int m = n - tail;
            unsigned k = 0;
            for (int i = 0; i < m; i++) { k += 1 + (unsigned)(rng() % 3); E[i] = ((unsigned long long)k << 32) | (unsigned)i; }
            for (int i = m; i < n; i++) {
                const unsigned kk = (unsigned)(E[rng() % (unsigned)m] >> 32) + (unsigned)(rng() % 3) - 1u;
                E[i] = ((unsigned long long)kk << 32) | (unsigned)i;
            }
        }
        std::vector<unsigned long long> A = E;
        std::sort(A.begin(), A.end(), [](unsigned long long a, unsigned long long b) { return (a >> 32) < (b >> 32); });
        std::vector<unsigned> rel((n + 31) / 32 + 1, 0u);
        if (relmode) {
            for (int i = 0; i < n;) {
                int j = i;
                while (j < n && (A[j] >> 32) == (A[i] >> 32)) j++;
                if (j - i >= 3) for (int k = i; k < j; k++) { const unsigned x = (unsigned)A[k] & 0xffffu; rel[x >> 5] |= 1u << (x & 31); }
                i = j;
            }
        }
        const unsigned* relp = relmode ? rel.data() : nullptr;
        if (lsm == 2) run_ls_global<128, 16>(E, 300 + (int)(rng() % 1748));
        else if (lsm == 3) run_ls_list<128, 16>(E, 100 + (int)(rng() % 1948), relp);
        else run_ls<128, 16>(E, relp);
        if (relmode) {            // every >= 3-point key: its points in std::sort's order; E a permutation
            std::vector<unsigned long long> B = E;
            std::sort(B.begin(), B.end());
            std::vector<unsigned long long> A2 = A;
            std::sort(A2.begin(), A2.end());
            bool ok = B == A2;
            std::vector<std::vector<unsigned>> ga, ge;
            auto order = [&](const std::vector<unsigned long long>& X) {
                std::vector<std::pair<unsigned, unsigned>> v;   // (key, index) of relevant points in X's order
                for (auto x : X) { const unsigned i = (unsigned)x & 0xffffu; if ((rel[i >> 5] >> (i & 31)) & 1u) v.push_back({(unsigned)(x >> 32), i}); }
                std::stable_sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first < b.first; });
                return v;
            };
            ok = ok && order(A) == order(E);
            if (!ok) { bad++; std::printf("rel mismatch trial %d n %d kinds %u mode %d\n", t, n, kinds, lsm); }
            continue;
        }
        if (A != E) {
            bad++;
            int first = 0;
            while (first < n && A[first] == E[first]) first++;
            std::printf("mismatch trial %d n %d kinds %u mode %d first diff at %d\n", t, n, kinds, lsm, first);
        }
    }
    std::printf("postorder segments %ld\n", (long)g_postorder.load());
    std::printf("trials %d mismatches %d\n", trials, bad);
    return bad != 0;
}
