// pcl_sort.hpp — PCL VoxelGrid's point order on gfx950: libstdc++ std::sort, replayed in parallel.
//
// pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.8.0, voxel_grid.hpp) pushes one (leaf index, point
// index) pair per point, std::sort's them by leaf index (an UNSTABLE introsort: the pairs of one leaf
// end up in an order that depends on the whole array) and sums every leaf's points in that order. The
// reference calls it at src/scanRegistration.cpp:401-405 (per scan line, leaf 0.2) and
// src/laserMapping.cpp:542-550 (the stacks), :788-801 (every surrounding map cube). fp32 sums depend on
// the order, so the device reproduces it exactly:
//
//   pcl_std_sort<NT, BIG>(E, n, scratch, nmax)             E in LDS
//   pcl_std_sort_global<NT>(gE, n, EL, cap, scratch)       E in global memory, staged through LDS
//
// leave E[0, n) (u64 = key << 32 | payload, compared by key only) in exactly the order
// std::sort(E, E + n, key-less) of libstdc++ produces. libstdc++'s sort is introsort_loop (median of
// first+1 / mid / last-1 moved to first, unguarded Hoare partition, recurse right, loop left, 16-element
// threshold, heap sort at depth 2 floor(log2 n)) followed by one insertion sort over the whole array.
//
// The partition of a segment [f, l) with pivot key K at f is computed, not simulated: with LS = the
// positions p in (f, l) with key >= K in ascending order ("left stops") and RS = the positions in
// [f, l) with key <= K in descending order ("right stops"), Hoare's two scans swap LS[j] <-> RS[j] for
// exactly the j < k with LS[j] < RS[j] (both sequences are monotone, so that is a prefix; LS[j] < RS[j]
// iff more than j right stops lie after LS[j]) and return cut = min(LS[k], RS[k-1]) (LS[k] when k = 0,
// RS[k-1] when LS runs out): every element a scan passes before a swap is untouched, and the first
// swapped element a scan meets stops it. The final insertion sort is stable and the partition property
// keeps every element inside its <= 16-element leaf, so each leaf is sorted (stable rank, lane-parallel)
// as soon as it forms. Depth-exhausted segments are heap-sorted by one lane, exactly as
// std::__partial_sort(first, last, last).
//
// Every step is element-parallel: a wave partitions a segment of <= PS_WMAX positions in 64-position
// chunks (chunk u = positions f + 64u + lane): one pass of ballots gives the stop masks, a DPP scan the
// per-chunk prefixes, and a second pass decides each left stop's swap from its own rank and its partner
// from the chunk prefixes held in the lanes (readlane), so no lane walks a mask bit by bit. Waves take
// segments from an LDS queue, push every right child for another wave and keep the left one
// (introsort's own recursion shape). Larger segments are first split level by level by the whole
// workgroup (per-thread chunks of <= 64 positions). Arrays in global memory are split by the workgroup
// until every segment fits the LDS buffer, then each segment is sorted there.
//
// The characterisation is checked against libstdc++ on the host (oracle/aloam_oracle.cpp
// oracle_pcl_replay_check, tests/test_oracle_pins.py), this file's code on the host by a per-lane
// thread emulation (tests/ps_emu.cpp, tests/test_pcl_sort_emu.py) and on the device by the VoxelGrid /
// scanRegistration / mapping parity tests against the oracle's PCL order.
#pragma once
#ifndef PS_HOST_EMU                          // tests/ps_emu.cpp compiles this file on the host
#include "aloam_device.hpp"
#endif

#ifndef PS_TS
#define PS_TS(level, k) do { } while (0)   // profiling builds: phase stamps (k_voxel.hip)
#endif
#ifndef PS_WSTAT
#define PS_CLK() 0ull                      // profiling builds: per-wave counters of the wave phase
#define PS_WSTAT(slot, v) do { } while (0)
#endif
// Work every lane of a wave does identically (same loads, same stores: SIMT executes each access for all
// lanes at once). The host emulator (tests/ps_emu.cpp) runs lanes as unsynchronised threads, so there one
// lane does it.
#ifdef PS_HOST_EMU
#define PS_SAME(...) do { if (lane_id() == 0) { __VA_ARGS__; } __builtin_amdgcn_wave_barrier(); } while (0)
#else
#define PS_SAME(...) do { __VA_ARGS__; } while (0)
#endif
#ifdef ALOAM_PS_CHECK                      // debug builds: report indices outside their segment
#define PS_CHECK(cond, ...) do { if (!(cond)) printf(__VA_ARGS__); } while (0)
#else
#define PS_CHECK(cond, ...) do { } while (0)
#endif

namespace aloam {

constexpr int PS_THRESHOLD = 16;    // libstdc++ _S_threshold
constexpr int PS_WMAX = 4096;       // segments one wave partitions (64 chunks of 64 positions)
constexpr int PS_MAX_CHUNK = 64;    // workgroup phase: positions per thread (u64 stop masks)
constexpr int PS_WGSEG = 32;        // workgroup phase: segments split at once (n <= NT * 64)
constexpr int PS_GLIST = 320;       // global sorts: segments staged through LDS (<= 2 per split x depth)
constexpr int PS_LANE_MAX = 64;     // segments of <= this many elements: one lane each (ps_lane_sort)

// Scratch (ints, LDS, 8-byte aligned): header | exscan words | workgroup phase arrays (BIG) | segment
// queue (3 ints per queued segment) [| staged-segment list (global sorts)]
__host__ __device__ constexpr int ps_wg_ints(int NT) { return 7 * (NT + 1) + 8 * PS_WGSEG; }
__host__ __device__ constexpr int ps_qcap(int n) { return n / (PS_THRESHOLD + 1) + 64; }   // (overflow: ps_wave_phase)
__host__ __device__ constexpr int ps_scratch_ints(int NT, int nmax, bool big) {
    return 16 + 2 * (NT / 64) + (big ? ps_wg_ints(NT) : 0) + 3 * ps_qcap(nmax);
}
__host__ __device__ constexpr int ps_scratch_ints_global(int NT, int cap) {
    return ps_scratch_ints(NT, cap, true) + 3 * PS_GLIST;
}

__device__ __forceinline__ unsigned ps_key(unsigned long long e) { return (unsigned)(e >> 32); }
// key of E[p] without the payload (high word, little endian)
__device__ __forceinline__ unsigned ps_keyat(const unsigned long long* E, int p) { return ((const unsigned*)E)[2 * p + 1]; }
// A wave-uniform value as such for the compiler (SGPR): the wave phase's loop bounds and branch
// conditions must be scalar, or the loops are compiled as divergent ones and run under narrowed exec
// masks, which breaks the ballots and scans inside them.
__device__ __forceinline__ int ps_u(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long ps_rl64(unsigned long long v, int lane) {
    return ((unsigned long long)(unsigned)readlane_i((int)(v >> 32), lane) << 32) | (unsigned)readlane_i((int)v, lane);
}
__device__ __forceinline__ int ps_msb(unsigned long long m) { return 63 - __builtin_clzll(m); }   // m != 0
// Single-writer updates inside the wave phase are done by the WHOLE wave, branch-free: an `if (lane ==
// 0)` block at a loop boundary was merged into the loop's exit mask by the compiler (lane 0 left the
// loop, lanes 1-63 kept iterating). Atomics: every lane adds, only lane 0 a non-zero amount, lane 0's
// old value broadcast; stores: every lane writes the same value.
__device__ __forceinline__ int ps_wave_add(int* p, int v, int order = __ATOMIC_RELAXED) {
    const int r = order == __ATOMIC_RELEASE
                      ? __hip_atomic_fetch_add(p, lane_id() == 0 ? v : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP)
                      : __hip_atomic_fetch_add(p, lane_id() == 0 ? v : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return ps_u(r);
}

template <bool G>
__device__ __forceinline__ void ps_bar() {
    if (G) __syncthreads();
    else lds_barrier();
}
// this wave's E accesses (LDS, or global with G) ordered before its next ones, across lanes
template <bool G>
__device__ __forceinline__ void ps_wsync() {
#ifndef PS_HOST_EMU
    if (G) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// position of the r-th set bit (0-based) of m (r < popcount(m))
__device__ __forceinline__ int ps_select_bit(unsigned long long m, int r) {
    int pos = 0;
    int c = __popc((unsigned)m);
    if (r >= c) { r -= c; m >>= 32; pos = 32; }
    unsigned x = (unsigned)m;
    c = __popc(x & 0xffffu);
    if (r >= c) { r -= c; x >>= 16; pos += 16; }
    c = __popc(x & 0xffu);
    if (r >= c) { r -= c; x >>= 8; pos += 8; }
    c = __popc(x & 0xfu);
    if (r >= c) { r -= c; x >>= 4; pos += 4; }
    c = __popc(x & 0x3u);
    if (r >= c) { r -= c; x >>= 2; pos += 2; }
    c = (int)(x & 1u);
    if (r >= c) pos += 1;
    return pos;
}

// stable insertion sort of E[f, l) by key (libstdc++ __insertion_sort / __unguarded_linear_insert)
__device__ __forceinline__ void ps_insertion_sort(unsigned long long* E, int f, int l) {
    for (int i = f + 1; i < l; i++) {
        const unsigned long long v = E[i];
        const unsigned kv = ps_key(v);
        int j = i;
        while (j > f && kv < ps_key(E[j - 1])) { E[j] = E[j - 1]; j--; }
        E[j] = v;
    }
}
// std::__adjust_heap / __push_heap on key order
__device__ inline void ps_adjust_heap(unsigned long long* first, int hole, int len, unsigned long long value) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (ps_key(first[child]) < ps_key(first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && ps_key(first[parent]) < ps_key(value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}
// std::__partial_sort(first, last, last): __make_heap then __sort_heap
__device__ inline void ps_heap_sort(unsigned long long* first, unsigned long long* last) {
    const int len = (int)(last - first);
    if (len >= 2) {
        int parent = (len - 2) / 2;
        while (true) {
            ps_adjust_heap(first, parent, len, first[parent]);
            if (parent == 0) break;
            parent--;
        }
    }
    while (last - first > 1) {
        --last;
        const unsigned long long v = *last;
        *last = *first;
        ps_adjust_heap(first, 0, (int)(last - first), v);
    }
}
// The whole std::sort by one thread (arrays beyond NT * PS_MAX_CHUNK elements): introsort_loop with an
// explicit stack (the right part is pushed, the left continued — disjoint ranges, same result), then
// __final_insertion_sort.
__device__ __noinline__ void ps_serial_std_sort(unsigned long long* E, int n) {
    if (n <= 1) return;
    int sf[64], sl[64], sd[64], sp = 0;
    sf[0] = 0; sl[0] = n; sd[0] = 2 * (31 - __builtin_clz((unsigned)n)); sp = 1;
    while (sp > 0) {
        sp--;
        int f = sf[sp], l = sl[sp], d = sd[sp];
        while (l - f > PS_THRESHOLD) {
            if (d == 0) { ps_heap_sort(E + f, E + l); break; }
            d--;
            const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
            const unsigned ka = ps_key(E[a]), kb = ps_key(E[b]), kc = ps_key(E[c]);
            const int pick = ka < kb ? (kb < kc ? b : (ka < kc ? c : a)) : (ka < kc ? a : (kb < kc ? c : b));
            { const unsigned long long t = E[f]; E[f] = E[pick]; E[pick] = t; }
            const unsigned kp = ps_key(E[f]);
            int lo = f + 1, hi = l;
            while (true) {
                while (ps_key(E[lo]) < kp) ++lo;
                --hi;
                while (kp < ps_key(E[hi])) --hi;
                if (!(lo < hi)) break;
                const unsigned long long t = E[lo]; E[lo] = E[hi]; E[hi] = t;
                ++lo;
            }
            sf[sp] = lo; sl[sp] = l; sd[sp] = d; sp++;
            l = lo;
        }
    }
    ps_insertion_sort(E, 0, n);   // == __final_insertion_sort: both are stable insertion sorts
}

// __move_median_to_first(first, first + 1, mid, last - 1): returns the pivot key
__device__ __forceinline__ unsigned ps_median_to_first(unsigned long long* E, int f, int l) {
    const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const unsigned ka = ps_key(E[a]), kb = ps_key(E[b]), kc = ps_key(E[c]);
    int pick;
    if (ka < kb) pick = kb < kc ? b : (ka < kc ? c : a);
    else pick = ka < kc ? a : (kb < kc ? c : b);
    const unsigned long long ef = E[f], ep = E[pick];
    E[f] = ep;
    E[pick] = ef;
    return ps_key(ep);
}

// One lane's whole std::sort of E[f0, l0) (l0 - f0 <= PS_LANE_MAX) from depth d: introsort_loop (right
// parts > 16 on a 3-entry register stack: they are disjoint, so at most 3 wait at once), then the final
// stable insertion sort over the segment (== sorting its <= 16-element leaves). No wave operations
// inside: the lanes of a wave run it on 64 different segments at once.
__device__ __forceinline__ void ps_lane_sort(unsigned long long* E, const int f0, const int l0, int d) {
    int f = f0, l = l0, sp = 0;
    int af = 0, al = 0, ad = 0, bf = 0, bl = 0, bd = 0, cf = 0, cl = 0, cd = 0;
    for (;;) {
        while (l - f > PS_THRESHOLD) {
            if (d == 0) { ps_heap_sort(E + f, E + l); break; }
            d--;
            const unsigned kp = ps_median_to_first(E, f, l);
            int lo = f + 1, hi = l;
            while (true) {
                while (ps_key(E[lo]) < kp) ++lo;
                --hi;
                while (kp < ps_key(E[hi])) --hi;
                if (!(lo < hi)) break;
                const unsigned long long t = E[lo]; E[lo] = E[hi]; E[hi] = t;
                ++lo;
            }
            if (l - lo > PS_THRESHOLD) {
                if (sp == 0) { af = lo; al = l; ad = d; }
                else if (sp == 1) { bf = lo; bl = l; bd = d; }
                else { cf = lo; cl = l; cd = d; }
                sp++;
            }
            l = lo;
        }
        if (sp == 0) break;
        sp--;
        if (sp == 0) { f = af; l = al; d = ad; }
        else if (sp == 1) { f = bf; l = bl; d = bd; }
        else { f = cf; l = cl; d = cd; }
    }
    ps_insertion_sort(E, f0, l0);
}

// ---- one wave ---------------------------------------------------------------------------------
// Leaf (m <= 16 elements): stable rank of every element by lane, then the scatter.
template <bool G>
__device__ __forceinline__ void ps_wave_leaf(unsigned long long* E, int f, int l) {
    const int m = l - f;
    if (m < 2) return;
    const int lane = lane_id();
    const bool act = lane < m;
    const unsigned long long v = act ? E[f + lane] : ~0ull;
    const unsigned kv = ps_key(v);
    int rank = 0;
#pragma unroll
    for (int i = 0; i < PS_THRESHOLD; i++) {
        const unsigned ki = (unsigned)__shfl((int)kv, i, WAVE);
        rank += (i < m) && (ki < kv || (ki == kv && i < lane));
    }
    ps_wsync<G>();
    if (act) E[f + rank] = v;
    ps_wsync<G>();
}

// Partition of E[f, l) (17 <= l - f <= PS_WMAX) by one wave; returns the cut. Chunk u = positions
// f + 64u + lane; lane u keeps chunk u's stop masks (myL, myR) and exclusive stop prefixes (pL, pR).
template <bool G>
__device__ int ps_wave_partition(unsigned long long* E, const int f, const int l) {
    const int lane = lane_id();
    int k0 = 0;
    PS_SAME(k0 = (int)ps_median_to_first(E, f, l));
    const unsigned K = (unsigned)ps_u(k0);
    ps_wsync<G>();
    const int nch = ps_u((l - f + 63) >> 6);
    unsigned long long myL = 0, myR = 0;
    for (int c0 = 0; c0 < nch; c0 += 4) {
        unsigned kk[4];
        bool in[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = f + ((c0 + u) << 6) + lane;
            in[u] = c0 + u < nch && p < l;
            kk[u] = in[u] ? ps_keyat(E, p) : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int p = f + ((c0 + u) << 6) + lane;
            const unsigned long long bl = __ballot(in[u] && p > f && kk[u] >= K);
            const unsigned long long br = __ballot(in[u] && kk[u] <= K);
            myL = lane == c0 + u ? bl : myL;
            myR = lane == c0 + u ? br : myR;
        }
    }
    const int cl = __popcll(myL), cr = __popcll(myR);
    const int iL = wave_incl_scan(cl), iR = wave_incl_scan(cr);
    const int pL = iL - cl, pR = iR - cr;
    const int nL = ps_u(readlane_i(iL, WAVE - 1)), nR = ps_u(readlane_i(iR, WAVE - 1));
    const bool valid = lane < nch;
    const unsigned long long lt = (1ull << lane) - 1ull, le = lt | (1ull << lane);
    // the swaps: left stop of rank j swaps with RS[j] iff more than j right stops lie after it; the
    // swapped ones are a prefix of the left stops, so the chunk loop ends at the first refusal
    int k = 0;
    for (int u = 0; u < nch; u++) {
        const unsigned long long bL = ps_rl64(myL, u);
        if (bL == 0ull) continue;
        const unsigned long long bR = ps_rl64(myR, u);
        const int pLu = ps_u(readlane_i(pL, u)), pRu = ps_u(readlane_i(pR, u));
        const int j = pLu + __popcll(bL & lt);
        const int after = nR - pRu - __popcll(bR & le);
        const bool sw = ((bL >> lane) & 1ull) && j < after;
        const unsigned long long bs = __ballot(sw);
        const int nsw = __popcll(bs);
        if (nsw > 0) {
            // partners: RS[j] = the right stop of ascending rank a = nR - 1 - j; this chunk's swaps
            // take ranks [aLo, aHi], found in chunks cLo..cHi (last chunk whose prefix is <= the rank)
            const int aHi = nR - 1 - pLu, aLo = aHi - nsw + 1;
            const int cHi = ps_msb(__ballot(valid && pR <= aHi)), cLo = ps_msb(__ballot(valid && pR <= aLo));
            const int a = nR - 1 - j;
            int q = -1;
            for (int c = cHi; c >= cLo; c--) {
                const int pRc = ps_u(readlane_i(pR, c));
                const unsigned long long mRc = ps_rl64(myR, c);
                if (sw && q < 0 && a >= pRc) q = f + (c << 6) + ps_select_bit(mRc, a - pRc);
            }
            if (sw) {
                const int p = f + (u << 6) + lane;
                PS_CHECK(p > f && p < l && q >= f && q < l && p < q, "ps swap: f %d l %d p %d q %d j %d nL %d nR %d\n", f, l, p, q, j, nL, nR);
                const unsigned long long ep = E[p], eq = E[q];
                E[p] = eq;
                E[q] = ep;
            }
        }
        k += nsw;
        if (nsw < __popcll(bL)) break;
    }
    k = ps_u(k);
    ps_wsync<G>();
    // the cut: LS[k] (k < nL) and RS[k-1] (k >= 1)
    int cut = 0x7fffffff;
    if (k < nL) {
        const int c = ps_msb(__ballot(valid && pL <= k));
        cut = f + (c << 6) + ps_select_bit(ps_rl64(myL, c), k - ps_u(readlane_i(pL, c)));
    }
    if (k >= 1) {
        const int a = nR - k;
        const int c = ps_msb(__ballot(valid && pR <= a));
        cut = min(cut, f + (c << 6) + ps_select_bit(ps_rl64(myR, c), a - ps_u(readlane_i(pR, c))));
    }
    cut = ps_u(cut);
    PS_CHECK(cut > f && cut < l, "ps cut: f %d l %d cut %d k %d nL %d nR %d\n", f, l, cut, k, nL, nR);
    return cut;
}

// Work queue of segments (f, l, depth + 1 as the ready mark). hdr: [1] head, [2] tail, [3] pending
// (queued or in progress). ps_push: ONE lane (the workgroup phase's thread 0); ps_push_wave: a whole
// wave, uniform arguments. False when the queue is full (the slot claimed past qcap is never filled: a
// wave waiting on it leaves when pending reaches zero).
__device__ __forceinline__ bool ps_push_wave(int* hdr, int* Q, int qcap, int f, int l, int d) {
    const int s = ps_wave_add(&hdr[2], 1);
    if (s >= qcap) return false;
    PS_CHECK(f >= 0 && l > f + PS_LANE_MAX, "ps push: f %d l %d d %d s %d qcap %d\n", f, l, d, s, qcap);
    ps_wave_add(&hdr[3], 1);
    Q[3 * s] = f;
    Q[3 * s + 1] = l;
    __hip_atomic_store(&Q[3 * s + 2], d + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return true;
}
__device__ __forceinline__ bool ps_push(int* tail, int* pend, int* Q, int qcap, int f, int l, int d) {
    const int s = __hip_atomic_fetch_add(tail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (s >= qcap) return false;
    PS_CHECK(f >= 0 && l >= f + 2, "ps push: f %d l %d d %d s %d qcap %d\n", f, l, d, s, qcap);
    __hip_atomic_fetch_add(pend, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    Q[3 * s] = f;
    Q[3 * s + 1] = l;
    __hip_atomic_store(&Q[3 * s + 2], d + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return true;
}

// every wave: take segments until no segment is queued or in progress. Every branch below is on a
// wave-uniform scalar (ps_u), so the wave runs it with its full exec mask. Segments of <= PS_LANE_MAX
// elements are collected, one per lane (lane i holds entry i), and sorted 64 at a time by ps_lane_sort.
template <bool G>
__device__ void ps_wave_phase(unsigned long long* E, int* hdr, int* Q, int qcap) {
    const int lane = lane_id();
    int lf = 0, ll = 0, ld = 0, ln = 0;                            // the collected small segments
    auto flush = [&]() {
        ps_wsync<G>();
        const unsigned long long tl = PS_CLK();
        if (lane < ln) ps_lane_sort(E, lf, ll, ld);
        ps_wsync<G>();
        PS_WSTAT(4, PS_CLK() - tl);
        PS_WSTAT(5, 1);
        ln = 0;
    };
    auto collect = [&](int f, int l, int d) {                      // uniform arguments
        if (ln == WAVE) flush();
        lf = lane == ln ? f : lf;
        ll = lane == ln ? l : ll;
        ld = lane == ln ? d : ld;
        ln = ps_u(ln + 1);
    };
    for (;;) {
        const int s = ps_wave_add(&hdr[1], 1);
        int mark = 0, quit = 0;
        const unsigned long long tw = PS_CLK();
        for (;;) {
            const int rdy = ps_u(s < qcap ? __hip_atomic_load(&Q[3 * min(s, qcap - 1) + 2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) : 0);
            const int pend = ps_u(__hip_atomic_load(&hdr[3], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (rdy != 0) { mark = rdy; break; }
            if (pend == 0) { quit = 1; break; }                    // nothing queued, nothing running
            __builtin_amdgcn_s_sleep(1);
        }
        PS_WSTAT(0, PS_CLK() - tw);
        if (ps_u(quit)) break;
        int f = ps_u(Q[3 * s]), l = ps_u(Q[3 * s + 1]);
        int d = ps_u(mark - 1);
        // right children the full queue refused stay with this wave: a stack held one entry per lane
        // (at most one per recursion level, <= 2 log2 n <= 32)
        int sp = 0, stf = 0, stl = 0, std_ = 0;
        for (;;) {
            for (;;) {                                             // introsort_loop on [f, l)
                if (l - f <= PS_LANE_MAX) {
                    if (l - f >= 2) collect(f, l, d);
                    break;
                }
                if (d == 0) {
                    PS_SAME(ps_heap_sort(E + f, E + l));           // (rare)
                    ps_wsync<G>();
                    break;
                }
                d = ps_u(d - 1);
                const unsigned long long tp = PS_CLK();
                const int cut = ps_wave_partition<G>(E, f, l);
                PS_WSTAT(1, PS_CLK() - tp);
                PS_WSTAT(2, 1);
                PS_WSTAT(3, l - f);
                if (l - cut > PS_LANE_MAX) {
                    if (!ps_push_wave(hdr, Q, qcap, cut, l, d)) {
                        stf = lane == sp ? cut : stf;
                        stl = lane == sp ? l : stl;
                        std_ = lane == sp ? d : std_;
                        sp = ps_u(sp + 1);
                    }
                } else if (l - cut >= 2) {
                    collect(cut, l, d);
                }
                l = ps_u(cut);
            }
            if (sp == 0) break;
            sp = ps_u(sp - 1);
            f = ps_u(readlane_i(stf, sp)); l = ps_u(readlane_i(stl, sp)); d = ps_u(readlane_i(std_, sp));
        }
        ps_wave_add(&hdr[3], -1, __ATOMIC_RELEASE);
    }
    if (ln > 0) flush();
}

// ---- the workgroup phase (segments > limit) ----------------------------------------------------
__device__ __forceinline__ int ps_count_before(const int* pref, const unsigned long long* mask, int p, int C) {
    const int t = p / C, o = p - t * C;
    return pref[t] + (o ? __popcll(mask[t] & ((1ull << o) - 1ull)) : 0);
}
// exclusive scan of (a, b) over the NT threads; ws >= 2 NT/64 ints. Threads still read ws on return:
// the caller's next barrier must come before ws is written again.
template <int NT>
__device__ __forceinline__ void ps_exscan2(int& a, int& b, int* ws, int& ta, int& tb) {
    constexpr int NW = NT / WAVE;
    const int lane = lane_id(), w = threadIdx.x / WAVE;
    const int ia = wave_incl_scan(a), ib = wave_incl_scan(b);
    if (lane == WAVE - 1) { ws[w] = ia; ws[NW + w] = ib; }
    lds_barrier();
    int ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const int x = ws[i], y = ws[NW + i];
        if (i < w) { ba += x; bb += y; }
        sa += x; sb += y;
    }
    a = ba + ia - a;
    b = bb + ib - b;
    ta = sa; tb = sb;
}
// stop with global index g: position, searching chunks [tlo, thi]
__device__ __forceinline__ int ps_select(const int* pref, const unsigned long long* mask, int g, int tlo, int thi, int C) {
    while (tlo < thi) {
        const int mid = (tlo + thi + 1) >> 1;
        if (pref[mid] <= g) tlo = mid;
        else thi = mid - 1;
    }
    return tlo * C + ps_select_bit(mask[tlo], g - pref[tlo]);
}
// the right stop before position q (exclusive) in the chunk masks, walking down: returns its position
__device__ __forceinline__ int ps_prev_stop(const unsigned long long* mask, int q, int C) {
    int t = q / C;
    unsigned long long rest = mask[t] & ((1ull << (q - t * C)) - 1ull);
    while (rest == 0ull && t > 0) rest = mask[--t];
    return t * C + ps_msb(rest);
}

// Split every segment listed in U's big list (Bf/Bl/Bd, sorted by f, hdr[0] entries) that is longer
// than `limit`, level by level, over positions [0, n): children > limit stay listed, the others are
// pushed to the sink queue (tail/pend/Qs/qcap; segments of <= 16 too: the wave phase sorts leaves).
// Elements stay in E (LDS, or global with G: loads are batched 8 at a time).
template <int NT, bool G>
__device__ void ps_wg_split(unsigned long long* E, const int n, int* sc, const int limit, int* tail, int* pend, int* Qs,
                            const int qcap) {
    const int tid = threadIdx.x;
    int* hdr = sc;
    int* ws = sc + 16;
    int* U = ws + 2 * (NT / WAVE);
    unsigned long long* maskL = (unsigned long long*)U;
    unsigned long long* maskR = maskL + NT + 1;
    int* prefL = (int*)(maskR + NT + 1);
    int* prefR = prefL + NT + 1;
    int* sidx = prefR + NT + 1;
    int* Bf = sidx + NT + 1;                         // big segments: f, l, depth, K, k, cut
    int* Bl = Bf + PS_WGSEG;
    int* Bd = Bl + PS_WGSEG;
    unsigned* Bk = (unsigned*)(Bd + PS_WGSEG);
    int* Bkk = Bd + 2 * PS_WGSEG;
    int* Bcut = Bd + 3 * PS_WGSEG;
    const int C = (n + NT - 1) / NT;
    const int nch = (n + C - 1) / C;
    for (int lvl = 0;; lvl++) {
        (void)lvl;
        const int nbig = ps_u(hdr[0]);
        PS_TS(lvl, 0);
        if (nbig == 0) break;
        // depth-exhausted segments: heap sort (rare), emptied from the list below
        for (int s = tid; s < nbig; s += NT)
            if (Bd[s] == 0) ps_heap_sort(E + Bf[s], E + Bl[s]);
        if (tid < nbig && Bd[tid] > 0) { Bk[tid] = ps_median_to_first(E, Bf[tid], Bl[tid]); Bkk[tid] = 0; }
        ps_bar<G>();
        int cl = 0, cr = 0;
        unsigned long long mL = 0, mR = 0;
        const int p0 = tid * C;
        int s0 = -1;
        if (tid < nch) {
            const int p1 = min(n, p0 + C);
            int lo = 0, hi = nbig;                       // s0 = the last segment with f <= p0 (-1: none)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (Bf[mid] <= p0) lo = mid + 1;
                else hi = mid;
            }
            int s = lo - 1;
            s0 = s;
            // the current segment in registers: f, l (l = f: inactive), K, and the next segment's f
            int cf = 0, ce = 0, nf = s + 1 < nbig ? Bf[s + 1] : 0x7fffffff;
            unsigned ck = 0;
            if (s >= 0) { cf = Bf[s]; ce = Bd[s] > 0 ? Bl[s] : cf; ck = Bk[s]; }
            for (int pb = p0; pb < p1; pb += 8) {
                unsigned kk[8];
#pragma unroll
                for (int i = 0; i < 8; i++) kk[i] = pb + i < p1 ? ps_keyat(E, pb + i) : 0u;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int p = pb + i;
                    if (p < p1) {
                        while (p >= nf) {
                            s++;
                            cf = Bf[s]; ce = Bd[s] > 0 ? Bl[s] : cf; ck = Bk[s];
                            nf = s + 1 < nbig ? Bf[s + 1] : 0x7fffffff;
                        }
                        if (p >= cf && p < ce) {
                            if (p > cf && kk[i] >= ck) mL |= 1ull << (p - p0);
                            if (kk[i] <= ck) mR |= 1ull << (p - p0);
                        }
                    }
                }
            }
            cl = __popcll(mL);
            cr = __popcll(mR);
        }
        int tl, tr;
        ps_exscan2<NT>(cl, cr, ws, tl, tr);
        if (tid < nch) { prefL[tid] = cl; prefR[tid] = cr; maskL[tid] = mL; maskR[tid] = mR; sidx[tid] = s0; }
        if (tid == 0) { prefL[nch] = tl; prefR[nch] = tr; maskL[nch] = 0ull; maskR[nch] = 0ull; }
        lds_barrier();
        PS_TS(lvl, 1);
        // k per segment: left stops with more right stops after them than left stops before them (this
        // thread's stops in registers; the segment's bounds once per segment)
        if (tid < nch && mL) {
            int s = s0, cur = -1, bL = 0, eR = 0, cnt = 0, j = 0;
            for (unsigned long long m = mL; m; m &= m - 1ull) {
                const int b = __builtin_ctzll(m), p = p0 + b;
                while (s + 1 < nbig && Bf[s + 1] <= p) s++;
                if (s != cur) {
                    if (cur >= 0 && cnt) atomicAdd(&Bkk[cur], cnt);
                    cur = s; cnt = 0;
                    bL = ps_count_before(prefL, maskL, Bf[s], C);
                    eR = ps_count_before(prefR, maskR, Bl[s], C);
                }
                j = cl + __popcll(mL & ((1ull << b) - 1ull)) - bL;
                const int after = eR - (cr + __popcll(mR & ((2ull << b) - 1ull)));
                cnt += j < after;
            }
            if (cur >= 0 && cnt) atomicAdd(&Bkk[cur], cnt);
        }
        lds_barrier();
        PS_TS(lvl, 2);
        // the swaps, 8 pairs in flight: partners from one select, then walking down the right stops
        if (tid < nch && mL) {
            int s = s0, cur = -1, bL = 0, eR = 0, k = 0, q = 0;
            unsigned long long m = mL;
            while (m) {
                int pp[8], qq[8];
                bool v[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    v[i] = false;
                    while (m && !v[i]) {
                        const int b = __builtin_ctzll(m), p = p0 + b;
                        m &= m - 1ull;
                        while (s + 1 < nbig && Bf[s + 1] <= p) s++;
                        if (s != cur) {
                            cur = s;
                            bL = ps_count_before(prefL, maskL, Bf[s], C);
                            eR = ps_count_before(prefR, maskR, Bl[s], C);
                            k = Bkk[s];
                            q = -1;
                        }
                        const int j = cl + __popcll(mL & ((1ull << b) - 1ull)) - bL;
                        if (j >= k) continue;
                        q = q < 0 ? ps_select(prefR, maskR, eR - 1 - j, Bf[s] / C, (Bl[s] - 1) / C, C) : ps_prev_stop(maskR, q, C);
                        PS_CHECK(p > Bf[s] && p < Bl[s] && q > p && q < Bl[s], "ps wg swap: f %d l %d p %d q %d\n", Bf[s], Bl[s], p, q);
                        pp[i] = p; qq[i] = q; v[i] = true;
                    }
                }
                unsigned long long ep[8], eq[8];
#pragma unroll
                for (int i = 0; i < 8; i++)
                    if (v[i]) { ep[i] = E[pp[i]]; eq[i] = E[qq[i]]; }
#pragma unroll
                for (int i = 0; i < 8; i++)
                    if (v[i]) { E[pp[i]] = eq[i]; E[qq[i]] = ep[i]; }
            }
        }
        if (tid < nbig && Bd[tid] > 0) {
            const int f = Bf[tid], l = Bl[tid], k = Bkk[tid];
            const int tlo = f / C, thi = (l - 1) / C;
            const int bL = ps_count_before(prefL, maskL, f, C), nL = ps_count_before(prefL, maskL, l, C) - bL;
            const int eR = ps_count_before(prefR, maskR, l, C);
            int cut;
            if (k < nL) {
                cut = ps_select(prefL, maskL, bL + k, tlo, thi, C);
                if (k > 0) cut = min(cut, ps_select(prefR, maskR, eR - k, tlo, thi, C));
            } else {
                cut = ps_select(prefR, maskR, eR - k, tlo, thi, C);
            }
            Bcut[tid] = cut;
        }
        ps_bar<G>();
        PS_TS(lvl, 3);
        // children: > limit stay listed, the rest go to the sink (a full sink: leaves sorted here,
        // longer ones stay listed)
        if (tid == 0) {
            int nn = 0;
            int nf[2 * PS_WGSEG], nl[2 * PS_WGSEG], nd[2 * PS_WGSEG];
            for (int s = 0; s < nbig; s++) {
                if (Bd[s] == 0) continue;
                const int d = Bd[s] - 1;
                const int ch[3] = {Bf[s], Bcut[s], Bl[s]};
                for (int h = 0; h < 2; h++) {
                    const int f = ch[h], l = ch[h + 1];
                    if (l - f > limit) { nf[nn] = f; nl[nn] = l; nd[nn] = d; nn++; }
                    else if (l - f >= 2 && !ps_push(tail, pend, Qs, qcap, f, l, d)) {
                        if (l - f <= PS_THRESHOLD) ps_insertion_sort(E, f, l);
                        else { nf[nn] = f; nl[nn] = l; nd[nn] = d; nn++; }
                    }
                }
            }
            for (int s = 0; s < nn; s++) { Bf[s] = nf[s]; Bl[s] = nl[s]; Bd[s] = nd[s]; }
            hdr[0] = nn;
        }
        ps_bar<G>();
        PS_TS(lvl, 4);
    }
}

// The sort of E[0, n) in LDS from depth d0 (the caller's segment of a larger sort: its remaining
// introsort depth). sc: ps_scratch_ints(NT, nmax, BIG) ints of LDS (8-byte aligned), nmax >= n. BIG =
// false: the caller guarantees n <= PS_WMAX. n <= NT * PS_MAX_CHUNK. All NT threads call it with the
// same arguments. Ends with a barrier.
template <int NT, bool BIG>
__device__ void ps_sort_lds(unsigned long long* E, const int n, const int d0, int* sc, const int nmax) {
    const int tid = threadIdx.x;
    int* hdr = sc;
    int* Q = sc + 16 + 2 * (NT / WAVE) + (BIG ? ps_wg_ints(NT) : 0);
    const int qcap = ps_qcap(nmax);
    for (int i = tid; i < 3 * qcap; i += NT) Q[i] = 0;
    if (tid < 16) hdr[tid] = 0;
    lds_barrier();
    if (!BIG || n <= PS_WMAX) {
        if (tid == 0) {
            if (n <= PS_THRESHOLD) ps_insertion_sort(E, 0, n);
            else if (d0 == 0) ps_heap_sort(E, E + n);
            else ps_push(&hdr[2], &hdr[3], Q, qcap, 0, n, d0);
        }
    } else {
        int* Bf = sc + 16 + 2 * (NT / WAVE) + 7 * (NT + 1);
        if (tid == 0) { Bf[0] = 0; Bf[PS_WGSEG] = n; Bf[2 * PS_WGSEG] = d0; hdr[0] = 1; }
        lds_barrier();
        ps_wg_split<NT, false>(E, n, sc, PS_WMAX, &hdr[2], &hdr[3], Q, qcap);
    }
    lds_barrier();
    PS_TS(60, 0);
    ps_wave_phase<false>(E, hdr, Q, qcap);
    lds_barrier();
    PS_TS(60, 1);
}

template <int NT, bool BIG>
__device__ void pcl_std_sort(unsigned long long* E, const int n, int* sc, const int nmax) {
    if (n <= 1) return;
    ps_sort_lds<NT, BIG>(E, n, 2 * (31 - __builtin_clz((unsigned)n)), sc, nmax);
}

// The sort of gE[0, n) in global memory (n <= NT * PS_MAX_CHUNK): the workgroup splits it until every
// segment fits EL (cap elements of LDS), then each segment is copied into EL, sorted there from its
// remaining depth and copied back. sc: ps_scratch_ints_global(NT, cap) ints of LDS. Ends with a barrier.
template <int NT>
__device__ void pcl_std_sort_global(unsigned long long* gE, const int n, unsigned long long* EL, const int cap, int* sc) {
    const int tid = threadIdx.x;
    if (n <= 1) return;
    int* hdr = sc;
    int* GL = sc + ps_scratch_ints(NT, cap, true);
    if (tid < 16) hdr[tid] = 0;
    for (int i = tid; i < 3 * PS_GLIST; i += NT) GL[i] = 0;
    int* Bf = sc + 16 + 2 * (NT / WAVE) + 7 * (NT + 1);
    const int D0 = 2 * (31 - __builtin_clz((unsigned)n));
    __syncthreads();
    if (tid == 0) {
        if (n > cap) { Bf[0] = 0; Bf[PS_WGSEG] = n; Bf[2 * PS_WGSEG] = D0; hdr[0] = 1; }
        else { GL[0] = 0; GL[1] = n; GL[2] = D0 + 1; hdr[4] = 1; }     // fits: one staged segment
    }
    __syncthreads();
    if (n > cap) ps_wg_split<NT, true>(gE, n, sc, cap, &hdr[4], &hdr[5], GL, PS_GLIST);
    __syncthreads();
    const int ns = min(ps_u(hdr[4]), PS_GLIST);
    for (int i = 0; i < ns; i++) {
        const int f = GL[3 * i], l = GL[3 * i + 1], d = GL[3 * i + 2] - 1;
        const int m = l - f;
        for (int t = tid; t < m; t += NT) EL[t] = gE[f + t];
        __syncthreads();
        ps_sort_lds<NT, true>(EL, m, d, sc, cap);
        for (int t = tid; t < m; t += NT) gE[f + t] = EL[t];
        __syncthreads();
    }
}

#ifndef PS_HOST_EMU
// CentroidPoint sum of the run of key k that starts at E[p]: x, y, z, intensity added in fp32 from zero
// in sorted order; the keys and points are loaded 8 ahead (the adds stay sequential). pt(i): point i.
template <typename PtF>
__device__ __forceinline__ float4 ps_run_sum(const unsigned long long* E, const int n, const int p, const unsigned k, PtF pt,
                                             int& cnt) {
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    cnt = 0;
    for (int t0 = p;; t0 += 8) {
        unsigned long long e[8];
        bool in[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            e[i] = t0 + i < n ? E[t0 + i] : 0ull;
            in[i] = t0 + i < n && ps_key(e[i]) == k;
        }
        float4 q[8];
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (in[i]) {
                PS_CHECK((int)(e[i] & 0xffffffffu) < n, "run payload %d n %d\n", (int)(e[i] & 0xffffffffu), n);
                q[i] = pt((int)(e[i] & 0xffffffffu));
            }
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (in[i]) { c.x += q[i].x; c.y += q[i].y; c.z += q[i].z; c.w += q[i].w; cnt++; }
        if (!in[7]) break;
    }
    return c;
}
#endif

}  // namespace aloam
