// pcl_sort.hpp — PCL VoxelGrid's point order on gfx950: libstdc++ std::sort building blocks.
//
// pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.8.0, voxel_grid.hpp) pushes one (leaf index, point
// index) pair per point, std::sort's them by leaf index (an UNSTABLE introsort: the pairs of one leaf
// end up in an order that depends on the whole array) and sums every leaf's points in that order. The
// reference calls it at src/scanRegistration.cpp:401-405 (per scan line, leaf 0.2) and
// src/laserMapping.cpp:542-550 (the stacks), :788-801 (every surrounding map cube). fp32 sums depend on
// the order, so the device reproduces it exactly (ls_sort.hpp). libstdc++'s sort is introsort_loop
// (median of first+1 / mid / last-1 moved to first, unguarded Hoare partition, recurse right, loop left,
// 16-element threshold, heap sort at depth 2 floor(log2 n)) followed by one insertion sort over the whole
// array. This file holds the pieces shared by ls_sort.hpp: keys (u64 = key << 32 | payload, compared by
// key only), the median move, heap sort, insertion sort, the one-thread whole sort (arrays beyond the
// parallel paths), block scans, the leaf sums, and the workgroup split of an array in global memory
// (ps_wg_split: segments above a limit partitioned level by level by the whole workgroup, each thread a
// chunk of <= 64 positions; children at or below the limit pushed to a sink list).
//
// The partition of a segment [f, l) with pivot key K at f is computed, not simulated: with LS = the
// positions p in (f, l) with key >= K in ascending order ("left stops") and RS = the positions in
// [f, l) with key <= K in descending order ("right stops"), Hoare's two scans swap LS[j] <-> RS[j] for
// exactly the j < k with LS[j] < RS[j] (both sequences are monotone, so that is a prefix; LS[j] < RS[j]
// iff more than j right stops lie after LS[j]) and return cut = min(LS[k], RS[k-1]) (LS[k] when k = 0,
// RS[k-1] when LS runs out): every element a scan passes before a swap is untouched, and the first
// swapped element a scan meets stops it. The final insertion sort is stable and the partition property
// keeps every element inside its <= 16-element leaf, so each leaf is sorted (stable rank) once it forms.
// Depth-exhausted segments are heap-sorted by one lane, exactly as std::__partial_sort(first, last, last).
//
// The characterisation is checked against libstdc++ on the host (oracle/aloam_oracle.cpp
// oracle_pcl_replay_check, tests/test_oracle_pins.py), the device code on the host by a per-lane thread
// emulation (tests/ps_emu.cpp, tests/test_pcl_sort_emu.py) and on the device by the VoxelGrid /
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
constexpr int PS_MAX_CHUNK = 64;    // workgroup phase: positions per thread (u64 stop masks)
constexpr int PS_WGSEG = 32;        // workgroup phase: segments split at once (n <= NT * 64)
constexpr int PS_GLIST = 320;       // global sorts: segments staged through LDS (<= 2 per split x depth)

// Scratch (ints, LDS, 8-byte aligned): header | exscan words | workgroup phase arrays (BIG) | segment
// queue (3 ints per queued segment) [| staged-segment list (global sorts)]
__host__ __device__ constexpr int ps_wg_ints(int NT) { return 7 * (NT + 1) + 8 * PS_WGSEG; }
__host__ __device__ constexpr int ps_qcap(int n) { return n / (PS_THRESHOLD + 1) + 64; }
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
#ifdef PS_EXP_NOHEAP                         // timing experiment only (results invalid): skip every heap sort
    return;
#endif
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
// Where PCL's order matters (relevance gating). A leaf's CentroidPoint sum starts at zero, so its first two
// terms commute, ((0 + a) + b) == ((0 + b) + a) bit for bit: the order std::sort leaves equal keys in only
// changes a centroid for leaves of >= 3 points. rel (may be null: everything matters) marks the points of
// such leaves, bit i for the point of payload index i (payload bits 0-15). A depth-exhausted introsort
// segment that holds fewer than two of them is left unsorted instead of heap-sorted: the caller's leaf
// sums take their order from an order-free sort of the keys, and each relevant point keeps the position
// range of its segment, which is all its leaf's order needs from it (segments are ordered by key).
__device__ inline bool ps_order_matters(const unsigned long long* E, int f, int l, const unsigned* rel) {
    if (!rel) return true;
    int c = 0;
    for (int p = f; p < l; p++) {
        const unsigned i = (unsigned)E[p] & 0xffffu;
        c += (int)((rel[i >> 5] >> (i & 31u)) & 1u);
        if (c >= 2) return true;
    }
    return false;
}
__device__ inline void ps_heap_sort_rel(unsigned long long* E, int f, int l, const unsigned* rel) {
    if (ps_order_matters(E, f, l, rel)) ps_heap_sort(E + f, E + l);
}

// ---- the heap sort by a whole wave ----------------------------------------------------------------
// One pop of libstdc++'s __adjust_heap(first, 0, hl, v) (after *last = *first) is, top-down: from the root
// hole, the larger child (the right one on a tie) moves up while its key is >= v's, then v fills the hole
// -- Floyd's descend-to-the-leaf-then-push-up gives the same array, as along the max-child path the keys
// do not increase. The wave resolves six levels per LDS round trip: lane r (< 63) loads the two children
// of the hole's subtree node r (relative heap numbering, depths 0-5) and votes (child chosen, moves up),
// the path is walked on the two ballots in scalar registers, and the path's lanes shift their winners up
// with one store.
// The hole's path through one six-level subtree from the two ballots (bit r: subtree node r's larger child
// moves up / is the right one), without a data-dependent loop: the six candidate nodes follow the `right`
// bits alone, the path length is the run of leading `go` bits along them. Returns the node where the path
// stops (< 63: the value goes there; 63..126 after six steps), the path's nodes in *pm, its length in *steps.
__device__ __forceinline__ int ws_path(const unsigned long long mgo, const unsigned long long mr, unsigned long long* pm, int* steps) {
    int rk[7];
    rk[0] = 0;
    unsigned gom = 0u;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        gom |= (unsigned)((mgo >> rk[k]) & 1ull) << k;
        rk[k + 1] = 2 * rk[k] + 1 + (int)((mr >> rk[k]) & 1ull);
    }
    const int st = __builtin_ctz(~gom);           // <= 6: gom < 64
    unsigned long long m = 0ull;
    int r = rk[0];
#pragma unroll
    for (int k = 0; k < 6; k++) {
        if (k < st) m |= 1ull << rk[k];
        if (k + 1 == st) r = rk[k + 1];
    }
    *pm = m;
    *steps = st;
    return r;
}
__device__ inline void ws_sift(unsigned long long* H, const int hl, const unsigned long long v) {
    const int lane = lane_id();
    const int dr = 31 - __builtin_clz((unsigned)(lane + 1));   // depth of subtree node `lane` (lane 63: unused)
    const int o = lane + 1 - (1 << dr);
    const unsigned vk = ps_key(v);
    int h = 0;
    for (;;) {
        int a = 0;
        bool go = false, right = false;
        unsigned long long w = 0ull;
        if (lane < 63) {
            a = ((h + 1) << dr) - 1 + o;
            const int c1 = 2 * a + 1;
            if (c1 < hl) {
                const unsigned long long e1 = H[c1];
                unsigned long long e2 = 0ull;
                if (c1 + 1 < hl) { e2 = H[c1 + 1]; right = !(ps_key(e2) < ps_key(e1)); }
                w = right ? e2 : e1;
                go = ps_key(w) >= vk;
            }
        }
        const unsigned long long mgo = __ballot(go), mr = __ballot(right);
        unsigned long long pm;
        int steps;
        const int r = ws_path(mgo, mr, &pm, &steps);
        if ((pm >> lane) & 1ull) H[a] = w;
        if (steps < 6) {                        // v fills the hole at subtree node r
            const int ar = readlane_i(a, r);
            if (lane == 0) H[ar] = v;
            ps_wsync<true>();
            return;
        }
        ps_wsync<true>();
        h = ((h + 1) << 6) - 1 + (r - 63);      // the hole went six levels down
    }
}
// The pops of __sort_heap on a heap in LDS. A wave's LDS operations complete in issue order, so no pop waits
// for its stores: the next pop's loads see them. Per pop: the root is carried in registers (the previous
// pop's new root), the re-inserted value H[hl] rides on lane 63 of the first six-level load, the popped
// root goes straight to its final slot, then ws_sift's six-level steps without the store waits. The
// result is std::__sort_heap's array (first npop pops).
__device__ inline bool ps_in_lds(const void* p) {
#if defined(PS_HOST_EMU)
    (void)p;
    return true;
#elif defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)p);
#else
    (void)p;
    return false;
#endif
}
__device__ inline void ws_sort_heap_lds(unsigned long long* H, const int len, const int npop) {
    const int lane = lane_id();
    const int dr = 31 - __builtin_clz((unsigned)(lane + 1));   // depth of subtree node `lane` (lane 63: the value)
    const int o = lane + 1 - (1 << dr);
    unsigned long long top = H[0];
    for (int i = 0; i < npop; i++) {
        const int hl = len - 1 - i;
        unsigned long long v = 0ull;
        unsigned vk = 0u;
        int h = 0;
        for (bool first = true;; first = false) {
            int a = 0;
            bool has = false, right = false;
            unsigned long long e1 = 0ull, e2 = 0ull, vv = 0ull;
            if (lane < 63) {
                a = ((h + 1) << dr) - 1 + o;
                const int c1 = 2 * a + 1;
                if (c1 < hl) {
                    has = true;
                    e1 = H[c1];
                    if (c1 + 1 < hl) { e2 = H[c1 + 1]; right = !(ps_key(e2) < ps_key(e1)); }
                }
            } else if (first) {
                vv = H[hl];
            }
            if (first) {
                v = ps_rl64(vv, 63);
                vk = ps_key(v);
                if (lane == 0) H[hl] = top;                 // after the load of H[hl] (issue order)
            }
            const unsigned long long w = right ? e2 : e1;
            const bool go = has && ps_key(w) >= vk;
            const unsigned long long mgo = __ballot(go), mr = __ballot(right);
            unsigned long long pm;
            int steps;
            const int r = ws_path(mgo, mr, &pm, &steps);
            if ((pm >> lane) & 1ull) H[a] = w;
            if (first) top = (mgo & 1ull) ? ps_rl64(w, 0) : v;   // the new root
            if (steps < 6) {                                 // v fills the hole at subtree node r
                const int ar = readlane_i(a, r);
                if (lane == 0) H[ar] = v;
                break;
            }
            h = ((h + 1) << 6) - 1 + (r - 63);               // the hole went six levels down
        }
        ps_wsync<false>();
    }
}
// ---- the pops with child flags (FH: len <= FH_MAX, heap and flags in LDS) -------------------------------
// A pop of __sort_heap moves the hole from the root along the larger-child path (the right child on a tie)
// to a leaf, then pushes the re-inserted value v = H[hl] up while its parent's key is < v's (pcl_sort.hpp
// ps_adjust_heap). The path depends only on which child of each path node is the larger one, so that bit
// is kept per node (1-based node m, children 2m and 2m + 1): F[m - 1] = !(key(right) < key(left)). A pop:
//   1. the top six levels: lane j (1..63) loads node j's bit (0 unless both children are in the heap), a
//      ballot gives the 63 bits, and the walk m <- 2m + bit(m) runs six steps (no branch: steps past the
//      heap are cut off afterwards); 2. the next five levels the same way from the level-6 node's
//      subtree; 3. the path's length L = the depths whose node lies in the heap (one ballot); lane t holds
//      path node p_t and loads x_t = H[p_t] and its sibling, every lane loads v; 4. v lands at p_J,
//      J = #{t >= 1: !(key(x_t) < key(v))} (path keys do not increase: a prefix), p_{t-1} <- x_t for t <= J,
//      the popped root goes to H[hl]; the only bits that change are those of p_0..p_{J-1} (their path
//      child got a new value): lane t recomputes p_{t-1}'s bit from p_t's new value and its sibling.
// Three LDS round trips per pop, everything else straight-line vector code: on one wave a taken branch
// costs ~32 cycles, a dependent scalar op ~8, a readlane -> scalar -> readlane link ~41 and a dependent
// vector op ~5 (micro/heap_bench.py), so the walks run on vector registers (fh_v launders the ballots
// there) and nothing branches inside a pop. Same array as std::__sort_heap (first npop pops). Bits of
// nodes whose right child left the heap are stale but never read (the heap-size test masks them).
constexpr int FH_MAX = 4095;            // depth <= 11: a six-level and a five-level walk; flag scratch: len bytes
#if defined(PS_HOST_EMU)
__device__ __forceinline__ unsigned fh_v(unsigned x) { return x; }
#else
// the value in a vector register (the compiler then keeps what is computed from it on the vector unit)
__device__ __forceinline__ unsigned fh_v(unsigned x) { unsigned r; asm("v_mov_b32 %0, %1" : "=v"(r) : "v"(x)); return r; }
#endif
// bit (k & 31) of x (v_bfe_u32: one instruction, the offset taken mod 32 like the hardware's)
#if defined(PS_HOST_EMU)
__device__ __forceinline__ unsigned fh_bit(unsigned x, unsigned k) { return (x >> (k & 31u)) & 1u; }
#else
__device__ __forceinline__ unsigned fh_bit(unsigned x, unsigned k) { return __builtin_amdgcn_ubfe(x, k, 1u); }
#endif
__device__ __forceinline__ unsigned long long fh_shl1(unsigned long long x) {   // lane l <- lane l + 1 (row of 16)
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)x, 0x101, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(x >> 32), 0x101, 0xF, 0xF, false);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PS_HOST_EMU)
#define PS_LDSP(T) __attribute__((address_space(3))) T*      // LDS pointer: ds_* instructions, not flat ones
#else
#define PS_LDSP(T) T*
#endif
template <bool DEEP>
__device__ __forceinline__ void fh_pops(PS_LDSP(unsigned long long) H, PS_LDSP(unsigned char) F, const int len, const int npop) {
    const int lane = lane_id();
    const unsigned dj = lane ? 31u - (unsigned)__builtin_clz((unsigned)lane) : 0u;   // lane j: subtree node j (1-based)
    const unsigned oj = (unsigned)lane - (1u << dj);
    for (int i = 0; i < npop; i++) {
        const int hl = len - 1 - i;                 // the descent's heap: 1-based nodes 1..hl; v = H[hl]
        // 1. top six levels
        const int jt = lane ? lane : 1;
        const unsigned char ft = F[min(jt, len) - 1];
        const unsigned long long Cb = __ballot(lane >= 1 && 2 * lane + 1 <= hl && ft);
        const unsigned Ctl = fh_v((unsigned)Cb), Cth = fh_v((unsigned)(Cb >> 32));
        unsigned m = fh_v(1u);
#pragma unroll
        for (int k = 0; k < 5; k++) m = (m << 1) | fh_bit(Ctl, m);   // nodes < 32: the low word (one bfe per step)
        m = (m << 1) | fh_bit(Cth, m);                                   // m in [32, 63]: bit m - 32 = m & 31 -> [64, 127]
        // 2. five more levels below the level-6 node m
        unsigned md = 32u;
        if (DEEP) {
            const unsigned nd = (m << dj) | oj;         // lane j: node j of m's subtree
            const unsigned char fd = F[min((int)nd, len) - 1];
            const unsigned Cd = fh_v((unsigned)__ballot(lane >= 1 && lane < 32 && (int)(2 * nd + 1) <= hl && fd));
            md = fh_v(1u);
#pragma unroll
            for (int k = 0; k < 5; k++) md = (md << 1) | fh_bit(Cd, md);   // md in [32, 63]
        }
        const unsigned me = (m << 5) | (md & 31u);    // the walk's node at depth 11
        // 3. path length and path nodes
        const int L = __popcll(__ballot(lane <= 11 && (int)(me >> (11 - min(lane, 11))) <= hl)) - 1;
        const unsigned p = lane <= 11 ? me >> (11 - lane) : 1u;    // lane t <= L: path node p_t
        const unsigned sb = p ^ 1u;                                  // its sibling (t >= 1)
        const unsigned long long x = H[min((int)p, hl + 1) - 1];
        const unsigned long long sv = H[max(min((int)sb, hl + 1), 1) - 1];
        const unsigned long long v = H[hl], root = H[0];            // (every lane: broadcast reads)
        const unsigned vk = ps_key(v);
        // 4. v's slot, the moves, the bits
        const int J = __popcll(__ballot(lane >= 1 && lane <= L && !(ps_key(x) < vk)));
        const unsigned long long xs = fh_shl1(x);                   // x_{t+1} in lane t (every lane: a collective)
        const unsigned long long nv = lane < J ? xs : v;            // p_t's new value (t <= J)
        const unsigned sk = ps_key(sv), nk = ps_key(nv);
        const unsigned char nf = (p & 1u) ? !(nk < sk) : !(sk < nk);   // p_{t-1}'s bit (p_t odd: the right child)
        // every lane stores (no exec-mask branches): lanes t <= J their path node, the others the popped
        // root into H[hl] (all the same value) and their bit into node hl + 1's byte, which no later pop
        // reads (the heap only shrinks)
        const bool wf = lane >= 1 && lane <= J && (int)sb <= hl;
        F[wf ? (int)(p >> 1) - 1 : hl] = nf;
        *(lane <= J ? H + (p - 1) : H + hl) = lane <= J ? nv : root;
        ps_wsync<false>();
    }
}
__device__ inline void fh_sort_heap_lds(unsigned long long* Hg, unsigned char* Fg, const int len_, const int npop_) {
    PS_LDSP(unsigned long long) H = (PS_LDSP(unsigned long long))Hg;
    PS_LDSP(unsigned char) F = (PS_LDSP(unsigned char))Fg;
    const int len = ps_u(len_), npop = ps_u(npop_);
    // the bits of every node with two children (1-based m: children 2m, 2m + 1 = 0-based 2m - 1, 2m)
    for (int m = lane_id() + 1; 2 * m + 1 <= len; m += WAVE) F[m - 1] = !(ps_key(H[2 * m]) < ps_key(H[2 * m - 1]));
    ps_wsync<false>();
    if (len > 127) fh_pops<true>(H, F, len, npop);
    else fh_pops<false>(H, F, len, npop);
}

// std::__partial_sort(E + f, E + l, E + l) (= __make_heap + __sort_heap) by one wave, E in LDS or global.
// __make_heap adjusts the parents (len - 2) / 2 .. 0 in turn; parents of one depth have disjoint subtrees,
// so each depth runs on the lanes at once, deepest first. With rel (rvg.hpp), only the order of the
// relevant points is needed: the pops stop once every element with a key >= the smallest relevant key has
// been popped into its final slot (pops go in decreasing key order); the rest stays in heap order.
// Nodes of the subtree of `node` in a heap of len slots, and a node's index in the heap's post-order
// (left subtree, right subtree, node).
__device__ inline int heap_subtree_size(int node, const int len) {
    int tot = 0;
    for (int k = 0;; k++) {
        const long long lo = ((long long)(node + 1) << k) - 1;
        if (lo >= len) break;
        tot += (int)(min((long long)len, lo + (1ll << k)) - lo);
    }
    return tot;
}
__device__ inline int heap_postorder(const int i, const int len) {
    const int di = 31 - __builtin_clz((unsigned)(i + 1));
    int a = 0, start = 0;
    for (int da = 0; da < di; da++) {
        const int anc = ((i + 1) >> (di - da - 1)) - 1;     // i's ancestor one level below a
        if (anc != 2 * a + 1) start += heap_subtree_size(2 * a + 1, len);
        a = anc;
    }
    return start + heap_subtree_size(i, len) - 1;
}
// __sort_heap without the pops, where that is provably the same for the relevant points (rvg.hpp): after
// __make_heap, the pops take the root, the larger child (the right one on a tie) moving up, so points of
// one key leave the heap in (node, right subtree, left subtree) pre-order of their slots -- the moves keep
// that order among equal keys -- and land in the reverse, the post-order (left, right, node). Only one
// thing breaks it: a point of the key taken as a pop's re-inserted value (the heap's last slot), which
// needs it to sit among the last c slots (c = points with keys >= its key: the pops until the key is out)
// and to stay there; a point taken this way with a larger key only moves larger points, whose order
// among themselves is not read. So when no relevant point sits in its danger zone, the segment is
// written in post-order of the heap slots (each relevant leaf's points then in PCL's order, the other
// points anywhere inside the segment, which rvg.hpp allows) and the pops are skipped. len <= 16 * 64.
// Checked against libstdc++'s heap sort by micro/cube_stats.cpp (POSTORDER "safe": every safe group
// right) and the host emulator. Returns false (nothing written) when some relevant point is in danger.
__device__ inline bool ws_heap_postorder(unsigned long long* H, const int len, const int npop, const unsigned* rel) {
    const int lane = lane_id();
    // candidates: relevant points in the last npop slots (npop = points >= the smallest relevant key)
    bool danger = false;
    for (int s0 = len - npop; s0 < len; s0 += WAVE) {
        const int sl = s0 + lane;
        unsigned long long e = 0ull;
        bool cand = false;
        if (sl < len) {
            e = H[sl];
            const unsigned i = (unsigned)e & 0xffffu;
            cand = (rel[i >> 5] >> (i & 31u)) & 1u;
        }
        unsigned long long cm = __ballot(cand);
        while (cm) {                                  // exact zone of each candidate: count_ge(key) >= len - slot
            const int b = __builtin_ctzll(cm);
            cm &= cm - 1ull;
            const unsigned kx = (unsigned)readlane_i((int)ps_key(e), b);
            const int sx = s0 + b;
            int c = 0;
            for (int p = lane; p < len; p += WAVE) c += ps_key(H[p]) >= kx;
            c = wave_sum_i(c);
            if (c >= len - sx) { danger = true; break; }
        }
        if (danger) break;
    }
    if (danger) return false;
#ifdef PS_POSTORDER_COUNT                           // host-emulator coverage counter (tests/ps_emu.cpp)
    if (lane == 0) PS_POSTORDER_COUNT++;
#endif
    unsigned long long ev[16];
    int dst[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int i = lane + WAVE * j;
        dst[j] = -1;
        if (i < len) { ev[j] = H[i]; dst[j] = heap_postorder(i, len); }
    }
    ps_wsync<true>();
#pragma unroll
    for (int j = 0; j < 16; j++)
        if (dst[j] >= 0) H[dst[j]] = ev[j];
    ps_wsync<true>();
    return true;
}

__device__ __noinline__ void ws_heap_sort(unsigned long long* E, const int f, const int l, const unsigned* rel,
                                          unsigned char* fscr = nullptr) {
    const int len = ps_u(l - f);          // scalar (arguments arrive in VGPRs): uniform loops, no exec masks
    if (len < 2) return;
    unsigned long long* H = E + ps_u(f);
    const int lane = lane_id();
    int npop = len - 1;
    if (rel) {
        unsigned km = 0xffffffffu;
        for (int p = lane; p < len; p += WAVE) {
            const unsigned long long e = H[p];
            const unsigned i = (unsigned)e & 0xffffu;
            if ((rel[i >> 5] >> (i & 31u)) & 1u) km = min(km, ps_key(e));
        }
        km = allreduce_u32<6>(km, [](unsigned x, unsigned y) { return x < y ? x : y; });
        int c = 0;
        for (int p = lane; p < len; p += WAVE) c += ps_key(H[p]) >= km;
        c = wave_sum_i(c);
        npop = ps_u(min(len - 1, c));
    }
    const bool lds = ps_in_lds(H);
    const int P = (len - 2) / 2;
    const int D = 31 - __builtin_clz((unsigned)(P + 1));
    for (int d = D; d >= 0; d--) {
        const int a0 = (1 << d) - 1, a1 = min((2 << d) - 2, P);
        for (int base = a0; base <= a1; base += WAVE) {
            const int node = base + lane;
            if (node <= a1) ps_adjust_heap(H, node, len, H[node]);
        }
        if (lds) ps_wsync<false>(); else ps_wsync<true>();
    }
#ifndef PS_NO_POSTORDER                      // A/B parity builds: the pops everywhere
    if (rel && len <= 16 * WAVE && ws_heap_postorder(H, len, npop, rel)) return;
#endif
#ifdef PS_NO_FH                              // A/B builds: the six-level pops everywhere
    fscr = nullptr;
#endif
    if (lds) {
        if (fscr && len <= FH_MAX) fh_sort_heap_lds(H, fscr, len, npop);   // fscr: len bytes of LDS
        else ws_sort_heap_lds(H, len, npop);
        return;
    }
    for (int i = 0; i < npop; i++) {
        const int hl = len - 1 - i;
        const unsigned long long v = H[hl], top = H[0];
        ps_wsync<true>();
        if (lane == 0) H[hl] = top;
        ps_wsync<true>();
        ws_sift(H, hl, v);
    }
}
// ps_order_matters by a wave (all lanes get the answer)
__device__ inline bool ws_order_matters(const unsigned long long* E, int f, int l, const unsigned* rel) {
    if (!rel) return true;
    int c = 0;
    for (int p = f + lane_id(); p < l; p += WAVE) {
        const unsigned i = (unsigned)E[p] & 0xffffu;
        c += (int)((rel[i >> 5] >> (i & 31u)) & 1u);
    }
    return wave_sum_i(c) >= 2;
}

// The whole std::sort by one thread (arrays beyond NT * PS_MAX_CHUNK elements): introsort_loop with an
// explicit stack (the right part is pushed, the left continued — disjoint ranges, same result), then
// __final_insertion_sort.
// Every call is counted (this translation unit's copy of the counter; aloam_serial_sort_fallbacks sums
// them): the one-thread sort is exact but slow, and a workload that reaches it should show.
#ifndef PS_HOST_EMU
static __device__ unsigned long long g_ps_serial_calls;
#endif
__device__ __noinline__ void ps_serial_std_sort(unsigned long long* E, int n) {
#ifndef PS_HOST_EMU
    atomicAdd(&g_ps_serial_calls, 1ull);
#endif
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
// (the four elements loaded together: one round trip on global memory)
__device__ __forceinline__ unsigned ps_median_to_first(unsigned long long* E, int f, int l) {
    const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const unsigned long long ef = E[f], ea = E[a], eb = E[b], ec = E[c];
    const unsigned ka = ps_key(ea), kb = ps_key(eb), kc = ps_key(ec);
    int pick;
    if (ka < kb) pick = kb < kc ? b : (ka < kc ? c : a);
    else pick = ka < kc ? a : (kb < kc ? c : b);
    const unsigned long long ep = pick == a ? ea : (pick == b ? eb : ec);
    E[f] = ep;
    E[pick] = ef;
    return ps_key(ep);
}

// Work queue of segments (f, l, depth + 1 as the ready mark). hdr: [1] head, [2] tail, [3] pending
// (queued or in progress). ps_push: ONE lane (the workgroup phase's thread 0); ps_push_wave: a whole
// wave, uniform arguments. False when the queue is full (the slot claimed past qcap is never filled: a
// wave waiting on it leaves when pending reaches zero).
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

// A[s] += c summed over the wave's lanes with the same s (s < 0 or c == 0: nothing); every lane calls it
__device__ __forceinline__ void ps_wave_add(int* A, int s, int c) {
    bool pend = s >= 0 && c != 0;
    for (;;) {
        const unsigned long long m = __ballot(pend);
        if (!m) break;
        const int lead = __builtin_ctzll(m);
        const int sl = readlane_i(s, lead);
        const bool mine = pend && s == sl;
        const int sum = wave_sum_i(mine ? c : 0);
        if (lane_id() == lead) atomicAdd(&A[sl], sum);
        pend = pend && !mine;
    }
}

// Split every segment listed in U's big list (Bf/Bl/Bd, sorted by f, hdr[0] entries) that is longer
// than `limit`, level by level, over positions [0, n): children > limit stay listed, the others are
// pushed to the sink queue (tail/pend/Qs/qcap; segments of <= 16 too: the wave phase sorts leaves).
// Elements stay in E (LDS, or global with G). limit >= 64: a 64-position word of the stop flags meets at most
// two listed segments. Per level (round 5, micro/split_bench.py): the flags by coalesced wave passes, the
// swaps by groups of 64 consecutive pairs per wave (both were per-thread chunks: one cache line per lane and
// load, bound by the CU's line rate on global memory), k summed per wave.
template <int NT, bool G>
__device__ void ps_wg_split(unsigned long long* E, const int n, int* sc, const int limit, int* tail, int* pend, int* Qs,
                            const int qcap, const unsigned* rel = nullptr) {
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
    constexpr int NW = NT / WAVE;
    const int lane = lane_id();
    for (int lvl = 0;; lvl++) {
        (void)lvl;
        const int nbig = ps_u(hdr[0]);
        PS_TS(lvl, 0);
        if (nbig == 0) break;
        // depth-exhausted segments: heap sort (rare), emptied from the list below
        for (int s = tid; s < nbig; s += NT)
            if (Bd[s] == 0) ps_heap_sort_rel(E, Bf[s], Bl[s], rel);
        if (tid < nbig && Bd[tid] > 0) { Bk[tid] = ps_median_to_first(E, Bf[tid], Bl[tid]); Bkk[tid] = 0; }
        ps_bar<G>();
        // A: the stop flags by ballot, 64 consecutive positions per wave pass (coalesced key loads, 4 passes in
        // flight); the 64-position words go to maskL / maskR and are read back below into each thread's
        // C-position masks (thread t: positions [t C, t C + C)) before those overwrite them
        const int nch64 = (n + 63) >> 6;
        for (int c0 = ps_u(tid / WAVE); c0 < nch64; c0 += 4 * NW) {
            unsigned kk[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int p = (c0 + u * NW) * 64 + lane;
                kk[u] = p < n ? ps_keyat(E, p) : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int c = c0 + u * NW;
                if (c >= nch64) break;
                const int p = c * 64 + lane;
                int lo = 0, hi = nbig;                   // the last segment with f <= 64 c, then this lane's
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (Bf[mid] <= c * 64) lo = mid + 1;
                    else hi = mid;
                }
                int s = lo - 1;
                if (s + 1 < nbig && Bf[s + 1] <= p) s++;
                bool isL = false, isR = false;
                if (s >= 0 && p < n) {
                    const int cf = Bf[s], ce = Bd[s] > 0 ? Bl[s] : cf;
                    const unsigned ck = Bk[s];
                    if (p >= cf && p < ce) { isL = p > cf && kk[u] >= ck; isR = kk[u] <= ck; }
                }
                const unsigned long long bl = __ballot(isL), br = __ballot(isR);
                if (lane == 0) { maskL[c] = bl; maskR[c] = br; }
            }
        }
        lds_barrier();
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
            s0 = lo - 1;
            const int w0 = p0 >> 6, o = p0 & 63, len = p1 - p0;
            unsigned long long wl = maskL[w0] >> o, wr = maskR[w0] >> o;
            if (o && w0 + 1 < nch64) { wl |= maskL[w0 + 1] << (64 - o); wr |= maskR[w0 + 1] << (64 - o); }
            const unsigned long long keep = len >= 64 ? ~0ull : (1ull << len) - 1ull;
            mL = wl & keep;
            mR = wr & keep;
            cl = __popcll(mL);
            cr = __popcll(mR);
        }
        int tl, tr;
        ps_exscan2<NT>(cl, cr, ws, tl, tr);              // (its barrier orders the reads above before the writes)
        if (tid < nch) { prefL[tid] = cl; prefR[tid] = cr; maskL[tid] = mL; maskR[tid] = mR; sidx[tid] = s0; }
        if (tid == 0) { prefL[nch] = tl; prefR[nch] = tr; maskL[nch] = 0ull; maskR[nch] = 0ull; }
        lds_barrier();
        PS_TS(lvl, 1);
        // k per segment: left stops with more right stops after them than left stops before them (this
        // thread's stops in registers; the segment's bounds once per segment); a chunk meets at most two
        // segments (listed segments are longer than `limit` >= 64), summed per wave before the LDS atomic
        {
            int sA = -1, cA = 0, sB = -1, cB = 0;
            if (tid < nch && mL) {
                int s = s0, cur = -1, bL = 0, eR = 0, cnt = 0, j = 0;
                for (unsigned long long m = mL; m; m &= m - 1ull) {
                    const int b = __builtin_ctzll(m), p = p0 + b;
                    while (s + 1 < nbig && Bf[s + 1] <= p) s++;
                    if (s != cur) {
                        if (cur >= 0 && cnt) {
                            if (sA < 0) { sA = cur; cA = cnt; }
                            else if (sB < 0) { sB = cur; cB = cnt; }
                            else atomicAdd(&Bkk[cur], cnt);
                        }
                        cur = s; cnt = 0;
                        bL = ps_count_before(prefL, maskL, Bf[s], C);
                        eR = ps_count_before(prefR, maskR, Bl[s], C);
                    }
                    j = cl + __popcll(mL & ((1ull << b) - 1ull)) - bL;
                    const int after = eR - (cr + __popcll(mR & ((2ull << b) - 1ull)));
                    cnt += j < after;
                }
                if (cur >= 0 && cnt) {
                    if (sA < 0) { sA = cur; cA = cnt; }
                    else if (sB < 0) { sB = cur; cB = cnt; }
                    else atomicAdd(&Bkk[cur], cnt);
                }
            }
            ps_wave_add(Bkk, sA, cA);
            ps_wave_add(Bkk, sB, cB);
        }
        lds_barrier();
        PS_TS(lvl, 2);
        // the swaps: segment s's pairs (left stop j, right stop j from the right), j < k_s, in groups of 64
        // consecutive j per wave pass (lane = j: neighbouring lanes touch neighbouring stops, so the loads
        // and stores coalesce), 4 groups in flight; a lane finds its pair by two rank selects in the masks
        {
            const int ks = lane < nbig && Bd[lane] > 0 ? Bkk[lane] : 0;
            const int gs = (ks + 63) >> 6;
            const int gincl = wave_incl_scan(gs);
            const int gtot = ps_u(readlane_i(gincl, WAVE - 1));
            for (int g0 = ps_u(tid / WAVE); g0 < gtot; g0 += 4 * NW) {
                int pp[4], qq[4];
                bool v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int g = g0 + u * NW;
                    v[u] = false;
                    pp[u] = qq[u] = 0;
                    if (g < gtot) {
                        const int sg = ps_u(__popcll(__ballot(lane < nbig && gincl <= g)));
                        const int gb = ps_u(readlane_i(gincl - gs, sg)), kseg = ps_u(readlane_i(ks, sg));
                        const int f = ps_u(Bf[sg]), l = ps_u(Bl[sg]);
                        const int j = (g - gb) * 64 + lane;
                        if (j < kseg) {
                            const int bL = ps_count_before(prefL, maskL, f, C), eR = ps_count_before(prefR, maskR, l, C);
                            pp[u] = ps_select(prefL, maskL, bL + j, f / C, (l - 1) / C, C);
                            qq[u] = ps_select(prefR, maskR, eR - 1 - j, f / C, (l - 1) / C, C);
                            v[u] = true;
                            PS_CHECK(pp[u] > f && pp[u] < l && qq[u] > pp[u] && qq[u] < l, "ps wg swap: f %d l %d p %d q %d\n", f, l,
                                     pp[u], qq[u]);
                        }
                    }
                }
                unsigned long long ep[4], eq[4];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (v[u]) { ep[u] = E[pp[u]]; eq[u] = E[qq[u]]; }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (v[u]) { E[pp[u]] = eq[u]; E[qq[u]] = ep[u]; }
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
