// pcl_sort.hpp — PCL VoxelGrid's point order on gfx950: libstdc++ std::sort, replayed in parallel.
//
// pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.8.0, voxel_grid.hpp) pushes one (leaf index, point
// index) pair per point, std::sort's them by leaf index (an UNSTABLE introsort: the pairs of one leaf
// end up in an order that depends on the whole array) and sums every leaf's points in that order. The
// reference calls it at src/scanRegistration.cpp:401-405 (per scan line, leaf 0.2) and
// src/laserMapping.cpp:542-550 (the stacks), :788-801 (every surrounding map cube). fp32 sums depend on
// the order, so the device reproduces it exactly:
//
//   pcl_std_sort<NT, G>(E, n, Lpos, Rpos, scratch, seg, segcap)
//
// leaves E[0, n) (u64 = key << 32 | payload, compared by key only) in exactly the order
// std::sort(E, E + n, key-less) of libstdc++ produces. libstdc++'s sort is introsort_loop (median of
// first+1 / mid / last-1 moved to first, unguarded Hoare partition, recurse right, loop left, 16-element
// threshold, heap sort at depth 2 floor(log2 n)) followed by one insertion sort over the whole array.
// This replays the loop level by level on one workgroup: all segments of a recursion level are
// partitioned at once. The partition of a segment [f, l) with pivot key K at f is computed, not
// simulated: with LS = the positions p in (f, l) with key >= K in ascending order ("left stops") and
// RS = the positions in [f, l) with key <= K in descending order ("right stops"), Hoare's scan swaps
// LS[j] <-> RS[j] for exactly the j < k with LS[j] < RS[j] (both sequences are monotone, so that is a
// prefix) and returns cut = min(LS[k], RS[k-1]) (LS[k] when k = 0, RS[k-1] when LS runs out): every
// element a scan passes before a swap is untouched, and the first swapped element a scan meets stops
// it. The stops are per-chunk bit masks + exclusive prefix counts (each thread owns C <= 64
// consecutive positions), scattered into position arrays by stop index, so the j-th stop of a
// segment is one lookup and k one binary search. Segments of <= 16 elements get their final
// insertion sort (stable, and the partition property keeps every element inside its leaf) as soon as
// they form; depth-exhausted segments are heap-sorted by one thread, exactly as
// std::__partial_sort(first, last, last) does. The characterisation is checked against libstdc++ on
// the host (oracle/aloam_oracle.cpp oracle_pcl_replay_check, tests/test_oracle_pins.py) and the device
// code by the VoxelGrid / scanRegistration / mapping parity tests against the oracle's PCL order.
#pragma once
#include "aloam_device.hpp"

namespace aloam {

constexpr int PS_THRESHOLD = 16;    // libstdc++ _S_threshold
constexpr int PS_MAX_CHUNK = 64;    // positions per thread (u64 stop masks)

// chunk scratch ints for NT threads (LDS); segment arrays: 9 ints per segment
__host__ __device__ constexpr int ps_scratch_ints(int NT) { return 8 + 2 * (NT / 64) + 7 * (NT + 1); }
__host__ __device__ constexpr int ps_seg_ints(int segcap) { return 9 * segcap; }
// segments a sort of n elements can have active at once (each holds > 16 elements)
__host__ __device__ constexpr int ps_segcap(int n) { return n / (PS_THRESHOLD + 1) + 1; }

__device__ __forceinline__ unsigned ps_key(unsigned long long e) { return (unsigned)(e >> 32); }

template <bool G>
__device__ __forceinline__ void ps_bar() {
    if (G) __syncthreads();
    else lds_barrier();
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
// The same order for a leaf of m <= 16 elements, in registers: odd-even transposition with adjacent
// swaps only where the keys are strictly out of order (a stable sort); padding sorts last.
__device__ __forceinline__ void ps_leaf_sort(unsigned long long* E, int f, int l) {
    const int m = l - f;
    if (m < 2) return;
    unsigned long long v[PS_THRESHOLD];
#pragma unroll
    for (int i = 0; i < PS_THRESHOLD; i++) v[i] = i < m ? E[f + i] : ~0ull;
#pragma unroll
    for (int r = 0; r < PS_THRESHOLD; r++) {
#pragma unroll
        for (int i = r & 1; i + 1 < PS_THRESHOLD; i += 2) {
            const unsigned long long a = v[i], b = v[i + 1];
            const bool sw = ps_key(b) < ps_key(a);
            v[i] = sw ? b : a;
            v[i + 1] = sw ? a : b;
        }
    }
#pragma unroll
    for (int i = 0; i < PS_THRESHOLD; i++)
        if (i < m) E[f + i] = v[i];
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
__device__ inline void ps_serial_std_sort(unsigned long long* E, int n) {
    if (n <= 1) return;
    int sf[64], sl[64], sd[64], sp = 0;
    sf[0] = 0; sl[0] = n; sd[0] = 2 * (31 - __clz(n)); sp = 1;
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

// number of stops at positions < p (pref: exclusive per-chunk prefix, mask: per-chunk stop bits)
__device__ __forceinline__ int ps_count_before(const int* pref, const unsigned long long* mask, int p, int C) {
    const int t = p / C, o = p - t * C;
    return pref[t] + (o ? __popcll(mask[t] & ((1ull << o) - 1ull)) : 0);
}
// last segment s with f[s] <= p (-1: none); f ascending
__device__ __forceinline__ int ps_find_seg(const int* f, int nseg, int p) {
    int lo = 0, hi = nseg - 1, r = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (f[mid] <= p) { r = mid; lo = mid + 1; }
        else hi = mid - 1;
    }
    return r;
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

// The sort. E, Lpos, Rpos (n ints each: the stops' positions by global stop index) and seg
// (ps_seg_ints(segcap) ints, segcap >= ps_segcap(n)) in LDS (G = false) or any of them in global
// memory (G = true: every exchange is then a full barrier); sc: ps_scratch_ints(NT) ints of LDS,
// 8-byte aligned. n <= NT * PS_MAX_CHUNK (the caller checks). All NT threads call it with the same
// n. Ends with a barrier.
template <int NT, bool G>
__device__ void pcl_std_sort(unsigned long long* E, const int n, int* Lpos, int* Rpos, int* sc, int* seg, const int segcap) {
    const int tid = threadIdx.x;
    if (n <= 1) return;
    if (n <= PS_THRESHOLD) {
        if (tid == 0) ps_leaf_sort(E, 0, n);
        ps_bar<G>();
        return;
    }
    constexpr int NW = NT / WAVE;
    int* shv = sc;                               // [0] active segments
    int* ws = sc + 8;
    unsigned long long* maskL = (unsigned long long*)(ws + 2 * NW);   // (8 + 2 NW ints: 8-byte aligned)
    unsigned long long* maskR = maskL + NT + 1;
    int* prefL = (int*)(maskR + NT + 1);
    int* prefR = prefL + NT + 1;
    int* sidx = prefR + NT + 1;
    int* sb = seg;
    int* Fa[2] = {sb, sb + segcap};
    int* La[2] = {sb + 2 * segcap, sb + 3 * segcap};
    unsigned* Kp = (unsigned*)(sb + 4 * segcap);
    int* BL = sb + 5 * segcap;
    int* TR = sb + 6 * segcap;
    int* KK = sb + 7 * segcap;
    int* CUT = sb + 8 * segcap;
    const int C = (n + NT - 1) / NT;
    const int nch = (n + C - 1) / C;
    int depth = 2 * (31 - __clz(n));
    if (tid == 0) { Fa[0][0] = 0; La[0][0] = n; shv[0] = 1; }
    lds_barrier();
    int cur = 0;
    for (;;) {
        const int nseg = shv[0];
        if (nseg == 0) break;
        const int* f = Fa[cur];
        const int* l = La[cur];
        if (depth == 0) {                       // introsort's depth limit: heap sort what is left
            for (int s = tid; s < nseg; s += NT) ps_heap_sort(E + f[s], E + l[s]);
            ps_bar<G>();
            break;
        }
        depth--;
        // (1) __move_median_to_first(first, first + 1, mid, last - 1)
        for (int s = tid; s < nseg; s += NT) {
            const int fs = f[s], a = fs + 1, b = fs + (l[s] - fs) / 2, c = l[s] - 1;
            const unsigned ka = ps_key(E[a]), kb = ps_key(E[b]), kc = ps_key(E[c]);
            int pick;
            if (ka < kb) pick = kb < kc ? b : (ka < kc ? c : a);
            else pick = ka < kc ? a : (kb < kc ? c : b);
            const unsigned long long ef = E[fs], ep = E[pick];
            E[fs] = ep;
            E[pick] = ef;
            Kp[s] = ps_key(ep);
        }
        ps_bar<G>();
        // (2) left / right stops of every chunk: bit masks, prefix counts, positions by stop index
        int cl = 0, cr = 0;
        unsigned long long mL = 0, mR = 0;
        const int p0 = tid * C;
        if (tid < nch) {
            const int p1 = min(n, p0 + C);
            int s = ps_find_seg(f, nseg, p0);
            sidx[tid] = s;
            for (int p = p0; p < p1; p++) {
                while (s + 1 < nseg && f[s + 1] <= p) s++;
                if (s >= 0 && p < l[s]) {
                    const unsigned kp = ps_key(E[p]), kv = Kp[s];
                    if (p > f[s] && kp >= kv) mL |= 1ull << (p - p0);
                    if (kp <= kv) mR |= 1ull << (p - p0);
                }
            }
            cl = __popcll(mL);
            cr = __popcll(mR);
        }
        int tl, tr;
        ps_exscan2<NT>(cl, cr, ws, tl, tr);
        if (tid < nch) {
            prefL[tid] = cl; prefR[tid] = cr; maskL[tid] = mL; maskR[tid] = mR;
            int g = cl;
            for (unsigned long long m = mL; m; m &= m - 1ull) Lpos[g++] = p0 + __builtin_ctzll(m);
            g = cr;
            for (unsigned long long m = mR; m; m &= m - 1ull) Rpos[g++] = p0 + __builtin_ctzll(m);
        }
        if (tid == 0) { prefL[nch] = tl; prefR[nch] = tr; maskL[nch] = 0ull; maskR[nch] = 0ull; }
        ps_bar<G>();
        // (3) per segment: swap count k (the first j with LS[j] >= RS[j]) and the cut
        for (int s = tid; s < nseg; s += NT) {
            const int fs = f[s], ls = l[s];
            const int bL = ps_count_before(prefL, maskL, fs, C), eL = ps_count_before(prefL, maskL, ls, C);
            const int bR = ps_count_before(prefR, maskR, fs, C), eR = ps_count_before(prefR, maskR, ls, C);
            const int nL = eL - bL, nR = eR - bR;
            int lo = 0, hi = min(nL, nR);
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (Lpos[bL + mid] < Rpos[eR - 1 - mid]) lo = mid + 1;
                else hi = mid;
            }
            const int k = lo;
            int cut;
            if (k < nL) {
                cut = Lpos[bL + k];
                if (k > 0) cut = min(cut, Rpos[eR - k]);
            } else {
                cut = Rpos[eR - k];
            }
            BL[s] = bL; TR[s] = eR; KK[s] = k; CUT[s] = cut;
        }
        ps_bar<G>();                             // (the segment arrays may be in global memory)
        // (4) the swaps: left stop j <-> right stop j for j < k (disjoint pairs, one thread each)
        if (tid < nch && mL) {
            int s = sidx[tid];
            int g = cl;
            for (unsigned long long m = mL; m; m &= m - 1ull) {
                const int p = p0 + __builtin_ctzll(m);
                while (s + 1 < nseg && f[s + 1] <= p) s++;
                const int j = g - BL[s];
                if (j < KK[s]) {
                    const int q = Rpos[TR[s] - 1 - j];
                    const unsigned long long ep = E[p], eq = E[q];
                    E[p] = eq;
                    E[q] = ep;
                }
                g++;
            }
        }
        ps_bar<G>();
        // (5) children: > 16 elements -> next level (in order), else their final insertion sort
        {
            const int per = (nseg + NT - 1) / NT;
            const int s0 = min(nseg, tid * per), s1 = min(nseg, s0 + per);
            int cnt = 0, dummy = 0;
            for (int s = s0; s < s1; s++) cnt += (CUT[s] - f[s] > PS_THRESHOLD) + (l[s] - CUT[s] > PS_THRESHOLD);
            int tot, td;
            ps_exscan2<NT>(cnt, dummy, ws, tot, td);
            int* nf = Fa[cur ^ 1];
            int* nl = La[cur ^ 1];
            for (int s = s0; s < s1; s++) {
                const int fs = f[s], c = CUT[s], ls = l[s];
                if (c - fs > PS_THRESHOLD) { nf[cnt] = fs; nl[cnt] = c; cnt++; }
                else ps_leaf_sort(E, fs, c);
                if (ls - c > PS_THRESHOLD) { nf[cnt] = c; nl[cnt] = ls; cnt++; }
                else ps_leaf_sort(E, c, ls);
            }
            if (tid == 0) shv[0] = tot;
        }
        ps_bar<G>();
        cur ^= 1;
    }
}

}  // namespace aloam
