// ls_sort.hpp — libstdc++ std::sort order of (leaf, index) pairs in LDS, level-synchronous.
//
// PCL's VoxelGrid (voxel_grid.hpp applyFilter, called at src/scanRegistration.cpp:401-405 and
// src/laserMapping.cpp:542-550,788-801) sums each leaf's points in the order an unstable std::sort by
// leaf leaves them. pcl_sort.hpp characterises one Hoare partition in closed form (LS = left stops,
// RS = right stops: swap LS[j] <-> RS[j] for the prefix j < k with LS[j] < RS[j], cut = min(LS[k],
// RS[k-1])); this file applies that characterisation to EVERY active segment of one introsort level at
// once, element-parallel over the whole workgroup, level after level:
//
//   A  stop flags of every position against its segment's pivot (one ballot pair per 64-position chunk)
//   B  exclusive scan of the chunk stop counts -> global stop ranks
//   C  per segment: its first left-stop rank, its right-stop range; every right stop writes its position
//      into RS_pos[global rank]
//   D  every left stop finds its partner RS[j] by one LDS read, swaps when LS[j] < RS[j]; the cut is the
//      minimum of the first non-swapping left stop and the partner of the last swapping one (LDS atomicMin,
//      at most two candidates per segment and chunk)
//   E  per segment: children (> 16 elements and depth left: next level, median moved to first; depth
//      exhausted: heap sort, std::__partial_sort; <= 16: a leaf), new segment list by a scan
//
// Chunk c (64 positions) belongs to wave c mod W. Every element carries the id of its position's segment
// in its payload's upper half (swaps never leave a segment); segment boundaries are kept as bits;
// the final insertion sort (stable, whole array) only moves elements inside their <= 16-element leaves,
// which a last pass sorts by stable rank.
//
// Cost per level: ~7 workgroup barriers + a few LDS accesses per position; the number of levels is the
// introsort's recursion depth (~1.5-2 log2(n / 16)). Replaces the wave-queue replay of pcl_sort.hpp for
// arrays that fit LDS (that one spent most of its time in lane-serial sorts of <= 64-element segments).
#pragma once
#include "pcl_sort.hpp"

#ifndef LS_TS
#define LS_TS(k) do { } while (0)     // profiling builds (micro/ls_bench.hip): phase stamps
#endif


namespace aloam {

constexpr int LS_INACT = 0xffff;
#ifndef LS_TAIL_DEF
#define LS_TAIL_DEF 256                   // (tests vary it)
#endif
constexpr int LS_TAIL = LS_TAIL_DEF;     // the waves take over when every active segment has <= this many elements

// LDS scratch (bytes, 8-byte aligned sections) for n <= nmax elements sorted by NT threads
__host__ __device__ constexpr int ls_nc(int nmax) { return (nmax + 63) / 64; }
__host__ __device__ constexpr int ls_smax(int nmax) { return nmax / 17 + 2; }
__host__ __device__ constexpr size_t ls_al8(size_t b) { return (b + 7) & ~(size_t)7; }
constexpr int LS_HQ = 128;                // depth-exhausted segments queued for the waves' heap sorts (rel)
__host__ __device__ constexpr size_t ls_scratch_bytes(int NT, int nmax) {
    return ls_al8(4 * (size_t)(16 + 2 * (NT / 64) + 2))          // hdr + scan words
           + 8 * (size_t)LS_HQ                                   // heap queue (f, l)
           + 4 * 8 * (size_t)(ls_nc(nmax) + 1)                   // maskL, maskR, boundary bits, maskV (relevant)
           + 8 * 64                                              // active-chunk bits (2 levels x 32 words)
           + ls_al8(3 * 4 * (size_t)(ls_nc(nmax) + 1))           // prefL, prefR, prefV
           + ls_al8(2 * (size_t)nmax)                            // RS_pos (u16)
           + 4 * (size_t)ls_smax(nmax) * 13;                     // 2 x (F, L, D, K) + bL, eR, nR, cut, idx
}

struct LsScr {
    int* hdr; int* ws;
    unsigned long long *maskL, *maskR, *bits, *act, *maskV;
    int *prefL, *prefR, *prefV;
    unsigned short* rs;
    int* seg0;           // 2 buffers x (F, L, D, K) x sm ints
    int sm;
    int* hq;             // heap queue: f, l per entry (count in hdr[6])
    int *bL, *eR, *nR, *cut, *idx;
    __device__ __forceinline__ int* seg(int b, int k) const { return seg0 + (b * 4 + k) * sm; }
    __device__ __forceinline__ LsScr(unsigned char* p, int NT, int nmax) {
        const int nc = ls_nc(nmax), sm = ls_smax(nmax);
        hdr = (int*)p; ws = hdr + 16;
        p += ls_al8(4 * (size_t)(16 + 2 * (NT / 64) + 2));
        hq = (int*)p;
        p += 8 * (size_t)LS_HQ;
        maskL = (unsigned long long*)p; maskR = maskL + nc + 1; bits = maskR + nc + 1; maskV = bits + nc + 1;
        p += 4 * 8 * (size_t)(nc + 1);
        act = (unsigned long long*)p;
        p += 8 * 64;
        prefL = (int*)p; prefR = prefL + nc + 1; prefV = prefR + nc + 1;
        p += ls_al8(3 * 4 * (size_t)(nc + 1));
        rs = (unsigned short*)p;
        p += ls_al8(2 * (size_t)nmax);
        int* q = (int*)p;
        seg0 = q; this->sm = sm;
        q += 8 * sm;
        bL = q; eR = bL + sm; nR = eR + sm; cut = nR + sm; idx = cut + sm;
    }
};

// stops at positions < p (p <= 64 * nc; mask[nc] = 0)
__device__ __forceinline__ int ls_before(const int* pref, const unsigned long long* mask, int p) {
    const int c = p >> 6, o = p & 63;
    return pref[c] + (o ? __popcll(mask[c] & ((1ull << o) - 1ull)) : 0);
}

// Segment id of the position an element sits on, kept in bits 16-31 of its payload (payloads are < 2^16
// here): every swap of the introsort stays inside one segment, so the id travels with the element and
// is correct for whichever position it lands on. Cleared by the final pass.
__device__ __forceinline__ int ls_seg(unsigned long long e) { return (int)((e >> 16) & 0xffffu); }
__device__ __forceinline__ unsigned long long ls_with_seg(unsigned long long e, int s) {
    return (e & ~0xffff0000ull) | ((unsigned long long)(unsigned)s << 16);
}

__device__ __forceinline__ unsigned long long ls_shfl64(unsigned long long v, int src) {
    return ((unsigned long long)(unsigned)__shfl((int)(v >> 32), src, WAVE) << 32) | (unsigned)__shfl((int)v, src, WAVE);
}

// __move_median_to_first(f, f + 1, mid, l - 1) as ps_median_to_first, also returning pick - f
__device__ __forceinline__ unsigned ls_median_to_first(unsigned long long* E, int f, int l, int* off) {
    const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const unsigned ka = ps_key(E[a]), kb = ps_key(E[b]), kc = ps_key(E[c]);
    int pick;
    if (ka < kb) pick = kb < kc ? b : (ka < kc ? c : a);
    else pick = ka < kc ? a : (kb < kc ? c : b);
    const unsigned long long ef = E[f], ep = E[pick];
    E[f] = ep;
    E[pick] = ef;
    *off = pick - f;
    return ps_key(ep);
}

// ---- one wave, one segment (the last, sparse levels) ----------------------------------------------------
// Whole introsort subtree of a segment [f, f + m), m <= 64, from depth d, in registers: lane i holds
// position f + i. Every level partitions all of its > 16-element sub-segments at once (each lane knows its
// sub-segment from the boundary bits): median of (a + 1, mid, b - 1) moved to a, the Hoare swaps LS[j] <->
// RS[j] for j < k as lane gathers, the cut from k. Depth exhausted: heap sort (std::__partial_sort) of the
// remaining > 16 sub-segments by one lane each. Then every final sub-segment of <= 16 is stably ranked (the
// final insertion sort) and written back.
// fb (may be null): LDS bytes at 2 x position free for the heap sorts' child flags (the RS region of the segment)
__device__ __forceinline__ void ws_small(unsigned long long* E, const int f, const int m, int d, const unsigned* rel = nullptr,
                                         unsigned char* fb = nullptr) {
    const int lane = lane_id();
    const unsigned long long lt = lanemask_lt64(), le = lt | (1ull << lane), gt = ~le;
    const unsigned long long all = m >= 64 ? ~0ull : ((1ull << m) - 1ull);
    const bool in = lane < m;
    unsigned long long e = in ? E[f + lane] : ~0ull;
    unsigned k = ps_key(e);
    unsigned long long starts = 1ull;
    int a = 0, b = m;
    for (;;) {
        a = ps_msb(starts & le);
        const unsigned long long nb = starts & gt & all;
        b = nb ? __builtin_ctzll(nb) : m;
        bool act = in && b - a > PS_THRESHOLD;
        if (rel) {                                       // sub-segments with < 2 relevant points retire (rvg.hpp)
            const unsigned i = (unsigned)e & 0xffffu;
            const unsigned long long mv = __ballot(in && ((rel[i >> 5] >> (i & 31u)) & 1u));
            const unsigned long long sg = (b >= 64 ? ~0ull : ((1ull << b) - 1ull)) & ~((1ull << a) - 1ull);
            act = act && __popcll(mv & sg) >= 2;
        }
        if (!__ballot(act)) break;
        if (d == 0) {                                    // (rare) heap sort the > 16 sub-segments
            if (in) E[f + lane] = e;
            ps_wsync<true>();
            unsigned long long hm = __ballot(act && lane == a);   // the sub-segments, each by the whole wave
            while (hm) {
                const int a2 = __builtin_ctzll(hm);
                hm &= hm - 1ull;
                const int b2 = readlane_i(b, a2);
                if (ws_order_matters(E, f + a2, f + b2, rel)) ws_heap_sort(E, f + a2, f + b2, rel, fb ? fb + 2 * (f + a2) : nullptr);
            }
            ps_wsync<true>();
            e = in ? E[f + lane] : ~0ull;
            k = ps_key(e);
            ps_wsync<false>();
            break;
        }
        d--;
        const int mid = a + (b - a) / 2;
        const unsigned ka = (unsigned)__shfl((int)k, act ? a + 1 : lane, WAVE);
        const unsigned kb = (unsigned)__shfl((int)k, act ? mid : lane, WAVE);
        const unsigned kc = (unsigned)__shfl((int)k, act ? b - 1 : lane, WAVE);
        int pick;
        if (ka < kb) pick = kb < kc ? mid : (ka < kc ? b - 1 : a + 1);
        else pick = ka < kc ? a + 1 : (kb < kc ? b - 1 : mid);
        int src = lane;
        if (act) src = lane == a ? pick : (lane == pick ? a : lane);
        e = ls_shfl64(e, src);
        k = ps_key(e);
        const unsigned K = (unsigned)__shfl((int)k, act ? a : lane, WAVE);
        const bool isL = act && lane > a && k >= K, isR = act && k <= K;
        const unsigned long long mL = __ballot(isL), mR = __ballot(isR);
        const unsigned long long segm = (b >= 64 ? ~0ull : ((1ull << b) - 1ull)) & ~((1ull << a) - 1ull);
        const unsigned long long sL = mL & segm, sR = mR & segm;
        const int nL = __popcll(sL), nR = __popcll(sR);
        src = lane;
        bool swL = false;
        if (isL) {
            const int j = __popcll(sL & lt);
            if (j < nR) {
                const int q = ps_select_bit(sR, nR - 1 - j);
                if (lane < q) { src = q; swL = true; }
            }
        }
        if (isR && !swL) {
            const int i = nR - 1 - __popcll(sR & lt);
            if (i < nL) {
                const int p2 = ps_select_bit(sL, i);
                if (p2 < lane) src = p2;
            }
        }
        e = ls_shfl64(e, src);
        k = ps_key(e);
        const int kk = __popcll(__ballot(swL) & segm);
        int cut = 0x7fffffff;
        if (kk < nL) cut = ps_select_bit(sL, kk);
        if (kk >= 1) cut = min(cut, ps_select_bit(sR, nR - kk));
        starts |= __ballot(act && lane == cut);
    }
    int r = lane;
    if (__ballot(in && b - a <= PS_THRESHOLD)) {
        int c = a;
#pragma unroll
        for (int i = 0; i < PS_THRESHOLD; i++) {
            const unsigned ki = (unsigned)__shfl((int)k, min(a + i, WAVE - 1), WAVE);
            c += a + i < b && (ki < k || (ki == k && a + i < lane));
        }
        if (b - a <= PS_THRESHOLD) r = c;
    }
    if (in) E[f + r] = e;
    ps_wsync<false>();
}

// Partition of [f, l) (l - f > 64) by one wave; returns the cut. Chunk u = positions f + 64u + lane; lane u
// keeps chunk u's stop masks and their exclusive prefixes (l - f <= 4096). Right stops are scattered to
// RS[f + ascending rank]; every left stop of rank j reads its partner RS[j] = RS[f + nR - 1 - j] and swaps
// when it lies before it (a prefix of the left stops: the loop ends at the first chunk with a refusal).
// cut = min(first non-swapping left stop, partners of the swapping ones).
__device__ __forceinline__ int ws_partition(unsigned long long* E, const int f, const int l, unsigned short* RS) {
    const int lane = lane_id();
    const unsigned long long lt = lanemask_lt64();
    int k0 = 0;
    PS_SAME(k0 = (int)ps_median_to_first(E, f, l));
    const unsigned K = (unsigned)ps_u(k0);
    ps_wsync<false>();
    const int nch = ps_u((l - f + 63) >> 6);
    unsigned long long myL = 0, myR = 0;
    for (int u = 0; u < nch; u++) {
        const int p = f + (u << 6) + lane;
        const bool inn = p < l;
        const unsigned kk = inn ? ps_keyat(E, p) : 0u;
        const unsigned long long bl = __ballot(inn && p > f && kk >= K);
        const unsigned long long br = __ballot(inn && kk <= K);
        myL = lane == u ? bl : myL;
        myR = lane == u ? br : myR;
    }
    const int cl = __popcll(myL), cr = __popcll(myR);
    const int iL = wave_incl_scan(cl), iR = wave_incl_scan(cr);
    const int pL = iL - cl, pR = iR - cr;
    const int nR = ps_u(readlane_i(iR, WAVE - 1));
    for (int u = 0; u < nch; u++) {
        const unsigned long long bR = ps_rl64(myR, u);
        const int pRu = ps_u(readlane_i(pR, u));
        if ((bR >> lane) & 1ull) RS[f + pRu + __popcll(bR & lt)] = (unsigned short)(f + (u << 6) + lane);
    }
    ps_wsync<false>();
    int cand = 0x7fffffff;
    for (int u = 0; u < nch; u++) {
        const unsigned long long bL = ps_rl64(myL, u);
        if (bL == 0ull) continue;
        const int pLu = ps_u(readlane_i(pL, u));
        const int p = f + (u << 6) + lane;
        const bool isL = (bL >> lane) & 1ull;
        bool sw = false;
        int q = 0;
        if (isL) {
            const int j = pLu + __popcll(bL & lt);
            if (j < nR) { q = RS[f + nR - 1 - j]; sw = p < q; }
            cand = min(cand, sw ? q : p);
        }
        if (sw) {
            const unsigned long long ep = E[p], eq = E[q];
            E[p] = eq;
            E[q] = ep;
        }
        if (__ballot(isL && !sw)) break;                 // the rest of the left stops do not swap
    }
    const int cut = ps_u((int)allreduce_u32<6>((unsigned)cand, [](unsigned x, unsigned y) { return x < y ? x : y; }));
    ps_wsync<false>();
    PS_CHECK(cut > f && cut < l, "ws cut: f %d l %d cut %d\n", f, l, cut);
    return cut;
}

// introsort_loop of one segment by one wave: partitions while > 64 elements (right children on a lane
// stack), the <= 64-element parts in registers
__device__ __forceinline__ void ws_segment(unsigned long long* E, int f, int l, int d, unsigned short* RS, const unsigned* rel = nullptr) {
    const int lane = lane_id();
    int sp = 0, stf = 0, stl = 0, std_ = 0;
    for (;;) {
        for (;;) {
            if (l - f <= WAVE) {
                if (l - f >= 2) ws_small(E, f, l - f, d, rel, (unsigned char*)RS);
                break;
            }
            if (d == 0) {   // the child flags in this segment's part of RS (its partitions are done)
                if (ws_order_matters(E, f, l, rel)) ws_heap_sort(E, f, l, rel, (unsigned char*)RS + 2 * f);
                ps_wsync<false>();
                break;
            }
            if (rel && !ws_order_matters(E, f, l, rel)) break;   // < 2 relevant points: retires (rvg.hpp)
            d = ps_u(d - 1);
            const int cut = ws_partition(E, f, l, RS);
            stf = lane == sp ? cut : stf;
            stl = lane == sp ? l : stl;
            std_ = lane == sp ? d : std_;
            sp = ps_u(sp + 1);
            l = ps_u(cut);
        }
        if (sp == 0) break;
        sp = ps_u(sp - 1);
        f = ps_u(readlane_i(stf, sp)); l = ps_u(readlane_i(stl, sp)); d = ps_u(readlane_i(std_, sp));
    }
}

// std::sort(E, E + n) by key (E[i] >> 32) as libstdc++ orders it, from introsort depth d0 (a whole sort:
// 2 floor(log2 n); a segment of a larger sort: its remaining depth), E and scratch in LDS, n <= NT * CPW,
// payloads (E[i] & 0xffffffff) < 2^16. All NT threads call it with the same arguments; it ends with a
// barrier.
template <int NT, int CPW>
__device__ __forceinline__ void ls_sort(unsigned long long* E, const int n, const int d0, unsigned char* scratch, const int nmax,
                                        const unsigned* rel = nullptr) {
    constexpr int W = NT / 64;
    static_assert(NT % 64 == 0 && CPW >= 1 && CPW <= 16, "ls_sort: chunks per wave, one segment per thread");
    const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
    if (n <= 1) return;
    LsScr S(scratch, NT, nmax);
    const int nc = (n + 63) >> 6;
    const unsigned long long lt = lanemask_lt64(), le = lt | (1ull << lane), gt = ~le;
    // boundary bits (position 0 starts a segment); active-chunk bits (chunks holding an active segment)
    for (int w = tid; w <= nc; w += NT) S.bits[w] = w == 0 ? 1ull : 0ull;
    if (tid < 16) S.hdr[tid] = 0;
    if (tid < 64) {                         // level 0 (buffer 0): chunks [0, nc); buffer 1 empty
        const int c0 = 64 * tid;
        S.act[tid] = tid >= 32 || c0 >= nc ? 0ull : (c0 + 64 <= nc ? ~0ull : (1ull << (nc - c0)) - 1ull);
    }
    int ns = 0;
    if (n > PS_THRESHOLD && d0 > 0) {
        ns = 1;
        if (tid == 0) {
            int o = 0;
            S.seg(0, 0)[0] = 0; S.seg(0, 1)[0] = n;
            S.seg(0, 3)[0] = (int)ls_median_to_first(E, 0, n, &o);
            S.seg(0, 2)[0] = d0 | (o << 8);
        }
    } else if (n > PS_THRESHOLD) {
        if (tid == 0) ps_heap_sort_rel(E, 0, n, rel);
    }
    lds_barrier();
    int b = 0;
    bool first = true;                      // level 0: every position in segment 0 (payload bits 16-31 = 0)
    while (ns > 0) {
        LS_TS(0);
        const int* F = S.seg(b, 0);
        const int* L = S.seg(b, 1);
        const int* D = S.seg(b, 2);
        const int* K = S.seg(b, 3);
        const unsigned long long* actb = S.act + (b ? 32 : 0);
        // A: every position's segment of this level (the child of last level's segment), stop flags, chunk
        // counts (inactive chunks: none)
#pragma unroll 2
        for (int c = wid; c < nc; c += W) {
            unsigned long long mL = 0ull, mR = 0ull, mV = 0ull;
            if ((actb[c >> 6] >> (c & 63)) & 1ull) {
                const int p = (c << 6) + lane;
                bool isL = false, isR = false, isV = false;
                if (p < n) {
                    unsigned long long e = E[p];
                    int s = ls_seg(e);
                    if (!first && s != LS_INACT) {
                        const int ix = S.idx[s];
                        const int s2 = p < S.cut[s] ? (ix & 0xffff) : (int)((unsigned)ix >> 16);
                        E[p] = ls_with_seg(e, s2);
                        s = s2;
                    }
                    if (s != LS_INACT) {
                        const unsigned key = ps_key(e), kp = (unsigned)K[s];
                        isL = p > F[s] && key >= kp;
                        isR = key <= kp;
                        if (rel) { const unsigned i = (unsigned)e & 0xffffu; isV = (rel[i >> 5] >> (i & 31u)) & 1u; }
                    }
                }
                mL = __ballot(isL);
                mR = __ballot(isR);
                if (rel) mV = __ballot(isV);
            }
            if (lane == 0) {
                S.maskL[c] = mL; S.maskR[c] = mR; S.prefL[c] = __popcll(mL); S.prefR[c] = __popcll(mR);
                if (rel) { S.maskV[c] = mV; S.prefV[c] = __popcll(mV); }
            }
        }
        first = false;
        lds_barrier();
        LS_TS(1);
        // B: exclusive scan of the chunk counts by wave 0 (nc <= 64 * 16)
        if (wid == 0) {
            int carryL = 0, carryR = 0;
            for (int c0 = 0; c0 < nc; c0 += 64) {
                const int c = c0 + lane;
                const int a = c < nc ? S.prefL[c] : 0, r = c < nc ? S.prefR[c] : 0;
                const int ia = wave_incl_scan(a), ir = wave_incl_scan(r);
                if (c < nc) { S.prefL[c] = carryL + ia - a; S.prefR[c] = carryR + ir - r; }
                carryL += readlane_i(ia, WAVE - 1);
                carryR += readlane_i(ir, WAVE - 1);
            }
            if (lane == 0) { S.prefL[nc] = carryL; S.prefR[nc] = carryR; S.maskL[nc] = 0ull; S.maskR[nc] = 0ull; }
        } else if (rel && wid == 1) {
            int carryV = 0;
            for (int c0 = 0; c0 < nc; c0 += 64) {
                const int c = c0 + lane;
                const int v = c < nc ? S.prefV[c] : 0;
                const int iv = wave_incl_scan(v);
                if (c < nc) S.prefV[c] = carryV + iv - v;
                carryV += readlane_i(iv, WAVE - 1);
            }
            if (lane == 0) { S.prefV[nc] = carryV; S.maskV[nc] = 0ull; }
        }
        lds_barrier();
        LS_TS(2);
        // C: per segment stop ranges; right stops -> RS_pos by global rank
        if (tid < ns) {
            const int f = F[tid], l = L[tid];
            const int eR = ls_before(S.prefR, S.maskR, l);
            S.bL[tid] = ls_before(S.prefL, S.maskL, f);
            S.eR[tid] = eR;
            S.nR[tid] = eR - ls_before(S.prefR, S.maskR, f);
            S.cut[tid] = 0x7fffffff;
            // fewer than two relevant points (rvg.hpp): the segment's order is never read, it retires here
            // (no swaps: no right stops; eR < 0 marks it for phase E)
            if (rel && ls_before(S.prefV, S.maskV, l) - ls_before(S.prefV, S.maskV, f) < 2) { S.nR[tid] = 0; S.eR[tid] = -1; }
        }
        for (int c = wid; c < nc; c += W) {
            const unsigned long long mR = S.maskR[c];
            if ((mR >> lane) & 1ull) S.rs[S.prefR[c] + __popcll(mR & lt)] = (unsigned short)((c << 6) + lane);
        }
        lds_barrier();
        LS_TS(3);
        // D: swaps and cut candidates
#pragma unroll 2
        for (int c = wid; c < nc; c += W) {
            const unsigned long long mL = S.maskL[c];
            if (mL == 0ull) continue;
            const int p = (c << 6) + lane;
            const bool isL = (mL >> lane) & 1ull;
            unsigned long long ep = 0ull;
            int s = -1;
            if (p < n) { ep = E[p]; s = ls_seg(ep); }
            PS_CHECK(!isL || (s >= 0 && s < ns), "ls D: p %d s %d ns %d\n", p, s, ns);
            bool sw = false;
            int q = 0;
            if (isL) {
                const int j = S.prefL[c] + __popcll(mL & lt) - S.bL[s];
                if (j < S.nR[s]) {
                    q = S.rs[S.eR[s] - 1 - j];
                    sw = p < q;
                }
            }
            if (sw) {
                const unsigned long long eq = E[q];
                E[p] = eq;
                E[q] = ep;
            }
            const int sprev = __shfl(s, lane == 0 ? 0 : lane - 1, WAVE);
            const unsigned long long bnd = __ballot(lane == 0 || s != sprev);
            const unsigned long long nswm = __ballot(isL && !sw), swm = __ballot(sw);
            const int lo = ps_msb(bnd & le);
            const unsigned long long nb = bnd & gt;
            const unsigned long long grp = (nb ? ((1ull << __builtin_ctzll(nb)) - 1ull) : ~0ull) & ~((1ull << lo) - 1ull);
            if (isL && !sw && (nswm & grp & lt) == 0ull && S.eR[s] >= 0) atomicMin(&S.cut[s], p);
            if (sw && (swm & grp & gt) == 0ull) atomicMin(&S.cut[s], q);
        }
        lds_barrier();
        LS_TS(4);
        // E: children -> next list (ids from a wave-aggregated counter; medians moved to first), active
        // chunks of the next level, heap sorts of depth-exhausted children
        {
            unsigned long long* actn = S.act + (b ? 0 : 32);
            int* cnt = &S.hdr[8 + (b ^ 1)];
            int* mx = &S.hdr[12 + (b ^ 1)];
            int aL = 0, aR = 0, f = 0, l = 0, cut = 0, d = 0;
            const bool retired = tid < ns && S.eR[tid] < 0;
            if (tid < ns && !retired) {
                f = F[tid]; l = L[tid]; d = (D[tid] & 0xff) - 1; cut = S.cut[tid];
                PS_CHECK(cut > f && cut < l, "ls cut: f %d l %d cut %d\n", f, l, cut);
                atomicOr(&S.bits[cut >> 6], 1ull << (cut & 63));
                // depth exhausted: heap sort (with rel: queued for the waves, after the levels)
                auto heap = [&](int f2, int l2) {
                    if (rel) {
                        const int q = atomicAdd(&S.hdr[6], 1);
                        if (q < LS_HQ) { S.hq[2 * q] = f2; S.hq[2 * q + 1] = l2; return; }
                    }
                    ps_heap_sort_rel(E, f2, l2, rel);
                };
                if (cut - f > PS_THRESHOLD) { if (d > 0) aL = 1; else heap(f, cut); }
                if (l - cut > PS_THRESHOLD) { if (d > 0) aR = 1; else heap(cut, l); }
            }
            const int mine = aL + aR;
            const int incl = wave_incl_scan(mine);
            int base = 0;
            if (lane == WAVE - 1 && incl) base = atomicAdd(cnt, incl);
            base = readlane_i(base, WAVE - 1) + incl - mine;
            int* Fn = S.seg(b ^ 1, 0);
            int* Ln = S.seg(b ^ 1, 1);
            int* Dn = S.seg(b ^ 1, 2);
            int* Kn = S.seg(b ^ 1, 3);
            if (tid < ns && retired) S.idx[tid] = LS_INACT | (LS_INACT << 16);
            if (tid < ns && !retired) {
                // D: depth | (median position - f) << 8 (the wave tail undoes the median move)
                int o = 0;
                if (aL) { Fn[base] = f; Ln[base] = cut; Kn[base] = (int)ls_median_to_first(E, f, cut, &o); Dn[base] = d | (o << 8); }
                if (aR) { Fn[base + aL] = cut; Ln[base + aL] = l; Kn[base + aL] = (int)ls_median_to_first(E, cut, l, &o); Dn[base + aL] = d | (o << 8); }
                S.idx[tid] = (aL ? base : LS_INACT) | ((aR ? base + aL : LS_INACT) << 16);
                const int big = max(aL ? cut - f : 0, aR ? l - cut : 0);
                if (big) atomicMax(mx, big);
                const int lo = aL ? f : cut, hi = aR ? l : cut;       // positions of the active children
                if (hi > lo) {
                    const int c0 = lo >> 6, c1 = (hi - 1) >> 6;          // their chunks, a word at a time
                    for (int w = c0 >> 6; w <= c1 >> 6; w++) {
                        const int a0 = max(c0, w << 6) - (w << 6), a1 = min(c1, (w << 6) + 63) - (w << 6);
                        const unsigned long long mk = (a1 == 63 ? ~0ull : ((2ull << a1) - 1ull)) & ~((1ull << a0) - 1ull);
                        atomicOr(&actn[w], mk);
                    }
                }
            }
        }
        lds_barrier();
        ns = S.hdr[8 + (b ^ 1)];
        // this level's counter and active chunks reset for the level after next
        if (tid == 0) { S.hdr[8 + b] = 0; S.hdr[12 + b] = 0; }
        if (tid < 32) S.act[(b ? 32 : 0) + tid] = 0ull;
        LS_TS(5);
        b ^= 1;
        // the sparse tail: once at most one active segment per wave is left and each is short, the waves
        // finish them independently (no workgroup barriers per level)
        if (ns > 0 && ns <= W && S.hdr[12 + b] <= LS_TAIL) {
            if (wid < ns) {
                const int sf = ps_u(S.seg(b, 0)[wid]), sl = ps_u(S.seg(b, 1)[wid]), sd = ps_u(S.seg(b, 2)[wid]);
                PS_SAME({ const unsigned long long t_ = E[sf]; E[sf] = E[sf + (sd >> 8)]; E[sf + (sd >> 8)] = t_; });   // undo the median move
                ps_wsync<false>();
                ws_segment(E, sf, sl, sd & 0xff, S.rs, rel);
            }
            ns = 0;
        }
    }
    LS_TS(6);
    if (rel) {                              // the queued heap sorts, one wave each
        if (!first) lds_barrier();
        const int nh = min(S.hdr[6], LS_HQ);
        for (int i = wid; i < nh; i += W) {
            const int hf = ps_u(S.hq[2 * i]), hl2 = ps_u(S.hq[2 * i + 1]);
            // child flags in the heap's own part of RS_pos (2 bytes per position; the levels are over)
            if (ws_order_matters(E, hf, hl2, rel)) ws_heap_sort(E, hf, hl2, rel, (unsigned char*)S.rs + 2 * hf);
        }
    }
    // final insertion sort (stable, whole array): every element ranked inside its leaf (<= 16 elements
    // between consecutive boundaries; longer runs were heap-sorted and stay), segment bits cleared
    if (!first) lds_barrier();
    unsigned long long ev[CPW];
    int np[CPW];
#pragma unroll
    for (int i = 0; i < CPW; i++) {
        const int p = ((wid + i * W) << 6) + lane;
        np[i] = -1;
        if (p < n) {
            const unsigned long long e = E[p];
            ev[i] = e & ~0xffff0000ull;
            const int w = p >> 6, o = p & 63;
            const unsigned long long bw = S.bits[w];
            const unsigned long long below = bw & ((2ull << o) - 1ull);   // boundaries <= p
            const int f = below ? (w << 6) + ps_msb(below) : ((w - 1) << 6) + ps_msb(S.bits[w - 1] | 1ull);
            const unsigned long long above = bw & ~((2ull << o) - 1ull);
            int nxt;
            if (above) nxt = (w << 6) + __builtin_ctzll(above);
            else {
                const unsigned long long m2 = w + 1 < nc ? S.bits[w + 1] : 0ull;
                nxt = m2 ? ((w + 1) << 6) + __builtin_ctzll(m2) : 0x7fffffff;
            }
            nxt = min(nxt, n);
            int pos = p;
            if (nxt - f <= PS_THRESHOLD) {
                const unsigned kp = ps_key(e);
                unsigned kk[PS_THRESHOLD];
#pragma unroll
                for (int j = 0; j < PS_THRESHOLD; j++) kk[j] = ps_keyat(E, min(f + j, n - 1));
                pos = f;
#pragma unroll
                for (int j = 0; j < PS_THRESHOLD; j++) pos += f + j < nxt && (kk[j] < kp || (kk[j] == kp && f + j < p));
            }
            np[i] = pos;
        }
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < CPW; i++)
        if (np[i] >= 0) E[np[i]] = ev[i];
    lds_barrier();
    LS_TS(7);
}

// The sort of gE[0, n) in global memory (n <= NT * PS_MAX_CHUNK): pcl_sort.hpp's workgroup phase splits
// it level by level until every segment fits EL (cap <= NT * CPW elements of LDS), then each segment is
// copied into EL, sorted there by ls_sort from its remaining depth and copied back. scratch:
// ls_global_scratch_bytes(NT, cap) bytes of LDS; the split's scratch and ls_sort's share one region.
__host__ __device__ constexpr size_t ls_max(size_t a, size_t b) { return a > b ? a : b; }
__host__ __device__ constexpr size_t ls_global_scratch_bytes(int NT, int cap) {
    return 4 * (size_t)(16 + 3 * PS_GLIST) + ls_max(4 * (size_t)ps_scratch_ints(NT, cap, true), ls_scratch_bytes(NT, cap));
}
// Not inlined (its register pressure stays out of the callers' LDS paths); the LDS buffers are passed as
// LDS-address-space pointers so the body keeps ds_* accesses.
#ifdef PS_HOST_EMU
typedef unsigned long long lds_u64;
typedef unsigned char lds_u8;
#else
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
typedef __attribute__((address_space(3))) unsigned char lds_u8;
#endif
template <int NT, int CPW>
__device__ __noinline__ void ls_sort_global_lds(unsigned long long* gE, const int n, lds_u64* ELs, const int cap, lds_u8* scrs) {
    unsigned long long* EL = (unsigned long long*)ELs;
    unsigned char* scratch = (unsigned char*)scrs;
    const int tid = threadIdx.x;
    if (n <= 1) return;
    int* H = (int*)scratch;                 // [4] staged segments, [5] pending (the split's sink counters)
    int* GL = H + 16;                       // staged segments: f, l, depth + 1
    int* wsc = GL + 3 * PS_GLIST;           // the split's scratch, then ls_sort's
    if (tid < 16) { H[tid] = 0; wsc[tid] = 0; }
    for (int i = tid; i < 3 * PS_GLIST; i += NT) GL[i] = 0;
    int* Bf = wsc + 16 + 2 * (NT / WAVE) + 7 * (NT + 1);
    const int D0 = 2 * (31 - __builtin_clz((unsigned)n));
    __syncthreads();
    if (tid == 0) {
        if (n > cap) { Bf[0] = 0; Bf[PS_WGSEG] = n; Bf[2 * PS_WGSEG] = D0; wsc[0] = 1; }
        else { GL[0] = 0; GL[1] = n; GL[2] = D0 + 1; H[4] = 1; }
    }
    __syncthreads();
    if (n > cap) ps_wg_split<NT, true>(gE, n, wsc, cap, &H[4], &H[5], GL, PS_GLIST);
    __syncthreads();
    const int ns = min(ps_u(H[4]), PS_GLIST);
    for (int i = 0; i < ns; i++) {
        const int f = GL[3 * i], l = GL[3 * i + 1], d = GL[3 * i + 2] - 1;
        const int m = l - f;
        for (int t = tid; t < m; t += NT) EL[t] = gE[f + t];
        __syncthreads();
        ls_sort<NT, CPW>(EL, m, d, (unsigned char*)wsc, cap);
        for (int t = tid; t < m; t += NT) gE[f + t] = EL[t];
        __syncthreads();
    }
}
template <int NT, int CPW>
__device__ __forceinline__ void ls_sort_global(unsigned long long* gE, const int n, unsigned long long* EL, const int cap, unsigned char* scratch) {
    ls_sort_global_lds<NT, CPW>(gE, n, (lds_u64*)EL, cap, (lds_u8*)scratch);
}

// ---- sorts over several workgroups -------------------------------------------------------------------
// A large array is split by one workgroup (the workgroup phase of pcl_sort.hpp on global memory) until
// every segment has <= limit elements; the segment list goes to global memory (gseg: count, then f, l,
// depth + 1 per segment) and the segments are then sorted by other workgroups in parallel (ls_sort_list),
// each independent of the others (introsort's recursion below a partition only sees its own range).
constexpr int LS_SEGL = 1 + 3 * PS_GLIST;       // ints per segment list
__host__ __device__ constexpr size_t ls_split_scratch_bytes(int NT, int limit) {
    return 4 * (size_t)(16 + 3 * PS_GLIST) + 4 * (size_t)ps_scratch_ints(NT, limit, true);
}
template <int NT>
__device__ __noinline__ void ls_split_to_list_lds(unsigned long long* gE, const int n, const int limit, int* gseg, lds_u8* scrs,
                                                  const unsigned* rel) {
    int* H = (int*)(unsigned char*)scrs;
    int* GL = H + 16;
    int* wsc = GL + 3 * PS_GLIST;
    const int tid = threadIdx.x;
    if (tid < 16) { H[tid] = 0; wsc[tid] = 0; }
    for (int i = tid; i < 3 * PS_GLIST; i += NT) GL[i] = 0;
    int* Bf = wsc + 16 + 2 * (NT / WAVE) + 7 * (NT + 1);
    const int D0 = n > 1 ? 2 * (31 - __builtin_clz((unsigned)n)) : 0;
    __syncthreads();
    if (tid == 0) {
        if (n > limit) { Bf[0] = 0; Bf[PS_WGSEG] = n; Bf[2 * PS_WGSEG] = D0; wsc[0] = 1; }
        else if (n >= 2) { GL[0] = 0; GL[1] = n; GL[2] = D0 + 1; H[4] = 1; }
    }
    __syncthreads();
    if (n > limit) ps_wg_split<NT, true>(gE, n, wsc, limit, &H[4], &H[5], GL, PS_GLIST, rel);
    __syncthreads();
    const int ns = min(H[4], PS_GLIST);
    for (int i = tid; i < 3 * ns; i += NT) gseg[1 + i] = GL[i];
    if (tid == 0) gseg[0] = ns;
}
template <int NT>
__device__ __forceinline__ void ls_split_to_list(unsigned long long* gE, const int n, const int limit, int* gseg, unsigned char* scratch,
                                                 const unsigned* rel = nullptr) {
    ls_split_to_list_lds<NT>(gE, n, limit, gseg, (lds_u8*)scratch, rel);
}
// Workgroup w of nw: the list's segments of > 64 elements w, w + nw, ... (in list order, counting only
// those), each copied into EL (cap elements of LDS), sorted by ls_sort from its remaining depth, copied
// back; the <= 64-element ones one per wave (all waves of all nw workgroups), in registers in place.
template <int NT, int CPW>
__device__ __forceinline__ void ls_sort_list(unsigned long long* gE, const int* gseg, int w, int nw, unsigned long long* EL,
                                             const int cap, unsigned char* scratch, const unsigned* rel = nullptr) {
    const int tid = threadIdx.x, wid = tid / WAVE;
    const int ns = min(gseg[0], PS_GLIST);
    int big = 0, small = 0;
    for (int i = 0; i < ns; i++) {
        const int f = gseg[1 + 3 * i], l = gseg[2 + 3 * i], d = gseg[3 + 3 * i] - 1;
        const int m = l - f;
        if (m > WAVE) {
            if (big++ % nw != w) continue;
            for (int t = tid; t < m; t += NT) EL[t] = gE[f + t];
            __syncthreads();
            ls_sort<NT, CPW>(EL, m, d, scratch, cap, rel);
            for (int t = tid; t < m; t += NT) gE[f + t] = EL[t];
            __syncthreads();
        } else if (m >= 2) {
            if (small++ % (nw * (NT / WAVE)) != w * (NT / WAVE) + wid) continue;
            ws_small(gE, f, m, d, rel);
        }
    }
}

}  // namespace aloam
