// rvg.hpp — PCL VoxelGrid leaf sums with PCL's order only where it can change a bit ("relevance").
//
// pcl::VoxelGrid::applyFilter (PCL 1.8.0) sums every leaf's points from zero in the order an unstable
// libstdc++ std::sort by leaf leaves them (src/scanRegistration.cpp:401-405, src/laserMapping.cpp:542-550,
// 788-801). fp32 addition is commutative, so ((0 + a) + b) == ((0 + b) + a) bit for bit: the sort's tie
// order changes a centroid only for leaves of three or more points. The filter therefore runs in three
// parts:
//   R2  an order-free sort S of the (leaf, point) pairs: the leaves in key order (PCL's output order), their
//       sizes, and `rel`, one bit per point of a >= 3-point leaf;
//   R3  only when some leaf is relevant: the exact replay of std::sort (ls_sort.hpp), where a depth-exhausted
//       segment is heap-sorted only if it holds two or more relevant points (pcl_sort.hpp
//       ps_order_matters); afterwards every relevant point's position orders it inside its leaf (segments
//       are ordered by key, and inside one only the exact parts' order is used);
//   R4  the sums: a leaf of <= 2 points in S's order, a relevant one in R3 position order.
// Checked against the oracle's PCL order (std::sort replica) by the VoxelGrid / mapping parity tests; the
// equivalence itself on every cube filter of a 60-frame sequence by micro/cube_stats.cpp (CS_RVG=1).
#pragma once
#include "pcl_sort.hpp"

namespace aloam {

__device__ __forceinline__ bool rvg_is_rel(const unsigned* rel, unsigned i) { return (rel[i >> 5] >> (i & 31u)) & 1u; }

// S (n pairs sorted by key, any tie order) -> rel bits (zeroed by the caller) for the points of >= 3-point
// leaves; *nrel (zeroed by the caller) += their count. Position q lies in such a leaf exactly when one of the
// three windows of 3 around it is constant; S is sorted, so a window is constant when its ends are equal:
// key[q-2] == key[q], key[q-1] == key[q+1] or key[q] == key[q+2]. One position per lane, consecutive lanes
// on consecutive positions (S in global memory: coalesced, no dependent loads; the leaf-walking form spent
// ~45 us of dependent loads on a 16k-point cube).
template <int NT>
__device__ __forceinline__ void rvg_mark(const unsigned long long* S, const int n, unsigned* rel, int* nrel) {
    int mine = 0;
    for (int q = threadIdx.x; q < n; q += NT) {
        const unsigned k = ps_keyat(S, q);
        const unsigned km2 = q >= 2 ? ps_keyat(S, q - 2) : ~k, km1 = q >= 1 ? ps_keyat(S, q - 1) : 0u;
        const unsigned kp1 = q + 1 < n ? ps_keyat(S, q + 1) : 0u, kp2 = q + 2 < n ? ps_keyat(S, q + 2) : ~k;
        const bool r = km2 == k || (q >= 1 && q + 1 < n && km1 == kp1) || kp2 == k;
        if (r) {
            const unsigned i = (unsigned)S[q] & 0xffffu;
            atomicOr(&rel[i >> 5], 1u << (i & 31u));
            mine++;
        }
    }
    mine = wave_sum_i(mine);
    if (lane_id() == 0 && mine) atomicAdd(nrel, mine);
}

// The same marks as bytes, relB[point] = 0 / 1 (every point's byte written, S holds each point once), for S and
// relB in global memory: plain byte stores instead of contended atomics on the bit words; rvg_pack_bits then
// builds the bit words (after a workgroup barrier). relB: 16-byte aligned, n + 31 bytes writable (the bytes
// from n up to the next multiple of 32 are zeroed here, so every byte rvg_pack_bits reads is exactly 0 or 1:
// its 4-bytes-to-4-bits fold relies on that; split cubes pass the 8 n + 512-byte rvg_T region).
template <int NT>
__device__ __forceinline__ void rvg_mark_bytes(const unsigned long long* S, const int n, unsigned char* relB, int* nrel) {
    if (threadIdx.x < (unsigned)(((n + 31) & ~31) - n)) relB[n + threadIdx.x] = 0;
    int mine = 0;
    for (int q0 = threadIdx.x; q0 < n; q0 += 4 * NT) {     // 4 positions per lane in flight
        unsigned kk[4][5], pi[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = q0 + u * NT;
#pragma unroll
            for (int d = 0; d < 5; d++) kk[u][d] = q + d - 2 >= 0 && q + d - 2 < n ? ps_keyat(S, q + d - 2) : 0xffffffffu - (unsigned)d;
            pi[u] = q < n ? (unsigned)S[q] & 0xffffu : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int q = q0 + u * NT;
            if (q >= n) continue;
            // (out-of-range neighbours hold distinct sentinels no key window can match with its ends)
            const bool r = kk[u][0] == kk[u][2] || (q >= 1 && q + 1 < n && kk[u][1] == kk[u][3]) || kk[u][4] == kk[u][2];
            relB[pi[u]] = r ? 1 : 0;
            mine += r;
        }
    }
    mine = wave_sum_i(mine);
    if (lane_id() == 0 && mine) atomicAdd(nrel, mine);
}
template <int NT>
__device__ __forceinline__ void rvg_pack_bits(const unsigned char* relB, const int n, unsigned* rel) {
    const int nw = (n + 31) >> 5;
    for (int w = threadIdx.x; w < nw; w += NT) {
        const unsigned* src = (const unsigned*)__builtin_assume_aligned(relB + 32 * (size_t)w, 16);
        unsigned x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = src[u];
        unsigned m = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) m |= ((x[u] | x[u] >> 7 | x[u] >> 14 | x[u] >> 21) & 0xfu) << (4 * u);   // bytes 0 / 1 -> 4 bits
        const int valid = n - 32 * w;
        rel[w] = valid >= 32 ? m : m & ((1u << valid) - 1u);
    }
}

// the final array E of the exact replay -> fpos[point] = position, for the relevant points
// (8 positions per thread in flight: E, then the relevance words, then the stores)
template <int NT>
__device__ __forceinline__ void rvg_positions(const unsigned long long* E, const int n, const unsigned* rel, int* fpos) {
    for (int p0 = threadIdx.x; p0 < n; p0 += 8 * NT) {
        unsigned i[8], w[8];
#pragma unroll
        for (int u = 0; u < 8; u++) i[u] = p0 + u * NT < n ? (unsigned)E[p0 + u * NT] & 0xffffu : 0u;
#pragma unroll
        for (int u = 0; u < 8; u++) w[u] = p0 + u * NT < n ? rel[i[u] >> 5] : 0u;
#pragma unroll
        for (int u = 0; u < 8; u++)
            if ((w[u] >> (i[u] & 31u)) & 1u) fpos[i[u]] = p0 + u * NT;
    }
}

// One relevant leaf S[q, e) (len >= 3) summed in fpos order (up to 16 points by a register sorting network,
// more by repeated selection).
template <typename PtF>
__device__ __forceinline__ float4 rvg_rel_sum(const unsigned long long* S, const int q, const int e, const int* fpos, PtF pt) {
    const int len = e - q;
    float4 cc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [&](unsigned i) {
        const float4 v = pt((int)i);
        cc.x += v.x; cc.y += v.y; cc.z += v.z; cc.w += v.w;
    };
    if (len <= 16) {
        unsigned v[16];                  // (position << 16) | point, sorted ascending = position order
#pragma unroll
        for (int u = 0; u < 16; u++) {
            const unsigned i = u < len ? ((unsigned)S[q + u] & 0xffffu) : 0u;
            v[u] = u < len ? (((unsigned)fpos[i] << 16) | i) : 0xffffffffu;
        }
#pragma unroll
        for (int r = 0; r < 16; r++) {   // odd-even transposition network
#pragma unroll
            for (int u = r & 1; u + 1 < 16; u += 2) {
                const unsigned a = v[u], b = v[u + 1];
                v[u] = a < b ? a : b;
                v[u + 1] = a < b ? b : a;
            }
        }
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (u < len) add(v[u] & 0xffffu);
    } else {
        int last = -1;
        for (int m = 0; m < len; m++) {
            int best = 0x7fffffff;
            unsigned bi = 0;
            for (int t = q; t < e; t++) {
                const unsigned i = (unsigned)S[t] & 0xffffu;
                const int fp = fpos[i];
                if (fp > last && fp < best) { best = fp; bi = i; }
            }
            add(bi);
            last = best;
        }
    }
    return cc;
}

// The same leaf sums with the thread's chunk read in batches of RB entries: the batch's S entries and
// their points are loaded together (independent loads in flight) and the leaves summed from registers
// in S order; a relevant leaf (rel bit at its head, its points then in fpos order) and a leaf running
// past the chunk take the per-leaf path. Same sums in the same order as rvg_reduce's loop.
template <int NT, int RB, typename PtF, typename OutF>
__device__ __forceinline__ int rvg_reduce_batched(const unsigned long long* S, const int n, const unsigned* rel, const int* fpos,
                                                  PtF pt, OutF out, int* sc) {
    const int C = (n + NT - 1) / NT;
    const int q0 = min(n, (int)threadIdx.x * C), q1 = min(n, q0 + C);
    int nh = 0;
    for (int qb = q0; qb < q1; qb += RB) {
        unsigned k[RB];
        const unsigned kp = qb > 0 ? ps_key(S[qb - 1]) : 0u;
#pragma unroll
        for (int j = 0; j < RB; j++) k[j] = qb + j < q1 ? ps_key(S[qb + j]) : 0u;
#pragma unroll
        for (int j = 0; j < RB; j++)
            if (qb + j < q1) nh += (qb + j == 0 || k[j] != (j ? k[j - 1] : kp));
    }
    int run = nh, dummy = 0, tot, td;
    ps_exscan2<NT>(run, dummy, sc, tot, td);
    // the open leaf: its head, whether it is summed here (a <= 2-point leaf) and the sum so far
    int head = -1;
    bool plain = false;
    float4 cc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto close = [&](int e) {            // the open leaf ends at e
        const int len = e - head;
        if (!plain) cc = rvg_rel_sum(S, head, e, fpos, pt);
        out(run, div4_by_count(cc, len));
        run++;
    };
    for (int qb = q0; qb < q1; qb += RB) {
        unsigned long long s[RB];
        float4 v[RB];
        const unsigned kp = qb > 0 ? ps_key(S[qb - 1]) : 0u;
#pragma unroll
        for (int j = 0; j < RB; j++) s[j] = qb + j < q1 ? S[qb + j] : 0ull;
#pragma unroll
        for (int j = 0; j < RB; j++) v[j] = qb + j < q1 ? pt((int)((unsigned)s[j] & 0xffffu)) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < RB; j++) {
            const int q = qb + j;
            if (q >= q1) continue;
            const unsigned kj = ps_key(s[j]);
            if (q == 0 || kj != (j ? ps_key(s[j - 1]) : kp)) {   // a leaf starts at q
                if (head >= 0) close(q);
                head = q;
                plain = !rvg_is_rel(rel, (unsigned)s[j] & 0xffffu);
                cc = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            if (head >= 0 && plain) { cc.x += v[j].x; cc.y += v[j].y; cc.z += v[j].z; cc.w += v[j].w; }
        }
    }
    if (head >= 0) {                     // the last leaf may run into the next chunk
        int e = q1;
        const unsigned kh = ps_key(S[head]);
        while (e < n && ps_key(S[e]) == kh) {
            if (plain) { const float4 w = pt((int)((unsigned)S[e] & 0xffffu)); cc.x += w.x; cc.y += w.y; cc.z += w.z; cc.w += w.w; }
            e++;
        }
        close(e);
    }
    return tot;
}

// Leaf sums: thread t owns the leaves starting in its chunk of S; out(r, centroid) for the r-th leaf in key
// order; returns the number of leaves (all threads). A relevant leaf's points are added in fpos order.
// fpos == null: S is PCL's order itself (every leaf summed in S order; payloads are then full 32-bit point
// indices). sc: 2 (NT / 64) + 2 ints of LDS. This is the leaf-at-a-time form (the exact mode's path, and
// the batched form's reference in tests/ps_emu.cpp).
template <int NT, typename PtF, typename OutF>
__device__ __forceinline__ int rvg_reduce_loop(const unsigned long long* S, const int n, const unsigned* rel, const int* fpos, PtF pt,
                                               OutF out, int* sc) {
    const bool exact = fpos == nullptr;
    const unsigned pm = exact ? 0xffffffffu : 0xffffu;
    const int C = (n + NT - 1) / NT;
    const int q0 = min(n, (int)threadIdx.x * C), q1 = min(n, q0 + C);
    int nh = 0;
    for (int q = q0; q < q1; q++) nh += (q == 0 || ps_key(S[q]) != ps_key(S[q - 1]));
    int run = nh, dummy = 0, tot, td;
    ps_exscan2<NT>(run, dummy, sc, tot, td);
    for (int q = q0; q < q1; q++) {
        const unsigned k = ps_key(S[q]);
        if (q > 0 && ps_key(S[q - 1]) == k) continue;
        int e = q + 1;
        while (e < n && ps_key(S[e]) == k) e++;
        const int len = e - q;
        float4 cc = make_float4(0.f, 0.f, 0.f, 0.f);
        auto add = [&](unsigned i) {
            const float4 v = pt((int)i);
            cc.x += v.x; cc.y += v.y; cc.z += v.z; cc.w += v.w;
        };
        if (len < 3 || exact) {
            for (int t = q; t < e; t++) add((unsigned)S[t] & pm);
        } else if (len <= 16) {
            unsigned v[16];                  // (position << 16) | point, sorted ascending = position order
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const unsigned i = u < len ? ((unsigned)S[q + u] & 0xffffu) : 0u;
                v[u] = u < len ? (((unsigned)fpos[i] << 16) | i) : 0xffffffffu;
            }
#pragma unroll
            for (int r = 0; r < 16; r++) {   // odd-even transposition network
#pragma unroll
                for (int u = r & 1; u + 1 < 16; u += 2) {
                    const unsigned a = v[u], b = v[u + 1];
                    v[u] = a < b ? a : b;
                    v[u + 1] = a < b ? b : a;
                }
            }
#pragma unroll
            for (int u = 0; u < 16; u++)
                if (u < len) add(v[u] & 0xffffu);
        } else {
            int last = -1;
            for (int m = 0; m < len; m++) {
                int best = 0x7fffffff;
                unsigned bi = 0;
                for (int t = q; t < e; t++) {
                    const unsigned i = (unsigned)S[t] & 0xffffu;
                    const int fp = fpos[i];
                    if (fp > last && fp < best) { best = fp; bi = i; }
                }
                add(bi);
                last = best;
            }
        }
        out(run, div4_by_count(cc, len));
        run++;
    }
    return tot;
}

// BATCHED: the batched form (S in global memory and registers to spare, k_rb_cubered); else the loop
// (S in LDS, or a kernel whose other phases already fill the 1024-thread register budget)
template <int NT, bool BATCHED = false, typename PtF, typename OutF>
__device__ __forceinline__ int rvg_reduce(const unsigned long long* S, const int n, const unsigned* rel, const int* fpos, PtF pt,
                                          OutF out, int* sc) {
    if (BATCHED && fpos) return rvg_reduce_batched<NT, 8>(S, n, rel, fpos, pt, out, sc);
    return rvg_reduce_loop<NT>(S, n, rel, fpos, pt, out, sc);
}

}  // namespace aloam
