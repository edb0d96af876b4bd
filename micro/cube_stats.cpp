// Analysis tool (not product code): statistics of the per-cube VoxelGrid inputs of laserMapping's map filter
// (src/laserMapping.cpp:788-801) over a synthetic HDL-64 sequence, from the oracle run with a compile-time hook.
// Per cube filter call: points, leaves by multiplicity (1, 2, >=3), whether the input is already one point per
// leaf in leaf order, and how libstdc++'s introsort treats it: elements that end in a heap-sorted segment, and
// whether any heap-sorted segment holds two or more points of a >=3-point leaf (the only case in which the heap
// sort's tie order can change a centroid's bits: a leaf sum from zero is commutative in its first two terms).
//
// build: g++ -O2 -std=c++17 -ffp-contract=off -I include -o /tmp/cube_stats micro/cube_stats.cpp \
//        lidar-visual-odometry_amd/tools/synth_scan.c -lm
// run:   /tmp/cube_stats FRAMES [report_every]
#include <cstdio>
#include <cstdlib>
#include <map>
#include <functional>
#include <vector>

struct PtI_;
namespace stats {
struct Acc {
    long calls = 0, pts = 0, leaves1 = 0, leaves2 = 0, leaves3 = 0, pts3 = 0, cubes_with3 = 0, cubes_sorted_unique = 0;
    long heap_elems = 0, heap_segs = 0, heap_calls = 0, heap_matter_calls = 0, heap_matter_segs = 0;
    long maxn = 0, heap_max = 0, matter_max = 0;
    long part_full = 0, part_pruned = 0, depth_full = 0, depth_pruned = 0;   // elements partitioned; max recursion depth
    long heap_steps_full = 0, heap_steps_pruned = 0, heap_steps_max_full = 0, heap_steps_max_pruned = 0;
    long sw_pops = 0, sw_max = 0, sw_segs = 0, sw_ok = 0, sw_bad = 0, es_pops = 0, es_max = 0;   // safe-switch analysis
    long po_segs = 0, po_grab = 0, po_ok = 0, po_bad = 0, po_grab_g = 0, po_safe = 0, po_safe_ok = 0, po_noown = 0, po_noown_ok = 0;   // post-order closed form checks
    long seg_safe_small = 0, seg_safe_big = 0, seg_unsafe = 0, pops_safe_small = 0, pops_safe_big = 0, pops_unsafe = 0, pops_safe_big_max = 0, pops_unsafe_max = 0;
};
Acc acc[5], frame_acc[5];
template <class V> void hook(const V& in, float leaf, int kind);
}  // namespace stats
#define ORACLE_CUBE_HOOK(arr, leaf, kind) stats::hook(arr, leaf, kind)
#include "../oracle/aloam_oracle.cpp"

extern "C" {
struct synth_config { int model, n_azimuth; double range_sigma, max_range; unsigned long long seed; double speed, yaw_amp_deg; };
int synth_generate(const synth_config* cfg, int k, float* out, int max_pts);
}

namespace stats {
// heap sort of [f, l) with the closed-form prediction for the relevant groups: after make_heap, every key
// group's pop order (ties go to the right child in __adjust_heap) is the (node, right, left) pre-order of its
// members' positions, so their final order is the (left, right, node) post-order -- exact as long as no
// element >= the group's key is taken as the re-inserted `value` (a "grab") before the group is popped.
template <class T, class Less>
static void heap_sort_check(T* first, T* last, Less less, const std::map<unsigned, int>& rel, Acc& A) {
    const long len = last - first;
    // make_heap
    if (len >= 2) { long parent = (len - 2) / 2; while (true) { T v = first[parent]; orc::adjust_heap(first, parent, len, v, less); if (parent == 0) break; parent--; } }
    const std::vector<T> hcopy(first, first + len);
    // conservative no-grab check per group: no member of G in the last c_G slots after make_heap
    std::map<unsigned, bool> safe;
    for (auto& kv : rel) {
        long cg = 0;
        for (long p = 0; p < len; p++) cg += first[p].idx >= kv.first;
        bool ok = true;
        for (long p = len - cg; p < len; p++) ok = ok && first[p].idx != kv.first;
        safe[kv.first] = ok;
    }
    // post-order positions per relevant group
    std::map<unsigned, std::vector<unsigned>> pred;
    std::function<void(long)> post = [&](long x) {
        if (x >= len) return;
        post(2 * x + 1); post(2 * x + 2);
        if (rel.count(first[x].idx)) pred[first[x].idx].push_back(first[x].ci);
    };
    post(0);
    // sort_heap with grab detection per group
    std::map<unsigned, bool> grabbed, grabbed_own;
    unsigned kmin = ~0u;
    for (auto& kv : rel) kmin = std::min(kmin, kv.first);
    long cmin = 0;
    for (long p = 0; p < len; p++) cmin += first[p].idx >= kmin;
    long tgrabs = 0;
    long l = len;
    while (l > 1) {
        --l;
        T v = first[l];
        if (len - 1 - l < cmin && v.idx >= kmin) tgrabs++;
        for (auto& kv : rel) if (v.idx == kv.first) grabbed_own[kv.first] = true;
        for (auto& kv : rel) if (v.idx >= kv.first) {
            // grab of an element >= K before group K is fully popped: group K still has members in [0, l)?
            bool left = false;
            for (long p = 0; p < l; p++) left = left || first[p].idx == kv.first;
            if (left) grabbed[kv.first] = true;
        }
        first[l] = first[0];
        orc::adjust_heap(first, 0L, l, v, less);
    }
    A.po_segs++;
    {   // segment-level closed form (ws_heap_postorder: every relevant group safe) by length, with its early-stop pops
        bool all = true;
        for (auto& kv : rel) all = all && safe[kv.first];
        const long pops = std::min(len - 1, cmin);
        if (all && len <= 1024) { A.seg_safe_small++; A.pops_safe_small += pops; }
        else if (all) { A.seg_safe_big++; A.pops_safe_big += pops; A.pops_safe_big_max = std::max(A.pops_safe_big_max, pops); }
        else { A.seg_unsafe++; A.pops_unsafe += pops; A.pops_unsafe_max = std::max(A.pops_unsafe_max, pops); }
    }
    // safe-switch analysis (a device design's prototype): pops until no relevant group has a member in its
    // danger window [len - c_G, h) (the window start stays fixed while G is popped: every pop takes an element
    // >= K_G and shrinks the heap by one), then the post-order closed form of the CURRENT heap for the rest.
    // Counts the pops simulated before the switch against the early-stop count, and checks the prediction.
    {
        std::vector<T> H(hcopy.begin(), hcopy.end());
        std::map<unsigned, long> wG;
        for (auto& kv : rel) { long cg = 0; for (long p = 0; p < len; p++) cg += H[p].idx >= kv.first; wG[kv.first] = len - cg; }
        long h = len, isafe = -1;
        for (long i = 0; h > 1; i++) {
            bool danger = false;
            for (long p = 0; p < h && !danger; p++) {
                auto it = wG.find(H[p].idx);
                if (it != wG.end() && p >= it->second) danger = true;
            }
            if (!danger) { isafe = i; break; }
            --h; T v = H[h]; H[h] = H[0]; orc::adjust_heap(H.data(), 0L, h, v, less);
        }
        if (isafe < 0) isafe = len - 1;
        isafe = std::min(isafe, std::min(len - 1, cmin));     // never more than the early stop's pops
        A.sw_pops += isafe; A.sw_max = std::max(A.sw_max, isafe); A.sw_segs++;
        A.es_pops += std::min(len - 1, cmin); A.es_max = std::max(A.es_max, std::min(len - 1, cmin));
        // prediction: members still in [0, h) in post-order of their slots, then the popped ones in slot order
        std::map<unsigned, std::vector<unsigned>> pr;
        std::function<void(long)> post2 = [&](long x) {
            if (x >= h) return;
            post2(2 * x + 1); post2(2 * x + 2);
            if (rel.count(H[x].idx)) pr[H[x].idx].push_back(H[x].ci);
        };
        post2(0);
        for (long p = h; p < len; p++) if (rel.count(H[p].idx)) pr[H[p].idx].push_back(H[p].ci);
        for (auto& kv : rel) {
            std::vector<unsigned> got;
            for (long p = 0; p < len; p++) if (first[p].idx == kv.first) got.push_back(first[p].ci);
            if (got == pr[kv.first]) A.sw_ok++; else A.sw_bad++;
        }
    }
    bool anyg = false;
    for (auto& kv : rel) {
        std::vector<unsigned> got;
        for (long p = 0; p < len; p++) if (first[p].idx == kv.first) got.push_back(first[p].ci);
        if (safe[kv.first]) { A.po_safe++; if (got == pred[kv.first]) A.po_safe_ok++; }
        if (!grabbed_own[kv.first]) { A.po_noown++; if (got == pred[kv.first]) A.po_noown_ok++; }
        if (grabbed[kv.first]) { A.po_grab_g++; anyg = true; continue; }
        if (got == pred[kv.first]) A.po_ok++; else A.po_bad++;
    }
    A.po_grab += anyg;
    if (getenv("CS_TGRAB")) printf("TGRAB len %ld cmin %ld grabs %ld\n", len, cmin, tgrabs);
}
// Relevance-pruned VoxelGrid (prototype of the device design): the leaf sums need PCL's order only inside
// leaves of >= 3 points ("relevant"); an introsort segment holding fewer than 2 relevant points is dropped
// from the replay, and each relevant point's position when its segment is dropped / becomes a <= 16 leaf /
// is heap-sorted orders it among its leaf's points.
static long g_rvg_calls = 0, g_rvg_bad = 0;
template <class V> static void rvg_check(const V& in, float leaf) {
    using orc::PtI;
    const size_t n = in.size();
    if (n == 0) return;
    std::vector<PtI> ref;
    orc::voxel_grid(std::vector<PtI>(in.begin(), in.end()), leaf, ref, 1);
    const float inv = 1.0f / leaf;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (const auto& p : in) { float c[3] = {p.x, p.y, p.z}; for (int d = 0; d < 3; d++) { mn[d] = std::min(mn[d], c[d]); mx[d] = std::max(mx[d], c[d]); } }
    int minb[3], maxb[3], divb[3];
    for (int d = 0; d < 3; d++) { minb[d] = (int)std::floor(mn[d] * inv); maxb[d] = (int)std::floor(mx[d] * inv); divb[d] = maxb[d] - minb[d] + 1; }
    const int mul1 = divb[0], mul2 = divb[0] * divb[1];
    struct IV { unsigned idx; unsigned ci; };
    std::vector<IV> iv(n);
    for (size_t i = 0; i < n; i++) {
        int i0 = (int)(std::floor(in[i].x * inv) - (float)minb[0]);
        int i1 = (int)(std::floor(in[i].y * inv) - (float)minb[1]);
        int i2 = (int)(std::floor(in[i].z * inv) - (float)minb[2]);
        iv[i] = {(unsigned)(i0 + i1 * mul1 + i2 * mul2), (unsigned)i};
    }
    // R2: order-free grouping
    std::vector<IV> srt = iv;
    std::stable_sort(srt.begin(), srt.end(), [](const IV& a, const IV& b) { return a.idx < b.idx; });
    std::vector<char> rel(n, 0);
    for (size_t i = 0; i < n;) { size_t j = i; while (j < n && srt[j].idx == srt[i].idx) j++; if (j - i >= 3) for (size_t k = i; k < j; k++) rel[srt[k].ci] = 1; i = j; }
    // R3: pruned replay; pos[ci] = final ordering position of relevant points
    std::vector<long> pos(n, -1);
    std::vector<IV> w = iv;
    auto less = [](const IV& a, const IV& b) { return a.idx < b.idx; };
    auto nrel = [&](IV* f, IV* l) { int c = 0; for (IV* p = f; p < l; p++) c += rel[p->ci]; return c; };
    auto record = [&](IV* f, IV* l) { for (IV* p = f; p < l; p++) if (rel[p->ci]) pos[p->ci] = p - w.data(); };
    std::function<void(IV*, IV*, long)> rec = [&](IV* first, IV* last, long depth) {
        while (last - first > 16) {
            if (nrel(first, last) < 2) { record(first, last); return; }
            if (depth == 0) { orc::heap_sort(first, last, less); record(first, last); return; }
            --depth;
            IV* mid = first + (last - first) / 2;
            orc::move_median_to_first(first, first + 1, mid, last - 1, less);
            IV* cut = orc::unguarded_partition(first + 1, last, first, less);
            rec(cut, last, depth);
            last = cut;
        }
        record(first, last);   // a <= 16 leaf: the final insertion sort keeps equal keys in position order
    };
    long lg = 63 - __builtin_clzl((unsigned long)n);
    rec(w.data(), w.data() + n, lg * 2);
    // R4: centroids in key order
    std::vector<PtI> out;
    for (size_t i = 0; i < n;) {
        size_t j = i; while (j < n && srt[j].idx == srt[i].idx) j++;
        std::vector<unsigned> mem;
        for (size_t k = i; k < j; k++) mem.push_back(srt[k].ci);
        if (j - i >= 3) std::sort(mem.begin(), mem.end(), [&](unsigned a, unsigned b) { return pos[a] < pos[b]; });
        float c[4] = {0.f, 0.f, 0.f, 0.f};
        for (unsigned ci : mem) { const PtI& p = in[ci]; c[0] += p.x; c[1] += p.y; c[2] += p.z; c[3] += p.intensity; }
        const float cnt = (float)(j - i);
        out.push_back({c[0] / cnt, c[1] / cnt, c[2] / cnt, c[3] / cnt});
        i = j;
    }
    g_rvg_calls++;
    if (out.size() != ref.size() || std::memcmp(out.data(), ref.data(), out.size() * sizeof(PtI)) != 0) g_rvg_bad++;
}
// introsort replica with instrumentation: records the heap-sorted segments
struct HS { long f, l; };
static std::vector<HS> g_heaps;
template <class T, class Less>
static void introsort_loop_i(T* base, T* first, T* last, long depth, Less less) {
    while (last - first > 16) {
        if (depth == 0) { g_heaps.push_back({first - base, last - base}); orc::heap_sort(first, last, less); return; }
        --depth;
        T* mid = first + (last - first) / 2;
        orc::move_median_to_first(first, first + 1, mid, last - 1, less);
        T* cut = orc::unguarded_partition(first + 1, last, first, less);
        introsort_loop_i(base, cut, last, depth, less);
        last = cut;
    }
}
template <class V> void hook(const V& in, float leaf, int kind) {
    using orc::PtI;
    const size_t n = in.size();
    if (n == 0) return;
    const float inv = 1.0f / leaf;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (const auto& p : in) { float c[3] = {p.x, p.y, p.z}; for (int d = 0; d < 3; d++) { mn[d] = std::min(mn[d], c[d]); mx[d] = std::max(mx[d], c[d]); } }
    int minb[3], maxb[3], divb[3];
    for (int d = 0; d < 3; d++) { minb[d] = (int)std::floor(mn[d] * inv); maxb[d] = (int)std::floor(mx[d] * inv); divb[d] = maxb[d] - minb[d] + 1; }
    const int mul1 = divb[0], mul2 = divb[0] * divb[1];
    struct IV { unsigned idx; unsigned ci; };
    std::vector<IV> iv(n);
    for (size_t i = 0; i < n; i++) {
        int i0 = (int)(std::floor(in[i].x * inv) - (float)minb[0]);
        int i1 = (int)(std::floor(in[i].y * inv) - (float)minb[1]);
        int i2 = (int)(std::floor(in[i].z * inv) - (float)minb[2]);
        iv[i] = {(unsigned)(i0 + i1 * mul1 + i2 * mul2), (unsigned)i};
    }
    bool uniq_sorted = true;
    for (size_t i = 1; i < n; i++) uniq_sorted = uniq_sorted && iv[i - 1].idx < iv[i].idx;
    std::map<unsigned, int> mult;
    for (auto& e : iv) mult[e.idx]++;
    Acc& A = frame_acc[kind];
    A.calls++; A.pts += n; A.maxn = std::max<long>(A.maxn, n);
    bool any3 = false;
    for (auto& kv : mult) {
        if (kv.second == 1) A.leaves1++; else if (kv.second == 2) A.leaves2++; else { A.leaves3++; A.pts3 += kv.second; any3 = true; }
    }
    A.cubes_with3 += any3; A.cubes_sorted_unique += uniq_sorted;
    g_heaps.clear();
    auto less = [](const IV& a, const IV& b) { return a.idx < b.idx; };
    long lg = 63 - __builtin_clzl((unsigned long)n);
    introsort_loop_i(iv.data(), iv.data(), iv.data() + n, lg * 2, less);
    if (!g_heaps.empty()) A.heap_calls++;
    bool matter = false;
    for (auto& h : g_heaps) {
        A.heap_segs++; A.heap_elems += h.l - h.f; A.heap_max = std::max(A.heap_max, h.l - h.f);
        std::map<unsigned, int> in_seg;
        for (long p = h.f; p < h.l; p++) if (mult[iv[p].idx] >= 3) in_seg[iv[p].idx]++;
        bool m = false;
        for (auto& kv : in_seg) m = m || kv.second >= 2;
        A.heap_matter_segs += m; matter = matter || m; if (m) A.matter_max = std::max(A.matter_max, h.l - h.f);
    }
    A.heap_matter_calls += matter;
    if (getenv("CS_RVG")) rvg_check(in, leaf);
    // pruned replay: a segment needs its exact order only if it holds >= 2 members of a >= 3-point leaf at group
    // ranks where the sum's order matters (not just the group's first two); heap sorts stop after the last
    // relevant group is popped
    {
        std::vector<IV> w(n);
        for (size_t i = 0; i < n; i++) w[i] = {0, (unsigned)i};
        for (size_t i = 0; i < n; i++) w[i].idx = 0;
        // recompute keys in the input order
        std::vector<unsigned> key(n);
        for (size_t i = 0; i < n; i++) {
            int i0 = (int)(std::floor(in[i].x * inv) - (float)minb[0]);
            int i1 = (int)(std::floor(in[i].y * inv) - (float)minb[1]);
            int i2 = (int)(std::floor(in[i].z * inv) - (float)minb[2]);
            key[i] = (unsigned)(i0 + i1 * mul1 + i2 * mul2);
            w[i] = {key[i], (unsigned)i};
        }
        long full_work = 0, pr_work = 0, dfull = 0, dpr = 0, hs_full = 0, hs_pr = 0;
        std::map<unsigned, int> before;   // unused
        auto relevant = [&](IV* f, IV* l, IV* base) {
            std::map<unsigned, int> c;
            for (IV* p = f; p < l; p++) if (mult[p->idx] >= 3) c[p->idx]++;
            for (auto& kv : c) {
                if (kv.second < 2) continue;
                if (kv.second >= 3) return true;
                // exactly 2 here: their group ranks = members before f + 1, + 2 (segments partition by key)
                int b = 0;
                for (IV* p = base; p < f; p++) b += p->idx == kv.first;
                if (b >= 1) return true;
            }
            return false;
        };
        std::function<void(IV*, IV*, long, int, bool)> rec = [&](IV* first, IV* last, long depth, int lev, bool prune_on) {
            while (last - first > 16) {
                bool rel = relevant(first, last, w.data());
                if (depth == 0) {
                    long m = last - first, lg2 = 64 - __builtin_clzl((unsigned long)m);
                    hs_full += m * lg2 * 3 / 2;
                    if (rel) {
                        unsigned kmin = ~0u;
                        std::map<unsigned, int> c;
                        for (IV* p = first; p < last; p++) if (mult[p->idx] >= 3) c[p->idx]++;
                        for (auto& kv : c) if (kv.second >= 2) kmin = std::min(kmin, kv.first);
                        long pops = 0;
                        for (IV* p = first; p < last; p++) pops += p->idx >= kmin;
                        hs_pr += m / 2 * 2 + pops * lg2;
                        if (getenv("CS_HEAPS")) {
                            std::map<unsigned, int> dk;
                            for (IV* p = first; p < last; p++) dk[p->idx]++;
                            int ng = 0, nm = 0, mx = 0, ge3 = 0;
                            for (auto& kv : c) if (kv.second >= 2) { ng++; nm += kv.second; }
                            for (auto& kv : dk) { mx = std::max(mx, kv.second); ge3 += kv.second >= 2; }
                            long below = 0;   // segment elements below the smallest relevant key
                            for (IV* p = first; p < last; p++) below += p->idx < kmin;
                            // refined: a group with exactly 2 points here and none of its points before the
                            // segment has them as its leaf's first two terms (commutative): order free
                            unsigned kref = ~0u;
                            for (auto& kv : c) {
                                if (kv.second < 2) continue;
                                int before = 0;
                                for (IV* p = w.data(); p < first; p++) before += p->idx == kv.first;
                                if (kv.second >= 3 || before >= 1) kref = std::min(kref, kv.first);
                            }
                            long pref = 0;
                            for (IV* p = first; p < last; p++) pref += kref != ~0u && p->idx >= kref;
                            printf("HEAP kind %d m %ld pops %ld n %zu groups %d members %d distinct %zu dupkeys %d maxmult %d below %ld refined_pops %ld\n",
                                   kind, m, pops, n, ng, nm, dk.size(), ge3, mx, below, pref);
                        }
                        std::map<unsigned, int> relg;
                        for (auto& kv : c) if (kv.second >= 2) relg[kv.first] = kv.second;
                        heap_sort_check(first, last, less, relg, A);
                        return;
                    }
                    orc::heap_sort(first, last, less);
                    return;
                }
                --depth;
                full_work += last - first;
                if (rel) pr_work += last - first;
                dfull = std::max<long>(dfull, lev + 1);
                if (rel) dpr = std::max<long>(dpr, lev + 1);
                IV* mid = first + (last - first) / 2;
                orc::move_median_to_first(first, first + 1, mid, last - 1, less);
                IV* cut = orc::unguarded_partition(first + 1, last, first, less);
                rec(cut, last, depth, lev + 1, prune_on);
                last = cut;
                lev++;
            }
        };
        rec(w.data(), w.data() + n, lg * 2, 0, true);
        A.part_full += full_work; A.part_pruned += pr_work;
        A.depth_full = std::max(A.depth_full, dfull); A.depth_pruned = std::max(A.depth_pruned, dpr);
        A.heap_steps_full += hs_full; A.heap_steps_pruned += hs_pr;
        A.heap_steps_max_full = std::max(A.heap_steps_max_full, hs_full); A.heap_steps_max_pruned = std::max(A.heap_steps_max_pruned, hs_pr);
    }
}
}  // namespace stats

int main(int argc, char** argv) {
    const int frames = argc > 1 ? atoi(argv[1]) : 60;
    const int every = argc > 2 ? atoi(argv[2]) : 20;
    aloam_params p{};
    p.scan_line = 64; p.minimum_range = 5.0f; p.mapping_skip_frame = 1; p.mapping_line_resolution = 0.4f;
    p.mapping_plane_resolution = 0.8f; p.input_is_dense = 1; p.odom_rounds = 10; p.map_rounds = 10; p.max_solver_iterations = 4;
    p.max_scan_points = 400000; p.max_map_points = 4000000;
    void* o = oracle_create(&p);
    oracle_set_voxel_order(o, 1);
    synth_config cfg{64, 2083, 0.02, 120.0, 2, 1.0, 2.0};
    std::vector<float> buf(64 * 2083 * 4);
    for (int k = 0; k < frames; k++) {
        int n = synth_generate(&cfg, k, buf.data(), 64 * 2083);
        for (auto& a : stats::frame_acc) a = stats::Acc{};
        if (getenv("CS_HEAPS")) printf("FRAME %d\n", k);
        oracle_process_scan(o, buf.data(), n, nullptr, nullptr);
        for (int w = 0; w < 5; w++) {
            auto& a = stats::frame_acc[w];
            auto& t = stats::acc[w];
            t.calls += a.calls; t.pts += a.pts; t.leaves1 += a.leaves1; t.leaves2 += a.leaves2; t.leaves3 += a.leaves3; t.pts3 += a.pts3;
            t.cubes_with3 += a.cubes_with3; t.cubes_sorted_unique += a.cubes_sorted_unique; t.heap_elems += a.heap_elems;
            t.heap_segs += a.heap_segs; t.heap_calls += a.heap_calls; t.heap_matter_calls += a.heap_matter_calls;
            t.part_full += a.part_full; t.part_pruned += a.part_pruned; t.depth_full = std::max(t.depth_full, a.depth_full);
            t.depth_pruned = std::max(t.depth_pruned, a.depth_pruned); t.heap_steps_full += a.heap_steps_full; t.heap_steps_pruned += a.heap_steps_pruned;
            t.heap_steps_max_full = std::max(t.heap_steps_max_full, a.heap_steps_max_full); t.heap_steps_max_pruned = std::max(t.heap_steps_max_pruned, a.heap_steps_max_pruned);
            t.po_safe += a.po_safe; t.po_safe_ok += a.po_safe_ok; t.po_noown += a.po_noown; t.po_noown_ok += a.po_noown_ok;
            t.po_segs += a.po_segs; t.po_grab += a.po_grab; t.po_ok += a.po_ok; t.po_bad += a.po_bad; t.po_grab_g += a.po_grab_g;
            t.sw_pops += a.sw_pops; t.sw_max = std::max(t.sw_max, a.sw_max); t.sw_segs += a.sw_segs; t.sw_ok += a.sw_ok; t.sw_bad += a.sw_bad;
            t.es_pops += a.es_pops; t.es_max = std::max(t.es_max, a.es_max);
            t.seg_safe_small += a.seg_safe_small; t.seg_safe_big += a.seg_safe_big; t.seg_unsafe += a.seg_unsafe;
            t.pops_safe_small += a.pops_safe_small; t.pops_safe_big += a.pops_safe_big; t.pops_unsafe += a.pops_unsafe;
            t.pops_safe_big_max = std::max(t.pops_safe_big_max, a.pops_safe_big_max); t.pops_unsafe_max = std::max(t.pops_unsafe_max, a.pops_unsafe_max);
            t.heap_matter_segs += a.heap_matter_segs; t.maxn = std::max(t.maxn, a.maxn); t.heap_max = std::max(t.heap_max, a.heap_max); t.matter_max = std::max(t.matter_max, a.matter_max);
            if ((k + 1) % every == 0)
                printf("frame %3d %s: cubes %ld (unique-sorted %ld, with >=3 leaf %ld, heap %ld, heap-order-matters %ld) pts %ld max %ld | "
                       "leaves 1:%ld 2:%ld >=3:%ld (pts in >=3: %ld) | heap elems %ld segs %ld (matter %ld)\n",
                       k, w ? "surf  " : "corner", a.calls, a.cubes_sorted_unique, a.cubes_with3, a.heap_calls, a.heap_matter_calls, a.pts,
                       a.maxn, a.leaves1, a.leaves2, a.leaves3, a.pts3, a.heap_elems, a.heap_segs, a.heap_matter_segs);
        }
    }
    static const char* NM[5] = {"corner", "surf  ", "stk-c ", "stk-s ", "lines "};
    for (int w = 0; w < 5; w++) {
        auto& t = stats::acc[w];
        printf("TOTAL %s: cubes %ld (unique-sorted %ld, with >=3 %ld, heap %ld, heap-order-matters %ld) pts %ld max %ld | leaves 1:%ld 2:%ld >=3:%ld pts3 %ld | heap elems %ld segs %ld matter %ld | heap max %ld matter max %ld\n",
               NM[w], t.calls, t.cubes_sorted_unique, t.cubes_with3, t.heap_calls, t.heap_matter_calls, t.pts, t.maxn,
               t.leaves1, t.leaves2, t.leaves3, t.pts3, t.heap_elems, t.heap_segs, t.heap_matter_segs, t.heap_max, t.matter_max);
    }
    for (int w = 0; w < 5; w++) {
        auto& t = stats::acc[w];
        printf("PRUNE %s: partition work full %ld pruned %ld | depth full %ld pruned %ld | heap steps full %ld (max/cube %ld) pruned %ld (max/cube %ld)\n",
               NM[w], t.part_full, t.part_pruned, t.depth_full, t.depth_pruned, t.heap_steps_full, t.heap_steps_max_full,
               t.heap_steps_pruned, t.heap_steps_max_pruned);
        printf("POSTORDER %s: relevant heap segments %ld (with a grab %ld) | groups predicted ok %ld wrong %ld grabbed %ld | safe %ld (post-order right %ld) | no own-member grab %ld (right %ld)\n",
               NM[w], t.po_segs, t.po_grab, t.po_ok, t.po_bad, t.po_grab_g, t.po_safe, t.po_safe_ok, t.po_noown, t.po_noown_ok);
        printf("SWITCH %s: relevant heap segments %ld | pops: early stop %ld (max %ld), safe switch %ld (max %ld) | prediction right %ld wrong %ld\n",
               NM[w], t.sw_segs, t.es_pops, t.es_max, t.sw_pops, t.sw_max, t.sw_ok, t.sw_bad);
        printf("SEGSAFE %s: all groups safe, <= 1024: %ld segs %ld pops | all safe, > 1024: %ld segs %ld pops (max %ld) | unsafe: %ld segs %ld pops (max %ld)\n",
               NM[w], t.seg_safe_small, t.pops_safe_small, t.seg_safe_big, t.pops_safe_big, t.pops_safe_big_max, t.seg_unsafe, t.pops_unsafe,
               t.pops_unsafe_max);
    }
    if (getenv("CS_RVG")) printf("RVG: %ld cube filters, %ld differ from PCL order\n", stats::g_rvg_calls, stats::g_rvg_bad);
    oracle_destroy(o);
    return 0;
}
