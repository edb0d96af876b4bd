// tests/map_cache_check.cpp — the mapping rounds' candidate cache (csrc/k_map.hip MapCache) restated on the
// host and checked against the oracle's kd-tree 5-NN on a synthetic HDL-64 sequence (test infrastructure,
// built and run by tests/test_map_cache.py).
//
// Per stack point and round, as the device does: round 0 (and any round where the point left its cache)
// collects the points of the 3x3x3 block of its 1.025 m grid cell within 1 + M of the point (M = 0.1, at
// most 64, else no cache); a later round uses the cached list when the point moved at most M - eps and its
// 1 m ball (+ eps) lies inside the cached block, taking the 5 nearest within 1 m by (d2, index) from the
// list. Every round's answer must equal the whole-map 5-NN (laserMapping.cpp:582-584, 648-650): the same 5
// indices in the same order when the 5th is within 1 m, fewer than 5 found otherwise. The grid follows
// k_grid.hip grid_params (float bbox origin, cell 1.025 m, float cell index).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace mc {
template <class V, class T> void hook(int it, const double* par, const V& cs, const V& ss, const T& tc, const T& ts);
}
#define ORACLE_ROUND_HOOK(it, par, cs, ss, tc, ts) mc::hook(it, par, cs, ss, tc, ts)
#include "../oracle/aloam_oracle.cpp"

extern "C" {
struct synth_config { int model, n_azimuth; double range_sigma, max_range; unsigned long long seed; double speed, yaw_amp_deg; };
int synth_generate(const synth_config* cfg, int k, float* out, int max_pts);
}

namespace mc {
constexpr int CAP = 64;
constexpr float M = 0.1f, EPS = 2e-3f;
struct Grid {
    float ox, oy, oz, cell, inv;
    int dx, dy, dz;
    std::vector<std::vector<int>> cells;   // point indices per cell
};
static Grid build(const std::vector<orc::PtI>& p) {
    Grid g{};
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const auto& q : p) {
        const float c[3] = {q.x, q.y, q.z};
        for (int a = 0; a < 3; a++) { mn[a] = std::min(mn[a], c[a]); mx[a] = std::max(mx[a], c[a]); }
    }
    float cell = 1.0f * 1.025f;
    int dims[3];
    for (int it = 0; it < 64; it++) {
        long long prod = 1;
        for (int a = 0; a < 3; a++) {
            float ext = mx[a] - mn[a];
            if (!(ext >= 0.f)) ext = 0.f;
            dims[a] = (int)(ext / cell) + 2;
            prod *= dims[a];
        }
        if (prod <= (1 << 23)) break;
        cell *= 1.25f;
    }
    g.ox = mn[0]; g.oy = mn[1]; g.oz = mn[2]; g.cell = cell; g.inv = 1.0f / cell;
    g.dx = dims[0]; g.dy = dims[1]; g.dz = dims[2];
    g.cells.assign((size_t)g.dx * g.dy * g.dz, {});
    for (size_t i = 0; i < p.size(); i++) {
        const int cx = (int)floorf((p[i].x - g.ox) * g.inv), cy = (int)floorf((p[i].y - g.oy) * g.inv), cz = (int)floorf((p[i].z - g.oz) * g.inv);
        g.cells[((size_t)cz * g.dy + cy) * g.dx + cx].push_back((int)i);
    }
    return g;
}
static inline float sqd(const orc::PtI& a, float x, float y, float z) {
    const float dx = a.x - x, dy = a.y - y, dz = a.z - z;
    return dx * dx + dy * dy + dz * dz;
}
struct Cache { float cx, cy, cz; int n; std::vector<int> idx; };
static std::vector<Cache> cache;
static long queries = 0, cached = 0, mismatches = 0, overflow = 0;

static void collect(const Grid& g, const std::vector<orc::PtI>& p, float x, float y, float z, Cache& c) {
    c.cx = x; c.cy = y; c.cz = z; c.idx.clear();
    const int cx = (int)floorf((x - g.ox) * g.inv), cy = (int)floorf((y - g.oy) * g.inv), cz = (int)floorf((z - g.oz) * g.inv);
    const int x0 = std::max(cx - 1, 0), x1 = std::min(cx + 1, g.dx - 1);
    int n = 0;
    for (int r = 0; r < 9; r++) {
        const int yy = cy + r % 3 - 1, zz = cz + r / 3 - 1;
        if (x0 > x1 || yy < 0 || yy >= g.dy || zz < 0 || zz >= g.dz) continue;
        for (int xx = x0; xx <= x1; xx++)
            for (int i : g.cells[((size_t)zz * g.dy + yy) * g.dx + xx])
                if (sqd(p[i], x, y, z) < (1.0f + M) * (1.0f + M)) { if (n < CAP) c.idx.push_back(i); n++; }
    }
    c.n = n <= CAP ? n : -1;
    if (c.n < 0) overflow++;
}
static bool ball_in_block(const Grid& g, const Cache& c, float x, float y, float z) {
    auto axis = [&](float cv, float qv, float o, int d) {
        const int cc = (int)floorf((cv - o) * g.inv);
        const float lo = cc - 1 <= 0 ? -INFINITY : o + (float)(cc - 1) * g.cell;
        const float hi = cc + 2 >= d ? INFINITY : o + (float)(cc + 2) * g.cell;
        return qv - (1.0f + EPS) >= lo && qv + (1.0f + EPS) <= hi;
    };
    return axis(c.cx, x, g.ox, g.dx) && axis(c.cy, y, g.oy, g.dy) && axis(c.cz, z, g.oz, g.dz);
}
template <class V, class T> void hook(int it, const double* par, const V& cs, const V& ss, const T& tc, const T& ts) {
    static Grid gc, gs;
    if (it == 0) { gc = build(tc.pts); gs = build(ts.pts); cache.assign(cs.size() + ss.size(), Cache{}); }
    for (size_t q = 0; q < cs.size() + ss.size(); q++) {
        const bool corner = q < cs.size();
        const orc::PtI& po = corner ? cs[q] : ss[q - cs.size()];
        const T& t = corner ? tc : ts;
        const Grid& g = corner ? gc : gs;
        const orc::PtI sel = orc::associate_to_map(par, po);
        Cache& c = cache[q];
        bool use = false;
        if (it > 0 && c.n >= 0) {
            const float ex = sel.x - c.cx, ey = sel.y - c.cy, ez = sel.z - c.cz;
            use = ex * ex + ey * ey + ez * ez <= (M - EPS) * (M - EPS) && ball_in_block(g, c, sel.x, sel.y, sel.z);
        }
        int got[5], found = 0;
        float gd[5];
        if (use) {
            cached++;
            for (int k = 0; k < 5; k++) { got[k] = -1; gd[k] = INFINITY; }
            for (int i : c.idx) {            // the cached list: 5 nearest within 1 m by (d2, index)
                const float d = sqd(t.pts[i], sel.x, sel.y, sel.z);
                if (!(d < 1.0f)) continue;
                if (!(d < gd[4] || (d == gd[4] && i < got[4]))) continue;
                int p = 4;
                while (p > 0 && (d < gd[p - 1] || (d == gd[p - 1] && i < got[p - 1]))) { gd[p] = gd[p - 1]; got[p] = got[p - 1]; p--; }
                gd[p] = d; got[p] = i;
            }
            for (int k = 0; k < 5; k++) found += got[k] >= 0;
        } else {
            collect(g, t.pts, sel.x, sel.y, sel.z, c);   // the device searches the grid here (exact) and re-centres
        }
        queries++;
        if (!use) continue;
        int ki[5];
        float kd[5];
        t.knn(sel, 5, ki, kd);
        const bool valid = kd[4] < 1.0;
        bool same = valid ? found == 5 : found < 5;
        if (valid && same) for (int k = 0; k < 5; k++) same = same && got[k] == ki[k];
        if (!same) {
            mismatches++;
            if (mismatches <= 5) std::printf("mismatch round %d query %zu: found %d valid %d\n", it, q, found, (int)valid);
        }
    }
}
}  // namespace mc

int main(int argc, char** argv) {
    const int frames = argc > 1 ? atoi(argv[1]) : 20;
    aloam_params p{};
    p.scan_line = 64; p.minimum_range = 5.0f; p.mapping_skip_frame = 1; p.mapping_line_resolution = 0.4f;
    p.mapping_plane_resolution = 0.8f; p.input_is_dense = 1; p.odom_rounds = 10; p.map_rounds = 10; p.max_solver_iterations = 4;
    p.max_scan_points = 400000; p.max_map_points = 4000000;
    void* o = oracle_create(&p);
    synth_config cfg{64, 2083, 0.02, 120.0, 2, 1.0, 2.0};
    std::vector<float> buf(64 * 2083 * 4);
    for (int k = 0; k < frames; k++) {
        const int n = synth_generate(&cfg, k, buf.data(), 64 * 2083);
        oracle_process_scan(o, buf.data(), n, nullptr, nullptr);
    }
    std::printf("queries %ld cached %ld overflow %ld mismatches %ld\n", mc::queries, mc::cached, mc::overflow, mc::mismatches);
    oracle_destroy(o);
    return mc::mismatches != 0 || mc::cached == 0;
}
