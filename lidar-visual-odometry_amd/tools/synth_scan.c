/*
 * synth_scan.c — seeded procedural-urban-scene lidar simulator (SURVEY §8(d) "Synthetic inputs").
 *
 * There is no KITTI data on this machine or the GPU box, so every benchmark and parity input is a
 * seeded synthetic sweep written in the KITTI velodyne .bin layout (float32 x,y,z,reflectance per
 * point, src/kittiHelper.cpp:25-35). The scene: ground plane, building blocks on both sides of a
 * road (vertical edges at every block corner), street poles (r = 0.15 m cylinders), parked cars
 * (boxes). Ranges get N(0, sigma) noise and beam elevations / azimuths get continuous jitter so no
 * two points coincide (the reference's std::sort / FLANN tie orders never matter).
 *
 * Points are ordered ring-major, each ring sweeping clockwise (increasing -atan2(y,x)) from behind
 * the vehicle, like a Velodyne HDL-64 packet stream re-grouped by laser.
 *
 * Deterministic: plain C, doubles, no FMA contraction (-ffp-contract=off), own PRNG.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct synth_config {
    int    model;          /* 16 = VLP-16, 64 = HDL-64E, 128 = generic 128-line (-25..+15 deg) */
    int    n_azimuth;      /* azimuth steps per revolution */
    double range_sigma;    /* range noise (m) */
    double max_range;      /* m */
    unsigned long long seed;
    double speed;          /* m per frame along +x */
    double yaw_amp_deg;    /* yaw oscillation amplitude */
} synth_config;

typedef struct { double lo[3], hi[3]; } box_t;
typedef struct { double x, y, r, h; } pole_t;

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double urand(uint64_t* s) { return (splitmix(s) >> 11) * (1.0 / 9007199254740992.0); }
static double nrand(uint64_t* s) {
    double u1 = urand(s), u2 = urand(s);
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

/* ---- scene (built once per seed; world frame, z up, ground at z = 0) ---- */
#define MAXB 4096
#define MAXP 1024
static box_t  g_box[MAXB];
static int    g_nbox = 0;
static pole_t g_pole[MAXP];
static int    g_npole = 0;
static unsigned long long g_scene_seed = ~0ull;

static void build_scene(unsigned long long seed) {
    if (g_scene_seed == seed) return;
    g_scene_seed = seed;
    uint64_t s = seed * 7919ull + 17ull;
    g_nbox = 0; g_npole = 0;
    for (int side = -1; side <= 1; side += 2) {
        double x = -150.0;
        while (x < 1200.0 && g_nbox < MAXB - 8) {
            double len = 8.0 + 22.0 * urand(&s);
            double setback = 8.0 + 7.0 * urand(&s);
            double depth = 8.0 + 14.0 * urand(&s);
            double height = 5.0 + 20.0 * urand(&s);
            box_t b;
            b.lo[0] = x; b.hi[0] = x + len;
            if (side > 0) { b.lo[1] = setback; b.hi[1] = setback + depth; }
            else { b.lo[1] = -setback - depth; b.hi[1] = -setback; }
            b.lo[2] = 0.0; b.hi[2] = height;
            g_box[g_nbox++] = b;
            /* occasional protruding annex: more vertical/horizontal edges */
            if (urand(&s) < 0.4) {
                box_t a = b;
                double al = 3.0 + 5.0 * urand(&s);
                a.lo[0] = x + 0.3 * len; a.hi[0] = a.lo[0] + al;
                if (side > 0) { a.lo[1] = setback - 1.5 - 1.0 * urand(&s); a.hi[1] = setback + 0.01; }
                else { a.lo[1] = -setback - 0.01; a.hi[1] = -setback + 1.5 + 1.0 * urand(&s); }
                a.hi[2] = 3.0 + 2.0 * urand(&s);
                g_box[g_nbox++] = a;
            }
            x += len + 2.0 + 10.0 * urand(&s);
        }
        /* poles */
        double px = -140.0 + 10.0 * urand(&s);
        while (px < 1200.0 && g_npole < MAXP) {
            pole_t p; p.x = px; p.y = side * (6.0 + 0.8 * urand(&s)); p.r = 0.12 + 0.08 * urand(&s); p.h = 4.0 + 4.0 * urand(&s);
            g_pole[g_npole++] = p;
            px += 10.0 + 10.0 * urand(&s);
        }
        /* parked cars */
        double cx = -140.0;
        while (cx < 1200.0 && g_nbox < MAXB - 2) {
            if (urand(&s) < 0.55) {
                box_t c;
                double cl = 3.8 + 1.2 * urand(&s), cw = 1.7 + 0.3 * urand(&s);
                double cy = side * (3.8 + 0.6 * urand(&s));
                c.lo[0] = cx; c.hi[0] = cx + cl;
                c.lo[1] = cy - cw / 2; c.hi[1] = cy + cw / 2;
                c.lo[2] = 0.15; c.hi[2] = 1.3 + 0.4 * urand(&s);
                g_box[g_nbox++] = c;
            }
            cx += 6.0 + 6.0 * urand(&s);
        }
    }
}

/* vehicle pose of frame k: rotation (row-major 3x3) and sensor origin */
void synth_pose(const synth_config* cfg, int k, double R[9], double o[3]) {
    double yaw = cfg->yaw_amp_deg * M_PI / 180.0 * sin(k / 17.0);
    double pitch = 0.4 * M_PI / 180.0 * sin(k / 11.0 + 0.3);
    double roll = 0.3 * M_PI / 180.0 * sin(k / 7.0 + 1.1);
    double cy = cos(yaw), sy = sin(yaw), cp = cos(pitch), sp = sin(pitch), cr = cos(roll), sr = sin(roll);
    /* R = Rz(yaw) Ry(pitch) Rx(roll) */
    R[0] = cy * cp; R[1] = cy * sp * sr - sy * cr; R[2] = cy * sp * cr + sy * sr;
    R[3] = sy * cp; R[4] = sy * sp * sr + cy * cr; R[5] = sy * sp * cr - cy * sr;
    R[6] = -sp;     R[7] = cp * sr;                R[8] = cp * cr;
    o[0] = cfg->speed * k;
    o[1] = 0.6 * sin(k / 23.0);
    o[2] = 1.73 + 0.03 * sin(k / 5.0);
}

static int elevations(int model, double* el) {
    if (model == 16) { for (int i = 0; i < 16; i++) el[i] = -15.0 + 2.0 * i; return 16; }
    if (model == 64) {
        for (int i = 0; i < 32; i++) el[i] = 2.0 - i / 3.0;
        for (int i = 0; i < 32; i++) el[32 + i] = -8.83 - 0.5 * i;
        return 64;
    }
    int n = model;
    for (int i = 0; i < n; i++) el[i] = -25.0 + 40.0 * i / (n - 1);
    return n;
}

static double ray_cast(const double o[3], const double d[3], double max_range) {
    double best = max_range;
    if (d[2] < -1e-9) { double t = -o[2] / d[2]; if (t > 0 && t < best) best = t; }
    for (int b = 0; b < g_nbox; b++) {
        const box_t* B = &g_box[b];
        /* cheap reject: box far from origin in xy */
        double cxb = 0.5 * (B->lo[0] + B->hi[0]) - o[0];
        if (cxb > best + 40.0 || cxb < -best - 40.0) continue;
        double tn = -1e300, tf = 1e300;
        int miss = 0;
        for (int a = 0; a < 3; a++) {
            if (fabs(d[a]) < 1e-12) { if (o[a] < B->lo[a] || o[a] > B->hi[a]) { miss = 1; break; } continue; }
            double t1 = (B->lo[a] - o[a]) / d[a], t2 = (B->hi[a] - o[a]) / d[a];
            if (t1 > t2) { double tt = t1; t1 = t2; t2 = tt; }
            if (t1 > tn) tn = t1;
            if (t2 < tf) tf = t2;
            if (tn > tf) { miss = 1; break; }
        }
        if (miss || tf <= 0) continue;
        if (tn > 1e-6 && tn < best) best = tn;
    }
    for (int p = 0; p < g_npole; p++) {
        const pole_t* P = &g_pole[p];
        double ox = o[0] - P->x, oy = o[1] - P->y;
        if (ox > best + 2 || ox < -best - 2) continue;
        double A = d[0] * d[0] + d[1] * d[1];
        if (A < 1e-12) continue;
        double Bq = 2.0 * (ox * d[0] + oy * d[1]);
        double Cq = ox * ox + oy * oy - P->r * P->r;
        double disc = Bq * Bq - 4 * A * Cq;
        if (disc < 0) continue;
        double t = (-Bq - sqrt(disc)) / (2 * A);
        if (t <= 1e-6 || t >= best) continue;
        double z = o[2] + t * d[2];
        if (z < 0 || z > P->h) continue;
        best = t;
    }
    return best;
}

/* Generate frame k into out (float4 x,y,z,reflectance in the SENSOR frame). Returns point count. */
int synth_generate(const synth_config* cfg, int k, float* out, int max_pts) {
    build_scene(cfg->seed);
    double el[256];
    int nl = elevations(cfg->model, el);
    double R[9], o[3];
    synth_pose(cfg, k, R, o);
    uint64_t s = cfg->seed * 1000003ull + (uint64_t)k * 7777777ull + 12345ull;
    int n = 0;
    const int naz = cfg->n_azimuth;
    for (int l = 0; l < nl; l++) {
        double e0 = el[l] + 0.004 * (urand(&s) - 0.5);
        double a_off = urand(&s) * (2.0 * M_PI / naz);
        for (int j = 0; j < naz; j++) {
            double e = (e0 + 0.002 * (urand(&s) - 0.5)) * M_PI / 180.0;
            /* clockwise sweep starting behind the vehicle: azimuth pi - 2 pi j / naz */
            double a = M_PI - a_off - 2.0 * M_PI * (j + 0.25 * (urand(&s) - 0.5)) / naz;
            double ds[3] = {cos(e) * cos(a), cos(e) * sin(a), sin(e)};
            double dw[3] = {R[0] * ds[0] + R[1] * ds[1] + R[2] * ds[2],
                            R[3] * ds[0] + R[4] * ds[1] + R[5] * ds[2],
                            R[6] * ds[0] + R[7] * ds[1] + R[8] * ds[2]};
            double t = ray_cast(o, dw, cfg->max_range);
            double ns = nrand(&s);
            double refl = urand(&s);
            if (t >= cfg->max_range) continue;
            double r = t + cfg->range_sigma * ns;
            if (r <= 0.5) continue;
            if (n >= max_pts) return -1;
            out[4 * n + 0] = (float)(r * ds[0]);
            out[4 * n + 1] = (float)(r * ds[1]);
            out[4 * n + 2] = (float)(r * ds[2]);
            out[4 * n + 3] = (float)refl;
            n++;
        }
    }
    return n;
}

/* Dense surface map of the scene in the world frame (C4's "2M-pt local map"): samples the ground,
 * box faces and pole surfaces on a lattice of step `step` within a box around (cx,cy), with
 * N(0, noise) jitter. Returns the number of points (<= max_pts). */
int synth_dense_map(unsigned long long seed, double cx, double cy, double half, double step, double noise,
                    float* out, int max_pts) {
    build_scene(seed);
    uint64_t s = seed * 31337ull + 99ull;
    int n = 0;
#define EMIT(X, Y, Z) do { if (n >= max_pts) return n; out[4*n] = (float)((X) + noise * nrand(&s)); \
        out[4*n+1] = (float)((Y) + noise * nrand(&s)); out[4*n+2] = (float)((Z) + noise * nrand(&s)); out[4*n+3] = 0.f; n++; } while (0)
    /* ground */
    for (double x = cx - half; x < cx + half; x += step)
        for (double y = cy - half; y < cy + half; y += step) EMIT(x, y, 0.0);
    /* box faces (the 4 vertical faces and the top) */
    for (int b = 0; b < g_nbox; b++) {
        const box_t* B = &g_box[b];
        if (B->hi[0] < cx - half || B->lo[0] > cx + half || B->hi[1] < cy - half || B->lo[1] > cy + half) continue;
        for (double z = B->lo[2]; z < B->hi[2]; z += step) {
            for (double x = B->lo[0]; x < B->hi[0]; x += step) { EMIT(x, B->lo[1], z); EMIT(x, B->hi[1], z); }
            for (double y = B->lo[1]; y < B->hi[1]; y += step) { EMIT(B->lo[0], y, z); EMIT(B->hi[0], y, z); }
        }
        for (double x = B->lo[0]; x < B->hi[0]; x += step)
            for (double y = B->lo[1]; y < B->hi[1]; y += step) EMIT(x, y, B->hi[2]);
    }
    for (int p = 0; p < g_npole; p++) {
        const pole_t* P = &g_pole[p];
        if (P->x < cx - half || P->x > cx + half) continue;
        int na = (int)(2 * M_PI * P->r / step) + 3;
        for (double z = 0; z < P->h; z += step)
            for (int a = 0; a < na; a++) EMIT(P->x + P->r * cos(2 * M_PI * a / na), P->y + P->r * sin(2 * M_PI * a / na), z);
    }
#undef EMIT
    return n;
}
