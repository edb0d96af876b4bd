// aloam_kitti — headless C++ host of the hot path: a KITTI velodyne sequence through the native
// pipeline (scanRegistration -> laserOdometry -> laserMapping) via the C ABI only, the way a ROS node
// shim would call it (SURVEY §8(b) "a headless benchmark driver calls the same ABI directly").
//
// Replaces the reference's kittiHelper player + the three nodes for offline runs
// (src/kittiHelper.cpp:25-35,130-151 read the .bin files; the nodes publish /aft_mapped_to_init).
// Output: one line per scan with the mapped pose as a KITTI 3x4 row-major [R|t] (the format of
// kittiHelper's ground-truth path), to stdout or -o FILE; a timing summary on stderr. Optional:
//   --map-path FILE   the /aft_mapped_path Path (laserMapping.cpp:866-873): every mapped pose appended,
//                     one "index tx ty tz qx qy qz qw" line each (TUM layout, the scan index as stamp)
//   --odom-path FILE  the /laser_odom_path Path (laserOdometry.cpp:598-607), same layout
//   --hf FILE         /aft_mapped_to_init_high_frec (laserMapping.cpp:218-246): each odometry pose mapped
//                     through the latest q/t_wmap_wodom (aloam_map_high_freq_pose), same layout
//
// usage: aloam_kitti [-l scan_line] [-s stages] [-n max_frames] [-o poses.txt] [--map-path F] [--odom-path F]
//                    [--hf F] file0.bin file1.bin ...
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "aloam_hip.h"

static bool read_bin(const char* path, std::vector<float>& out) {   // kittiHelper.cpp:25-35
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long bytes = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize((size_t)bytes / sizeof(float));
    const size_t got = std::fread(out.data(), sizeof(float), out.size(), f);
    std::fclose(f);
    return got == out.size() && out.size() % 4 == 0;
}

static void write_pose(FILE* o, const double q[4], const double t[3]) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
                         2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                         2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)};
    std::fprintf(o, "%.9e %.9e %.9e %.9e %.9e %.9e %.9e %.9e %.9e %.9e %.9e %.9e\n", R[0], R[1], R[2], t[0], R[3], R[4],
                 R[5], t[1], R[6], R[7], R[8], t[2]);
}

static void write_tum(FILE* o, long index, const double q[4], const double t[3]) {
    if (o) std::fprintf(o, "%ld %.9e %.9e %.9e %.12e %.12e %.12e %.12e\n", index, t[0], t[1], t[2], q[0], q[1], q[2], q[3]);
}

static FILE* open_out(const char* path) {
    if (!path) return nullptr;
    FILE* f = std::fopen(path, "w");
    if (!f) { std::perror(path); std::exit(1); }
    return f;
}

int main(int argc, char** argv) {
    int scan_line = 64, stages = 2, max_frames = -1;
    const char* out_path = nullptr;
    const char *map_path = nullptr, *odom_path = nullptr, *hf_path = nullptr;
    std::vector<const char*> files;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "-l") && i + 1 < argc) scan_line = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "-s") && i + 1 < argc) stages = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "-n") && i + 1 < argc) max_frames = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "-o") && i + 1 < argc) out_path = argv[++i];
        else if (!std::strcmp(argv[i], "--map-path") && i + 1 < argc) map_path = argv[++i];
        else if (!std::strcmp(argv[i], "--odom-path") && i + 1 < argc) odom_path = argv[++i];
        else if (!std::strcmp(argv[i], "--hf") && i + 1 < argc) hf_path = argv[++i];
        else files.push_back(argv[i]);
    }
    if (files.empty()) {
        std::fprintf(stderr, "usage: %s [-l scan_line] [-s stages] [-n max_frames] [-o poses.txt] [--map-path F] [--odom-path F] "
                             "[--hf F] scans.bin...\n", argv[0]);
        return 2;
    }
    if (max_frames >= 0 && (size_t)max_frames < files.size()) files.resize(max_frames);
    aloam_params p;
    aloam_default_params(&p, scan_line);
    aloam_pipeline* pl = aloam_pipeline_create(&p, 0, stages);
    if (!pl) {
        std::fprintf(stderr, "aloam_pipeline_create failed: %s\n", aloam_last_error(nullptr));
        return 1;
    }
    FILE* o = out_path ? std::fopen(out_path, "w") : stdout;
    if (!o) { std::perror(out_path); return 1; }
    FILE *fmap = open_out(map_path), *fodom = open_out(odom_path), *fhf = open_out(hf_path);
    // the mapping stage's context holds q/t_wmap_wodom (the last context of the pipeline)
    aloam_ctx* mctx = aloam_pipeline_context(pl, stages >= 2 ? 1 : 0);
    std::vector<float> bufs[2];     // a pushed sweep is read until the next push returns: alternate buffers
    size_t mapped = 0, pushed = 0;
    long odom_n = 0;
    double busy_s = 0;
    auto on_odom = [&](const aloam_odom_result& r) {
        write_tum(fodom, odom_n, r.q_w_curr, r.t_w_curr);
        if (fhf) {                  // laserMapping's odometry callback: the pose in the map frame right away
            double q[4], t[3];
            if (aloam_map_high_freq_pose(mctx, r.q_w_curr, r.t_w_curr, q, t) == ALOAM_OK) write_tum(fhf, odom_n, q, t);
        }
        odom_n++;
    };
    auto on_map = [&](const aloam_map_result& r) {
        write_pose(o, r.q_w_curr, r.t_w_curr);
        write_tum(fmap, (long)mapped, r.q_w_curr, r.t_w_curr);   // the Path grows by one pose per mapped scan
        mapped++;
    };
    for (const char* path : files) {
        std::vector<float>& pts = bufs[pushed++ & 1];
        if (!read_bin(path, pts)) {
            std::fprintf(stderr, "cannot read %s\n", path);
            return 1;
        }
        aloam_odom_result od;
        aloam_map_result mp;
        int have_od = 0, have_mp = 0;
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = aloam_pipeline_push(pl, pts.data(), (int)(pts.size() / 4), 0, &od, &have_od, &mp, &have_mp);
        busy_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (rc) {
            std::fprintf(stderr, "%s: rc=%d %s\n", path, rc, aloam_pipeline_last_error(pl));
            return 1;
        }
        if (have_od) on_odom(od);
        if (have_mp) on_map(mp);
    }
    aloam_odom_result od;
    aloam_map_result mp, mp2;
    for (;;) {                      // until nothing is left in flight
        int ho = 0, hm = 0, hm2 = 0;
        if (aloam_pipeline_flush(pl, &od, &ho, &mp, &hm, &mp2, &hm2)) {
            std::fprintf(stderr, "flush: %s\n", aloam_pipeline_last_error(pl));
            return 1;
        }
        if (ho) on_odom(od);
        if (hm) on_map(mp);
        if (hm2) on_map(mp2);
        if (!ho && !hm && !hm2) break;
    }
    if (o != stdout) std::fclose(o);
    for (FILE* f : {fmap, fodom, fhf}) if (f) std::fclose(f);
    aloam_pipeline_destroy(pl);
    std::fprintf(stderr, "aloam_kitti: %zu scans, %zu mapped poses, %.3f ms/scan (incl. .bin upload)\n", files.size(),
                 mapped, 1e3 * busy_s / files.size());
    return 0;
}
