/*
 * aloam_hip.h — C ABI of the MI355X-native A-LOAM per-scan hot path.
 *
 * This is the drop-in boundary: plain C types, host pointers + sizes, no torch
 * or HIP types in any signature. Every entry point replaces an inline hot block
 * of the reference's three ROS nodes (reference = ucmmesa/Lidar-Visual-Odometry,
 * an A-LOAM fork; citations are path:line relative to its repo root):
 *
 *   aloam_scan_registration  ->  src/scanRegistration.cpp:114-411   (laserCloudHandler body)
 *   aloam_odometry           ->  src/laserOdometry.cpp:331-641      (main-loop body, incl. 10x Ceres solve)
 *   aloam_mapping            ->  src/laserMapping.cpp:305-848       (process() body, incl. 10x Ceres solve)
 *   aloam_factor (+ eval)    ->  src/lidarFactor.hpp:12-172         (LidarEdge/Plane/PlaneNorm/Distance factors)
 *
 * Threading: one caller thread per context, synchronous calls,
 * one HIP stream per context. Several contexts may coexist in one process.
 *
 * Errors: 0 = ok, < 0 = error (ALOAM_E_*); aloam_last_error() has the text.
 * The reference's soft conditions are NOT errors: "less correspondence!"
 * (laserOdometry.cpp:566-568) still solves, and a too-small map skips the
 * solve (laserMapping.cpp:554,730-733); both are reported in the result structs.
 */
#ifndef ALOAM_HIP_H
#define ALOAM_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define ALOAM_ABI_VERSION 7

/* error codes */
#define ALOAM_OK             0
#define ALOAM_E_ARG         -1   /* bad argument (NULL pointer, negative size)            */
#define ALOAM_E_CAPACITY    -2   /* input larger than the capacity given at create time   */
#define ALOAM_E_HIP         -3   /* HIP runtime error                                      */
#define ALOAM_E_SCAN_LINES  -4   /* scan_line not in {16,32,64} and generic rule not opted in
                                    (reference aborts: scanRegistration.cpp:201-205,472-476) */
#define ALOAM_E_STATE       -5   /* call out of order (e.g. odometry before any features)  */
#define ALOAM_E_NODEVICE    -6   /* no HIP device / extension unusable                     */

/* flags for aloam_scan_registration */
#define ALOAM_INPUT_DEVICE   1   /* xyzr points at device memory (already resident in HBM) */

/* Launch parameters (launch/aloam_velodyne_*.launch) and the reference's
 * hard-coded constants, which are kept overridable for tests. */
typedef struct aloam_params {
    int   scan_line;                /* scanRegistration.cpp:466 "scan_line" (16/32/64)              */
    float minimum_range;            /* scanRegistration.cpp:468 "minimum_range"                     */
    int   mapping_skip_frame;       /* laserOdometry.cpp:274   "mapping_skip_frame"                 */
    float mapping_line_resolution;  /* laserMapping.cpp:902    "mapping_line_resolution"            */
    float mapping_plane_resolution; /* laserMapping.cpp:903    "mapping_plane_resolution"           */
    int   input_is_dense;           /* PointCloud2 is_dense: 1 => removeNaNFromPointCloud is a copy */
    int   generic_scan_lines;       /* opt-in linear elevation->line rule for other line counts    */
    float generic_min_elev_deg;     /*   lowest beam elevation (deg) for the generic rule          */
    float generic_max_elev_deg;     /*   highest beam elevation (deg)                              */
    int   odom_rounds;              /* laserOdometry.cpp:364  (10 in this fork)                    */
    int   map_rounds;               /* laserMapping.cpp:562   (10 in this fork)                    */
    int   max_solver_iterations;    /* laserOdometry.cpp:573 / laserMapping.cpp:715 (4)            */
    int   max_scan_points;          /* capacity: raw points per scan                               */
    int   max_map_points;           /* capacity: points of corner+surf map                         */
} aloam_params;

/* A point cloud in caller-owned host memory: n points of float4 (x,y,z,intensity)
 * = pcl::PointXYZI without its padding (include/aloam_velodyne/common.h:43). */
typedef struct aloam_cloud {
    float* pts;   /* n*4 floats                                   */
    int    n;     /* [out] number of points written               */
    int    cap;   /* [in]  capacity of pts in points              */
} aloam_cloud;

/* Outputs of scanRegistration (the five topics, scanRegistration.cpp:413-441). */
typedef struct aloam_features {
    aloam_cloud full;        /* /velodyne_cloud_2       (laserCloud, line-ordered)      */
    aloam_cloud sharp;       /* /laser_cloud_sharp                                      */
    aloam_cloud less_sharp;  /* /laser_cloud_less_sharp                                 */
    aloam_cloud flat;        /* /laser_cloud_flat                                       */
    aloam_cloud less_flat;   /* /laser_cloud_less_flat  (per-line VoxelGrid 0.2 m)      */
    int*   sharp_idx;        /* optional (may be NULL): index into full of each sharp  */
    int*   less_sharp_idx;   /* optional: index into full of each less_sharp           */
    int*   flat_idx;         /* optional: index into full of each flat                 */
    float* curvature;        /* optional: full.n floats; entries outside [5,n-5) are 0 */
} aloam_features;

/* Ceres-equivalent solve summary of one outer round. */
typedef struct aloam_lm_summary {
    int    iterations;         /* LM iterations executed (<= max_solver_iterations)  */
    int    successful_steps;
    int    termination;        /* 0 max-iter, 1 function tol, 2 param tol, 3 gradient tol, 4 no residuals, 5 invalid steps */
    int    num_residual_blocks;
    double initial_cost;
    double final_cost;
} aloam_lm_summary;

#define ALOAM_MAX_ROUNDS 16

/* laserOdometry result (/laser_odom_to_init, laserOdometry.cpp:588-598). */
typedef struct aloam_odom_result {
    double q_w_curr[4];        /* x,y,z,w  (Eigen coeff order)                        */
    double t_w_curr[3];
    double q_last_curr[4];     /* para_q (laserOdometry.cpp:131)                       */
    double t_last_curr[3];     /* para_t                                               */
    int    optimized;          /* 0 on the initialising frame (laserOdometry.cpp:355)  */
    int    rounds;
    int    corner_correspondence[ALOAM_MAX_ROUNDS];
    int    plane_correspondence[ALOAM_MAX_ROUNDS];
    aloam_lm_summary lm[ALOAM_MAX_ROUNDS];
    int    publish_to_mapping;  /* frameCount % skipFrameNum == 0 (laserOdometry.cpp:643) */
} aloam_odom_result;

/* laserMapping result (/aft_mapped_to_init, laserMapping.cpp:854-865). */
typedef struct aloam_map_result {
    double q_w_curr[4];
    double t_w_curr[3];
    int    optimized;           /* 0 if the map was too small (laserMapping.cpp:554)   */
    int    map_corner_num;      /* laserCloudCornerFromMapNum                          */
    int    map_surf_num;        /* laserCloudSurfFromMapNum                            */
    int    corner_stack_num;
    int    surf_stack_num;
    int    rounds;
    int    corner_num[ALOAM_MAX_ROUNDS];
    int    surf_num[ALOAM_MAX_ROUNDS];
    aloam_lm_summary lm[ALOAM_MAX_ROUNDS];
    int    map_total_points;    /* all cubes, corner + surf                            */
    /* the odometry -> map correction after this frame's transformUpdate (laserMapping.cpp:148-152),
     * which /aft_mapped_to_init_high_frec applies to every later odometry pose (:197-229) */
    double q_wmap_wodom[4];
    double t_wmap_wodom[3];
    int    frame_count;         /* frameCount of this frame: mapping frames processed before it      */
    int    pub_surround;        /* frameCount % 5 == 0: /laser_cloud_surround is published (:806)     */
    int    pub_map;             /* frameCount % 20 == 0: /laser_cloud_map is published (:823)         */
    int    uncached_queries;    /* stack points beyond the rounds' candidate-cache slots (65,536): they
                                 * search the map grid in every round (exact, slower); 0 on HDL-64       */
} aloam_map_result;

/* One residual block of lidarFactor.hpp, flattened.
 *  type 0 LidarEdgeFactor      (lidarFactor.hpp:12-55):  cp, a = last_point_a, b = last_point_b
 *  type 1 LidarPlaneFactor     (lidarFactor.hpp:57-104): cp, a = last_point_j, b = ljm_norm (unit)
 *  type 2 LidarPlaneNormFactor (lidarFactor.hpp:106-138): cp, a = plane_unit_norm, b[0] = negative_OA_dot_norm
 *  type 3 LidarDistanceFactor  (lidarFactor.hpp:141-172): cp, a = closed_point
 * s (interpolation ratio) is 1 on the whole hot path (DISTORTION 0, laserOdometry.cpp:67). */
typedef struct aloam_factor {
    int    type;
    int    pad;
    double cp[3];
    double a[3];
    double b[3];
} aloam_factor;

/* ---- context ---------------------------------------------------------------------- */
typedef struct aloam_ctx aloam_ctx;

void        aloam_default_params(aloam_params* p, int scan_line);
aloam_ctx*  aloam_create(const aloam_params* p, int device);
void        aloam_destroy(aloam_ctx* ctx);
const char* aloam_last_error(const aloam_ctx* ctx);
int         aloam_abi_version(void);

/* ---- stage 1: scanRegistration (scanRegistration.cpp:114-411) ---------------------- */
/* xyzr: n points of float4 (x,y,z,reflectance) = KITTI .bin / PointCloud2 of PointXYZ(I).
 * The features stay resident in the context for aloam_odometry(); fetch them with
 * aloam_get_features(). */
int aloam_scan_registration(aloam_ctx* ctx, const float* xyzr, int n, int flags);
/* The same from a sensor_msgs/PointCloud2 data blob as the /velodyne_points callback receives it
 * (scanRegistration.cpp:114,131-133): n records of point_step bytes (multiple of 4, >= 12) with
 * float32 x, y, z at byte offsets 0, 4, 8 (pcl::PointXYZ / PointXYZI / velodyne XYZIR layouts;
 * 16 = KITTI .bin, 32 = pcl::PointXYZI). Other fields are ignored, as by pcl::fromROSMsg into the
 * reference's PointXYZ cloud. Host blob, or device blob with ALOAM_INPUT_DEVICE. */
int aloam_scan_registration_pc2(aloam_ctx* ctx, const void* data, int n, int point_step, int flags);
int aloam_feature_counts(aloam_ctx* ctx, int counts[5]); /* full, sharp, less_sharp, flat, less_flat */
int aloam_get_features(aloam_ctx* ctx, aloam_features* out);

/* ---- stage 2: laserOdometry (laserOdometry.cpp:331-641) ---------------------------- */
/* Consumes the features produced by the last aloam_scan_registration(). */
int aloam_odometry(aloam_ctx* ctx, aloam_odom_result* out);
/* Teacher-forcing input: load features from host clouds (float4 x,y,z,intensity),
 * replacing the ones aloam_scan_registration() left in the context. */
int aloam_set_features(aloam_ctx* ctx,
                       const float* sharp, int n_sharp, const float* less_sharp, int n_less_sharp,
                       const float* flat, int n_flat, const float* less_flat, int n_less_flat);
/* Overwrite the odometry state (warm start para_q/para_t, pose, last clouds). */
int aloam_set_odom_state(aloam_ctx* ctx, const double q_last_curr[4], const double t_last_curr[3],
                         const double q_w_curr[4], const double t_w_curr[3],
                         const float* corner_last, int n_corner, const float* surf_last, int n_surf);

/* ---- stage 3: laserMapping (laserMapping.cpp:305-848) ------------------------------ */
/* Consumes laserOdometry's corner_last / surf_last / pose of the same frame. */
int aloam_mapping(aloam_ctx* ctx, aloam_map_result* out);
/* Teacher-forcing input for mapping (corner_last, surf_last in the scan frame). */
int aloam_set_mapping_input(aloam_ctx* ctx, const float* corner_last, int n_corner,
                            const float* surf_last, int n_surf,
                            const double q_wodom_curr[4], const double t_wodom_curr[3]);
/* Map clouds: which = 0 surround (/laser_cloud_surround, laserMapping.cpp:806-821),
 * 1 whole map (/laser_cloud_map, :823-836). */
int aloam_get_map_cloud(aloam_ctx* ctx, int which, aloam_cloud* out);
/* /velodyne_cloud_registered (laserMapping.cpp:838-848): last full cloud in the map frame. */
int aloam_get_registered_cloud(aloam_ctx* ctx, aloam_cloud* out);
/* /aft_mapped_to_init_high_frec (laserOdometryHandler, laserMapping.cpp:197-229): an odometry pose
 * (/laser_odom_to_init) through the correction of the latest completed mapping frame,
 * q_out = q_wmap_wodom * q_wodom, t_out = q_wmap_wodom * t_wodom + t_wmap_wodom (Eigen's double
 * quaternion product and _transformVector; identity before the first mapping frame). Host
 * arithmetic only: callable from any thread (the reference calls it from the ROS spin thread while
 * process() runs), also while a pipeline worker runs the context's mapping. */
int aloam_map_high_freq_pose(aloam_ctx* ctx, const double q_wodom[4], const double t_wodom[3], double q_out[4],
                             double t_out[3]);

/* ---- whole per-scan pipeline: scanRegistration -> laserOdometry -> laserMapping ----- */
/* map_out may be NULL. With ALOAM_NO_MAPPING in flags the call stops after laserOdometry and
 * leaves the published corner/surf/full clouds + pose for aloam_forward_mapping_input. */
#define ALOAM_NO_MAPPING 2
int aloam_process_scan(aloam_ctx* ctx, const float* xyzr, int n, int flags,
                       aloam_odom_result* odom_out, aloam_map_result* map_out);
/* The /laser_cloud_corner_last, /laser_cloud_surf_last, /velodyne_cloud_3 and /laser_odom_to_init
 * hand-off (laserOdometry.cpp:588-663 -> laserMapping.cpp:192-234) between two contexts on the
 * same device, device to device: `src` ran laserOdometry (front end), `dst` runs laserMapping.
 * Lets the two stages of consecutive scans run concurrently on two streams, as the reference's
 * separate ROS nodes do. */
int aloam_forward_mapping_input(aloam_ctx* src, aloam_ctx* dst);
/* The scanRegistration -> laserOdometry topics (/velodyne_cloud_2, /laser_cloud_sharp,
 * /laser_cloud_less_sharp, /laser_cloud_flat, /laser_cloud_less_flat: scanRegistration.cpp:413-449
 * -> laserOdometry.cpp:280-292) between two contexts, device to device: `src` ran
 * aloam_scan_registration, `dst` then runs aloam_odometry. With it the three stages of three
 * consecutive scans run concurrently, like the reference's three nodes. */
int aloam_forward_features(aloam_ctx* src, aloam_ctx* dst);

/* ---- lower-level entry points (tests, tools) -------------------------------------- */
/* Residuals (3 per factor; plane types fill 1) and the tangent-space Jacobian
 * (3x6 per factor, row-major; columns = 3 rotation (left-multiplicative quaternion
 * tangent of EigenQuaternionParameterization) + 3 translation), Huber(0.1)-corrected
 * when robust != 0, plus the normal equations neq[28] = 21 upper JtJ + 6 Jtr + cost. */
int aloam_eval_factors(aloam_ctx* ctx, const aloam_factor* f, int n, const double x[7], int robust,
                       double* residuals, double* jacobians, double neq[28]);
/* One Ceres-equivalent Solve (LM, Huber 0.1, EigenQuaternionParameterization,
 * max_solver_iterations) over x = (qx,qy,qz,qw,tx,ty,tz), in place. */
int aloam_lm_solve(aloam_ctx* ctx, const aloam_factor* f, int n, double x[7], aloam_lm_summary* s);
/* PCL VoxelGrid (downsample_all_data, x,y,z,intensity centroids) on one cloud. */
int aloam_voxel_grid(aloam_ctx* ctx, const float* pts, int n, float leaf, aloam_cloud* out);
/* Exact radius k-NN (k <= 8, radius > 0) of each query in a point set by float L2 on x,y,z,
 * sorted by distance, ties by index; idx = -1 / d2 = +inf when fewer than k points lie within
 * the radius — the KdTreeFLANN::nearestKSearch + distance gate of laserMapping.cpp:582-584,648-650
 * (host buffers). */
int aloam_knn(aloam_ctx* ctx, const float* pts, int n, const float* queries, int nq, int k,
              float radius, int* idx, float* d2);
/* The same search on device-resident data (~240k queries against a ~2M-point
 * local map): d_pts / d_queries are device float4 (x, y, z, w) arrays, d_idx / d_d2 device arrays
 * of nq * k; the index is built in context memory grown on demand. Synchronous. Two-phase: a fine
 * grid's 3x3x3 block first (exact when the k-th neighbour is closer than 0.99 fine cells), the
 * radius-edge block for the rest; ALOAM_KNN_FINE = fine cell / radius (default 0.3; 0 = one phase).
 * Replaces the KdTreeFLANN::nearestKSearch calls of laserMapping.cpp:582,648 at C4 scale. */
int aloam_knn_device(aloam_ctx* ctx, const float* d_pts, int n, const float* d_queries, int nq, int k,
                     float radius, int* d_idx, float* d_d2);
/* The same search split into build and query, so repeated queries against one map pay for the
 * index once — laserMapping.cpp builds its map kd-trees once per frame (kdtreeCornerFromMap /
 * kdtreeSurfFromMap->setInputCloud, :558-559) and queries them in every round (nearestKSearch, :582,
 * :648). aloam_knn_build indexes the n device float4 points for radius-`radius` searches (both grids of
 * the two-phase search; the points are copied into the index, so d_pts may change afterwards);
 * aloam_knn_query answers nq device queries against the last built index (same results as
 * aloam_knn_device with the same points and radius; ALOAM_E_STATE before any build). Synchronous.
 * aloam_knn_device = aloam_knn_build + aloam_knn_query. Device buffers passed by pointer must be complete
 * when the call is made: the context's stream does not wait for another stream that is still filling
 * them (or filling the output arrays). */
int aloam_knn_build(aloam_ctx* ctx, const float* d_pts, int n, float radius);
int aloam_knn_query(aloam_ctx* ctx, const float* d_queries, int nq, int k, int* d_idx, float* d_d2);
/* Name of the search kernel the context's last aloam_knn_device / aloam_knn_query call launched (e.g. "k_knn_2phase<5,8>";
 * "" before the first call), so a timing of that call can be attributed to a kernel. ALOAM_KNN_TILE=1
 * (read per call) selects the LDS-tiled phase 1 ("k_knn_tile<...>"). Valid until the next call. */
const char* aloam_knn_kernel(const aloam_ctx* ctx);

/* TicToc stage names of the reference (printf'ed per scan), as indices of aloam_timing.tictoc_ms */
#define ALOAM_TT_PREPARE            0   /* "prepare time"              scanRegistration.cpp:128-254 */
#define ALOAM_TT_SEPARATE_POINTS    1   /* "seperate points time"      :269-410 (includes "sort q time" :287-289) */
#define ALOAM_TT_SCAN_REGISTRATION  2   /* "scan registration time"    :127-456 */
#define ALOAM_TT_DATA_ASSOCIATION   3   /* "data association time"     laserOdometry.cpp:382-564, summed over rounds */
#define ALOAM_TT_SOLVER             4   /* "solver time"               :570-577, summed over rounds */
#define ALOAM_TT_OPTIMIZATION_TWICE 5   /* "optimization twice time"   :363-579 */
#define ALOAM_TT_PUBLICATION        6   /* "publication time"          :585-664 (compose, last clouds, kd-trees, publish) */
#define ALOAM_TT_WHOLE_ODOMETRY     7   /* "whole laserOdometry time"  :353-665 */
#define ALOAM_TT_MAP_PREPARE        8   /* "map prepare time"          laserMapping.cpp:311-552 (recentring, surround, stacks) */
#define ALOAM_TT_BUILD_TREE         9   /* "build tree time"           :557-560 */
#define ALOAM_TT_MAP_ASSOCIATION   10   /* "mapping data assosiation time" :574-710, summed over rounds */
#define ALOAM_TT_MAP_SOLVER        11   /* "mapping solver time"       :712-721, summed over rounds */
#define ALOAM_TT_MAP_OPTIMIZATION  12   /* "mapping optimization time" :556-728 */
#define ALOAM_TT_ADD_POINTS        13   /* "add points time"           :736-784 (transformUpdate + insertion) */
#define ALOAM_TT_FILTER            14   /* "filter time"               :787-802 */
#define ALOAM_TT_MAPPING_PUB       15   /* "mapping pub time"          :804-850 (registered cloud) */
#define ALOAM_TT_WHOLE_MAPPING     16   /* "whole mapping time"        :307-852 */
#define ALOAM_TICTOC_N             17

/* Timing of the last pipeline call, measured with HIP events on the context's stream. */
typedef struct aloam_timing {
    float scan_registration_ms;
    float odometry_ms;
    float mapping_ms;
    float odom_search_ms;     /* sum over rounds of the odometry correspondence-search kernel */
    float map_search_ms;      /* sum over rounds of the mapping correspondence-search kernel  */
    int   odom_search_launches;
    int   map_search_launches;
    double map_search_bytes;  /* algorithmic bytes of the mapping searches     */
    double odom_search_bytes;
    float knn_ms;             /* aloam_knn_device: search kernel time (HIP events)              */
    int   knn_launches;
    double knn_bytes;         /* its algorithmic bytes: sum_q (16 + 16 |C27(q)|) + 8 k Q         */
    double knn_streamed_bytes;/* bytes it actually streamed (both phases of the two-phase search)   */
    float knn_build_ms;       /* aloam_knn_build / aloam_knn_device: index build time (HIP events)  */
    /* the reference's TicToc stage surface (tic_toc.h; printed by the three nodes), GPU time of the
     * same phases from HIP events on the stage's stream, indexed by ALOAM_TT_* below */
    float tictoc_ms[ALOAM_TICTOC_N];
} aloam_timing;
int aloam_set_profiling(aloam_ctx* ctx, int enable);
int aloam_get_timing(aloam_ctx* ctx, aloam_timing* t);
/* Restricts the context's streams to a set of CUs (bit i of mask[i / 32] = CU i; nwords = 0 lifts the
 * restriction). Used to give concurrent pipeline stages disjoint CUs. The context must be idle. */
int aloam_set_cu_mask(aloam_ctx* ctx, const unsigned* mask, int nwords);
/* Number of VoxelGrid / segment sorts (process-wide, all contexts on the current device) that exceeded
 * the workgroup replay's reach (n > 65,536) and ran the exact one-thread std::sort instead: correct but
 * slow, so a workload that reaches it is visible (bench.py reports it). Blocking: it reads the device
 * counters with a synchronous copy on the CALLING thread's current HIP device (call it between frames,
 * with that device current). */
int aloam_serial_sort_fallbacks(unsigned long long* count);

/* ---- native pipeline: the reference's node split on one GPU ---------------------------------
 * scanRegistration, laserOdometry and laserMapping run as three ROS processes in the reference, one
 * hot thread each (scanRegistration.cpp:461-503, laserOdometry.cpp:311, laserMapping.cpp:934). The
 * pipeline owns one context per stage and one native worker thread per later stage; push() runs the
 * first stage of scan k on the caller's thread while the workers run the later stages of earlier
 * scans, and hands data over device to device. stages = 2: [scanRegistration + laserOdometry] ||
 * [laserMapping]; stages = 3: one stage per node. Every scan passes every stage in order, so the
 * results equal aloam_process_scan's. */
typedef struct aloam_pipeline aloam_pipeline;
aloam_pipeline* aloam_pipeline_create(const aloam_params* p, int device, int stages);
void            aloam_pipeline_destroy(aloam_pipeline* pl);
const char*     aloam_pipeline_last_error(const aloam_pipeline* pl);
/* stage 0 = scanRegistration context, 1 = laserOdometry (== 0 when stages == 2), 2 = laserMapping */
aloam_ctx*      aloam_pipeline_context(aloam_pipeline* pl, int stage);
/* Feeds one sweep (flags as aloam_scan_registration). Outputs the odometry result completed in this
 * step (*have_od: scan k-1 for both stages 2 and 3 — scan k for stages 2 with profiling on) and the
 * mapping result completed in it (*have_mp: scan k-3 for stages 2 — k-2 with ALOAM_PIPE_LAG=1 —,
 * k-1 with profiling on, k-2 for stages 3). od / mp may be NULL. Stages 2 returns once scan k is
 * issued: its input (host or device) is read until the next push or flush returns. */
int aloam_pipeline_push(aloam_pipeline* pl, const float* xyzr, int n, int flags,
                        aloam_odom_result* od, int* have_od, aloam_map_result* mp, int* have_mp);
/* Drains the pipeline: the odometry result still in flight (stages 3), the mapping job in flight
 * (mp) and the mapping of that last odometry result (mp2); stages 2: the issued scan's odometry
 * result (od) and up to two of the mapping results still in flight, oldest first. Call again until it
 * returns nothing (*have_od, *have_mp and *have_mp2 all 0). */
int aloam_pipeline_flush(aloam_pipeline* pl, aloam_odom_result* od, int* have_od, aloam_map_result* mp, int* have_mp,
                         aloam_map_result* mp2, int* have_mp2);
/* HIP-event timing of each stage's last completed job (profiling on). */
int aloam_pipeline_set_profiling(aloam_pipeline* pl, int enable);
int aloam_pipeline_timing(aloam_pipeline* pl, int stage, aloam_timing* t);

/* ---- scan-to-map registration, sharded over ranks (BASELINE configs[3]) ----
 * The registration half of laserMapping::process (src/laserMapping.cpp:556-727: 10 rounds of
 * pointAssociateToMap + 5-NN within 1 m + line / plane fit + one ceres::Solve) against a local map
 * the caller supplies, for a corner / surf query stack of any size (the C4 stress set is a whole
 * 240k-point sweep against a 2M-point map). The query slots (corner stack, then surf stack: the
 * reference's AddResidualBlock order) are cut into ALOAM_S2M_RECORDS fixed blocks; a rank of a
 * world of W associates and evaluates the contiguous run of blocks aloam_shard_slot_range() gives
 * it, and every LM pass exchanges one record of 32 doubles per block (21 JtJ + 6 Jtr + cost +
 * count + corner / surf correspondences) with an RCCL all-gather over xGMI; every rank reduces the
 * ALOAM_S2M_RECORDS records in block order and runs the identical LM tail, so the pose is
 * bit-identical for every world size and no broadcast is needed. The map is replicated (2M points
 * = 32 MB of HBM per rank). */
#define ALOAM_S2M_RECORDS 256

typedef struct aloam_s2m_result {
    double q_w_curr[4];          /* parameters after the last round (laserMapping.cpp:129)   */
    double t_w_curr[3];
    int    optimized;            /* 0: map too small, solve skipped (laserMapping.cpp:554)   */
    int    rounds;
    int    corner_num[ALOAM_MAX_ROUNDS];   /* correspondences per round, all ranks          */
    int    surf_num[ALOAM_MAX_ROUNDS];
    aloam_lm_summary lm[ALOAM_MAX_ROUNDS];
    int    slot_begin, slot_end; /* this rank's query slots                                 */
    int    world;
} aloam_s2m_result;

/* The local map (laserCloudCornerFromMap / laserCloudSurfFromMap, map frame): float4 arrays of
 * nc / ns points, host memory or, with ALOAM_INPUT_DEVICE, device memory. Builds its search index. */
int aloam_s2m_set_map(aloam_ctx* ctx, const float* corner, int nc, const float* surf, int ns, int flags);
/* The query stacks (laserCloudCornerStack / laserCloudSurfStack, body frame, already downsampled;
 * laserMapping.cpp:542-550). Every rank passes the same full stacks. */
int aloam_s2m_set_queries(aloam_ctx* ctx, const float* corner, int ncq, const float* surf, int nsq, int flags);
/* Runs the rounds from x = (qx,qy,qz,qw,tx,ty,tz) in place. With a shard communicator
 * (aloam_shard_init) this is a collective: every rank calls it with the same x. */
int aloam_s2m_register(aloam_ctx* ctx, double x[7], aloam_s2m_result* out);
/* The same registration for `world` contexts driven from one thread (rank r = ctxs[r], one GPU or
 * several): the record exchange is a peer copy between the contexts' streams instead of RCCL.
 * out (may be NULL) receives world results. */
int aloam_s2m_register_group(aloam_ctx** ctxs, int world, double x[7], aloam_s2m_result* out);
/* RCCL communicator for the exchange (librccl.so.1 is loaded on first use). Rank 0 creates the
 * 128-byte id, the caller distributes it (e.g. torch.distributed), then every rank calls
 * aloam_shard_init (collective). world = 1 needs no id: with id NULL there is no exchange, with an
 * id a one-rank communicator is created and the exchange still goes through RCCL. */
int aloam_shard_unique_id(unsigned char id[128]);
int aloam_shard_init(aloam_ctx* ctx, int rank, int world, const unsigned char* id);
/* The exchange on the device, no host and no RCCL in it (replaces the per-pass ncclAllGather of
 * aloam_s2m_register; the reference's counterpart is ceres::Solve's in-process evaluation,
 * laserMapping.cpp:714-721). Each rank exports a small uncached buffer (records + arrival counters);
 * aloam_shard_peer_handle returns its IPC handle, the caller all-gathers the world's handles (e.g.
 * torch.distributed), every rank calls aloam_shard_peer_open with them (rank r's handle at
 * handles + r * ALOAM_PEER_HANDLE_BYTES), then a barrier, then aloam_s2m_register as usual: every Solve
 * is one persistent launch per rank whose workgroups publish their block records, wait on the peers'
 * monotonic arrival counters and gather the peers' records over xGMI themselves; results are
 * bit-identical to the RCCL exchange. World <= 8, one rank per GPU (or several processes on one GPU
 * with ALOAM_S2M_SOLVE_G x world <= the CU count), the same ALOAM_S2M_SOLVE_G on every rank. While open it
 * takes precedence over a shard communicator. A peer that never arrives ends the Solve after ~2 s
 * with ALOAM_E_HIP and closes the exchange (open it again on every rank). */
#define ALOAM_PEER_HANDLE_BYTES 64
int aloam_shard_peer_handle(aloam_ctx* ctx, unsigned char handle[ALOAM_PEER_HANDLE_BYTES]);
int aloam_shard_peer_open(aloam_ctx* ctx, const unsigned char* handles, int world, int rank);
int aloam_shard_peer_close(aloam_ctx* ctx);
/* [begin, end) query slots of `rank` among n_slots (pure host function, no device needed). */
int aloam_shard_slot_range(int n_slots, int rank, int world, int* begin, int* end);

#ifdef __cplusplus
}
#endif
#endif /* ALOAM_HIP_H */
