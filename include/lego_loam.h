/* lego_loam.h — C-ABI of the MI355X-native LeGO-LOAM per-scan hot path.
 *
 * The reference's "plugin API" for this path is its ROS node/topic surface
 * (SURVEY.md §8b).  Each entry point below replaces one node callback and
 * keeps that topic's payload:
 *
 *   lego_ip_process   <- ImageProjection::cloudHandler
 *                        (LeGO-LOAM/src/imageProjection.cpp:181-197)
 *                        in : /velodyne_points        (PointCloud2, PointXYZIR)
 *                        out: /segmented_cloud, /segmented_cloud_info
 *                             (cloud_msgs/msg/cloud_info.msg:1-12),
 *                             /outlier_cloud (+ gated /full_cloud_projected,
 *                             /ground_cloud, /segmented_cloud_pure)
 *   lego_fa_process   <- FeatureAssociation::runFeatureAssociation
 *                        (LeGO-LOAM/src/featureAssociation.cpp:1817-1860)
 *                        out: /laser_cloud_{sharp,less_sharp,flat,less_flat},
 *                             /laser_odom_to_init, /laser_cloud_{corner,surf}_last,
 *                             /outlier_cloud_last
 *   lego_mo_process   <- mapOptimization::run scan-to-map part
 *                        (LeGO-LOAM/src/mapOptmization.cpp:1487-1522,
 *                         376-606, 956-1350)
 *   lego_odom_batch   the device-resident hot path: ip+fa (incl. the two-step
 *                        LM odometry) over K consecutive scans of one stream,
 *                        one pose record per scan (what bench.py times).
 *
 * Conventions (mirroring the reference):
 *   - all functions return a lego_status; nothing throws across the ABI;
 *   - a non-dense input cloud is LEGO_E_NOT_DENSE (the reference ROS_ERRORs and
 *     shuts down, imageProjection.cpp:174-177);
 *   - output buffers are library-owned and valid until the next call on the
 *     same context (the reference reuses member clouds the same way);
 *   - a context is NOT thread-safe; distinct contexts are independent.
 */
#ifndef LEGO_LOAM_H_
#define LEGO_LOAM_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  LEGO_OK = 0,
  LEGO_E_NOT_DENSE = 1, /* input has non-finite xyz (imageProjection.cpp:174) */
  LEGO_E_CAPACITY = 2,  /* more points than the context was sized for */
  LEGO_E_DEVICE = 3,    /* HIP runtime error / no device */
  LEGO_E_ARG = 4,       /* bad argument (null, empty cloud, bad config) */
  LEGO_E_STATE = 5      /* call out of order (e.g. mo before any fa) */
} lego_status;

/* /velodyne_points point: the velodyne PointCloud2 wire layout, point_step 32
 * (x@0 y@4 z@8 intensity@16 ring@20) = PointXYZIR, utility.h:153-165. */
typedef struct lego_point_xyzir {
  float x, y, z, _pad0;
  float intensity;
  uint16_t ring;
  uint16_t _pad1;
  uint32_t _pad2[2];
} lego_point_xyzir;

/* PointType = pcl::PointXYZI (utility.h:51), packed to 16 bytes. */
typedef struct lego_point_xyzi {
  float x, y, z, intensity;
} lego_point_xyzi;

/* Runtime form of the compile-time constants of utility.h:53-136. */
typedef struct lego_sensor_cfg {
  int32_t n_scan;            /* N_SCAN            utility.h:63 */
  int32_t horizon_scan;      /* Horizon_SCAN      utility.h:64 */
  float ang_res_x;           /* utility.h:65 */
  float ang_res_y;           /* utility.h:66 */
  float ang_bottom;          /* utility.h:67 */
  int32_t ground_scan_ind;   /* groundScanInd     utility.h:68 */
  int32_t use_cloud_ring;    /* utility.h:60 */
  float sensor_minimum_range;/* utility.h:111 */
  float sensor_mount_angle;  /* utility.h:112 */
  float segment_theta;       /* utility.h:113 */
  int32_t segment_valid_point_num; /* utility.h:114 */
  int32_t segment_valid_line_num;  /* utility.h:115 */
  float segment_alpha_x;     /* utility.h:116 (derived) */
  float segment_alpha_y;     /* utility.h:117 (derived) */
  float edge_threshold;      /* utility.h:123 */
  float surf_threshold;      /* utility.h:124 */
  float nearest_feature_search_sq_dist; /* utility.h:125 */
  float scan_period;         /* utility.h:107 */
  double mapping_process_interval; /* utility.h:105 */
  float surrounding_keyframe_search_radius; /* utility.h:129 */
  int32_t skip_frame_num;    /* featureAssociation.cpp:284 */
} lego_sensor_cfg;

/* Presets: "VLP-16" (utility.h:63-68), "HDL-32E" (:71-76), "VLS-128" (:79-84),
 * "OS1-16" (:89-94), "OS1-64" (:97-102), and "HDL-64E" (64x2048, KITTI-shaped:
 * no preset in the reference, README.md:86; derived in DESIGN.md). */
int lego_sensor_preset(const char* name, lego_sensor_cfg* out);

/* cloud_msgs/cloud_info (cloud_info.msg:1-12).  The three per-point arrays have
 * length N_SCAN*Horizon_SCAN like the reference (imageProjection.cpp:128-130);
 * only the first n_segmented entries are meaningful. */
typedef struct lego_cloud_info {
  double stamp;
  const int32_t* start_ring_index; /* [n_scan] */
  const int32_t* end_ring_index;   /* [n_scan] */
  float start_orientation;
  float end_orientation;
  float orientation_diff;
  const uint8_t* segmented_cloud_ground_flag; /* [P] */
  const uint32_t* segmented_cloud_col_ind;    /* [P] */
  const float* segmented_cloud_range;         /* [P] */
} lego_cloud_info;

typedef struct lego_ip_out {
  lego_cloud_info info;                  /* /segmented_cloud_info */
  const lego_point_xyzi* segmented_cloud;/* /segmented_cloud */
  int32_t n_segmented;
  const lego_point_xyzi* outlier_cloud;  /* /outlier_cloud */
  int32_t n_outlier;
  /* gated outputs / range-image debug view; NULL unless LEGO_IP_IMAGES set */
  const lego_point_xyzi* full_cloud;     /* /full_cloud_projected [P] */
  const float* range_image;              /* rangeMat  [P] */
  const int8_t* ground_image;            /* groundMat [P] */
  const int32_t* label_image;            /* labelMat  [P] */
  /* the topics the reference publishes only with a subscriber
   * (imageProjection.cpp:480-506); NULL / 0 unless LEGO_IP_GATED is set.
   * Node-shaped calls (lego_ip_process, lego_ip_process_pc2) only. */
  const lego_point_xyzi* full_info_cloud;      /* /full_cloud_info [P]: intensity = range (:252-254) */
  const lego_point_xyzi* ground_cloud;         /* /ground_cloud: groundMat == 1, rows <= groundScanInd (:301-308) */
  int32_t n_ground;
  const lego_point_xyzi* segmented_cloud_pure; /* /segmented_cloud_pure: labels, intensity = label (:357-367) */
  int32_t n_segmented_pure;
} lego_ip_out;

#define LEGO_IP_IMAGES 1u /* full_cloud and the range / ground / label images */
#define LEGO_IP_GATED 2u  /* full_info_cloud, ground_cloud, segmented_cloud_pure */

typedef struct lego_fa_out {
  double stamp;
  /* /laser_cloud_sharp, _less_sharp, _flat, _less_flat (camera frame) */
  const lego_point_xyzi* sharp;      int32_t n_sharp;
  const lego_point_xyzi* less_sharp; int32_t n_less_sharp;
  const lego_point_xyzi* flat;       int32_t n_flat;
  const lego_point_xyzi* less_flat;  int32_t n_less_flat;
  /* /laser_odom_to_init (featureAssociation.cpp:1727-1744) */
  int32_t odom_valid;        /* 0 on the initialisation scan (:1846-1849) */
  float transform_cur[6];
  float transform_sum[6];
  double odom_quat[4];       /* x,y,z,w exactly as published (:1731-1734) */
  double odom_pos[3];
  /* hand-off to mapping every (skip_frame_num+1)-th scan (:1790-1814) */
  int32_t publish_to_mapping;
  const lego_point_xyzi* corner_last;  int32_t n_corner_last;
  const lego_point_xyzi* surf_last;    int32_t n_surf_last;
  const lego_point_xyzi* outlier_last; int32_t n_outlier_last;
} lego_fa_out;

typedef struct lego_mo_out {
  int32_t processed;          /* mapping ran this call (interval gate :1499) */
  int32_t optimized;          /* scan2MapOptimization guard passed (:1331) */
  int32_t iterations;
  float transform_tobe_mapped[6];
  float transform_aft_mapped[6];
  float transform_bef_mapped[6];
  int32_t n_corner_map_ds, n_surf_map_ds, n_corner_scan_ds, n_surf_scan_ds;
  int32_t n_rows_last;        /* laserCloudOri size at the last iteration */
} lego_mo_out;

/* One performLoopClosure (mapOptmization.cpp:875-945; loopClosureThread runs
 * it at 1 Hz when loopClosureEnableFlag is set, utility.h:104): the history
 * keyframe search (detectLoopClosure :814-872), the ICP of the latest
 * keyframe against the +-25 keyframes around the closest old one, and the
 * loop constraint the reference adds to iSAM2 (:919-939).  GTSAM is not part
 * of this library: the constraint is returned for the caller's pose graph. */
typedef struct lego_loop_out {
  int32_t detected;        /* a keyframe > 30 s old within 7 m of the robot */
  int32_t converged;       /* icp.hasConverged() */
  int32_t accepted;        /* converged && fitness <= historyKeyframeFitnessScore: the factor is added */
  int32_t latest_id;       /* latestFrameIDLoopCloure */
  int32_t closest_id;      /* closestHistoryFrameID */
  int32_t iterations;      /* ICP iterations run */
  int32_t n_source;        /* latestSurfKeyFrameCloud (intensity >= 0) */
  int32_t n_target;        /* nearHistorySurfKeyFrameCloudDS */
  double fitness;          /* icp.getFitnessScore() = the constraint's noise variance */
  float icp_transform[16]; /* getFinalTransformation(), row-major (camera frame) */
  double from_rotation[9]; /* gtsam poseFrom (corrected latest keyframe), row-major */
  double from_translation[3];
  double to_rotation[9];   /* poseTo (the history keyframe) */
  double to_translation[3];
  double between_rotation[9];  /* poseFrom.between(poseTo): the BetweenFactor's measurement */
  double between_translation[3];
} lego_loop_out;

/* /imu_raw message (sensor_msgs/Imu; utility.h:54): the fields the
 * reference's imuHandlers read (featureAssociation.cpp:431-458,
 * mapOptmization.cpp:643-652). */
typedef struct lego_imu_msg {
  double stamp;                  /* header.stamp.toSec() */
  double orientation[4];         /* x, y, z, w */
  double angular_velocity[3];    /* x, y, z */
  double linear_acceleration[3]; /* x, y, z */
} lego_imu_msg;

/* One record per scan from the batch path (64 bytes, also the RCCL gather
 * unit of the multi-GPU bench). */
typedef struct lego_pose_rec {
  double stamp;
  float transform_sum[6];
  int32_t n_segmented;
  int32_t n_sharp, n_less_sharp, n_flat, n_less_flat;
  int32_t odom_valid;
  int32_t flags;   /* LEGO_REC_* bits: which paths this scan took (diagnostic) */
  int32_t _pad;
} lego_pose_rec;
/* lego_pose_rec.flags */
#define LEGO_REC_RING0_REDONE 2  /* ring 0 re-extracted with the stream's real carry (SURVEY.md §9.7 residue) */
#define LEGO_REC_SORT_TIES 4     /* a sector had equal curvatures: sorted by the std::sort restatement
                                    (featureAssociation.cpp:699), not the bitonic network */
#define LEGO_REC_ODOM_HBM 8      /* the LM ran on HBM-resident last clouds (LDS caps exceeded) */

typedef struct lego_ctx lego_ctx;

/* Creates a per-stream context on HIP device `device`, sized for scans of up to
 * max_points points and batches of up to max_batch scans. */
int lego_create(const lego_sensor_cfg* cfg, int device, int32_t max_points,
                int32_t max_batch, lego_ctx** out);
/* A fleet: n_streams independent lidar streams in one context on one device,
 * run together by lego_odom_batch (one launch per stage for all of them; the
 * device's CUs split between the streams' odometry chains).  Batches are
 * stream-major: nscans = n_streams x K, scans [s*K, s*K + K) are K consecutive
 * scans of stream s, K <= scans_per_stream.  Each stream's results equal those
 * of its own lego_create context.  The node-shaped calls (lego_fa_process,
 * lego_mo_*) need a single-stream context (LEGO_E_ARG otherwise).
 * No reference counterpart: the reference runs one stream per process. */
int lego_fleet_create(const lego_sensor_cfg* cfg, int device, int32_t n_streams,
                      int32_t max_points, int32_t scans_per_stream, lego_ctx** out);

/* Per-context options, fixed at creation (lego_create_ex /
 * lego_fleet_create_ex; lego_create and lego_fleet_create use the defaults).
 * Scheduling and diagnostic switches: none of them changes a result, which
 * the tests check by running both settings against the oracle.  Nothing in
 * the library reads the environment.  No reference counterpart (the
 * reference's schedule is fixed by its ROS nodes). */
typedef struct lego_ctx_opts {
  int32_t size;            /* sizeof(lego_ctx_opts); lego_ctx_opts_init sets it */
  int32_t node_overlap;    /* 1 (default): lego_fa_process runs the per-ring less-flat VoxelGrid on a
                              second stream beside the LM; 0: one stream */
  int32_t front_parts;     /* a fleet batch's projection + extraction in this many parts of whole
                              streams on their own HIP streams (default 2; reduced to a divisor) */
  int32_t lfv_wave;        /* 1 (default): small rings' VoxelGrids by one wave each; 0: by workgroups */
  int32_t lfv_block_rings; /* large rings per VoxelGrid workgroup; 0 (default): by the launch size */
  int32_t lfv_wide;        /* 1: every ring's VoxelGrid by a 1024-thread workgroup, 0: 256 threads,
                              -1 (default): 1024 for launches of <= 128 rings */
  int32_t ccl_tiles;       /* 1 (default): the HBM union-find in LDS column tiles + seams; 0: per edge in HBM */
  int32_t seg_hbm;         /* 1: every image through the HBM union-find (diagnostic; default 0) */
  int32_t odom_workgroups; /* odometry workgroups per stream; 0 (default): by the sensor and the CUs */
  int32_t odom_gridless;   /* 1 / 0: NN without / with grids; -1 (default): by the workgroup count */
  int32_t odom_integ;      /* 1 / 0: the integration on its own workgroup or the lead's;
                              -1 (default): its own when there are >= 2 workgroups */
  int32_t odom_silent_wg;  /* diagnostic: this workgroup publishes into private exchange copies
                              (the others steal its work); -1 (default): none */
  int32_t odom_late_wg;    /* diagnostic: this workgroup starts after the lead ends; -1: none */
  int32_t lf_wait_ms;      /* the node hand-off's bound on waiting for the VoxelGrid's stream
                              (default 2000; 0: never waits, i.e. a forced LEGO_E_DEVICE, for tests) */
  int32_t mo_cand_cache;   /* 1 (default): mapping keeps a candidate cache of map points */
  int32_t kf_cap;          /* keyframe store capacity cap; 0 (default): sized from the arena */
  int32_t vg_rounds;       /* mapping VoxelGrids' partition rounds; -1 (default): by the cloud size */
  int32_t fa_synccheck;    /* diagnostic: synchronise after every extraction launch and name the
                              kernel that failed (stderr); default 0 */
  int32_t mo_hostprof;     /* diagnostic: the mapping step's host enqueue times (stderr); default 0 */
  int32_t mo_evprof;       /* diagnostic: the mapping step's chain times (stderr); default 0 */
  int32_t ip_fused;        /* 1 (default): a batch of VLP-16-class scans is projected, ground-walked
                              and segmented by one kernel, a workgroup per scan (k_ip_lds);
                              0: four kernels (k_project, k_pixels, k_ground, k_seg_lds) */
  int32_t reserved[11];
} lego_ctx_opts;
void lego_ctx_opts_init(lego_ctx_opts* opts);
/* lego_create / lego_fleet_create with options (NULL: the defaults). */
int lego_create_ex(const lego_sensor_cfg* cfg, int device, int32_t max_points, int32_t max_batch,
                   const lego_ctx_opts* opts, lego_ctx** out);
int lego_fleet_create_ex(const lego_sensor_cfg* cfg, int device, int32_t n_streams, int32_t max_points,
                         int32_t scans_per_stream, const lego_ctx_opts* opts, lego_ctx** out);
int lego_destroy(lego_ctx* ctx);
/* Resets the per-stream state (odometry, residues) to construction values.
 * Needed after a LEGO_E_DEVICE of the odometry's hand-off wait (the stream's
 * state is then not advanced; lego_fa_process and the batch calls return
 * LEGO_E_STATE until the reset). */
int lego_reset(lego_ctx* ctx);

int lego_ip_process(lego_ctx* ctx, const lego_point_xyzir* pts, int32_t n,
                    double stamp, uint32_t flags, lego_ip_out* out);
int lego_fa_process(lego_ctx* ctx, const lego_ip_out* in, lego_fa_out* out);

/* Device-resident batch: scans k=0..nscans-1 are the points
 * pts[offsets[k] .. offsets[k+1]).  pts/offsets are device pointers when
 * on_device != 0, host pointers otherwise.  Runs ip + fa + odometry for every
 * scan in stream order and writes one record per scan to recs (host).  On a
 * fleet context the batch is stream-major (lego_fleet_create) and nscans a
 * multiple of n_streams (LEGO_E_ARG otherwise).
 * offsets[k+1] > offsets[k] (an empty scan is LEGO_E_ARG, nothing runs) and
 * every scan <= max_points (LEGO_E_CAPACITY).  A non-finite point anywhere in
 * the batch is LEGO_E_NOT_DENSE, detected on the device after the batch ran:
 * the stream state is then undefined and the caller must lego_reset (the
 * reference shuts the node down, imageProjection.cpp:174-177). */
int lego_odom_batch(lego_ctx* ctx, const lego_point_xyzir* pts,
                    const int64_t* offsets, const double* stamps,
                    int32_t nscans, int32_t on_device, lego_pose_rec* recs);
/* /imu_raw: delivers messages to the featureAssociation and mapOptimization
 * IMU queues in order (featureAssociation.cpp:431-458 imuHandler +
 * AccumulateIMUShiftAndRotation :392-429; mapOptmization.cpp:643-652), as
 * the ROS callbacks would between two scans.  Single-stream contexts. */
int lego_imu_push(lego_ctx* ctx, const lego_imu_msg* msgs, int32_t n);
/* lego_odom_batch with the IMU messages that arrive during the batch:
 * imu[0 .. imu_before[k]) are delivered before scan k is processed
 * (imu_before non-decreasing, <= n_imu), the rest after the last scan.
 * Deskew (adjustDistortion :525-614), the initial guess (updateInitialGuess
 * :1639-1664), integration and the hand-off then use the IMU terms once the
 * stream has received a message.  Single-stream contexts. */
int lego_odom_batch_imu(lego_ctx* ctx, const lego_point_xyzir* pts,
                        const int64_t* offsets, const double* stamps,
                        int32_t nscans, int32_t on_device, const lego_imu_msg* imu,
                        int32_t n_imu, const int32_t* imu_before, lego_pose_rec* recs);
/* Asynchronous form: lego_odom_batch_submit enqueues a batch (arguments as
 * lego_odom_batch_imu; pass imu = NULL, n_imu = 0 without IMU) and returns;
 * lego_odom_batch_wait blocks for the oldest submitted batch and writes its
 * cap >= nscans records.  At most two batches are in flight (LEGO_E_STATE
 * otherwise): the second one's projection and extraction run while the
 * first one's odometry chain does.  The node-shaped calls and lego_reset
 * need no batch in flight.  Host input arrays may be reused once submit
 * returns; device inputs must stay valid until the wait. */
int lego_odom_batch_submit(lego_ctx* ctx, const lego_point_xyzir* pts,
                           const int64_t* offsets, const double* stamps,
                           int32_t nscans, int32_t on_device, const lego_imu_msg* imu,
                           int32_t n_imu, const int32_t* imu_before);
int lego_odom_batch_wait(lego_ctx* ctx, lego_pose_rec* recs, int32_t cap, int32_t* nscans);
/* After lego_odom_batch: fetch full per-scan outputs of scan k of that batch. */
int lego_batch_fetch(lego_ctx* ctx, int32_t k, lego_ip_out* ip, lego_fa_out* fa);

/* ---- Wire formats: sensor_msgs/PointCloud2 and
 * cloud_msgs/cloud_info as they travel between the ROS nodes. */

/* sensor_msgs/PointField datatypes. */
enum { LEGO_PF_INT8 = 1, LEGO_PF_UINT8 = 2, LEGO_PF_INT16 = 3, LEGO_PF_UINT16 = 4,
       LEGO_PF_INT32 = 5, LEGO_PF_UINT32 = 6, LEGO_PF_FLOAT32 = 7, LEGO_PF_FLOAT64 = 8 };

typedef struct lego_pc2_field {
  char name[16];
  uint32_t offset;
  uint8_t datatype;
  uint32_t count;
} lego_pc2_field;

/* A sensor_msgs/PointCloud2 (header stamp as seconds).  data holds
 * height x row_step bytes; host or device memory as the call says. */
typedef struct lego_pc2_msg {
  double stamp;
  uint32_t height, width, point_step, row_step;
  uint8_t is_bigendian, is_dense;
  int32_t n_fields;
  const lego_pc2_field* fields;
  const uint8_t* data;
} lego_pc2_msg;

/* pcl::fromROSMsg into PointXYZIR (imageProjection.cpp:166, 172): each of
 * x, y, z, intensity (FLOAT32) and ring (UINT16) is copied from the field of
 * that name, datatype and count 1; a field without a match stays 0 (PCL
 * warns and skips it).  Big-endian data is LEGO_E_ARG.  is_dense == 0 is
 * LEGO_E_NOT_DENSE (:173-176).  Decoding runs on the device; out is host
 * memory with room for height x width points. */
int lego_pc2_decode(lego_ctx* ctx, const lego_pc2_msg* msg, lego_point_xyzir* out,
                    int32_t cap, int32_t* n_out);
/* cloudHandler on a raw /velodyne_points message (decode + lego_ip_process). */
int lego_ip_process_pc2(lego_ctx* ctx, const lego_pc2_msg* msg, uint32_t flags, lego_ip_out* out);
/* lego_odom_batch over nscans raw messages (msgs[k].data: device pointers
 * when on_device != 0, host otherwise); stamps from the messages. */
int lego_odom_batch_pc2(lego_ctx* ctx, const lego_pc2_msg* msgs, int32_t nscans,
                        int32_t on_device, lego_pose_rec* recs);

/* pcl::toROSMsg of a PointXYZI cloud (the /segmented_cloud, /outlier_cloud,
 * /laser_cloud_* payloads): fields x@0 y@4 z@8 intensity@16 FLOAT32,
 * point_step 32, height 1, dense.  Writes 32 * n bytes to data (bytes 12-15
 * carry PCL's data[3] = 1.0f, the rest of the padding is 0) and the 4
 * fields to fields4. */
int lego_pc2_encode_xyzi(const lego_point_xyzi* pts, int32_t n, uint8_t* data,
                         lego_pc2_field* fields4);
/* ROS1 wire bytes of a cloud_msgs/cloud_info (cloud_info.msg:1-12):
 * Header {seq, stamp = ros::Time::fromSec(info->stamp), frame_id}, then the
 * arrays with their uint32 lengths — startRingIndex / endRingIndex n_scan,
 * the three per-point arrays P = n_scan x horizon_scan (the reference
 * publishes them at full length, imageProjection.cpp:125-130).  *len gets
 * the size; with buf == NULL only the size is computed. */
int lego_cloud_info_serialize(const lego_cloud_info* info, int32_t n_scan, int32_t horizon_scan,
                              uint32_t seq, const char* frame_id, uint8_t* buf, uint64_t cap,
                              uint64_t* len);

/* Mapping (scan-to-map).  lego_mo_set_map installs a fixed surrounding map
 * (config 5) instead of the keyframe-built one; pass NULLs to go back to the
 * keyframe map of mapOptmization.cpp:1001-1056. */
int lego_mo_set_map(lego_ctx* ctx, const lego_point_xyzi* corner, int32_t n_corner,
                    const lego_point_xyzi* surf, int32_t n_surf);
/* Mapping options (mapOptimization's compile-time switches, utility.h:104,130). */
typedef struct lego_mo_opts {
  /* 1: an installed fixed map goes through the map VoxelGrids and the NN
   * index build on every mapping step, as extractSurroundingKeyFrames and
   * scan2MapOptimization do with the surrounding map (mapOptmization.cpp:
   * 1058-1064, 1333-1334).  0 (default): filtered and indexed once per
   * lego_mo_set_map (the filter of an unchanged cloud is the same cloud, so
   * results are identical). */
  int32_t fixed_map_per_step;
  /* loopClosureEnableFlag (utility.h:104, default false).  1: the surrounding
   * map is the most recent surrounding_keyframe_search_num keyframes
   * (:961-999) instead of the radius search, every saved keyframe goes into
   * the context's pose graph, an accepted lego_mo_loop_closure adds its loop
   * factor, and the next mapping step re-optimises the graph and corrects the
   * keyframe poses (correctPoses :1456-1478).  Keyframe-built map only. */
  int32_t loop_closure_enable;
  int32_t surrounding_keyframe_search_num; /* utility.h:130; <= 0 selects 50 */
  int32_t _pad;
} lego_mo_opts;
/* Sets the options; takes effect at the next lego_mo_process.  Switching
 * loop_closure_enable needs a context with no saved keyframe (LEGO_E_STATE). */
int lego_mo_configure(lego_ctx* ctx, const lego_mo_opts* opts);
/* mapOptimization::run's scan-to-map step on the published clouds of `in`
 * (mapOptmization.cpp:1487-1522).  When `in` is this context's own last
 * lego_fa_process / lego_batch_fetch output, unchanged (its corner / surf /
 * outlier pointers and counts, no projection, extraction or batch call in
 * between), the clouds are read where that call copied them from, on the
 * device: no upload.  The host buffers are then not read, so a caller that
 * edits them in place must pass a copy; any other clouds are uploaded. */
int lego_mo_process(lego_ctx* ctx, const lego_fa_out* in, lego_mo_out* out);
/* performLoopClosure over the keyframes the mapping calls have saved (needs
 * the keyframe-built map, i.e. no lego_mo_set_map); LEGO_E_ARG otherwise. */
int lego_mo_loop_closure(lego_ctx* ctx, lego_loop_out* out);

/* transformFusion (transformFusion.cpp:94-239): /integrated_to_init, the
 * odometry pose composed with the latest mapping correction.  Host math, per
 * message, in the context's fusion state. */
typedef struct lego_fusion_out {
  double stamp;
  float transform_mapped[6];
  double quat[4];  /* orientation x, y, z, w as published (:189-196) */
  double pos[3];
} lego_fusion_out;
/* laserOdometryHandler (:174-205): one /laser_odom_to_init message (the
 * odom_quat / odom_pos / stamp of a lego_fa_out). */
int lego_fusion_odometry(lego_ctx* ctx, const lego_fa_out* odom, lego_fusion_out* out);
/* odomAftMappedHandler (:207-227): the /aft_mapped_to_init message of a
 * processed lego_mo_out (mapOptmization.cpp:654-679 publishTF). */
int lego_fusion_aft_mapped(lego_ctx* ctx, const lego_mo_out* mo);

/* ---- featureAssociation's hand-off to the serial mapping consumer
 * (publishCloudsLast, featureAssociation.cpp:1790-1815) as one packet per
 * batch, so streams running on other GPUs can be mapped on rank 0.
 *
 * Packet (little-endian, 8-byte aligned): a lego_handoff_hdr, nscans
 * lego_handoff_scan entries, then for every scan with publish_to_mapping set
 * its /laser_cloud_corner_last, /laser_cloud_surf_last and
 * /outlier_cloud_last points (lego_point_xyzi, the published forms, the
 * outliers axis-swapped as adjustOutlierCloud does, :1746-1757) at the entry's
 * offset, in that order. */
#define LEGO_HANDOFF_MAGIC 0x4f48474cu /* "LGHO" */
typedef struct lego_handoff_hdr {
  uint32_t magic, version; /* LEGO_HANDOFF_MAGIC, 1 */
  int32_t nscans, npub;    /* scans of the batch, scans published to mapping */
  uint64_t bytes;          /* the whole packet */
  uint64_t _pad;
} lego_handoff_hdr;
typedef struct lego_handoff_scan {
  lego_pose_rec rec;       /* the batch record of the scan */
  float transform_cur[6];
  int32_t publish_to_mapping;
  int32_t n_corner_last, n_surf_last, n_outlier_last; /* 0 unless published */
  uint64_t offset;         /* byte offset of the corner points in the packet */
  uint64_t _pad[2];
} lego_handoff_scan;
/* Packs the last batch lego_odom_batch / lego_odom_batch_wait returned into a
 * device buffer owned by the context (*packet, *bytes), complete when the
 * call returns; valid until the next batch call on the context. */
int lego_handoff_pack(lego_ctx* ctx, const void** packet, uint64_t* bytes);
/* The same into caller-owned device memory dst (cap bytes, on the context's
 * device; LEGO_E_CAPACITY if smaller); dst == NULL only sets *bytes. */
int lego_handoff_pack_into(lego_ctx* ctx, void* dst, uint64_t cap, uint64_t* bytes);
/* Host-side view of scan k of a packet in host memory: its record and, in
 * out, the lego_fa_out lego_mo_process consumes (stamp, transform_sum /
 * _cur, odom_quat / _pos, publish flag, the three clouds pointing into the
 * packet; the feature clouds are not part of the hand-off and stay NULL).
 * Needs no device.  LEGO_E_ARG for a malformed packet or k out of range. */
int lego_handoff_unpack(const void* packet, uint64_t bytes, int32_t k, lego_pose_rec* rec, lego_fa_out* out);

/* Native collective for the hand-off (RCCL over xGMI): one communicator per
 * process and GPU, ranks 0..nranks-1 sharing the unique id rank 0 created
 * (the caller broadcasts the 128 bytes, e.g. over MPI or torch.distributed). */
typedef struct lego_comm lego_comm;
int lego_comm_unique_id(uint8_t id[128]);
/* Every wait a call makes on the communicator's stream is bounded (default
 * 60000 ms, lego_comm_set_timeout): a peer that never joins a collective
 * makes the waiting call abort the communicator and return LEGO_E_DEVICE with
 * the wait named in lego_last_error, instead of blocking the process. */
int lego_comm_create(const uint8_t id[128], int32_t nranks, int32_t rank, int32_t device, lego_comm** out);
/* The bound of every later wait on the communicator's stream, ms >= 1. */
int lego_comm_set_timeout(lego_comm* comm, int32_t timeout_ms);
int lego_comm_destroy(lego_comm* comm);
/* The communicator's rank count as RCCL reports it (ncclCommCount). */
int lego_comm_count(lego_comm* comm, int32_t* nranks);
/* Aborts the communicator (ncclCommAbort): every operation still queued on it
 * is cancelled, so its stream drains, and every later call returns
 * LEGO_E_STATE.  Call it on every rank once any rank reports a failed gather
 * (the caller agrees on that over its own control channel): a failure on root
 * after the size exchange (a receive buffer it cannot allocate, a copy error)
 * aborts only root's communicator, and the other ranks' sends of that gather,
 * queued with LEGO_COMM_DEVICE_RESULT, would otherwise never complete; their
 * next lego_comm_wait or gather would block.  lego_comm_destroy after an abort
 * does not block. */
int lego_comm_abort(lego_comm* comm);
/* Collective over all ranks: every rank packs its context's last batch
 * (lego_handoff_pack) and root receives every rank's packet (ncclGather of
 * the sizes, then ncclSend / ncclRecv of the packets in one group).  Returns
 * once the packets are in root's host memory (lego_comm_handoff).
 * = lego_comm_gather_handoff_ex(comm, ctx, root, 0). */
int lego_comm_gather_handoff(lego_comm* comm, lego_ctx* ctx, int32_t root);
/* flags: LEGO_COMM_DEVICE_RESULT keeps the gathered packets in root's device
 * memory (lego_comm_handoff_device) and returns once the send / receive is
 * enqueued on the communicator's stream: root waits only for the 8-byte
 * sizes, no packet crosses PCIe and no rank waits for the transfer (the next
 * call, lego_comm_wait or a device synchronisation does).  A rank whose pack
 * fails still takes part with an empty packet (the others do not hang) and
 * returns the pack's status; an RCCL or device error after the communicator
 * was used aborts it (ncclCommAbort) and every later call returns
 * LEGO_E_STATE (the other ranks then call lego_comm_abort, above).
 * The send reads the context's packet buffer (lego_handoff_pack's) while it
 * is in flight: a lego_handoff_pack on the same context waits for that send
 * before it rewrites or regrows the buffer (the gather records a fence on the
 * context), so repacking in between is safe; lego_handoff_pack_into writes the
 * caller's buffer and does not wait. */
#define LEGO_COMM_DEVICE_RESULT 1u
int lego_comm_gather_handoff_ex(lego_comm* comm, lego_ctx* ctx, int32_t root, uint32_t flags);
/* Blocks until the last gather on the communicator has completed (within the
 * lego_comm_set_timeout bound, see lego_comm_create). */
int lego_comm_wait(lego_comm* comm);
/* On root after lego_comm_gather_handoff: rank r's packet in host memory,
 * valid until the next gather on the communicator. */
int lego_comm_handoff(lego_comm* comm, int32_t rank, const void** packet, uint64_t* bytes);
/* On root after either gather: rank r's packet in device memory (complete
 * once lego_comm_wait returns), valid until the next gather. */
int lego_comm_handoff_device(lego_comm* comm, int32_t rank, const void** dpacket, uint64_t* bytes);

/* pcl::VoxelGrid<PointXYZI> (leaf size `leaf`, downsample_all_data, no
 * field filter) of a host cloud on the context's device: the filter every
 * mapping VoxelGrid call runs (mapOptmization.cpp:1058-1091), including PCL's
 * std::sort order of each voxel's points.  out holds up to n points; *n_out
 * the voxels written.  Non-finite points are skipped, as PCL does for a cloud
 * that is not dense. */
int lego_voxel_grid(lego_ctx* ctx, const lego_point_xyzi* in, int32_t n, float leaf, lego_point_xyzi* out,
                    int32_t* n_out);
/* Counters of the last lego_voxel_grid: [0] finite points sorted, [1] voxels,
 * [2] partition rounds launched, [3] segments sorted in one workgroup,
 * [4] of them still above the workgroup size after the rounds, [5] heap-sorted
 * segments (depth budget spent), [6] non-finite points, [7] device time in
 * microseconds.  Diagnostics for tests and benchmarks. */
int lego_voxel_grid_stats(lego_ctx* ctx, int32_t stats[8]);
/* The permutation libstdc++'s std::sort gives (key, index) pairs compared by
 * key alone — the sort pcl::VoxelGrid::applyFilter runs on (voxel idx, point)
 * (voxel_grid.hpp; featureAssociation.cpp:778-782, mapOptmization.cpp:1058-1091),
 * whose order of equal keys is the VoxelGrid's summation order — computed on
 * the device: perm[i] = the input index at sorted position i.  wave = 0: the
 * workgroup sort the VoxelGrids use (n <= 8192); wave = 1: the one-wave sort
 * of the per-ring less-flat VoxelGrid (n <= 512).  wave = 2 / 3: the workgroup
 * sort as the VoxelGrids run it, with 256 threads (n <= 2048) / 1024 threads
 * (n <= 8192): heap-sorted pieces whose voxel sums do not depend on their
 * order (each key at most twice, the smallest not continuing the preceding
 * piece) come back in stable order instead of std::sort's, every other
 * position as std::sort leaves it.  Modes 4..8 cover the rest of the
 * workgroup sort's two forms (segment ids in registers, "reg", or in LDS,
 * "lds") by block size and rule, each compiled under the register budget of
 * the kernel that runs it (256 threads: k_lf_voxel's): 4 reg/256/exact,
 * 5 reg/256/sum-order, 6 lds/256/exact, 7 lds/1024/exact, 8 lds/1024/sum-order
 * (mode 0 = reg/1024/exact, 2 = lds/256/sum-order, 3 = reg/1024/sum-order).
 * 256-thread modes hold n <= 2048.  heap_pieces (may be NULL): how many pieces
 * the depth budget sent to std::__partial_sort. */
int lego_sort_permutation(lego_ctx* ctx, const uint32_t* keys, int32_t n, int32_t wave, int32_t* perm,
                          int32_t* heap_pieces);

/* Last device error string (static storage). */
const char* lego_last_error(void);

/* Per-stage device timings of the last lego_odom_batch call (ms), for bench:
 * names[i] / ms[i], i < *n. */
int lego_stage_times(lego_ctx* ctx, const char** names, float* ms, int32_t cap,
                     int32_t* n);

/* Diagnostic in-kernel phase counters of the odometry kernel (wall clock at
 * 100 MHz): enable = 1/0 turns stamping on/off and zeroes the counters,
 * enable = -1 leaves it unchanged; out32 (may be NULL) receives
 * {surf NN iters, surf iters, corner NN iters, corner iters, solve, integrate,
 *  to_end, NN grid build, LDS residency, #surf iters, #corner iters, #NN rounds,
 *  nn query, -, #shell-1 queries, #brute-force queries, then group-0 splits of
 *  the NN loop: to_start, grid NN, scan-line, #queries; 12 spare}. */
int lego_odom_profile(lego_ctx* ctx, int32_t enable, uint64_t* out32);
/* Diagnostic phase stamps of the feature-extraction kernel (one workgroup per
 * scan and ring), summed over workgroups while lego_odom_profile stamping is
 * on (wall clock at 100 MHz): {window load + sector sorts, picking walk,
 * picked copies + less-flat set, per-ring VoxelGrid, #rings, #sector
 * re-walks of the speculative picking, #rings picked speculatively, sum over
 * workgroups of the workgroups in flight when each started}. */
int lego_extract_profile(lego_ctx* ctx, uint64_t* out8);

#ifdef __cplusplus
}
#endif
#endif /* LEGO_LOAM_H_ */
