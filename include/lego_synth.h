/* lego_synth.h — deterministic synthetic lidar source.
 *
 * The reference is validated by replaying rosbags (README.md:90-106), which are
 * not available offline; this generator ray-casts a seeded scene instead and
 * emits scans in the velodyne PointCloud2 layout (lego_point_xyzir), in firing
 * order (column-major, ring inner), with intra-scan ego motion.  Own PRNG
 * (splitmix64) only — no std::*_distribution, whose output is
 * implementation-defined.
 */
#ifndef LEGO_SYNTH_H_
#define LEGO_SYNTH_H_
#include <stdint.h>
#include "lego_loam.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lego_synth_cfg {
  int32_t n_scan, horizon_scan;
  float vert_min_deg, vert_max_deg; /* ring r elevation: linear in r */
  float mount_height;               /* sensor height above the ground plane */
  float ground_tilt_deg;            /* max ground tilt */
  float noise_sigma;                /* range noise (m) */
  float dropout;                    /* fraction of returns dropped */
  float max_range;                  /* no return beyond */
  float dup_frac;                   /* fraction of re-fired (colliding) points */
  float azimuth_jitter;             /* fraction of a column */
  float speed_mps, yaw_rate_dps, scan_period;
  int32_t n_boxes, n_cylinders, n_walls;
  uint64_t seed;
} lego_synth_cfg;

/* "VLP-16", "HDL-64E", "VLS-128" (SURVEY.md §8d C1-C5), and the reference's
 * other presets "HDL-32E", "OS1-16", "OS1-64" (utility.h:70-102). */
int lego_synth_preset(const char* name, uint64_t seed, lego_synth_cfg* out);
/* Upper bound on the points of one scan. */
int32_t lego_synth_max_points(const lego_synth_cfg* cfg);
/* Scan `scan_index` of the stream: stamp = scan_index * scan_period. */
int lego_synth_scan(const lego_synth_cfg* cfg, int32_t scan_index,
                    lego_point_xyzir* out, int32_t cap, int32_t* n_out,
                    double* stamp);
/* /imu_raw messages of the same ego motion at rate_hz, stamps
 * phase + i / rate_hz within [t0, t1): orientation (ego yaw plus a small
 * roll / pitch sway), gyro and accelerometer (specific force incl. gravity)
 * in the ROS body frame (x forward, y left, z up), with seeded noise. */
int lego_synth_imu(const lego_synth_cfg* cfg, double t0, double t1, double rate_hz, double phase,
                   lego_imu_msg* out, int32_t cap, int32_t* n_out);
/* Config-5 surrounding map: planes (surf, ~0.4 m spacing) and vertical edges
 * (corner, ~0.2 m spacing) within `radius` of the origin, in the mapping
 * frame (camera convention: x left, y up, z forward as in
 * featureAssociation.cpp:500-502). */
int lego_synth_map(uint64_t seed, float radius, int32_t n_surf, int32_t n_corner,
                   lego_point_xyzi* surf, lego_point_xyzi* corner);

#ifdef __cplusplus
}
#endif
#endif
