// lego_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
// hot path, used as the parity checker by tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg.  Never linked into the product.
//
// PARITY STATUS: "parity unpinned" against the reference binary — the
// reference cannot be built here (needs ROS, PCL, OpenCV, GTSAM; SURVEY.md
// §8c) and ships no tests or golden vectors.  What IS pinned:
// the libm shim it uses (bit-exact vs this host's glibc, tests/test_numerics_shim.py),
// libstdc++ std::sort (called directly, the same library the reference links),
// and hand-derived known-answer tests (tests/test_oracle_kat.py).
#pragma once
#include "lego_loam.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lego_oracle lego_oracle;

int lego_oracle_sensor_preset(const char* name, lego_sensor_cfg* out);
int lego_oracle_create(const lego_sensor_cfg* cfg, lego_oracle** out);
int lego_oracle_destroy(lego_oracle* o);
/* Options: the VoxelGrid in-voxel summation order.  Bit 0: featureAssociation's
 * per-ring VoxelGrid (featureAssociation.cpp:778-780), bit 1: mapOptimization's
 * VoxelGrids (mapOptmization.cpp:1058-1091, 1363).  A set bit sums each voxel
 * in PCL's order (std::sort of (idx, point) by idx, unstable: the reference's
 * behaviour), a clear bit in input order (std::stable_sort).  The default
 * (LEGO_ORACLE_DEFAULT_OPTS) is the product's: both bits set. */
#define LEGO_ORACLE_VG_FA 1u
#define LEGO_ORACLE_VG_MO 2u
#define LEGO_ORACLE_DEFAULT_OPTS (LEGO_ORACLE_VG_FA | LEGO_ORACLE_VG_MO)
int lego_oracle_set_options(lego_oracle* o, uint32_t opts);
int lego_oracle_ip_process(lego_oracle* o, const lego_point_xyzir* pts, int32_t n,
                           double stamp, uint32_t flags, lego_ip_out* out);
int lego_oracle_fa_process(lego_oracle* o, const lego_ip_out* in, lego_fa_out* out);
int lego_oracle_mo_set_map(lego_oracle* o, const lego_point_xyzi* corner, int32_t n_corner,
                           const lego_point_xyzi* surf, int32_t n_surf);
int lego_oracle_mo_process(lego_oracle* o, const lego_fa_out* in, lego_mo_out* out);
int lego_oracle_mo_loop_closure(lego_oracle* o, lego_loop_out* out);
int lego_oracle_mo_configure(lego_oracle* o, const lego_mo_opts* opts);
/* transformFusion's two handlers. */
int lego_oracle_fusion_odometry(lego_oracle* o, const lego_fa_out* odom, lego_fusion_out* out);
int lego_oracle_fusion_aft_mapped(lego_oracle* o, const lego_mo_out* mo);
/* /imu_raw messages delivered to both nodes' imuHandlers, in order. */
int lego_oracle_imu_push(lego_oracle* o, const lego_imu_msg* msgs, int32_t n);

/* LM statistics: scans, surf iterations, corner iterations, NN rounds, rows. */
int lego_oracle_stats(lego_oracle* o, long* out5);

/* Diagnostic: record the dense systems handed to the OpenCV-shaped solvers
 * (kind 0: odometry AtA|AtB 12 floats; 1: mapping AtA|AtB 42; 2: mapping
 * plane-fit A0 15; 3: mapping corner covariance 9), up to 4096 per kind.
 * enable resets the log.  lego_oracle_systems copies up to cap floats of a
 * kind and reports the total in *n. */
int lego_oracle_log_systems(lego_oracle* o, int32_t enable);
int lego_oracle_systems(lego_oracle* o, int32_t kind, float* out, int32_t cap, int32_t* n);

/* Stand-alone pieces for known-answer tests. */
int lego_oracle_voxel_grid(const lego_point_xyzi* in, int32_t n, float leaf,
                           int32_t pcl_sort, lego_point_xyzi* out, int32_t* n_out);
/* libstdc++'s std::sort of (key, index) pairs by key (PCL VoxelGrid's
 * sort): perm[i] = the index at sorted position i. */
int lego_oracle_sort_permutation(const uint32_t* keys, int32_t n, int32_t* perm);
float lego_oracle_atan2f(float y, float x);
float lego_oracle_sinf(float x);
float lego_oracle_cosf(float x);
float lego_oracle_asinf(float x);

#ifdef __cplusplus
}
#endif
