/* Prints sizeof/offsetof of the C-ABI structs (include/lego_loam.h,
 * include/lego_synth.h) so tests/test_abi.py can check the ctypes mirror. */
#include <stddef.h>
#include <stdio.h>
#include "lego_loam.h"
#include "lego_synth.h"
#define S(t) printf(#t " %zu\n", sizeof(t))
#define O(t, f) printf(#t "." #f " %zu\n", offsetof(t, f))
int main(void) {
  S(lego_point_xyzir); O(lego_point_xyzir, intensity); O(lego_point_xyzir, ring);
  S(lego_point_xyzi);
  S(lego_sensor_cfg); O(lego_sensor_cfg, mapping_process_interval); O(lego_sensor_cfg, skip_frame_num);
  S(lego_cloud_info); O(lego_cloud_info, segmented_cloud_range);
  S(lego_ip_out); O(lego_ip_out, n_segmented); O(lego_ip_out, label_image);
  O(lego_ip_out, full_info_cloud); O(lego_ip_out, n_ground); O(lego_ip_out, n_segmented_pure);
  S(lego_fa_out); O(lego_fa_out, odom_valid); O(lego_fa_out, odom_quat); O(lego_fa_out, publish_to_mapping);
  O(lego_fa_out, n_outlier_last);
  S(lego_mo_out); O(lego_mo_out, transform_bef_mapped); O(lego_mo_out, n_rows_last);
  S(lego_pose_rec); O(lego_pose_rec, n_segmented); O(lego_pose_rec, flags);
  S(lego_loop_out); O(lego_loop_out, fitness); O(lego_loop_out, icp_transform); O(lego_loop_out, from_rotation);
  O(lego_loop_out, between_translation);
  S(lego_mo_opts); O(lego_mo_opts, loop_closure_enable); O(lego_mo_opts, surrounding_keyframe_search_num);
  S(lego_synth_cfg); O(lego_synth_cfg, seed);
  S(lego_ctx_opts); O(lego_ctx_opts, lf_wait_ms); O(lego_ctx_opts, mo_evprof); O(lego_ctx_opts, reserved);
  return 0;
}
