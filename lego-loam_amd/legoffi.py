"""ctypes bindings for the lego C-ABI (include/lego_loam.h, include/lego_synth.h).

This is the Python face of the drop-in boundary: the same struct layouts a
ROS adapter would bind, used by tests/ and bench.py.

Libraries (all built in-tree by __graft_entry__.build()):
  lego-loam_amd/build/liblego_hip.so    product: HIP kernels + C-ABI
  lego-loam_amd/build/liblego_synth.so  synthetic lidar source
  oracle/build/liblego_oracle.so        CPU oracle (tests / cpu_baseline only)
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import weakref
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
BUILD = PKG_DIR / "build"
HIP_LIB = BUILD / "liblego_hip.so"
if os.environ.get("LEGO_HIP_LIB_AB"):  # A/B timing of two builds on one box (scripts/ab.sh); diagnostic
    HIP_LIB = Path(os.environ["LEGO_HIP_LIB_AB"]).resolve()
SYNTH_LIB = BUILD / "liblego_synth.so"
ORACLE_LIB = REPO / "oracle" / "build" / "liblego_oracle.so"

LEGO_OK, LEGO_E_NOT_DENSE, LEGO_E_CAPACITY, LEGO_E_DEVICE, LEGO_E_ARG, LEGO_E_STATE = range(6)
LEGO_IP_IMAGES = 1
LEGO_IP_GATED = 2

f32p = C.POINTER(C.c_float)


class PointXYZIR(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("_pad0", C.c_float),
                ("intensity", C.c_float), ("ring", C.c_uint16), ("_pad1", C.c_uint16),
                ("_pad2", C.c_uint32 * 2)]


class PointXYZI(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("intensity", C.c_float)]


XYZIR_DTYPE = np.dtype({"names": ["x", "y", "z", "_pad0", "intensity", "ring", "_pad1", "_pad2"],
                        "formats": ["<f4", "<f4", "<f4", "<f4", "<f4", "<u2", "<u2", ("<u4", 2)],
                        "offsets": [0, 4, 8, 12, 16, 20, 22, 24], "itemsize": 32})
XYZI_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("intensity", "<f4")])
assert C.sizeof(PointXYZIR) == 32 and C.sizeof(PointXYZI) == 16


class SensorCfg(C.Structure):
    _fields_ = [("n_scan", C.c_int32), ("horizon_scan", C.c_int32), ("ang_res_x", C.c_float),
                ("ang_res_y", C.c_float), ("ang_bottom", C.c_float), ("ground_scan_ind", C.c_int32),
                ("use_cloud_ring", C.c_int32), ("sensor_minimum_range", C.c_float),
                ("sensor_mount_angle", C.c_float), ("segment_theta", C.c_float),
                ("segment_valid_point_num", C.c_int32), ("segment_valid_line_num", C.c_int32),
                ("segment_alpha_x", C.c_float), ("segment_alpha_y", C.c_float),
                ("edge_threshold", C.c_float), ("surf_threshold", C.c_float),
                ("nearest_feature_search_sq_dist", C.c_float), ("scan_period", C.c_float),
                ("mapping_process_interval", C.c_double),
                ("surrounding_keyframe_search_radius", C.c_float), ("skip_frame_num", C.c_int32)]


class CloudInfo(C.Structure):
    _fields_ = [("stamp", C.c_double), ("start_ring_index", C.POINTER(C.c_int32)),
                ("end_ring_index", C.POINTER(C.c_int32)), ("start_orientation", C.c_float),
                ("end_orientation", C.c_float), ("orientation_diff", C.c_float),
                ("segmented_cloud_ground_flag", C.POINTER(C.c_uint8)),
                ("segmented_cloud_col_ind", C.POINTER(C.c_uint32)),
                ("segmented_cloud_range", f32p)]


class IpOut(C.Structure):
    _fields_ = [("info", CloudInfo), ("segmented_cloud", C.POINTER(PointXYZI)),
                ("n_segmented", C.c_int32), ("outlier_cloud", C.POINTER(PointXYZI)),
                ("n_outlier", C.c_int32), ("full_cloud", C.POINTER(PointXYZI)),
                ("range_image", f32p), ("ground_image", C.POINTER(C.c_int8)),
                ("label_image", C.POINTER(C.c_int32)),
                ("full_info_cloud", C.POINTER(PointXYZI)), ("ground_cloud", C.POINTER(PointXYZI)),
                ("n_ground", C.c_int32), ("segmented_cloud_pure", C.POINTER(PointXYZI)),
                ("n_segmented_pure", C.c_int32)]


class FaOut(C.Structure):
    _fields_ = [("stamp", C.c_double),
                ("sharp", C.POINTER(PointXYZI)), ("n_sharp", C.c_int32),
                ("less_sharp", C.POINTER(PointXYZI)), ("n_less_sharp", C.c_int32),
                ("flat", C.POINTER(PointXYZI)), ("n_flat", C.c_int32),
                ("less_flat", C.POINTER(PointXYZI)), ("n_less_flat", C.c_int32),
                ("odom_valid", C.c_int32), ("transform_cur", C.c_float * 6),
                ("transform_sum", C.c_float * 6), ("odom_quat", C.c_double * 4),
                ("odom_pos", C.c_double * 3), ("publish_to_mapping", C.c_int32),
                ("corner_last", C.POINTER(PointXYZI)), ("n_corner_last", C.c_int32),
                ("surf_last", C.POINTER(PointXYZI)), ("n_surf_last", C.c_int32),
                ("outlier_last", C.POINTER(PointXYZI)), ("n_outlier_last", C.c_int32)]


class MoOut(C.Structure):
    _fields_ = [("processed", C.c_int32), ("optimized", C.c_int32), ("iterations", C.c_int32),
                ("transform_tobe_mapped", C.c_float * 6), ("transform_aft_mapped", C.c_float * 6),
                ("transform_bef_mapped", C.c_float * 6), ("n_corner_map_ds", C.c_int32),
                ("n_surf_map_ds", C.c_int32), ("n_corner_scan_ds", C.c_int32),
                ("n_surf_scan_ds", C.c_int32), ("n_rows_last", C.c_int32)]


class MoOpts(C.Structure):  # lego_mo_opts
    _fields_ = [("fixed_map_per_step", C.c_int32), ("loop_closure_enable", C.c_int32),
                ("surrounding_keyframe_search_num", C.c_int32), ("_pad", C.c_int32)]


class LoopOut(C.Structure):  # lego_loop_out (performLoopClosure)
    _fields_ = [("detected", C.c_int32), ("converged", C.c_int32), ("accepted", C.c_int32),
                ("latest_id", C.c_int32), ("closest_id", C.c_int32), ("iterations", C.c_int32),
                ("n_source", C.c_int32), ("n_target", C.c_int32), ("fitness", C.c_double),
                ("icp_transform", C.c_float * 16), ("from_rotation", C.c_double * 9),
                ("from_translation", C.c_double * 3), ("to_rotation", C.c_double * 9),
                ("to_translation", C.c_double * 3), ("between_rotation", C.c_double * 9),
                ("between_translation", C.c_double * 3)]


def loop_to_dict(o: LoopOut) -> dict:
    return {k: (np.array(list(getattr(o, k))) if isinstance(getattr(o, k), C.Array) else getattr(o, k))
            for k, _ in LoopOut._fields_}


class FusionOut(C.Structure):  # lego_fusion_out (/integrated_to_init)
    _fields_ = [("stamp", C.c_double), ("transform_mapped", C.c_float * 6), ("quat", C.c_double * 4),
                ("pos", C.c_double * 3)]


class PoseRec(C.Structure):
    _fields_ = [("stamp", C.c_double), ("transform_sum", C.c_float * 6),
                ("n_segmented", C.c_int32), ("n_sharp", C.c_int32), ("n_less_sharp", C.c_int32),
                ("n_flat", C.c_int32), ("n_less_flat", C.c_int32), ("odom_valid", C.c_int32),
                ("flags", C.c_int32), ("_pad", C.c_int32)]


assert C.sizeof(PoseRec) == 64


class HandoffHdr(C.Structure):  # lego_handoff_hdr
    _fields_ = [("magic", C.c_uint32), ("version", C.c_uint32), ("nscans", C.c_int32), ("npub", C.c_int32),
                ("bytes", C.c_uint64), ("_pad", C.c_uint64)]


class HandoffScan(C.Structure):  # lego_handoff_scan
    _fields_ = [("rec", PoseRec), ("transform_cur", C.c_float * 6), ("publish_to_mapping", C.c_int32),
                ("n_corner_last", C.c_int32), ("n_surf_last", C.c_int32), ("n_outlier_last", C.c_int32),
                ("offset", C.c_uint64), ("_pad", C.c_uint64 * 2)]


assert C.sizeof(HandoffHdr) == 32 and C.sizeof(HandoffScan) == 128
HANDOFF_MAGIC = 0x4F48474C


# lego_imu_msg (include/lego_loam.h): the sensor_msgs/Imu fields the handlers read
IMU_DTYPE = np.dtype([("stamp", np.float64), ("orientation", np.float64, 4),
                      ("angular_velocity", np.float64, 3), ("linear_acceleration", np.float64, 3)])
assert IMU_DTYPE.itemsize == 88


class Pc2Field(C.Structure):  # lego_pc2_field (sensor_msgs/PointField)
    _fields_ = [("name", C.c_char * 16), ("offset", C.c_uint32), ("datatype", C.c_uint8),
                ("count", C.c_uint32)]


class Pc2Msg(C.Structure):  # lego_pc2_msg (sensor_msgs/PointCloud2)
    _fields_ = [("stamp", C.c_double), ("height", C.c_uint32), ("width", C.c_uint32),
                ("point_step", C.c_uint32), ("row_step", C.c_uint32), ("is_bigendian", C.c_uint8),
                ("is_dense", C.c_uint8), ("n_fields", C.c_int32), ("fields", C.POINTER(Pc2Field)),
                ("data", C.c_void_p)]


PF = {"INT8": 1, "UINT8": 2, "INT16": 3, "UINT16": 4, "INT32": 5, "UINT32": 6, "FLOAT32": 7, "FLOAT64": 8}


def pc2_msg(data: np.ndarray, fields: list[tuple[str, int, int, int]], point_step: int, width: int,
            height: int = 1, row_step: int | None = None, stamp: float = 0.0, is_dense: int = 1,
            is_bigendian: int = 0):
    """A Pc2Msg over the uint8 buffer `data` (kept alive by the caller);
    fields: (name, offset, datatype, count)."""
    arr = (Pc2Field * max(1, len(fields)))()
    for i, (nm, off, dt, cnt) in enumerate(fields):
        arr[i].name = nm.encode()
        arr[i].offset = off
        arr[i].datatype = dt
        arr[i].count = cnt
    m = Pc2Msg()
    m.stamp = stamp
    m.height, m.width, m.point_step = height, width, point_step
    m.row_step = row_step if row_step is not None else width * point_step
    m.is_bigendian, m.is_dense = is_bigendian, is_dense
    m.n_fields = len(fields)
    m.fields = C.cast(arr, C.POINTER(Pc2Field))
    m.data = data.ctypes.data
    m._keep = (arr, data)
    return m


class SynthCfg(C.Structure):
    _fields_ = [("n_scan", C.c_int32), ("horizon_scan", C.c_int32), ("vert_min_deg", C.c_float),
                ("vert_max_deg", C.c_float), ("mount_height", C.c_float),
                ("ground_tilt_deg", C.c_float), ("noise_sigma", C.c_float),
                ("dropout", C.c_float), ("max_range", C.c_float), ("dup_frac", C.c_float),
                ("azimuth_jitter", C.c_float), ("speed_mps", C.c_float),
                ("yaw_rate_dps", C.c_float), ("scan_period", C.c_float), ("n_boxes", C.c_int32),
                ("n_cylinders", C.c_int32), ("n_walls", C.c_int32), ("seed", C.c_uint64)]


# ------------------------------------------------------------------ loading
_libs: dict[str, C.CDLL] = {}


def _load(path: Path, key: str) -> C.CDLL:
    if key not in _libs:
        if not path.exists():
            raise RuntimeError(f"{path} is not built; run __graft_entry__.build()")
        _libs[key] = C.CDLL(str(path))
    return _libs[key]


def synth_lib() -> C.CDLL:
    lib = _load(SYNTH_LIB, "synth")
    lib.lego_synth_preset.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(SynthCfg)]
    lib.lego_synth_max_points.argtypes = [C.POINTER(SynthCfg)]
    lib.lego_synth_max_points.restype = C.c_int32
    lib.lego_synth_scan.argtypes = [C.POINTER(SynthCfg), C.c_int32, C.c_void_p, C.c_int32,
                                    C.POINTER(C.c_int32), C.POINTER(C.c_double)]
    lib.lego_synth_map.argtypes = [C.c_uint64, C.c_float, C.c_int32, C.c_int32, C.c_void_p,
                                   C.c_void_p]
    lib.lego_synth_imu.argtypes = [C.POINTER(SynthCfg), C.c_double, C.c_double, C.c_double, C.c_double,
                                   C.c_void_p, C.c_int32, C.POINTER(C.c_int32)]
    return lib


def oracle_lib() -> C.CDLL:
    """TEST INFRASTRUCTURE: the CPU oracle.  Only tests/, smoke() and bench's
    cpu_baseline leg may call this."""
    lib = _load(ORACLE_LIB, "oracle")
    lib.lego_oracle_sensor_preset.argtypes = [C.c_char_p, C.POINTER(SensorCfg)]
    lib.lego_oracle_create.argtypes = [C.POINTER(SensorCfg), C.POINTER(C.c_void_p)]
    lib.lego_oracle_sort_permutation.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    lib.lego_oracle_destroy.argtypes = [C.c_void_p]
    lib.lego_oracle_set_options.argtypes = [C.c_void_p, C.c_uint32]
    lib.lego_oracle_ip_process.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_double,
                                           C.c_uint32, C.POINTER(IpOut)]
    lib.lego_oracle_fa_process.argtypes = [C.c_void_p, C.POINTER(IpOut), C.POINTER(FaOut)]
    lib.lego_oracle_mo_set_map.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]
    lib.lego_oracle_mo_process.argtypes = [C.c_void_p, C.POINTER(FaOut), C.POINTER(MoOut)]
    lib.lego_oracle_mo_loop_closure.argtypes = [C.c_void_p, C.POINTER(LoopOut)]
    lib.lego_oracle_mo_configure.argtypes = [C.c_void_p, C.POINTER(MoOpts)]
    lib.lego_oracle_imu_push.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    lib.lego_oracle_fusion_odometry.argtypes = [C.c_void_p, C.POINTER(FaOut), C.POINTER(FusionOut)]
    lib.lego_oracle_fusion_aft_mapped.argtypes = [C.c_void_p, C.POINTER(MoOut)]
    lib.lego_oracle_log_systems.argtypes = [C.c_void_p, C.c_int32]
    lib.lego_oracle_systems.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)]
    lib.lego_oracle_voxel_grid.argtypes = [C.c_void_p, C.c_int32, C.c_float, C.c_int32,
                                           C.c_void_p, C.POINTER(C.c_int32)]
    for fn in ("atan2f",):
        getattr(lib, "lego_oracle_" + fn).argtypes = [C.c_float, C.c_float]
        getattr(lib, "lego_oracle_" + fn).restype = C.c_float
    for fn in ("sinf", "cosf", "asinf"):
        getattr(lib, "lego_oracle_" + fn).argtypes = [C.c_float]
        getattr(lib, "lego_oracle_" + fn).restype = C.c_float
    return lib


class CtxOpts(C.Structure):
    """lego_ctx_opts (include/lego_loam.h): a context's scheduling and
    diagnostic switches, fixed at creation."""
    _fields_ = [(n, C.c_int32) for n in (
        "size", "node_overlap", "front_parts", "lfv_wave", "lfv_block_rings", "lfv_wide", "ccl_tiles",
        "seg_hbm", "odom_workgroups", "odom_gridless", "odom_integ", "odom_silent_wg", "odom_late_wg",
        "lf_wait_ms", "mo_cand_cache", "kf_cap", "vg_rounds", "fa_synccheck", "mo_hostprof", "mo_evprof",
        "ip_fused")] + [("reserved", C.c_int32 * 11)]


# Tooling only (bench.py, scripts/): the A/B scripts switch a context's
# options through the environment; the library itself reads none.
ENV_OPTS = {"LEGO_NODE_OVERLAP": "node_overlap", "LEGO_FRONT_PARTS": "front_parts", "LEGO_LFV_WAVE": "lfv_wave",
            "LEGO_LFV_BLOCK_RINGS": "lfv_block_rings", "LEGO_LFV_WIDE": "lfv_wide", "LEGO_CCL_TILES": "ccl_tiles",
            "LEGO_SEG_HBM": "seg_hbm", "LEGO_ODOM_WORKGROUPS": "odom_workgroups",
            "LEGO_ODOM_GRIDLESS": "odom_gridless", "LEGO_ODOM_INTEG": "odom_integ",
            "LEGO_ODOM_SILENT_WG": "odom_silent_wg", "LEGO_ODOM_LATE_WG": "odom_late_wg",
            "LEGO_MO_CAND": "mo_cand_cache", "LEGO_KF_CAP": "kf_cap", "LEGO_VG_ROUNDS": "vg_rounds",
            "LEGO_FA_SYNCCHECK": "fa_synccheck", "LEGO_MO_HOSTPROF": "mo_hostprof", "LEGO_MO_EVPROF": "mo_evprof",
            "LEGO_IP_FUSED": "ip_fused"}


def opts_from_env() -> dict:
    """The LEGO_* A/B variables of the tooling's environment as option values."""
    return {f: int(os.environ[e]) for e, f in ENV_OPTS.items() if os.environ.get(e, "") != ""}


def ctx_opts(lib: C.CDLL | None = None, **over) -> CtxOpts:
    lib = lib or hip_lib()
    o = CtxOpts()
    lib.lego_ctx_opts_init(C.byref(o))
    for k, v in over.items():
        setattr(o, k, int(v))
    return o


HIP_EXPORTS = ["lego_sensor_preset", "lego_create", "lego_fleet_create", "lego_destroy", "lego_reset",
               "lego_ctx_opts_init", "lego_create_ex", "lego_fleet_create_ex", "lego_comm_set_timeout",
               "lego_ip_process", "lego_fa_process", "lego_odom_batch", "lego_odom_batch_imu",
               "lego_imu_push", "lego_odom_batch_submit", "lego_odom_batch_wait", "lego_batch_fetch", "lego_pc2_decode", "lego_ip_process_pc2",
               "lego_odom_batch_pc2", "lego_pc2_encode_xyzi", "lego_cloud_info_serialize",
               "lego_fusion_odometry", "lego_fusion_aft_mapped",
               "lego_mo_set_map", "lego_mo_configure", "lego_mo_process", "lego_mo_loop_closure", "lego_last_error", "lego_stage_times",
               "lego_odom_profile", "lego_extract_profile", "lego_handoff_pack", "lego_handoff_pack_into", "lego_handoff_unpack", "lego_comm_unique_id",
               "lego_comm_create", "lego_comm_destroy", "lego_comm_gather_handoff", "lego_comm_handoff",
               "lego_comm_gather_handoff_ex", "lego_comm_wait", "lego_comm_handoff_device", "lego_comm_abort",
               "lego_comm_count", "lego_voxel_grid", "lego_voxel_grid_stats", "lego_sort_permutation"]


def hip_lib() -> C.CDLL:
    """The product library.  Loading never falls back to anything else."""
    lib = _load(HIP_LIB, "hip")
    lib.lego_sensor_preset.argtypes = [C.c_char_p, C.POINTER(SensorCfg)]
    lib.lego_create.argtypes = [C.POINTER(SensorCfg), C.c_int, C.c_int32, C.c_int32,
                                C.POINTER(C.c_void_p)]
    lib.lego_fleet_create.argtypes = [C.POINTER(SensorCfg), C.c_int, C.c_int32, C.c_int32, C.c_int32,
                                      C.POINTER(C.c_void_p)]
    lib.lego_ctx_opts_init.argtypes = [C.POINTER(CtxOpts)]
    lib.lego_ctx_opts_init.restype = None
    lib.lego_create_ex.argtypes = [C.POINTER(SensorCfg), C.c_int, C.c_int32, C.c_int32, C.POINTER(CtxOpts),
                                   C.POINTER(C.c_void_p)]
    lib.lego_fleet_create_ex.argtypes = [C.POINTER(SensorCfg), C.c_int, C.c_int32, C.c_int32, C.c_int32,
                                         C.POINTER(CtxOpts), C.POINTER(C.c_void_p)]
    lib.lego_comm_set_timeout.argtypes = [C.c_void_p, C.c_int32]
    lib.lego_destroy.argtypes = [C.c_void_p]
    lib.lego_reset.argtypes = [C.c_void_p]
    lib.lego_ip_process.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_double, C.c_uint32,
                                    C.POINTER(IpOut)]
    lib.lego_fa_process.argtypes = [C.c_void_p, C.POINTER(IpOut), C.POINTER(FaOut)]
    lib.lego_odom_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                    C.c_int32, C.c_void_p]
    lib.lego_odom_batch_imu.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                        C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
    lib.lego_imu_push.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    lib.lego_fusion_odometry.argtypes = [C.c_void_p, C.POINTER(FaOut), C.POINTER(FusionOut)]
    lib.lego_fusion_aft_mapped.argtypes = [C.c_void_p, C.POINTER(MoOut)]
    lib.lego_odom_batch_submit.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                           C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
    lib.lego_odom_batch_wait.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)]
    lib.lego_pc2_decode.argtypes = [C.c_void_p, C.POINTER(Pc2Msg), C.c_void_p, C.c_int32, C.POINTER(C.c_int32)]
    lib.lego_ip_process_pc2.argtypes = [C.c_void_p, C.POINTER(Pc2Msg), C.c_uint32, C.POINTER(IpOut)]
    lib.lego_odom_batch_pc2.argtypes = [C.c_void_p, C.POINTER(Pc2Msg), C.c_int32, C.c_int32, C.c_void_p]
    lib.lego_pc2_encode_xyzi.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.POINTER(Pc2Field)]
    lib.lego_cloud_info_serialize.argtypes = [C.POINTER(CloudInfo), C.c_int32, C.c_int32, C.c_uint32,
                                              C.c_char_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    lib.lego_batch_fetch.argtypes = [C.c_void_p, C.c_int32, C.POINTER(IpOut), C.POINTER(FaOut)]
    lib.lego_mo_set_map.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]
    lib.lego_mo_process.argtypes = [C.c_void_p, C.POINTER(FaOut), C.POINTER(MoOut)]
    lib.lego_mo_configure.argtypes = [C.c_void_p, C.POINTER(MoOpts)]
    lib.lego_mo_loop_closure.argtypes = [C.c_void_p, C.POINTER(LoopOut)]
    lib.lego_handoff_pack.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
    lib.lego_handoff_pack_into.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    lib.lego_handoff_unpack.argtypes = [C.c_void_p, C.c_uint64, C.c_int32, C.POINTER(PoseRec), C.POINTER(FaOut)]
    lib.lego_comm_unique_id.argtypes = [C.c_void_p]
    lib.lego_comm_create.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
    lib.lego_comm_destroy.argtypes = [C.c_void_p]
    lib.lego_comm_gather_handoff.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    lib.lego_comm_handoff.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
    lib.lego_comm_gather_handoff_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_uint32]
    lib.lego_comm_wait.argtypes = [C.c_void_p]
    lib.lego_comm_abort.argtypes = [C.c_void_p]
    lib.lego_comm_count.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
    lib.lego_comm_handoff_device.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
    lib.lego_voxel_grid.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_float, C.c_void_p,
                                    C.POINTER(C.c_int32)]
    lib.lego_voxel_grid_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
    lib.lego_sort_permutation.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                          C.POINTER(C.c_int32)]
    lib.lego_last_error.restype = C.c_char_p
    lib.lego_odom_profile.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    lib.lego_extract_profile.argtypes = [C.c_void_p, C.c_void_p]
    lib.lego_stage_times.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), f32p, C.c_int32,
                                     C.POINTER(C.c_int32)]
    return lib


_hiprt = None


def hip_memcpy_d2h(dst: int, src: int, n: int) -> int:
    """hipMemcpy device -> host through the HIP runtime already loaded."""
    global _hiprt
    if _hiprt is None:
        hip_lib()  # the runtime liblego_hip.so links is then loaded: take that one
        for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
            try:
                _hiprt = C.CDLL(name)
                break
            except OSError:
                continue
        if _hiprt is None:
            raise OSError("no HIP runtime (libamdhip64.so) to copy the packet with")
        _hiprt.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    return _hiprt.hipMemcpy(C.c_void_p(dst), C.c_void_p(src), n, 2)  # hipMemcpyDeviceToHost


def handoff_unpack(packet: np.ndarray, k: int, lib: C.CDLL | None = None) -> tuple:
    """lego_handoff_unpack of scan k of a host packet: (PoseRec, fa dict)."""
    lib = lib or hip_lib()
    rec, fa = PoseRec(), FaOut()
    packet = np.ascontiguousarray(packet, np.uint8)
    check(lib.lego_handoff_unpack(packet.ctypes.data, packet.nbytes, k, C.byref(rec), C.byref(fa)),
          "lego_handoff_unpack", lib)
    return rec, fa_to_dict(fa)


def handoff_header(packet: np.ndarray) -> HandoffHdr:
    return HandoffHdr.from_buffer_copy(bytes(packet[:C.sizeof(HandoffHdr)]))


def check(st: int, what: str, lib: C.CDLL | None = None) -> None:
    if st != LEGO_OK:
        msg = ""
        if lib is not None and hasattr(lib, "lego_last_error"):
            try:
                msg = (lib.lego_last_error() or b"").decode()
            except Exception:  # noqa: BLE001
                msg = ""
        raise RuntimeError(f"{what} failed with status {st} {msg}")


# ------------------------------------------------------------------ helpers
def synth_cfg(name: str = "VLP-16", seed: int = 0, **over) -> SynthCfg:
    lib = synth_lib()
    cfg = SynthCfg()
    check(lib.lego_synth_preset(name.encode(), seed, C.byref(cfg)), "synth_preset")
    for k, v in over.items():
        setattr(cfg, k, v)
    return cfg


def synth_scan(cfg: SynthCfg, k: int) -> tuple[np.ndarray, float]:
    lib = synth_lib()
    cap = lib.lego_synth_max_points(C.byref(cfg))
    buf = np.zeros(cap, dtype=XYZIR_DTYPE)
    n = C.c_int32()
    st = C.c_double()
    check(lib.lego_synth_scan(C.byref(cfg), k, buf.ctypes.data, cap, C.byref(n), C.byref(st)),
          "synth_scan")
    return buf[: n.value].copy(), st.value


def synth_imu(cfg: SynthCfg, t0: float, t1: float, rate_hz: float = 100.0,
              phase: float = 0.0037) -> np.ndarray:
    """/imu_raw messages of the synthetic ego motion with stamps in [t0, t1)."""
    lib = synth_lib()
    cap = int((t1 - t0) * rate_hz) + 2
    buf = np.zeros(cap, dtype=IMU_DTYPE)
    n = C.c_int32()
    check(lib.lego_synth_imu(C.byref(cfg), t0, t1, rate_hz, phase, buf.ctypes.data, cap, C.byref(n)),
          "synth_imu")
    return buf[: n.value].copy()


def synth_map(seed: int, radius: float, n_surf: int, n_corner: int):
    lib = synth_lib()
    surf = np.zeros(n_surf, dtype=XYZI_DTYPE)
    corner = np.zeros(n_corner, dtype=XYZI_DTYPE)
    check(lib.lego_synth_map(seed, radius, n_surf, n_corner, surf.ctypes.data, corner.ctypes.data),
          "synth_map")
    return surf, corner


def sensor_cfg(name: str = "VLP-16", lib: C.CDLL | None = None) -> SensorCfg:
    lib = lib or oracle_lib()
    cfg = SensorCfg()
    fn = lib.lego_sensor_preset if hasattr(lib, "lego_sensor_preset") else lib.lego_oracle_sensor_preset
    check(fn(name.encode(), C.byref(cfg)), "sensor_preset")
    return cfg


def _arr(ptr, n, dtype):
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(n * np.dtype(dtype).itemsize,)).view(dtype).copy()


def ip_to_dict(o: IpOut, cfg: SensorCfg, images: bool = False) -> dict:
    P = cfg.n_scan * cfg.horizon_scan
    ns = o.n_segmented
    d = {
        "start_orientation": o.info.start_orientation,
        "end_orientation": o.info.end_orientation,
        "orientation_diff": o.info.orientation_diff,
        "start_ring_index": _arr(o.info.start_ring_index, cfg.n_scan, np.int32),
        "end_ring_index": _arr(o.info.end_ring_index, cfg.n_scan, np.int32),
        "ground_flag": _arr(o.info.segmented_cloud_ground_flag, ns, np.uint8),
        "col_ind": _arr(o.info.segmented_cloud_col_ind, ns, np.uint32),
        "range": _arr(o.info.segmented_cloud_range, ns, np.float32),
        "segmented": _arr(o.segmented_cloud, ns, XYZI_DTYPE),
        "outlier": _arr(o.outlier_cloud, o.n_outlier, XYZI_DTYPE),
    }
    if images:
        d["range_image"] = _arr(o.range_image, P, np.float32)
        d["ground_image"] = _arr(o.ground_image, P, np.int8)
        d["label_image"] = _arr(o.label_image, P, np.int32)
        d["full_cloud"] = _arr(o.full_cloud, P, XYZI_DTYPE)
    if o.full_info_cloud:  # LEGO_IP_GATED
        d["full_info_cloud"] = _arr(o.full_info_cloud, P, XYZI_DTYPE)
        d["ground_cloud"] = _arr(o.ground_cloud, o.n_ground, XYZI_DTYPE)
        d["segmented_cloud_pure"] = _arr(o.segmented_cloud_pure, o.n_segmented_pure, XYZI_DTYPE)
    return d


def fa_to_dict(o: FaOut) -> dict:
    return {
        "sharp": _arr(o.sharp, o.n_sharp, XYZI_DTYPE),
        "less_sharp": _arr(o.less_sharp, o.n_less_sharp, XYZI_DTYPE),
        "flat": _arr(o.flat, o.n_flat, XYZI_DTYPE),
        "less_flat": _arr(o.less_flat, o.n_less_flat, XYZI_DTYPE),
        "odom_valid": o.odom_valid,
        "transform_cur": np.array(list(o.transform_cur), dtype=np.float32),
        "transform_sum": np.array(list(o.transform_sum), dtype=np.float32),
        "odom_quat": np.array(list(o.odom_quat)),
        "odom_pos": np.array(list(o.odom_pos)),
        "publish_to_mapping": o.publish_to_mapping,
        "corner_last": _arr(o.corner_last, o.n_corner_last, XYZI_DTYPE),
        "surf_last": _arr(o.surf_last, o.n_surf_last, XYZI_DTYPE),
        "outlier_last": _arr(o.outlier_last, o.n_outlier_last, XYZI_DTYPE),
    }


class Oracle:
    """TEST INFRASTRUCTURE: stateful oracle pipeline (one stream)."""

    VG_FA = 1  # featureAssociation's per-ring VoxelGrid in PCL's std::sort order
    VG_MO = 2  # mapOptimization's VoxelGrids in PCL's std::sort order
    DEFAULT_OPTS = VG_FA | VG_MO  # LEGO_ORACLE_DEFAULT_OPTS: the reference's order everywhere

    def __init__(self, cfg: SensorCfg, vg_opts: int | None = None):
        """vg_opts: None keeps the default (the reference's VoxelGrid order,
        which the product reproduces); 0 sums every voxel in input order."""
        self.lib = oracle_lib()
        self.cfg = cfg
        self.h = C.c_void_p()
        check(self.lib.lego_oracle_create(C.byref(cfg), C.byref(self.h)), "oracle_create")
        if vg_opts is not None:
            check(self.lib.lego_oracle_set_options(self.h, int(vg_opts)), "oracle_set_options")
        self._ip = IpOut()
        self._fa = FaOut()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.lego_oracle_destroy(self.h)
            self.h = None

    def ip(self, pts: np.ndarray, stamp: float, images: bool = False, gated: bool = False) -> dict:
        pts = np.ascontiguousarray(pts, dtype=XYZIR_DTYPE)
        flags = (LEGO_IP_IMAGES if images else 0) | (LEGO_IP_GATED if gated else 0)
        check(self.lib.lego_oracle_ip_process(self.h, pts.ctypes.data, len(pts), stamp, flags, C.byref(self._ip)),
              "oracle_ip")
        return ip_to_dict(self._ip, self.cfg, images)

    def imu(self, msgs: np.ndarray) -> None:
        """Delivers /imu_raw messages to the featureAssociation and
        mapOptimization handlers, in order."""
        msgs = np.ascontiguousarray(msgs, dtype=IMU_DTYPE)
        check(self.lib.lego_oracle_imu_push(self.h, msgs.ctypes.data, len(msgs)), "oracle_imu")

    def fa(self) -> dict:
        check(self.lib.lego_oracle_fa_process(self.h, C.byref(self._ip), C.byref(self._fa)),
              "oracle_fa")
        return fa_to_dict(self._fa)

    def mo_set_map(self, corner: np.ndarray, surf: np.ndarray) -> None:
        check(self.lib.lego_oracle_mo_set_map(self.h, corner.ctypes.data, len(corner),
                                              surf.ctypes.data, len(surf)), "oracle_mo_set_map")

    def mo_configure(self, fixed_map_per_step: bool = False, loop_closure: bool = False,
                     keyframe_search_num: int = 0) -> None:
        o = MoOpts(int(fixed_map_per_step), int(loop_closure), int(keyframe_search_num), 0)
        check(self.lib.lego_oracle_mo_configure(self.h, C.byref(o)), "oracle_mo_configure")

    def loop_closure(self) -> dict:
        out = LoopOut()
        check(self.lib.lego_oracle_mo_loop_closure(self.h, C.byref(out)), "oracle_mo_loop_closure")
        return loop_to_dict(out)

    def log_systems(self, enable: bool = True) -> None:
        """Records the dense systems the OpenCV-shaped solvers receive."""
        check(self.lib.lego_oracle_log_systems(self.h, int(enable)), "oracle_log_systems")

    SYSTEM_WIDTH = {0: 12, 1: 42, 2: 15, 3: 9}  # odometry AtA|AtB, mapping AtA|AtB, plane A0, corner cov

    def systems(self, kind: int) -> np.ndarray:
        """The logged systems of `kind`, one row each (see SYSTEM_WIDTH)."""
        n = C.c_int32()
        check(self.lib.lego_oracle_systems(self.h, kind, None, 0, C.byref(n)), "oracle_systems")
        out = np.zeros(n.value, np.float32)
        check(self.lib.lego_oracle_systems(self.h, kind, out.ctypes.data, n.value, C.byref(n)), "oracle_systems")
        return out.reshape(-1, self.SYSTEM_WIDTH[kind])

    def mo(self) -> dict:
        out = MoOut()
        check(self.lib.lego_oracle_mo_process(self.h, C.byref(self._fa), C.byref(out)), "oracle_mo")
        self._mo = out
        return {k: (np.array(list(getattr(out, k)), dtype=np.float32)
                    if k.startswith("transform") else getattr(out, k)) for k, _ in MoOut._fields_}

    def fusion(self) -> np.ndarray:
        """transformFusion: the last mapping output (if any) then the last
        odometry message -> /integrated_to_init transform_mapped."""
        if getattr(self, "_mo", None) is not None:
            check(self.lib.lego_oracle_fusion_aft_mapped(self.h, C.byref(self._mo)), "oracle_fusion_aft")
            self._mo = None
        out = FusionOut()
        check(self.lib.lego_oracle_fusion_odometry(self.h, C.byref(self._fa), C.byref(out)), "oracle_fusion")
        return np.array(list(out.transform_mapped), np.float32)


_live: "weakref.WeakSet[Lego]" = weakref.WeakSet()


@atexit.register
def _close_live_contexts():
    """Destroys the contexts still open at interpreter exit, while the HIP
    runtime (and torch's use of it) is still up: a context's destructor frees
    device memory, pinned host buffers, events and streams."""
    for g in list(_live):
        g.close()


class Lego:
    """The product pipeline (HIP) behind the C-ABI, one stream per context."""

    def __init__(self, cfg: SensorCfg, device: int = 0, max_points: int = 300000,
                 max_batch: int = 1, streams: int = 0, opts: dict | None = None):
        """streams > 0: a fleet context (lego_fleet_create) of that many
        streams, max_batch scans per stream; batches are stream-major.
        opts: lego_ctx_opts fields over the library defaults (lego_create_ex)."""
        self.lib = hip_lib()
        self.cfg = cfg
        self.h = C.c_void_p()
        o = C.byref(ctx_opts(self.lib, **opts)) if opts else None
        if streams > 0:
            check(self.lib.lego_fleet_create_ex(C.byref(cfg), device, streams, max_points, max_batch, o,
                                                C.byref(self.h)), "lego_fleet_create", self.lib)
        else:
            check(self.lib.lego_create_ex(C.byref(cfg), device, max_points, max_batch, o, C.byref(self.h)),
                  "lego_create", self.lib)
        self._ip = IpOut()
        self._fa = FaOut()
        _live.add(self)

    def close(self):
        if getattr(self, "h", None):
            self.lib.lego_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def reset(self):
        check(self.lib.lego_reset(self.h), "lego_reset", self.lib)

    def ip(self, pts: np.ndarray, stamp: float, images: bool = False, gated: bool = False) -> dict:
        pts = np.ascontiguousarray(pts, dtype=XYZIR_DTYPE)
        flags = (LEGO_IP_IMAGES if images else 0) | (LEGO_IP_GATED if gated else 0)
        check(self.lib.lego_ip_process(self.h, pts.ctypes.data, len(pts), stamp, flags, C.byref(self._ip)),
              "lego_ip_process", self.lib)
        return ip_to_dict(self._ip, self.cfg, images)

    def fa(self) -> dict:
        check(self.lib.lego_fa_process(self.h, C.byref(self._ip), C.byref(self._fa)),
              "lego_fa_process", self.lib)
        return fa_to_dict(self._fa)

    def mo_set_map(self, corner: np.ndarray, surf: np.ndarray) -> None:
        corner = np.ascontiguousarray(corner, dtype=XYZI_DTYPE)
        surf = np.ascontiguousarray(surf, dtype=XYZI_DTYPE)
        check(self.lib.lego_mo_set_map(self.h, corner.ctypes.data, len(corner), surf.ctypes.data, len(surf)),
              "lego_mo_set_map", self.lib)

    def mo_configure(self, fixed_map_per_step: bool = False, loop_closure: bool = False,
                     keyframe_search_num: int = 0) -> None:
        """lego_mo_configure (mapOptimization's switches, utility.h:104,130)."""
        o = MoOpts(int(fixed_map_per_step), int(loop_closure), int(keyframe_search_num), 0)
        check(self.lib.lego_mo_configure(self.h, C.byref(o)), "lego_mo_configure", self.lib)

    def mo(self) -> dict:
        """Scan-to-map on the last fa() output (mapOptimization::run)."""
        out = MoOut()
        check(self.lib.lego_mo_process(self.h, C.byref(self._fa), C.byref(out)), "lego_mo_process", self.lib)
        self._mo = out
        return {k: (np.array(list(getattr(out, k)), dtype=np.float32)
                    if k.startswith("transform") else getattr(out, k)) for k, _ in MoOut._fields_}

    def loop_closure(self) -> dict:
        """performLoopClosure on the device (lego_mo_loop_closure)."""
        out = LoopOut()
        check(self.lib.lego_mo_loop_closure(self.h, C.byref(out)), "lego_mo_loop_closure", self.lib)
        return loop_to_dict(out)

    def fusion(self) -> np.ndarray:
        """transformFusion (lego_fusion_aft_mapped with the last mapping
        output, then lego_fusion_odometry with the last odometry)."""
        if getattr(self, "_mo", None) is not None:
            check(self.lib.lego_fusion_aft_mapped(self.h, C.byref(self._mo)), "lego_fusion_aft_mapped", self.lib)
            self._mo = None
        out = FusionOut()
        check(self.lib.lego_fusion_odometry(self.h, C.byref(self._fa), C.byref(out)), "lego_fusion_odometry",
              self.lib)
        return np.array(list(out.transform_mapped), np.float32)

    def odom_batch(self, pts: np.ndarray, offsets: np.ndarray, stamps: np.ndarray,
                   imu: np.ndarray | None = None, imu_before: np.ndarray | None = None) -> np.ndarray:
        """imu / imu_before: lego_odom_batch_imu (messages imu[:imu_before[k]]
        delivered before scan k, the rest after the batch)."""
        pts = np.ascontiguousarray(pts, dtype=XYZIR_DTYPE)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        stamps = np.ascontiguousarray(stamps, dtype=np.float64)
        k = len(offsets) - 1
        recs = (PoseRec * k)()
        if imu is None:
            check(self.lib.lego_odom_batch(self.h, pts.ctypes.data, offsets.ctypes.data,
                                           stamps.ctypes.data, k, 0, recs), "lego_odom_batch", self.lib)
        else:
            imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
            before = np.ascontiguousarray(imu_before, dtype=np.int32)
            check(self.lib.lego_odom_batch_imu(self.h, pts.ctypes.data, offsets.ctypes.data,
                                               stamps.ctypes.data, k, 0, imu.ctypes.data, len(imu),
                                               before.ctypes.data, recs), "lego_odom_batch_imu", self.lib)
        return recs

    def imu(self, msgs: np.ndarray) -> None:
        """Delivers /imu_raw messages to the featureAssociation and
        mapOptimization queues (lego_imu_push)."""
        msgs = np.ascontiguousarray(msgs, dtype=IMU_DTYPE)
        check(self.lib.lego_imu_push(self.h, msgs.ctypes.data, len(msgs)), "lego_imu_push", self.lib)

    def submit_device(self, pts_ptr: int, offsets_ptr: int, stamps: np.ndarray, k: int) -> None:
        """lego_odom_batch_submit on device-resident inputs (returns at once)."""
        stamps = np.ascontiguousarray(stamps, dtype=np.float64)
        self._stamps_keep = stamps
        check(self.lib.lego_odom_batch_submit(self.h, C.c_void_p(pts_ptr), C.c_void_p(offsets_ptr),
                                              stamps.ctypes.data, k, 1, None, 0, None),
              "lego_odom_batch_submit", self.lib)

    def wait(self, recs) -> int:
        """lego_odom_batch_wait: the oldest submitted batch's records."""
        n = C.c_int32()
        check(self.lib.lego_odom_batch_wait(self.h, recs, len(recs), C.byref(n)), "lego_odom_batch_wait",
              self.lib)
        return n.value

    def odom_batch_device(self, pts_ptr: int, offsets_ptr: int, stamps: np.ndarray, k: int, recs):
        check(self.lib.lego_odom_batch(self.h, C.c_void_p(pts_ptr), C.c_void_p(offsets_ptr),
                                       stamps.ctypes.data, k, 1, recs), "lego_odom_batch", self.lib)

    def batch_fetch(self, k: int, images: bool = False) -> tuple[dict, dict]:
        check(self.lib.lego_batch_fetch(self.h, k, C.byref(self._ip), C.byref(self._fa)),
              "lego_batch_fetch", self.lib)
        return ip_to_dict(self._ip, self.cfg, images), fa_to_dict(self._fa)

    def voxel_grid(self, pts: np.ndarray, leaf: float) -> tuple[np.ndarray, dict]:
        """lego_voxel_grid of an XYZI cloud on the device: (filtered cloud,
        lego_voxel_grid_stats as a dict)."""
        pts = np.ascontiguousarray(pts, dtype=XYZI_DTYPE)
        out = np.zeros(max(len(pts), 1), XYZI_DTYPE)
        n = C.c_int32()
        check(self.lib.lego_voxel_grid(self.h, pts.ctypes.data, len(pts), leaf, out.ctypes.data, C.byref(n)),
              "lego_voxel_grid", self.lib)
        st = (C.c_int32 * 8)()
        check(self.lib.lego_voxel_grid_stats(self.h, st), "lego_voxel_grid_stats", self.lib)
        keys = ("sorted", "voxels", "rounds", "local_segments", "slow_segments", "heap_segments", "nonfinite",
                "device_us")
        return out[:n.value].copy(), dict(zip(keys, list(st)))

    def sort_permutation(self, keys: np.ndarray, wave: bool | int = False) -> tuple[np.ndarray, int]:
        """lego_sort_permutation: std::sort's permutation of (key, index) by key
        on the device and the heap-sorted piece count; `wave` is the mode
        (False / 0: block sort, True / 1: one wave, 2..8: the block sort's
        forms and rules, lego_loam.h)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        perm = np.zeros(max(len(keys), 1), np.int32)
        heap = C.c_int32()
        check(self.lib.lego_sort_permutation(self.h, keys.ctypes.data, len(keys), int(wave), perm.ctypes.data,
                                             C.byref(heap)), "lego_sort_permutation", self.lib)
        return perm[:len(keys)].copy(), heap.value

    def handoff_packet(self) -> np.ndarray:
        """lego_handoff_pack of the last waited batch, copied to the host
        (uint8 array)."""
        ptr, n = C.c_void_p(), C.c_uint64()
        check(self.lib.lego_handoff_pack(self.h, C.byref(ptr), C.byref(n)), "lego_handoff_pack", self.lib)
        out = np.zeros(n.value, np.uint8)
        err = hip_memcpy_d2h(out.ctypes.data, ptr.value, n.value)
        assert err == 0, err
        return out

    def handoff_tensor(self, device):
        """lego_handoff_pack_into a torch uint8 tensor in HBM (the packet of
        the last waited batch, ready for a device-side gather)."""
        import torch

        n = C.c_uint64()
        check(self.lib.lego_handoff_pack_into(self.h, None, 0, C.byref(n)), "lego_handoff_pack_into", self.lib)
        t = torch.empty(n.value, dtype=torch.uint8, device=device)
        check(self.lib.lego_handoff_pack_into(self.h, C.c_void_p(t.data_ptr()), n.value, C.byref(n)),
              "lego_handoff_pack_into", self.lib)
        return t

    def mo_handoff(self, packet: np.ndarray, k: int) -> dict:
        """mapOptimization::run on scan k of a hand-off packet (another
        stream's, e.g. gathered from another GPU): lego_handoff_unpack into
        the context's lego_fa_out, then lego_mo_process."""
        packet = np.ascontiguousarray(packet, np.uint8)
        self._handoff_keep = packet  # the fa_out points into it
        check(self.lib.lego_handoff_unpack(packet.ctypes.data, packet.nbytes, k, None, C.byref(self._fa)),
              "lego_handoff_unpack", self.lib)
        return self.mo()

    def stage_times(self) -> dict:
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        n = C.c_int32()
        check(self.lib.lego_stage_times(self.h, names, ms, 64, C.byref(n)), "stage_times", self.lib)
        return {names[i].decode(): ms[i] for i in range(n.value)}
