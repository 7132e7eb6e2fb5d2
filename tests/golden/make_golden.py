#!/usr/bin/env python3
"""Regenerates tests/golden/*.npz from the CPU oracle (test infrastructure).

The reference ships no golden data and cannot be built here (SURVEY.md §4,
§8c), so these fixtures are the oracle's own outputs on seeded synthetic
inputs.  They pin the oracle against regressions and carry the inputs to the
GPU box, where tests/test_golden.py checks the HIP product against them.

  python tests/golden/make_golden.py
"""
import hashlib
import importlib.util
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
OUT = Path(__file__).resolve().parent


def ffi():
    spec = importlib.util.spec_from_file_location("legoffi", REPO / "lego-loam_amd" / "legoffi.py")
    m = importlib.util.module_from_spec(spec)
    sys.modules["legoffi"] = m
    spec.loader.exec_module(m)
    return m


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def scan_fixture(L, sensor, seed, k, name, full=True):
    sc = L.synth_cfg(sensor, seed)
    pts, stamp = L.synth_scan(sc, k)
    ora = L.Oracle(L.sensor_cfg(sensor))
    ip = ora.ip(pts, stamp, images=True)
    fa = ora.fa()
    d = {"input": pts.view(np.uint8), "stamp": np.float64(stamp), "input_sha": np.bytes_(sha(pts))}
    keys_ip = ["start_ring_index", "end_ring_index", "ground_flag", "col_ind", "range", "segmented", "outlier",
               "label_image", "ground_image", "range_image"]
    for key in keys_ip:
        if full or key in ("start_ring_index", "end_ring_index"):
            d["ip_" + key] = ip[key].view(np.uint8) if ip[key].dtype.names else ip[key]
        d["sha_ip_" + key] = np.bytes_(sha(ip[key]))
    d["orient"] = np.array([ip["start_orientation"], ip["end_orientation"], ip["orientation_diff"]], np.float32)
    for key in ("sharp", "less_sharp", "flat", "less_flat"):
        if full:
            d["fa_" + key] = fa[key].view(np.uint8)
        d["sha_fa_" + key] = np.bytes_(sha(fa[key]))
    if not full:
        del d["input"]
    np.savez_compressed(OUT / f"{name}.npz", **d)


def stream_fixture(L, sensor, seed, n, name):
    sc = L.synth_cfg(sensor, seed)
    ora = L.Oracle(L.sensor_cfg(sensor))
    sums, counts, shas, in_shas = [], [], [], []
    for k in range(n):
        pts, stamp = L.synth_scan(sc, k)
        in_shas.append(sha(pts))
        ip = ora.ip(pts, stamp)
        fa = ora.fa()
        sums.append(fa["transform_sum"])
        counts.append([len(ip["segmented"]), len(fa["sharp"]), len(fa["less_sharp"]), len(fa["flat"]),
                       len(fa["less_flat"]), fa["odom_valid"], fa["publish_to_mapping"]])
        shas.append(sha(np.concatenate([fa[k2].view(np.uint8) for k2 in
                                        ("sharp", "less_sharp", "flat", "less_flat")])))
    np.savez_compressed(OUT / f"{name}.npz", transform_sum=np.array(sums, np.float32),
                        counts=np.array(counts, np.int32), feat_sha=np.array(shas, dtype="S64"),
                        input_sha=np.array(in_shas, dtype="S64"), sensor=np.bytes_(sensor),
                        seed=np.int64(seed))


def mapping_fixture(L, sensor, seed, n, name, fixed_map):
    """Scan-to-map after every scan of a stream: the keyframe-built map
    (fixed_map None) or a fixed synthetic map (seed, radius, n_surf, n_corner)."""
    sc = L.synth_cfg(sensor, seed)
    ora = L.Oracle(L.sensor_cfg(sensor))
    if fixed_map:
        surf, corner = L.synth_map(*fixed_map)
        ora.mo_set_map(corner, surf)
    aft, info = [], []
    for k in range(n):
        pts, stamp = L.synth_scan(sc, k)
        ora.ip(pts, stamp)
        ora.fa()
        o = ora.mo()
        aft.append(o["transform_aft_mapped"])
        info.append([o["processed"], o["optimized"], o["iterations"], o["n_rows_last"], o["n_corner_map_ds"],
                     o["n_surf_map_ds"], o["n_corner_scan_ds"], o["n_surf_scan_ds"]])
    np.savez_compressed(OUT / f"{name}.npz", transform_aft_mapped=np.array(aft, np.float32),
                        info=np.array(info, np.int32), sensor=np.bytes_(sensor), seed=np.int64(seed),
                        fixed_map=np.array(fixed_map or [], np.float64))


def imu_before(imu, stamps, period):
    """Delivery rule of the IMU fixtures: the messages stamped before the end
    of scan k's sweep (stamp + scan period) reach the handlers before scan k
    is processed."""
    return np.searchsorted(imu["stamp"], np.asarray(stamps) + period, side="left").astype(np.int32)


def imu_fixture(L, sensor, seed, n, name, imu_t0, rate_hz):
    """The VLP-16 stream with /imu_raw from imu_t0 on (the first scans see no
    message: the imuPointerLast < 0 branch, then the switch-over), odometry
    and keyframe scan-to-map after every scan."""
    sc = L.synth_cfg(sensor, seed)
    ora = L.Oracle(L.sensor_cfg(sensor))
    period = float(sc.scan_period)
    imu = L.synth_imu(sc, imu_t0, n * period + period, rate_hz)
    stamps = [L.synth_scan(sc, k)[1] for k in range(n)]
    before = imu_before(imu, stamps, period)
    sums, counts, shas, aft, info = [], [], [], [], []
    j = 0
    for k in range(n):
        pts, stamp = L.synth_scan(sc, k)
        ora.imu(imu[j:before[k]])
        j = before[k]
        ip = ora.ip(pts, stamp)
        fa = ora.fa()
        o = ora.mo()
        sums.append(fa["transform_sum"])
        counts.append([len(ip["segmented"]), len(fa["sharp"]), len(fa["less_sharp"]), len(fa["flat"]),
                       len(fa["less_flat"]), fa["odom_valid"], fa["publish_to_mapping"]])
        shas.append(sha(np.concatenate([fa[k2].view(np.uint8) for k2 in
                                        ("sharp", "less_sharp", "flat", "less_flat")])))
        aft.append(o["transform_aft_mapped"])
        info.append([o["processed"], o["optimized"], o["iterations"], o["n_rows_last"], o["n_corner_map_ds"],
                     o["n_surf_map_ds"], o["n_corner_scan_ds"], o["n_surf_scan_ds"]])
    np.savez_compressed(OUT / f"{name}.npz", transform_sum=np.array(sums, np.float32),
                        counts=np.array(counts, np.int32), feat_sha=np.array(shas, dtype="S64"),
                        transform_aft_mapped=np.array(aft, np.float32), info=np.array(info, np.int32),
                        imu=imu.view(np.uint8), imu_before=before, sensor=np.bytes_(sensor),
                        seed=np.int64(seed))


def main():
    L = ffi()
    scan_fixture(L, "VLP-16", 0, 0, "vlp16_seed0_scan0", full=True)
    scan_fixture(L, "HDL-64E", 2, 0, "hdl64_seed2_scan0", full=False)
    stream_fixture(L, "VLP-16", 1, 20, "vlp16_seed1_stream20")
    mapping_fixture(L, "VLP-16", 6, 24, "vlp16_seed6_keyframe_map24", None)
    mapping_fixture(L, "VLP-16", 3, 10, "vlp16_seed3_fixed_map10", (3, 50.0, 200000, 40000))
    imu_fixture(L, "VLP-16", 6, 24, "vlp16_seed6_imu100_map24", 0.25, 100.0)
    for p in sorted(OUT.glob("*.npz")):
        print(p.name, p.stat().st_size)


if __name__ == "__main__":
    main()
