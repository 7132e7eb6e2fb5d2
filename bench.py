#!/usr/bin/env python3
"""bench.py — scans/sec of LeGO-LOAM's per-scan hot path on MI355X.

Workload (BASELINE.json configs[1]): one synthetic VLP-16
(16x1800) stream at 10 Hz — projection + ground + segmentation + features +
two-step LM odometry for every scan, in stream order.  A "step" is one batch
of `--batch` consecutive scans of the stream through lego_odom_batch with the
points already resident in HBM.  With --gpus N each rank runs its own stream
(seed 10 + rank, config C4) and every step's hand-off packet (the 64-B pose
records plus the corner / surf / outlier clouds published to mapping) is
gathered to rank 0 over RCCL (the hand-off to the serial pose graph).

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import contextlib
import datetime
import ctypes as C
import importlib.util
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def load_ffi():
    spec = importlib.util.spec_from_file_location("legoffi", REPO / "lego-loam_amd" / "legoffi.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["legoffi"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_multistream():
    sys.path.insert(0, str(REPO / "lego-loam_amd"))
    import multistream

    return multistream


def make_stream(L, sensor: str, seed: int, nscans: int):
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(nscans)]
    pts = np.concatenate([s[0] for s in scans])
    off = np.zeros(nscans + 1, np.int64)
    off[1:] = np.cumsum([len(s[0]) for s in scans])
    stamps = np.array([s[1] for s in scans], np.float64)
    maxn = int(max(len(s[0]) for s in scans))
    return pts, off, stamps, maxn


def odom_alg_bytes(recs) -> float:
    """Compulsory HBM bytes of k_odom per launch: per scan it
    reads the four feature clouds once (16 B/pt) and writes the
    TransformToEnd'ed less-sharp / less-flat clouds twice, as the next scan's
    "last" clouds and as the per-scan output (2 x 16 B/pt).  The NN index is an
    implementation structure, not algorithmic traffic."""
    tot = 0.0
    for r in recs:
        f = r.n_sharp + r.n_less_sharp + r.n_flat + r.n_less_flat
        last = r.n_less_sharp + r.n_less_flat
        tot += 16 * f + 32 * last
    return tot


def pipeline_alg_bytes(cfg, npts, rec) -> float:
    """SURVEY.md §8d's whole-pipeline algorithmic bytes of one scan, from its
    actual counts: projection 16N + 16P + 4P, ground 12(g+1)H + 9P, CCL 9P,
    compaction 21P + 25Ns, curvature / occlusion 13Ns, sort / extract
    10Ns + 16F, deskew and TransformToEnd 32Ns, and the odometry as k_odom's
    compulsory bytes (odom_alg_bytes: 16F + 32 last).  Outliers (a few
    hundred points) are left out."""
    P = cfg.n_scan * cfg.horizon_scan
    H, g = cfg.horizon_scan, cfg.ground_scan_ind
    ns = rec.n_segmented
    f = rec.n_sharp + rec.n_less_sharp + rec.n_flat + rec.n_less_flat
    last = rec.n_less_sharp + rec.n_less_flat
    return (16 * npts + 20 * P + 12 * (g + 1) * H + 9 * P + 9 * P + 21 * P + 25 * ns + 13 * ns + 10 * ns
            + 16 * f + 32 * ns + 16 * f + 32 * last)


def cpu_baseline(L, sensor, seed, nscans, budget_s):
    """The oracle (C++ restatement, 1 thread) over the same stream, repeated
    until ~budget_s of CPU work."""
    cfg = L.sensor_cfg(sensor)
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(nscans)]
    done = 0
    t0 = time.perf_counter()
    passes = 0
    ref = []  # the first pass's transformSum per scan (the pose reference of the bench line)
    while True:
        ora = L.Oracle(cfg)
        for pts, st in scans:
            ora.ip(pts, st)
            f = ora.fa()
            if passes == 0:
                ref.append(f["transform_sum"])
            done += 1
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return done / dt, done, passes, ref


def pose_delta_vs_oracle(gpu_recs: dict, ref: list, B: int):
    """The metric's "pose delta vs ref": every timed scan's transformSum from
    the GPU records against the oracle's run over the same stream (bit-exact
    count and max |delta|; the north-star tolerance is 1e-4)."""
    worst, exact, n = 0.0, 0, 0
    for j, rc in gpu_recs.items():
        for k in range(B):
            o = np.asarray(ref[j * B + k], np.float32)
            g = np.array(list(rc[k].transform_sum), np.float32)
            worst = max(worst, float(np.max(np.abs(g.astype(np.float64) - o.astype(np.float64)))))
            exact += int(np.array_equal(g.view(np.uint32), o.view(np.uint32)))
            n += 1
    return {"scans": n, "max_abs": worst, "bit_exact": exact, "tolerance": 1e-4,
            "reference": "oracle (CPU restatement, oracle/) over the same stream"}


def cpu_all_cores(L, sensor, threads, nscans, budget_s):
    """The oracle on `threads` host threads, thread t running its own stream
    (seed 10 + t; the oracle releases the GIL inside its C++ calls), each
    repeating its stream until ~budget_s.  SURVEY.md §8d's "all cores" line:
    the CPU counterpart of several streams per host."""
    import threading

    cfg = L.sensor_cfg(sensor)
    streams = [None] * threads
    done = [0] * threads

    def synth(t):
        sc = L.synth_cfg(sensor, 10 + t)
        streams[t] = [L.synth_scan(sc, k) for k in range(nscans)]

    def work(t, t0):
        while time.perf_counter() - t0 < budget_s:
            ora = L.Oracle(cfg)
            for pts, st in streams[t]:
                ora.ip(pts, st)
                ora.fa()
                done[t] += 1

    th = [threading.Thread(target=synth, args=(t,)) for t in range(threads)]
    [x.start() for x in th]
    [x.join() for x in th]
    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(t, t0)) for t in range(threads)]
    [x.start() for x in th]
    [x.join() for x in th]
    dt = time.perf_counter() - t0
    quota = cgroup_cpus()
    return {"value": sum(done) / dt, "unit": "scans/s", "cores": threads, "kind": "port",
            "cgroup_cpu_quota": quota,
            "sample": f"{sum(done)} scans: {threads} threads (min(streams, cores), BASELINE.md), each its own "
                      f"{nscans}-scan {sensor} stream (seeds 10..{9 + threads}) through oracle ip+fa incl. LM, "
                      f"~{budget_s:.0f} s" + (f"; the cgroup caps the process at {quota:g} cores" if quota else "")}


def cgroup_cpus():
    """The CPU quota of this process's cgroup (cpu.max), in cores, or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def host_info():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    return {"nproc": os.cpu_count(), "affinity": share, "cgroup_cpu_quota": cgroup_cpus(), "cpu_model": model}


def mapping_handoff(gpu, B: int) -> dict:
    """Auxiliary, outside the timed region: featureAssociation's
    hand-off to mapping over the last timed batch.  publishCloudsLast sends the
    last clouds every skipFrameNum + 1 scans (featureAssociation.cpp:1798-1815);
    lego_batch_fetch brings one scan's outputs (features, the three *_last
    clouds, the pose) to the host, the step a mapping consumer on another
    process pays per published scan."""
    pub, dts, sizes = [], [], []
    for k in range(B):
        t0 = time.perf_counter()
        _, fa = gpu.batch_fetch(k)
        dts.append((time.perf_counter() - t0) * 1e3)
        if fa["publish_to_mapping"]:
            pub.append(k)
            sizes.append((len(fa["corner_last"]), len(fa["surf_last"]), len(fa["outlier_last"])))
    gaps = [b - a for a, b in zip(pub, pub[1:])]
    return {"scans": B, "published": len(pub), "every_n_scans": (statistics.mean(gaps) if gaps else None),
            "fetch_ms_per_scan": statistics.median(dts),
            "clouds_per_published_scan": ([round(statistics.mean(c)) for c in zip(*sizes)] if sizes else None),
            "clouds": "corner_last, surf_last, outlier_last points"}


def c5_alg_bytes(m_raw: int, m_ds: int, q: int, iters: int) -> float:
    """SURVEY.md §8d's algorithmic bytes of one C5 mapping step: the map
    VoxelGrids read and write 16 B per raw point (2·16·M_raw), the hash index
    reads and writes 16 B per filtered point (2·16·M), and each LM iteration
    moves 112 B per query (the query, its 5 neighbours' indices and row)."""
    return 2 * 16 * m_raw + 2 * 16 * m_ds + 112 * q * iters


def mapping_bench(L, steps: int, cpu: bool):
    """Auxiliary (not the headline metric): config C5 scan-to-map — consecutive
    VLS-128 scans (seed 3) handed to mapping against a fixed synthetic map of
    1.0 M surf / 200 k corner points.  Like for like with
    the reference: with `fixed_map_per_step` every step runs the map VoxelGrids
    and the NN index build over the 1.2 M points (mapOptmization.cpp:1058-1064,
    1333-1334), as the oracle leg does, then <= 10 LM iterations.  Only the
    mapping calls are timed (ip + fa of the scans in between are not): host
    wall clock around lego_mo_process, which includes the scan clouds' upload
    and the result read-back.  The install-once mode (map filtered / indexed at
    lego_mo_set_map, identical results) is timed on the same steps beside it."""
    sensor = "VLS-128"
    sc = L.synth_cfg(sensor, 3)
    surf, corner = L.synth_map(3, 50.0, 1_000_000, 200_000)
    res = {"workload": "C5: consecutive VLS-128 scans (seed 3) vs fixed map 1.0M surf + 200k corner, "
                       "map VoxelGrid + index every step, <= 10 LM iterations", "steps": steps}
    cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc)) + 16

    def run(eng, per_step, nsteps):
        if per_step is not None:
            eng.mo_configure(fixed_map_per_step=per_step)
        eng.mo_set_map(corner, surf)
        dts, outs, k = [], [], 0
        while len(dts) < nsteps:
            eng.ip(*L.synth_scan(sc, k))
            eng.fa()
            k += 1
            t0 = time.perf_counter()
            o = eng.mo()
            dt = (time.perf_counter() - t0) * 1e3
            if o["processed"]:
                dts.append(dt)
                outs.append(o)
        return dts, outs

    # a throwaway context's first step loads the mapping kernels' code: the
    # timed contexts then time steps 1..steps, the same steps the CPU leg runs
    warm = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, opts=L.opts_from_env())
    run(warm, True, 1)
    warm.close()
    gpu = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, opts=L.opts_from_env())
    dts, outs = run(gpu, True, steps)
    gpu.close()
    gpu = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, opts=L.opts_from_env())
    dts1, _ = run(gpu, False, steps)
    gpu.close()
    its = [o["iterations"] for o in outs]
    rows = [o["n_rows_last"] for o in outs]
    q = outs[-1]["n_corner_scan_ds"] + outs[-1]["n_surf_scan_ds"]
    med = statistics.median(dts)
    alg = statistics.mean(c5_alg_bytes(len(surf) + len(corner), o["n_corner_map_ds"] + o["n_surf_map_ds"],
                                       o["n_corner_scan_ds"] + o["n_surf_scan_ds"], o["iterations"]) for o in outs)
    res.update({"gpu_ms_per_step": med, "gpu_ms_per_step_mean": statistics.mean(dts),
                "gpu_ms_per_step_min": min(dts),
                "gpu_ms_per_step_map_installed_once": statistics.median(dts1),
                "iterations_per_step": statistics.mean(its), "iterations": its, "rows_last_mean": statistics.mean(rows),
                "map_ds": [outs[-1]["n_corner_map_ds"], outs[-1]["n_surf_map_ds"]], "queries": q,
                "roofline": {"bound": "hbm", "alg_bytes_per_step": alg, "achieved_gbs": alg / (med * 1e-3) / 1e9,
                             "peak_gbs": HBM_PEAK_GBS, "frac": alg / (med * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "note": "SURVEY §8d C5 bytes (2*16*M_raw + 2*16*M_ds + 112*Q*iters) / median step"}})
    if cpu:
        n = 5
        cdts, couts = run(L.Oracle(L.sensor_cfg(sensor)), None, n)
        res["cpu_ms_per_step"] = statistics.median(cdts)
        res["cpu_iterations"] = [o["iterations"] for o in couts]
        res["cpu_sample"] = (f"first {n} mapping steps of the same consecutive scans through the oracle (1 thread; "
                             "map VoxelGrid + kd-tree build every step, as the reference)")
        res["same_iterations_as_gpu"] = res["cpu_iterations"] == its[:n]
        res["gpu_ms_per_step_steps_1_to_%d" % n] = statistics.median(dts[:n])
        res["cpu_over_gpu_same_steps"] = res["cpu_ms_per_step"] / statistics.median(dts[:n])
        res["cpu_vs_gpu_steps"] = (f"like for like: the oracle's steps 1..{n} (median) against the GPU's steps "
                                   f"1..{n} (median, gpu_ms_per_step_steps_1_to_{n}); gpu_ms_per_step is the median "
                                   f"of all {steps} GPU steps")
    return res


def loop_bench(L, nscans: int, calls: int, cpu: bool):
    """Auxiliary (not the headline metric): performLoopClosure
    (lego_mo_loop_closure) after a synthetic VLP-16 drive in a 3.8 m circle
    (15 deg/s, 1 m/s) long enough to revisit 30 s old keyframes, mapping on
    the keyframe-built map.  GPU: host wall clock per call (detection, the
    history cloud's gather / VoxelGrid / index, the ICP and the fitness),
    median of `calls`; CPU: the oracle's same call."""
    sc = L.synth_cfg("VLP-16", 6, yaw_rate_dps=15.0, speed_mps=1.0)
    cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc))
    scans = [L.synth_scan(sc, k) for k in range(nscans)]
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=cap, opts=L.opts_from_env())
    for pts, stamp in scans:
        gpu.ip(pts, stamp)
        gpu.fa()
        gpu.mo()
    g = gpu.loop_closure()  # warm-up (allocates the loop buffers)
    dts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        g = gpu.loop_closure()
        dts.append((time.perf_counter() - t0) * 1e3)
    gpu.close()
    res = {"workload": f"loop closure after {nscans} VLP-16 scans in a 3.8 m circle (keyframe map)",
           "gpu_ms_per_call": statistics.median(dts), "detected": g["detected"], "accepted": g["accepted"],
           "iterations": g["iterations"], "n_source": g["n_source"], "n_target": g["n_target"],
           "fitness": g["fitness"]}
    if cpu:
        ora = L.Oracle(L.sensor_cfg("VLP-16"))
        for pts, stamp in scans:
            ora.ip(pts, stamp)
            ora.fa()
            ora.mo()
        cd = []
        for _ in range(calls):
            t0 = time.perf_counter()
            ora.loop_closure()
            cd.append((time.perf_counter() - t0) * 1e3)
        res["cpu_ms_per_call"] = statistics.median(cd)
        res["cpu_sample"] = f"median of {calls} calls of the oracle (1 thread; kd-tree ICP as PCL)"
    return res


def node_path_bench(L, nscans: int, cpu: bool, cpu_scans: int = 40, sensor: str = "VLP-16", seed: int = 1):
    """Auxiliary (not the headline metric): the per-scan latency of the
    node-shaped drop-in path a ROS deployment runs at 10 Hz (INTEGRATION.md's
    adapter; imageProjection.cpp:181-197 cloudHandler, featureAssociation.cpp:
    1817-1860 runFeatureAssociation, mapOptmization.cpp:1487-1522 run): for
    every scan of the C2 stream (VLP-16, seed 1; or `sensor` / `seed`), one at a time from HOST
    buffers, lego_ip_process -> lego_fa_process -> lego_mo_process (the
    keyframe-built map, the reference's default; the call returns at once when
    mapOptimization's 0.3 s gate is closed).  Host wall clock per scan around
    the three calls, uploads and the library's host outputs included.  A
    throwaway context runs first so module loading is not in the numbers.  CPU
    leg: the oracle's same three calls over the first `cpu_scans` scans, with
    the GPU's summary over those same scans beside it (gpu_same_scans)."""
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(nscans)]
    cap = max(len(p) for p, _ in scans) + 16

    def run(lib, h, ipf, faf, mof, n):
        """per scan: (total, ip, fa, mo) ms and whether mapping ran"""
        ip, fa = L.IpOut(), L.FaOut()
        out = []
        for pts, stamp in scans[:n]:
            pts = np.ascontiguousarray(pts, dtype=L.XYZIR_DTYPE)
            mo = L.MoOut()
            t0 = time.perf_counter()
            L.check(ipf(h, pts.ctypes.data, len(pts), stamp, 0, C.byref(ip)), "ip", lib)
            t1 = time.perf_counter()
            L.check(faf(h, C.byref(ip), C.byref(fa)), "fa", lib)
            t2 = time.perf_counter()
            L.check(mof(h, C.byref(fa), C.byref(mo)), "mo", lib)
            t3 = time.perf_counter()
            out.append(((t3 - t0) * 1e3, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, bool(mo.processed)))
        return out

    def pct(v, q):
        v = sorted(v)
        return v[min(len(v) - 1, int(round(q * (len(v) - 1))))] if v else None

    def summary(recs):
        per = [r[0] for r in recs]
        t_mo = [r[3] for r in recs if not r[4]]
        t_map = [r[3] for r in recs if r[4]]
        return {"scans": len(per), "ms_per_scan_median": statistics.median(per), "ms_per_scan_p99": pct(per, 0.99),
                "ms_per_scan_max": max(per), "ms_per_scan_mean": statistics.mean(per),
                "ip_ms_median": statistics.median(r[1] for r in recs),
                "fa_ms_median": statistics.median(r[2] for r in recs),
                "mo_gate_closed_ms_median": statistics.median(t_mo) if t_mo else None,
                "mapping_steps": len(t_map),
                "mapping_step_ms_median": statistics.median(t_map) if t_map else None,
                "mapping_step_ms_max": max(t_map) if t_map else None}

    lib = L.hip_lib()
    warm = L.Lego(L.sensor_cfg(sensor, lib), max_points=cap, opts=L.opts_from_env())
    run(lib, warm.h, lib.lego_ip_process, lib.lego_fa_process, lib.lego_mo_process, 8)
    warm.close()
    gpu = L.Lego(L.sensor_cfg(sensor, lib), max_points=cap, opts=L.opts_from_env())
    name = "C2 stream (VLP-16 seed 1)" if (sensor, seed) == ("VLP-16", 1) else f"{sensor} seed {seed} stream"
    res = {"workload": f"{name} one scan at a time from host buffers through the node API: "
                       f"lego_ip_process -> lego_fa_process -> lego_mo_process (keyframe map), {nscans} scans"}
    recs = run(lib, gpu.h, lib.lego_ip_process, lib.lego_fa_process, lib.lego_mo_process, nscans)
    gpu.close()
    res["gpu"] = summary(recs)
    res["gpu"]["fits_10hz"] = res["gpu"]["ms_per_scan_max"] < 100.0
    if cpu:
        olib = L.oracle_lib()
        ora = L.Oracle(L.sensor_cfg(sensor))
        res["cpu"] = summary(run(olib, ora.h, olib.lego_oracle_ip_process, olib.lego_oracle_fa_process,
                                 olib.lego_oracle_mo_process, cpu_scans))
        res["cpu"]["sample"] = f"the oracle's same three calls over scans 0..{cpu_scans - 1} (1 thread)"
        # like for like: the GPU's calls on the same scans (the mapping gate
        # opens on the same scans of both)
        res["gpu_same_scans"] = summary(recs[:cpu_scans])
        res["gpu_vs_cpu_note"] = (f"cpu and gpu_same_scans cover the same scans 0..{cpu_scans - 1} (medians and p99 "
                                  f"comparable); gpu covers all {nscans}")
    return res


def dense_bench(L, nscans: int, batch: int, device: int, cpu: bool = False, budget_s: float = 5.0):
    """Auxiliary (not the headline metric): config C3, the HDL-64E-shaped
    synthetic stream (64 x 2048) through the same pipeline
    on one GPU, two batches in flight.  Host wall clock, like the headline."""
    import torch

    cfg = L.sensor_cfg("HDL-64E", L.hip_lib())
    nscans = max(nscans, 3 * batch)  # two warm-up batches and at least one timed one
    pts, off, stamps, maxn = make_stream(L, "HDL-64E", 2, nscans)
    nb = nscans // batch
    d_pts = torch.from_numpy(pts.view(np.uint8)).to(device)
    d_off = [torch.from_numpy(off[i * batch:(i + 1) * batch + 1].astype(np.int64)).to(device) for i in range(nb)]
    g = L.Lego(cfg, device=device, max_points=maxn + 16, max_batch=batch, opts=L.opts_from_env())
    recs = (L.PoseRec * batch)()
    sub = lambda j: g.submit_device(d_pts.data_ptr(), d_off[j].data_ptr(), stamps[j * batch:(j + 1) * batch],  # noqa: E731
                                    batch)
    got = {}  # batch index -> its records (copied after each wait; the pose check runs after the timing)
    order = []

    def wait():
        g.wait(recs)
        cp = (L.PoseRec * batch)()
        C.memmove(cp, recs, C.sizeof(recs))
        got[order.pop(0)] = cp

    warm = 2  # as the headline loop: two warm-up batches, then the rest two deep
    for j in range(warm):
        sub(j)
        order.append(j)
    for j in range(warm):
        wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    inflight = 0
    for j in range(warm, nb):
        if inflight == 2:
            wait()
            inflight -= 1
        sub(j)
        order.append(j)
        inflight += 1
    while inflight:
        wait()
        inflight -= 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    g.close()
    n = (nb - warm) * batch
    j = nb - 1  # recs: the last batch's records
    per_scan = statistics.mean(pipeline_alg_bytes(cfg, int(off[j * batch + k + 1] - off[j * batch + k]), got[j][k])
                               for k in range(batch))
    res = {"workload": f"C3: HDL-64E 64x2048 synthetic stream (seed 2), {batch} scans per call, two in flight",
           "scans": n, "scans_per_s": n / dt, "ms_per_scan": dt / n * 1e3, "points_per_scan": int(maxn),
           "roofline": {"bound": "hbm", "alg_bytes_per_scan": per_scan, "achieved_gbs": per_scan * n / dt / 1e9,
                        "peak_gbs": HBM_PEAK_GBS, "frac": per_scan * n / dt / 1e9 / HBM_PEAK_GBS,
                        "note": "SURVEY §8d whole-pipeline bytes per scan (pipeline_alg_bytes, the last batch's "
                                "counts) x scans/s"}}
    if cpu:  # the oracle on one core over the same stream (scans synthesised beforehand): the CPU
        # leg times its first ~budget_s, and the whole stream is the pose reference of every GPU scan
        sc = L.synth_cfg("HDL-64E", 2)
        ora = L.Oracle(L.sensor_cfg("HDL-64E"))
        ref, done, tc, timing = [], 0, 0.0, True
        for k in range(nb * batch):
            scan = L.synth_scan(sc, k)
            t0 = time.perf_counter()
            ora.ip(*scan)
            f = ora.fa()
            if timing:
                tc += time.perf_counter() - t0
                done += 1
                timing = tc < budget_s
            ref.append(f["transform_sum"])
        v = done / tc
        res["cpu_baseline"] = {"value": v, "unit": "scans/s", "cores": 1, "kind": "port",
                               "sample": f"the first {done} scans of the same HDL-64E stream through oracle ip+fa "
                                         "incl. LM, 1 thread"}
        res["gpu_over_cpu"] = res["scans_per_s"] / v
        res["pose_delta_vs_oracle"] = pose_delta_vs_oracle({j: got[j] for j in range(warm, nb)}, ref, batch)
        res["pose_delta_vs_oracle"]["note"] = f"the {n} timed scans (batches {warm}..{nb - 1})"
    return res


def fleet_bench(L, streams: int, k: int, steps: int, device: int, check: bool = False):
    """Auxiliary (not the headline metric): `streams` independent VLP-16
    streams in one fleet context (lego_fleet_create) on one GPU, k scans per
    stream per call, the stream-major batch resident in HBM.  Whole-GPU
    scans/s over `steps` calls (host wall clock, like the headline).  Every
    stream is its own synthetic drive (seed 10 + s), synthesised on the host's
    cores beforehand."""
    import torch
    from concurrent.futures import ThreadPoolExecutor

    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    nwin = steps + 1

    def synth(d):  # the synthesis library runs outside the GIL
        sc = L.synth_cfg("VLP-16", 10 + d)
        return [L.synth_scan(sc, j)[0] for j in range(k * nwin)]

    with ThreadPoolExecutor(max_workers=max(1, min(16, host_info()["affinity"]))) as ex:
        src = list(ex.map(synth, range(streams)))
    maxn = max(len(p) for s in src for p in s)
    wins, npts = [], []
    for w in range(nwin):
        scans = [src[s][w * k + j] for s in range(streams) for j in range(k)]
        npts.append([len(p) for p in scans])
        off = np.zeros(len(scans) + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p in scans])
        st = np.concatenate([np.arange(w * k, (w + 1) * k) * 0.1] * streams)
        wins.append((torch.from_numpy(np.concatenate(scans).view(np.uint8)).to(device),
                     torch.from_numpy(off).to(device), st))
    fl = L.Lego(cfg, device=device, max_points=maxn + 16, max_batch=k, streams=streams, opts=L.opts_from_env())
    recs = (L.PoseRec * (streams * k))()
    sub = lambda w: fl.submit_device(w[0].data_ptr(), w[1].data_ptr(), w[2], streams * k)  # noqa: E731
    sub(wins[0])  # warm-up (initialises every stream)
    fl.wait(recs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):  # two calls in flight, as the headline loop
        sub(wins[1 + i])
        if i:
            fl.wait(recs)
    fl.wait(recs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    fl.close()
    # recs hold the last call's records (window nwin - 1), stream-major like its points
    per_scan = statistics.mean(pipeline_alg_bytes(cfg, npts[-1][i], recs[i]) for i in range(streams * k))
    sps = streams * k * steps / dt
    pose = None
    if check:  # every stream's last-call poses against the oracle's run of that stream (host threads, untimed)
        ocfg = L.sensor_cfg("VLP-16")

        def oracle_stream(d):
            ora = L.Oracle(ocfg)
            out = None
            for j in range(k * nwin):
                ora.ip(src[d][j], j * 0.1)
                f = ora.fa()
                if j >= k * (nwin - 1):
                    out = f["transform_sum"] if out is None else np.vstack([out, f["transform_sum"]])
            return out

        with ThreadPoolExecutor(max_workers=max(1, min(16, host_info()["affinity"]))) as ex:
            refs = list(ex.map(oracle_stream, range(streams)))
        worst, exact = 0.0, 0
        for d in range(streams):
            for j in range(k):
                g = np.array(list(recs[d * k + j].transform_sum), np.float32)
                o = np.asarray(refs[d][j], np.float32)
                worst = max(worst, float(np.max(np.abs(g.astype(np.float64) - o.astype(np.float64)))))
                exact += int(np.array_equal(g.view(np.uint32), o.view(np.uint32)))
        pose = {"scans": streams * k, "max_abs": worst, "bit_exact": exact, "tolerance": 1e-4,
                "reference": f"the oracle's run of every stream over its {k * nwin} scans; the last call's "
                             f"{k} scans of each of the {streams} streams compared"}
    return {"pose_delta_vs_oracle": pose,
            "workload": f"fleet: {streams} independent VLP-16 streams (seeds 10..{9 + streams}) x {k} scans per "
                        "call on one GPU (lego_fleet_create, two calls in flight), full per-scan pipeline incl. LM "
                        "odometry",
            "streams": streams, "scans_per_stream_per_call": k, "calls": steps,
            "scans_per_s": sps, "ms_per_call": dt / steps * 1e3,
            "roofline": {"bound": "hbm", "alg_bytes_per_scan": per_scan, "achieved_gbs": per_scan * sps / 1e9,
                         "peak_gbs": HBM_PEAK_GBS, "frac": per_scan * sps / 1e9 / HBM_PEAK_GBS,
                         "note": "SURVEY §8d whole-pipeline bytes per scan (pipeline_alg_bytes, the last call's "
                                 "counts) x scans/s"}}


@contextlib.contextmanager
def stdout_to_stderr():
    """File descriptor 1 onto 2 for the block: gloo's connection messages
    ("[Gloo] Rank r is connected to ...", printed to stdout by every rank)
    stay out of the one JSON line rank 0 prints."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=100, help="scans per step")
    ap.add_argument("--stream-len", type=int, default=600, help="synthetic stream length (C2: 600)")
    ap.add_argument("--sensor", default="VLP-16")
    ap.add_argument("--seed", type=int, default=None, help="stream seed at N=1 (default 1: C2; C3 is 2)")
    ap.add_argument("--no-handoff", action="store_true",
                    help="skip the untimed mapping hand-off fetches (profiling runs: only the timed work)")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of oracle work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--odom-profile", action="store_true", help="in-kernel phase stamps (diagnostic)")
    ap.add_argument("--mapping-steps", type=int, default=15, help="C5 scan-to-map steps (aux; 0 = skip)")
    ap.add_argument("--fleet-streams", type=int, default=256,
                    help="streams of the fleet aux line (0 = skip); 256 = one odometry workgroup per stream and CU")
    ap.add_argument("--loop-scans", type=int, default=340, help="loop-closure aux stream length (0 = skip)")
    ap.add_argument("--dense-scans", type=int, default=200, help="C3 HDL-64E scans of the aux line (0 = skip)")
    ap.add_argument("--node-scans", type=int, default=120,
                    help="scans of the node-API latency line (aux.node_path; 0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for the N > 1 path on a one-GPU box (never used by the
    # driver): every rank on device 0, the pose gather over gloo on the host.
    if os.environ.get("LEGO_BENCH_SHARE_GPU"):
        local = 0
    backend = os.environ.get("LEGO_BENCH_BACKEND", "nccl")  # nccl = RCCL on ROCm
    import torch

    dist = None
    ms = load_multistream()
    # N > 1 fails fast and says where: finite timeouts on the process groups
    # (LEGO_BENCH_PG_TIMEOUT_S) and a per-rank watchdog (LEGO_BENCH_WATCHDOG_S)
    # that ends a rank making no progress with a message naming the step and
    # phase (multistream.Watchdog: os._exit, never a re-exec).  The native
    # gather's own waits are bounded by lego_comm_set_timeout (LEGO_COMM_TIMEOUT_MS
    # in the environment, multistream.native_comm).
    wd = None
    pg_timeout = datetime.timedelta(seconds=float(os.environ.get("LEGO_BENCH_PG_TIMEOUT_S", "300")))
    if world > 1:
        import torch.distributed as dist

        wd = ms.Watchdog(float(os.environ.get("LEGO_BENCH_WATCHDOG_S", "240")), rank)
        wd.mark(None, "init_process_group")
        torch.cuda.set_device(local)
        with stdout_to_stderr():
            dist.init_process_group(backend, timeout=pg_timeout)
    dev = torch.device("cuda", local)

    def mark(step, phase):
        if wd is not None:
            wd.mark(step, phase)

    L = load_ffi()
    lib = L.hip_lib()
    cfg = L.sensor_cfg(args.sensor, lib)
    # N=1: the C2 stream (seed 1).  N>1: C4, stream `rank` (seed 10 + rank).
    seed = (args.seed if args.seed is not None else 1) if world == 1 else ms.stream_seed(
        ms.streams_of_rank(world, world, rank)[0])
    pts, off, stamps, maxn = make_stream(L, args.sensor, seed, args.stream_len)
    B = args.batch
    nb = args.stream_len // B
    # inputs resident in HBM before the timed region
    d_pts = torch.from_numpy(pts.view(np.uint8)).to(dev)
    d_off = [torch.from_numpy((off[i * B:(i + 1) * B + 1] - 0).astype(np.int64)).to(dev)
             for i in range(nb)]
    torch.cuda.synchronize()
    gpu = L.Lego(cfg, device=local, max_points=maxn + 16, max_batch=B, opts=L.opts_from_env())
    n_en = C.c_int32()
    on = (C.c_float * 1)()
    lib.lego_stage_times(gpu.h, None, on, 0, C.byref(n_en))  # enable the stage timer
    if args.odom_profile:
        lib.lego_odom_profile(gpu.h, 1, None)
    recs = (L.PoseRec * B)()
    # N > 1 hand-off transport: the C-ABI's own collective (lego_comm_gather_handoff_ex,
    # RCCL send/recv over xGMI, packets kept in rank 0's HBM) when every rank has
    # its GPU; the one-GPU rehearsal (gloo, shared device) gathers over torch.
    # The choice is collective (ms.HandoffTransport): the ranks agree over a gloo
    # control group after the communicator's creation and after every native
    # gather, and a failure on any rank moves EVERY rank to the torch gather at
    # the same step (never RCCL on some ranks and torch on others: a hang).
    comm, transport = None, None
    comm_ranks = None
    if dist is not None:
        mark(None, "control group")
        with stdout_to_stderr():
            ctrl = dist.new_group(backend="gloo", timeout=pg_timeout) if backend != "gloo" else None
        want_native = backend == "nccl"
        create_error = None
        if want_native:
            mark(None, "lego_comm_create")
            try:
                comm = ms.native_comm(L, dist, local)
            except Exception as e:  # noqa: BLE001
                create_error = f"lego_comm_create: {e}"
        mark(None, "transport agreement")
        transport = ms.HandoffTransport(dist, ctrl, want_native and comm is not None, create_error)
        if not transport.native and comm is not None:
            lib.lego_comm_abort(comm)
            lib.lego_comm_destroy(comm)
            comm = None
        if comm is not None:  # the communicator's rank count as RCCL reports it
            n = C.c_int32()
            comm_ranks = int(n.value) if lib.lego_comm_count(comm, C.byref(n)) == L.LEGO_OK else None
        else:
            comm_ranks = dist.get_world_size()

    # Steps are pipelined two deep (lego_odom_batch_submit / _wait): step i+1's
    # projection + extraction run while step i's odometry chain does.
    inflight = []

    def retire():
        i = inflight.pop(0)
        mark(i, "lego_odom_batch_wait")
        gpu.wait(recs)
        cp = (L.PoseRec * B)()
        C.memmove(cp, recs, C.sizeof(recs))
        # N > 1: the step's hand-off packet (pose records + the published
        # corner / surf / outlier clouds) gathered to rank 0 right here, before
        # the slot is reused: by the native collective, or (every rank at once)
        # by the torch gather of the packet packed into HBM
        pkt = None
        if transport is not None:
            mark(i, "hand-off gather (" + transport.name + ")")

            def fallback():
                t = gpu.handoff_tensor(dev)
                return ms.gather_packets(t if backend == "nccl" else t.cpu(), dist, to_host=False)

            _, pkt = transport.step(lambda: ms.native_gather_handoff(L, comm, gpu, 0, device=True), fallback,
                                    lambda: lib.lego_comm_abort(comm) if comm is not None else None)
        return i, gpu.stage_times(), cp, pkt

    def submit(i):
        j = i % nb
        done = []
        if j == 0 and i > 0:
            gpu.reset()  # a new pass over the stream starts from a fresh state (in stream order)
        if len(inflight) == 2:
            done.append(retire())
        mark(i, "lego_odom_batch_submit")
        gpu.submit_device(d_pts.data_ptr(), d_off[j].data_ptr(), stamps[j * B:(j + 1) * B], B)
        inflight.append(i)
        return done

    for i in range(args.warmup):
        submit(i)
    while inflight:
        retire()
    if dist:
        mark(None, "barrier before the timed region")
        dist.barrier()
    torch.cuda.synchronize()
    if transport is not None:  # per-step host costs of the timed steps only
        transport.t_gather = transport.t_agree = 0.0
    stage_acc: dict[str, float] = {}
    gathered = None
    t0 = time.perf_counter()
    alg_bytes = 0.0

    gpu_recs = {}  # batch index within the stream -> its pose records (each pass starts from reset)
    pipe_bytes = 0.0

    def account(done):
        nonlocal alg_bytes, gathered, pipe_bytes
        for i, st, rc, pkt in done:
            gpu_recs[i % nb] = rc
            j = i % nb
            pipe_bytes += sum(pipeline_alg_bytes(cfg, int(off[j * B + k + 1] - off[j * B + k]), rc[k])
                              for k in range(B))
            for k, v in st.items():
                stage_acc[k] = stage_acc.get(k, 0.0) + v
            alg_bytes += odom_alg_bytes(rc)
            if dist:  # gathered in retire(): rank 0's copies of every rank's packet
                gathered = pkt

    for i in range(args.steps):
        account(submit(args.warmup + i))
    while inflight:
        account([retire()])
    torch.cuda.synchronize()
    if dist:
        mark(None, "barrier after the timed region")
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        mark(None, "max-over-ranks all_reduce")
        t = torch.tensor([dt], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        wd.disarm()
    total_scans = args.steps * B * world
    value = total_scans / dt
    ms_per_step = dt / args.steps * 1e3

    handoff = None
    if rank == 0:
        handoff = mapping_handoff(gpu, B) if not args.no_handoff else {}
        if gathered is not None:  # the last step's packets as rank 0 received them
            if transport.native:
                L.check(lib.lego_comm_wait(comm), "lego_comm_wait", lib)
                hdrs = []
                for ptr, nbytes in gathered:
                    h = L.HandoffHdr()
                    if ptr and nbytes >= C.sizeof(h):
                        L.hip_memcpy_d2h(C.addressof(h), ptr, C.sizeof(h))
                    hdrs.append(h)
                sizes = [int(nb) for _, nb in gathered]
                how = ("lego_comm_gather_handoff_ex (C-ABI; RCCL ncclGather of sizes + ncclSend/ncclRecv "
                       "of packets, LEGO_COMM_DEVICE_RESULT), every step in the timed region")
            else:
                hdrs = [L.handoff_header(g.cpu().numpy()) for g in gathered]
                sizes = [int(g.numel()) for g in gathered]
                how = f"torch.distributed gather ({backend}) of lego_handoff_pack_into packets, in the timed region"
            handoff["gathered_to_rank0"] = {
                "ranks": len(hdrs), "scans_per_rank": [h.nscans for h in hdrs],
                "published_per_rank": [h.npub for h in hdrs], "bytes_per_rank": [h.bytes for h in hdrs],
                "valid": len(hdrs) == world and all(h.magic == L.HANDOFF_MAGIC and h.nscans == B and h.bytes == n
                                                    for h, n in zip(hdrs, sizes)),
                "transport": how}
        # the batch runs as chunks (lego_api.hip run_batch): k_odom launches per step
        launches = {k[2:]: v / args.steps for k, v in stage_acc.items() if k.startswith("n:")}
        stage_acc = {k: v for k, v in stage_acc.items() if not k.startswith("n:")}
        odom_ms = stage_acc.get("odom.lm", 0.0) / args.steps
        n_odom = max(1.0, launches.get("odom.lm", 1.0))
        achieved = (alg_bytes / args.steps) / (odom_ms * 1e-3) / 1e9 if odom_ms > 0 else 0.0
        # roofline.traffic: the PMC figure (FETCH_SIZE x2 + WRITE_SIZE, separate
        # rocprofv3 passes over this command, scripts/gpu_profile.sh) of the newest
        # committed summary, labelled with the commit it was measured at
        traffic, traffic_src = None, None
        pmcs = sorted((REPO / "profiles").glob("r[0-9][0-9]_pmc_summary.json"), reverse=True)
        for pmc in pmcs:
            if pmc.exists():
                try:
                    js = json.loads(pmc.read_text())
                    traffic = js.get("k_odom_hbm_bytes_per_launch")
                    traffic_src = f"profiles/{pmc.name} (measured at commit {js.get('commit', '?')}, not in this run)"
                except Exception:  # noqa: BLE001
                    traffic = None
                break
        cpu = None
        cpu_all = None
        pose_delta = None
        if not args.no_cpu and world == 1:  # the CPU baseline is an N = 1 line
            v, n, passes, ref = cpu_baseline(L, args.sensor, seed, args.stream_len, args.cpu_budget)
            pose_delta = pose_delta_vs_oracle(gpu_recs, ref, B)
            cpu = {"value": v, "unit": "scans/s", "cores": 1, "kind": "port",
                   "sample": f"{n} scans ({passes} pass(es) over the {args.stream_len}-scan "
                             f"{args.sensor} stream, seed {seed}) through oracle ip+fa incl. LM, 1 thread"}
            # min(streams, cores) threads, the streams being the fleet line's
            # (the cores this process may use: its affinity, capped by the cgroup's quota)
            usable = host_info()["affinity"]
            if cgroup_cpus():
                usable = min(usable, max(1, int(cgroup_cpus())))
            thr = max(1, min(max(args.fleet_streams, 1), usable))
            # each thread repeats its own stream; the streams' synthesis is kept to ~3.8 k scans
            cpu_all = cpu_all_cores(L, args.sensor, thr, max(10, 3840 // thr), args.cpu_budget)
        if args.odom_profile:
            prof = (C.c_uint64 * 32)()
            lib.lego_odom_profile(gpu.h, -1, prof)
            names = ["surf_nn", "surf", "corner_nn", "corner", "solve", "integrate", "to_end",
                     "build", "resident", "", "", "", "nn_shells"]
            nsc = (args.steps + args.warmup) * B
            for i, nm in enumerate(names):
                if nm:
                    print(f"  odom.{nm:10s} {prof[i] / 100.0 / nsc:9.2f} us/scan", file=sys.stderr)
            print(f"  iters/scan surf {prof[9] / nsc:.2f} corner {prof[10] / nsc:.2f} nn {prof[11] / nsc:.2f}"
                  f"  per scan: nn shell-1 {prof[14] / nsc:.1f}, nn exhaustive {prof[15] / nsc:.1f},"
                  f" scan-line indexed {prof[20] / nsc:.1f}, scan-line literal {prof[13] / nsc:.1f}",
                  file=sys.stderr)
            for i, nm in ((21, "rows (excl. reduce)"), (22, "solve_qr+eig it0"), (23, "solve_qr it>0"),
                          (24, "nn local work"), (25, "to_end loop (wave 1)"),                           (26, "build: pass 1"), (27, "build: key tables+scan"), (29, "build: scatter pass"),
                          (31, "build: bucket ends")):
                print(f"  odom.{nm:20s} {prof[i] / 100.0 / nsc:9.2f} us/scan", file=sys.stderr)
            nq0 = max(prof[30], 1)
            for i, nm in ((28, "wave0 q: nn i1"), (16, "wave0 q: to_start"), (17, "wave0 q: closest"),
                          (18, "wave0 q: scan lines")):
                print(f"  odom.{nm:20s} {prof[i] / 100.0 / nq0:9.2f} us/query ({prof[30] / nsc:.1f} q/scan)",
                      file=sys.stderr)
        if args.stages:
            tot = sum(stage_acc.values())
            for k, v in sorted(stage_acc.items(), key=lambda kv: -kv[1]):
                print(f"  {k:14s} {v / args.steps:9.3f} ms/step  {100 * v / max(tot, 1e-9):5.1f}%",
                      file=sys.stderr)
        # The headline context is done: close it before the aux lines.  A
        # process's HIP streams share GPU_MAX_HW_QUEUES (4) hardware queues, and
        # an idle context's two streams left open make a later context's
        # extraction and odometry streams share a queue (C3 measured 4.0 k
        # instead of 5.1 k scans/s that way, scripts/dense_probe3.py).
        if comm is not None:
            lib.lego_comm_destroy(comm)
            comm = None
        gpu.close()
        gpu = None
        aux = {"mapping_handoff": handoff}
        t_aux = time.perf_counter()

        def progress(leg):  # one stderr line per aux leg (a long run is seen to advance)
            print(f"bench: {leg} at {time.perf_counter() - t_aux:.0f} s", file=sys.stderr, flush=True)

        if args.mapping_steps > 0 and world == 1:
            progress("C5")
            aux["scan_to_map_c5"] = mapping_bench(L, args.mapping_steps, not args.no_cpu)
        if args.fleet_streams > 0 and world == 1:
            progress("fleet")
            aux["fleet_vlp16"] = fleet_bench(L, args.fleet_streams, 20, 3, local, check=not args.no_cpu)
        if args.dense_scans > 0 and world == 1:
            progress("C3")
            aux["dense_hdl64_c3"] = dense_bench(L, args.dense_scans, 20, local, cpu=not args.no_cpu)
        if args.loop_scans > 0 and world == 1:
            progress("loop closure")
            aux["loop_closure"] = loop_bench(L, args.loop_scans, 5, not args.no_cpu)
        if args.node_scans > 0 and world == 1:
            progress("node path")
            aux["node_path"] = node_path_bench(L, args.node_scans, not args.no_cpu)
            progress("node path VLS-128")
            # the dense single-scan path (VLS-128: 128 rings per VoxelGrid launch)
            aux["node_path_vls128"] = node_path_bench(L, max(8, args.node_scans // 3), not args.no_cpu,
                                                      cpu_scans=8, sensor="VLS-128", seed=3)
        if cpu_all:
            aux["cpu_all_cores"] = cpu_all
        aux["host"] = host_info()
        line = {
            "metric": "scans/sec (projection+seg+feat+LM) VLP-16 16x1800",
            "value": value,
            "unit": "scans/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded ray-cast VLP-16 stream, 1 m/s + 5 deg/s)",
            "config": {"workload": (f"C2: {args.sensor} stream @10Hz, full per-scan pipeline incl. "
                                    f"2-step LM odometry, {B} scans/step" if world == 1 else
                                    f"C4: one {args.sensor} stream per GPU (seeds 10..{9 + world}) @10Hz, full "
                                    f"per-scan pipeline incl. 2-step LM odometry, {B} scans/step, hand-off "
                                    "gathered to rank 0 every step"),
                       "scans_per_step": B, "stream_len": args.stream_len, "seed": seed,
                       "parallelism": f"stream-per-gpu x{world}",
                       "gather": ((("lego_comm (C-ABI RCCL send/recv)" if transport.native
                                    else f"torch.distributed ({backend})")
                                   + ": per step, pose records + published clouds to rank 0, one transport on every "
                                     "rank (agreed over a gloo control group)") if transport else None),
                       "gather_native_error": (transport.errors or None) if transport else None,
                       "gather_fallback_from_step": transport.switched_at if transport else None,
                       "comm_ranks": comm_ranks,
                       "gather_host_ms_per_step": ({
                           "gather": transport.t_gather / args.steps * 1e3,
                           "agreement": transport.t_agree / args.steps * 1e3,
                           "note": "rank 0's host time per timed step in the hand-off call (native: pack, size "
                                   "gather and root's sync on the sizes, send/recv enqueue) and in the gloo "
                                   "agreement after it"} if transport else None)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_over_alg": (traffic / (alg_bytes / args.steps * 1.0 / n_odom)
                                              if traffic and alg_bytes else None),
                         "kernel": "k_odom", "launch_ms": odom_ms / n_odom, "launches_per_step": n_odom,
                         "kernel_ms_per_step": odom_ms,
                         "pipeline": {"alg_bytes_per_scan": pipe_bytes / (args.steps * B),
                                      "achieved_gbs": pipe_bytes * world / dt / 1e9,
                                      "frac": pipe_bytes * world / dt / 1e9 / HBM_PEAK_GBS,
                                      "note": "SURVEY §8d whole-pipeline bytes of every timed scan (pipeline_alg_bytes) "
                                              "over the timed region, all ranks"}},
            "cpu_baseline": cpu,
            "pose_delta_vs_oracle": pose_delta,
            "stages_ms_per_step": {k: v / args.steps for k, v in stage_acc.items()},
            "aux": aux,
        }
        print(json.dumps(line))
    if comm is not None:
        lib.lego_comm_destroy(comm)
    if gpu is not None:
        gpu.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
