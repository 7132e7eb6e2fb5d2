#!/usr/bin/env python3
"""Fleet throughput on one GPU: S independent VLP-16 streams in one fleet
context (lego_fleet_create), K scans per stream per call, the stream-major
batch resident in HBM.  Prints whole-GPU scans/s per (S, K).  Diagnostic;
bench.py's headline stays one stream per GPU."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,8,32,64")
    ap.add_argument("--k", type=int, default=20, help="scans per stream per call")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--distinct", type=int, default=4)
    ap.add_argument("--workgroups", type=int, default=0)
    ap.add_argument("--extract-profile", action="store_true", help="k_extract phase stamps (diagnostic)")
    args = ap.parse_args()
    import torch

    if args.workgroups:
        os.environ["LEGO_ODOM_WORKGROUPS"] = str(args.workgroups)
    L = bench.load_ffi()
    lib = L.hip_lib()
    cfg = L.sensor_cfg("VLP-16", lib)
    K = args.k
    nwin = args.steps + 1
    src = []
    for d in range(args.distinct):
        sc = L.synth_cfg("VLP-16", 10 + d)
        src.append([L.synth_scan(sc, k)[0] for k in range(K * nwin)])
    stamps_one = np.arange(K * nwin) * 0.1
    maxn = max(len(p) for s in src for p in s)
    for S in (int(v) for v in args.streams.split(",")):
        wins = []
        for w in range(nwin):  # stream-major window w: stream s's scans [w*K, w*K + K)
            scans = [src[s % args.distinct][w * K + k] for s in range(S) for k in range(K)]
            off = np.zeros(len(scans) + 1, np.int64)
            off[1:] = np.cumsum([len(p) for p in scans])
            d_pts = torch.from_numpy(np.concatenate(scans).view(np.uint8)).to("cuda:0")
            d_off = torch.from_numpy(off).to("cuda:0")
            st = np.concatenate([stamps_one[w * K:(w + 1) * K]] * S)
            wins.append((d_pts, d_off, st))
        torch.cuda.synchronize()
        fl = L.Lego(cfg, device=0, max_points=maxn + 16, max_batch=K, streams=S, opts=L.opts_from_env())
        n_en = C.c_int32()
        lib.lego_stage_times(fl.h, None, (C.c_float * 1)(), 0, C.byref(n_en))  # enable the stage timer
        recs = (L.PoseRec * (S * K))()
        d_pts, d_off, st = wins[0]
        fl.odom_batch_device(d_pts.data_ptr(), d_off.data_ptr(), st, S * K, recs)  # warm-up
        torch.cuda.synchronize()
        if args.extract_profile:
            lib.lego_odom_profile(fl.h, 1, None)
        t0 = time.perf_counter()
        for i in range(args.steps):
            d_pts, d_off, st = wins[1 + i]
            fl.odom_batch_device(d_pts.data_ptr(), d_off.data_ptr(), st, S * K, recs)
        dt = time.perf_counter() - t0
        stg = fl.stage_times()
        valid = sum(r.odom_valid for r in recs)
        xph = None
        if args.extract_profile:
            xp = (C.c_uint64 * 8)()
            lib.lego_extract_profile(fl.h, xp)
            rings = max(xp[4], 1)
            xph = {nm: round(xp[i] / 100.0 / rings, 2) for i, nm in
                   enumerate(("sorts", "picking", "copies+lessflat", "voxelgrid"))}
            xph["rings"] = xp[4]
            xph["rings_parallel_picking"] = xp[6]
            xph["sector_rewalks"] = xp[5]
            xph["mean_workgroups_in_flight_at_start"] = round(xp[7] / rings, 1)
            op = (C.c_uint64 * 32)()
            lib.lego_odom_profile(fl.h, -1, op)
            nsc = S * K * (args.steps + 1)  # stamps of every workgroup 0 of a stream... summed over all workgroups
            xph["odom_us_per_scan_summed_over_workgroups"] = {
                nm: round(op[i] / 100.0 / nsc, 2) for i, nm in
                ((0, "surf_nn"), (2, "corner_nn"), (3, "corner"), (4, "solve"), (5, "integrate"), (6, "to_end"),
                 (7, "build"), (12, "nn_shells"), (21, "rows"), (23, "solve_qr"), (24, "nn_local"))}
            xph["odom_iters_per_scan"] = {"surf": op[9] / nsc, "corner": op[10] / nsc, "nn": op[11] / nsc}
        fl.close()
        print(json.dumps({"streams": S, "k": K, "scans_per_s": S * K * args.steps / dt,
                          "ms_per_call": dt / args.steps * 1e3, "valid_last": valid,
                          "stages_ms_last": {k: round(v, 3) for k, v in stg.items()},
                          "extract_us_per_ring_workgroup": xph}), flush=True)
        del wins


if __name__ == "__main__":
    main()
