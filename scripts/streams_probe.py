#!/usr/bin/env python3
"""Several independent VLP-16 streams on ONE GPU, one context (and HIP
stream) per lidar stream, each driven by its own host thread (ctypes drops
the GIL for the duration of lego_odom_batch).  Prints scans/s of the whole
GPU for each stream count.  Diagnostic for the concurrency of the per-stream
pipeline; not the headline metric."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,4")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--stream-len", type=int, default=400)
    ap.add_argument("--workgroups", type=int, default=0, help="cap on k_odom workgroups per stream")
    ap.add_argument("--distinct", type=int, default=4, help="distinct synthetic streams (reused round-robin)")
    args = ap.parse_args()
    import os

    import torch

    if args.workgroups:
        os.environ["LEGO_ODOM_WORKGROUPS"] = str(args.workgroups)

    L = bench.load_ffi()
    lib = L.hip_lib()
    cfg = L.sensor_cfg("VLP-16", lib)
    B = args.batch
    nb = args.stream_len // B
    smax = max(int(s) for s in args.streams.split(","))
    data = []
    for s in range(min(smax, args.distinct)):
        pts, off, stamps, maxn = bench.make_stream(L, "VLP-16", 10 + s, args.stream_len)
        d_pts = torch.from_numpy(pts.view(np.uint8)).to("cuda:0")
        d_off = [torch.from_numpy(off[i * B:(i + 1) * B + 1].astype(np.int64)).to("cuda:0") for i in range(nb)]
        data.append((d_pts, d_off, stamps, maxn))
    data = [data[s % len(data)] for s in range(smax)]
    torch.cuda.synchronize()
    out = {}
    for S in (int(s) for s in args.streams.split(",")):
        if S * (args.workgroups or 48) > 256:  # keep every launched workgroup co-resident (one per CU)
            continue
        ctxs = [L.Lego(cfg, device=0, max_points=data[s][3] + 16, max_batch=B) for s in range(S)]
        errs = []

        def run(s, nsteps, first):
            d_pts, d_off, stamps, _ = data[s]
            recs = (L.PoseRec * B)()
            try:
                for i in range(first, first + nsteps):
                    j = i % nb
                    if j == 0:
                        ctxs[s].reset()
                    ctxs[s].odom_batch_device(d_pts.data_ptr(), d_off[j].data_ptr(), stamps[j * B:(j + 1) * B], B,
                                              recs)
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        for s in range(S):  # warm-up, serial
            run(s, 1, 0)
        th = [threading.Thread(target=run, args=(s, args.steps, 1)) for s in range(S)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        for c in ctxs:
            c.close()
        out[S] = {"scans_per_s": S * args.steps * B / dt, "errors": errs}
        print(json.dumps({"streams": S, "workgroups": args.workgroups, **out[S]}), flush=True)


if __name__ == "__main__":
    main()
