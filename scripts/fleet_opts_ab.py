#!/usr/bin/env python3
"""Fleet A/B over lego_ctx_opts settings: bench.py's fleet line (256 VLP-16
streams, seeds 10.., 20 scans per stream per call, two calls in flight), one
context per setting and round (created, warmed by one call, CALLS calls
timed, closed: two open contexts would share the process's hardware queues),
the settings alternating over ROUNDS rounds.  Prints scans/s per setting and
round.  Diagnostic.

  python scripts/fleet_opts_ab.py --settings "ip_fused=1;ip_fused=0"
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import bench  # noqa: E402


def parse(setting: str) -> dict:
    return {k: int(v) for k, v in (kv.split("=") for kv in setting.split(",") if kv)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--windows", type=int, default=3)
    ap.add_argument("--calls", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--settings", default="ip_fused=1;ip_fused=0")
    args = ap.parse_args()
    import torch

    L = bench.load_ffi()
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    S, K = args.streams, args.k

    def synth(d):
        sc = L.synth_cfg("VLP-16", 10 + d)
        return [L.synth_scan(sc, j)[0] for j in range(K * args.windows)]

    with ThreadPoolExecutor(max_workers=16) as ex:
        src = list(ex.map(synth, range(S)))
    maxn = max(len(p) for s in src for p in s)
    wins = []
    for w in range(args.windows):
        scans = [src[s][w * K + j] for s in range(S) for j in range(K)]
        off = np.zeros(len(scans) + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p in scans])
        st = np.concatenate([np.arange(w * K, (w + 1) * K) * 0.1] * S)
        wins.append((torch.from_numpy(np.concatenate(scans).view(np.uint8)).to("cuda:0"),
                     torch.from_numpy(off).to("cuda:0"), st))
    del src
    recs = (L.PoseRec * (S * K))()
    for r in range(args.rounds):
        for setting in args.settings.split(";"):
            fl = L.Lego(cfg, device=0, max_points=maxn + 16, max_batch=K, streams=S, opts=parse(setting))
            n = [0]

            def sub():
                w = wins[n[0] % len(wins)]
                n[0] += 1
                fl.submit_device(w[0].data_ptr(), w[1].data_ptr(), w[2], S * K)

            sub()  # untimed
            fl.wait(recs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.calls):
                sub()
                if i:
                    fl.wait(recs)
            fl.wait(recs)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"round": r, "setting": setting, "scans_per_s": round(S * K * args.calls / dt),
                              "ms_per_call": round(dt / args.calls * 1e3, 3),
                              "valid": sum(x.odom_valid for x in recs)}), flush=True)
            fl.close()


if __name__ == "__main__":
    main()
