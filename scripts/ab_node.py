"""Node-API latency A/B (GPU box): bench.node_path_bench in this process, the
variant chosen by the environment the caller sets (e.g. LEGO_LFV_BLOCK_RINGS,
read once per process; SENSOR / SEED pick the stream, default the C2 one).  Prints one line: label, median / p99 ms per scan, ip
and fa medians.  Diagnostic, not a test."""
import os
import sys

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "lego-loam_amd"))
import bench  # noqa: E402
import legoffi as L  # noqa: E402

res = bench.node_path_bench(L, int(os.environ.get("SCANS", "120")), cpu=False, sensor=os.environ.get("SENSOR", "VLP-16"),
                            seed=int(os.environ.get("SEED", "1")))["gpu"]
print(f"{os.environ.get('LABEL', '?'):4s} median {res['ms_per_scan_median']:.3f} p99 {res['ms_per_scan_p99']:.3f} "
      f"ip {res['ip_ms_median']:.3f} fa {res['fa_ms_median']:.3f} map {res['mapping_step_ms_median']:.3f}", flush=True)
