"""The segmentation angle test (imageProjection.cpp:421-423) as the kernels
evaluate it (lego_seg.h seg_edge_fast: decided from the quotient away from
the threshold, atan2f near it) equals the reference's expression on random,
near-threshold and corner-case range pairs for the presets' alphas and four
thresholds (tests/native/seg_edge_check.cpp, gcc -ffp-contract=off)."""
import subprocess
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def test_seg_edge_fast_equals_atan2f(tmp_path):
    exe = tmp_path / "seg_edge_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", str(REPO / "include"),
                    "-I", str(REPO / "lego-loam_amd/csrc"), str(REPO / "tests/native/seg_edge_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
