#!/usr/bin/env python3
"""Writes tests/golden/vg_killer.npz: VoxelGrid key sequences that drive
libstdc++'s std::sort (PCL's sort of (voxel idx, point)) into its heap-sort
fallback, with ties, and (heaps_<case>) how many heap-sorted pieces std::sort
takes on each — McIlroy's adversary run against the real std::sort by
tests/native/vgsort_check.cpp, keys divided to make voxels of 1-3 points.

  python tests/golden/make_vg_killer.py
"""
import subprocess
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
CASES = {"n8000_div3": (8000, 3), "n30000_div3": (30000, 3), "n20000_div1": (20000, 1),
         # for the one-wave sort (<= 512 keys) and the block sort's small arrays
         "n64_div1": (64, 1), "n200_div1": (200, 1), "n500_div3": (500, 3), "n512_div1": (512, 1),
         "n3000_div2": (3000, 2)}


def main():
    with tempfile.TemporaryDirectory() as d:
        exe = Path(d) / "vgsort_check"
        subprocess.run(["g++", "-O2", "-std=c++17", str(REPO / "tests/native/vgsort_check.cpp"), "-o", str(exe)],
                       check=True)
        out = {}
        for name, (n, div) in CASES.items():
            raw = subprocess.run([str(exe), "killer", str(n), str(div)], check=True, capture_output=True).stdout
            out[name] = np.frombuffer(raw, np.uint32).copy()
            assert out[name].size == n
            # how many heap-sorted pieces std::sort takes on them (the emulation, checked equal to it)
            kf = Path(d) / "keys.bin"
            kf.write_bytes(raw)
            out["heaps_" + name] = np.array([int(subprocess.run([str(exe), "heaps", str(kf)], check=True,
                                                                capture_output=True, text=True).stdout)], np.int64)
    np.savez_compressed(Path(__file__).resolve().parent / "vg_killer.npz", **out)


if __name__ == "__main__":
    main()
