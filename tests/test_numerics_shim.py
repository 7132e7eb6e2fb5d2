"""The float libm restatement (lego_numerics.h) that both the oracle and the
gfx950 kernels use must equal this host's glibc bit for bit — the reference
calls glibc's atan2f/sinf/cosf/asinf on its hot path.
LEGO_EXHAUSTIVE=1 checks every float (≈1 min on 8 cores)."""
import os
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def _build(tmp_path, name, src):
    exe = tmp_path / name
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", str(src), "-o", str(exe)],
                   check=True)
    return exe


def test_libm_shim_matches_glibc(tmp_path):
    exe = _build(tmp_path, "shim_check", REPO / "tests/native/shim_check.cpp")
    stride = "1" if os.environ.get("LEGO_EXHAUSTIVE") else "97"
    r = subprocess.run([str(exe), stride, "2000000"], capture_output=True, text=True, timeout=900)
    print(r.stdout)
    assert r.returncode == 0, r.stdout


def test_introsort_port_matches_std_sort(tmp_path):
    exe = _build(tmp_path, "introsort_check", REPO / "tests/native/introsort_check.cpp")
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout


def test_vgsort_partition_rules_match_std_sort(tmp_path):
    """lego_vgsort.h's parallel partition rules (prefix-count pairing, cut,
    level order, stable blocks, heap-sort fallback) give std::sort's order of
    equal VoxelGrid keys — the order PCL sums a voxel's points in."""
    exe = _build(tmp_path, "vgsort_check", REPO / "tests/native/vgsort_check.cpp")
    r = subprocess.run([str(exe), "6000"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout


def test_vgsort_sum_order_rule(tmp_path):
    """lego_vgsort.h's sumOrder: a heap-sorted piece ranked stably instead
    (each key at most twice in it, its smallest not also in the preceding
    leaf) must give every voxel the same float sum from 0 as std::sort's
    order.  Replayed over C2 scan 465's ring keys, the adversary fixtures and
    tied random keys, with both kinds of piece present."""
    import numpy as np

    exe = _build(tmp_path, "vgsum_check", REPO / "tests/native/vgsum_check.cpp")
    arrays = list(np.load(REPO / "tests/golden/c2_ring_keys.npz").values())
    z = np.load(REPO / "tests/golden/vg_killer.npz")
    arrays += [z[k] for k in z.files if not k.startswith("heaps_")]
    rng = np.random.default_rng(4)
    for n in (300, 900, 2000, 5000):
        for div in (1, 2, 3):  # ascending runs with ties: std::sort's degenerate splits
            a = np.sort(rng.integers(0, n // div + 1, n))
            b = np.sort(rng.integers(0, n // div + 1, n))
            arrays.append(np.concatenate([a, b]))
    dump = tmp_path / "keys.bin"
    with open(dump, "wb") as f:
        for k in arrays:
            k = np.asarray(k, np.int64)
            k = (k - k.min()).astype(np.uint32)
            np.array([len(k)], np.int32).tofile(f)
            k.tofile(f)
    r = subprocess.run([str(exe), str(dump)], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    ranked, exact = (int(x) for x in r.stdout.split("shortcuts")[1].split("bad")[0].replace("flagged", "").split())
    assert ranked > 0 and exact > 0, r.stdout


def test_eigen3_register_form_matches_generic(tmp_path):
    """The device solver's register-resident 3x3 Jacobi (cv_eigen_sym3) must
    equal the OpenCV JacobiImpl_ restatement (cv_eigen_sym<3>) bit for bit."""
    exe = _build(tmp_path, "eigen3_check", REPO / "tests/native/eigen3_check.cpp")
    r = subprocess.run([str(exe), "300000"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout


def test_eig_min_shortcut_is_sound(tmp_path):
    """The odometry skips the iteration-0 Jacobi when an LDL^T test proves
    every eigenvalue of AtA exceeds 10 by a margin; the Jacobi restatement
    must then agree that nothing is degenerate."""
    exe = _build(tmp_path, "eigmin_check", REPO / "tests/native/eigmin_check.cpp")
    r = subprocess.run([str(exe), "300000"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout


def test_jacobi_svd3_and_umeyama(tmp_path):
    """The loop closure's Eigen JacobiSVD / umeyama / PCL convergence-criteria
    restatement (lego_icp.h): reconstruction, orthonormality, ordering, exact
    rigid-motion recovery, criteria branches."""
    exe = _build(tmp_path, "svd3_check", REPO / "tests/native/svd3_check.cpp")
    r = subprocess.run([str(exe), "200000"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout


def test_segmentation_alpha_constants(L):
    """sin/cos of segmentAlphaX/Y (imageProjection.cpp:421) — bit patterns
    recorded in SURVEY.md §9.3 for VLP-16."""
    import numpy as np

    cfg = L.sensor_cfg("VLP-16")
    lib = L.oracle_lib()
    sx, cx = lib.lego_oracle_sinf(cfg.segment_alpha_x), lib.lego_oracle_cosf(cfg.segment_alpha_x)
    sy, cy = lib.lego_oracle_sinf(cfg.segment_alpha_y), lib.lego_oracle_cosf(cfg.segment_alpha_y)
    assert float(np.float32(sx)).hex() == "0x1.c986d40000000p-9"
    assert float(np.float32(cx)).hex() == "0x1.ffff340000000p-1"
    assert float(np.float32(sy)).hex() == "0x1.1de58c0000000p-5"
    assert float(np.float32(cy)).hex() == "0x1.ffb0280000000p-1"
    assert float(np.float32(cfg.segment_theta)).hex() == "0x1.0c15240000000p+0"  # 0x3f860a92


def test_pack_pool_matches_one_thread(tmp_path):
    """The node call's threaded upload pass (lego_pack_host.h): thousands of
    back-to-back jobs of random sizes on one pool give the one-thread
    packing's words and non-finite flag, with the DMA runs in order."""
    exe = tmp_path / "pack_pool_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", str(REPO / "include"), "-I",
                    str(REPO / "lego-loam_amd/csrc"), str(REPO / "tests/native/pack_pool_check.cpp"), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), "3000"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
