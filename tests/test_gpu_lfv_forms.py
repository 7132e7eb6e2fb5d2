"""k_lf_voxel (the per-ring less-flat VoxelGrid, featureAssociation.cpp:
778-782) at both of its block sizes, through the product path against the
oracle, on the call sequence of round 4's only GPU fault record.

That record was a work-in-progress build whose k_lf_voxel
ran the register form of the block sort (segment ids in registers,
vg_block_sort): lego_fa_process on VLS-128 scan 0, right after two
lego_voxel_grid calls on the same context, ended with an illegal memory
access.  Round 5 built the register form back into k_lf_voxel behind a
diagnostic switch and ran this sequence: its 1024-thread instance faulted
deterministically (a VM fault, fa_synccheck naming k_lf_voxel), its
256-thread instance and the LDS-id form at both sizes ran bit-exact, and the
sort itself is exact at both sizes in kernels of its own
(tests/test_gpu_sort_perm.py).  The register form is therefore not built
into k_lf_voxel; this file keeps the sequence as a regression test of the
product's kernel (LDS-id form) in 256- (wide=0) and 1024-thread (wide=1)
workgroups (lego_ctx_opts::lfv_wide).  A payload no sort can produce is
reported as LEGO_E_DEVICE (kBadPermutation), not clamped."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _eq(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("wide", [0, 1])
def test_fault_record_sequence(L, wide):
    """The fault record's calls on one context: lego_voxel_grid on C5's 1.0 M
    surf map (leaf 0.4) and 200 k corner map (leaf 0.2), then lego_ip_process
    / lego_fa_process on VLS-128 seed 3 scans 0..2 (scripts/vg_probe.py), with
    k_lf_voxel in 256- (wide=0) or 1024-thread (wide=1) workgroups.  Features
    and poses bit-exact vs the oracle."""
    sensor = "VLS-128"
    sc = L.synth_cfg(sensor, 3)
    surf, corner = L.synth_map(3, 50.0, 1_000_000, 200_000)
    cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc)) + 16
    g = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=cap, opts={"lfv_wide": wide})
    ora = L.Oracle(L.sensor_cfg(sensor))
    try:
        g.voxel_grid(surf, 0.4)
        g.voxel_grid(corner, 0.2)
        for k in range(3):
            pts, stamp = L.synth_scan(sc, k)
            g.ip(pts, stamp)
            ora.ip(pts, stamp)
            gf, of = g.fa(), ora.fa()
            for key in ("sharp", "less_sharp", "flat", "less_flat"):
                assert _eq(gf[key], of[key]), (k, key, len(gf[key]), len(of[key]))
            assert np.array_equal(gf["transform_sum"].astype(np.float32), of["transform_sum"].astype(np.float32)), k
    finally:
        g.close()
