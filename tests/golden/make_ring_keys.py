"""Makes tests/golden/c2_ring_keys.npz: the voxel keys of every per-ring
less-flat VoxelGrid (featureAssociation.cpp:778-782) of scan 465 of the C2
stream (VLP-16, seed 1), in the order the oracle sorts them (its
LEGO_ORACLE_VG_DUMP diagnostic).  ring6 (840 keys) holds heap-sorted pieces of
both kinds the device's sum-order sort distinguishes (lego_vgsort.h, sumOrder).

Also tests/golden/dense_ring_keys.npz: the same keys of every ring of the
dense sensors' scans with more than 16 points (a node call's 1024-thread
k_lf_voxel sorts every ring with its workgroup; a batch's only those above
512): VLS-128 seed 3 scan 0 (the scan round 4's fault record names) and
HDL-64E seed 2 scan 0, as vls128_ring<r> / hdl64_ring<r>.

    python tests/golden/make_ring_keys.py
"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))


def ring_keys(L, sensor, seed, scan):
    """the oracle's per-ring sort keys of one scan, ring by ring"""
    sc = L.synth_cfg(sensor, seed)
    ora = L.Oracle(L.sensor_cfg(sensor))
    fd, dump = tempfile.mkstemp(suffix=".bin")
    os.close(fd)
    os.unlink(dump)
    for k in range(scan + 1):
        ora.ip(*L.synth_scan(sc, k))
        if k == scan:
            os.environ["LEGO_ORACLE_VG_DUMP"] = dump
        ora.fa()
    del os.environ["LEGO_ORACLE_VG_DUMP"]
    d = np.fromfile(dump, np.int32)
    os.unlink(dump)
    rings, i = [], 0
    while i < len(d):
        m = int(d[i])
        rings.append(d[i + 1:i + 1 + m].astype(np.uint32))
        i += 1 + m
    return rings


def main():
    import __graft_entry__ as g

    L = g._ffi()
    rings = {f"ring{r}": k for r, k in enumerate(ring_keys(L, "VLP-16", 1, 465))}
    np.savez_compressed(REPO / "tests/golden/c2_ring_keys.npz", **rings)
    print({k: len(v) for k, v in rings.items()})
    dense = {}
    for tag, sensor, seed in (("vls128", "VLS-128", 3), ("hdl64", "HDL-64E", 2)):
        for r, k in enumerate(ring_keys(L, sensor, seed, 0)):
            if len(k) > 16:  # a sort with at least one partition level
                dense[f"{tag}_ring{r}"] = k
    np.savez_compressed(REPO / "tests/golden/dense_ring_keys.npz", **dense)
    print(len(dense), "dense rings:", sorted(len(v) for v in dense.values()))


if __name__ == "__main__":
    main()
