"""Makes tests/golden/c2_ring_keys.npz: the voxel keys of every per-ring
less-flat VoxelGrid (featureAssociation.cpp:778-782) of scan 465 of the C2
stream (VLP-16, seed 1), in the order the oracle sorts them (its
LEGO_ORACLE_VG_DUMP diagnostic).  ring6 (840 keys) holds heap-sorted pieces of
both kinds the device's sum-order sort distinguishes (lego_vgsort.h, sumOrder).

    python tests/golden/make_ring_keys.py
"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))


def main():
    import __graft_entry__ as g

    L = g._ffi()
    sc = L.synth_cfg("VLP-16", 1)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    fd, dump = tempfile.mkstemp(suffix=".bin")
    os.close(fd)
    os.unlink(dump)
    for k in range(466):
        ora.ip(*L.synth_scan(sc, k))
        if k == 465:
            os.environ["LEGO_ORACLE_VG_DUMP"] = dump
        ora.fa()
    del os.environ["LEGO_ORACLE_VG_DUMP"]
    d = np.fromfile(dump, np.int32)
    os.unlink(dump)
    rings, i = {}, 0
    while i < len(d):
        m = int(d[i])
        rings[f"ring{len(rings)}"] = d[i + 1:i + 1 + m].astype(np.uint32)
        i += 1 + m
    np.savez_compressed(REPO / "tests/golden/c2_ring_keys.npz", **rings)
    print({k: len(v) for k, v in rings.items()})


if __name__ == "__main__":
    main()
