"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the synthetic source and the oracle still reproduce them exactly.
GPU: the HIP product reproduces them exactly (inputs travel in the fixture,
so this holds even if the synthetic generator changes)."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def load(name):
    return np.load(GOLD / f"{name}.npz", allow_pickle=False)


def check_scan(L, g, ip, fa, full):
    for key in ("start_ring_index", "end_ring_index", "ground_flag", "col_ind", "range", "segmented",
                "outlier", "label_image", "ground_image", "range_image"):
        assert sha(ip[key]) == g["sha_ip_" + key].item().decode(), key
    np.testing.assert_array_equal(
        np.array([ip["start_orientation"], ip["end_orientation"], ip["orientation_diff"]], np.float32).view(np.uint32),
        g["orient"].view(np.uint32))
    for key in ("sharp", "less_sharp", "flat", "less_flat"):
        assert sha(fa[key]) == g["sha_fa_" + key].item().decode(), key
    if full:
        np.testing.assert_array_equal(ip["label_image"], g["ip_label_image"])
        np.testing.assert_array_equal(ip["segmented"].view(np.uint8), g["ip_segmented"])


def test_synth_reproduces_inputs(L):
    g = load("vlp16_seed0_scan0")
    pts, stamp = L.synth_scan(L.synth_cfg("VLP-16", 0), 0)
    assert sha(pts) == g["input_sha"].item().decode()
    s = load("vlp16_seed1_stream20")
    sc = L.synth_cfg("VLP-16", 1)
    for k in (0, 7, 19):
        assert sha(L.synth_scan(sc, k)[0]) == s["input_sha"][k].decode()


def test_oracle_reproduces_scan_fixture(L):
    g = load("vlp16_seed0_scan0")
    pts = g["input"].view(L.XYZIR_DTYPE)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    ip = ora.ip(pts, float(g["stamp"]), images=True)
    check_scan(L, g, ip, ora.fa(), True)


def test_oracle_reproduces_hdl64_fixture(L):
    g = load("hdl64_seed2_scan0")
    pts, stamp = L.synth_scan(L.synth_cfg("HDL-64E", 2), 0)
    assert sha(pts) == g["input_sha"].item().decode()
    ora = L.Oracle(L.sensor_cfg("HDL-64E"))
    ip = ora.ip(pts, stamp, images=True)
    check_scan(L, g, ip, ora.fa(), False)


def test_oracle_reproduces_stream_fixture(L):
    s = load("vlp16_seed1_stream20")
    sc = L.synth_cfg("VLP-16", 1)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    for k in range(len(s["counts"])):
        pts, stamp = L.synth_scan(sc, k)
        ip = ora.ip(pts, stamp)
        fa = ora.fa()
        np.testing.assert_array_equal(fa["transform_sum"].view(np.uint32), s["transform_sum"][k].view(np.uint32))
        feats = np.concatenate([fa[key].view(np.uint8) for key in ("sharp", "less_sharp", "flat", "less_flat")])
        assert sha(feats) == s["feat_sha"][k].decode()


@pytest.mark.gpu
def test_product_reproduces_scan_fixture(L):
    g = load("vlp16_seed0_scan0")
    pts = g["input"].view(L.XYZIR_DTYPE)
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=len(pts) + 16)
    ip = gpu.ip(pts, float(g["stamp"]), images=True)
    check_scan(L, g, ip, gpu.fa(), True)
    gpu.close()


@pytest.mark.gpu
def test_product_reproduces_stream_fixture(L):
    """Features and poses bit-exact per scan (the north star's 1e-4 is the
    contract; bit-identity is what the product delivers and what is asserted)."""
    s = load("vlp16_seed1_stream20")
    sc = L.synth_cfg("VLP-16", 1)
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000)
    exact = 0
    for k in range(len(s["counts"])):
        pts, stamp = L.synth_scan(sc, k)
        gpu.ip(pts, stamp)
        fa = gpu.fa()
        feats = np.concatenate([fa[key].view(np.uint8) for key in ("sharp", "less_sharp", "flat", "less_flat")])
        assert sha(feats) == s["feat_sha"][k].decode(), k
        d = np.abs(fa["transform_sum"].astype(np.float64) - s["transform_sum"][k])
        assert d.max() <= 1e-4, (k, d)
        exact += int(np.array_equal(fa["transform_sum"].view(np.uint32), s["transform_sum"][k].view(np.uint32)))
    gpu.close()
    print(f"bit-exact poses: {exact}/{len(s['counts'])}")
    assert exact == len(s["counts"])


def _run_mapping(L, g, engine_factory, gpu):
    sensor = g["sensor"].item().decode()
    sc = L.synth_cfg(sensor, int(g["seed"]))
    eng = engine_factory(sensor)
    fm = g["fixed_map"]
    if len(fm):
        surf, corner = L.synth_map(int(fm[0]), float(fm[1]), int(fm[2]), int(fm[3]))
        eng.mo_set_map(corner, surf)
    out = []
    for k in range(len(g["info"])):
        pts, stamp = L.synth_scan(sc, k)
        eng.ip(pts, stamp)
        eng.fa()
        out.append(eng.mo())
    if gpu:
        eng.close()
    return out


@pytest.mark.parametrize("name", ["vlp16_seed6_keyframe_map24", "vlp16_seed3_fixed_map10"])
def test_oracle_reproduces_mapping_fixture(L, name):
    g = load(name)
    out = _run_mapping(L, g, lambda s: L.Oracle(L.sensor_cfg(s)), False)
    for k, o in enumerate(out):
        info = [o["processed"], o["optimized"], o["iterations"], o["n_rows_last"], o["n_corner_map_ds"],
                o["n_surf_map_ds"], o["n_corner_scan_ds"], o["n_surf_scan_ds"]]
        np.testing.assert_array_equal(info, g["info"][k], err_msg=str(k))
        np.testing.assert_array_equal(o["transform_aft_mapped"].view(np.uint32),
                                      g["transform_aft_mapped"][k].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["vlp16_seed6_keyframe_map24", "vlp16_seed3_fixed_map10"])
def test_product_reproduces_mapping_fixture(L, name):
    """Decisions, LM iteration counts, last-iteration row counts and filtered
    sizes exact; mapped poses bit-exact (the 1e-4 north star checked too)."""
    g = load(name)
    out = _run_mapping(L, g, lambda s: L.Lego(L.sensor_cfg(s, L.hip_lib()), max_points=40000), True)
    exact = 0
    for k, o in enumerate(out):
        info = [o["processed"], o["optimized"], o["iterations"], o["n_rows_last"], o["n_corner_map_ds"],
                o["n_surf_map_ds"], o["n_corner_scan_ds"], o["n_surf_scan_ds"]]
        np.testing.assert_array_equal(info, g["info"][k], err_msg=str(k))
        d = np.abs(o["transform_aft_mapped"].astype(np.float64) - g["transform_aft_mapped"][k])
        assert d.max() <= 1e-4, (k, d)
        exact += int(np.array_equal(o["transform_aft_mapped"].view(np.uint32),
                                    g["transform_aft_mapped"][k].view(np.uint32)))
    print(f"{name}: bit-exact mapped poses {exact}/{len(out)}")
    assert exact == len(out)


# ---------------------------------------------------------------- /imu_raw
def _imu_fixture_run(L, g, eng, gpu):
    """Node-shaped replay of the IMU fixture: the messages before each scan,
    then ip -> fa -> mo."""
    sensor = g["sensor"].item().decode()
    sc = L.synth_cfg(sensor, int(g["seed"]))
    imu = g["imu"].view(L.IMU_DTYPE)
    before = g["imu_before"]
    outs = []
    j = 0
    for k in range(len(before)):
        pts, stamp = L.synth_scan(sc, k)
        eng.imu(imu[j:before[k]])
        j = int(before[k])
        ip = eng.ip(pts, stamp)
        fa = eng.fa()
        outs.append((ip, fa, eng.mo()))
    return outs


def _check_imu_fixture(g, outs):
    """Counts and features exact; odometry and mapped poses, LM iteration and
    row counts bit-exact.  Every differing scan is collected first, so a
    failure names the first scan, the field and its |delta|."""
    bad = []
    for k, (ip, fa, mo) in enumerate(outs):
        c = [len(ip["segmented"]), len(fa["sharp"]), len(fa["less_sharp"]), len(fa["flat"]),
             len(fa["less_flat"]), fa["odom_valid"], fa["publish_to_mapping"]]
        np.testing.assert_array_equal(c, g["counts"][k], err_msg=str(k))
        feats = np.concatenate([fa[key].view(np.uint8) for key in ("sharp", "less_sharp", "flat", "less_flat")])
        assert sha(feats) == g["feat_sha"][k].decode(), k
        ts = np.asarray(fa["transform_sum"], np.float32)
        assert np.abs(ts.astype(np.float64) - g["transform_sum"][k]).max() <= 1e-4, k
        if not np.array_equal(ts.view(np.uint32), g["transform_sum"][k].view(np.uint32)):
            bad.append((k, "transform_sum", float(np.abs(ts.astype(np.float64) - g["transform_sum"][k]).max())))
        info = [mo["processed"], mo["optimized"], mo["iterations"], mo["n_rows_last"], mo["n_corner_map_ds"],
                mo["n_surf_map_ds"], mo["n_corner_scan_ds"], mo["n_surf_scan_ds"]]
        if not np.array_equal(info, g["info"][k]):
            bad.append((k, "info", (info, list(g["info"][k]))))
        tam = mo["transform_aft_mapped"]
        assert np.abs(tam.astype(np.float64) - g["transform_aft_mapped"][k]).max() <= 1e-4, k
        if not np.array_equal(tam.view(np.uint32), g["transform_aft_mapped"][k].view(np.uint32)):
            bad.append((k, "transform_aft_mapped",
                        float(np.abs(tam.astype(np.float64) - g["transform_aft_mapped"][k]).max())))
    assert not bad, f"{len(bad)} differing (scan, field, delta), first: {bad[:6]}"


def test_oracle_reproduces_imu_fixture(L):
    g = load("vlp16_seed6_imu100_map24")
    outs = _imu_fixture_run(L, g, L.Oracle(L.sensor_cfg("VLP-16")), False)
    _check_imu_fixture(g, outs)


@pytest.mark.gpu
def test_product_reproduces_imu_fixture(L):
    """/imu_raw through lego_imu_push + the node calls: IMU deskew, initial
    guess, integration, hand-off and the mapping blend."""
    g = load("vlp16_seed6_imu100_map24")
    eng = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000)
    outs = _imu_fixture_run(L, g, eng, True)
    eng.close()
    _check_imu_fixture(g, outs)


@pytest.mark.gpu
def test_product_reproduces_imu_fixture_batched(L):
    """The same stream through lego_odom_batch_imu in three batches, the
    messages of each batch scheduled by imu_before."""
    g = load("vlp16_seed6_imu100_map24")
    sc = L.synth_cfg("VLP-16", int(g["seed"]))
    imu = g["imu"].view(L.IMU_DTYPE)
    before = g["imu_before"].astype(np.int64)
    n = len(before)
    scans = [L.synth_scan(sc, k) for k in range(n)]
    eng = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=10)
    recs = []
    j0 = 0
    for lo, hi in ((0, 7), (7, 15), (15, n)):
        pts = np.concatenate([p for p, _ in scans[lo:hi]])
        off = np.zeros(hi - lo + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p, _ in scans[lo:hi]])
        j1 = int(before[hi]) if hi < n else len(imu)  # this batch's messages end where the next scan's start
        b = (before[lo:hi] - j0).astype(np.int32)
        recs += list(eng.odom_batch(pts, off, np.array([s for _, s in scans[lo:hi]]), imu[j0:j1], b))
        j0 = j1
    eng.close()
    bad = []
    for k, r in enumerate(recs):
        c = [r.n_segmented, r.n_sharp, r.n_less_sharp, r.n_flat, r.n_less_flat, r.odom_valid]
        np.testing.assert_array_equal(c, g["counts"][k][:6], err_msg=str(k))
        ts = np.array(list(r.transform_sum), np.float32)
        assert np.abs(ts.astype(np.float64) - g["transform_sum"][k]).max() <= 1e-4, k
        if not np.array_equal(ts.view(np.uint32), g["transform_sum"][k].view(np.uint32)):
            bad.append((k, float(np.abs(ts.astype(np.float64) - g["transform_sum"][k]).max())))
    assert not bad, f"{len(bad)} scans' poses differ, first (scan, delta): {bad[:6]}"


@pytest.mark.gpu
def test_product_fusion_matches_oracle(L):
    """transformFusion after every scan of the keyframe-mapping stream: the
    product's /integrated_to_init equals the oracle's (mapping corrections
    arriving every 0.3 s)."""
    g = load("vlp16_seed6_keyframe_map24")
    sc = L.synth_cfg("VLP-16", int(g["seed"]))
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000)
    exact = 0
    for k in range(len(g["info"])):
        pts, stamp = L.synth_scan(sc, k)
        for e in (ora, gpu):
            e.ip(pts, stamp)
            e.fa()
            e.mo()
        a, b = ora.fusion(), gpu.fusion()
        assert np.abs(a.astype(np.float64) - b).max() <= 1e-4, (k, a, b)
        exact += int(np.array_equal(a.view(np.uint32), b.view(np.uint32)))
    gpu.close()
    print(f"fusion: bit-exact {exact}/{len(g['info'])}")
    assert exact == len(g["info"])
