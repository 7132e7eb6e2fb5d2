"""The drop-in boundary: the C-ABI library loads on this (GPU-less) host and
exports every entry point include/*.h declares; the ctypes mirror used by
tests/bench matches the C struct layouts; product presets equal the oracle's
restatement of utility.h bit for bit.  No compute calls here."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def declared(header: Path, prefix: str):
    txt = header.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"[a-z0-9_]+)\s*\(", txt)))


def test_hip_library_exports_every_declared_symbol(L):
    lib = C.CDLL(str(L.HIP_LIB))
    names = declared(REPO / "include/lego_loam.h", "lego_")
    assert len(names) >= 12, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(L.HIP_EXPORTS) <= set(names)


def test_synth_library_exports(L):
    lib = C.CDLL(str(L.SYNTH_LIB))
    names = declared(REPO / "include/lego_synth.h", "lego_synth_")
    assert names and all(hasattr(lib, n) for n in names)


def test_oracle_library_exports(L):
    lib = C.CDLL(str(L.ORACLE_LIB))
    names = declared(REPO / "oracle/lego_oracle.h", "lego_oracle_")
    assert names and all(hasattr(lib, n) for n in names)


def test_struct_layouts_match_ctypes(L, tmp_path):
    exe = tmp_path / "abi_layout"
    subprocess.run(["gcc", "-std=c99", "-I", str(REPO / "include"), str(REPO / "tests/native/abi_layout.c"),
                    "-o", str(exe)], check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                             check=True).stdout.splitlines())
    m = {"lego_point_xyzir": L.PointXYZIR, "lego_point_xyzi": L.PointXYZI, "lego_sensor_cfg": L.SensorCfg,
         "lego_cloud_info": L.CloudInfo, "lego_ip_out": L.IpOut, "lego_fa_out": L.FaOut,
         "lego_mo_out": L.MoOut, "lego_pose_rec": L.PoseRec, "lego_synth_cfg": L.SynthCfg,
         "lego_loop_out": L.LoopOut, "lego_mo_opts": L.MoOpts, "lego_ctx_opts": L.CtxOpts}
    for key, val in out.items():
        if "." in key:
            t, f = key.split(".")
            assert getattr(m[t], f).offset == int(val), key
        else:
            assert C.sizeof(m[key]) == int(val), key
    assert L.XYZIR_DTYPE.itemsize == 32 and L.XYZIR_DTYPE.fields["ring"][1] == 20


@pytest.mark.parametrize("name", ["VLP-16", "HDL-32E", "VLS-128", "OS1-16", "OS1-64", "HDL-64E"])
def test_presets_product_equals_oracle(L, name):
    a = L.sensor_cfg(name, L.hip_lib())
    b = L.sensor_cfg(name)
    assert bytes(a) == bytes(b)


def test_bad_inputs_rejected_without_device(L):
    lib = L.hip_lib()
    cfg = L.SensorCfg()
    assert lib.lego_sensor_preset(b"nope", C.byref(cfg)) == L.LEGO_E_ARG
    h = C.c_void_p()
    assert lib.lego_create(None, 0, 10, 1, C.byref(h)) == L.LEGO_E_ARG
    good = L.sensor_cfg("VLP-16", lib)
    bad = L.SensorCfg.from_buffer_copy(bytes(good))
    bad.n_scan = 4096  # > kMaxRings
    assert lib.lego_create(C.byref(bad), 0, 10, 1, C.byref(h)) == L.LEGO_E_ARG


def test_ctx_opts_defaults_and_validation(L):
    """lego_ctx_opts_init's defaults (host only, no device needed) and the
    size check of lego_create_ex."""
    lib = L.hip_lib()
    o = L.ctx_opts(lib)
    assert o.size == C.sizeof(L.CtxOpts)
    assert (o.node_overlap, o.front_parts, o.lfv_wave, o.lfv_wide, o.ccl_tiles, o.seg_hbm) == (1, 2, 1, -1, 1, 0)
    assert (o.odom_workgroups, o.odom_gridless, o.odom_integ, o.odom_silent_wg, o.odom_late_wg) == (0, -1, -1, -1, -1)
    assert (o.lf_wait_ms, o.mo_cand_cache, o.kf_cap, o.vg_rounds) == (2000, 1, 0, -1)
    bad = L.ctx_opts(lib)
    bad.size = 8
    h = C.c_void_p()
    cfg = L.sensor_cfg("VLP-16", lib)
    assert lib.lego_create_ex(C.byref(cfg), 0, 1000, 1, C.byref(bad), C.byref(h)) == L.LEGO_E_ARG
    neg = L.ctx_opts(lib, lf_wait_ms=-1)
    assert lib.lego_create_ex(C.byref(cfg), 0, 1000, 1, C.byref(neg), C.byref(h)) == L.LEGO_E_ARG


def test_no_environment_reads_in_the_library():
    """The shipped library's schedule is fixed by lego_ctx_opts at creation:
    no getenv anywhere in its sources."""
    import re
    src = REPO / "lego-loam_amd" / "csrc"
    hits = [f"{p.name}:{i + 1}" for p in sorted(src.iterdir()) if p.suffix in (".hip", ".h", ".cpp")
            and p.name != "lego_synth.cpp"
            for i, line in enumerate(p.read_text().splitlines()) if re.search(r"\bgetenv\b", line)]
    assert not hits, hits
