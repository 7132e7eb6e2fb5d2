"""Register budget of the sort kernels, read from the built code object (CPU).

Both GPU faults of rounds 4-5 came from builds of k_lf_voxel that carried the
register form of the VoxelGrid block sort (vg_block_sort) and spilled VGPRs
under the kernel's 128-VGPR cap; every spill-free kernel that
runs the same sort has passed the permutation and parity tests.  The product
therefore keeps the register form out of k_lf_voxel, and this test keeps the
rule checkable: every kernel that runs a workgroup sort of lego_vgsort.h
(either form) is built without VGPR spills or scratch.

The metadata come from liblego_hip.so's gfx950 code object
(.hip_fatbin -> clang-offload-bundler -> llvm-readelf --notes)."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
LIB = REPO / "lego-loam_amd/build/liblego_hip.so"
LLVM = Path("/opt/rocm/llvm/bin")

# kernels running vg_block_sort (register form) or vg_block_sort_sid (LDS-id
# form), by mangled-name prefix
SORT_KERNELS = ["_ZN4lego16k_vg_local_small", "_ZN4lego10k_vg_localE", "_ZN4lego11k_sort_perm",
                "_ZN4lego16k_sort_perm_form", "_ZN4lego10k_lf_voxel"]


def kernel_metadata(tmp: Path) -> dict:
    objcopy = shutil.which("objcopy")
    bundler, readelf = LLVM / "clang-offload-bundler", LLVM / "llvm-readelf"
    if not (objcopy and bundler.exists() and readelf.exists()):
        pytest.skip("binutils / ROCm LLVM tools not found")
    if not LIB.exists():
        from conftest import ensure_built

        ensure_built()
    fat = tmp / "fatbin.bin"
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", str(LIB), str(tmp / "lib.tmp")], check=True)
    raw = fat.read_bytes()  # one offload bundle per translation unit, back to back
    starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", raw)] + [len(raw)]
    notes = ""
    for i in range(len(starts) - 1):
        part, co = tmp / f"bundle{i}.bin", tmp / f"co{i}.elf"
        part.write_bytes(raw[starts[i]:starts[i + 1]])
        subprocess.run([str(bundler), "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes += subprocess.run([str(readelf), "--notes", str(co)], check=True, capture_output=True,
                                text=True).stdout
    out, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.match(r"\s+\.(private_segment_fixed_size|vgpr_spill_count|vgpr_count|sgpr_spill_count):\s+(\d+)", line)
        if m and cur is not None:
            out[cur][m.group(1)] = int(m.group(2))
    return out


def test_sort_kernels_build_without_spills(tmp_path):
    md = kernel_metadata(tmp_path)
    sort = {k: v for k, v in md.items() if any(k.startswith(p) for p in SORT_KERNELS)}
    assert any(k.startswith("_ZN4lego10k_lf_voxel") for k in sort), sorted(md)[:20]
    assert any(k.startswith("_ZN4lego16k_vg_local_small") for k in sort)
    for k, v in sorted(sort.items()):
        print(f"{k:70s} vgpr {v.get('vgpr_count')} spill {v.get('vgpr_spill_count')} "
              f"scratch {v.get('private_segment_fixed_size')}")
    bad = {k: v for k, v in sort.items() if v.get("vgpr_spill_count", 0) or v.get("private_segment_fixed_size", 0)}
    assert not bad, f"sort kernels spilling VGPRs / using scratch: {bad}"
