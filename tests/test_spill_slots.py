"""Spill-slot audit of the product library's machine code (CPU).

Round 5's k_lf_voxel fault was never tied to an instruction.
Round 6 rebuilt the faulting instance (the register-form block sort in
k_lf_voxel<1024>, 9b2ac0a's tree: 128 VGPRs, 9 VGPRs and 23 SGPRs spilled, 40 B
of scratch) and audited its spills (tests/amdgcn_spills.py): no SGPR spill
slot is clobbered, no reload of one bypasses its write, every VGPR spill
store is in the prologue at full EXEC, and each of its 16 global memory
operations takes a base SGPR pair that is never spilled plus a checked or
lane-constant offset.  The spills are therefore not
the mechanism in that reconstruction.  What this test keeps is the pattern
that audit checks, for every kernel of the shipped library:
  * no SGPR spill slot's VGPR is written by anything but v_writelane, and none
    is stored to scratch (a partial-EXEC store would lose its lanes);
  * in the VoxelGrid sort kernels, no slot is reloaded on a control-flow path
    that skips every write of it.  (Other kernels have such reloads whose
    value is dead on that path, e.g. loop-carried restores; the path search is
    not path-sensitive, so they are listed, not failed.)"""
import os
import shutil
from pathlib import Path

import pytest

import amdgcn_spills as A

REPO = Path(__file__).resolve().parents[1]
LIB = REPO / "lego-loam_amd" / "build" / "liblego_hip.so"
SORT_KERNELS = ("k_lf_voxel", "k_vg_local", "k_sort_perm")


@pytest.fixture(scope="module")
def audits():
    if not (shutil.which("objcopy") and (A.LLVM / "llvm-objdump").exists()):
        pytest.skip("binutils / ROCm LLVM tools not found")
    if not LIB.exists():
        from conftest import ensure_built

        ensure_built()
    return {f: A.audit(ins) for f, ins in A.functions(A.disassemble(LIB)).items()}


def test_no_spill_slot_is_clobbered(audits):
    bad = {f: r["clobbers"][:3] for f, r in audits.items() if r["clobbers"]}
    assert not bad, bad
    assert sum(len(r["slots"]) for r in audits.values()) > 100  # the audit saw the spills (k_odom's among them)


def test_sort_kernels_reload_only_written_slots(audits):
    seen = [f for f in audits if any(k in f for k in SORT_KERNELS)]
    assert len(seen) >= 4, seen
    bad = {f: audits[f]["bypass"][:3] for f in seen if audits[f]["bypass"]}
    assert not bad, bad
    others = {f[:48]: len(r["bypass"]) for f, r in audits.items() if r["bypass"]}
    print("reloads on paths without a write (not asserted outside the sort kernels):", others)
