"""Spill-slot audit of gfx950 machine code (CPU; test infrastructure).

An SGPR the register allocator spills goes to a lane of a VGPR it reserves
(v_writelane_b32 vX, sY, L) and comes back with v_readlane_b32 sZ, vX, L.
Two ways such a slot can hand back a wrong value, the patterns round 5's
k_lf_voxel fault analysis checked:
  * the slot VGPR is written by anything else (a VALU op, a load, DPP), or is
    itself spilled to scratch (a partial-EXEC store would lose lanes);
  * a reload is reachable from the kernel's entry on a control-flow path that
    never executes a write of that slot (e.g. the write sits in a region an
    s_cbranch_execz skips).
audit() disassembles every kernel of a code object and reports both."""
from __future__ import annotations

import re
import subprocess
import tempfile
from collections import deque
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def disassemble(lib: Path) -> str:
    """llvm-objdump of every gfx950 code object bundled in a HIP shared library."""
    tmp = Path(tempfile.mkdtemp())
    fat = tmp / "fat.bin"
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(lib), str(tmp / "x")], check=True)
    raw = fat.read_bytes()
    starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", raw)] + [len(raw)]
    asm = ""
    for i in range(len(starts) - 1):
        part, co = tmp / f"b{i}", tmp / f"c{i}.co"
        part.write_bytes(raw[starts[i]:starts[i + 1]])
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        asm += subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", str(co)], check=True,
                              capture_output=True, text=True).stdout
    return asm


def functions(asm: str) -> dict[str, list[tuple[int, str]]]:
    """name -> [(address, instruction text)]"""
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = out.setdefault(m.group(1), [])
            continue
        m = re.search(r"//\s*([0-9A-F]{12}):", line)
        if cur is not None and m:
            cur.append((int(m.group(1), 16), line.split("//")[0].strip()))
    return out


def _vregs(s: str) -> list[int]:
    r = []
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", s):
        r += [int(m.group(3))] if m.group(3) else list(range(int(m.group(1)), int(m.group(2)) + 1))
    return r


_NO_VDST = ("s_", "v_cmp", "v_readlane", "v_readfirstlane", "ds_write", "ds_store", "global_store",
            "buffer_store", "scratch_store", "v_writelane")


def audit(ins: list[tuple[int, str]]) -> dict:
    wr, rd = {}, {}
    for i, (_, t) in enumerate(ins):
        m = re.match(r"v_writelane_b32 v(\d+), s\d+, (\d+)$", t)
        if m:
            wr.setdefault((int(m.group(1)), int(m.group(2))), []).append(i)
        m = re.match(r"v_readlane_b32 s\d+, v(\d+), (\d+)$", t)
        if m:
            rd.setdefault((int(m.group(1)), int(m.group(2))), []).append(i)
    slots = {k for k in wr if k in rd}
    vset = {v for v, _ in slots}
    clobbers = []
    for _, t in ins:
        op = t.split()[0]
        if op.startswith("scratch_store") and set(_vregs(t)) & vset:
            clobbers.append(t)
        if op.startswith(_NO_VDST) and not ("atomic" in op and "rtn" in op):
            continue
        args = t[len(op):].strip()
        d = re.split(r",(?![^\[]*\])", args)[0] if args else ""
        if set(_vregs(d)) & vset:
            clobbers.append(t)
    # control flow
    at = {a: i for i, (a, _) in enumerate(ins)}

    def succ(i):
        a, t = ins[i]
        op = t.split()[0]
        if op == "s_endpgm":
            return []
        out = [] if op in ("s_branch", "s_setpc_b64") else ([i + 1] if i + 1 < len(ins) else [])
        if op.startswith("s_cbranch") or op == "s_branch":
            k = int(t.split()[1])
            k = k - 65536 if k >= 32768 else k
            out.append(at[a + 4 + 4 * k])
        return out

    bypass = []
    for s in sorted(slots):
        block = set(wr[s])
        seen, q = {0}, deque([0])
        while q:
            i = q.popleft()
            for j in succ(i):
                if j not in seen and j not in block:
                    seen.add(j)
                    q.append(j)
        bypass += [(s, ins[r][0]) for r in rd[s] if r in seen]
    return {"slots": sorted(slots), "clobbers": clobbers, "bypass": bypass}
