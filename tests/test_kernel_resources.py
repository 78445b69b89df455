"""Build-time register budget of the reduce kernel (CPU: hipcc cross-compiles gfx950).

``wc_reduce_buckets`` must not spill VGPRs to scratch.  A round-6 build whose
reduce batch spilled 1-2 VGPRs (16 B/lane) lost and misattributed records
(``test_gpu_engine.py::test_random_vs_oracle[0]``: 76 keys missing, 166 with wrong
counts or first offsets) while the same logic built without the spill (one
record fewer in flight per lane) passed the whole GPU suite
(``profiles/r6_session.md`` §6).  Until that is explained, a reduce that spills
does not ship: this test reads the compiler's resource report of every
instance and fails on scratch use.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="hipcc not installed")
def test_reduce_kernel_does_not_spill(tmp_path):
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    out = subprocess.run(
        [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
         "-I" + os.path.join(ROOT, "src"), "-I/opt/rocm/include", "-c",
         os.path.join(ROOT, "src", "kernels", "reduce.hip"), "-o", str(tmp_path / "reduce.o"),
         "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    name = None
    found = {}
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name and "wc_reduce_buckets" in name:
            found[name] = int(m.group(1))
    assert found, "no wc_reduce_buckets instance in the resource report"
    assert all(v == 0 for v in found.values()), f"wc_reduce_buckets spills to scratch: {found}"


def _loops_with(asm_lines, start, end, marker, max_len=800):
    """(label, first, last) of every innermost-sized loop (a backward branch to a
    label) in asm_lines[start:end] whose body holds `marker`."""
    labels = {}
    out = []
    for i in range(start, end):
        m = re.match(r"^(\.LBB\d+_\d+):", asm_lines[i])
        if m:
            labels[m.group(1)] = i
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", asm_lines[i])
        if m and m.group(1) in labels and i - labels[m.group(1)] < max_len:
            a = labels[m.group(1)]
            if any(marker in l for l in asm_lines[a:i + 1]):
                out.append((m.group(1), a, i))
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="hipcc not installed")
def test_map_token_steps_do_not_touch_scratch(tmp_path):
    """The map runs at 16 waves per CU (128 VGPRs per wave) and spills a few
    VGPRs, but only outside its token loop (``profiles/r6_map_geometry.md``):
    every step loop — the loops that hold the hot-table probe, four
    ``ds_read_b128`` of candidate groups — must be free of scratch traffic in
    every ``wc_map`` instance.  A change that moves a spill into a step (a
    longer-lived value across the step, as tried in ``r6_session.md`` §22) fails
    here before it reaches a GPU."""
    hipcc = HIPCC if os.path.exists(HIPCC) else shutil.which("hipcc")
    asm = tmp_path / "map.s"
    out = subprocess.run(
        [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
         "-I" + os.path.join(ROOT, "src"), "-I/opt/rocm/include", "--cuda-device-only", "-S",
         os.path.join(ROOT, "src", "kernels", "map.hip"), "-o", str(asm)],
        capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = asm.read_text().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_ZN2wc3dev6wc_mapILb[01]ELb[01]EEEvNS_7MapArgsENS_7HotArgsE:", l)]
    assert len(starts) == 4, "expected the four wc_map instances"
    for s in starts:
        e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
        loops = _loops_with(lines, s, e, "ds_read_b128")
        assert loops, f"no probe loop found in {lines[s]}"
        for label, a, b in loops:
            bad = [l.strip() for l in lines[a:b + 1] if re.match(r"\s*(scratch|buffer)_(load|store)", l)]
            assert not bad, f"{lines[s].split(':')[0]} step loop {label} touches scratch: {bad[:4]}"
