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
