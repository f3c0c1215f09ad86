"""Register budget of the hot kernels: the production 8-phase GEMM (and its split-K fix-up instantiation) must
compile for gfx950 with NO scratch (private-memory spills). A device call added to the kernel once made the compiler
spill 872 bytes per lane inside the main loop and the layer-1 GEMM ran 16 ms instead of 1.1 (profiles/r6_fixup) —
no numerics test notices that, so the compiler's own resource report is checked here, on the CPU (hipcc
cross-compiles without a GPU)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "netsdb_amd", "csrc", "kernels")


def _resources(src: str):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    p = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o", os.devnull,
                        "-Rpass-analysis=kernel-resource-usage"], cwd=KDIR, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-2000:]
    out, cur = {}, None
    for line in p.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).split()[0]] = int(m.group(2))
    return out


def test_gemm_8phase_kernels_do_not_spill():
    res = _resources("gemm.hip")
    hot = {k: v for k, v in res.items() if "gemm_nt_256_8ph" in k}
    assert len(hot) >= 4, sorted(res)                  # EPI 0 / 1 / 2 / 3 + the 32x32x16 loop
    for name, r in hot.items():
        assert r.get("ScratchSize", 0) == 0, (name, r)
        assert r.get("Occupancy", 0) >= 2, (name, r)   # two waves per SIMD: the ping-pong wave groups
