"""Host-side sanitizer builds (the reference's CI runs --check-bounds=yes,
.github/workflows/CI.yml:72): libsrhip's host C++ (the compiler and its 64-shard code cache, the
persistent host pool, background teardown, finalize) built with AddressSanitizer + UBSan and with
ThreadSanitizer (host side only: -Xarch_host), driven by tools/host_stress.cpp from 8 threads at once.
Any sanitizer report fails the run (-fno-sanitize-recover=all; TSan exits 66 on a race).  No device is
used here; the GPU box runs the same drivers' device phase (coalescer, submitted evaluations, the split
optimiser)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_host_code_under_sanitizer(san):
    pkg = os.path.join(ROOT, "symbolicregression.jl_amd")
    if not os.path.exists(os.path.join(pkg, "build", "srhip_grad.o")):
        pytest.skip("device objects not built (run __graft_entry__.build())")
    subprocess.run(["make", "-s", "-j8", "-C", pkg, san], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools"), san], check=True)
    exe = os.path.join(ROOT, "tools", "build", f"host_stress_{san}")
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([exe, "8", "40"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "host_stress ok" in r.stdout and "Sanitizer" not in r.stderr, r.stderr[-6000:]
