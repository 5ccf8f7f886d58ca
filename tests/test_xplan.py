"""The multi-GPU combines' host bookkeeping (zipkin_amd/csrc/zdl_xplan.h, used by zdl.hip's
sparse gathers and the insertion-order MIN across a job) against simulated ranks on the CPU:
tests/xplan_check.cpp includes the product header, builds every transfer plan for 1-8 ranks
(empty lists included), executes it with memcpy and checks the gathered buffers, the per-cell
sums and DependencyLinker.merge's order (DependencyLinker.java:189-204)."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("san", [[], ["-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]],
                         ids=["plain", "asan_ubsan"])
def test_xplan_against_simulated_ranks(san):
    """(asan_ubsan: the same header under AddressSanitizer + UBSan, the host-code sanitizer build
    SURVEY §5 lists; GPU sanitizers are not available on the pool)"""
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "xplan_check")
        subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", *san,
                        os.path.join(ROOT, "tests", "xplan_check.cpp"), "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
        assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
