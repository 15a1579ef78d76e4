"""The host worker pool of the C ABI (sng_api.cpp HostPool / parallel_ranges), built on its own with g++
from the library's source text and stressed: ragged sections on 1-16 threads, every item exactly once,
no deadlock (ThreadSanitizer when the toolchain has it)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "smart-nanogrid-gym_amd", "csrc", "sng_api.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_pool_sections(tmp_path):
    text = open(SRC).read()
    a, b = text.index("class HostPool {"), text.index("// FNV-1a over a byte range")
    (tmp_path / "host_pool.inc").write_text(text[a:b])
    exe = str(tmp_path / "pool")
    base = ["g++", "-O2", "-std=c++17", "-I", str(tmp_path), os.path.join(ROOT, "tests", "native", "host_pool_check.cpp"),
            "-o", exe, "-lpthread"]
    if subprocess.run(base[:1] + ["-fsanitize=thread"] + base[1:], capture_output=True).returncode != 0:
        subprocess.run(base, check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "pool ok" in out.stdout, out.stdout + out.stderr
