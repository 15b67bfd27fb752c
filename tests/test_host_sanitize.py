"""CPU sanitizer build of the host code (VERDICT r3
item 8): the parsers that read file bytes on the host -- the FFV1
configuration record and the slice-footer walk (csrc/ffv1host.cpp), the p02
byte scanners (csrc/scan.cpp) -- and the swscale filter construction
(csrc/filters.cpp) built with g++ -fsanitize=address,undefined
(`make -C processing-chain_amd sanitize`) and fuzzed by csrc/fuzz_host.cpp
with seeded mutations: at least 10k corrupt packets and records per seed, no
sanitizer report, and every accepted slice table inside its frame."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "processing-chain_amd")


@pytest.fixture(scope="module")
def fuzzer():
    if not shutil.which("g++"):
        pytest.skip("no g++")
    p = subprocess.run(["make", "-C", PKG, "sanitize"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    return os.path.join(PKG, "build", "san", "fuzz_host")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_host_parsers_under_asan_ubsan(fuzzer, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([fuzzer, "20000", str(seed)], capture_output=True, text=True, timeout=600, env=env)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out and "LeakSanitizer" not in out
    counts = dict(zip(*[iter(p.stdout.split())] * 2))
    assert int(counts["records"]) >= 10000 and int(counts["packets"]) >= 10000 and counts["failures"] == "0"
