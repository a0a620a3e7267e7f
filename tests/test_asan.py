"""Host-side AddressSanitizer run of the C-ABI runtime (SURVEY §5 "race
detection / sanitizers"): tools/asan_build.sh instruments sw_api.cpp and the
driver tests/abi_asan.cpp (-Xarch_host -fsanitize=address; device code is
not instrumented).  CPU: the entry points that need no GPU; GPU: the whole
lifecycle of three model/stepper/precision combinations."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "asan_bin", "abi_asan")


def _run(*args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1")
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=300, env=env)


def test_asan_host_paths_without_gpu():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_build.sh")], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _run()
    assert r.returncode == 0 and "abi_asan: ok" in r.stdout, (r.stdout + r.stderr)[-3000:]
    assert "AddressSanitizer" not in r.stderr


@pytest.mark.gpu
def test_asan_full_lifecycle_on_gpu():
    if not os.path.exists(BIN):
        pytest.skip("tests/asan_bin/abi_asan not built (tools/asan_build.sh; __graft_entry__.build())")
    env_leaks = "detect_leaks=0"  # the HIP runtime's own allocations are not libsw's
    r = subprocess.run([BIN, "--gpu"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS=env_leaks + ":halt_on_error=1"))
    assert r.returncode == 0 and "abi_asan: ok" in r.stdout, (r.stdout + r.stderr)[-3000:]
    assert "AddressSanitizer" not in r.stderr
