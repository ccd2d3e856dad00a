"""Host sanitizer runs of the native runtime (race detection / sanitizers).

``csrc/runtime/rccl_comm.cpp`` (RCCL communicator, watchdog thread, bucket reducer) is compiled for the CPU with
ThreadSanitizer and with AddressSanitizer + UndefinedBehaviorSanitizer and linked against the HIP / RCCL fakes of
``csrc/tests/rt_sanitize.cpp``; the harness drives the watchdog-timeout + abort path against a hot issue loop,
the reducer with concurrent graph-replay tracking, and destroy with pending work.  Any sanitizer report or
fake-RCCL protocol violation (collective on an aborted communicator, abort during an enqueue) fails the test.
GPU sanitizers are not available on the MI355X pool; this covers the host threads, where the races live.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "runtime", "rccl_comm.cpp"), os.path.join(ROOT, "csrc", "tests", "rt_sanitize.cpp")]


def _build_and_run(tmp_path, flags, env_extra, argv=()):
    cxx = shutil.which("g++")
    if cxx is None or not os.path.exists("/opt/rocm/include/rccl/rccl.h"):
        pytest.skip("host C++ toolchain / ROCm headers not available")
    exe = str(tmp_path / "rt_sanitize")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-Wno-unused-result",
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", *SRC, "-o", exe, "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, *argv], capture_output=True, text=True, timeout=240, env=env)
    return r


def test_runtime_threadsanitizer(tmp_path):
    r = _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"})
    out = r.stdout + r.stderr
    assert "ThreadSanitizer" not in out, out[-4000:]
    assert r.returncode == 0 and "rt_sanitize: OK" in out, out[-4000:]


def test_runtime_address_ub_sanitizer(tmp_path):
    r = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                       {"ASAN_OPTIONS": "detect_leaks=1"})
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0 and "rt_sanitize: OK" in out, out[-4000:]


def test_abort_escalates_when_owner_is_stuck_inside_rccl(tmp_path):
    """Timeout action "abort" while the owning thread is blocked inside an RCCL enqueue (holding the issue
    lock): the watchdog must not abort underneath the call; it publishes error 4 and exits with code 3
    (advisor r3: the escalation was undocumented and untested)."""
    r = _build_and_run(tmp_path, [], {}, argv=("stuck",))
    out = r.stdout + r.stderr
    assert r.returncode == 3, out[-4000:]
    assert "stuck inside RCCL" in out and "rt_sanitize: stuck escalation observed" in out, out[-4000:]
