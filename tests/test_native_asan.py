"""The native host runtime (csrc/runtime.cpp: block allocator, scheduler, safetensors reader)
compiled alone under AddressSanitizer + UndefinedBehaviorSanitizer and driven by a C++ test
(tests/native/runtime_host_test.cpp) - SURVEY 5.2's host-code sanitizer run. CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "runtime_host_test")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", os.path.join(HERE, "native", "runtime_host_test.cpp"), "-o", exe,
           "-pthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload other libraries ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    import resource

    def _few_fds():  # 3000 failing opens below leak-check the reader's fd / mapping cleanup
        resource.setrlimit(resource.RLIMIT_NOFILE, (512, 512))

    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120, env=env,
                       preexec_fn=_few_fds)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout


CTRL_MODES = ("threads", "timeout", "procs", "dead")


def _ctrl_build(tmp_path, name, sanitize):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer"] + sanitize + [
        os.path.join(HERE, "native", "ctrl_host_test.cpp"), "-o", exe, "-pthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return exe


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_ctrl_ring_under_asan_ubsan(tmp_path):
    """The shared-memory control ring (csrc/ctrl_ring.h, the leader -> follower step records of serving/driver.py)
    under ASan + UBSan: producer / 3 readers as threads on one mapping with wrap-around, fragmentation and a slow
    reader; both timeouts; two processes through the named ring; a producer process dying inside a fragmented
    message (tests/native/ctrl_host_test.cpp)."""
    exe = _ctrl_build(tmp_path, "ctrl_asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    for mode in CTRL_MODES:  # one process per mode: no fork after threads
        r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=180, env=env)
        assert r.returncode == 0 and "ALL OK" in r.stdout, (mode, r.stdout + r.stderr)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_ctrl_ring_under_tsan(tmp_path):
    """The same stress under ThreadSanitizer: the threads mode shares ONE mapping between the producer and the
    readers, so every access of the release/acquire protocol (write_pos, read_pos, the data bytes) is checked."""
    exe = _ctrl_build(tmp_path, "ctrl_tsan", ["-fsanitize=thread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    for mode in CTRL_MODES:
        r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0 and "ALL OK" in r.stdout and "ThreadSanitizer" not in r.stderr, \
            (mode, r.stdout + r.stderr)
