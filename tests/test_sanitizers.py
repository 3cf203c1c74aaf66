"""Sanitizer builds of the host code (race detection /
sanitizers): the CPU oracle under AddressSanitizer + UBSan, and libjfsx's
host scheduling code (async queue, aggregator, per-device dispatchers,
multi-device context; juicefs_amd/csrc/jfsx_agg.cpp over the stub engine)
under ThreadSanitizer.  Host code only: GPU sanitizers are not used."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _run(cmd_build, exe, env=None):
    subprocess.check_call(cmd_build)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "WARNING: ThreadSanitizer" not in out.stderr, \
        out.stderr[-4000:]
    assert "runtime error" not in out.stderr, out.stderr[-4000:]
    return out.stdout


def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_asan")
    out = _run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                "-fno-omit-frame-pointer", "-o", exe, os.path.join(HERE, "harness", "oracle_asan.c"),
                "-lpthread", "-ldl"], exe,
               env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0"))
    assert "oracle sanitizer run ok" in out


# ROCm's clang: its TSan runtime intercepts pthread_cond_clockwait, which
# libstdc++ 11 uses for condition_variable::wait_until; GCC 11's TSan runtime
# does not, and then reports a spurious "double lock of a mutex".
CLANGXX = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANGXX), reason="ROCm clang++ not present")
def test_scheduler_under_tsan(tmp_path):
    exe = str(tmp_path / "agg_tsan")
    out = _run([CLANGXX, "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-I", os.path.join(ROOT, "include"),
                "-o", exe, os.path.join(HERE, "harness", "agg_tsan.cpp"), "-lpthread"], exe,
               env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1"))
    assert "scheduler sanitizer run ok" in out


def test_zstd_decoder_under_asan(tmp_path):
    # checksummed frames decoded into exactly sized outputs: the XXH64 tail
    # must not read past the decoded bytes (jfsx_zstd.h xxh64)
    exe = str(tmp_path / "zstd_asan")
    out = _run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                "-fno-omit-frame-pointer", "-o", exe, os.path.join(HERE, "harness", "zstd_asan.cpp"), "-ldl"], exe,
               env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0"))
    assert "zstd sanitizer run ok" in out
