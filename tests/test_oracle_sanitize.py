"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (race /
memory checking of the CPU restatement): oracle/sanitize_main.c drives every routine of
oracle/sph_oracle.c -- lists, the single-phase and multiphase styles, integrators, fix
phase_change over CommBrick's swaps -- on small systems; any ASan/UBSan report or failed
invariant fails the test.  Host code only (no GPU sanitizer exists on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_clean_under_asan_ubsan(tmp_path):
    exe = tmp_path / "sanitize_check"
    b = subprocess.run(["gcc", "-O1", "-g", "-fno-omit-frame-pointer",
                        "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                        "-ffp-contract=off", "-std=c99", "-Wall", "-o", str(exe),
                        os.path.join(ROOT, "oracle", "sanitize_main.c"),
                        os.path.join(ROOT, "oracle", "sph_oracle.c"), "-lm"],
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    assert "atoms inserted" in r.stdout and "all oracle routines clean" in r.stdout
