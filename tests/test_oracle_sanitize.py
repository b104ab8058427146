"""CPU: the oracle (C restatement, test infrastructure) under AddressSanitizer
and UndefinedBehaviorSanitizer.  oracle/sanitize/driver.c
calls every oracle entry point -- the three PFDR solvers in all their modes,
the metric projection, the CP reduced-problem builder and the CP graph
steps -- on small synthetic graphs (including an edgeless one, a path, a
self-loop and a duplicate edge); any out-of-bounds access, leak-free misuse
or undefined operation aborts the run with a non-zero status."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "..", "oracle", "sanitize", "driver.c")


def test_oracle_clean_under_asan_ubsan(tmp_path):
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc absent")
    exe = str(tmp_path / "oracle_sanitized")
    flags = ["-std=c99", "-O1", "-g", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-ffp-contract=off"]
    r = subprocess.run([cc, *flags, "-o", exe, DRIVER, "-lm"], capture_output=True, text=True)
    if r.returncode != 0 and "asan" in (r.stderr or "").lower():
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-4000:])
    assert "projection ok" in r.stdout
    assert r.stdout.count("solvers, CP steps ok") == 4
