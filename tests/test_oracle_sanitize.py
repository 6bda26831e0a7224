"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer.

`make -C oracle sanitize` builds oracle/build/liboracle_san.so from the same source with
-fsanitize=address,undefined (no recovery: any report aborts).  A child Python with libasan and
libubsan preloaded loads it through KZGO_LIB and runs the whole oracle test module (golden
vectors, MSM identities, shard sums, compressed/invalid encodings, powers and Fiat-Shamir
modes).  Host code only: GPU sanitizers are not available on the GPU pool."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", "-print-file-name=%s" % name], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_under_asan_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc sanitizer runtimes not installed")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    san = os.path.join(ROOT, "oracle", "build", "liboracle_san.so")
    env = dict(os.environ, LD_PRELOAD="%s:%s" % (asan, ubsan), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", KZGO_LIB=san, OMP_NUM_THREADS="4")
    probe = ("import sys; sys.path.insert(0, %r); from oracle import oracle as O; O.lib(); "
             "print(sum('liboracle_san.so' in l for l in open('/proc/self/maps')) > 0)" % ROOT)
    r = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "True", (r.stdout, r.stderr[-2000:])
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.join(ROOT, "tests", "test_oracle.py"), "-x", "-q",
                        "-p", "no:cacheprovider"], env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr
