"""Compile checks of the diagnostic variants kept in csrc/ (every preprocessor branch
is compiled either by the shipped build or by a test).  Only KZ_PROBE_STAMPS remains: the pairing
interpreter's per-round-class cycle counters (s_memtime sums printed by thread 0), used for the
breakdowns in profiles/.  hipcc cross-compiles gfx950 without a GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kzg-batch-verification-scheme_amd")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("curve,mode", [(0, "1"), (1, "1"), (0, "2")])
def test_probe_stamps_variant_compiles(tmp_path, curve, mode):
    """KZ_PROBE_STAMPS=1: per-phase stamps in every round; =2: loop-top stamps only."""
    out = tmp_path / "pairing_stamps.o"
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wno-unused-result",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "csrc"),
           "-DKZ_CURVE=%d" % curve, "-DKZ_PROBE_STAMPS=" + mode, "-c", os.path.join(PKG, "csrc", "launch_pairing.hip"),
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert out.stat().st_size > 0


def test_no_stale_ab_knobs():
    """The shipped sources name no A/B variant macro other than the kept ones."""
    import re
    allowed = {"KZ_DEV", "KZ_CURVE", "KZ_CURVE_T", "KZ_STR", "KZ_STR2", "KZ_TAIL_PRIO", "KZ_OPS_TABLE", "KZ_ROUTE",
               "KZ_STAMP", "KZ_STAMP_ARG", "KZ_STC", "KZ_PROBE_STAMPS", "KZ_PHASE_STAMPS", "KZ_CALL", "KZ_HD",
               # tuning constants with their shipped default defined in place (#ifndef X / #define X)
               "KZ_ACC_QUEUE_FACTOR", "KZ_ACC_QUEUE_FROM", "KZ_ACC29_WAVES", "KZ_ACC29_WAVES_BN", "KZ_SGC_WAVES",
               "KZ_PAR_THREADS"}
    found = set()
    csrc = os.path.join(PKG, "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hpp", ".hip")):
            with open(os.path.join(csrc, f)) as fh:
                found |= set(re.findall(r"\bKZ_[A-Z0-9_]+", fh.read()))
    assert found <= allowed, sorted(found - allowed)
