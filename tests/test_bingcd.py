"""The word-level binary GCD inversion (csrc/bingcd.hpp, used by fp_inv on the device for MSM
results and by the pairing's Fp inversion), built for the host from the same header
(tools/bingcd_check.cpp) and checked against Python's pow(y, -1, m) on the four moduli of the
library (BLS12-381 p and r, BN254 p and r): edge values and random ones.  The device build runs
in every GPU MSM-encoding and pairing parity test."""
import os
import random
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODULI = {  # modulus: 32-bit limbs of the library's Fp<P>
    0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab: 12,
    0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001: 8,
    0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47: 8,
    0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001: 8,
}


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("bingcd") / "bingcd_check")
    subprocess.run([hipcc, "-O2", "-o", out, os.path.join(ROOT, "tools", "bingcd_check.cpp")], check=True,
                   capture_output=True, text=True)
    return out


def test_inverse_matches_pow(checker):
    rng = random.Random(20261017)
    cases = []
    for m, n in MODULI.items():
        ys = [1, 2, 3, m - 1, m - 2, (m + 1) // 2, 1 << 200, 1 << (m.bit_length() - 1), (1 << 64) - 1]
        ys += [rng.randrange(1, m) for _ in range(500)]
        ys += [rng.randrange(1, 1 << rng.randrange(1, m.bit_length())) for _ in range(200)]  # short values
        cases += [(n, m, y) for y in ys]
    inp = "".join(f"{n} {m.bit_length()} {m:x} {y:x}\n" for n, m, y in cases)
    out = subprocess.run([checker], input=inp, capture_output=True, text=True, check=True).stdout.split()
    assert len(out) == len(cases)
    bad = [(hex(m), hex(y)) for (n, m, y), o in zip(cases, out) if int(o, 16) != pow(y, -1, m)]
    assert not bad, bad[:3]


def test_zero_maps_to_zero(checker):
    m, n = next(iter(MODULI.items()))
    out = subprocess.run([checker], input=f"{n} {m.bit_length()} {m:x} 0\n", capture_output=True, text=True,
                         check=True).stdout.split()
    assert int(out[0], 16) == 0
