"""The generated constant headers are what their generators produce now.

tools/gen_params29.py also runs check_bounds(): the value bounds of every step of the radix-2^29
accumulation loop, its doubling and the record addition/doubling, per curve, with the biases the
loop uses (msm.hpp acc_loop29) -- so this test fails if a bias role, NKP or a bias constant is
changed without the bounds still closing.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kzg-batch-verification-scheme_amd")


def _stdout(gen):
    return subprocess.run([sys.executable, os.path.join(PKG, "tools", gen)], check=True,
                          capture_output=True, text=True).stdout


def test_params29_in_sync_and_bounds_close():
    with open(os.path.join(PKG, "csrc", "params29_gen.hpp")) as f:
        assert _stdout("gen_params29.py") == f.read()


def test_params_lp_in_sync():
    with open(os.path.join(PKG, "csrc", "params_lp_gen.hpp")) as f:
        assert _stdout("gen_params_lp.py") == f.read()


def test_bound_checker_rejects_a_short_bias():
    """BN254 with the 1p negation bias (round 3's first attempt): the Montgomery conversion
    leaves points below (p / R29 + 1) p = 1.006 p, so 1p - y can go negative."""
    sys.path.insert(0, os.path.join(PKG, "tools"))
    try:
        import gen_params29 as g
    finally:
        sys.path.pop(0)
    name, p, n, r32, b, nkp, roles = g.CURVES[1]
    assert name == "Bn254Fp29"
    g.check_bounds(p, n, nkp, roles)
    bad = dict(roles, ACC_NEG=1)
    try:
        g.check_bounds(p, n, nkp, bad)
    except AssertionError:
        return
    raise AssertionError("check_bounds accepted ACC_NEG = 1p on BN254")


def test_bilinear_program_alias_ranges():
    """tools/gen_bilinear.py: every round's output block is disjoint from its input blocks as
    RANGES (pairing_par.hpp writes outputs straight into the register file with no barrier after
    the round's reads), for the shipped programs of both curves; an op whose output starts inside
    an input block (same start or not) is rejected."""
    import pytest
    sys.path.insert(0, os.path.join(PKG, "tools"))
    try:
        import gen_bilinear as g
    finally:
        sys.path.pop(0)
    for cv in ("bls12_381", "bn254"):
        g.build_program(cv)  # asserts on every op / op2
        P = g.Prog(cv)
        assert g.op_shape("LL", cv) == (6, 6, 12)
        with pytest.raises(AssertionError):
            P.op("MUL", P.g(0), P.g(1), P.g(0) + 6)   # output starts inside input A
        with pytest.raises(AssertionError):
            P.op("LL", P.e(0), P.e(0) + 6, P.e(0) + 3)
        with pytest.raises(AssertionError):
            P.op2("SQR", P.g(0), None, P.g(1), "LL", P.e(0), P.e(0) + 6, P.g(1) + 6)  # outputs overlap
        P.op("MUL", P.g(0), P.g(1), P.g(2))             # disjoint: accepted


def test_bilinear_cyc_runs_same_result_and_header_in_sync():
    """compress_cyc_runs (K_CYCRUN: chained cyclotomic squarings decoded once by the interpreter)
    leaves the program's result unchanged: check_program runs the compressed bytecode numerically
    against a direct Miller product + naive final exponentiation, for both curves; and the shipped
    header holds the compressed programs (NPROG)."""
    sys.path.insert(0, os.path.join(PKG, "tools"))
    try:
        import gen_bilinear as g
    finally:
        sys.path.pop(0)
    with open(os.path.join(PKG, "csrc", "bilinear_gen.hpp")) as f:
        hdr = f.read()
    for cv in ("bls12_381", "bn254"):
        tables = {name: g.build_op(fn, cv) for name, fn in g.OPS}
        P, res = g.build_program(cv)
        n0 = len(P.code)
        g.compress_cyc_runs(P)
        assert len(P.code) < n0
        assert any(ins[0] == g.K_CYCRUN for ins in P.code)
        g.check_program(cv, tables, P, res)
        assert "NPROG = %d," % len(P.code) in hdr
