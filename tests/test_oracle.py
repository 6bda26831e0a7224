"""C oracle vs the golden fixtures produced by the independent Python spec (CPU only).

Pins the oracle before it is trusted as the checker for the HIP path (task rule 3).
Parity against the reference itself is unpinned: the reference holds no code or vectors.
"""
import hashlib
import random

import pytest

from oracle import oracle as O
from oracle.pyspec import curves as pc
from oracle.pyspec import kzg as pk

CURVES = ["bls12_381", "bn254"]
SIZES = {"bls12_381": [4, 16, 256], "bn254": [4, 16, 64]}


def h(x):
    return bytes.fromhex(x)


def test_sha256_and_randomizers():
    for m in [b"", b"abc", bytes(range(55)), bytes(range(56)), bytes(range(64)), bytes(200)]:
        assert O.sha256(m) == hashlib.sha256(m).digest()
    seed = bytes(range(32))
    for i in [0, 1, 2, 1 << 20, (1 << 63) + 5]:
        assert O.randomizer(seed, i) == pk.randomizer(seed, i)
        assert 0 < O.randomizer(seed, i) < 1 << 127


@pytest.mark.parametrize("curve", CURVES)
def test_pairing_kat(curve, golden):
    g = golden("%s_pairing.json" % curve)
    assert O.pairing(curve, h(g["g1"]), h(g["g2"])).hex() == g["e_g1_g2"]
    assert O.pairing(curve, h(g["aP"]), h(g["bQ"])).hex() == g["e_aP_bQ"]


@pytest.mark.parametrize("curve", CURVES)
def test_msm_golden(curve, golden):
    g = golden("%s_msm.json" % curve)
    for case in g["cases"]:
        got = O.msm_g1(curve, h(case["points"]), h(case["scalars"]), case["n"])
        assert got.hex() == case["expected"], case["name"]


@pytest.mark.parametrize("curve", CURVES)
def test_batch_golden(curve, golden):
    for n in SIZES[curve]:
        g = golden("%s_batch_n%d.json" % (curve, n))
        for key in ["valid", "neg_flip_y", "neg_swap_proofs"]:
            src = g if key == "valid" else g[key]
            exp = g[key]
            ok, A, B = O.batch_verify(curve, h(src["commitments"]), h(src["zs"]), h(src["ys"]),
                                      h(src["proofs"]), n, h(g["g2"]), h(g["tau_g2"]), h(g["seed"]),
                                      want_ab=True)
            assert ok == exp["ok"], (n, key)
            assert A.hex() == exp["A"], (n, key)
            assert B.hex() == exp["B"], (n, key)


@pytest.mark.parametrize("curve", CURVES)
def test_tuned_verifier_golden(curve, golden):
    """The tuned CPU verifier (oracle/c/pippenger_tuned_tmpl.h, bench.py's CPU baseline) gives
    the golden A, B and verdict bit for bit -- at several window widths and with point ranges
    cut into several tasks (chunk 3: ragged last chunks, G1 only in the first)."""
    for n in SIZES[curve]:
        g = golden("%s_batch_n%d.json" % (curve, n))
        for key in ["valid", "neg_flip_y", "neg_swap_proofs"]:
            src = g if key == "valid" else g[key]
            exp = g[key]
            for c, chunk in ((4, 3), (9, 0), (13, 0), (11, 5)):
                ok, A, B = O.batch_verify_tuned(curve, h(src["commitments"]), h(src["zs"]), h(src["ys"]),
                                                h(src["proofs"]), n, h(g["g2"]), h(g["tau_g2"]), h(g["seed"]),
                                                wbits=c, chunk=chunk, pairing=c == 13)
                assert (A.hex(), B.hex()) == (exp["A"], exp["B"]), (n, key, c, chunk)
                assert ok == (exp["ok"] if c == 13 else None), (n, key, c, chunk)


@pytest.mark.parametrize("curve", CURVES)
def test_tuned_pairing_equals_oracle(curve, golden):
    """The tuned verifier's pairing (Miller program precomputed from Q, easy part + 4-term
    Frobenius multi-exponent hard part with cyclotomic squarings, oracle/gen_fexp.py) gives the
    oracle's 12 Fp values bit for bit, on the golden pairs and on the point at infinity."""
    g = golden("%s_pairing.json" % curve)
    for P, Q in ((g["g1"], g["g2"]), (g["aP"], g["bQ"]), (g["g1"], g["bQ"])):
        assert O.pairing_fast(curve, h(P), h(Q)) == O.pairing(curve, h(P), h(Q))
    inf = bytes([0x40]) + bytes(95) if curve == "bls12_381" else bytes(64)
    assert O.pairing_fast(curve, inf, h(g["g2"])) == O.pairing(curve, inf, h(g["g2"]))


@pytest.mark.parametrize("curve", CURVES)
def test_tuned_verifier_vs_oracle_random(curve):
    """Random points (not openings: the verdict is False) with repeated and infinity points,
    A, B of the tuned verifier == the oracle's; empty batch accepts; errors as the oracle's."""
    C = pc.CURVES[curve]
    rng = random.Random(7)
    n = 300
    ks = [rng.randrange(C.r) for _ in range(n)]
    ks[5] = ks[9] = ks[17]   # equal points: doublings inside the buckets
    ks[11] = 0               # the point at infinity
    ks[12] = C.r - ks[13]    # P and -P
    pts = O.g1_mul_gen(curve, b"".join(pk.fr_to_bytes(k) for k in ks), n)
    cm, pf = pts, O.g1_mul_gen(curve, b"".join(pk.fr_to_bytes(k * 3 % C.r) for k in ks), n)
    zs = b"".join(pk.fr_to_bytes(rng.randrange(C.r)) for _ in range(n))
    ys = b"".join(pk.fr_to_bytes(rng.randrange(C.r)) for _ in range(n))
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, 99)
    seed = bytes(range(32))
    want = O.batch_verify(curve, cm, zs, ys, pf, n, g2, tg2, seed, want_ab=True)
    assert O.batch_verify_tuned(curve, cm, zs, ys, pf, n, g2, tg2, seed) == want
    assert O.batch_verify_tuned(curve, cm, zs, ys, pf, n, g2, tg2, seed, wbits=7, chunk=64,
                                pairing=False) == (None,) + want[1:]
    assert O.batch_verify_tuned(curve, b"", b"", b"", b"", 0, g2, tg2, seed)[0] is True
    bad = bytearray(zs)
    bad[32:64] = C.r.to_bytes(32, "big")
    with pytest.raises(O.OracleError) as e:
        O.batch_verify_tuned(curve, cm, bytes(bad), ys, pf, n, g2, tg2, seed)
    assert e.value.code == -4


@pytest.mark.parametrize("curve", CURVES)
def test_genuine_kzg(curve, golden):
    g = golden("%s_genuine_kzg.json" % curve)
    ok = O.batch_verify(curve, h(g["commitments"]), h(g["zs"]), h(g["ys"]), h(g["proofs"]), g["n"],
                        h(g["g2"]), h(g["tau_g2"]), h(g["seed"]))
    assert ok is True


@pytest.mark.parametrize("curve", CURVES)
def test_empty_batch_and_errors(curve, golden):
    g = golden("%s_batch_n4.json" % curve)
    assert O.batch_verify(curve, b"", b"", b"", b"", 0, h(g["g2"]), h(g["tau_g2"]), h(g["seed"]))
    C = pc.CURVES[curve]
    # non-canonical scalar -> error code, not ok=0
    zs = bytearray(h(g["zs"]))
    zs[0:32] = (C.r).to_bytes(32, "big")
    with pytest.raises(O.OracleError) as e:
        O.batch_verify(curve, h(g["commitments"]), bytes(zs), h(g["ys"]), h(g["proofs"]), 4,
                       h(g["g2"]), h(g["tau_g2"]), h(g["seed"]))
    assert e.value.code == -4
    # off-curve commitment
    cm = bytearray(h(g["commitments"]))
    cm[2 * C.fp_bytes - 1] ^= 1
    with pytest.raises(O.OracleError) as e:
        O.batch_verify(curve, bytes(cm), h(g["zs"]), h(g["ys"]), h(g["proofs"]), 4,
                       h(g["g2"]), h(g["tau_g2"]), h(g["seed"]))
    assert e.value.code == -3


@pytest.mark.parametrize("curve", CURVES)
def test_msm_discrete_log_identity(curve):
    """MSM(k_i G, s_i) == (sum k_i s_i) G: size-independent known-answer identity."""
    C = pc.CURVES[curve]
    rng = random.Random(11)
    n = 3000
    ks = [rng.randrange(C.r) for _ in range(n)]
    ss = [rng.randrange(C.r) for _ in range(n)]
    pts = O.g1_mul_gen(curve, b"".join(pk.fr_to_bytes(k) for k in ks), n)
    got = O.msm_g1(curve, pts, b"".join(pk.fr_to_bytes(s) for s in ss), n)
    tot = sum(k * s for k, s in zip(ks, ss)) % C.r
    assert got == O.g1_mul_gen(curve, pk.fr_to_bytes(tot), 1)


def test_sharded_msm_equals_unsharded():
    """The multi-GPU decomposition (split the point range, add partials) on the oracle."""
    curve = "bls12_381"
    C = pc.CURVES[curve]
    rng = random.Random(3)
    n = 700
    ks = [rng.randrange(C.r) for _ in range(n)]
    ss = [rng.randrange(C.r) for _ in range(n)]
    pts = O.g1_mul_gen(curve, b"".join(pk.fr_to_bytes(k) for k in ks), n)
    scs = b"".join(pk.fr_to_bytes(s) for s in ss)
    full = pk.g1_from_bytes(O.msm_g1(curve, pts, scs, n), C)
    acc = None
    for lo, hi in [(0, 100), (100, 350), (350, 351), (351, 700)]:
        part = O.msm_g1(curve, pts[lo * 96:hi * 96], scs[lo * 32:hi * 32], hi - lo)
        acc = pc.g1_add(acc, pk.g1_from_bytes(part, C), C)
    assert acc == full


# ---------------------------------------------------------------- SURVEY.md 8f item 1
@pytest.mark.parametrize("curve", CURVES)
def test_compressed_roundtrip_oracle_vs_spec(curve, golden):
    """Compressed encodings: C oracle == Python spec, both directions, on golden points."""
    C = pc.CURVES[curve]
    g = golden("%s_batch_n16.json" % curve)
    pts = bytes.fromhex(g["commitments"]) + bytes.fromhex(g["proofs"])
    n = len(pts) // (2 * C.fp_bytes)
    comp = O.g1_compress(curve, pts, n)
    g1b, fb = 2 * C.fp_bytes, C.fp_bytes
    assert comp == b"".join(pk.g1_to_bytes_compressed(pk.g1_from_bytes(pts[i * g1b:(i + 1) * g1b], C), C)
                            for i in range(n))
    rc, back = O.g1_decompress(curve, comp, n)
    assert rc == 0 and back == pts
    for i in range(n):
        assert pk.g1_from_bytes_compressed(comp[i * fb:(i + 1) * fb], C) == pk.g1_from_bytes(pts[i * g1b:(i + 1) * g1b], C)
    inf = pk.g1_to_bytes_compressed(None, C)
    assert O.g1_decompress(curve, inf, 1) == (0, pk.g1_to_bytes(None, C))


@pytest.mark.parametrize("curve", CURVES)
def test_invalid_compressed(curve):
    from pointcases import invalid_compressed
    C = pc.CURVES[curve]
    for enc, want in invalid_compressed(C):
        rc, _ = O.g1_decompress(curve, enc, 1)
        assert rc == want, (enc.hex(), rc, want)
        with pytest.raises(ValueError):
            pk.g1_from_bytes_compressed(enc, C)


@pytest.mark.parametrize("curve", ["bls12_381", "bn254"])
def test_invalid_uncompressed_cases(curve):
    """The uncompressed cases the GPU validation test expects errors for are the ones the
    Python spec's decoder rejects, and the valid ones decode to the identity."""
    import random
    from pointcases import invalid_uncompressed
    C = pc.CURVES[curve]
    for enc, want in invalid_uncompressed(C, random.Random(41)):
        if want is None:
            assert pk.g1_from_bytes(enc, C) is None
        else:
            with pytest.raises(ValueError):
                pk.g1_from_bytes(enc, C)


def test_subgroup_definition():
    """Oracle subgroup check ([r]P == O) on members, random non-members and small-order points."""
    from pointcases import subgroup_cases
    C = pc.BLS12_381
    for P, member in subgroup_cases():
        assert O.g1_subgroup_check("bls12_381", pk.g1_to_bytes(P, C), 1) is member
        assert pc.g1_in_subgroup(P, C) is member


# ---------------------------------------------------------------- SURVEY.md 8f item 2
def test_fs_zero_chunk_constant():
    """kFsZeroChunk in csrc/fs.hpp == root of an all-zero 4096-slot subtree."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "kzg-batch-verification-scheme_amd", "csrc",
                            "fs.hpp")).read()
    words = re.search(r"kFsZeroChunk\[8\] = \{([^}]*)\}", src).group(1)
    const = b"".join(int(w.strip().rstrip("u"), 16).to_bytes(4, "big") for w in words.split(","))
    assert const == pk.merkle_root([bytes(32)] * 4096)


@pytest.mark.parametrize("curve", CURVES)
def test_powers_mode_oracle_vs_spec(curve, golden):
    """r_i = r^i with the Fiat-Shamir r: C oracle == Python spec (A, B, verdict), incl. shards."""
    from fsref import fs_challenge_bytes
    C = pc.CURVES[curve]
    g = golden("%s_batch_n16.json" % curve)
    h = bytes.fromhex
    n, g1b = 16, 2 * C.fp_bytes
    cm, pf, zb, yb = h(g["commitments"]), h(g["proofs"]), h(g["zs"]), h(g["ys"])
    pts = lambda b: [pk.g1_from_bytes(b[i * g1b:(i + 1) * g1b], C) for i in range(n)]  # noqa: E731
    ints = lambda b: [int.from_bytes(b[32 * i:32 * i + 32], "big") for i in range(n)]  # noqa: E731
    r = pk.fs_challenge(pts(cm), ints(zb), ints(yb), pts(pf), C)
    assert r == fs_challenge_bytes(curve, cm, zb, yb, pf, n)
    ok, A, B = O.batch_verify_powers(curve, cm, zb, yb, pf, n, h(g["g2"]), h(g["tau_g2"]), r)
    As, Bs = pk.batch_combination(pts(cm), ints(zb), ints(yb), pts(pf), b"", C, powers_of=r)
    assert ok is True and A == pk.g1_to_bytes(As, C) and B == pk.g1_to_bytes(Bs, C)
    # shard partials with offsets add up to the whole
    _, A0, B0 = O.batch_verify_powers(curve, cm[:5 * g1b], zb[:160], yb[:160], pf[:5 * g1b], 5, h(g["g2"]),
                                      h(g["tau_g2"]), r, offset=0, pairing=False)
    _, A1, B1 = O.batch_verify_powers(curve, cm[5 * g1b:], zb[160:], yb[160:], pf[5 * g1b:], 11, h(g["g2"]),
                                      h(g["tau_g2"]), r, offset=5, pairing=False)
    assert pc.g1_add(pk.g1_from_bytes(A0, C), pk.g1_from_bytes(A1, C), C) == As
    assert pc.g1_add(pk.g1_from_bytes(B0, C), pk.g1_from_bytes(B1, C), C) == Bs
    yb2 = bytearray(yb)
    yb2[31] ^= 1
    assert O.batch_verify_powers(curve, cm, zb, bytes(yb2), pf, n, h(g["g2"]), h(g["tau_g2"]), r)[0] is False


@pytest.mark.parametrize("curve", CURVES)
def test_fiat_shamir_mode_oracle_vs_spec(curve, golden):
    """KZGMI_FLAG_FIAT_SHAMIR: seeded 127-bit r_i with seed = be32(r_FS): C oracle == spec."""
    C = pc.CURVES[curve]
    g = golden("%s_batch_n16.json" % curve)
    h = bytes.fromhex
    n, g1b = 16, 2 * C.fp_bytes
    cm, pf, zb, yb = h(g["commitments"]), h(g["proofs"]), h(g["zs"]), h(g["ys"])
    pts = lambda b: [pk.g1_from_bytes(b[i * g1b:(i + 1) * g1b], C) for i in range(n)]  # noqa: E731
    ints = lambda b: [int.from_bytes(b[32 * i:32 * i + 32], "big") for i in range(n)]  # noqa: E731
    seed = pk.fs_seed(pts(cm), ints(zb), ints(yb), pts(pf), C)
    ok, A, B = O.batch_verify(curve, cm, zb, yb, pf, n, h(g["g2"]), h(g["tau_g2"]), seed, want_ab=True)
    As, Bs = pk.batch_combination(pts(cm), ints(zb), ints(yb), pts(pf), seed, C)
    assert ok is True and A == pk.g1_to_bytes(As, C) and B == pk.g1_to_bytes(Bs, C)
    assert all(pk.randomizer(seed, i) < 1 << 127 for i in range(n))
