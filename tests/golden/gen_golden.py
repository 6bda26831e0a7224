"""Generate the committed golden fixtures from the pure-Python spec (oracle/pyspec).

The reference snapshot has no golden vectors (LICENSE only), so
these fixtures are produced by the independent Python big-int specification and pin both
the C oracle and the HIP product.  Deterministic (fixed seeds).  Run from the repo root:

    python tests/golden/gen_golden.py

Outputs tests/golden/*.json plus MANIFEST.json (sha256 of each file).
"""
import hashlib
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.pyspec.curves import (BLS12_381, BN254, g1_add, g1_mul, g1_msm, g1_neg,  # noqa: E402
                                  g2_mul)
from oracle.pyspec.kzg import (batch_combination, fr_to_bytes, g1_to_bytes, g2_to_bytes,  # noqa: E402
                               poly_commit_and_open, randomizer, toy_srs, valid_tuples)
from oracle.pyspec.pairing import flat_to_tower, pairing, multi_pairing_is_one  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def hx(b: bytes) -> str:
    return b.hex()


def fp12_hex(f, C):
    return hx(b"".join(v.to_bytes(C.fp_bytes, "big") for v in flat_to_tower(f, C)))


def constants():
    d = {}
    for C in (BLS12_381, BN254):
        d[C.name] = {
            "p": hex(C.p), "r": hex(C.r), "b": C.b, "xi": list(C.xi), "twist": C.twist,
            "g1": hx(g1_to_bytes(C.g1, C)), "g2": hx(g2_to_bytes(C.g2, C)),
            "loop": hex(C.loop), "loop_negative": C.loop_negative,
        }
    return d


def pairing_kat(C, rng):
    a = rng.randrange(1, C.r)
    b = rng.randrange(1, C.r)
    P = g1_mul(C.g1, a, C)
    Q = g2_mul(C.g2, b, C)
    return {
        "g1": hx(g1_to_bytes(C.g1, C)), "g2": hx(g2_to_bytes(C.g2, C)),
        "e_g1_g2": fp12_hex(pairing(C.g1, C.g2, C), C),
        "a": hex(a), "b": hex(b),
        "aP": hx(g1_to_bytes(P, C)), "bQ": hx(g2_to_bytes(Q, C)),
        "e_aP_bQ": fp12_hex(pairing(P, Q, C), C),
        "note": "e is the optimal-ate pairing; BLS12-381 values are e^3 (see pairing.py)",
    }


def msm_cases(C, rng):
    cases = []
    G = C.g1
    pts = [g1_mul(G, rng.randrange(1, C.r), C) for _ in range(6)]
    # edge cases
    defs = [
        ("single", [pts[0]], [rng.randrange(C.r)]),
        ("zero_scalar", [pts[0], pts[1]], [0, rng.randrange(C.r)]),
        ("infinity_point", [None, pts[1]], [rng.randrange(C.r), rng.randrange(C.r)]),
        ("cancel", [pts[2], g1_neg(pts[2], C)], [12345, 12345]),
        ("doubling_same_bucket", [pts[3], pts[3]], [7, 7]),
        ("r_minus_1", [pts[4]], [C.r - 1]),
        ("all_zero", [pts[0], pts[1]], [0, 0]),
        ("small_digits", pts, [1, 2, 3, 2**16 - 1, 2**16, 2**15]),
        ("top_window", pts[:3], [C.r - 2, (1 << 254) + 5 if (1 << 254) < C.r else C.r - 7, 2**127]),
    ]
    big_pts = [g1_mul(G, rng.randrange(1, C.r), C) for _ in range(33)]
    big_sc = [rng.randrange(C.r) for _ in range(33)]
    defs.append(("random_33", big_pts, big_sc))
    for name, P, S in defs:
        cases.append({
            "name": name, "n": len(P),
            "points": hx(b"".join(g1_to_bytes(p, C) for p in P)),
            "scalars": hx(b"".join(fr_to_bytes(s) for s in S)),
            "expected": hx(g1_to_bytes(g1_msm(P, S, C), C)),
        })
    return cases


def batch_fixture(C, n, seed_int):
    rng = random.Random(seed_int)
    tau = rng.randrange(2, C.r)
    g1, g2, tg2 = toy_srs(tau, C)
    tup = valid_tuples(n, tau, rng, C)
    seed = hashlib.sha256(b"kzgmi-golden-%d" % seed_int).digest()
    cm = [t[0] for t in tup]
    zs = [t[1] for t in tup]
    ys = [t[2] for t in tup]
    ps = [t[3] for t in tup]

    def enc(cm, zs, ys, ps):
        return {
            "commitments": hx(b"".join(g1_to_bytes(p, C) for p in cm)),
            "zs": hx(b"".join(fr_to_bytes(z) for z in zs)),
            "ys": hx(b"".join(fr_to_bytes(y) for y in ys)),
            "proofs": hx(b"".join(g1_to_bytes(p, C) for p in ps)),
        }

    def result(cm, zs, ys, ps):
        A, B = batch_combination(cm, zs, ys, ps, seed, C)
        ok = multi_pairing_is_one([(A, tg2), (g1_neg(B, C), g2)], C)
        return {"A": hx(g1_to_bytes(A, C)), "B": hx(g1_to_bytes(B, C)), "ok": ok}

    d = {"curve": C.name, "n": n, "tau": hex(tau), "seed": hx(seed),
         "g2": hx(g2_to_bytes(g2, C)), "tau_g2": hx(g2_to_bytes(tg2, C)),
         "randomizers_head": [hex(randomizer(seed, i)) for i in range(min(n, 8))]}
    d.update(enc(cm, zs, ys, ps))
    d["valid"] = result(cm, zs, ys, ps)
    assert d["valid"]["ok"]
    # negative 1: one y flipped
    ys_bad = list(ys)
    ys_bad[n // 2] = (ys_bad[n // 2] + 1) % C.r
    neg1 = enc(cm, zs, ys_bad, ps)
    neg1["what"] = "y[%d] += 1" % (n // 2)
    neg1.update(result(cm, zs, ys_bad, ps))
    assert not neg1["ok"]
    d["neg_flip_y"] = neg1
    if n >= 2:
        ps_sw = list(ps)
        ps_sw[0], ps_sw[1] = ps_sw[1], ps_sw[0]
        neg2 = enc(cm, zs, ys, ps_sw)
        neg2["what"] = "proofs 0 and 1 swapped"
        neg2.update(result(cm, zs, ys, ps_sw))
        assert not neg2["ok"]
        d["neg_swap_proofs"] = neg2
    return d


def genuine_kzg(C):
    """Proper KZG openings of degree-7 polynomials with an SRS of powers of tau."""
    rng = random.Random(99)
    tau = rng.randrange(2, C.r)
    g1, g2, tg2 = toy_srs(tau, C)
    out = {"tau": hex(tau), "g2": hx(g2_to_bytes(g2, C)), "tau_g2": hx(g2_to_bytes(tg2, C)),
           "seed": hx(hashlib.sha256(b"genuine").digest())}
    cm, zs, ys, ps = [], [], [], []
    for _ in range(4):
        coeffs = [rng.randrange(C.r) for _ in range(8)]
        z = rng.randrange(C.r)
        Cm, y, Pi = poly_commit_and_open(coeffs, z, tau, C)
        cm.append(Cm); zs.append(z); ys.append(y); ps.append(Pi)
    out.update({
        "n": 4,
        "commitments": hx(b"".join(g1_to_bytes(p, C) for p in cm)),
        "zs": hx(b"".join(fr_to_bytes(z) for z in zs)),
        "ys": hx(b"".join(fr_to_bytes(y) for y in ys)),
        "proofs": hx(b"".join(g1_to_bytes(p, C) for p in ps)),
        "ok": True,
    })
    return out


def main():
    files = {}
    files["constants.json"] = constants()
    for C, sizes in ((BLS12_381, (4, 16, 256)), (BN254, (4, 16, 64))):
        rng = random.Random(7)
        files["%s_pairing.json" % C.name] = pairing_kat(C, rng)
        files["%s_msm.json" % C.name] = {"curve": C.name, "cases": msm_cases(C, rng)}
        files["%s_genuine_kzg.json" % C.name] = genuine_kzg(C)
        for n in sizes:
            files["%s_batch_n%d.json" % (C.name, n)] = batch_fixture(C, n, 1000 + n)
            print("generated", C.name, n, flush=True)
    manifest = {}
    for name, obj in files.items():
        data = json.dumps(obj, indent=1, sort_keys=True).encode()
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(data)
        manifest[name] = hashlib.sha256(data).hexdigest()
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(files), "fixtures")


if __name__ == "__main__":
    main()
