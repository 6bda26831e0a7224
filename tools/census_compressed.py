"""Per-point operation census of the compressed-input front end:
k_decompress_points + k_subgroup_check (csrc/points.hpp) for BLS12-381 against the chain lengths
and the measured mad issue rate.

Counts come from the generated chain data (csrc/params_gen.hpp: the (p+1)/4 window, |x|) and the
formulas as written in points.hpp (dbl-2009-l, madd-2007-bl, add-2007-bl); radix-2^29 products
cost 301 (squaring) / 392 (product) v_mad_u64_u32 (field29.hpp, bench.py hw_floor).  The floor
is the mad stream alone at the measured 0.4596 wave-instructions per SIMD per ns
(profiles/r01/probes/mad_rate.txt) on 1024 SIMDs.

  python tools/census_compressed.py [bench_detail.json] > profiles/r05/census_compressed.txt
"""
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = (ROOT / "kzg-batch-verification-scheme_amd/csrc/params_gen.hpp").read_text()
bls = SRC.split("struct Bls12_381FpParams", 1)[1].split("\n};", 1)[0]
sqr_steps = [int(v) for v in re.search(r"SQRT_SQR\[\d+\] = \{([^}]*)\}", bls).group(1).split(",")]
idx = [int(v) for v in re.search(r"SQRT_IDX\[\d+\] = \{([^}]*)\}", bls).group(1).split(",")]
x_abs = int(re.search(r"X_ABS = (0x[0-9a-f]+)ull", SRC).group(1), 16)

SQR_MADS, MUL_MADS = 301, 392
MAD_RATE, SIMDS = 0.4596, 1024  # wave-instructions per SIMD per ns; SIMDs


def row(name, sq, mu, note=""):
    return (name, sq, mu, note)


# ---- decompression (radix 29 inside fp_pow_sqrt29; the rest in the 32-bit form)
dec = [
    row("table x^2, x^(2k+1) k<8", 1, 7),
    row("(p+1)/4 window: squarings", sum(sqr_steps), 0, "%d steps" % len(sqr_steps)),
    row("(p+1)/4 window: table products", 0, sum(1 for k in idx if k != 255)),
]
dec32 = 4  # x^3 + b (sqr, mul), the y^2 check, to/from Montgomery: 32-bit-limb products
# ---- membership [x^2]P = [|x|]([|x|]P) vs -phi(P)
nbits = x_abs.bit_length()
nadd = bin(x_abs).count("1") - 1
ndbl = 2 * (nbits - 1)
sgc = [
    row("doublings (dbl-2009-l: 5S + 2M)", 5 * ndbl, 2 * ndbl, "%d doublings" % ndbl),
    row("chain 1 additions (madd-2007-bl: 4S + 8M, 1 zero test)", 4 * nadd, 8 * nadd, "%d additions" % nadd),
    row("chain 2 additions (add-2007-bl: 5S + 11M)", 5 * nadd, 11 * nadd, "%d additions" % nadd),
]
sgc32 = 5  # beta x, Z^2, Z^3, two comparisons' products (32-bit form)


def total(rows):
    sq = sum(r[1] for r in rows)
    mu = sum(r[2] for r in rows)
    return sq, mu, sq * SQR_MADS + mu * MUL_MADS


lines = ["# Compressed-input front end, BLS12-381: per-point operation census (tools/census_compressed.py)", ""]
for title, rows, extra in (("k_decompress_points", dec, dec32), ("k_subgroup_check", sgc, sgc32)):
    lines.append("## %s" % title)
    for name, sq, mu, note in rows:
        lines.append("  %-58s %5d sqr %5d mul  %s" % (name, sq, mu, note))
    sq, mu, mads = total(rows)
    lines.append("  %-58s %5d sqr %5d mul  = %d radix-29 products, %.1f K mads (+%d 32-bit products)"
                 % ("total", sq, mu, sq + mu, mads / 1e3, extra))
    lines.append("")
sq, mu, mads = total(dec + sgc)
pts = 2 << 20  # configs[2]: 2^20 commitments + 2^20 proofs
wave_instr = pts / 64 * mads
floor_ms = wave_instr / (MAD_RATE * SIMDS) / 1e6
lines += [
    "## per batch (configs[2]: 2^21 compressed points)",
    "  radix-29 products per point: %d (%d sqr + %d mul), %.1f K v_mad_u64_u32" % (sq + mu, sq, mu, mads / 1e3),
    "  mad-stream floor at %.4f wave-instr/SIMD/ns x %d SIMDs: %.1f ms per batch" % (MAD_RATE, SIMDS, floor_ms),
]
if len(sys.argv) > 1:
    d = json.load(open(sys.argv[1]))
    leg = d["secondary"]["compressed_subgroup"] if "secondary" in d else d["compressed_subgroup"]
    conv = leg["phase_ms_single_batch"]["convert"]
    acc = leg["phase_ms_single_batch"]["accumulate"]
    rate = leg["batch_verifies_per_s"]
    lines += [
        "  measured convert phase (single batch): %.1f ms = %.2f of the mad floor (%s)" % (conv, floor_ms / conv,
                                                                                       sys.argv[1]),
        "  measured pipelined rate: %.1f batch-verifies/s (%.1f ms per batch)" % (rate, 1e3 / rate),
        "  ceiling at 100%% of the mad floor + the accumulation (%.1f ms): %.1f/s  -> 30/s is out of reach"
        % (acc, 1e3 / (floor_ms + acc)),
    ]
lines += [
    "",
    "## why the chains are not shorter",
    "  - membership: any test [a]P + [b]phi(P) = O that accepts G1 needs a + b*lambda = 0 mod r; then the norm",
    "    a^2 - ab + b^2 is a nonzero multiple of r, so max(|a|, |b|) >= sqrt(r/3) ~ 2^126.7 and Straus pays ~126 doublings:",
    "    Scott's [x^2] (126 doublings, |x| has %d set bits) is at that bound.  A single [|x|] cannot kill G1: x" % (nadd + 1),
    "    is not in Z[lambda] (lambda = -x^2; odd powers of x never reduce to even ones mod x^4 - x^2 + 1).",
    "  - random-combination batch membership is unsound here: the cofactor has the small factors 3 and 11,",
    "    so a random coefficient kills a non-member's order-3 component with probability 1/3.",
    "  - the (p+1)/4 window: %d squarings are the exponent's length; a better addition chain can only trim the" % (
        sum(sqr_steps)),
    "    %d table products (<= %.0f %% of the point's products, bounded by removing all of them)." % (
        sum(1 for k in idx if k != 255) + 7, 100.0 * (sum(1 for k in idx if k != 255) + 7) / (sq + mu)),
    "  - dbl-2009-l (7 products) is the cheapest a = 0 doubling; XYZZ costs 9, projective 8+.",
]
print("\n".join(lines))
