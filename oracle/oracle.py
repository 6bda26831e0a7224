"""ctypes binding of the C oracle (oracle/build/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker / CPU baseline.  Never by the product package.  Parity unpinned by the reference
(LICENSE-only snapshot); pinned against the Python spec's golden fixtures in tests/golden.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# KZGO_LIB: an alternative build of the same source (the ASan/UBSan one, `make -C oracle sanitize`)
LIB_PATH = os.environ.get("KZGO_LIB") or os.path.join(HERE, "build", "liboracle.so")
CURVE_IDS = {"bls12_381": 0, "bn254": 1}
FP_BYTES = {"bls12_381": 48, "bn254": 32}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c = ctypes
        L.kzgo_batch_verify.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p,
                                        c.c_size_t, c.c_char_p, c.c_char_p, c.c_char_p,
                                        c.POINTER(c.c_int), c.c_char_p, c.c_char_p]
        L.kzgo_batch_combination.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t,
                                             c.c_uint64, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p]
        L.kzgo_pairing_check.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.POINTER(c.c_int)]
        L.kzgo_msm_g1.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_size_t, c.c_char_p]
        L.kzgo_g1_mul_gen.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_char_p]
        L.kzgo_batch_verify_powers.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t,
                                               c.c_uint64, c.c_char_p, c.c_char_p, c.c_char_p, c.c_int,
                                               c.POINTER(c.c_int), c.c_char_p, c.c_char_p]
        L.kzgo_g1_decompress.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_char_p]
        L.kzgo_g1_compress.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_char_p]
        L.kzgo_g1_subgroup_check.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.POINTER(c.c_int)]
        L.kzgo_pairing.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p]
        L.kzgo_g2_mul.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p]
        L.kzgo_randomizer_bytes.argtypes = [c.c_char_p, c.c_uint64, c.c_char_p]
        L.kzgo_sha256.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t]
        L.kzgo_batch_verify_g1.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t,
                                           c.c_uint64, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_int,
                                           c.POINTER(c.c_int), c.c_char_p, c.c_char_p]
        L.kzgo_batch_verify_tuned.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, c.c_size_t,
                                              c.c_char_p, c.c_char_p, c.c_char_p, c.c_int, c.c_size_t, c.c_int,
                                              c.POINTER(c.c_int), c.c_char_p, c.c_char_p]
        L.kzgo_pairing_fast.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_char_p]
        L.kzgo_fr_dot.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_size_t, c.c_char_p]
        L.kzgo_set_threads.argtypes = [c.c_int]
        L.kzgo_get_threads.restype = c.c_int
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__("oracle error %d" % code)
        self.code = code


def _check(rc):
    if rc != 0:
        raise OracleError(rc)


def set_threads(n: int):
    lib().kzgo_set_threads(int(n))


def threads() -> int:
    return lib().kzgo_get_threads()


def batch_verify(curve, commitments: bytes, zs: bytes, ys: bytes, proofs: bytes, n: int,
                 g2: bytes, tau_g2: bytes, seed: bytes, want_ab=False):
    g1b = 2 * FP_BYTES[curve]
    ok = ctypes.c_int(-1)
    a = ctypes.create_string_buffer(g1b)
    b = ctypes.create_string_buffer(g1b)
    _check(lib().kzgo_batch_verify(CURVE_IDS[curve], commitments, zs, ys, proofs, n, g2, tau_g2,
                                   seed, ctypes.byref(ok), a, b))
    if want_ab:
        return bool(ok.value), a.raw, b.raw
    return bool(ok.value)


def batch_verify_tuned(curve, commitments: bytes, zs: bytes, ys: bytes, proofs: bytes, n: int,
                       g2: bytes, tau_g2: bytes, seed: bytes, wbits: int = 0, chunk: int = 0, pairing: bool = True):
    """The tuned CPU verifier (c/pippenger_tuned_tmpl.h: signed windows, XYZZ buckets, fused
    MSMs, OpenMP tasks) -- the CPU baseline bench.py quotes; same A, B and verdict as
    batch_verify.  wbits = 0 picks the window width from n.  Returns (ok or None, A, B)."""
    g1b = 2 * FP_BYTES[curve]
    ok = ctypes.c_int(-1)
    a = ctypes.create_string_buffer(g1b)
    b = ctypes.create_string_buffer(g1b)
    _check(lib().kzgo_batch_verify_tuned(CURVE_IDS[curve], commitments, zs, ys, proofs, n, g2, tau_g2, seed,
                                         int(wbits), int(chunk), 1 if pairing else 0, ctypes.byref(ok), a, b))
    return (bool(ok.value) if pairing else None), a.raw, b.raw


def batch_combination(curve, commitments, zs, ys, proofs, n, offset, g2, tau_g2, seed):
    """(A, B) encodings for tuples [offset, offset + n) of a global batch (shard partials)."""
    g1b = 2 * FP_BYTES[curve]
    a = ctypes.create_string_buffer(g1b)
    b = ctypes.create_string_buffer(g1b)
    _check(lib().kzgo_batch_combination(CURVE_IDS[curve], commitments, zs, ys, proofs, n, offset, g2, tau_g2,
                                        seed, a, b))
    return a.raw, b.raw


def batch_verify_g1(curve, commitments, zs, ys, proofs, n, g1, g2, tau_g2, seed, offset=0, pairing=True):
    """Batch check against an SRS whose G1 element is `g1` (None = the standard generator).
    Returns (ok or None, A, B); pairing=False gives the shard partials of [offset, offset + n)."""
    g1b = 2 * FP_BYTES[curve]
    ok = ctypes.c_int(-1)
    a = ctypes.create_string_buffer(g1b)
    b = ctypes.create_string_buffer(g1b)
    _check(lib().kzgo_batch_verify_g1(CURVE_IDS[curve], commitments, zs, ys, proofs, n, offset, g1, g2, tau_g2, seed,
                                      1 if pairing else 0, ctypes.byref(ok), a, b))
    return (bool(ok.value) if pairing else None), a.raw, b.raw


def fr_dot(curve, a: bytes, b: bytes, n: int) -> int:
    """sum_i a_i b_i mod r (32-B big-endian canonical Fr values): with points a_i G1 and
    scalars b_i, [fr_dot] G1 is the MSM (SURVEY.md 4.3 discrete-log identity)."""
    out = ctypes.create_string_buffer(32)
    _check(lib().kzgo_fr_dot(CURVE_IDS[curve], a, b, n, out))
    return int.from_bytes(out.raw, "big")


def pairing_check(curve, A: bytes, B: bytes, g2: bytes, tau_g2: bytes) -> bool:
    ok = ctypes.c_int(-1)
    _check(lib().kzgo_pairing_check(CURVE_IDS[curve], A, B, g2, tau_g2, ctypes.byref(ok)))
    return bool(ok.value)


def batch_verify_powers(curve, commitments, zs, ys, proofs, n, g2, tau_g2, r: int, offset=0, pairing=True):
    """Powers mode: r_i = r^(offset + i).  Returns (ok or None, A, B)."""
    g1b = 2 * FP_BYTES[curve]
    ok = ctypes.c_int(-1)
    a = ctypes.create_string_buffer(g1b)
    b = ctypes.create_string_buffer(g1b)
    _check(lib().kzgo_batch_verify_powers(CURVE_IDS[curve], commitments, zs, ys, proofs, n, offset, g2, tau_g2,
                                          int(r).to_bytes(32, "big"), 1 if pairing else 0, ctypes.byref(ok), a, b))
    return (bool(ok.value) if pairing else None), a.raw, b.raw


def g1_decompress(curve, data: bytes, n: int):
    """(error code of the first invalid encoding or 0, n uncompressed encodings)."""
    out = ctypes.create_string_buffer(n * 2 * FP_BYTES[curve])
    rc = lib().kzgo_g1_decompress(CURVE_IDS[curve], data, n, out)
    return rc, out.raw


def g1_compress(curve, points: bytes, n: int) -> bytes:
    out = ctypes.create_string_buffer(n * FP_BYTES[curve])
    _check(lib().kzgo_g1_compress(CURVE_IDS[curve], points, n, out))
    return out.raw


def g1_subgroup_check(curve, points: bytes, n: int) -> bool:
    """True iff every (uncompressed, valid) point satisfies [r]P == O."""
    ok = ctypes.c_int(-1)
    _check(lib().kzgo_g1_subgroup_check(CURVE_IDS[curve], points, n, ctypes.byref(ok)))
    return bool(ok.value)


def msm_g1(curve, points: bytes, scalars: bytes, n: int) -> bytes:
    out = ctypes.create_string_buffer(2 * FP_BYTES[curve])
    _check(lib().kzgo_msm_g1(CURVE_IDS[curve], points, scalars, n, out))
    return out.raw


def g1_mul_gen(curve, scalars: bytes, n: int) -> bytes:
    out = ctypes.create_string_buffer(max(1, n * 2 * FP_BYTES[curve]))
    _check(lib().kzgo_g1_mul_gen(CURVE_IDS[curve], scalars, n, out))
    return out.raw[: n * 2 * FP_BYTES[curve]]


def pairing(curve, g1: bytes, g2: bytes) -> bytes:
    out = ctypes.create_string_buffer(12 * FP_BYTES[curve])
    _check(lib().kzgo_pairing(CURVE_IDS[curve], g1, g2, out))
    return out.raw


def pairing_fast(curve, g1: bytes, g2: bytes) -> bytes:
    """The tuned verifier's pairing (same value as pairing())."""
    out = ctypes.create_string_buffer(12 * FP_BYTES[curve])
    _check(lib().kzgo_pairing_fast(CURVE_IDS[curve], g1, g2, out))
    return out.raw


def g2_mul(curve, q: bytes, k: int) -> bytes:
    out = ctypes.create_string_buffer(4 * FP_BYTES[curve])
    _check(lib().kzgo_g2_mul(CURVE_IDS[curve], q, int(k).to_bytes(32, "big"), out))
    return out.raw


def randomizer(seed: bytes, i: int) -> int:
    out = ctypes.create_string_buffer(32)
    lib().kzgo_randomizer_bytes(seed, i, out)
    return int.from_bytes(out.raw, "big")


def sha256(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().kzgo_sha256(out, msg, len(msg))
    return out.raw
