"""Byte-level restatement of the Fiat-Shamir transcript (oracle/pyspec/kzg.py fs_challenge) for
large batches: compressed encodings from the C oracle, hashing with hashlib.  Test
infrastructure only."""
import hashlib

from oracle import oracle as O
from oracle.pyspec import curves as pc
from oracle.pyspec import kzg as pk


def fs_challenge_bytes(curve, commitments, zs, ys, proofs, n, compressed=False):
    C = pc.CURVES[curve]
    fb = C.fp_bytes
    cc = commitments if compressed else O.g1_compress(curve, commitments, n)
    pp = proofs if compressed else O.g1_compress(curve, proofs, n)
    leaves = [hashlib.sha256(pk.FS_LEAF_TAG + i.to_bytes(8, "big") + cc[i * fb:(i + 1) * fb] + pp[i * fb:(i + 1) * fb]
                             + zs[32 * i:32 * i + 32] + ys[32 * i:32 * i + 32]).digest() for i in range(n)]
    leaves += [bytes(32)] * (pk.fs_slots(n) - n)
    h = hashlib.sha256(pk.FS_ROOT_TAG + n.to_bytes(8, "big") + pk.merkle_root(leaves)).digest()
    r = int.from_bytes(h, "big") % C.r
    return r if r else 1
