"""Python big-int specification of the KZG batch verifier (TEST INFRASTRUCTURE ONLY).

Never imported by the product path.  See oracle/README.md.
"""
from .curves import BLS12_381, BN254, CURVES  # noqa: F401
