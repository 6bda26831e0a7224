"""CPU-only checks of the drop-in boundary: libkzgmi.so loads, exports every symbol declared
in include/kzgmi.h, and fails loudly (KZGMI_ERR_DEVICE) without a GPU -- no CPU fallback."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "kzgmi.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(kzgmi_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_python_binding():
    import kzgmi
    assert header_symbols() == sorted(kzgmi.exported_symbols())


def test_library_exports_every_header_symbol():
    import kzgmi
    lib = kzgmi.lib()
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert b"gfx950" in lib.kzgmi_version()
    # the version string reports the header's ABI revision (it is built from KZGMI_ABI_VERSION)
    assert ("abi %d" % lib.kzgmi_abi_version()).encode() in lib.kzgmi_version()
    assert lib.kzgmi_abi_version() == kzgmi.ABI_VERSION


def test_library_contains_gfx950_code_object():
    import kzgmi
    with open(kzgmi.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob or b"gfx950" in blob


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import kzgmi
    with pytest.raises(kzgmi.KzgmiError) as e:
        kzgmi.Context(0)
    assert e.value.code == -5


def test_shard_range():
    from kzgmi.distributed import shard_range
    for n in [0, 1, 7, 1 << 20, (1 << 20) + 3]:
        for w in [1, 2, 3, 8]:
            parts = [shard_range(n, w, r) for r in range(w)]
            assert sum(c for _, c in parts) == n
            off = 0
            for o, c in parts:
                assert o == off
                off += c
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
            aligned = [shard_range(n, w, r, align=4096) for r in range(w)]
            assert sum(c for _, c in aligned) == n
            assert all(o % 4096 == 0 or c == 0 for o, c in aligned)
            assert [o for o, c in aligned if c] == sorted(o for o, c in aligned if c)
