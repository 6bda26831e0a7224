"""The literal drop-in path: batch_verify from HOST buffers (SURVEY.md 8b/8d "secondary:
includes the H2D copy"), through kzgmi_batch_verify_ex_async and the synchronous
kzgmi_batch_verify that wraps it.

Three kinds of host memory take two different copy paths in the library, and every one is
checked against the oracle / the golden fixtures:
  - pinned (kzgmi_host_alloc -> kzgmi.HostBuffer, or kzgmi_host_register'ed numpy arrays):
    DMA'd directly on the slot's stream, the call returns at once;
  - pageable (numpy arrays, bytes): staged through the slot's pinned ring by the copy pool
    before the call returns (the caller may overwrite its arrays right after the call).

Bar: verdicts and the combined points A, B bit-exact vs the golden fixtures (n = 256) and vs
the C oracle at n = 2^20; errors as the device path's.
"""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from oracle.pyspec import curves as pc  # noqa: E402
from oracle.pyspec import kzg as pk  # noqa: E402


def h(x):
    return bytes.fromhex(x)


@pytest.fixture(scope="module")
def ctx():
    import kzgmi
    c = kzgmi.Context(0, 4)
    yield c
    c.close()


def _host_kinds(raw):
    """The same bytes as: bytes, a pageable numpy array, a pinned HostBuffer view."""
    import kzgmi
    hb = kzgmi.HostBuffer(max(1, len(raw)))
    hb.array[:len(raw)] = np.frombuffer(raw, dtype=np.uint8)
    return {"bytes": raw, "numpy": np.frombuffer(raw, dtype=np.uint8).copy(), "pinned": hb.view(0, len(raw)),
            "_keep": hb}


@pytest.mark.parametrize("curve", ["bls12_381", "bn254"])
def test_host_async_golden(ctx, curve, golden):
    """Golden batches (n = 256 / 64) through the async host entry on every slot, with every kind
    of host memory: verdicts as the fixtures; A, B (slot 0) bit-exact."""
    n = 256 if curve == "bls12_381" else 64
    g = golden("%s_batch_n%d.json" % (curve, n))
    srs = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))
    for key in ["valid", "neg_flip_y", "neg_swap_proofs"]:
        src = g if key == "valid" else g[key]
        exp = g[key]
        arrs = {k: _host_kinds(h(src[k])) for k in ("commitments", "zs", "ys", "proofs")}
        for kind in ("bytes", "numpy", "pinned"):
            args = [arrs[k][kind] for k in ("commitments", "zs", "ys", "proofs")]
            # slot 0 first (its A, B are readable), then the other slots in flight together
            ctx.batch_verify_host_async(srs, 0, *args, seed=h(g["seed"]))
            assert ctx.wait(0) == exp["ok"], (key, kind)
            A, B = ctx.last_combination(curve)
            assert (A.hex(), B.hex()) == (exp["A"], exp["B"]), (key, kind)
            for s in range(1, 4):
                ctx.batch_verify_host_async(srs, s, *args, seed=h(g["seed"]))
            assert [ctx.wait(s) for s in range(1, 4)] == [exp["ok"]] * 3, (key, kind)
            # the synchronous wrapper (kzgmi_batch_verify_ex = async on slot 0 + wait)
            assert ctx.batch_verify(srs, *args, seed=h(g["seed"])) == exp["ok"], (key, kind)


def test_pageable_inputs_may_be_reused_after_the_call(ctx, golden):
    """Pageable arrays are staged before the call returns: overwriting them right away must
    not change the verdict of the batch already enqueued."""
    g = golden("bls12_381_batch_n256.json")
    srs = ctx.load_srs("bls12_381", h(g["g2"]), h(g["tau_g2"]))
    arrs = [np.frombuffer(h(g[k]), dtype=np.uint8).copy() for k in ("commitments", "zs", "ys", "proofs")]
    ctx.batch_verify_host_async(srs, 1, *arrs, seed=h(g["seed"]))
    arrs[2][:] = np.frombuffer(h(g["neg_flip_y"]["ys"]), dtype=np.uint8)  # now an invalid batch
    ctx.batch_verify_host_async(srs, 2, *arrs, seed=h(g["seed"]))
    assert ctx.wait(1) is True
    assert ctx.wait(2) is False


def test_registered_numpy_is_dmad(ctx, golden):
    """kzgmi_host_register'ed numpy arrays (pinned in place) verify like the others."""
    import kzgmi
    g = golden("bls12_381_batch_n16.json")
    srs = ctx.load_srs("bls12_381", h(g["g2"]), h(g["tau_g2"]))
    arrs = [np.frombuffer(h(g[k]), dtype=np.uint8).copy() for k in ("commitments", "zs", "ys", "proofs")]
    for a in arrs:
        kzgmi.register_host(a)
    try:
        with pytest.raises(kzgmi.KzgmiError):
            kzgmi.register_host(arrs[0])  # twice
        ctx.batch_verify_host_async(srs, 3, *arrs, seed=h(g["seed"]))
        assert ctx.wait(3) is True
    finally:
        for a in arrs:
            kzgmi.unregister_host(a)
    with pytest.raises(kzgmi.KzgmiError):
        kzgmi.unregister_host(arrs[0])


def test_host_async_errors(ctx, golden):
    import kzgmi
    C = pc.CURVES["bls12_381"]
    g = golden("bls12_381_batch_n4.json")
    srs = ctx.load_srs("bls12_381", h(g["g2"]), h(g["tau_g2"]))
    args = [h(g[k]) for k in ("commitments", "zs", "ys", "proofs")]
    ctx.batch_verify_host_async(srs, 1, *args, seed=h(g["seed"]))
    with pytest.raises(kzgmi.KzgmiError) as e:  # slot busy
        ctx.batch_verify_host_async(srs, 1, *args, seed=h(g["seed"]))
    assert e.value.code == -1
    assert ctx.wait(1) is True
    zs = bytearray(args[1])
    zs[0:32] = C.r.to_bytes(32, "big")
    ctx.batch_verify_host_async(srs, 1, args[0], bytes(zs), args[2], args[3], seed=h(g["seed"]))
    with pytest.raises(kzgmi.KzgmiError) as e:  # non-canonical scalar: reported by the wait
        ctx.wait(1)
    assert e.value.code == -4
    ctx.batch_verify_host_async(srs, 1, b"", b"", b"", b"", n=0, seed=h(g["seed"]))
    assert ctx.wait(1) is True
    mc = kzgmi.Context(slots=1, devices=[0, 0])
    try:
        msrs = mc.load_srs("bls12_381", h(g["g2"]), h(g["tau_g2"]))
        # ABI 5: a multi-device context runs a whole host-buffer batch on the slot's device
        mc.batch_verify_host_async(msrs, 0, *args, seed=h(g["seed"]))
        with pytest.raises(kzgmi.KzgmiError) as e:  # slot busy, on the routed device too
            mc.batch_verify_host_async(msrs, 0, *args, seed=h(g["seed"]))
        assert e.value.code == -1
        with pytest.raises(kzgmi.KzgmiError) as e:  # the synchronous split needs every first slot idle
            mc.batch_verify(msrs, *args, seed=h(g["seed"]))
        assert e.value.code == -1
        assert mc.wait(0) is True
        with pytest.raises(kzgmi.KzgmiError) as e:  # slot 1 does not exist (slots=1)
            mc.batch_verify_host_async(msrs, 1, *args, seed=h(g["seed"]))
        assert e.value.code == -1
        assert mc.batch_verify(msrs, *args, seed=h(g["seed"])) is True
        del msrs
    finally:
        mc.close()


@pytest.mark.slow
def test_host_async_full_size_vs_oracle(ctx):
    """configs[2] through the host path: one 2^20 BLS12-381 batch from pinned memory and the
    same batch from pageable memory, in flight together on two slots; the pinned one's A, B
    (slot 0) bit-exact vs the oracle, both verdicts True; a corrupted copy rejected."""
    import kzgmi
    import torch
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n, tau = 1 << 20, 0xC0FFEE + 11
    g1b = 2 * C.fp_bytes
    d = [torch.empty(n * w, dtype=torch.uint8, device="cuda") for w in (g1b, 32, 32, g1b)]
    ctx.gen_tuples(curve, tau, hashlib.sha256(b"host-cfg2").digest(), n, *d)
    host = [t.cpu().numpy() for t in d]
    pinned = kzgmi.HostBuffer(n * (2 * g1b + 64))
    views, off = [], 0
    for a in host:
        v = pinned.view(off, a.nbytes)
        v[:] = a
        views.append(v)
        off += a.nbytes
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    vseed = hashlib.sha256(b"host-cfg2-verify").digest()
    ctx.reserve(curve, n)
    ctx.batch_verify_host_async(srs, 0, *views, seed=vseed)
    ctx.batch_verify_host_async(srs, 1, *host, seed=vseed)
    assert ctx.wait(0) is True
    A, B = ctx.last_combination(curve)
    assert ctx.wait(1) is True
    ok, Ao, Bo = O.batch_verify(curve, *(a.tobytes() for a in host), n, g2, tg2, vseed, want_ab=True)
    assert ok is True and A == Ao and B == Bo
    host[2][32 * (n - 1) + 31] ^= 1
    assert ctx.batch_verify(srs, *host, seed=vseed) is False
    del srs
    pinned.free()


def _context_env(**env):
    import os
    import kzgmi
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return kzgmi.Context(0, 4)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.slow
@pytest.mark.parametrize("curve,trusted", [("bls12_381", False), ("bls12_381", True), ("bn254", False)])
def test_sync_host_chunked_matches_unsplit(ctx, curve, trusted):
    """The synchronous host-buffer call splits a large batch into point ranges whose work starts
    while the next range copies (csrc/api.hip batch_host_chunked): one bucket store for every
    range (the default without flags or with trusted_g1; BN254 and trusted points take the GLV
    form) and shard partials per range (KZGMI_HOST_CHUNK_MODE=1, the form for the other flags)
    both give the verdict and A, B of a
    context that never splits (KZGMI_HOST_CHUNKS=1) and of the oracle; a corrupted y in the last
    range and in a middle range (second store + merge, then more accumulation) rejects; a
    non-canonical z in an inner range reports the unsplit call's error.  With n = 2^19 + 5000 the
    ranges are [0, 65536), then three of ~154 K (api.hip enqueue_batch_chunked): index 66536 is
    in range 1, n / 2 in range 2."""
    import kzgmi
    import torch
    C = pc.CURVES[curve]
    n, tau = (1 << 19) + 5000, 0xC0FFEE + 12  # 4 ranges
    g1b = 2 * C.fp_bytes
    d = [torch.empty(n * w, dtype=torch.uint8, device="cuda") for w in (g1b, 32, 32, g1b)]
    ctx.gen_tuples(curve, tau, hashlib.sha256(b"host-chunked").digest(), n, *d)
    host = [t.cpu().numpy() for t in d]
    del d
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    seed = hashlib.sha256(b"host-chunked-verify").digest()
    c1 = _context_env(KZGMI_HOST_CHUNKS="1")
    c2 = _context_env(KZGMI_HOST_CHUNK_MODE="1")
    try:
        s1 = c1.load_srs(curve, g2, tg2)
        kw = {"trusted_g1": trusted}
        assert c1.batch_verify(s1, *host, seed=seed, **kw) is True
        want = c1.last_combination(curve)
        ok, Ao, Bo = O.batch_verify(curve, *(a.tobytes() for a in host), n, g2, tg2, seed, want_ab=True)
        assert ok is True and want == (Ao, Bo)
        bad_y = [a.copy() for a in host]
        bad_y[2][32 * (n - 1) + 31] ^= 1  # y of the last tuple
        bad_ymid = [a.copy() for a in host]
        bad_ymid[2][32 * (n // 2) + 31] ^= 1  # y of a tuple in range 2
        iz = (1 << 16) + 1000  # range 1
        bad_z = [a.copy() for a in host]
        bad_z[1][32 * iz:32 * (iz + 1)] = np.frombuffer(C.r.to_bytes(32, "big"), dtype=np.uint8)  # z = r
        with pytest.raises(kzgmi.KzgmiError) as e1:
            c1.batch_verify(s1, *bad_z, seed=seed, **kw)
        for c in (ctx, c2):
            srs = c.load_srs(curve, g2, tg2)
            assert c.batch_verify(srs, *host, seed=seed, **kw) is True
            assert c.last_combination(curve) == want
            assert c.batch_verify(srs, *bad_y, seed=seed, **kw) is False
            assert c.batch_verify(srs, *bad_ymid, seed=seed, **kw) is False
            with pytest.raises(kzgmi.KzgmiError) as e:
                c.batch_verify(srs, *bad_z, seed=seed, **kw)
            assert e.value.code == e1.value.code == -4
            assert c.batch_verify(srs, *host, seed=seed, **kw) is True  # the context recovers
            del srs
        del s1
    finally:
        c1.close()
        c2.close()


def test_ctx_destroy_releases_chunked_workspaces():
    """kzgmi_ctx_destroy releases every slot buffer (the second bucket store of
    chunked host batches -- acc29b, cntb, offb -- and the small-call tree were left allocated,
    ~60 MB per context at 2^17 tuples).  A one-slot context also takes the one-store chunked form
    (its ranges all run on slot 0).  Device free memory must come back after each
    create / chunked verify / small verify / destroy cycle."""
    import kzgmi
    import torch
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n, tau = 1 << 17, 0xC0FFEE + 21
    g1b = 2 * C.fp_bytes
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    seed = hashlib.sha256(b"destroy-cycle").digest()
    d = [torch.empty(n * w, dtype=torch.uint8, device="cuda") for w in (g1b, 32, 32, g1b)]
    c0 = kzgmi.Context(0, 1)
    try:
        c0.gen_tuples(curve, tau, hashlib.sha256(b"destroy-cycle-tuples").digest(), n, *d)
    finally:
        c0.close()
    host = [t.cpu().numpy() for t in d]
    small = [a[: 64 * (len(a) // n)] for a in host]
    del d
    torch.cuda.synchronize()

    def cycle():
        c = kzgmi.Context(0, 1)
        try:
            srs = c.load_srs(curve, g2, tg2)
            assert c.batch_verify(srs, *host, seed=seed) is True
            assert c.batch_verify(srs, *small, seed=seed) is True
            del srs
        finally:
            c.close()

    cycle()  # runtime pools, code objects
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(3):
        cycle()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 < (32 << 20), (free0 - free1) / 2**20
