"""The drop-in boundary of SURVEY.md 8b on the GPU: the SRS's G1 element, the multi-device
context (kzgmi_ctx_create over a device list), stream ordering against torch, slot-0 guards, argument
checks, and shard partials compared one by one with the oracle.

Bar: bit-exact against the C oracle (oracle/c) for every point; verdicts as the oracle's.
"""
import hashlib
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from oracle.pyspec import curves as pc  # noqa: E402
from oracle.pyspec import kzg as pk  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def h(x):
    return bytes.fromhex(x)


@pytest.fixture(scope="module")
def ctx():
    import kzgmi
    c = kzgmi.Context(0, 2)
    yield c
    c.close()


def _dev(b):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()


def _host(t):
    return t.cpu().numpy().tobytes()


def _gen_batch(ctx, curve, n, tau, seed):
    import torch
    g1b = 2 * pc.CURVES[curve].fp_bytes
    Cm = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.gen_tuples(curve, tau, seed, n, Cm, z, y, P)
    return Cm, z, y, P


def _scale_points(curve, pts: bytes, n: int, k: int) -> bytes:
    """[k] P_i for each of n encodings (oracle MSMs of one term)."""
    g1b = 2 * pc.CURVES[curve].fp_bytes
    kb = pk.fr_to_bytes(k)
    return b"".join(O.msm_g1(curve, pts[i * g1b:(i + 1) * g1b], kb, 1) for i in range(n))


@pytest.mark.parametrize("curve", ["bls12_381", "bn254"])
def test_srs_g1_element(ctx, curve, golden):
    """srs = {G1, [1]_2, [tau]_2}: with [1]_1 = 3 G the openings C' = 3 C, pi' = 3 pi verify
    only against the SRS that carries 3 G; A, B bit-exact vs the oracle with the same g1."""
    g = golden("%s_batch_n16.json" % curve)
    n = g["n"]
    g1_3 = O.g1_mul_gen(curve, pk.fr_to_bytes(3), 1)
    C3 = _scale_points(curve, h(g["commitments"]), n, 3)
    P3 = _scale_points(curve, h(g["proofs"]), n, 3)
    srs3 = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]), g1=g1_3)
    srs1 = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))
    seed = h(g["seed"])
    assert ctx.batch_verify(srs3, C3, h(g["zs"]), h(g["ys"]), P3, seed=seed) is True
    A, B = ctx.last_combination(curve)
    ok, Ao, Bo = O.batch_verify_g1(curve, C3, h(g["zs"]), h(g["ys"]), P3, n, g1_3, h(g["g2"]), h(g["tau_g2"]), seed)
    assert ok is True and A == Ao and B == Bo
    assert ctx.batch_verify(srs1, C3, h(g["zs"]), h(g["ys"]), P3, seed=seed) is False
    ok, Ao, Bo = O.batch_verify_g1(curve, C3, h(g["zs"]), h(g["ys"]), P3, n, None, h(g["g2"]), h(g["tau_g2"]), seed)
    A, B = ctx.last_combination(curve)
    assert ok is False and A == Ao and B == Bo
    # the standard generator passed explicitly == g1 omitted
    srs_g = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]), g1=O.g1_mul_gen(curve, pk.fr_to_bytes(1), 1))
    assert ctx.batch_verify(srs_g, h(g["commitments"]), h(g["zs"]), h(g["ys"]), h(g["proofs"]), seed=seed) is True
    assert ctx.last_combination(curve) == (h(g["valid"]["A"]), h(g["valid"]["B"]))


def test_srs_g1_rejected(ctx, golden):
    import kzgmi
    from pointcases import non_subgroup_points
    curve = "bls12_381"
    C = pc.CURVES[curve]
    g = golden("%s_batch_n4.json" % curve)
    g1 = bytearray(O.g1_mul_gen(curve, pk.fr_to_bytes(5), 1))
    g1[-1] ^= 1
    cases = [(bytes(g1), -3), (b"\x40" + bytes(95), -1),
             (pk.g1_to_bytes(non_subgroup_points(1, seed=4)[0], C), -7)]
    for enc, code in cases:
        with pytest.raises(kzgmi.KzgmiError) as e:
            ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]), g1=enc)
        assert e.value.code == code
    srs = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))  # context still usable
    assert ctx.batch_verify(srs, h(g["commitments"]), h(g["zs"]), h(g["ys"]), h(g["proofs"]), seed=h(g["seed"]))


@pytest.mark.parametrize("curve", ["bls12_381", "bn254"])
def test_shard_partials_vs_oracle(ctx, curve):
    """Three uneven shards (one of a single tuple): every shard's A_k, B_k equals the oracle's
    combination of the same global index range; their combination verifies, and the
    combined A, B equal the oracle's unsharded A, B."""
    import torch
    C = pc.CURVES[curve]
    n, tau = 2500, 4242
    seed = hashlib.sha256(b"shard").digest()
    Cm, z, y, P = _gen_batch(ctx, curve, n, tau, seed)
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    pb = ctx.partial_bytes(curve)
    g1b = 2 * C.fp_bytes
    hb = [_host(t) for t in (Cm, z, y, P)]
    bounds = [0, 1000, 1001, n]
    parts = torch.empty(3 * 2 * pb, dtype=torch.uint8, device="cuda")
    for k in range(3):
        lo, hi = bounds[k], bounds[k + 1]
        rec = parts[k * 2 * pb:(k + 1) * 2 * pb]
        ctx.batch_partial(srs, Cm[lo * g1b:hi * g1b], z[lo * 32:hi * 32], y[lo * 32:hi * 32], P[lo * g1b:hi * g1b],
                          hi - lo, lo, seed, rec)
        Ak, Bk = ctx.partial_encode(curve, rec, 2)
        Ao, Bo = O.batch_combination(curve, hb[0][lo * g1b:hi * g1b], hb[1][lo * 32:hi * 32], hb[2][lo * 32:hi * 32],
                                     hb[3][lo * g1b:hi * g1b], hi - lo, lo, g2, tg2, seed)
        assert (Ak, Bk) == (Ao, Bo), k
    assert ctx.batch_combine(srs, parts, 3) is True
    ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, seed, want_ab=True)
    assert ok is True and ctx.last_combination(curve) == (Ao, Bo)
    # MSM shards: each partial vs the oracle MSM of its range, combination vs the whole
    pts, sc = Cm[:2000 * g1b], z[:2000 * 32]
    mp = torch.empty(2 * pb, dtype=torch.uint8, device="cuda")
    ctx.msm_partial(curve, pts[:700 * g1b], sc[:700 * 32], 700, mp[:pb])
    ctx.msm_partial(curve, pts[700 * g1b:], sc[700 * 32:], 1300, mp[pb:])
    e0, e1 = ctx.partial_encode(curve, mp, 2)
    assert e0 == O.msm_g1(curve, hb[0][:700 * g1b], hb[1][:700 * 32], 700)
    assert e1 == O.msm_g1(curve, hb[0][700 * g1b:2000 * g1b], hb[1][700 * 32:2000 * 32], 1300)
    assert ctx.msm_combine(curve, mp, 2) == O.msm_g1(curve, hb[0][:2000 * g1b], hb[1][:2000 * 32], 2000)


def test_stream_order_and_buffer_reuse(ctx):
    """Inputs written by torch immediately before the call (no explicit synchronize) are read
    complete: a valid batch then the same buffers corrupted in place, alternately, through the
    one-shot sharded path (world-1 RCCL) and the single-device path."""
    import torch
    import torch.distributed as dist
    from kzgmi.distributed import sharded_batch_verify, sharded_msm
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n, tau = 3000, 31337
    seed = hashlib.sha256(b"order").digest()
    Cm, z, y, P = _gen_batch(ctx, curve, n, tau, seed)
    g2 = pk.g2_to_bytes(C.g2, C)
    srs = ctx.load_srs(curve, g2, O.g2_mul(curve, g2, tau))
    y_good = y.clone()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    created = not dist.is_initialized()
    if created:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        big = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
        for it in range(3):
            y.copy_(y_good)
            big.fill_(it)                 # keep torch's stream busy ahead of the corruption
            if it % 2:
                y[32 * 77 + 31] ^= 1
            want = it % 2 == 0
            assert sharded_batch_verify(ctx, srs, Cm, z, y, P, n, 0, seed) is want, it
            assert ctx.batch_verify(srs, Cm, z, y, P, seed=seed, n=n) is want, it
        want_msm = O.msm_g1(curve, _host(Cm[:500 * 96]), _host(z[:500 * 32]), 500)
        assert sharded_msm(ctx, curve, Cm[:500 * 96], z[:500 * 32], 500) == want_msm
    finally:
        if created:
            dist.destroy_process_group()


def test_slot0_busy_guard_and_args(ctx, golden):
    """A synchronous slot-0 call while an async job is pending on slot 0 is refused (and does
    not disturb that job's verdict); seed / challenge / powers-offset arguments are checked."""
    import kzgmi
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n, tau = 1000, 555
    seed = hashlib.sha256(b"busy").digest()
    Cm, z, y, P = _gen_batch(ctx, curve, n, tau, seed)
    g2 = pk.g2_to_bytes(C.g2, C)
    srs = ctx.load_srs(curve, g2, O.g2_mul(curve, g2, tau))
    ybad = y.clone()
    ybad[31] ^= 1
    ctx.batch_verify_async(srs, 0, Cm, z, ybad, P, n, seed=seed)
    for call in (lambda: ctx.msm_g1(curve, Cm, z, n=n),
                 lambda: ctx.load_srs(curve, g2, g2),
                 lambda: ctx.last_combination(curve),
                 lambda: ctx.pairing(curve, Cm[:96].cpu().numpy().tobytes(), g2)):
        with pytest.raises(kzgmi.KzgmiError) as e:
            call()
        assert e.value.code == -1
    assert ctx.wait(0) is False        # the pending job's own verdict
    with pytest.raises(ValueError):
        ctx.batch_verify_async(srs, 0, Cm, z, y, P, n, seed=b"short")
    with pytest.raises(ValueError):
        ctx.batch_verify_async(srs, 0, Cm, z, y, P, n, challenge=1 << 256)
    with pytest.raises(ValueError):
        ctx.batch_verify_async(srs, 0, Cm, z, y, P, n + 1, seed=seed)  # tensors hold n tuples
    out = Cm.new_empty(2 * ctx.partial_bytes(curve))
    with pytest.raises(kzgmi.KzgmiError) as e:
        ctx.batch_partial_async(srs, 0, Cm, z, y, P, n, (1 << 32) - 100, None, out, challenge=12345)
    assert e.value.code == -1
    assert ctx.batch_verify(srs, Cm, z, y, P, seed=seed, n=n) is True


@pytest.mark.parametrize("curve", ["bls12_381", "bn254"])
def test_multi_device_context(curve):
    """kzgmi_ctx_create over the device list [0, 0] (two shard contexts on the one GPU of
    the test box; on a node the list names distinct GPUs): host-buffer batch_verify and msm_g1
    are split over both, partials gathered with hipMemcpyPeer and combined on the primary --
    A, B and the MSM bit-exact vs the oracle, the negative batch rejected, Fiat-Shamir mode
    equal to the single-device result, device-resident shards through *_multi_device."""
    import kzgmi
    import torch
    C = pc.CURVES[curve]
    g1b = 2 * C.fp_bytes
    mc = kzgmi.Context(slots=1, devices=[0, 0])
    sc = kzgmi.Context(0, 1)
    try:
        assert mc.num_devices() == 2
        n, tau = 9001, 0xABCDEF
        seed = hashlib.sha256(b"multi").digest()
        Cm, z, y, P = _gen_batch(sc, curve, n, tau, seed)
        hb = [_host(t) for t in (Cm, z, y, P)]
        g2 = pk.g2_to_bytes(C.g2, C)
        tg2 = O.g2_mul(curve, g2, tau)
        srs = mc.load_srs(curve, g2, tg2)
        assert mc.batch_verify(srs, hb[0], hb[1], hb[2], hb[3], seed=seed) is True
        ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, seed, want_ab=True)
        assert ok is True and mc.last_combination(curve) == (Ao, Bo)
        ybad = bytearray(hb[2])
        ybad[32 * (n - 1) + 31] ^= 1
        assert mc.batch_verify(srs, hb[0], hb[1], bytes(ybad), hb[3], seed=seed) is False
        # Fiat-Shamir: the whole-batch transcript across shards == the single-device challenge
        ssrs = sc.load_srs(curve, g2, tg2)
        assert mc.batch_verify(srs, hb[0], hb[1], hb[2], hb[3], fiat_shamir=True) is True
        ab_multi = mc.last_combination(curve)
        assert sc.batch_verify(ssrs, Cm, z, y, P, n=n, fiat_shamir=True) is True
        assert ab_multi == sc.last_combination(curve)
        # MSM
        assert mc.msm_g1(curve, hb[0], hb[1]) == O.msm_g1(curve, hb[0], hb[1], n)
        # device-resident shards (uneven; global order = shard order)
        cut = 4000
        shards = [(Cm[:cut * g1b], z[:cut * 32], y[:cut * 32], P[:cut * g1b], cut),
                  (Cm[cut * g1b:], z[cut * 32:], y[cut * 32:], P[cut * g1b:], n - cut)]
        assert mc.batch_verify_multi(srs, shards, seed=seed) is True
        assert mc.last_combination(curve) == (Ao, Bo)
        assert mc.msm_g1_multi(curve, [(Cm[:cut * g1b], z[:cut * 32], cut), (Cm[cut * g1b:], z[cut * 32:], n - cut)]) \
            == O.msm_g1(curve, hb[0], hb[1], n)
        # an invalid scalar on the second device is an error, and the context recovers
        zbad = z.clone()
        zbad[32 * (n - 5):32 * (n - 4)] = torch.frombuffer(bytearray(C.r.to_bytes(32, "big")), dtype=torch.uint8).cuda()
        with pytest.raises(kzgmi.KzgmiError) as e:
            mc.batch_verify_multi(srs, [(Cm[:cut * g1b], zbad[:cut * 32], y[:cut * 32], P[:cut * g1b], cut),
                                        (Cm[cut * g1b:], zbad[cut * 32:], y[cut * 32:], P[cut * g1b:], n - cut)],
                                  seed=seed)
        assert e.value.code == -4
        assert mc.batch_verify_multi(srs, shards, seed=seed) is True
    finally:
        mc.close()
        sc.close()


def test_two_rank_gloo_pipeline_on_gpu():
    """Two processes share the GPU over gloo and drive the real HIP ShardedPipeline (RCCL
    refuses two ranks per device; the driver's N > 1 runs use RCCL): every rank's shard
    partial A_k, B_k and the combined A, B are checked against the oracle, and the pipeline's
    verdicts come back in submission order (tests/gpu_dist_worker.py)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = []
    for r in range(2):
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "gpu_dist_worker.py")],
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
        assert "RANK OK" in out, out[-3000:]


@pytest.mark.parametrize("curve,mode", [("bls12_381", {}), ("bls12_381", {"trusted_g1": True}),
                                        ("bls12_381", {"fiat_shamir": True}), ("bn254", {})])
def test_reserve_leaves_nothing_to_allocate(curve, mode):
    """kzgmi_ctx_reserve sizes every slot for the mode: pipelined batches of at most that size then
    make no workspace allocation (kzgmi_alloc_count unchanged), and verify as the oracle does."""
    import kzgmi
    n, slots = 5000, 3
    c = kzgmi.Context(0, slots)
    try:
        tau = 0x1234567890ABCDEF
        srs = c.load_srs(curve, kzgmi.G2_GENERATOR[curve], c.g2_mul(curve, kzgmi.G2_GENERATOR[curve], tau))
        Cm, z, y, P = _gen_batch(c, curve, n, tau, hashlib.sha256(b"reserve").digest())
        c.reserve(curve, n, **mode)
        a0 = kzgmi.alloc_count()
        seed = None if mode.get("fiat_shamir") else hashlib.sha256(b"r").digest()
        for k in range(2 * slots):                      # every slot used twice, two sizes
            s = k % slots
            if k >= slots:
                assert c.wait(s)
            c.batch_verify_async(srs, s, Cm, z, y, P, n if k % 2 == 0 else n - 17, seed=seed, **mode)
        for s in range(slots):
            assert c.wait(s)
        assert kzgmi.alloc_count() == a0, "a reserved context allocated inside the steady state"
        c.batch_verify_async(srs, 0, Cm, z, y, P, n, seed=seed, **mode)  # still accepts after the reuse
        assert c.wait(0)
        # a larger batch than reserved still works (the workspace grows)
        Cm2, z2, y2, P2 = _gen_batch(c, curve, 2 * n, tau, hashlib.sha256(b"reserve2").digest())
        assert c.batch_verify(srs, Cm2, z2, y2, P2, seed=seed, n=2 * n, **mode)
        assert kzgmi.alloc_count() > a0
    finally:
        c.close()


def test_reserve_argument_checks(ctx):
    import kzgmi
    assert kzgmi.lib().kzgmi_ctx_reserve(ctx.handle, 0, 1 << 27, 0) == -1   # above the 2^26 per-call limit
    assert kzgmi.lib().kzgmi_ctx_reserve(ctx.handle, 0, 16, 1 << 10) == -1  # unknown flag
    with pytest.raises(kzgmi.KzgmiError):
        ctx.reserve("bls12_381", 16, fiat_shamir=True, powers=True)  # exclusive modes
    assert kzgmi.lib().kzgmi_abi_version() == kzgmi.ABI_VERSION


@pytest.mark.parametrize("curve", ["bls12_381", "bn254"])
def test_failed_shard_partial_is_marked(curve):
    """a shard partial whose inputs fail validation is written MARKED, and
    every combine that reads it fails -- with the shard's own code (device-marked record) or
    KZGMI_ERR_SHARD (record the caller filled with 0xFF) -- so no rank of a multi-GPU batch can
    accept it.  Also the chained combine on the failing slot and the MSM partials."""
    import torch
    import kzgmi
    c = kzgmi.Context(0, 3)
    try:
        tau, n = 0x7777, 64
        srs = c.load_srs(curve, kzgmi.G2_GENERATOR[curve], c.g2_mul(curve, kzgmi.G2_GENERATOR[curve], tau))
        Cm, z, y, P = _gen_batch(c, curve, 2 * n, tau, hashlib.sha256(b"mark").digest())
        g1b = 2 * pc.CURVES[curve].fp_bytes
        seed = hashlib.sha256(b"mark-seed").digest()
        pb = c.partial_bytes(curve)
        good = torch.empty(2 * pb, dtype=torch.uint8, device="cuda")
        bad = torch.empty(2 * pb, dtype=torch.uint8, device="cuda")
        c.batch_partial(srs, Cm[: n * g1b], z[: 32 * n], y[: 32 * n], P[: n * g1b], n, 0, seed, good)
        Cbad = Cm[n * g1b:].clone()
        Cbad[5 * g1b + g1b - 1] ^= 1  # off the curve
        with pytest.raises(kzgmi.KzgmiError) as e:
            c.batch_partial(srs, Cbad, z[32 * n:], y[32 * n:], P[n * g1b:], n, n, seed, bad)
        assert e.value.code == -3
        both = torch.cat([good, bad])
        with pytest.raises(kzgmi.KzgmiError) as e:  # a remote rank's view: the shard's own code
            c.batch_combine(srs, both, 2)
        assert e.value.code == -3
        # chained on the failing slot (the eager schedule): its wait reports the shard's error
        c.batch_partial_async(srs, 1, Cbad, z[32 * n:], y[32 * n:], P[n * g1b:], n, n, seed, bad)
        c.batch_combine_async(srs, 1, torch.cat([good, bad]), 2)
        with pytest.raises(kzgmi.KzgmiError) as e:
            c.wait(1)
        assert e.value.code == -3
        # caller-marked record (rejected before anything ran): KZGMI_ERR_SHARD on every rank
        bad.fill_(0xFF)
        with pytest.raises(kzgmi.KzgmiError) as e:
            c.batch_combine(srs, torch.cat([good, bad]), 2)
        assert e.value.code == -8
        # the good shards alone still combine to the valid unsharded verdict
        ok_part = torch.empty(2 * pb, dtype=torch.uint8, device="cuda")
        c.batch_partial(srs, Cm[n * g1b:], z[32 * n:], y[32 * n:], P[n * g1b:], n, n, seed, ok_part)
        assert c.batch_combine(srs, torch.cat([good, ok_part]), 2) is True
        # MSM partials
        mg = torch.empty(pb, dtype=torch.uint8, device="cuda")
        mb = torch.empty(pb, dtype=torch.uint8, device="cuda")
        c.msm_partial(curve, Cm[: n * g1b], z[: 32 * n], n, mg)
        with pytest.raises(kzgmi.KzgmiError):
            c.msm_partial(curve, Cbad, z[32 * n:], n, mb)
        with pytest.raises(kzgmi.KzgmiError) as e:
            c.msm_combine(curve, torch.cat([mg, mb]), 2)
        assert e.value.code == -3
        assert c.msm_combine(curve, mg, 1) == c.msm_g1(curve, Cm[: n * g1b], z[: 32 * n], n=n)
    finally:
        c.close()


@pytest.mark.parametrize("curve,n_gold", [("bls12_381", 256), ("bn254", 64)])
def test_multi_device_async_pipeline(curve, n_gold, golden):
    """a device-list context pipelines WHOLE batches per device through the
    async entry points -- caller slot s runs on device s % D (kzgmi_slot_device) with its own
    lane pipeline there, no collective.  On the box's one GPU the list is [0, 0] (two device
    contexts).  Golden batches (valid / flipped y / swapped proofs) from host buffers on every
    slot, verdicts as the fixtures'; A, B of a routed slot's partial bit-exact vs the golden; a
    2^20 batch and its corrupted copy in flight on the two devices at once."""
    import kzgmi
    import torch
    g = golden("%s_batch_n%d.json" % (curve, n_gold))
    mc = kzgmi.Context(slots=4, devices=[0, 0])
    try:
        assert mc.num_devices() == 2 and mc.slots == 4
        assert [mc.slot_device(s) for s in range(4)] == [0, 0, 0, 0]
        srs = mc.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))
        seed = h(g["seed"])
        cases = ["valid", "neg_flip_y", "neg_swap_proofs", "valid", "neg_flip_y", "valid", "neg_swap_proofs", "valid"]
        pend = {}
        got = []
        for k, key in enumerate(cases):
            s = k % 4
            if s in pend:
                got.append((pend.pop(s), mc.wait(s)))
            src = g if key == "valid" else g[key]
            mc.batch_verify_host_async(srs, s, h(src["commitments"]), h(src["zs"]), h(src["ys"]), h(src["proofs"]),
                                       seed=seed)
            pend[s] = key
        for s in sorted(pend):
            got.append((pend[s], mc.wait(s)))
        assert sorted(got) == sorted((key, g[key]["ok"]) for key in cases)
        # A, B through a slot on the second device (caller slot 1): partial of the whole batch
        pb = mc.partial_bytes(curve)
        rec = torch.empty(2 * pb, dtype=torch.uint8, device="cuda")
        dev = [_dev(h(g[k])) for k in ("commitments", "zs", "ys", "proofs")]
        mc.batch_partial_async(srs, 1, *dev, n_gold, 0, seed, rec)
        assert mc.wait(1) is True
        A, B = mc.partial_encode(curve, rec, 2)
        assert (A.hex(), B.hex()) == (g["valid"]["A"], g["valid"]["B"])
        # full size: one valid 2^20 batch on device 0 (slot 2), its corrupted copy on device 1 (slot 3)
        sc = kzgmi.Context(0, 1)
        try:
            n, tau = 1 << 20, 0x1F2E3D4C
            Cm, z, y, P = _gen_batch(sc, curve, n, tau, hashlib.sha256(b"multi-async").digest())
            g2 = kzgmi.G2_GENERATOR[curve]
            srs2 = mc.load_srs(curve, g2, mc.g2_mul(curve, g2, tau))
            ybad = y.clone()
            ybad[32 * 777 + 31] ^= 1
            torch.cuda.synchronize()
            mc.batch_verify_async(srs2, 2, Cm, z, y, P, n, seed=seed)
            mc.batch_verify_async(srs2, 3, Cm, z, ybad, P, n, seed=seed)
            assert mc.wait(2) is True
            assert mc.wait(3) is False
        finally:
            sc.close()
        with pytest.raises(kzgmi.KzgmiError):
            mc.wait(5)
    finally:
        mc.close()
