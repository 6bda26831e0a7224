"""kzgmi -- MI355X-native KZG batch verifier (Python host side over the C-ABI).

`batch_verify(commitments, zs, ys, proofs, srs)` is the north-star entry point
(BASELINE.json:5).  The reference repository contains no code
(/root/reference/LICENSE:1-201), so its "plugin interface" is the signature named in
BASELINE.json; this module mirrors it and calls libkzgmi.so (hand-written gfx950 HIP
kernels) through ctypes.  There is no CPU fallback: without the built library or without a
HIP device every call raises.

Inputs may be `bytes`/`bytearray`/`memoryview`, numpy uint8 arrays, or torch uint8 tensors.
CUDA(HIP) tensors are passed by device pointer (no PCIe copy: the HBM-resident path);
host buffers go through the host-pointer entry points.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# KZGMI_LIB selects an alternative build (timing experiments); default: the in-tree library
LIB_PATH = os.environ.get("KZGMI_LIB") or os.path.join(_HERE, "libkzgmi.so")

ABI_VERSION = 5  # include/kzgmi.h KZGMI_ABI_VERSION
CURVES = {"bls12_381": 0, "bn254": 1}
FP_BYTES = {"bls12_381": 48, "bn254": 32}
PHASES = ["convert", "scalars", "sort", "accumulate", "reduce", "combine", "pairing", "h2d"]

ERR_NAMES = {-1: "ARG", -2: "ENCODING", -3: "NOT_ON_CURVE", -4: "SCALAR", -5: "DEVICE", -6: "OOM",
             -7: "NOT_IN_SUBGROUP", -8: "SHARD"}


class KzgmiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("kzgmi error %d (%s): %s" % (code, ERR_NAMES.get(code, "?"), msg))
        self.code = code


_lib = None


def lib():
    """Load libkzgmi.so (fails loudly if the HIP extension was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libkzgmi.so not built (run __graft_entry__.build()): %s" % LIB_PATH)
    # One HIP runtime per process: torch-ROCm ships its own libamdhip64 with the same
    # soname (libamdhip64.so.7).  Loading torch first makes libkzgmi bind to that copy, so
    # device pointers, streams and RCCL all live in one runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    c = ctypes
    vp, sz, u8p, ip = c.c_void_p, c.c_size_t, c.c_char_p, c.POINTER(c.c_int)
    sig = {
        "kzgmi_version": ([], c.c_char_p),
        "kzgmi_last_error": ([], c.c_char_p),
        "kzgmi_phase_names": ([], c.c_char_p),
        "kzgmi_ctx_create": ([c.POINTER(vp), c.POINTER(c.c_int), c.c_int, c.c_int], c.c_int),
        "kzgmi_ctx_create_device": ([c.POINTER(vp), c.c_int, c.c_int], c.c_int),
        "kzgmi_ctx_destroy": ([vp], None),
        "kzgmi_srs_load": ([vp, c.c_int, u8p, u8p, u8p, c.POINTER(vp)], c.c_int),
        "kzgmi_ctx_num_devices": ([vp], c.c_int),
        "kzgmi_slot_device": ([vp, c.c_int], c.c_int),
        "kzgmi_abi_version": ([], c.c_int),
        "kzgmi_ctx_reserve": ([vp, c.c_int, sz, c.c_uint32], c.c_int),
        "kzgmi_alloc_count": ([], c.c_uint64),
        "kzgmi_stream_wait": ([vp, c.c_int, vp], c.c_int),
        "kzgmi_slot_signal": ([vp, c.c_int, vp], c.c_int),
        "kzgmi_host_alloc": ([sz, c.POINTER(vp)], c.c_int),
        "kzgmi_host_free": ([vp], None),
        "kzgmi_host_register": ([vp, sz], c.c_int),
        "kzgmi_host_unregister": ([vp], c.c_int),
        "kzgmi_partial_encode_device": ([vp, c.c_int, vp, sz, u8p], c.c_int),
        "kzgmi_batch_verify_multi_device": ([vp, vp, c.POINTER(vp), c.POINTER(vp), c.POINTER(vp), c.POINTER(vp),
                                             c.POINTER(sz), u8p, c.c_uint32, ip], c.c_int),
        "kzgmi_msm_g1_multi_device": ([vp, c.c_int, c.POINTER(vp), c.POINTER(vp), c.POINTER(sz), u8p], c.c_int),
        "kzgmi_srs_free": ([vp], None),
        "kzgmi_batch_verify": ([vp, vp, vp, vp, vp, vp, sz, u8p, ip], c.c_int),
        "kzgmi_batch_verify_device": ([vp, vp, vp, vp, vp, vp, sz, u8p, ip], c.c_int),
        "kzgmi_batch_verify_device_async": ([vp, vp, c.c_int, vp, vp, vp, vp, sz, u8p], c.c_int),
        "kzgmi_batch_verify_ex": ([vp, vp, vp, vp, vp, vp, sz, u8p, c.c_uint32, ip], c.c_int),
        "kzgmi_batch_verify_ex_async": ([vp, vp, c.c_int, vp, vp, vp, vp, sz, u8p, c.c_uint32], c.c_int),
        "kzgmi_batch_verify_device_ex_async": ([vp, vp, c.c_int, vp, vp, vp, vp, sz, u8p, c.c_uint32], c.c_int),
        "kzgmi_g1_validate_device": ([vp, c.c_int, vp, sz, c.c_uint32], c.c_int),
        "kzgmi_g1_compress_device": ([vp, c.c_int, vp, sz, vp], c.c_int),
        "kzgmi_ck_load": ([vp, c.c_int, u8p, sz, c.POINTER(c.c_void_p)], c.c_int),
        "kzgmi_ck_free": ([vp], None),
        "kzgmi_commit": ([vp, vp, u8p, sz, u8p], c.c_int),
        "kzgmi_commit_device": ([vp, vp, vp, sz, u8p], c.c_int),
        "kzgmi_fs_challenge_device": ([vp, c.c_int, vp, vp, vp, vp, sz, c.c_uint32, u8p], c.c_int),
        "kzgmi_fs_chunk_digests_device": ([vp, c.c_int, vp, vp, vp, vp, sz, c.c_uint64, c.c_uint32, vp], c.c_int),
        "kzgmi_fs_challenge_from_digests_device": ([vp, c.c_int, vp, sz, c.c_uint64, u8p], c.c_int),
        "kzgmi_slot_wait": ([vp, c.c_int, ip], c.c_int),
        "kzgmi_last_combination": ([vp, u8p, u8p], c.c_int),
        "kzgmi_msm_g1": ([vp, c.c_int, vp, vp, sz, u8p], c.c_int),
        "kzgmi_msm_g1_device": ([vp, c.c_int, vp, vp, sz, u8p], c.c_int),
        "kzgmi_msm_g1_device_async": ([vp, c.c_int, c.c_int, vp, vp, sz], c.c_int),
        "kzgmi_msm_wait": ([vp, c.c_int, u8p], c.c_int),
        "kzgmi_set_glv": ([vp, c.c_int, c.c_int], c.c_int),
        "kzgmi_commit_device_async": ([vp, vp, c.c_int, vp, sz], c.c_int),
        "kzgmi_set_trusted_g1": ([vp, c.c_int], c.c_int),
        "kzgmi_set_split_acc": ([vp, c.c_int], c.c_int),
        "kzgmi_msm_partial_device_async": ([vp, c.c_int, c.c_int, vp, vp, sz, vp], c.c_int),
        "kzgmi_msm_combine_device_async": ([vp, c.c_int, c.c_int, vp, c.c_int], c.c_int),
        "kzgmi_partial_bytes": ([c.c_int], sz),
        "kzgmi_batch_partial_device": ([vp, vp, vp, vp, vp, vp, sz, c.c_uint64, u8p, vp], c.c_int),
        "kzgmi_batch_combine_device": ([vp, vp, vp, c.c_int, ip], c.c_int),
        "kzgmi_batch_partial_device_async": ([vp, vp, c.c_int, vp, vp, vp, vp, sz, c.c_uint64, u8p, c.c_uint32, vp],
                                             c.c_int),
        "kzgmi_batch_combine_device_async": ([vp, vp, c.c_int, vp, c.c_int], c.c_int),
        "kzgmi_msm_partial_device": ([vp, c.c_int, vp, vp, sz, vp], c.c_int),
        "kzgmi_msm_combine_device": ([vp, c.c_int, vp, c.c_int, u8p], c.c_int),
        "kzgmi_pairing": ([vp, c.c_int, u8p, u8p, u8p], c.c_int),
        "kzgmi_gen_g1": ([vp, c.c_int, vp, sz, vp], c.c_int),
        "kzgmi_gen_tuples": ([vp, c.c_int, u8p, u8p, sz, vp, vp, vp, vp], c.c_int),
        "kzgmi_g2_mul": ([vp, c.c_int, u8p, u8p, u8p], c.c_int),
        "kzgmi_probe_fpmul": ([vp, c.c_int, c.POINTER(c.c_double)], c.c_int),
        "kzgmi_set_profiling": ([vp, c.c_int], c.c_int),
        "kzgmi_get_phase_ms": ([vp, c.POINTER(c.c_double), c.c_int], c.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    if L.kzgmi_abi_version() != ABI_VERSION:  # include/kzgmi.h KZGMI_ABI_VERSION
        raise ImportError("libkzgmi.so ABI %d, this binding expects %d (rebuild: __graft_entry__.build())"
                          % (L.kzgmi_abi_version(), ABI_VERSION))
    _lib = L
    return L


def exported_symbols():
    return [
        "kzgmi_version", "kzgmi_last_error", "kzgmi_phase_names", "kzgmi_ctx_create", "kzgmi_ctx_create_device",
        "kzgmi_ctx_destroy", "kzgmi_srs_load", "kzgmi_srs_free", "kzgmi_batch_verify",
        "kzgmi_batch_verify_device", "kzgmi_batch_verify_device_async", "kzgmi_slot_wait",
        "kzgmi_batch_verify_ex", "kzgmi_batch_verify_device_ex_async", "kzgmi_g1_validate_device",
        "kzgmi_g1_compress_device", "kzgmi_ck_load", "kzgmi_ck_free", "kzgmi_commit", "kzgmi_commit_device",
        "kzgmi_fs_challenge_device", "kzgmi_fs_chunk_digests_device",
        "kzgmi_fs_challenge_from_digests_device",
        "kzgmi_last_combination", "kzgmi_msm_g1", "kzgmi_msm_g1_device", "kzgmi_msm_g1_device_async",
        "kzgmi_msm_wait", "kzgmi_set_glv", "kzgmi_commit_device_async", "kzgmi_set_trusted_g1", "kzgmi_set_split_acc", "kzgmi_msm_partial_device_async", "kzgmi_msm_combine_device_async", "kzgmi_partial_bytes",
        "kzgmi_batch_partial_device", "kzgmi_batch_combine_device", "kzgmi_batch_partial_device_async",
        "kzgmi_batch_combine_device_async", "kzgmi_msm_partial_device",
        "kzgmi_msm_combine_device", "kzgmi_pairing", "kzgmi_gen_g1", "kzgmi_gen_tuples",
        "kzgmi_g2_mul", "kzgmi_probe_fpmul", "kzgmi_set_profiling", "kzgmi_get_phase_ms",
        "kzgmi_ctx_num_devices", "kzgmi_slot_device", "kzgmi_stream_wait", "kzgmi_slot_signal", "kzgmi_partial_encode_device",
        "kzgmi_batch_verify_multi_device", "kzgmi_msm_g1_multi_device",
        "kzgmi_abi_version", "kzgmi_ctx_reserve", "kzgmi_alloc_count", "kzgmi_batch_verify_ex_async",
        "kzgmi_host_alloc", "kzgmi_host_free", "kzgmi_host_register", "kzgmi_host_unregister",
    ]


FLAG_COMPRESSED = 1
FLAG_SUBGROUP_CHECK = 2
FLAG_POWERS = 4
FLAG_FIAT_SHAMIR = 8
FLAG_TRUSTED_G1 = 16
ERR_NOT_IN_SUBGROUP = -7
FS_CHUNK = 4096


def _flags(compressed: bool = False, subgroup_check: bool = False, fiat_shamir: bool = False,
           challenge=None, trusted_g1: bool = False) -> int:
    return ((FLAG_COMPRESSED if compressed else 0) | (FLAG_SUBGROUP_CHECK if subgroup_check else 0)
            | (FLAG_FIAT_SHAMIR if fiat_shamir else 0) | (FLAG_POWERS if challenge is not None else 0)
            | (FLAG_TRUSTED_G1 if trusted_g1 else 0))


def _challenge_seed(seed, challenge):
    """The 32-byte seed argument of the C-ABI (the library reads exactly 32 bytes from it).
    KZGMI_FLAG_POWERS passes r (int < 2^256 or 32 big-endian bytes) in its place."""
    if challenge is None:
        if seed is None:
            return None
        sd = bytes(seed)
        if len(sd) != 32:
            raise ValueError("seed must be 32 bytes, got %d" % len(sd))
        return sd
    if seed is not None:
        raise ValueError("pass either seed or challenge")
    if isinstance(challenge, int):
        if not 0 <= challenge < (1 << 256):
            raise ValueError("challenge must be in [0, 2^256)")
        return challenge.to_bytes(32, "big")
    sd = bytes(challenge)
    if len(sd) != 32:
        raise ValueError("challenge must be 32 bytes, got %d" % len(sd))
    return sd


def _check(rc: int):
    if rc != 0:
        msg = lib().kzgmi_last_error()
        raise KzgmiError(rc, msg.decode() if msg else "")


def _is_device_tensor(x) -> bool:
    return hasattr(x, "is_cuda") and x.is_cuda


def _host_bytes(x) -> bytes:
    if x is None:
        return b""
    if isinstance(x, (bytes, bytearray, memoryview)):
        return bytes(x)
    if hasattr(x, "cpu"):  # torch tensor
        return x.detach().cpu().contiguous().numpy().tobytes()
    if hasattr(x, "tobytes"):  # numpy
        return x.tobytes()
    raise TypeError("unsupported buffer type %r" % type(x))


def _host_ptr(x):
    """(address, nbytes, keepalive) of a host buffer, without copying it: bytes, bytearray,
    memoryview, numpy arrays (C-contiguous) and CPU torch tensors.  The keepalive object must
    outlive every use of the address."""
    if x is None:
        return 0, 0, None
    if isinstance(x, bytes):
        cp = ctypes.c_char_p(x)  # points into the bytes object itself
        return ctypes.cast(cp, ctypes.c_void_p).value or 0, len(x), (x, cp)
    if isinstance(x, HostBuffer):
        return x.ptr, x.nbytes, x
    import numpy as np
    if hasattr(x, "data_ptr") and hasattr(x, "is_cuda"):  # torch CPU tensor
        t = x.detach()
        if not t.is_contiguous():
            t = t.contiguous()
        return t.data_ptr(), t.numel() * t.element_size(), t
    if isinstance(x, (bytearray, memoryview)):
        x = np.frombuffer(x, dtype=np.uint8)
    if not isinstance(x, np.ndarray):
        try:  # any other buffer-protocol object (array.array, mmap, ...)
            x = np.frombuffer(memoryview(x).cast("B"), dtype=np.uint8)
        except TypeError:
            raise TypeError("unsupported buffer type %r" % type(x)) from None
    if not x.flags["C_CONTIGUOUS"]:
        x = np.ascontiguousarray(x)
    return x.ctypes.data, x.nbytes, x


class HostBuffer:
    """Page-locked host memory from kzgmi_host_alloc: host-buffer batch_verify calls whose arrays
    live here are DMA'd to HBM at PCIe rate, asynchronously (no staging copy).  `array` is a
    writable numpy uint8 view; free() (or garbage collection) releases it -- only when no job
    reading it is in flight."""

    def __init__(self, nbytes: int):
        import numpy as np
        p = ctypes.c_void_p()
        _check(lib().kzgmi_host_alloc(int(nbytes), ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, int(nbytes)
        raw = (ctypes.c_uint8 * self.nbytes).from_address(self.ptr)
        raw._kzgmi_owner = self  # every numpy view's base chain ends here: the block outlives its views
        self.array = np.ctypeslib.as_array(raw)

    def view(self, offset: int, nbytes: int):
        """numpy view of [offset, offset + nbytes) (also accepted by the host entry points)."""
        return self.array[offset:offset + nbytes]

    def free(self):
        """Release the block now (the caller guarantees no view is used afterwards and no job
        reading it is in flight); otherwise it is released when the last view goes away."""
        if getattr(self, "ptr", None):
            self.array = None
            lib().kzgmi_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def register_host(arr) -> None:
    """Pin an existing C-contiguous numpy array in place (kzgmi_host_register) so host-buffer
    calls DMA from it directly; unregister_host(arr) before freeing it."""
    _check(lib().kzgmi_host_register(arr.ctypes.data, arr.nbytes))


def unregister_host(arr) -> None:
    _check(lib().kzgmi_host_unregister(arr.ctypes.data))


def _dptr(x, nbytes: Optional[int] = None) -> int:
    """Device pointer of a contiguous tensor holding at least `nbytes` bytes."""
    if not x.is_contiguous():
        raise ValueError("device tensors must be contiguous")
    if nbytes is not None and x.numel() * x.element_size() < nbytes:
        raise ValueError("device tensor holds %d bytes, the call reads %d" % (x.numel() * x.element_size(), nbytes))
    return x.data_ptr()


def _current_stream(device: int):
    import torch
    return torch.cuda.current_stream(device).cuda_stream


@dataclass
class Srs:
    """{G1, [1]_2, [tau]_2} with device-side Miller-loop line tables."""
    ctx: "Context"
    curve: str
    handle: ctypes.c_void_p

    def __del__(self):
        try:
            if self.handle:
                lib().kzgmi_srs_free(self.handle)
                self.handle = None
        except Exception:
            pass


class CommitKey:
    """Prover commit key: [tau^i]_1 powers + fixed-base tables on the device."""
    ctx: "Context"
    curve: str
    n: int
    handle: ctypes.c_void_p

    def __del__(self):
        try:
            if self.handle:
                lib().kzgmi_ck_free(self.handle)
                self.handle = None
        except Exception:
            pass


class Context:
    """One GPU (device_id) with `slots` independent workspaces/streams; or, with
    devices=[d0, d1, ...], one context over several GPUs (kzgmi_ctx_create's device list: the
    synchronous host-buffer batch_verify / msm_g1 are sharded over them, d0 being the primary
    device; the async entry points run whole batches per device -- slot s on device
    slot_device(s) = devices[s % len(devices)], device tensors passed to it must live there).

    Device-tensor arguments are read on the library's own streams: every call first orders
    the slot's stream after torch's current stream (kzgmi_stream_wait), so tensors written by
    torch just before the call are seen complete."""

    def __init__(self, device: int = 0, slots: int = 1, devices=None):
        h = ctypes.c_void_p()
        devs = [int(d) for d in devices] if devices is not None else [int(device)]
        arr = (ctypes.c_int * len(devs))(*devs)
        _check(lib().kzgmi_ctx_create(ctypes.byref(h), arr, len(devs), int(slots)))
        device = devs[0]
        self.handle = h
        self.device = device
        self.slots = slots
        self.ndev = len(devs)

    def num_devices(self) -> int:
        return int(lib().kzgmi_ctx_num_devices(self.handle))

    def slot_device(self, slot: int) -> int:
        """The device id slot `slot` runs on (kzgmi_slot_device)."""
        d = int(lib().kzgmi_slot_device(self.handle, int(slot)))
        if d < 0:
            _check(d)
        return d

    def reserve(self, curve: str, n: int, compressed: bool = False, subgroup_check: bool = False,
                fiat_shamir: bool = False, powers: bool = False, trusted_g1: bool = False):
        """kzgmi_ctx_reserve: size every slot's workspace for batches of up to n tuples in this
        mode (and create the profiling events) -- later calls of that size allocate nothing."""
        fl = _flags(compressed, subgroup_check, fiat_shamir, 0 if powers else None, trusted_g1)
        _check(lib().kzgmi_ctx_reserve(self.handle, CURVES[curve], int(n), fl))

    def _order(self, slot: int = 0):
        """Order `slot`'s next job after torch's current stream on the slot's device (device
        inputs written by torch)."""
        dev = self.device if self.ndev == 1 else self.slot_device(slot)
        _check(lib().kzgmi_stream_wait(self.handle, int(slot), _current_stream(dev)))

    def signal(self, slot: int, stream=None):
        """kzgmi_slot_signal: order later work on `stream` (a torch.cuda.Stream; default torch's
        current stream) after everything enqueued so far on `slot` -- no host sync."""
        dev = self.device if self.ndev == 1 else self.slot_device(slot)
        st = stream.cuda_stream if stream is not None else _current_stream(dev)
        _check(lib().kzgmi_slot_signal(self.handle, int(slot), st))

    def close(self):
        if getattr(self, "handle", None):
            lib().kzgmi_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ SRS
    def load_srs(self, curve: str, g2: bytes, tau_g2: bytes, g1: Optional[bytes] = None) -> Srs:
        """srs = {G1, [1]_2, [tau]_2}; g1 None = the standard generator."""
        h = ctypes.c_void_p()
        _check(lib().kzgmi_srs_load(self.handle, CURVES[curve], None if g1 is None else bytes(g1), bytes(g2),
                                    bytes(tau_g2), ctypes.byref(h)))
        return Srs(self, curve, h)

    # ------------------------------------------------------------------ batch verify
    def batch_verify(self, srs: Srs, commitments, zs, ys, proofs, seed: Optional[bytes] = None,
                     n: Optional[int] = None, compressed: bool = False, subgroup_check: bool = False,
                     fiat_shamir: bool = False, challenge=None, trusted_g1: bool = False) -> bool:
        """BASELINE.json:5 batch_verify.  compressed: C/pi are compressed G1 encodings;
        subgroup_check: reject points outside G1 (KZGMI_ERR_NOT_IN_SUBGROUP); fiat_shamir:
        randomisers seeded with a challenge hashed from the inputs on the GPU; challenge:
        r_i = r^i for a caller-supplied r (e.g. the EIP-4844 transcript's); trusted_g1: the
        points are known G1 members (enables GLV on BLS12-381)."""
        flags = _flags(compressed, subgroup_check, fiat_shamir, challenge, trusted_g1)
        g1b = (1 if compressed else 2) * FP_BYTES[srs.curve]
        ok = ctypes.c_int(-1)
        sd = _challenge_seed(seed, challenge)
        if seed is not None and len(sd) != 32:
            raise ValueError("seed must be 32 bytes")
        if _is_device_tensor(commitments):
            if n is None:
                n = commitments.numel() // g1b
            ptrs = (_dptr(commitments, n * g1b), _dptr(zs, 32 * n), _dptr(ys, 32 * n), _dptr(proofs, n * g1b))
            self._order(0)
            if flags:
                _check(lib().kzgmi_batch_verify_device_ex_async(self.handle, srs.handle, 0, *ptrs, n, sd, flags))
                return self.wait(0)
            _check(lib().kzgmi_batch_verify_device(self.handle, srs.handle, *ptrs, n, sd, ctypes.byref(ok)))
        else:
            ptrs, keep = self._host_inputs(commitments, zs, ys, proofs, n, g1b)
            n = ptrs[-1]
            _check(lib().kzgmi_batch_verify_ex(self.handle, srs.handle, *ptrs[:4], n, sd, flags, ctypes.byref(ok)))
            del keep
        return bool(ok.value)

    @staticmethod
    def _host_inputs(commitments, zs, ys, proofs, n, g1b):
        """Addresses of the four host arrays (no copies) in C-ABI order (C, z, y, pi) + n."""
        (pc, lc, kc), (pz, lz, kz), (py, ly, ky), (pp, lp, kp) = (
            _host_ptr(v) for v in (commitments, zs, ys, proofs))
        if n is None:
            n = lc // g1b
        if lc < n * g1b or lp < n * g1b or lz < 32 * n or ly < 32 * n:
            raise ValueError("input buffers shorter than n tuples")
        return (pc, pz, py, pp, n), (kc, kz, ky, kp)

    def batch_verify_host_async(self, srs: Srs, slot: int, commitments, zs, ys, proofs, n: Optional[int] = None,
                                seed: Optional[bytes] = None, compressed: bool = False,
                                subgroup_check: bool = False, fiat_shamir: bool = False, challenge=None,
                                trusted_g1: bool = False):
        """kzgmi_batch_verify_ex_async: host arrays -> HBM on `slot`'s stream ahead of the batch's
        kernels; wait(slot) returns the verdict.  Arrays in a HostBuffer (or register_host'ed) are
        DMA'd asynchronously and must stay untouched until the wait; others are staged through
        the slot's pinned ring before this returns."""
        g1b = (1 if compressed else 2) * FP_BYTES[srs.curve]
        ptrs, keep = self._host_inputs(commitments, zs, ys, proofs, n, g1b)
        _check(lib().kzgmi_batch_verify_ex_async(self.handle, srs.handle, int(slot), *ptrs,
                                                 _challenge_seed(seed, challenge),
                                                 _flags(compressed, subgroup_check, fiat_shamir, challenge,
                                                        trusted_g1)))
        # the DMA may read the arrays until wait(slot); a failed call (e.g. slot busy) keeps the
        # pending job's keepalive
        self._host_keep = getattr(self, "_host_keep", {})
        self._host_keep[slot] = keep

    def batch_verify_async(self, srs: Srs, slot: int, commitments, zs, ys, proofs, n: int,
                           seed: Optional[bytes] = None, compressed: bool = False, subgroup_check: bool = False,
                           fiat_shamir: bool = False, challenge=None, trusted_g1: bool = False):
        g1b = (1 if compressed else 2) * FP_BYTES[srs.curve]
        ptrs = (_dptr(commitments, n * g1b), _dptr(zs, 32 * n), _dptr(ys, 32 * n), _dptr(proofs, n * g1b))
        sd = _challenge_seed(seed, challenge)
        self._order(slot)
        _check(lib().kzgmi_batch_verify_device_ex_async(self.handle, srs.handle, int(slot), *ptrs, n, sd,
                                                        _flags(compressed, subgroup_check, fiat_shamir, challenge,
                                                               trusted_g1)))

    def batch_verify_multi(self, srs: Srs, shards, seed: Optional[bytes] = None, compressed: bool = False,
                           subgroup_check: bool = False, fiat_shamir: bool = False, challenge=None,
                           trusted_g1: bool = False) -> bool:
        """Multi-device context: shards[d] = (commitments, zs, ys, proofs[, n]) device tensors on
        device d of the context's list (global tuple order = shard order)."""
        g1b = (1 if compressed else 2) * FP_BYTES[srs.curve]
        D = len(shards)
        if D != self.num_devices():
            raise ValueError("need one shard per device (%d), got %d" % (self.num_devices(), D))
        cols = [[], [], [], []]
        ns = []
        for sh in shards:
            C, z, y, P = sh[:4]
            n = sh[4] if len(sh) > 4 else C.numel() // g1b
            ns.append(n)
            for i, (t, nb) in enumerate(((C, n * g1b), (z, 32 * n), (y, 32 * n), (P, n * g1b))):
                cols[i].append(_dptr(t, nb) if n else None)
        import torch
        for sh in shards:  # inputs written by torch on each device's current stream
            torch.cuda.current_stream(sh[0].device).synchronize()
        arr = [(ctypes.c_void_p * D)(*c) for c in cols]
        nn = (ctypes.c_size_t * D)(*ns)
        ok = ctypes.c_int(-1)
        _check(lib().kzgmi_batch_verify_multi_device(self.handle, srs.handle, *arr, nn, _challenge_seed(seed, challenge),
                                                     _flags(compressed, subgroup_check, fiat_shamir, challenge,
                                                            trusted_g1), ctypes.byref(ok)))
        return bool(ok.value)

    def msm_g1_multi(self, curve: str, shards) -> bytes:
        """Multi-device context: shards[d] = (points, scalars[, n]) device tensors on device d."""
        g1b = 2 * FP_BYTES[curve]
        D = len(shards)
        if D != self.num_devices():
            raise ValueError("need one shard per device (%d), got %d" % (self.num_devices(), D))
        pp, ss, ns = [], [], []
        import torch
        for sh in shards:
            n = sh[2] if len(sh) > 2 else sh[0].numel() // g1b
            ns.append(n)
            pp.append(_dptr(sh[0], n * g1b) if n else None)
            ss.append(_dptr(sh[1], 32 * n) if n else None)
            torch.cuda.current_stream(sh[0].device).synchronize()
        out = ctypes.create_string_buffer(g1b)
        _check(lib().kzgmi_msm_g1_multi_device(self.handle, CURVES[curve], (ctypes.c_void_p * D)(*pp),
                                               (ctypes.c_void_p * D)(*ss), (ctypes.c_size_t * D)(*ns), out))
        return out.raw

    # ------------------------------------------------------------------ prover commit
    def load_commit_key(self, curve: str, g1_powers: bytes, n: Optional[int] = None) -> CommitKey:
        """g1_powers: n uncompressed G1 encodings [tau^i]_1 (host bytes)."""
        pb = _host_bytes(g1_powers)
        if n is None:
            n = len(pb) // (2 * FP_BYTES[curve])
        h = ctypes.c_void_p()
        _check(lib().kzgmi_ck_load(self.handle, CURVES[curve], pb, n, ctypes.byref(h)))
        ck = CommitKey()
        ck.ctx, ck.curve, ck.n, ck.handle = self, curve, n, h
        return ck

    def commit(self, ck: CommitKey, coeffs, m: Optional[int] = None) -> bytes:
        """sum_i coeff_i [tau^i]_1 for m <= ck.n coefficients (32 B canonical Fr each)."""
        out = ctypes.create_string_buffer(2 * FP_BYTES[ck.curve])
        if _is_device_tensor(coeffs):
            if m is None:
                m = coeffs.numel() // 32
            p = _dptr(coeffs, 32 * m)
            self._order(0)
            _check(lib().kzgmi_commit_device(self.handle, ck.handle, p, m, out))
        else:
            cb = _host_bytes(coeffs)
            if m is None:
                m = len(cb) // 32
            _check(lib().kzgmi_commit(self.handle, ck.handle, cb, m, out))
        return out.raw

    # ------------------------------------------------------------------ Fiat-Shamir
    def commit_async(self, ck: CommitKey, slot: int, coeffs, m: int):
        """Enqueue a fixed-base commitment of m device-resident coefficients on `slot`;
        msm_wait(slot) returns it."""
        self._msm_curve = getattr(self, "_msm_curve", {})
        self._msm_curve[slot] = ck.curve
        p = _dptr(coeffs, 32 * m)
        self._order(slot)
        _check(lib().kzgmi_commit_device_async(self.handle, ck.handle, int(slot), p, int(m)))

    def fs_challenge(self, curve: str, commitments, zs, ys, proofs, n: int, compressed: bool = False) -> int:
        """r of KZGMI_FLAG_FIAT_SHAMIR for device-resident inputs."""
        out = ctypes.create_string_buffer(32)
        g1b = (1 if compressed else 2) * FP_BYTES[curve]
        ptrs = (_dptr(commitments, n * g1b), _dptr(zs, 32 * n), _dptr(ys, 32 * n), _dptr(proofs, n * g1b))
        self._order(0)
        _check(lib().kzgmi_fs_challenge_device(self.handle, CURVES[curve], *ptrs, n, _flags(compressed), out))
        return int.from_bytes(out.raw, "big")

    def fs_chunk_digests(self, curve: str, commitments, zs, ys, proofs, n: int, index_offset: int, out,
                         compressed: bool = False):
        """Shard's 4096-leaf subtree roots (ceil(n / 4096) x 32 B) into device tensor `out`."""
        g1b = (1 if compressed else 2) * FP_BYTES[curve]
        ptrs = (_dptr(commitments, n * g1b), _dptr(zs, 32 * n), _dptr(ys, 32 * n), _dptr(proofs, n * g1b))
        po = _dptr(out, 32 * ((n + FS_CHUNK - 1) // FS_CHUNK))
        self._order(0)
        _check(lib().kzgmi_fs_chunk_digests_device(self.handle, CURVES[curve], *ptrs, n, int(index_offset),
                                                   _flags(compressed), po))

    def fs_challenge_from_digests(self, curve: str, digests, nchunks: int, n_total: int) -> int:
        out = ctypes.create_string_buffer(32)
        p = _dptr(digests, 32 * nchunks)
        self._order(0)
        _check(lib().kzgmi_fs_challenge_from_digests_device(self.handle, CURVES[curve], p, nchunks,
                                                            int(n_total), out))
        return int.from_bytes(out.raw, "big")

    def g1_validate(self, curve: str, points, n: int, compressed: bool = False, subgroup_check: bool = False):
        """Raise KzgmiError unless all n device-resident G1 encodings are valid."""
        p = _dptr(points, n * (1 if compressed else 2) * FP_BYTES[curve])
        self._order(0)
        _check(lib().kzgmi_g1_validate_device(self.handle, CURVES[curve], p, n, _flags(compressed, subgroup_check)))

    def g1_compress(self, curve: str, points, n: int, out):
        """Device utility: uncompressed G1 encodings -> compressed (no validation)."""
        pi, po = _dptr(points, 2 * n * FP_BYTES[curve]), _dptr(out, n * FP_BYTES[curve])
        self._order(0)
        _check(lib().kzgmi_g1_compress_device(self.handle, CURVES[curve], pi, n, po))

    def wait(self, slot: int) -> bool:
        ok = ctypes.c_int(-1)
        try:
            _check(lib().kzgmi_slot_wait(self.handle, int(slot), ctypes.byref(ok)))
        finally:
            getattr(self, "_host_keep", {}).pop(slot, None)
        return bool(ok.value)

    def last_combination(self, curve: str):
        g1b = 2 * FP_BYTES[curve]
        a = ctypes.create_string_buffer(g1b)
        b = ctypes.create_string_buffer(g1b)
        _check(lib().kzgmi_last_combination(self.handle, a, b))
        return a.raw, b.raw

    # ------------------------------------------------------------------ MSM
    def msm_g1(self, curve: str, points, scalars, n: Optional[int] = None) -> bytes:
        g1b = 2 * FP_BYTES[curve]
        out = ctypes.create_string_buffer(g1b)
        if _is_device_tensor(points):
            if n is None:
                n = points.numel() // g1b
            pp, ps = _dptr(points, n * g1b), _dptr(scalars, 32 * n)
            self._order(0)
            _check(lib().kzgmi_msm_g1_device(self.handle, CURVES[curve], pp, ps, n, out))
        else:
            (pp, lp, kp), (ps, ls, ks) = _host_ptr(points), _host_ptr(scalars)
            if n is None:
                n = lp // g1b
            if lp < n * g1b or ls < 32 * n:
                raise ValueError("input buffers shorter than n points")
            _check(lib().kzgmi_msm_g1(self.handle, CURVES[curve], pp, ps, n, out))
            del kp, ks
        return out.raw

    def msm_g1_async(self, curve: str, slot: int, points, scalars, n: int):
        """Enqueue sum k_i P_i (device tensors) on workspace `slot`; msm_wait(slot) returns it."""
        self._msm_curve = getattr(self, "_msm_curve", {})
        self._msm_curve[slot] = curve
        pp, ps = _dptr(points, n * 2 * FP_BYTES[curve]), _dptr(scalars, 32 * n)
        self._order(slot)
        _check(lib().kzgmi_msm_g1_device_async(self.handle, CURVES[curve], int(slot), pp, ps, int(n)))

    def msm_wait(self, slot: int) -> bytes:
        g1b = 2 * FP_BYTES[self._msm_curve[slot]]
        out = ctypes.create_string_buffer(g1b)
        _check(lib().kzgmi_msm_wait(self.handle, int(slot), out))
        return out.raw

    # ------------------------------------------------------------------ multi-GPU pieces
    def tensor_device(self):
        import torch
        return torch.device("cuda", self.device)

    def partial_bytes(self, curve: str) -> int:
        return int(lib().kzgmi_partial_bytes(CURVES[curve]))

    def _batch_ptrs(self, curve, commitments, zs, ys, proofs, n, compressed=False):
        g1b = (1 if compressed else 2) * FP_BYTES[curve]
        return (_dptr(commitments, n * g1b), _dptr(zs, 32 * n), _dptr(ys, 32 * n), _dptr(proofs, n * g1b))

    def batch_partial(self, srs: Srs, commitments, zs, ys, proofs, n: int, index_offset: int, seed: bytes, out):
        ptrs = self._batch_ptrs(srs.curve, commitments, zs, ys, proofs, n)
        po = _dptr(out, 2 * self.partial_bytes(srs.curve))
        sd = _challenge_seed(seed, None)
        self._order(0)
        _check(lib().kzgmi_batch_partial_device(self.handle, srs.handle, *ptrs, n, int(index_offset), sd, po))

    def batch_combine(self, srs: Srs, partials, n_parts: int) -> bool:
        ok = ctypes.c_int(-1)
        p = _dptr(partials, 2 * n_parts * self.partial_bytes(srs.curve))
        self._order(0)
        _check(lib().kzgmi_batch_combine_device(self.handle, srs.handle, p, int(n_parts), ctypes.byref(ok)))
        return bool(ok.value)

    def partial_encode(self, curve: str, records, count: int) -> list:
        """G1 encodings of `count` device-resident partial records (e.g. a shard's [A_k, B_k])."""
        g1b = 2 * FP_BYTES[curve]
        p = _dptr(records, count * self.partial_bytes(curve))
        out = ctypes.create_string_buffer(count * g1b)
        self._order(0)
        _check(lib().kzgmi_partial_encode_device(self.handle, CURVES[curve], p, int(count), out))
        return [out.raw[i * g1b:(i + 1) * g1b] for i in range(count)]

    def batch_partial_async(self, srs: Srs, slot: int, commitments, zs, ys, proofs, n: int, index_offset: int,
                            seed, out, compressed: bool = False, subgroup_check: bool = False, challenge=None,
                            trusted_g1: bool = False):
        """Enqueue this shard's partial (A_k, B_k) on `slot`; complete with wait(slot).
        challenge: r_i = r^(index_offset + i) (pass seed=None)."""
        ptrs = self._batch_ptrs(srs.curve, commitments, zs, ys, proofs, n, compressed)
        po = _dptr(out, 2 * self.partial_bytes(srs.curve))
        sd = _challenge_seed(seed, challenge)
        self._order(slot)
        _check(lib().kzgmi_batch_partial_device_async(self.handle, srs.handle, int(slot), *ptrs, n, int(index_offset),
                                                      sd, _flags(compressed, subgroup_check, False, challenge,
                                                                 trusted_g1), po))

    def batch_combine_async(self, srs: Srs, slot: int, partials, n_parts: int):
        """Enqueue sum-of-partials + pairing check on `slot`; wait(slot) returns the verdict."""
        p = _dptr(partials, 2 * n_parts * self.partial_bytes(srs.curve))
        self._order(slot)
        _check(lib().kzgmi_batch_combine_device_async(self.handle, srs.handle, int(slot), p, int(n_parts)))

    def msm_partial(self, curve: str, points, scalars, n: int, out):
        pp, ps = _dptr(points, n * 2 * FP_BYTES[curve]), _dptr(scalars, 32 * n)
        po = _dptr(out, self.partial_bytes(curve))
        self._order(0)
        _check(lib().kzgmi_msm_partial_device(self.handle, CURVES[curve], pp, ps, n, po))

    def msm_partial_async(self, curve: str, slot: int, points, scalars, n: int, out):
        pp, ps = _dptr(points, n * 2 * FP_BYTES[curve]), _dptr(scalars, 32 * n)
        po = _dptr(out, self.partial_bytes(curve))
        self._order(slot)
        _check(lib().kzgmi_msm_partial_device_async(self.handle, CURVES[curve], int(slot), pp, ps, int(n), po))

    def msm_combine_async(self, curve: str, slot: int, partials, n_parts: int):
        self._msm_curve = getattr(self, "_msm_curve", {})
        self._msm_curve[slot] = curve
        p = _dptr(partials, n_parts * self.partial_bytes(curve))
        self._order(slot)
        _check(lib().kzgmi_msm_combine_device_async(self.handle, CURVES[curve], int(slot), p, int(n_parts)))

    def msm_combine(self, curve: str, partials, n_parts: int) -> bytes:
        out = ctypes.create_string_buffer(2 * FP_BYTES[curve])
        p = _dptr(partials, n_parts * self.partial_bytes(curve))
        self._order(0)
        _check(lib().kzgmi_msm_combine_device(self.handle, CURVES[curve], p, int(n_parts), out))
        return out.raw

    # ------------------------------------------------------------------ utilities
    def pairing(self, curve: str, g1: bytes, g2: bytes) -> bytes:
        out = ctypes.create_string_buffer(12 * FP_BYTES[curve])
        _check(lib().kzgmi_pairing(self.handle, CURVES[curve], bytes(g1), bytes(g2), out))
        return out.raw

    def gen_g1(self, curve: str, scalars_dev, n: int, out_dev):
        ps, po = _dptr(scalars_dev, 32 * n), _dptr(out_dev, n * 2 * FP_BYTES[curve])
        self._order(0)
        _check(lib().kzgmi_gen_g1(self.handle, CURVES[curve], ps, n, po))

    def gen_tuples(self, curve: str, tau: int, seed: bytes, n: int, C, z, y, pi):
        ptrs = self._batch_ptrs(curve, C, z, y, pi, n)
        sd = _challenge_seed(seed, None)
        self._order(0)
        _check(lib().kzgmi_gen_tuples(self.handle, CURVES[curve], int(tau).to_bytes(32, "big"), sd, n, *ptrs))

    def g2_mul(self, curve: str, g2: bytes, k: int) -> bytes:
        out = ctypes.create_string_buffer(4 * FP_BYTES[curve])
        _check(lib().kzgmi_g2_mul(self.handle, CURVES[curve], bytes(g2), int(k).to_bytes(32, "big"), out))
        return out.raw

    def toy_srs(self, curve: str, tau: int):
        """(G2 generator, [tau]_2) encodings computed on the GPU (test/bench SRS)."""
        g2 = G2_GENERATOR[curve]
        return g2, self.g2_mul(curve, g2, tau)

    def probe_fpmul(self, curve: str) -> float:
        v = ctypes.c_double()
        _check(lib().kzgmi_probe_fpmul(self.handle, CURVES[curve], ctypes.byref(v)))
        return v.value

    def set_glv(self, msm: bool = True, batch: bool = True):
        """GLV split of full Fr scalars for MSMs / batch verification."""
        _check(lib().kzgmi_set_glv(self.handle, int(bool(msm)), int(bool(batch))))

    def set_trusted_g1(self, on: bool = True):
        """MSM inputs on this context are known G1 members (BLS12-381 MSMs may then use GLV)."""
        _check(lib().kzgmi_set_trusted_g1(self.handle, int(bool(on))))

    def set_split_acc(self, mode: int = -1):
        """Split accumulation of a batch's two MSMs: -1 auto (large synchronous calls), 0 never, 1 always."""
        _check(lib().kzgmi_set_split_acc(self.handle, int(mode)))

    def set_profiling(self, on: bool):
        _check(lib().kzgmi_set_profiling(self.handle, 1 if on else 0))

    def phase_ms(self) -> dict:
        arr = (ctypes.c_double * len(PHASES))()
        lib().kzgmi_get_phase_ms(self.handle, arr, len(PHASES))
        return dict(zip(PHASES, list(arr)))


# ---------------------------------------------------------------------- north-star API
# Standard G2 generators (ZCash / EIP-197 encodings, imaginary part first)
G2_GENERATOR = {
    "bls12_381": bytes.fromhex(
        "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
        "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8"
        "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be"
        "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801"),
    "bn254": b"".join(v.to_bytes(32, "big") for v in (
        11559732032986387107991004021392285783925812861821192530917403151452391805634,
        10857046999023057135944570762232829481370756359578518086990519993285655852781,
        4082367875863433681332203403145435568316851327593401208105741076214120093531,
        8495653923123431417604973247489272438418190587263600148770280649306958101930)),
}

_default_ctx: Optional[Context] = None


def alloc_count() -> int:
    """Process-wide number of device workspace allocations made by the library so far."""
    return int(lib().kzgmi_alloc_count())


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0, 1)
    return _default_ctx


def load_srs(curve: str, g2: bytes, tau_g2: bytes, ctx: Optional[Context] = None, g1: Optional[bytes] = None) -> Srs:
    return (ctx or default_context()).load_srs(curve, g2, tau_g2, g1=g1)


def batch_verify(commitments, zs, ys, proofs, srs: Srs, seed: Optional[bytes] = None, compressed: bool = False,
                 subgroup_check: bool = False, fiat_shamir: bool = False, challenge=None,
                 trusted_g1: bool = False) -> bool:
    """BASELINE.json:5 batch_verify(commitments, zs, ys, proofs, srs) on the GPU."""
    return srs.ctx.batch_verify(srs, commitments, zs, ys, proofs, seed=seed, compressed=compressed,
                                subgroup_check=subgroup_check, fiat_shamir=fiat_shamir, challenge=challenge,
                                trusted_g1=trusted_g1)


def msm_g1(curve: str, points, scalars, ctx: Optional[Context] = None) -> bytes:
    return (ctx or default_context()).msm_g1(curve, points, scalars)


def tuple_scalars_host(seed: bytes, i: int, tag: str) -> int:
    """The 253-bit synthetic scalar kzgmi_gen_tuples derives (for host-side checks)."""
    import hashlib
    h = hashlib.sha256(bytes(seed) + int(i).to_bytes(8, "little") + tag.encode()).digest()
    return int.from_bytes(h, "big") & ((1 << 253) - 1)
