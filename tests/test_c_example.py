"""The drop-in boundary from plain C (examples/verify_files.c): gcc against include/kzgmi.h and
libkzgmi.so, no Python in the verifying process.  CPU: it links, runs, and fails loudly
(KZGMI_ERR_DEVICE, exit 2) without a GPU.  GPU: golden batches verified through the host-pointer
entry point, verdict and combined points bit-exact with the fixtures (the oracle's values)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "kzg-batch-verification-scheme_amd", "kzgmi")


@pytest.fixture(scope="module")
def c_binary(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "libkzgmi.so")):
        pytest.fail("libkzgmi.so not built (run __graft_entry__.build())")
    out = str(tmp_path_factory.mktemp("cex") / "verify_files")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "verify_files.c"), "-L", LIBDIR, "-lkzgmi",
                    "-Wl,-rpath," + LIBDIR, "-Wl,-rpath-link,/opt/rocm/lib", "-o", out],
                   check=True, capture_output=True, text=True)
    return out


def run_case(binary, tmp_path, curve, g, src):
    files = {}
    for k, v in (("g2", g["g2"]), ("tau", g["tau_g2"]), ("cm", src["commitments"]), ("zs", src["zs"]),
                 ("ys", src["ys"]), ("pf", src["proofs"]), ("seed", g["seed"])):
        files[k] = str(tmp_path / (k + ".bin"))
        with open(files[k], "wb") as f:
            f.write(bytes.fromhex(v))
    return subprocess.run([binary, curve, str(g["n"]), files["g2"], files["tau"], files["cm"], files["zs"],
                           files["ys"], files["pf"], files["seed"]], capture_output=True, text=True, timeout=120)


def golden(name):
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        return json.load(f)


def test_c_caller_without_gpu_fails_loudly(c_binary, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    g = golden("bls12_381_batch_n4.json")
    r = run_case(c_binary, tmp_path, "bls12_381", g, g)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "kzgmi error -5" in r.stderr, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["bls12_381", "bn254"])
def test_c_caller_golden_batch(c_binary, tmp_path, curve):
    g = golden("%s_batch_n16.json" % curve)
    for key in ["valid", "neg_flip_y"]:
        src = g if key == "valid" else g[key]
        r = run_case(c_binary, tmp_path, curve, g, src)
        assert r.returncode == 0, (r.returncode, r.stderr)
        exp = g[key]
        assert r.stdout.split() == ["ok=%d" % int(exp["ok"]), "A=" + exp["A"], "B=" + exp["B"]], (key, r.stdout)
