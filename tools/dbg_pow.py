import sys, os, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "kzg-batch-verification-scheme_amd")); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch, kzgmi
from oracle.pyspec import curves as pc
ctx = kzgmi.Context(0, 2)
h = bytes.fromhex
for curve in ["bls12_381", "bn254"]:
    C = pc.CURVES[curve]
    g = json.load(open("tests/golden/%s_batch_n16.json" % curve))
    cm, pf, zb, yb = h(g["commitments"]), h(g["proofs"]), h(g["zs"]), h(g["ys"])
    srs = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))
    for r in [1, 2, C.r - 1, 0x1234567890ABCDEF << 100, C.r]:
        try:
            ok = ctx.batch_verify(srs, cm, zb, yb, pf, challenge=r)
        except kzgmi.KzgmiError as e:
            ok = "err %d" % e.code
        try:
            torch.cuda.synchronize()
            st = "sync ok"
        except Exception as e:
            st = "SYNC FAIL %s" % e
        print(curve, hex(r)[:12], ok, st, flush=True)
        if st != "sync ok":
            sys.exit(1)
ctx.close()
try:
    x = torch.ones(4, device="cuda") + 1
    torch.cuda.synchronize()
    print("after close: torch ok", x.sum().item())
except Exception as e:
    print("after close: TORCH FAIL", e)
ctx2 = kzgmi.Context(0, 2)
try:
    d = torch.frombuffer(bytearray(64), dtype=torch.uint8).cuda()
    print("ctx2 + torch ok")
except Exception as e:
    print("ctx2: TORCH FAIL", e)
