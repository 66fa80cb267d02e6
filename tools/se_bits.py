"""Steepest-edge state after K pivots at C3 (and m = 2048 with the dense
B_w operand off), printed as a hash of the weights, x_b and the objective's
bits: compare two builds (SPX_LIB) for bit-identity.  python tools/se_bits.py"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

out = {}
for (m, n, k) in ((4096, 16384, 700), (2048, 8192, 400), (300, 1200, 250)):
    with spx.Context(m=m, n=n, seed=0, device=0, pricing=spx.PRICING_STEEPEST) as ctx:
        st, p = ctx.iterate(k)
        w = ctx.weights()
        s = ctx.state()
        h = hashlib.sha256(w.tobytes() + s["x_b"].tobytes() + s["b_ixs"].tobytes()).hexdigest()[:16]
        out[f"{m}x{n}"] = [int(st), p, ctx.objective().hex(), h]
print(json.dumps({"lib": os.environ.get("SPX_LIB", "default")[-40:], **out}))
