"""Graph-launch time per pass for one 63-pass window (fold included) at C3,
per library build (SPX_LIB), interleaved over 3 rounds, best of 6 windows
each: the A/B of whole passes (tools/ab_libs.py gives the event-timed kernel
split).  Also used for timing-only builds whose pivots do not advance (one
graph launch still runs 63 passes).
    python tools/pass_ab.py default simplex_method_gpu_amd/_build/xNAME/libsimplex.so ...
    SPX_DEFER_TAIL=0 python tools/pass_ab.py default   # env knobs apply to every build
    python tools/pass_ab.py env:SPX_FTRAN_RPW=1 env:SPX_FTRAN_RPW=4   # knobs per entry
    PASS_AB_M=1024 PASS_AB_N=4096 python tools/pass_ab.py ...          # another LP size
    PASS_AB_PRICING=2 python tools/pass_ab.py ...                      # steepest edge
    PASS_AB_WINDOW=64 python tools/pass_ab.py ...                      # Context(window=...)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, json
sys.path.insert(0, %r)
import simplex_method_gpu_amd as spx
best = 1e9
with spx.Context(m=int(os.environ.get('PASS_AB_M', 4096)), n=int(os.environ.get('PASS_AB_N', 16384)), seed=0, device=0,
                 pricing=int(os.environ.get('PASS_AB_PRICING', 0)), window=int(os.environ.get('PASS_AB_WINDOW', 0))) as ctx:
    ctx.iterate(63)
    for r in range(6):
        t0 = time.perf_counter()
        ctx.iterate(63)
        best = min(best, time.perf_counter() - t0)
print(json.dumps({"us_per_pass": round(best / 63 * 1e6, 2)}))
''' % ROOT
libs = sys.argv[1:] or ["default"]
res = {l: [] for l in libs}
for r in range(3):
    for l in libs:
        env = dict(os.environ)
        if l.startswith("env:"):  # env:VAR=VAL[,VAR=VAL]: the default build with these knobs
            for kv in l[4:].split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        elif l != "default":
            env["SPX_LIB"] = os.path.join(ROOT, l)
        out = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, env=env, timeout=200)
        line = [x for x in out.stdout.splitlines() if x.startswith("{")]
        if not line:
            print(out.stdout[-500:], out.stderr[-1500:], flush=True)
            sys.exit(1)
        res[l].append(json.loads(line[-1])["us_per_pass"])
        print(l, res[l][-1], flush=True)
print(json.dumps({l: min(v) for l, v in res.items()}))
