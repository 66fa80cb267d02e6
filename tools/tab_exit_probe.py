"""Exit-path probe: one window-tableau context (persistent k_tab_loop), a few
passes, close, interpreter exit.  Run under rocprofv3 to check teardown."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

persist = os.environ.get("PROBE_PERSIST", "1") == "1"
ctx = spx.Context(m=1024, n=4096, seed=0, tableau=True, persist=persist)
print(ctx.iterate(100), ctx.config().get("persistent"))
ctx.close()
print("closed", flush=True)
