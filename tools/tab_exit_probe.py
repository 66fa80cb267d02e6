"""Exit-path probe: one persistent-loop context (k_tab_loop, or k_loop with
PROBE_TAB=0), a few passes, close, interpreter exit.  Run under rocprofv3 to
check teardown (SPX_LOOP_COOP=1: the round-1 cooperative launch; PROBE_SEGV=1:
the native stack of a crash, tools/segv_trace.c); writes /proc/self/maps to PROBE_MAPS (if set) just before exit
so the PCs of a crash stack in the same process can be mapped to libraries."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import simplex_method_gpu_amd as spx  # noqa: E402

if os.environ.get("PROBE_SEGV") == "1":  # native stack of a fatal signal (tools/segv_trace.c)
    import ctypes

    ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsegv_trace.so")).segv_trace_install()

persist = os.environ.get("PROBE_PERSIST", "1") == "1"
tab = os.environ.get("PROBE_TAB", "1") == "1"
ctx = spx.Context(m=1024, n=4096, seed=0, tableau=tab, persist=persist, window=64)
print(ctx.iterate(100), ctx.config().get("persistent"))
ctx.close()
print("closed", flush=True)
maps = os.environ.get("PROBE_MAPS")
if maps:
    with open("/proc/self/maps") as f, open(maps, "w") as g:
        g.write(f.read())
