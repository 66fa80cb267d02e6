"""One rank of tests/test_watchdog.py (gloo on the CPU): bench.py's Watchdog
around a barrier (rank 0) while rank 1 stalls inside its own watched phase,
or (mode "ok") phases that end within the bound."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch.distributed as dist  # noqa: E402

from bench import Watchdog  # noqa: E402


class FakeCtx:
    last_pivots = 1234

    def dispatch_stats(self):
        return {"eager_passes": 3, "graph_launches": 7}


def main():
    mode = sys.argv[1]
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    wd = Watchdog(2.0, rank)
    if mode == "ok":
        for k in range(3):
            with wd.phase(f"window {k}", FakeCtx()):
                time.sleep(0.5)
                dist.barrier()
        time.sleep(3.0)  # disarmed: no bound
        dist.destroy_process_group()
        print("done", flush=True)
        return
    if rank == 1:
        with wd.phase("timed window", FakeCtx()):
            time.sleep(60)  # a stalled peer
    else:
        with wd.phase("next window 1", FakeCtx()):
            dist.barrier()  # waits for rank 1 forever
    print("unreachable", flush=True)


if __name__ == "__main__":
    main()
