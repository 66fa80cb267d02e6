"""Multi-rank check of the column-sharded pricing path (RCCL all-gather MINLOC).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 tools/dist_check.py [--m 512 --n 2048 --k 300]

Every rank runs the same LP with its pricing shard; rank 0 also runs the
single-rank solve.  The sharded run must reproduce the single-rank run bit for
bit (same pivots, b_ixs, x_b, y) on every rank — within 1e-9 with
--row-shard, where s_y is evaluated from the gathered c_B.alpha sum.  Ranks map to devices
LOCAL_RANK % device_count, so it also runs (RCCL permitting) with several
ranks on one GPU.  The out-of-band id exchange uses a gloo group.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--k", type=int, default=300)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--row-shard", action="store_true")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ndev = torch.cuda.device_count()
    dev = int(os.environ.get("LOCAL_RANK", "0")) % max(ndev, 1)
    import simplex_method_gpu_amd as spx

    ctx = spx.Context(m=a.m, n=a.n, seed=a.seed, device=dev, rank=rank, nranks=world, row_shard=a.row_shard)
    obj = [spx.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    ctx.attach_comm(obj[0])
    st, piv = ctx.iterate(a.k)
    s = ctx.state()
    z = ctx.objective()
    ctx.close()
    # gather everything on rank 0 and compare to the single-rank run
    mine = {"status": int(st), "pivots": piv, "z": z, "b_ixs": s["b_ixs"].tolist(), "x_b": s["x_b"].tolist(),
            "y": s["y"].tolist()}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    ok = True
    if rank == 0:
        with spx.Context(m=a.m, n=a.n, seed=a.seed, device=dev) as ref:
            rst, rpiv = ref.iterate(a.k)
            rs = ref.state()
            rz = ref.objective()
        def close(u, v):  # row-sharded storage reassociates s_y: 1e-9 instead of bitwise
            u, v = np.asarray(u), np.asarray(v)
            return np.array_equal(u, v) if not a.row_shard else \
                float(np.max(np.abs(u - v))) <= 1e-9 * max(1.0, float(np.max(np.abs(v))))

        for r, d in enumerate(allr):
            same = (d["status"] == int(rst) and d["pivots"] == rpiv and close([d["z"]], [rz])
                    and d["b_ixs"] == rs["b_ixs"].tolist()
                    and close(d["x_b"], rs["x_b"]) and close(d["y"], rs["y"]))
            print(f"rank {r}: status={d['status']} pivots={d['pivots']} z={d['z']!r} identical_to_1rank={same}")
            ok &= same
        print("DIST_CHECK", "PASS" if ok else "FAIL", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
