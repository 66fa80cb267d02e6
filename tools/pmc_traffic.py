"""Turn rocprofv3 --pmc CSVs (FETCH_SIZE pass, WRITE_SIZE pass) into HBM bytes
per launch of each hot kernel, with the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE reads exactly half the bytes of a wide
(16 B/lane) coalesced stream, so it is doubled; WRITE_SIZE is exact for 16-B
stores.  Both counters are in KiB.  The warmup dispatches are skipped.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --m 4096 --n 16384 --out profiles/traffic_r01.json
"""
import argparse
import csv
import json
import statistics


KERNELS = ("k_price", "k_ftran_bc", "k_update", "k_tab_fold", "k_cfold", "k_fold", "k_bc_gather")


def per_kernel(path, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            key = next((k for k in KERNELS if k in name), None)
            if key:
                vals.setdefault(key, []).append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--skip", type=int, default=20, help="warmup launches to drop")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f = per_kernel(a.fetch_csv, "FETCH_SIZE")
    w = per_kernel(a.write_csv, "WRITE_SIZE")
    out = {"m": a.m, "n": a.n, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes)",
           "correction": "FETCH_SIZE x2 (gfx950 wide-stream half count), KiB -> bytes"}
    for k in KERNELS:
        skip = a.skip if "fold" not in k else 0  # a fold runs once per window
        fv = f.get(k, [])[skip:]
        wv = w.get(k, [])[skip:]
        if not fv or not wv:
            continue
        rd = 2.0 * 1024.0 * statistics.median(fv)
        wr = 1024.0 * statistics.median(wv)
        out[k] = {"launches": len(fv), "read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
                  "raw_fetch_kib_median": statistics.median(fv), "raw_write_kib_median": statistics.median(wv)}
        if k == "k_tab_fold":  # 8-byte-per-lane tile loads: the x2 stream correction may not hold
            out[k]["note"] = "8 B/lane loads: read_bytes assumes the x2 correction; raw x1 = %.0f" % (
                1024.0 * statistics.median(fv))
    if "k_price" in out:
        out["price_hbm_bytes_per_launch"] = out["k_price"]["hbm_bytes"]
    upd = "k_ftran_bc" if "k_ftran_bc" in out else "k_update"
    if upd in out:
        out["update_kernel"] = upd
        out["update_hbm_bytes_per_launch"] = out[upd]["hbm_bytes"]
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
