# First-window attribution: fresh processes, timed windows
# starting 0..3 windows later (same pivot ranges at different positions), C3
# and C2, each window's streamed pricing bytes beside its rate.
set -o pipefail
OUT=gpurun_out/${1:-r6win}
mkdir -p $OUT
for rep in 1 2; do for c in C3 C2; do for sh in 0 1 2 3; do
  timeout -k 10 120 python3 -u tools/window_fresh.py --config $c --nw 4 --shift $sh >> $OUT/fresh.jsonl 2>/dev/null || exit 1
done; done; done
python3 - $OUT/fresh.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
for c in ("C3", "C2"):
    by = collections.defaultdict(list)
    for r in rows:
        if r["config"] != c: continue
        for k, (v, p) in enumerate(zip(r["it_s"], r["piv0"])):
            by[p].append((k, v))
    for p in sorted(by):
        print(c, "piv0", p, " ".join(f"pos{k}:{v:.0f}" for k, v in sorted(by[p])))
PY
