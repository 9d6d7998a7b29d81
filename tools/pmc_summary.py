"""Summarise rocprofv3 --pmc counter_collection.csv: per kernel, mean counter value per dispatch.
    python tools/pmc_summary.py <csv> [kernel-substring ...]"""
import csv
import collections
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
want = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"]
    if want and not any(w in k for w in want):
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("FETCH_SIZE", 0))):
    n = len(disp[k])
    nm = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    print(nm[:40].ljust(40), n, " ".join(f"{c}={x / n:.4g}" for c, x in sorted(v.items())))
