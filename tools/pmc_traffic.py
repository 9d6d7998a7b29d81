"""HBM traffic per launch of the edge kernels from rocprofv3 FETCH_SIZE /
WRITE_SIZE passes (tools/prof_pmc.sh), written to profiles/<name>_traffic.json.

Units and corrections (MI355X_MICROARCH.md §HBM, and our own calibration in
profiles/r02_fetch_calibration.json, made by tools/fetch_calib.hip +
tools/calib_pmc.sh on known byte counts past the Infinity Cache):
  * FETCH_SIZE / WRITE_SIZE are KiB per dispatch;
  * WRITE_SIZE is exact for 4- and 16-byte-per-lane stores;
  * FETCH_SIZE reads 1/2 of a fully coalesced stream (4 or 16 B/lane alike)
    and 0.625 of the edge kernels' own pattern (16-lane groups reading 64-byte
    runs of different channel rows): reads are corrected by 1/0.625 = 1.6;
    the guide's 2.0 (upper bound) is reported beside it.

    python tools/pmc_traffic.py gpurun_out/pmc_xxx r02b128 [E F B [pass-dir prefix]]
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
d, name = sys.argv[1], sys.argv[2]
E = int(sys.argv[3]) if len(sys.argv) > 3 else 16 * 2394 * 128
F = int(sys.argv[4]) if len(sys.argv) > 4 else 10
B = int(sys.argv[5]) if len(sys.argv) > 5 else 8
cal = json.load(open(os.path.join(ROOT, "profiles", "r02_fetch_calibration.json")))
read_cal = cal["edge_read_correction"]


def kname(full):
    """'void (anonymous namespace)::km_source_bwd<10, 1, true>(EdgeGeo, ...)' ->
    'km_source_bwd<10>' (the Fdim only: the precision / mask template flags of
    one edge path are one kernel per step)"""
    k = full.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    if k.startswith(("km_", "k_")) and "<" in k:
        k = k.split("<")[0] + "<" + k.split("<")[1].split(",")[0].rstrip(">") + ">"
    return k


# the profiled edge path's MFMA kernels: 1 = mfma (the default path; its
# forward kernels at PREC 0), 4 = bf16x6
PREC = os.environ.get("PFSGNN_PMC_PREC", "1")
PATH_OF = {"4": "bf16x6", "1": "mfma", "0": "mfma32", "3": "bf16x3"}


def per_dispatch(path, counter):
    agg, n = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        full = r["Kernel_Name"]
        if "km_" in full and "forward" not in full:
            # only the headline path's kernels (bench.py also times other
            # paths): <F, PREC[, TM]>, the forward kernels' PREC being 0 for it
            tmpl = full.split("<")[1].split(">")[0].split(",")
            want = ("0" if PREC == "1" else PREC) if kname(full).split("<")[0] in (
                "km_edge_mlp_fwd", "km_source_fwd", "km_source_fwd_ft", "km_target_fwd") else PREC
            if tmpl[1].strip() != want:
                continue
        k = kname(r["Kernel_Name"])
        agg[k] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    return {k: agg[k] / len(n[k]) * 1024.0 for k in agg}   # KiB -> bytes


def algorithmic(kernel):
    """Algorithmic bytes per launch (bench.py:kernel_bytes_per_edge x E)."""
    import bench
    per = bench.kernel_bytes_per_edge(F)
    base = kernel.split("<")[0].replace("km_", "").replace("k_", "")
    base = {"source_fwd_ft": "source_fwd"}.get(base, base)   # (the fiber-tile grid: same bytes)
    if base not in per:
        return None
    if base == "edge_mlp_bwd":          # block 0 writes no input gradient
        return (per[base] * (B - 1) + 3 * 4 * F) * E / B
    return per[base] * E


pre = sys.argv[6] if len(sys.argv) > 6 else ""     # pass directories <d>/<pre>fetch, <pre>write
fetch = per_dispatch(os.path.join(d, pre + "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
write = per_dispatch(os.path.join(d, pre + "write", "run_counter_collection.csv"), "WRITE_SIZE")
out = {"E": E, "F": F, "edge_path": PATH_OF.get(PREC, PREC), "read_calibration": read_cal,
       "calibration": "profiles/r02_fetch_calibration.json (rdrows pattern)",
       "note": "traffic_bytes = FETCH_SIZE*read_calibration + WRITE_SIZE per launch; "
               "traffic_bytes_guide2x uses the guide's 2.0 read correction (upper bound)",
       "kernels": {}}
for k in sorted(fetch):
    if "<" not in k:
        continue
    fb, wb = fetch[k], write.get(k, 0.0)
    alg = algorithmic(k)
    rec = {"fetch_bytes_raw": fb, "write_bytes": wb, "traffic_bytes": fb * read_cal + wb,
           "traffic_bytes_guide2x": fb * 2.0 + wb}
    if alg:
        rec["algorithmic_bytes"] = alg
        rec["traffic_over_algorithmic"] = round(rec["traffic_bytes"] / alg, 3)
        rec["traffic_over_algorithmic_guide2x"] = round(rec["traffic_bytes_guide2x"] / alg, 3)
    out["kernels"][k] = rec
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
path = os.path.join(ROOT, "profiles", f"{name}_traffic.json")
json.dump(out, open(path, "w"), indent=1)
for k, v in out["kernels"].items():
    if "algorithmic_bytes" in v:
        print(f"{k:26s} traffic {v['traffic_bytes'] / 1e6:8.1f} MB/launch (x{v['traffic_over_algorithmic']:.2f} "
              f"of algorithmic {v['algorithmic_bytes'] / 1e6:.1f}; guide 2x: x{v['traffic_over_algorithmic_guide2x']:.2f})")
print("read calibration", read_cal, "->", path)
