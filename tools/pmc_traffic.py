"""HBM traffic per launch of the edge kernels from rocprofv3 FETCH_SIZE /
WRITE_SIZE passes (tools/prof_pmc.sh), written to profiles/<name>_traffic.json.

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  WRITE_SIZE reads dword stores
exactly (MI355X_MICROARCH.md, HBM section).  FETCH_SIZE under-reports wide
coalesced reads on gfx950 and is uncalibrated for other widths, so it is
calibrated on OUR access pattern: k_edge_bn_sums reads exactly the two edge
tensors g and y (2*F*4 bytes per edge, 4-byte-per-lane coalesced rows, the
pattern of every edge kernel) and nothing else of size.

    python tools/pmc_traffic.py gpurun_out/pmc3 r01 [E F]
"""
import collections
import csv
import json
import os
import sys

d, name = sys.argv[1], sys.argv[2]
E = int(sys.argv[3]) if len(sys.argv) > 3 else 16 * 2394 * 128
F = int(sys.argv[4]) if len(sys.argv) > 4 else 10


def kname(full):
    """'void (anonymous namespace)::km_source_bwd<10>(EdgeGeo, ...)' -> 'km_source_bwd<10>'"""
    return full.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def per_dispatch(path, counter):
    agg, n = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = kname(r["Kernel_Name"])
        agg[k] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    return {k: agg[k] / len(n[k]) * 1e3 for k in agg}   # KB -> bytes


fetch = per_dispatch(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
write = per_dispatch(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
cal_key = [k for k in fetch if k.startswith("k_edge_bn_sums")][0]
read_cal = (2 * F * 4 * E) / fetch[cal_key]
out = {"E": E, "F": F, "calibration_kernel": cal_key, "read_calibration": read_cal,
       "note": "traffic_bytes = FETCH_SIZE*read_calibration + WRITE_SIZE, per launch", "kernels": {}}
for k in sorted(fetch):
    if "<" not in k:
        continue
    fb, wb = fetch[k], write.get(k, 0.0)
    out["kernels"][k] = {"fetch_bytes_raw": fb, "write_bytes": wb,
                         "traffic_bytes": fb * read_cal + wb}
os.makedirs("profiles", exist_ok=True)
path = os.path.join("profiles", f"{name}_traffic.json")
json.dump(out, open(path, "w"), indent=1)
for k, v in out["kernels"].items():
    print(f"{k:28s} traffic {v['traffic_bytes'] / 1e6:8.1f} MB/launch "
          f"(fetch raw {v['fetch_bytes_raw'] / 1e6:7.1f}, write {v['write_bytes'] / 1e6:7.1f})")
print("read calibration", read_cal, "->", path)
