"""Per-step summary of a kernel-stats CSV (tools/rocpd_stats.py output):
launches and time per step, edge vs node level, the top node kernels.

    python tools/node_summary.py profiles/<name>_kernel_stats.csv STEPS [TOP]
"""
import csv
import sys

path, S = sys.argv[1], int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
edge = ("km_", "k_loss_fwd", "k_loss_bwd", "k_edge_bn_sums")
tn = tt = et = 0
for r in rows:
    n, t = int(r["Calls"]), float(r["TotalDurationNs"])
    if n < S:
        continue
    tn += n
    tt += t
    if any(k in r["Name"] for k in edge):
        et += t
print("launches/step %.1f  kernel ms/step %.3f  edge %.3f  node %.3f"
      % (tn / S, tt / S / 1e6, et / S / 1e6, (tt - et) / S / 1e6))
k = 0
for r in rows:
    if int(r["Calls"]) < S or any(e in r["Name"] for e in edge):
        continue
    print(f"{int(r['Calls']) / S:6.1f}/step {float(r['TotalDurationNs']) / 1e6 / S:7.3f}ms "
          f"avg {float(r['AverageNs']) / 1e3:7.1f}us  {r['Name'][:90]}")
    k += 1
    if k >= top:
        break
