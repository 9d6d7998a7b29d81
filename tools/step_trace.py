"""Per-step kernel summary of a rocprofv3 --kernel-trace run of bench.py.

    python tools/step_trace.py <run_kernel_trace.csv> [step_index]

Steps are delimited by k_adam launches; prints calls / total us per kernel
name for one step (default: the 9th, inside the timed replays)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 8


def name(s):
    s = s.replace("void ", "").replace("(anonymous namespace)::", "")
    s = re.sub(r"\(.*", "", s)
    m = re.search(r"(Fill|CUDAFunctorOnSelf_add|CUDAFunctor_add|direct_copy|MulFunctor|reduce_kernel)", s)
    if s.startswith("at::native") and m:
        s = "torch_" + m.group(1)
    return s[:40]


ends = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
seg = rows[ends[which - 1] + 1:ends[which] + 1]
t0 = int(seg[0]["Start_Timestamp"])
t1 = int(seg[-1]["End_Timestamp"])
cnt, tot = collections.Counter(), collections.Counter()
for r in seg:
    n = name(r["Kernel_Name"])
    cnt[n] += 1
    tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print(f"step {which}: {len(seg)} kernels, {(t1 - t0) / 1e3:.1f} us wall, "
      f"{sum(tot.values()):.1f} us busy")
for n, _ in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{n:42s} {cnt[n]:4d} {tot[n]:9.1f} us  {tot[n] / cnt[n]:7.1f} avg")
