"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

want = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, {}
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|"
                  r"Occupancy \[waves/SIMD\]|SGPRs): (\d+)", l)
    if m and cur:
        rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
for k, v in rows.items():
    if want in k:
        print(k[:44].ljust(44), " ".join(f"{a}={b}" for a, b in v.items()))
