"""Instruction mix of the kernels in a hipcc -S listing: python tools/isamix.py file.s [filter]."""
import collections
import re
import sys

s = open(sys.argv[1]).read().split("\n")
want = sys.argv[2] if len(sys.argv) > 2 else ""
starts = [(i, l.split(":")[0]) for i, l in enumerate(s) if re.match(r"^_Z\w+:", l)]
for idx, (i, name) in enumerate(starts):
    if want not in name:
        continue
    end = starts[idx + 1][0] if idx + 1 < len(starts) else len(s)
    c = collections.Counter()
    for l in s[i:end]:
        l = l.strip()
        if not l or l.startswith((".", ";")) or l.endswith(":"):
            continue
        op = l.split()[0]
        if op.startswith(("v_readlane", "v_writelane")):
            c["lane"] += 1
        elif op.startswith(("s_load", "s_buffer_load")):
            c["s_load"] += 1
        elif op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith(("v_fma", "v_pk_fma", "v_fmac", "v_mac")):
            c["fma"] += 1
        elif op.startswith("ds_"):
            c["ds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif op.startswith("s_waitcnt"):
            c["wait"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    print(name[:34].ljust(34), " ".join(f"{k}={v}" for k, v in sorted(c.items())))
