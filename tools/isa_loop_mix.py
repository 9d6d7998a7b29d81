"""Instruction mix of the hottest loop of a kernel in a hipcc -S listing.

    python tools/isa_loop_mix.py <file.s> <mangled-name-substring> [...]

The loop is the largest region [label, backward branch to it]; counts MFMA,
VALU, LDS, VMEM, SALU and waitcnt instructions in it."""
import re
import sys

src = open(sys.argv[1]).read().split("\n")
starts = [i for i, l in enumerate(src) if re.match(r"^_Z\S*:", l)]
for pat in sys.argv[2:]:
    for si in starts:
        name = src[si].split(":")[0]
        if pat not in name:
            continue
        end = next(i for i in range(si, len(src)) if src[i].startswith(".Lfunc_end"))
        body = src[si:end]
        labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S*:", l)}
        best = None
        for i, l in enumerate(body):
            m = re.match(r"\s*s_cbranch_\w+\s+(\.LBB\S+)|\s*s_branch\s+(\.LBB\S+)", l)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in labels and labels[tgt] < i and (best is None or i - labels[tgt] > best[1] - best[0]):
                    best = (labels[tgt], i)
        if best is None:
            continue
        cnt = {}
        for l in body[best[0]:best[1] + 1]:
            t = l.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            op = t.split()[0]
            k = ("mfma" if "mfma" in op else "waitcnt" if op.startswith("s_waitcnt") else
                 "lds" if op.startswith("ds_") else "vmem" if op.startswith(("buffer_", "global_")) else
                 "dpp" if "dpp" in t else "valu" if op.startswith("v_") else
                 "salu" if op.startswith("s_") else "other")
            cnt[k] = cnt.get(k, 0) + 1
        print(name[:70], "loop lines", best[1] - best[0], cnt)
