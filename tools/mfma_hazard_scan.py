"""Wait states between each MFMA and the next instructions touching its
destination VGPRs, from a kernel's .s (hipcc --cuda-device-only -S): every
path out of the MFMA (fall-through and branch targets) is walked up to a
horizon, counting one state per instruction and N+1 per s_nop N (inline asm
markers and labels count nothing -- an empty asm emits no instruction).  An
access of a destination register before `need` states is reported, except a
following MFMA that takes the whole destination as its C and writes it again
(an accumulation chain, which the hardware forwards).
    python tools/mfma_hazard_scan.py file.s kernel_symbol [need]"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def parse(path, sym):
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    en = next((i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end")), len(lines))
    ins, labels = [], {}
    for l in lines[st + 1:en]:
        s = l.split(";")[0].strip()
        if not s or s.startswith("."):
            if re.match(r"^\.LBB\w+:", s):
                labels[s[:-1]] = len(ins)
            continue
        ins.append(s)
    return ins, labels


def states(s):
    m = re.match(r"s_nop\s+(\d+)", s)
    return int(m.group(1)) + 1 if m else 1


def operands(s):
    op, _, rest = s.partition(" ")
    parts = [p.strip() for p in rest.split(",")]
    return op, parts


def succ(ins, labels, i):
    op, parts = operands(ins[i])
    out = []
    if op.startswith("s_cbranch") or op == "s_branch":
        out.append(labels.get(parts[0]))
    if op != "s_branch" and op != "s_endpgm" and i + 1 < len(ins):
        out.append(i + 1)
    return [o for o in out if o is not None]


def scan(ins, labels, need, war=True):
    found = []
    for i, s in enumerate(ins):
        op, parts = operands(s)
        if not op.startswith("v_mfma"):
            continue
        dst = regs(parts[0])
        ab = regs(parts[1]) | regs(parts[2])
        srcs = (ab | regs(parts[3])) - dst
        stack, seen = [(j, states(s) - 1) for j in succ(ins, labels, i)], set()
        while stack:
            j, ws = stack.pop()
            if (j, ws) in seen or ws >= need:
                continue
            seen.add((j, ws))
            t = ins[j]
            o2, p2 = operands(t)
            touched = regs(",".join(p2)) & dst if p2 and p2[0] else set()
            if touched:
                # an MFMA taking the whole destination as its C (the LLVM model's
                # full-overlap SrcC case: no states) is not reported
                chain = (o2.startswith("v_mfma") and regs(p2[3]) == dst
                         and not (regs(p2[1]) | regs(p2[2])) & dst)
                if not chain:
                    found.append((i, j, ws, s, t, "RAW/WAW on D"))
                if not chain or regs(p2[0]) == dst:
                    continue   # (a chained MFMA owns the registers from here)
            # WAR: a write of one of this MFMA's source registers
            if war and p2 and p2[0] and not o2.startswith(("s_", "buffer_store", "global_store", "ds_write")):
                w = regs(p2[0]) & srcs
                if w:
                    found.append((i, j, ws, s, t, "WAR on " + ("A/B" if w & ab else "C")))
            stack += [(k, ws + states(t)) for k in succ(ins, labels, j)]
    return found


if __name__ == "__main__":
    path, sym = sys.argv[1], sys.argv[2]
    need = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    ins, labels = parse(path, sym)
    f = scan(ins, labels, need)
    print(f"{len(ins)} instructions, {sum(1 for s in ins if s.startswith('v_mfma'))} MFMAs, "
          f"{len(f)} accesses of an MFMA destination within {need} states")
    for i, j, ws, s, t, kind in f:
        print(f"  [{i}] {s}\n     -> [{j}] {kind} after {ws} states: {t}")
