"""Basic blocks of one kernel in a hipcc -S listing: instruction counts by class and branch
targets, to see what a traversal step costs.  usage: python tools/asm_blocks.py FILE.s SYMBOL"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\w+|" + re.escape(sym) + r"):", l)
    if m:
        cur = {"name": m.group(1), "ins": []}
        blocks.append(cur)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    if cur is not None:
        cur["ins"].append(t.split(";")[0].strip())


def cls(op):
    if op.startswith("v_"):
        return "f64" if "_f64" in op else "valu"
    if op.startswith("s_"):
        return "salu" if not op.startswith(("s_cbranch", "s_branch", "s_waitcnt")) else "ctl"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


for b in blocks:
    c = {}
    for i in b["ins"]:
        k = cls(i.split()[0])
        c[k] = c.get(k, 0) + 1
    br = [i for i in b["ins"] if i.startswith(("s_cbranch", "s_branch"))]
    print(f"{b['name']:14s} n={len(b['ins']):4d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())) +
          ("  -> " + ", ".join(x.split()[-1] + ("(" + x.split()[0][10:] + ")" if x.startswith("s_cbranch") else "") for x in br) if br else ""))
