"""Instruction mix of the hottest loop of one kernel in a device .s file:
the loop = the basic blocks between a label and the backward branch to it
that contains the most v_exp_f32.  Usage: asm_loop_mix.py file.s symbol_regex"""
import re
import sys
from collections import Counter

path, pat = sys.argv[1], re.compile(sys.argv[2])
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^[A-Za-z_]\S*:", l) and pat.search(l.split(":")[0]))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {l[:-1]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:$", l)}
best = None
for i, l in enumerate(body):
    m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\S+)|^\s+s_branch\s+(\.LBB\S+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    j = labels.get(tgt)
    if j is None or j >= i:
        continue
    seg = body[j:i + 1]
    nexp = sum("v_exp_f32" in s for s in seg)
    if best is None or nexp > best[0] or (nexp == best[0] and i - j < best[2] - best[1]):
        best = (nexp, j, i)
_, j, i = best
seg = [s.strip().split()[0] for s in body[j:i + 1] if s.startswith("\t") and not s.strip().startswith((";", "."))]
c = Counter()
for op in seg:
    if op.startswith("v_mfma"):
        c["mfma"] += 1
    elif op.startswith("v_"):
        c["valu"] += 1
        c["valu:" + op] += 1
    elif op.startswith("ds_"):
        c["lds"] += 1
    elif op.startswith(("global_", "buffer_")):
        c["vmem"] += 1
    elif op.startswith("s_"):
        c["salu/ctrl"] += 1
print(f"loop lines {j}-{i} of {body[0][:80]}")
for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
    print(f"  {v:5d}  {k}")
