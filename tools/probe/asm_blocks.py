"""Per-basic-block instruction counts of the hottest loop (see asm_loop_mix.py):
one line per block with its label, MFMA / VALU / LDS / VMEM counts and the
branch it ends with.  Usage: asm_blocks.py file.s symbol_regex"""
import re
import sys

path, pat = sys.argv[1], re.compile(sys.argv[2])
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^[A-Za-z_]\S*:", l) and pat.search(l.split(":")[0]))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {l[:-1]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:$", l)}
best = None
for i, l in enumerate(body):
    m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
    if m and labels.get(m.group(1), 1 << 30) < i:
        j = labels[m.group(1)]
        n = sum("v_exp_f32" in s for s in body[j:i + 1])
        if best is None or n > best[0]:
            best = (n, j, i)
_, j, i = best
blk = {"name": body[j][:-1], "mfma": 0, "valu": 0, "lds": 0, "vmem": 0, "exp": 0}
for s in body[j + 1:i + 1] + [".end:"]:
    t = s.strip()
    if re.match(r"^\.\w+:$", t):
        print(f"{blk['name']:14s} mfma {blk['mfma']:3d} valu {blk['valu']:3d} (exp {blk['exp']:2d}) lds {blk['lds']:2d} "
              f"vmem {blk['vmem']:2d}  {blk.get('br', '')}")
        blk = {"name": t[:-1], "mfma": 0, "valu": 0, "lds": 0, "vmem": 0, "exp": 0}
        continue
    if not t or t.startswith((";", ".")):
        continue
    op = t.split()[0]
    if op.startswith("v_mfma"):
        blk["mfma"] += 1
    elif op.startswith("v_"):
        blk["valu"] += 1
        blk["exp"] += op.startswith("v_exp")
    elif op.startswith("ds_"):
        blk["lds"] += 1
    elif op.startswith(("global_", "buffer_")):
        blk["vmem"] += 1
    elif op.startswith(("s_cbranch", "s_branch")):
        blk["br"] = t
        print(f"{blk['name']:14s} mfma {blk['mfma']:3d} valu {blk['valu']:3d} (exp {blk['exp']:2d}) lds {blk['lds']:2d} "
              f"vmem {blk['vmem']:2d}  {blk.get('br', '')}")
        blk = {"name": "  (fallthru)", "mfma": 0, "valu": 0, "lds": 0, "vmem": 0, "exp": 0}
