"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (static counts).

    python tools/isa_blocks.py <file.s> <mangled kernel name> [min_insts]

Prints each block with its MFMA / VALU / SALU / LDS / global counts and the branch targets, so
the loop bodies (backward branches) can be read off and weighted by their trip counts."""
import re
import sys
from collections import OrderedDict

path, name = sys.argv[1], sys.argv[2]
minn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
blocks = OrderedDict()
cur = "entry"
blocks[cur] = {"mfma": 0, "valu": 0, "salu": 0, "lds": 0, "gl": 0, "wait": 0, "br": [], "line": start}
for i in range(start + 1, len(lines)):
    l = lines[i].split(";")[0].strip()
    if l.startswith(".Lfunc_end"):
        break
    if not l:
        continue
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        cur = m.group(1)
        blocks[cur] = {"mfma": 0, "valu": 0, "salu": 0, "lds": 0, "gl": 0, "wait": 0, "br": [], "line": i + 1}
        continue
    if l.startswith("."):
        continue
    op = l.split()[0]
    b = blocks[cur]
    if op.startswith("v_mfma"):
        b["mfma"] += 1
    elif op.startswith("v_"):
        b["valu"] += 1
    elif op.startswith("ds_"):
        b["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        b["gl"] += 1
    elif op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        b["wait"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"):
        b["br"].append(l.split()[-1])
        b["salu"] += 1
    elif op.startswith("s_"):
        b["salu"] += 1
tot = {"mfma": 0, "valu": 0, "salu": 0, "lds": 0, "gl": 0}
order = list(blocks)
for k, b in blocks.items():
    n = b["mfma"] + b["valu"] + b["salu"] + b["lds"] + b["gl"]
    for t in tot:
        tot[t] += b[t]
    back = [t for t in b["br"] if t in blocks and order.index(t) <= order.index(k)]
    if n >= minn or back:
        print(f"{k:14s} L{b['line']:6d} mfma {b['mfma']:4d} valu {b['valu']:5d} salu {b['salu']:4d} lds {b['lds']:4d} gl {b['gl']:3d}"
              f"  br {','.join(b['br'])}{'  <-- back ' + ','.join(back) if back else ''}")
print("total", tot)
