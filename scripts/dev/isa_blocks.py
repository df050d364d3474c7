"""Per-basic-block instruction mix of one kernel in a hipcc -S listing
(dev tool: python scripts/dev/isa_blocks.py file.s kernel_symbol)."""
import re, sys
src, sym = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
blocks, cur = [], {"label": "entry", "line": start, "n": {}, "br": []}
for i in range(start + 1, end + 1):
    l = lines[i].strip()
    if re.match(r"^\.?LBB\w+:", l):
        blocks.append(cur); cur = {"label": l.split(":")[0], "line": i + 1, "n": {}, "br": []}; continue
    if not l or l.startswith((";", ".", "//")): continue
    op = l.split()[0]
    k = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(("s_load", "s_buffer", "s_waitcnt", "s_cbranch", "s_branch")) else
         "smem" if op.startswith(("s_load", "s_buffer")) else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else
         "lds" if op.startswith("ds_") else "br" if op.startswith(("s_cbranch", "s_branch")) else "wait" if op.startswith("s_waitcnt") else "other")
    cur["n"][k] = cur["n"].get(k, 0) + 1
    if k == "br" and len(l.split()) > 1: cur["br"].append(l.split()[1])
blocks.append(cur)
idx = {b["label"]: j for j, b in enumerate(blocks)}
tot = {}
for j, b in enumerate(blocks):
    back = [t for t in b["br"] if t in idx and idx[t] <= j]
    for k, v in b["n"].items(): tot[k] = tot.get(k, 0) + v
    print(f"{j:4d} {b['label']:>22s} L{b['line']:6d} valu {b['n'].get('valu',0):4d} salu {b['n'].get('salu',0):3d} "
          f"vmem {b['n'].get('vmem',0):2d} smem {b['n'].get('smem',0):2d} lds {b['n'].get('lds',0):2d}"
          + (f"  LOOP->{','.join(back)}" if back else ""))
print("total", tot)
