"""Static instruction mix of one kernel by source region (dev tool).

  hipcc ... -g -S -o k.s ; python scripts/dev/isa_regions.py k.s <kernel symbol>

Each instruction is attributed to the innermost source function of its
`.loc` line (kernels/*.hip, *.h); functions are grouped into regions
(intersection, rng, camera, nee, shading, bookkeeping).  Loops (backward
branches) are listed with their own mix, so a per-ray budget can be formed
as loop body x trip count."""
import re
import sys
from collections import defaultdict
from pathlib import Path

src, sym = sys.argv[1], sys.argv[2]
lines = Path(src).read_text().split("\n")
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
    if m:
        d = Path(m.group(2))
        if not d.is_absolute() and 0 in files:  # (relative to the compilation directory, file 0's)
            d = Path(files[0]).parent.parent.parent / d if files[0].endswith(".hip") else d
        files[int(m.group(1))] = str(d / m.group(3))

# function line ranges of the kernel sources
FUNC_RE = re.compile(r'^(?:template\s*<[^>]*>\s*)?(?:__device__|__global__|static|inline|constexpr)[^;{(]*?\b([A-Za-z_]\w*)\s*\(')
ranges = {}
for fid, path in files.items():
    if not Path(path).exists() or "repo" not in path:
        continue
    text = Path(path).read_text().split("\n")
    cur, out = "<file>", []
    for i, l in enumerate(text, 1):
        m = FUNC_RE.match(l)
        if m:
            cur = m.group(1)
        out.append(cur)
    ranges[fid] = out

REGION = {
    "intersection": ["fdot", "bw_plane", "bw_test", "bw_test2", "bw_plane2", "tri_test", "tri_test2", "tri_test_ref",
                     "edge_ref", "sphere_test", "plane_nd", "tri_outside", "leaf_closest", "leaf_occluded", "load_prim",
                     "prim_sphere", "take_hit", "box_hit", "fdot2", "fma2"],
    "rng": ["philox", "philox_round", "rng", "rng_nee2", "u01", "mulhilo", "mad64", "philox10"],
    "camera": ["camera_dir", "camera_dir_ref"],
    "rootpass": ["root_pass", "push_children", "push_ray", "count_rays", "wave_sum"],
    "slots": ["shade_slot", "wave_hist_rank", "wave_key_rank", "claim_block", "block_range", "path_pixel", "put_res"],
    "nee": ["nee_sample", "light_of", "light_sample"],
    "shading": ["shade_vertex", "normalize", "cross", "dot", "length", "sincos2pi", "mulv", "xyz", "mk", "ld3"],
}
fn2reg = {f: r for r, fs in REGION.items() for f in fs}

start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
loc = (0, 0)
insts = []  # (index, kind, region, fn)
labels = {}
for i in range(start + 1, end + 1):
    l = lines[i].strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = (int(m.group(1)), int(m.group(2)))
        continue
    m = re.match(r"^(\.?LBB\w+):", l)
    if m:
        labels[m.group(1)] = len(insts)
        continue
    if not l or l.startswith((";", ".", "//")):
        continue
    op = l.split()[0]
    kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(
        ("s_load", "s_buffer", "s_waitcnt", "s_cbranch", "s_branch", "s_nop")) else
            "smem" if op.startswith(("s_load", "s_buffer")) else
            "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else
            "lds" if op.startswith("ds_") else "br" if op.startswith(("s_cbranch", "s_branch")) else "other")
    fid, ln = loc
    fn = ranges.get(fid, [])[ln - 1] if fid in ranges and 0 < ln <= len(ranges[fid]) else "?"
    insts.append((kind, fn2reg.get(fn, "bookkeeping"), fn, l))

tot = defaultdict(lambda: defaultdict(int))
for kind, reg, fn, _ in insts:
    tot[reg][kind] += 1
print("static mix by region:")
for reg, d in sorted(tot.items()):
    print(f"  {reg:14s} " + " ".join(f"{k} {v:5d}" for k, v in sorted(d.items())))
# loops: backward branches
print("loops (backward branches):")
for j, (kind, reg, fn, l) in enumerate(insts):
    if kind != "br":
        continue
    parts = l.split()
    if len(parts) < 2 or parts[1] not in labels:
        continue
    tgt = labels[parts[1]]
    if tgt > j:
        continue
    body = insts[tgt:j + 1]
    d = defaultdict(int)
    regs = defaultdict(int)
    for k2, r2, f2, _ in body:
        d[k2] += 1
        if k2 == "valu":
            regs[r2] += 1
    print(f"  [{tgt:5d}..{j:5d}] " + " ".join(f"{k} {v}" for k, v in sorted(d.items())) +
          "  valu by region: " + ", ".join(f"{r} {v}" for r, v in sorted(regs.items(), key=lambda x: -x[1])))
if len(sys.argv) > 3:
    fnv = defaultdict(int)
    for kind, reg, fn, _ in insts:
        if kind == "valu" and reg == sys.argv[3]:
            fnv[fn] += 1
    print(sys.argv[3], "valu by function:", sorted(fnv.items(), key=lambda x: -x[1])[:20])
