#!/usr/bin/env python3
"""Headline benchmark: Mrays/s and ms/frame of the breadth-first wide-BVH path
tracer at 1024x1024, 256 spp, 8 bounces (BASELINE.json metric), on N GPUs.

The headline workload is BASELINE.json configs[1]:
the diffuse Cornell box CBempty.dae.  The same JSON line carries the other
single-GPU configs of the metric (config 3: CBspheres, glass + mirror; config
4: CBbunny, 28,588 triangles, deep wide BVH, and the ~100k-triangle dragon
proxy of cuda-raytracer_amd/scenes.py) measured the same way in the same run,
under "configs".

A step is one full frame: every rank renders its interleaved 32x32 tiles of the
1024x1024 image at 256 spp (strong scaling: the frame is fixed, ranks split it),
then the framebuffer is gathered to rank 0 over RCCL and copied to the host
(ms/frame ends with the accumulated image on the host; one
rank: pt_get_image_async into a pinned buffer, more ranks: a non-blocking
copy of the gathered frame; either copy overlaps the next frame's rendering,
and the last frame's copy is waited for inside the timed region).  Timed
frames are queued with PT_FLAG_ASYNC: on the single-leaf scenes one frame's
path kernel runs while the previous frame's per-path results are summed
(same sums, same order); the wavefront scenes render synchronously.  Rays are
the rays traced (camera +
extension + shadow), counted on the device: SURVEY §8(d) counts the rays cast
through the traversal, so camera rays that pt_render resolves on the host
(pixels whose whole footprint misses the scene's root box: radiance 0, never
launched; pt_stats.culled_rays) are reported beside the value as
"culled_rays_per_frame", not in it.

BASELINE config 5 (the dragon proxy at 2048x2048, 1024 spp) runs tiled over
all ranks when n_gpus >= 8; on fewer GPUs the line carries it as single-GPU
measurements (the whole frame on one GPU, and one rank's 1/8 tile share),
labelled as such -- not a scaling figure.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts the N
ranks itself (a torch.distributed.run child process on 127.0.0.1, before
anything touches the GPU) and exits with its status; it refuses to start when
fewer than N GPUs are visible.  "n_gpus" is the world the gather ran over.

Rank 0 prints one JSON line.  "roofline" describes the workload's dominant
kernel, timed by HIP events attached to its dispatch packets in one extra,
instrumented frame (the headline frames run without events):
  * the level kernels (k_trace_real / k_trace_leaves / k_trace_level: BVH
    levels >= 1, HBM-bound): algorithmic bytes = 32 B per (ray, node) visit
    (4 B queue id + 28 B of ray) + 4 B per id they push;
    "line_frac" prices the same visits at the 128-B line a random record
    gather fetches;
  * k_shade_push (shading + the fused root pass): 96 B per shaded vertex +
    the root pass's share of the traversal bytes (40 B per ray entering the
    root + 4 B per id it pushes);
  * k_path_leaf (scenes whose BVH root is a leaf: each path runs to completion
    in registers, no HBM stream): VALU-bound, algorithmic FP32 FLOPs of the
    primitive tests (every primitive of the leaf per ray; an FMA counts 2, an
    add / mul / div / sqrt 1, compares and selects 0: 42 per ray-triangle
    test, 19 per ray-sphere test) against the 157.3 TFLOP/s vector peak (which
    also counts an FMA as 2); PMC VALU activity beside it when profiled.
Each workload also reports "ms_1spp" (one 1-spp frame, outside the timed
steps) and, under "trace", the traversal passes of a frame and ms per pass
(SURVEY §8(d)).  The stdout line stays compact (< 12 KB, compact_line: the
headline, its roofline and cpu_baseline, and per other workload its value,
ms/frame and roofline fraction); every workload's full record -- per-level
traces, notes, PMC sources -- goes to --detail-out, which the line names.
"traffic" is HBM bytes per launch from rocprofv3 PMC passes (FETCH_SIZE x 2 +
WRITE_SIZE, MI355X_MICROARCH.md) when a matching summary is committed under
profiles/ (scripts/pmc.sh, scripts/pmc_summary.py), else null.
cpu_baseline: the CPU oracle run through the Scotty3D PathTracer surface
(oracle/scotty_cpu.cpp over scotty::PathTracerT: 32x32-tile work queue,
std::thread::hardware_concurrency() workers, raytrace_tile -> raytrace_pixel;
pathtracer.cpp:183-213, 499-558) on a bounded sample of the headline frame's
tiles, on this host.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
VALU_PEAK_TFLOPS = 157.3    # MI355X FP32 vector peak, same guide
# FP32 FLOPs per primitive test (FMA = 2; trace.hip tri_test: N.d 5, N.o and
# the plane offset 6, the division 1, P = o + t d 6, three edge tests 8 each;
# sphere_test: o - c 3, b 5, c 6, disc 2, sqrt 1, the two roots 2)
FLOP_TRI, FLOP_SPHERE = 42, 19
# a cluster box (slab) test: 6 FMAs for the slab distances (compares free)
FLOP_BOX = 12
# the newest round's PMC summaries (scripts/profile_round.sh -> profiles/rNN/)
PMC_DIR = max((d for d in (ROOT / "profiles").glob("r[0-9][0-9]") if any(d.glob("pmc_*.json"))),
              default=ROOT / "profiles" / "r02")



def _ordinal(n):
    """2 -> '2nd', 11 -> '11th', 23 -> '23rd' (the CPU sample's tile stride)."""
    suf = "th" if 10 <= n % 100 <= 20 else {1: "st", 2: "nd", 3: "rd"}.get(n % 10, "th")
    return f"{n}{suf}"

def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scene", default="CBempty", help="headline scene (configs[1] = CBempty)")
    p.add_argument("--configs", default="CBspheres,CBbunny,bunny,dragon_proxy,dragon_proxy_gpubvh",
                   help="other single-GPU configs measured in the same run ('' = none)")
    p.add_argument("--width", type=int, default=1024)
    p.add_argument("--height", type=int, default=1024)
    p.add_argument("--spp", type=int, default=256)
    p.add_argument("--bounces", type=int, default=8)
    p.add_argument("--batch", type=int, default=0, help="paths in flight per batch (0 = auto)")
    p.add_argument("--tile", type=int, default=32)
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="target length of the CPU baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--seed", type=int, default=15618)
    p.add_argument("--config5", choices=["auto", "on", "off"], default="auto",
                   help="BASELINE config 5 (dragon proxy, 2048x2048, 1024 spp): tiled over all ranks when "
                        "n_gpus >= 8 (auto/on), else one GPU's whole frame and 1/8 tile share (on; auto at 1 GPU)")
    p.add_argument("--config5-size", default="2048x2048x1024",
                   help="WxHxSPP of config 5 (BASELINE: 2048x2048x1024; tests shrink it to run the 8-rank branch)")
    p.add_argument("--save-config5", default=None,
                   help="rank 0 saves config 5's gathered frame when it runs tiled over >= 8 ranks (.npy; tests)")
    p.add_argument("--no-1spp", action="store_true",
                   help="skip the ms_1spp frame (profiler runs: keeps per-launch averages to full frames)")
    p.add_argument("--no-executed", action="store_true",
                   help="skip the PT_FLAG_COUNT_TESTS frame of k_path_leaf workloads (profiler runs: its counting "
                        "kernel would join the profiled kernel's per-launch averages)")
    p.add_argument("--stats-in-timed", action="store_true",
                   help="record per-kernel HIP events inside the timed steps (default: one extra instrumented frame)")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="collective backend of the frame gather (nccl = RCCL over xGMI; gloo: tests only -- ranks "
                        "may share a GPU, device LOCAL_RANK %% device_count, the gather runs on host tensors)")
    p.add_argument("--force-gather", action="store_true",
                   help="tests: initialise the process group and gather the frame even at WORLD_SIZE=1 (runs "
                        "the nccl path -- local_sums_tensor on the device, dist.gather, index_copy_ -- on one GPU)")
    p.add_argument("--save-frame", default=None, help="rank 0 saves the last headline frame (.npy; tests)")
    p.add_argument("--detail-out", default="gpurun_out/bench_detail.json",
                   help="rank 0 writes every workload's full record (per-level traces, notes, PMC sources) here; "
                        "the stdout line stays compact and names this file ('' = none)")
    p.add_argument("--ref-arith", default="CBbunny",
                   help="workloads also measured with PT_FLAG_REF_ARITH, the reference kernels' literal "
                        "arithmetic ('' = none)")
    return p.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus(topology="/sys/class/kfd/kfd/topology/nodes", env=None):
    """GPUs this process may use, counted without touching the HIP runtime:
    KFD topology nodes with SIMDs (CPU nodes have simd_count 0), narrowed by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES."""
    env = os.environ if env is None else env
    n = 0
    for props in sorted(Path(topology).glob("*/properties")):
        try:
            kv = dict(l.split()[:2] for l in props.read_text().splitlines() if len(l.split()) >= 2)
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [s for s in v.split(",") if s.strip() != ""]
            n = min(n, len(ids))
    return n


def launch_ranks(args):
    """--gpus N > 1 without a torch.distributed launcher around us: start the
    N ranks as a child torch.distributed.run (one process per GPU) and return
    its exit status.  Nothing here touches the GPU or the HIP runtime (the
    GPUs are counted from the KFD topology in sysfs), so the ranks own their
    devices."""
    import subprocess
    n = visible_gpus()
    if n < args.gpus and args.backend == "nccl":
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {n}", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve()),
           *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def _cpu_share():
    """CPUs this process may use: affinity mask and cgroup quota (the GPU box
    shows the whole machine in nproc / hardware_concurrency)."""
    out = {}
    try:
        out["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        out["cgroup_quota_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return out


def usable_cpus():
    """(CPUs this process can actually run on: the affinity mask capped by the
    cgroup CPU quota, the share dict)."""
    sh = _cpu_share()
    n = sh.get("affinity") or os.cpu_count() or 1
    q = sh.get("cgroup_quota_cpus")
    if q:
        n = min(n, max(1, int(q)))
    return n, sh


def cpu_baseline(desc, args):
    """The oracle through the Scotty3D PathTracer surface on this host, one
    worker per usable CPU (affinity mask / cgroup quota; the GPU box's
    hardware_concurrency reports the whole machine): a bounded sample of the
    same frame (same spp and bounces, every k-th 32x32 tile), sized to about
    --cpu-seconds."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle
    ncpu, share = usable_cpus()
    ntiles = -(-args.width // 32) * -(-args.height // 32)
    cal = max(1, ntiles // 16)  # calibration: 1/16 of the tiles (at least one) at 4 spp
    _, rays, dt, thr = pyoracle.scotty_render(desc, args.width, args.height, 4, args.bounces, seed=args.seed,
                                              tile_stride=cal, threads=ncpu)
    full_s = dt * cal * args.spp / 4  # estimated seconds for the whole frame
    # the smallest tile stride whose share fits --cpu-seconds (a 10-30 s sample)
    stride = min(ntiles, max(1, int(-(-full_s // args.cpu_seconds))))
    _, rays, dt, thr = pyoracle.scotty_render(desc, args.width, args.height, args.spp, args.bounces,
                                              seed=args.seed, tile_stride=stride, threads=ncpu)
    nt = len(range(0, ntiles, stride))
    out = {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": thr, "kind": "port",
           "sample": f"{args.scene} {args.width}x{args.height}: {nt} of {ntiles} 32x32 tiles (every {_ordinal(stride)}), "
                     f"{args.spp} spp, {args.bounces} bounces, through the Scotty3D PathTracer surface "
                     f"({thr} worker threads = the usable CPUs); {rays} rays in {dt:.1f} s",
           "hardware_concurrency": os.cpu_count()}
    out.update(share)
    return out


def pmc_kernel(scene, kernel):
    """The committed PMC summary of `kernel` in `scene`'s profile, if any."""
    f = PMC_DIR / f"pmc_{scene}.json"
    if not f.exists():
        return None, None
    try:
        d = json.loads(f.read_text())
        return d["kernels"][kernel], f"{f.relative_to(ROOT)} ({d.get('config', '')})"
    except (KeyError, ValueError):
        return None, None


def pmc_traffic(scene, kernel):
    """HBM bytes per launch of `kernel` from a committed PMC summary, if any.
    kernel may be a tuple: the launch-weighted mean over those kernels (the
    level roofline covers k_trace_real, k_trace_leaves and k_trace_level)."""
    names = kernel if isinstance(kernel, tuple) else (kernel,)
    tot = n = 0
    src = None
    for kn in names:
        k, s = pmc_kernel(scene, kn)
        if not k or "hbm_bytes_per_launch" not in k:
            continue
        tot += k["hbm_bytes_per_launch"] * k.get("dispatches", 1)
        n += k.get("dispatches", 1)
        src = s
    return (int(tot / n), src) if n else (None, None)


# gfx950: 256 CUs x 4 SIMDs, 8 XCDs; a wave64 fp32 VALU instruction occupies
# its SIMD for 2 cycles (32 lanes per cycle: 157.3 TF = 1024 SIMDs x 2.4 GHz x
# 32 FMA x 2); GRBM_GUI_ACTIVE is summed over the 8 XCDs.
N_SIMD, N_XCD, VALU_CYCLES_PER_INST = 1024, 8, 2


def pmc_valu_busy(scene, kernel):
    """Fraction of SIMD cycles issuing VALU work during `kernel`'s launches
    (SQ_INSTS_VALU x 2 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)); transcendental
    and 64-bit ops take longer, so this is a lower bound.  kernel: a name or
    a tuple of names (summed)."""
    names = kernel if isinstance(kernel, tuple) else (kernel,)
    vi = ga = 0.0
    for kn in names:
        k, _ = pmc_kernel(scene, kn)
        if k and "SQ_INSTS_VALU" in k and "GRBM_GUI_ACTIVE" in k:
            vi += k["SQ_INSTS_VALU"]
            ga += k["GRBM_GUI_ACTIVE"]
    return round(vi * VALU_CYCLES_PER_INST / (N_SIMD * ga / N_XCD), 3) if ga else None


def root_leaf_flops(desc):
    """(flop per ray, prims) of the single-leaf test: every primitive of the root leaf."""
    import numpy as np
    import ctypes as C
    n = desc.nodes[0]
    if n.prim_count <= 0:
        return 0, 0
    q = np.ctypeslib.as_array(C.cast(desc.prims, C.POINTER(C.c_float)), shape=(desc.n_prims, 24))
    meta = q[n.prim_start:n.prim_start + n.prim_count, 3].view(np.uint32) >> 28
    import ptrace
    nsph = int((meta == ptrace.PT_PRIM_SPHERE).sum())
    ntri = n.prim_count - nsph
    return ntri * FLOP_TRI + nsph * FLOP_SPHERE, n.prim_count


def run_workload(name, args, ctx, rank, world, dev, dist, share=None, flags=0):
    """One workload (scene + args' frame shape) timed over args.steps frames.
    share=(r, n): render only tile share r of n on this one GPU (no gather);
    flags: extra render flags (PT_FLAG_REF_ARITH)."""
    import torch
    import ptrace
    import ptdist
    import scenes
    tb = time.perf_counter()
    scene = scenes.load(name)
    build_ms = (time.perf_counter() - tb) * 1e3  # scene assembly + BVH build (outside the timed frames)
    ctx.load_scene(scene)
    desc = scene.desc()

    # the frame lands in pinned host memory (one rank: pt_get_image; more: the
    # RCCL gather to rank 0, then rank 0's copy to the host)
    host = torch.empty((args.height, args.width, 4), dtype=torch.float32, pin_memory=True)
    t_rank, t_world = share if share else (rank, world)
    sums = [None]  # this rank's owned-pixel sums, reused frame to frame

    def frame(stats):
        ctx.clear()
        ctx.render(args.width, args.height, args.spp, max_bounces=args.bounces, seed=args.seed,
                   batch_paths=args.batch, tile_size=args.tile, rank=t_rank, nranks=t_world,
                   flags=flags | (ptrace.PT_FLAG_STATS if stats else ptrace.PT_FLAG_ASYNC))
        if world > 1 or args.force_gather:
            # RCCL gathers device tensors; gloo (tests) host tensors
            sdev = dev if args.backend == "nccl" else "cpu"
            sums[0] = ptdist.local_sums_tensor(ctx, sdev, out=sums[0])
            img = ptdist.gather_frame(sums[0], args.width, args.height, args.tile, args.spp)
            if img is not None:
                # (queued on torch's stream: overlaps the next frame's
                # rendering on the library's stream, like get_image_async)
                host.copy_(img, non_blocking=True)
        else:
            ctx.get_image_async(out=host)

    for _ in range(args.warmup):
        frame(False)
    ctx.reset_stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame(args.stats_in_timed)
    ctx.wait_image()  # (the last frame's image is on the host inside the timed region)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st0 = ctx.stats()  # device counters, no instrumentation needed
    # traced rays only: camera rays culled on the host never reach the GPU
    rays, culled = st0.rays - st0.culled_rays, st0.culled_rays
    instrumented_ms = None
    if not args.stats_in_timed:
        # per-kernel times of one more, instrumented frame (HIP events attached
        # to each dispatch packet); the timed frames above ran without them
        ctx.reset_stats()
        t1 = time.perf_counter()
        frame(True)
        ctx.wait_image()
        torch.cuda.synchronize()
        instrumented_ms = (time.perf_counter() - t1) * 1e3
    st = ctx.stats()
    # one 1-spp frame of the same workload (outside the timed
    # steps; this rank's tiles, no gather)
    ms_1spp = None
    if not args.no_1spp:
        ctx.clear()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ctx.render(args.width, args.height, 1, max_bounces=args.bounces, seed=args.seed, batch_paths=args.batch,
                   tile_size=args.tile, rank=t_rank, nranks=t_world, flags=flags)
        torch.cuda.synchronize()
        ms_1spp = (time.perf_counter() - t2) * 1e3
    lvl_ms = sum(st.ms_level[l] for l in range(1, 16))
    V = [st.level_visits[l] for l in range(16)]
    # 40 B per ray entering the root (record written at generation
    # + final hit word), 32 B per visit, 4 B per push.  The root pass runs inside
    # the producers (k_camera_push / k_shade_push): their share is 40 R + 4 B per
    # id pushed into the first queued level l0; the level kernels' share is
    # 32 B per visit + 4 B per id they push (into the levels below l0)
    l0 = next((l for l in range(1, 16) if V[l] > 0), 1)
    lvl_bytes = sum(32 * V[l] for l in range(1, 16)) + sum(4 * V[l] for l in range(l0 + 1, 16))
    traced = st.rays - st.culled_rays
    root_bytes = 40 * traced + 4 * V[l0]
    lvl_launches = sum(st.level_launches[l] for l in range(1, 16))
    flop_ray, _ = root_leaf_flops(desc)
    path_flops = flop_ray * traced
    if dist:
        rdev = dev if args.backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays, culled], dtype=torch.float64, device=rdev)
        dist.all_reduce(r)
        rays, culled = float(r[0].item()), float(r[1].item())
    save = getattr(args, "save_path", None) or (args.save_frame if name == args.scene else None)
    if save and rank == 0 and share is None and not flags:
        import numpy as np
        np.save(save, host.numpy())
    ms_step = elapsed / args.steps * 1e3
    if st.ms_path >= lvl_ms:
        kernel, launches = "k_path_leaf", st.path_launches
        ach = path_flops / (st.ms_path * 1e-3) / 1e12 if st.ms_path > 0 else 0.0
        traffic, src = pmc_traffic(name, kernel)
        roof = {"bound": "valu", "achieved": round(ach, 2), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / VALU_PEAK_TFLOPS, 4), "traffic": traffic, "kernel": kernel,
                "launches": int(launches), "avg_launch_us": round(st.ms_path * 1e3 / max(1, launches), 2),
                "flop_per_launch": int(path_flops / max(1, launches)),
                "valu_busy": pmc_valu_busy(name, kernel),
                "note": "single-leaf BVH: paths run to completion in registers; FP32 VALU, not HBM, bounds it; "
                        "achieved counts the reference's intersection work per ray (every leaf primitive, FMA = 2; "
                        "the kernel's candidate clusters execute only part of it, DESIGN.md §3/§4), valu_busy (PMC) "
                        "is the share of SIMD cycles issuing any VALU instruction (shading, NEE, RNG included)"}
    else:
        kernel, launches = "k_trace_level", lvl_launches
        ach = (lvl_bytes / (lvl_ms * 1e-3) / 1e9) if lvl_ms > 0 else 0.0
        lk = ("k_trace_level", "k_trace_real", "k_trace_leaves")
        traffic, src = pmc_traffic(name, lk)
        avg_s = lvl_ms * 1e-3 / max(1, launches)
        # the same visits priced at the hardware's fetch granularity: a random
        # 32-B record gather is one 128-B DRAM line (scripts/cal/gather_cal.hip)
        line_bytes = sum(132 * V[l] for l in range(1, 16)) + sum(4 * V[l] for l in range(2, 16))
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": "k_trace_real+k_trace_leaves+k_trace_level",
                "launches": int(launches), "avg_launch_us": round(avg_s * 1e6, 2),
                "bytes_per_launch": int(lvl_bytes / max(1, launches)), "valu_busy": pmc_valu_busy(name, lk),
                "traffic_gbs": round(traffic / avg_s / 1e9, 1) if traffic and avg_s > 0 else None,
                "line_bytes_per_launch": int(line_bytes / max(1, launches)),
                "line_frac": round(line_bytes / max(lvl_ms * 1e-3, 1e-12) / 1e9 / HBM_PEAK_GBS, 4),
                "note": "achieved/frac: SURVEY 8(d)'s 32 B per visit + 4 B per push; line_frac: the same visits at "
                        "the 128-B line a random record gather fetches; traffic_gbs: PMC HBM bytes per launch / "
                        "average launch time"}
    if kernel == "k_path_leaf" and not flags and not args.no_executed:
        # the work the kernel executes: one more frame
        # through the counting build (PT_FLAG_COUNT_TESTS, not timed: the
        # counters cost it time), priced like the reference's work -- 42 flop
        # per triangle candidate tested (an upper bound: a shadow candidate the
        # division-free pre-test rejects does less), 19 per sphere, 12 per
        # cluster box test (a slab test's 6 FMAs; the shadow rays' box-overlap
        # tests do compares only) -- over the same launch time as `achieved`
        ctx.reset_stats()
        ctx.clear()
        ctx.render(args.width, args.height, args.spp, max_bounces=args.bounces, seed=args.seed,
                   batch_paths=args.batch, tile_size=args.tile, rank=t_rank, nranks=t_world,
                   flags=ptrace.PT_FLAG_COUNT_TESTS)
        sc = ctx.stats()
        ntest = sc.prim_tests_tri + sc.prim_tests_sph
        if ntest > 0 and st.ms_path > 0:
            ex = FLOP_TRI * sc.prim_tests_tri + FLOP_SPHERE * sc.prim_tests_sph + FLOP_BOX * sc.cluster_box_tests
            exa = ex / (st.ms_path * 1e-3) / 1e12
            roof.update({"executed_flop": int(ex / max(1, launches)), "executed_achieved": round(exa, 2),
                         "executed_frac": round(exa / VALU_PEAK_TFLOPS, 4),
                         "executed_tests_per_ray": round(ntest / max(1, traced), 3),
                         "leaf_tests_per_ray": int(desc.nodes[0].prim_count),
                         "box_tests_per_ray": round(sc.cluster_box_tests / max(1, traced), 3)})
            roof["note"] += ("; executed_*: the tests the kernel actually ran (PT_FLAG_COUNT_TESTS frame), "
                             "42 flop per triangle candidate, 19 per sphere, 12 per cluster box test")
    if src:
        roof["traffic_source"] = src
    others = []
    if st.shade_launches > 0:
        # shading with the fused root pass: 96 B per shaded path
        # vertex (hit 8 + path state 44 read + 44 write) + the root pass's share
        # of the traversal bytes (root_bytes above)
        sbytes = 96 * st.shaded + root_bytes
        ach = sbytes / (st.ms_shade_push * 1e-3) / 1e9 if st.ms_shade_push > 0 else 0.0
        straffic, ssrc = pmc_traffic(name, "k_shade_push")
        sroof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": straffic, "kernel": "k_shade_push",
                 "launches": int(st.shade_launches),
                 "avg_launch_us": round(st.ms_shade_push * 1e3 / max(1, st.shade_launches), 2),
                 "bytes_per_launch": int(sbytes / max(1, st.shade_launches)), "shaded_vertices": int(st.shaded),
                 "valu_busy": pmc_valu_busy(name, "k_shade_push")}
        sroof["note"] = ("96 B per shaded vertex + the fused root pass's traversal share (40 B per ray "
                         "entering the root + 4 B per id it pushes); the first fill's camera rays (k_camera_push, "
                         "<= 2 % of the rays) are counted here too")
        savg = st.ms_shade_push * 1e-3 / max(1, st.shade_launches)
        sroof["traffic_gbs"] = round(straffic / savg / 1e9, 1) if straffic and savg > 0 else None
        if ssrc:
            sroof["traffic_source"] = ssrc
        if st.ms_shade_push > lvl_ms:  # the dominant kernel first
            roof, sroof = sroof, roof
        others.append(sroof)
    out = {
        "scene": name,
        "value": round(rays / elapsed / 1e6, 2),
        "ms_per_frame": round(ms_step, 2),
        "rays_per_frame": int(rays / args.steps),
        "culled_rays_per_frame": int(culled / args.steps),
        "batch_paths": st.batch_paths,
        "scene_build_ms": round(build_ms, 1),
        "bvh": {"nodes": int(desc.n_nodes), "levels": int(desc.n_levels), "prims": int(desc.n_prims),
                "gpu_build_ms": round(getattr(scene, "build_ms", 0.0), 2) or None},
        "roofline": roof,
        "roofline_other": others,
        "ms_1spp": None if ms_1spp is None else round(ms_1spp, 2),
        "trace": {"visits_per_ray": round(st.visits / max(1, traced), 2),
                  "instrumented_frame_ms": None if instrumented_ms is None else round(instrumented_ms, 2),
                  "passes": int(st.passes),
                  "ms_per_pass": None if instrumented_ms is None else round(instrumented_ms / max(1, st.passes), 3),
                  "ms_path": round(st.ms_path, 1), "ms_trace": round(st.ms_trace, 1),
                  "ms_shade": round(st.ms_shade, 1), "ms_shade_push": round(st.ms_shade_push, 1),
                  "ms_root": round(st.ms_root, 1),
                  "ms_scan": round(st.ms_scan, 1), "ms_levels": round(lvl_ms, 1),
                  "levels": [{"level": l, "ms": round(st.ms_level[l], 2), "visits": int(st.level_visits[l]),
                              "leaf_visits": int(st.level_leaf_visits[l]), "items": int(st.level_items[l]),
                              "scan_ms": round(st.ms_scan_level[l], 2),
                              "Gvisits_per_s": round(st.level_visits[l] / max(st.ms_level[l], 1e-9) / 1e6, 2)}
                             for l in range(1, st.n_levels) if st.level_launches[l] > 0]},
    }
    return out, scene


LINE_MAX = 12000  # the driver parses the stdout line; keep it well under its limit
_ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "launches", "avg_launch_us",
              "flop_per_launch", "bytes_per_launch", "valu_busy", "traffic_gbs", "line_frac", "executed_flop",
              "executed_frac", "executed_tests_per_ray")


def _short_roof(r, keys=_ROOF_KEYS):
    return {k: r[k] for k in keys if k in r and r[k] is not None} if r else None


def detail_record(head, others, cpu, args, world):
    """Everything a workload measured (per-level traces, notes, PMC sources):
    written to --detail-out, referenced from the stdout line."""
    return {"argv": sys.argv[1:], "n_gpus": world, "headline": head, "configs": others, "cpu_baseline": cpu}


def compact_line(head, others, cpu, args, world, detail_path=None):
    """The one JSON line rank 0 prints (the driver's contract): the headline
    fields, its roofline and cpu_baseline, and each other workload as
    {scene, value, ms_per_frame, roofline: {kernel, frac, achieved, traffic}}.
    Everything else goes to the detail file.  Bounded by LINE_MAX."""
    configs = []
    for o in others:
        r = o.get("roofline") or {}
        c = {"scene": o["scene"], "value": o["value"], "ms_per_frame": o["ms_per_frame"],
             "culled_rays_per_frame": o["culled_rays_per_frame"],
             "roofline": {k: r.get(k) for k in ("kernel", "frac", "achieved", "traffic")}}
        if o.get("config"):
            c["config"] = o["config"]
        ro = (o.get("roofline_other") or [None])[0]
        if ro:
            c["roofline_other"] = {k: ro.get(k) for k in ("kernel", "frac", "achieved", "traffic")}
        configs.append(c)
    tr = head.get("trace") or {}
    out = {
        "metric": f"Mrays/sec at {args.width}x{args.height}, {args.spp} spp, {args.bounces} bounces",
        "value": head["value"],
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_frame"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic rays (Philox seed {args.seed}) on scene {args.scene} (reference media, flattened fixture)",
        "config": {"workload": f"{args.scene} {args.width}x{args.height} {args.spp}spp {args.bounces} bounces",
                   "scene": args.scene, "width": args.width, "height": args.height, "spp": args.spp,
                   "max_bounces": args.bounces, "batch_paths": head["batch_paths"],
                   "parallelism": f"tiles{args.tile}x{world}"},
        "ms_per_frame": head["ms_per_frame"],
        "ms_1spp": head.get("ms_1spp"),
        "rays_per_frame": head["rays_per_frame"],
        "culled_rays_per_frame": head["culled_rays_per_frame"],
        "roofline": _short_roof(head["roofline"]),
        "roofline_other": [_short_roof(r) for r in head.get("roofline_other") or []],
        "trace": {k: tr.get(k) for k in ("visits_per_ray", "passes", "ms_per_pass", "ms_path", "ms_levels",
                                         "ms_shade_push") if k in tr},
        "configs": configs,
    }
    if cpu is not None:
        out["cpu_baseline"] = {k: cpu[k] for k in ("value", "unit", "cores", "kind", "sample") if k in cpu}
    if detail_path:
        out["detail"] = str(detail_path)
    line = json.dumps(out, separators=(",", ":"))
    if len(line) > LINE_MAX:  # never print a line the driver cannot take: drop the extras first
        for k in ("trace", "roofline_other", "ms_1spp"):
            out.pop(k, None)
        for c in out["configs"]:
            c.pop("roofline_other", None)
            c.pop("config", None)
        line = json.dumps(out, separators=(",", ":"))
    return line


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import ptrace
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the world", file=sys.stderr)
    dist = None
    # one GPU per rank (gloo test runs may put several ranks on one GPU)
    gpu = local if args.backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    if world > 1 or args.force_gather:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
        world = dist.get_world_size()
    dev = torch.device("cuda", gpu)
    ctx = ptrace.Context(gpu)

    head, head_scene = run_workload(args.scene, args, ctx, rank, world, dev, dist)
    others = []
    for name in [s for s in args.configs.split(",") if s not in ("", "none", '""') and s != args.scene]:
        o, _ = run_workload(name, args, ctx, rank, world, dev, dist)
        o["config"] = f"{args.width}x{args.height} {args.spp}spp {args.bounces} bounces"
        others.append(o)
    # the cost of reference parity: the same frame with PT_FLAG_REF_ARITH, the
    # reference kernels' literal arithmetic (triangles with diffuse / mirror /
    # emission BSDFs only)
    for name in [s for s in args.ref_arith.split(",") if s not in ("", "none", '""')]:
        o, _ = run_workload(name, args, ctx, rank, world, dev, dist, flags=ptrace.PT_FLAG_REF_ARITH)
        o["config"] = f"{args.width}x{args.height} {args.spp}spp {args.bounces} bounces, PT_FLAG_REF_ARITH"
        o["flags"] = "PT_FLAG_REF_ARITH"
        others.append(o)
    import copy
    a5 = copy.copy(args)
    a5.width, a5.height, a5.spp = (int(v) for v in args.config5_size.lower().split("x"))
    a5.save_path = args.save_config5
    if world >= 8 and args.config5 in ("auto", "on"):
        # BASELINE config 5: the dragon proxy at 2048x2048, 1024 spp, the
        # framebuffer tiled over all ranks and gathered over RCCL
        a5.steps, a5.warmup = 1, 1
        o, _ = run_workload("dragon_proxy", a5, ctx, rank, world, dev, dist)
        o["config"] = (f"config 5: {a5.width}x{a5.height} {a5.spp}spp {a5.bounces} bounces, tiles over all ranks "
                       f"+ {'RCCL' if args.backend == 'nccl' else args.backend} gather")
        others.append(o)
    elif world == 1 and (args.config5 == "on" or (args.config5 == "auto" and args.configs)):
        # config 5's workload on ONE GPU (not a scaling figure): one rank's
        # share of the 8-GPU tiling (every 8th 32x32 tile), then the whole frame
        a5.steps, a5.warmup, a5.save_path = 1, 1, None
        o, _ = run_workload("dragon_proxy", a5, ctx, 0, 1, dev, None, share=(0, 8))
        o["config"] = (f"config 5 workload, single GPU: rank 0's 1/8 tile share of {a5.width}x{a5.height} "
                       f"{a5.spp}spp {a5.bounces} bounces (the per-GPU work of the 8-GPU run, no gather)")
        others.append(o)
        a5.warmup, a5.save_path = 0, args.save_config5
        o, _ = run_workload("dragon_proxy", a5, ctx, 0, 1, dev, None)
        o["config"] = (f"config 5 workload, single GPU: the whole {a5.width}x{a5.height} {a5.spp}spp "
                       f"{a5.bounces}-bounce frame on one MI355X")
        others.append(o)
    if rank == 0:
        cpu = cpu_baseline(head_scene.desc(), args) if world == 1 and not args.no_cpu else None
        detail = detail_record(head, others, cpu, args, world)
        line = compact_line(head, others, cpu, args, world, detail_path=args.detail_out)
        if args.detail_out:
            p = Path(args.detail_out)
            p.parent.mkdir(parents=True, exist_ok=True)
            p.write_text(json.dumps(detail, indent=1) + "\n")
        print(line, flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
