#!/usr/bin/env python3
"""Copy one round's GPU profile outputs into profiles/<round>/ (run locally
after scripts/profile_round.sh came back in gpurun_out/):

  python scripts/collect_profiles.py r02

* bench_default.json                      the bench line (gpurun_out/bench.log)
* bench_detail.json                       its detail side file (gpurun_out/bench_detail.json)
* rocprof_kernel_stats_<scene>.csv        rocprofv3 --stats of one frame per workload
* detail_<scene>.json                     that run's bench detail file (per-level visits)
* pmc_<scene>.json                        per-kernel PMC totals (scripts/pmc_summary.py)
"""
import glob
import json
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "gpurun_out"


def main():
    rnd = sys.argv[1]
    dst = ROOT / "profiles" / rnd
    dst.mkdir(parents=True, exist_ok=True)
    log = OUT / "bench.log"
    if log.exists():
        line = [x for x in log.read_text().splitlines() if x.startswith("{")]
        if line:
            rec = json.loads(line[-1])
            det = OUT / "bench_detail.json"
            if det.exists():  # the line's side file travels with it
                shutil.copy(det, dst / "bench_detail.json")
                rec["detail"] = f"profiles/{rnd}/bench_detail.json"
            (dst / "bench_default.json").write_text(json.dumps(rec, indent=1) + "\n")
    for d in sorted(OUT.glob("prof_*")):
        if not d.is_dir():
            continue
        sc = d.name[len("prof_"):]
        stats = glob.glob(str(d / "**" / "*kernel_stats.csv"), recursive=True)
        if stats:
            shutil.copy(stats[0], dst / f"rocprof_kernel_stats_{sc}.csv")
        det = OUT / f"prof_{sc}.detail.json"  # (that run's per-level visits: scripts/dev/level_table.py)
        if det.exists():
            shutil.copy(det, dst / f"detail_{sc}.json")
    scenes = sorted({p.name[len("pmc_"):].rsplit("_", 1)[0] for p in OUT.glob("pmc_*") if p.is_dir()})
    for sc in scenes:
        files = sorted(glob.glob(str(OUT / f"pmc_{sc}_[0-9]*" / "**" / "*counter_collection.csv"), recursive=True))
        if not files:
            continue
        cfg = f"{sc} 1024x1024 256spp 8 bounces, bench.py --scene {sc} --configs none --config5 off --steps 1 " \
              f"--warmup 0 --no-cpu --no-1spp --ref-arith none (2 frames)"
        subprocess.run([sys.executable, str(ROOT / "scripts" / "pmc_summary.py"), *files, "--json",
                        str(dst / f"pmc_{sc}.json"), "--config", cfg], check=True, stdout=subprocess.DEVNULL)
        print("pmc", sc, len(files), "passes")


if __name__ == "__main__":
    main()
