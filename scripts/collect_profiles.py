#!/usr/bin/env python3
"""Copy one round's GPU results from gpurun_out/ into profiles/ (the committed evidence):
bench JSON lines (scripts/bench_round.sh), rocprofv3 kernel-trace summaries
(scripts/profile_round.sh, scripts/ens_profiles.sh), HBM traffic from the PMC passes
(scripts/hbm_traffic.py) and the det kernel's SQ timing counters.
    python scripts/collect_profiles.py <tag>
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def traffic(tag, fetch, write, line):
    c = line["config"]
    args = [fetch, write, tag, c["slots"], c["tile"], c["n_reaches"], c["T"]]
    if c["members_per_gpu"] > 1:
        args.append(c["members_per_gpu"])
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "hbm_traffic.py")] +
                   [str(a) for a in args], check=True, cwd=ROOT)


def sq_counters(tag):
    tot, names = {}, set()
    for f in glob.glob(os.path.join(O, f"{tag}_sq_p*", "**", "*counter_collection.csv"),
                       recursive=True):
        for r in csv.DictReader(open(f)):
            if "wavefront_flow" not in r["Kernel_Name"]:
                continue
            names.add(r["Kernel_Name"])
            key = (r["Counter_Name"], r["Dispatch_Id"])
            tot[key] = tot.get(key, 0.0) + float(r["Counter_Value"])
    per = {}
    for (name, _), v in tot.items():
        per.setdefault(name, []).append(v)
    c = {k: sum(v) / len(v) for k, v in sorted(per.items())}
    wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    rec = {"kernel": sorted(names), "workload": "Texas det, bench --steps 1; per dispatch average",
           "counters": c,
           "ratios": {"wait_any/wave_cycles": c.get("SQ_WAIT_ANY", 0) / wc,
                      "wait_inst_any/wave_cycles": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                      "active_inst_any/wave_cycles": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                      "active_valu/wave_cycles": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                      "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1)},
           "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles "
                   "(MI355X_MICROARCH.md); ratios are unit-free"}
    json.dump(rec, open(os.path.join(P, f"{tag}_det_sq_counters.json"), "w"), indent=1)


def main():
    tag = sys.argv[1]
    lines = {}
    for f in sorted(glob.glob(os.path.join(O, f"bench_{tag}_*.log"))):
        name = os.path.basename(f)[len(f"bench_{tag}_"):-4]
        lines[name] = last_json(f)
        json.dump(lines[name], open(os.path.join(P, f"{tag}_bench_{name}.json"), "w"), indent=1)
    for name in ("det", "ens64", "enkf32", "enkf256", "kf"):
        src = os.path.join(O, f"prof_{name}", "run_kernel_stats.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(P, f"{tag}_{name}_kernel_stats.csv"))
    src = os.path.join(O, f"prof_{tag}_conus", "run_kernel_stats.csv")
    if os.path.exists(src):
        shutil.copy(src, os.path.join(P, f"{tag}_conus_kernel_stats.csv"))
    if "det" in lines and os.path.isdir(os.path.join(O, f"{tag}_hbm_p1")):
        traffic(tag, os.path.join(O, f"{tag}_hbm_p1"), os.path.join(O, f"{tag}_hbm_p2"),
                lines["det"])
    for name, key in (("ens64", "ens64"), ("conus", "conus")):
        if name in lines and os.path.isdir(os.path.join(O, f"{tag}_{key}_fetch")):
            traffic(tag, os.path.join(O, f"{tag}_{key}_fetch"),
                    os.path.join(O, f"{tag}_{key}_write"), lines[name])
    if glob.glob(os.path.join(O, f"{tag}_sq_p*")):
        sq_counters(tag)
    # the bench lines ran before this round's PMC passes: annotate them with the traffic measured
    # for the same workload in the same session (as bench.py reports it on later runs)
    for name, suffix in (("det", ""), ("ens64", "_ens64"), ("conus", "_ens16")):
        tf = os.path.join(P, f"{tag}_hbm_traffic{suffix}.json")
        if name not in lines or not os.path.exists(tf):
            continue
        rec, line = json.load(open(tf)), lines[name]
        roof = line["roofline"]
        roof["traffic"] = rec["traffic_bytes_per_launch"]
        roof["traffic_source"] = os.path.relpath(tf, ROOT)
        roof["traffic_gbs"] = round(rec["traffic_bytes_per_launch"] / (roof["avg_launch_us"] * 1e-6)
                                    / 1e9, 3)
        json.dump(line, open(os.path.join(P, f"{tag}_bench_{name}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
