#!/usr/bin/env python3
"""Copy one round's final GPU evidence (scripts/r03_final_a.sh, r03_final_b.sh) from gpurun_out/
into profiles/: bench JSON lines, the GPU suite / smoke logs, rocprofv3 kernel-trace summaries,
the PMC HBM traffic records (already stamped with the source hash on the box), the det kernel's
SQ counters and the EnKF256 MFMA counters.
    python scripts/collect_round.py r03z
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
O = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")
F64_MFMA_PEAK_TFLOPS = 78.6            # MI355X_MICROARCH.md, dense f64 matrix


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def short(kernel_name):
    """Kernel name without the anonymous namespace and the parameter list."""
    return kernel_name.replace("(anonymous namespace)::", "").split("(")[0]


def counters(name, match):
    """{counter: [per-dispatch value]} for kernels whose name contains `match`, and the kernel
    names (one PMC pass serialises dispatches: values are per dispatch)."""
    tot, names = {}, {}
    for f in glob.glob(os.path.join(O, name, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match not in r["Kernel_Name"]:
                continue
            k = short(r["Kernel_Name"])
            key = (k, r["Counter_Name"], r["Dispatch_Id"])
            tot[key] = tot.get(key, 0.0) + float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = k
    out = {}
    for (k, c, _), v in tot.items():
        out.setdefault(k, {}).setdefault(c, []).append(v)
    return out


def durations(name):
    """{kernel: [duration ns]} from the pass's kernel trace."""
    out = {}
    for f in glob.glob(os.path.join(O, name, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            out.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def sq(tag):
    c = {}
    for i in (1, 2, 3):
        for k, cs in counters(f"{tag}_pmc_det_sq{i}", "wavefront_flow").items():
            for n, v in cs.items():
                c[n] = sum(v) / len(v)
    wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    rec = {"kernel": "wavefront_flow (Texas det, bench --steps 1 --warmup 0)",
           "counters": c,
           "ratios": {"wait_any/wave_cycles": c.get("SQ_WAIT_ANY", 0) / wc,
                      "wait_inst_any/wave_cycles": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                      "active_inst_any/wave_cycles": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                      "active_valu/wave_cycles": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                      "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1)},
           "note": "per dispatch average; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count "
                   "quad-cycles (MI355X_MICROARCH.md): the ratios are unit-free"}
    json.dump(rec, open(os.path.join(P, f"{tag}_det_sq_counters.json"), "w"), indent=1)


def mfma(tag):
    name = f"{tag}_pmc_enkf256_mfma"
    cs = counters(name, "")
    du = durations(name)
    rec = {"command": "rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES "
                      "SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE -- python3 bench.py --members "
                      "256 --enkf --steps 1 --warmup 0 --no-cpu --no-api --timing-runs 1",
           "notes": "per dispatch (the PMC pass serialises dispatches); flops = "
                    "SQ_INSTS_VALU_MFMA_MOPS_F64 x 512; GRBM_GUI_ACTIVE is summed over the 8 XCDs, "
                    "so mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); "
                    f"f64 MFMA dense peak {F64_MFMA_PEAK_TFLOPS} TFLOP/s",
           "kernels": {}}
    for k, c in cs.items():
        mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64")
        if not mops or sum(mops) == 0:
            continue
        n = len(mops)
        flops = sum(mops) / n * 512
        us = sum(du.get(k, [0])) / max(len(du.get(k, [])), 1) / 1e3
        busy = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0])) / n
        gui = sum(c.get("GRBM_GUI_ACTIVE", [0])) / n
        rec["kernels"][k] = {
            "dispatches": n, "flops_per_dispatch": flops, "avg_us": us,
            "tflops": flops / (us * 1e-6) / 1e12 if us else None,
            "frac_of_f64_mfma_peak": flops / (us * 1e-6) / 1e12 / F64_MFMA_PEAK_TFLOPS if us else None,
            "mfma_busy": busy / (gui / 8 * 1024) if gui else None}
    json.dump(rec, open(os.path.join(P, f"{tag}_enkf256_mfma.json"), "w"), indent=1)


def main():
    tag = sys.argv[1]
    for f in sorted(glob.glob(os.path.join(O, f"{tag}_bench_*.json"))):
        json.dump(last_json(f), open(os.path.join(P, os.path.basename(f)), "w"), indent=1)
    for f in (f"{tag}_pytest_gpu.txt", f"{tag}_smoke.log"):
        if os.path.exists(os.path.join(O, f)):
            shutil.copy(os.path.join(O, f), os.path.join(P, f))
    for f in (f"{tag}_subbasins.json",):
        if os.path.exists(os.path.join(O, f)):
            json.dump(last_json(os.path.join(O, f)), open(os.path.join(P, f), "w"), indent=1)
    for src in glob.glob(os.path.join(O, f"{tag}_prof_*", "run_kernel_stats.csv")):
        name = os.path.basename(os.path.dirname(src))[len(f"{tag}_prof_"):]
        shutil.copy(src, os.path.join(P, f"{tag}_{name}_kernel_stats.csv"))
    for src in glob.glob(os.path.join(O, f"{tag}_profiles", "*.json")):
        shutil.copy(src, os.path.join(P, os.path.basename(src)))
    if glob.glob(os.path.join(O, f"{tag}_pmc_det_sq1")):
        sq(tag)
    if glob.glob(os.path.join(O, f"{tag}_pmc_enkf256_mfma")):
        mfma(tag)


if __name__ == "__main__":
    main()
