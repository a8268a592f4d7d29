#!/usr/bin/env python3
"""Wave-time breakdown of every kernel in rocprofv3 --pmc passes (scripts/gpu_pmc.sh output):
parked at s_waitcnt / barrier (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY), issuing
(SQ_ACTIVE_INST_ANY; of which VALU / LDS), as fractions of SQ_WAVE_CYCLES summed over the
kernel's dispatches (all quad-cycle counters, so the ratios are unit-free).
    python scripts/sq_breakdown.py gpurun_out/<tag>_p1 [more pass dirs ...]
"""
import csv
import glob
import os
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")


def main(dirs):
    tot = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                c = tot.setdefault(k, {})
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if not wc:
            continue
        f = lambda n: c.get(n, 0.0) / wc                      # noqa: E731
        print(f"{k[:58]:58s} waves {c.get('SQ_WAVES', 0):9.0f} wave_qcyc {wc:9.3e} "
              f"parked {f('SQ_WAIT_ANY'):.2f} stall {f('SQ_WAIT_INST_ANY'):.2f} "
              f"issue {f('SQ_ACTIVE_INST_ANY'):.2f} (valu {f('SQ_ACTIVE_INST_VALU'):.2f} "
              f"lds {f('SQ_ACTIVE_INST_LDS'):.2f}) insts_valu {c.get('SQ_INSTS_VALU', 0):.3e}")


if __name__ == "__main__":
    main(sys.argv[1:])
