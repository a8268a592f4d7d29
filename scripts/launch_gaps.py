#!/usr/bin/env python3
"""Diagnostic: durations of the last `count` launches of a kernel and the idle gaps between them,
from a rocprofv3 --kernel-trace CSV.
    python scripts/launch_gaps.py <run_kernel_trace.csv> <kernel-name substring> <count>
"""
import csv
import sys


def main():
    path, name, count = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows][-count:]
    gaps = [(t[i][0] - t[i - 1][1]) / 1e3 for i in range(1, len(t))]
    durs = [(b - a) / 1e3 for a, b in t]
    print("durations us:", [round(x) for x in durs])
    print("gaps us:", [round(x, 1) for x in gaps])
    print("sum gaps", round(sum(gaps), 1), "sum durations", round(sum(durs), 1))


if __name__ == "__main__":
    main()
