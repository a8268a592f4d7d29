#!/usr/bin/env python3
"""HBM traffic per launch of the routing kernel from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE; they cannot share a pass on gfx950).  Correction per MI355X_MICROARCH.md (HBM):
FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950 -> doubled; WRITE_SIZE as is.
Writes profiles/<tag>_hbm_traffic.json, stamped with the library's source hash (_build.
source_hash); bench.py reports it as roofline.traffic only when the workload AND the hash match
the running build.
    python scripts/hbm_traffic.py <fetch_dir> <write_dir> <tag> <slots> <tile> <n> <T> [E]
(E = members per GPU, default 1; ensembles go to profiles/<tag>_hbm_traffic_ens<E>.json)
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tx-fast-hydrology_amd"))
from tx_fast_hydrology_amd._build import source_hash  # noqa: E402


def per_dispatch(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "wavefront" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            out[k] = (r["Kernel_Name"], out.get(k, (None, 0.0))[1] + float(r["Counter_Value"]))
    return out


def main():
    fdir, wdir, tag, slots, tile, n, T = sys.argv[1:8]
    E = int(sys.argv[8]) if len(sys.argv) > 8 else 1
    fe = per_dispatch(fdir, "FETCH_SIZE")
    wr = per_dispatch(wdir, "WRITE_SIZE")
    if not fe or not wr:
        sys.exit("no wavefront dispatches with FETCH_SIZE / WRITE_SIZE found")
    # rocprofv3 derives both in KB
    fetch_kb = sum(v for _, v in fe.values()) / len(fe)
    write_kb = sum(v for _, v in wr.values()) / len(wr)
    kernel = sorted({k for k, _ in fe.values()})
    rec = {"kernel": kernel, "dispatches": [len(fe), len(wr)],
           "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
           "read_bytes": 2.0 * fetch_kb * 1024, "write_bytes": write_kb * 1024,
           "traffic_bytes_per_launch": 2.0 * fetch_kb * 1024 + write_kb * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE x1",
           "workload": {"slots": int(slots), "tile": int(tile), "n": int(n), "T": int(T)},
           "source_hash": source_hash()}
    if E > 1:
        rec["workload"]["E"] = E
    os.makedirs("profiles", exist_ok=True)
    out = f"profiles/{tag}_hbm_traffic" + (f"_ens{E}" if E > 1 else "") + ".json"
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
