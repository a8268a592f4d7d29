#!/usr/bin/env python3
"""HBM traffic per launch of the routing kernel from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE; they cannot share a pass on gfx950).  Correction per MI355X_MICROARCH.md (HBM):
FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950 -> doubled; WRITE_SIZE as is.
Writes profiles/<tag>_hbm_traffic.json, stamped with the library's source hash (_build.
source_hash); bench.py reports it as roofline.traffic only when the workload AND the hash match
the running build.
    python scripts/hbm_traffic.py <fetch_dir> <write_dir> <tag> <slots> <tile> <n> <T> [E]
        [--launches L]
(E = members per GPU, default 1; ensembles go to profiles/<tag>_hbm_traffic_ens<E>.json)

Only the bench horizons may be counted.  The PMC passes run `bench.py --no-api` (scripts/
gpu_pmc.sh), so every routing dispatch of the pass belongs to one of its identical horizons; the
dispatches are split into horizons of L consecutive launches (--launches, or the smallest L whose
horizons agree) and the set is REFUSED unless every horizon moves the same bytes within 2 % --
a pass that also recorded other launches (e.g. the drop-in API's chunk launches, which move other
byte counts) cannot be averaged into a per-launch figure.
"""
import argparse
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tx-fast-hydrology_amd"))

TOL = 0.02


def per_dispatch(d, counter, match="wavefront"):
    """{dispatch id: (kernel name, counter value summed over the dispatch's rows)}."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            out[k] = (r["Kernel_Name"], out.get(k, (None, 0.0))[1] + float(r["Counter_Value"]))
    return out


def _horizons(vals, L):
    return [sum(vals[h * L:(h + 1) * L]) for h in range(len(vals) // L)]


def _consistent(tot):
    lo, hi = min(tot), max(tot)
    return hi > 0 and (hi - lo) <= TOL * hi


def split_horizons(disp, launches=None):
    """Per-launch mean of a dispatch set made of identical horizons: returns (mean per launch,
    L, number of horizons).  Raises ValueError when the set is not such a set (mixed kernels,
    a count that L does not divide, horizons whose bytes disagree by more than TOL)."""
    if not disp:
        raise ValueError("no routing dispatches found")
    names = {k for k, _ in disp.values()}
    if len(names) != 1:
        raise ValueError(f"dispatches of several kernels: {sorted(names)}")
    vals = [disp[k][1] for k in sorted(disp)]
    cands = [launches] if launches else [L for L in range(1, len(vals) // 2 + 1)
                                         if len(vals) % L == 0]
    for L in cands:
        if L is None or L < 1 or len(vals) % L or len(vals) // L < 1:
            continue
        tot = _horizons(vals, L)
        if (len(tot) >= 2 or launches) and _consistent(tot):
            return sum(tot) / len(tot) / L, L, len(tot)
    raise ValueError(
        f"{len(vals)} dispatches do not form identical horizons (per-dispatch values "
        f"{[round(v) for v in vals[:12]]}{' ...' if len(vals) > 12 else ''}): the pass recorded "
        "launches other than the bench horizons (run bench.py with --no-api)")


def traffic(fdir, wdir, launches=None):
    fe = per_dispatch(fdir, "FETCH_SIZE")
    wr = per_dispatch(wdir, "WRITE_SIZE")
    fetch_kb, Lf, hf = split_horizons(fe, launches)
    write_kb, Lw, hw = split_horizons(wr, launches)
    if Lf != Lw:
        raise ValueError(f"the two passes split into horizons of {Lf} and {Lw} launches")
    kernel = sorted({k for k, _ in fe.values()})
    # rocprofv3 derives both in KB
    return {"kernel": kernel, "dispatches": [len(fe), len(wr)], "launches_per_horizon": Lf,
            "horizons": [hf, hw], "fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
            "read_bytes": 2.0 * fetch_kb * 1024, "write_bytes": write_kb * 1024,
            "traffic_bytes_per_launch": 2.0 * fetch_kb * 1024 + write_kb * 1024,
            "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE x1",
            "selection": f"bench horizons only: {Lf} launches each, horizons agree within "
                         f"{TOL:.0%}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("tag")
    ap.add_argument("slots", type=int)
    ap.add_argument("tile", type=int)
    ap.add_argument("n", type=int)
    ap.add_argument("T", type=int)
    ap.add_argument("E", type=int, nargs="?", default=1)
    ap.add_argument("--launches", type=int, default=None)
    a = ap.parse_args()
    from tx_fast_hydrology_amd._build import source_hash
    try:
        rec = traffic(a.fetch_dir, a.write_dir, a.launches)
    except ValueError as e:
        sys.exit(f"refused: {e}")
    rec["workload"] = {"slots": a.slots, "tile": a.tile, "n": a.n, "T": a.T}
    if a.E > 1:
        rec["workload"]["E"] = a.E
    rec["source_hash"] = source_hash()
    os.makedirs("profiles", exist_ok=True)
    out = f"profiles/{a.tag}_hbm_traffic" + (f"_ens{a.E}" if a.E > 1 else "") + ".json"
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
