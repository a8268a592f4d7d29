"""Host logic of bench.py (no GPU): workload presets, the per-workload defaults and the lookup of
the PMC-measured HBM traffic that the bench line reports as roofline.traffic."""
import json
import sys

import pytest

import bench


def parse(*argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_defaults_are_baseline_config_1():
    a = parse()
    assert (a.n, a.basins, a.depth, a.T, a.dt, a.members) == (190_000, 300, 1500, 288, 300.0, 1)
    assert not a.enkf and not a.conus


def test_conus_preset_is_baseline_config_4():
    a = parse("--conus")
    assert (a.n, a.basins, a.depth, a.members) == (2_700_000, 4000, 7000, 16)
    assert parse("--conus", "--members", "8").members == 8


def test_measured_traffic_matches_the_exact_workload(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    det = {"workload": {"slots": 192, "tile": 16, "n": 190000, "T": 288},
           "traffic_bytes_per_launch": 7.0e8}
    ens = {"workload": {"slots": 256, "tile": 64, "n": 190000, "T": 288, "E": 64},
           "traffic_bytes_per_launch": 2.1e9}
    old = {"workload": {"slots": 384, "tile": 32, "n": 190000, "T": 288},
           "traffic_bytes_per_launch": 6.9e8}
    (prof / "r01a_hbm_traffic.json").write_text(json.dumps(old))
    (prof / "r01b_hbm_traffic.json").write_text(json.dumps(det))
    (prof / "r01b_hbm_traffic_ens64.json").write_text(json.dumps(ens))
    (prof / "r01c_hbm_traffic.json").write_text("not json")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got = bench.measured_traffic({"slots": 192, "tile": 16}, 190000, 288)
    assert got["traffic_bytes_per_launch"] == 7.0e8 and got["file"].endswith("r01b_hbm_traffic.json")
    got = bench.measured_traffic({"slots": 256, "tile": 64}, 190000, 288, E=64)
    assert got["traffic_bytes_per_launch"] == 2.1e9
    assert bench.measured_traffic({"slots": 256, "tile": 64}, 190000, 288, E=32) is None
    assert bench.measured_traffic({"slots": 448, "tile": 16}, 190000, 288) is None


@pytest.mark.parametrize("E,enkf,want", [(1, False, "texas-det"), (64, False, "texas-ens64"),
                                         (32, True, "texas-enkf")])
def test_workload_names(E, enkf, want):
    from types import SimpleNamespace
    ek = SimpleNamespace(E_total=E, n_an=24, m=500) if enkf else None
    wl = SimpleNamespace(enkf=ek, n=190000)
    assert bench.workload_name(wl, E).startswith(want)
