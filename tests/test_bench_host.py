"""Host logic of bench.py (no GPU): workload presets, the N-rank launch decision, the per-workload
defaults and the lookup of the PMC-measured HBM traffic that the bench line reports as
roofline.traffic (only for the build it was measured on)."""
import json

import pytest

import bench


def parse(*argv, world=1):
    return bench.parse(list(argv), world=world)


def test_defaults_are_baseline_config_1():
    a = parse()
    assert (a.n, a.basins, a.depth, a.T, a.dt, a.members) == (190_000, 300, 1500, 288, 300.0, 1)
    assert not a.enkf and not a.conus


def test_multi_gpu_default_is_the_sharded_256_member_enkf():
    """BASELINE configs[3]: with N > 1 ranks the headline is the 256-member EnKF, members
    sharded over the ranks; --det keeps the replicated deterministic run."""
    a = parse(world=8)
    assert a.members == 256 and a.enkf
    d = parse("--det", world=8)
    assert d.members == 1 and not d.enkf
    e = parse("--members", "64", world=4)
    assert e.members == 64 and not e.enkf


def test_conus_preset_is_baseline_config_4():
    a = parse("--conus")
    assert (a.n, a.basins, a.depth, a.members) == (2_700_000, 4000, 7000, 16)
    assert parse("--conus", "--members", "8").members == 8
    assert parse("--conus", world=8).members == 16


def test_huc8_preset_is_baseline_config_0():
    a = parse("--huc8")
    assert (a.n, a.basins, a.depth, a.members) == (1000, 1, 100, 1) and not a.enkf
    assert parse("--huc8", world=4).members == 1       # deterministic replicas, not the EnKF


def test_huc8_network_is_one_sub_basin():
    from tx_fast_hydrology_amd import synthetic
    import numpy as np
    end = synthetic.huc8(seed=0, n=1000, max_depth=100)
    assert end.size == 1000 and int((end == np.arange(1000)).sum()) == 1


def test_launch_plan():
    # no launcher: --gpus N > 1 spawns N ranks as a child, --gpus 1 runs here
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(1, {}) == ("run", 1)
    # under torch.distributed.run: --gpus must equal the world size
    env = {"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "4"}
    assert bench.launch_plan(4, env) == ("run", 4)
    with pytest.raises(SystemExit):
        bench.launch_plan(1, env)
    with pytest.raises(SystemExit):
        bench.launch_plan(8, env)
    assert bench.launch_plan(1, {"RANK": "0", "WORLD_SIZE": "1"}) == ("run", 1)
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def test_spawn_ranks_runs_a_child_launcher(monkeypatch):
    seen = {}

    def call(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return 3

    monkeypatch.setattr(bench.subprocess, "call", call)
    monkeypatch.setattr(bench.sys, "argv", ["bench.py", "--gpus", "2", "--steps", "4"])
    assert bench.spawn_ranks(2) == 3
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "4"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_measured_traffic_matches_the_exact_workload_and_build(tmp_path, monkeypatch):
    from tx_fast_hydrology_amd._build import source_hash
    h = source_hash()
    prof = tmp_path / "profiles"
    prof.mkdir()
    det = {"workload": {"slots": 192, "tile": 16, "n": 190000, "T": 288},
           "traffic_bytes_per_launch": 7.0e8, "source_hash": h, "launches_per_horizon": 1}
    ens = {"workload": {"slots": 256, "tile": 64, "n": 190000, "T": 288, "E": 64},
           "traffic_bytes_per_launch": 2.1e9, "source_hash": h, "launches_per_horizon": 23}
    old = {"workload": {"slots": 384, "tile": 32, "n": 190000, "T": 288},
           "traffic_bytes_per_launch": 6.9e8, "source_hash": h, "launches_per_horizon": 1}
    stale = {"workload": {"slots": 192, "tile": 16, "n": 190000, "T": 288},
             "traffic_bytes_per_launch": 9.9e8, "source_hash": "0" * 16,
             "launches_per_horizon": 1}
    # a profile of this build written before the bench-horizon selection: never quoted
    mixed = {"workload": {"slots": 192, "tile": 16, "n": 190000, "T": 288},
             "traffic_bytes_per_launch": 4.9e8, "source_hash": h}
    (prof / "r01e_hbm_traffic.json").write_text(json.dumps(mixed))
    (prof / "r01a_hbm_traffic.json").write_text(json.dumps(old))
    (prof / "r01b_hbm_traffic.json").write_text(json.dumps(det))
    (prof / "r01b_hbm_traffic_ens64.json").write_text(json.dumps(ens))
    (prof / "r01c_hbm_traffic.json").write_text("not json")
    (prof / "r01d_hbm_traffic.json").write_text(json.dumps(stale))   # newer, other build
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    got, note = bench.measured_traffic({"slots": 192, "tile": 16}, 190000, 288)
    assert got["traffic_bytes_per_launch"] == 7.0e8 and got["file"].endswith("r01b_hbm_traffic.json")
    got, _ = bench.measured_traffic({"slots": 256, "tile": 64}, 190000, 288, E=64)
    assert got["traffic_bytes_per_launch"] == 2.1e9
    assert bench.measured_traffic({"slots": 256, "tile": 64}, 190000, 288, E=32)[0] is None
    assert bench.measured_traffic({"slots": 448, "tile": 16}, 190000, 288)[0] is None
    # only a profile of another build: refused, and the note names it
    (prof / "r01b_hbm_traffic.json").unlink()
    got, note = bench.measured_traffic({"slots": 192, "tile": 16}, 190000, 288)
    assert got is None and "r01d_hbm_traffic.json" in note and h in note


def test_compulsory_bytes():
    # det Texas: outflows 288 n 8 + forcing 25 n 8 + coefficients 4 n 8 + state 4 n 8
    assert bench.compulsory_bytes(190000, 1, 288, 25) == 8.0 * 190000 * (288 + 25 + 4 + 4)
    assert bench.compulsory_bytes(10, 4, 3, 2) == 8.0 * 10 * (12 + 8 + 4 + 16)


@pytest.mark.parametrize("E,enkf,want", [(1, False, "texas-det"), (64, False, "texas-ens64"),
                                         (32, True, "texas-enkf")])
def test_workload_names(E, enkf, want):
    from types import SimpleNamespace
    ek = SimpleNamespace(E_total=E, n_an=24, m=500) if enkf else None
    wl = SimpleNamespace(enkf=ek, n=190000)
    assert bench.workload_name(wl, E).startswith(want)
