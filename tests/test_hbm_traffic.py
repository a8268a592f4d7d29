"""scripts/hbm_traffic.py (no GPU): the PMC traffic of the routing kernel is averaged over the bench
horizons only, and a counter pass that also recorded other launches is refused (VERDICT r4 item 1:
the det pass had averaged the drop-in API's six chunk launches into the two bench launches)."""
import csv
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("hbm_traffic",
                                               os.path.join(ROOT, "scripts", "hbm_traffic.py"))
hbm = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(hbm)

KFLOW = "void mcr::(anonymous namespace)::wavefront_flow<192, 2, false>(mcr::WaveArgs)"
KDET = "void mcr::(anonymous namespace)::wavefront_det<256, 2, false>(mcr::WaveArgs)"


def write_pass(d, counter, rows):
    """rows: [(dispatch id, kernel, value)] -> d/run_counter_collection.csv (rocprofv3 columns)."""
    os.makedirs(d, exist_ok=True)
    cols = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id",
            "Grid_Size", "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size",
            "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Counter_Name",
            "Counter_Value", "Start_Timestamp", "End_Timestamp"]
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, cols)
        w.writeheader()
        w.writerow(dict.fromkeys(cols, 0) | {"Dispatch_Id": 1, "Kernel_Name": "__amd_rocclr_copyBuffer",
                                             "Counter_Name": counter, "Counter_Value": 2.0})
        for k, name, v in rows:
            w.writerow(dict.fromkeys(cols, 0) | {"Dispatch_Id": k, "Kernel_Name": name,
                                                 "Counter_Name": counter, "Counter_Value": v})


def test_det_pass_with_api_launches_is_refused(tmp_path):
    # the r04p det write pass: two bench launches + six API chunk launches
    vals = [600063.0, 600063.0, 402005.0, 288829.0, 402005.0, 288829.0, 402005.0, 288829.0]
    write_pass(tmp_path / "w", "WRITE_SIZE", [(24 + i, KFLOW, v) for i, v in enumerate(vals)])
    write_pass(tmp_path / "f", "FETCH_SIZE", [(24 + i, KFLOW, 48000.0) for i in range(8)])
    with pytest.raises(ValueError, match="identical horizons"):
        hbm.traffic(str(tmp_path / "f"), str(tmp_path / "w"))
    with pytest.raises(ValueError):
        hbm.traffic(str(tmp_path / "f"), str(tmp_path / "w"), launches=1)


def test_det_bench_launches_only(tmp_path):
    write_pass(tmp_path / "w", "WRITE_SIZE", [(24, KFLOW, 600063.0), (25, KFLOW, 600063.0)])
    write_pass(tmp_path / "f", "FETCH_SIZE", [(24, KFLOW, 48271.0), (25, KFLOW, 48252.0)])
    rec = hbm.traffic(str(tmp_path / "f"), str(tmp_path / "w"))
    assert rec["launches_per_horizon"] == 1 and rec["horizons"] == [2, 2]
    assert rec["write_bytes"] == pytest.approx(600063.0 * 1024)
    assert rec["read_bytes"] == pytest.approx(2 * 48261.5 * 1024)


def test_multi_launch_horizons_found(tmp_path):
    # two horizons of 5 launches whose bytes ramp up and down (first / last launches run fewer
    # workgroups): the per-launch mean is the horizon total / 5
    h = [10.0, 40.0, 50.0, 40.0, 10.0]
    write_pass(tmp_path / "w", "WRITE_SIZE", [(i, KDET, v) for i, v in enumerate(h + h)])
    write_pass(tmp_path / "f", "FETCH_SIZE", [(i, KDET, v / 10) for i, v in enumerate(h + h)])
    rec = hbm.traffic(str(tmp_path / "f"), str(tmp_path / "w"))
    assert rec["launches_per_horizon"] == 5
    assert rec["write_size_kb"] == pytest.approx(30.0)


def test_mixed_kernels_refused(tmp_path):
    write_pass(tmp_path / "w", "WRITE_SIZE", [(1, KFLOW, 5.0), (2, KDET, 5.0)])
    write_pass(tmp_path / "f", "FETCH_SIZE", [(1, KFLOW, 5.0), (2, KDET, 5.0)])
    with pytest.raises(ValueError, match="several kernels"):
        hbm.traffic(str(tmp_path / "f"), str(tmp_path / "w"))
