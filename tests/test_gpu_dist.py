"""Member-sharded ensemble analysis (ensemble.py + mc_ens_* stages) with two ranks on the device:
scripts/dist_enkf_check.py under torch.distributed.run, gloo backend (RCCL refuses two ranks on
the one GPU of a test box: "Duplicate GPU detected"), device buffers staged through host memory
for the collectives.  Rank 0 compares the gathered members with the one-session analysis of the
whole ensemble: bit-identical."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(240)
def test_two_rank_device_analysis_bitexact():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517",
           os.path.join(ROOT, "scripts", "dist_enkf_check.py"), "--backend", "gloo",
           "--reaches", "8000", "--members", "8", "--gauges", "40"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=220)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "bitexact=True" in out, out[-3000:]


@pytest.mark.timeout(420)
def test_bench_two_ranks_gloo_line():
    """bench.py's N > 1 branch end to end on the one GPU of a test box: two ranks (gloo,
    host-staged collectives), the member-sharded configs[3] EnKF as the headline (3 analysis
    steps to bound the run), the replicated det run beside it, the CPU baseline timed on rank 0."""
    import json
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend",
           "gloo", "--steps", "1", "--warmup", "0", "--timing-runs", "1", "--no-api",
           "--obs-hours", "0.25", "--cpu-seconds", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["parallelism"] == "members sharded x2"
    assert line["config"]["members"] == 256 and line["config"]["members_per_gpu"] == 128
    assert line["value"] > 0 and line["value"] == line["value"]          # finite, not NaN
    assert line["det_replicas"]["parallelism"] == "replicas x2"
    assert line["det_replicas"]["value"] > 0
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1
