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
