"""bench.py's N > 1 path end to end on one GPU: two ranks under torch.distributed.run (gloo
rendezvous, 127.0.0.1), sharing the card through the host debug transport (RCCL refuses two
ranks on one device). Checks the one JSON line the driver parses — the same code the driver's
multi-GPU run executes with RCCL, minus the transport."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_host_transport():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--grid", "48", "--transport", "host"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]  # rank 0 prints exactly one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["unit"] == "V-cycles/s" and d["higher_is_better"] is True
    assert d["scaling"] == "strong" and d["dtype"] == "f64"
    assert d["config"]["n"] == 48 ** 3 and d["config"]["transport"] == "host"
    assert "host debug transport" in d["config"]["parallelism"]
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1.5
    assert d["cpu_baseline"] is None  # rank 0 at N = 1 only
    assert d["final_residual"] > 0
    # N > 1 diagnostics: per-level ms with the max over ranks, and the
    # ghost-exchange times per level / per cycle
    lv = d["levels"]
    assert len(lv) == d["config"]["levels"] and lv[0]["ms"]["residual"] > 0
    assert all(lv[l]["ms_max_over_ranks"][op] >= lv[l]["ms"][op] for l in range(len(lv)) for op in lv[l]["ms"])
    ex = d["exchange"]
    assert ex["per_level"][0]["exchanges_per_cycle"]["A"] == 3 and ex["per_level"][0]["ms_per_exchange"]["A"] > 0
    assert ex["ms_per_cycle_upper_bound"] >= ex["per_level"][0]["ms_per_cycle"] > 0
