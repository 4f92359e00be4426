"""The N>1 path's RCCL calls on a one-GPU box.

RCCL refuses two ranks on one device, so the multi-rank rehearsals of bench.py use gloo
(tools/rehearse_multi.sh). This test runs the driver's own launch form instead --
`python -m torch.distributed.run ... bench.py --gpus 1` -- with FM_BENCH_PG=1, which builds a
one-rank "nccl" group: init_process_group with `device_id`, the timing barrier, the all-reduce
(MAX) of a device tensor, gather_object of the rank records and destroy_process_group all run
through RCCL, as they do on every rank of an 8-GPU run.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_bench_one_rank_rccl_group():
    env = dict(os.environ, FM_BENCH_PG="1", FM_BENCH_BACKEND="nccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
           "--steps", "3", "--warmup", "2", "--no-cpu-baseline", "--no-host-fed", "--no-mjpeg", "--no-side"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["ranks"]["group_backend"] == "nccl" and line["ranks"]["world_size_seen"] == 1
    assert [d["rank"] for d in line["ranks"]["devices"]] == [0] and line["ranks"]["devices"][0]["device"] == 0
