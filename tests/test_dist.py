"""Multi-process path on CPU (gloo, world size 2): stream sharding, timing reduction and gather.

Each rank runs its contiguous block of synthetic streams through a
StreamGroup (per-frame results from the CPU oracle engine, tests/fake_engine.py)
and rank 0 gathers the per-stream run_vid tuples plus written-frame lists.
The gathered result must equal a single-process run over all streams: the
path has no cross-stream dependency, so sharding is exact.
"""
import os
import socket

import pytest
import torch.multiprocessing as mp

W, H, N, S_PER_RANK = 160, 90, 20, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_streams(streams, tmpdir):
    from fake_engine import OracleEngine
    from find_motion_amd import motion, videoio

    caps = [videoio.SyntheticCapture(W, H, N - 3 * (s % 3), s) for s in streams]
    names = [os.path.join(tmpdir, f"s{s}") for s in streams]
    grp = motion.StreamGroup(names, batch=4, captures=caps, engine=OracleEngine, box_size=80, threshold=12,
                             cache_time=0.2, min_time=0.1, outdir=tmpdir)
    res = grp.find_motion()
    return [(os.path.basename(r[1]), r[0], r[2], v.written_indices) for r, v in zip(res, grp.videos)]


def _worker(rank, world, port, tmpdir, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from find_motion_amd import dist

    p = dist.placement_from_env()
    active = dist.init(p, "gloo")
    streams = dist.rank_streams(p, S_PER_RANK)
    dist.barrier(active)
    res = _run_streams(streams, tmpdir)
    t = dist.max_over_ranks(float(rank + 1), active)
    gathered = dist.gather_to_root(res, p, active)
    if p.is_root:
        q.put((t, [r for part in gathered for r in part]))
    dist.finalize(active)


def test_two_rank_sharding_equals_single_process(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for pr in procs:
        pr.start()
    t, gathered = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert t == 2.0  # max over ranks
    serial = _run_streams(list(range(world * S_PER_RANK)), str(tmp_path / "serial") if os.makedirs(
        tmp_path / "serial", exist_ok=True) is None else None)
    assert [g[0] for g in gathered] == [f"s{s}" for s in range(world * S_PER_RANK)]
    assert [g[1:] for g in gathered] == [s[1:] for s in serial]
    assert any(g[3] for g in gathered)


def _one_rank_worker(port, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    from find_motion_amd import dist

    p = dist.placement_from_env()
    active = dist.init(p, "gloo", force=True)
    dist.barrier(active)
    out = (active, dist.world_size(active), dist.max_over_ranks(2.5, active), dist.gather_to_root("r0", p, active))
    dist.finalize(active)
    q.put(out)


def test_forced_one_rank_group():
    """bench.py's FM_BENCH_PG=1: a one-rank group runs every call the N>1 path makes (gloo here; RCCL on the box)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_one_rank_worker, args=(_free_port(), q))
    pr.start()
    out = q.get(timeout=120)
    pr.join(timeout=60)
    assert pr.exitcode == 0
    assert out == (True, 1, 2.5, ["r0"])


def test_placement_and_shards():
    from find_motion_amd import dist

    p = dist.Placement(rank=3, world=8, local_rank=3)
    assert dist.rank_streams(p, 8) == list(range(24, 32))
    assert not dist.init(dist.Placement(0, 1, 0), "gloo")
    assert dist.max_over_ranks(1.5, False) == 1.5
    assert dist.gather_to_root("x", dist.Placement(0, 1, 0), False) == ["x"]
