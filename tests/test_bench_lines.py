"""bench.py's labelling and roofline arithmetic (CPU): which BASELINE config a run is filed under at world
size 1 / 2 / 8 (configs[3] = 64 x 1080p, 8 streams per GPU on 8 GPUs, find_motion.py:1054-1122), and the
launch-time consistency check of the roofline (a launch of one stream's serialised pixel kernels can never
average more than a step)."""
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    saved = os.environ.get("GPU_MAX_HW_QUEUES")  # bench.py sets it at import (for its own process)
    sys.path.insert(0, ROOT)
    try:
        yield importlib.import_module("bench")
    finally:
        if saved is None:
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = saved


@pytest.mark.parametrize("S,world,mode,want", [
    (1, 1, "F", "configs[1]"),
    (1, 1, "D", "configs[1] (mode D)"),
    (1, 8, "F", "configs[1] x 8 GPUs"),
    (8, 1, "F", "configs[2]"),
    (8, 1, "D", "configs[2] (mode D)"),
    (8, 8, "F", "configs[3]"),
    (8, 2, "F", "configs[3] family: 8 streams per GPU x 2 GPUs"),
    (8, 4, "F", "configs[3] family: 8 streams per GPU x 4 GPUs"),
])
def test_config_name_is_world_aware(bench, S, world, mode, want):
    assert bench.config_name(S, 1920, 1080, mode, 5, world=world) == want


def test_config_name_other_shapes(bench):
    assert bench.config_name(4, 3840, 2160, "F", 21, haar=True) == "configs[4]"
    assert bench.config_name(4, 3840, 2160, "F", 21) == "configs[4] geometry (no Haar stage)"
    assert bench.config_name(3, 1920, 1080, "F", 5, world=2).startswith("3 x 1080p streams per GPU x 2 GPU(s)")
    assert bench.config_name(1, 640, 480, "F", 5) == "custom shape"


def _cfg(S=1, T=256, mode="F"):
    h, w = (1080, 1920) if mode == "F" else (56, 100)
    return {"streams_per_gpu": S, "frames_per_step": T, "H": 1080, "W": 1920, "h": h, "w": w,
            "workload": "test"}


def test_roofline_frac_and_launch_check(bench):
    cfg = _cfg()
    # 20 stamped launches of 450 us each inside 500 us steps
    roof = bench.roofline_of({"pix": (20 * 0.450, 20)}, cfg, ms_per_step=0.5)
    assert roof["kernel"] == "pix" and roof["launches_timed"] == 20
    assert roof["avg_launch_us"] == pytest.approx(450.0)
    assert roof["bytes_per_launch"] == 2_073_600 * (4 * 256 + 16)
    assert roof["frac"] == pytest.approx(roof["bytes_per_launch"] / 450e-6 / 1e9 / 8000.0, abs=1e-4)
    assert roof["launch_le_step"] is True
    # a launch longer than the step is a timing fault, flagged in the line
    bad = bench.roofline_of({"pix": (20 * 0.709, 20)}, cfg, ms_per_step=0.6555)
    assert bad["launch_le_step"] is False


def test_roofline_mode_d_prices_the_resize(bench):
    cfg = _cfg(mode="D")
    roof = bench.roofline_of({"pix": (10 * 0.3, 10), "resize_area": (10 * 0.29, 10)}, cfg, ms_per_step=0.4)
    assert roof["kernel"] == "resize_area"
    assert roof["bytes_per_launch"] == 256 * (1920 * 1080 * 3 + 56 * 100 * 3)
    assert roof["launch_le_step"] is True


def test_roofline_carries_the_launch_spread(bench):
    roof = bench.roofline_of({"pix": (20 * 0.6, 20)}, _cfg(), ms_per_step=0.62, kstd={"pix": 0.0214})
    assert roof["launch_std_us"] == pytest.approx(21.4)
    assert "launch_std_us" not in bench.roofline_of({"pix": (20 * 0.6, 20)}, _cfg(), ms_per_step=0.62)


def test_roofline_of_overlapping_launches_uses_their_union(bench):
    """Mode D's resizes of consecutive batches run on two input streams: each launch lasts ~2 steps, but at most
    two run at once, so the kernel's throughput is its bytes over the union of the launch windows."""
    cfg = _cfg(mode="D")
    ktimes = {"resize_area": (60 * 0.55, 60)}
    roof = bench.roofline_of(ktimes, cfg, ms_per_step=0.31, kbusy={"resize_area": 60 * 0.3})
    assert roof["launches_overlap"] and roof["launch_le_step"]
    assert roof["avg_launch_us"] == pytest.approx(550.0)
    assert roof["busy_us_per_launch"] == pytest.approx(300.0)
    assert roof["frac"] == pytest.approx(roof["bytes_per_launch"] / 300e-6 / 1e9 / 8000.0, abs=1e-4)
    assert roof["frac_per_launch_duration"] == pytest.approx(roof["bytes_per_launch"] / 550e-6 / 1e9 / 8000.0, abs=1e-4)
    # no overlap: the busy time equals the summed launch times and nothing changes
    plain = bench.roofline_of(ktimes, cfg, ms_per_step=0.6, kbusy={"resize_area": 60 * 0.55})
    assert "launches_overlap" not in plain and plain["frac"] == pytest.approx(roof["frac_per_launch_duration"], abs=1e-4)


def test_default_line_legs_have_committed_pmc_traffic(bench):
    """Every workload of the default line (configs[1], and the side legs mode D, configs[2], configs[4] with and
    without its Haar stage) has a PMC entry in profiles/traffic.json under the exact workload string the line
    carries, so no leg's roofline reports traffic null (verdict r05 item 6)."""
    from find_motion_amd import make_gaussian, work_height
    want = {
        "F": bench.workload_name(1, 1920, 1080, "F", 1920, 384, make_gaussian(1920, 384), 256, 256, 64),
        "mode_d": bench.workload_name(1, 1920, 1080, "D", 100, 20, make_gaussian(100, 20), 256, 256, 64),
        "configs2": bench.workload_name(8, 1920, 1080, "F", 1920, 384, make_gaussian(1920, 384), 128, 256, 64),
        "configs4": bench.workload_name(4, 3840, 2160, "F", 3840, 183, 21, 64, 64, 16, haar=True),
        "configs4_no_haar": bench.workload_name(4, 3840, 2160, "F", 3840, 183, 21, 64, 64, 16),
    }
    assert make_gaussian(3840, 183) == 21 and work_height(2160, 3840, 3840) == 2160
    for leg, wl in want.items():
        kernel = "resize_area" if leg == "mode_d" else "pix"
        traffic, src, sq = bench.pmc_traffic(kernel, {"workload": wl})
        assert traffic and traffic > 0, (leg, wl)
        assert os.path.exists(os.path.join(ROOT, src)), src


def test_side_legs_run_in_child_processes(bench, monkeypatch):
    """bench.py runs each side leg as `bench.py --side-leg NAME` in a process of its own and takes its last JSON
    line; a failed child gives an error entry, not a crash of the default line."""
    import json
    import subprocess
    assert set(bench.SIDE_LEGS) == {"mode_d", "configs2", "configs4", "configs4_no_haar"}
    seen = []

    class R:
        def __init__(self, rc, out):
            self.returncode, self.stdout = rc, out

    def fake_run(cmd, stdout=None, text=None, timeout=None, env=None):
        seen.append((cmd, env))
        return R(0, "noise\n" + json.dumps({"value": 1.0}) + "\n") if "mode_d" in cmd else R(1, "")

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setenv("FM_BENCH_PG", "1")
    args = type("A", (), {"warmup": 5, "batch": 256, "all_ktimes": False, "no_ktimes": False})()
    assert bench.side_child("mode_d", args) == {"value": 1.0}
    assert "error" in bench.side_child("configs4", args)
    cmd, env = seen[0]
    assert cmd[1].endswith("bench.py") and cmd[2:4] == ["--side-leg", "mode_d"]
    # the parent's one-rank process group is not rebuilt by the child on the parent's rendezvous
    assert "FM_BENCH_PG" not in env and env.get("PATH") == os.environ.get("PATH")
