"""bench.py --gpus N: the N-rank job it launches for itself, and the rank-count checks
(the -T fan-out it stands in for: reference engine.py:386-422).  CPU only: no rank starts."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_command_shape():
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "20", "--warmup", "3"], 8, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-port=29512" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    # the child re-runs this very script with the caller's arguments unchanged
    j = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[j + 1:] == ["--gpus", "8", "--steps", "20", "--warmup", "3"]


def test_resolve_world_without_launcher():
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(2, {}) == (2, True)
    assert bench.resolve_world(8, {}) == (8, True)
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


def test_resolve_world_under_launcher():
    # the driver's form: torch.distributed.run ... bench.py --gpus N
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(None, {"WORLD_SIZE": "2"}) == (2, False)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.resolve_world(8, {"WORLD_SIZE": "2"})


def test_free_port_is_bindable():
    import socket
    p = bench.free_port()
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", p))


def test_mismatch_exits_before_any_gpu_work():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_trace_stage_time_filters_the_scan_forms(tmp_path):
    """roofline's time: the kernel-trace pass holds every kernel of the child process; only the
    scan stage's forms count, each averaged without its first (cold) dispatch, forms summed."""
    import csv
    import bench
    p = tmp_path / "kernel_trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for i, d in enumerate([9000, 2000, 2200]):
            w.writerow(["void mp::scan_kernel<1, false>(mp::ScanArgs)", 10 * i, 10 * i + d])
        for d in [5000, 700, 900]:
            w.writerow(["void mp::scan_kernel<1, false, 8>(mp::ScanArgs)", 0, d])
        w.writerow(["void at::native::vectorized_elementwise_kernel<4>", 0, 10 ** 9])
        w.writerow(["void mp::tail_kernel<false>(mp::ScanArgs)", 0, 10 ** 6])
    got = bench.trace_stage_ns(str(p), "scan_kernel|dense_kernel")
    assert got["_trace_stage_ns"] == 2100 + 800
    assert sorted(got["_trace_forms"]) == ["void mp::scan_kernel<1, false, 8>(mp::ScanArgs)",
                                           "void mp::scan_kernel<1, false>(mp::ScanArgs)"]


def test_roofline_time_never_takes_the_all_dispatch_mean():
    """The roofline's time: this command's trace pass first, then a committed profile's isolated
    mean, then the events -- never a profile's mean over every (overlapped) dispatch."""
    assert bench.roofline_time({"_trace_stage_ns": 2.0e6, "avg_duration_ns_trace_isolated": 2.5e6}, 9e-3)[0] == 2.0e-3
    t, src = bench.roofline_time({"avg_duration_ns_trace": 3.16e6, "avg_duration_ns_trace_isolated": 2.06e6}, 9e-3)
    assert t == 2.06e-3 and "isolated" in src
    t, src = bench.roofline_time({"avg_duration_ns_trace": 3.16e6}, 2.1e-3)
    assert t == 2.1e-3 and "events" in src
    assert bench.roofline_time(None, 1e-3) == (1e-3, "HIP events (no trace pass)")
