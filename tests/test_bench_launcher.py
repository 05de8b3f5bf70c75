"""bench.py driver contract on the CPU: ``--gpus N`` spawns N ranks (torch.distributed.run as
a child process), rank 0 prints ONE JSON line with n_gpus == N, the parent relays it and
fails loudly when a rank fails (``--cpu-dry-run``: gloo + the fp32 oracle, no GPU)."""
import json
import re
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None, timeout=300):
    e = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=timeout, env=e, cwd=ROOT)


@pytest.mark.parametrize("n", [1, 2, 4])
def test_launcher_spawns_n_ranks_one_json_line(n):
    r = _bench("--cpu-dry-run", "--gpus", str(n), "--steps", "3", "--warmup", "1",
               "--batch", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == 4 * n
    assert rec["config"]["parallelism"] == f"dp{n}"
    assert rec["rank_ms_per_step_max"] >= rec["rank_ms_per_step_min"] > 0
    assert rec["value"] > 0 and rec["dry_run"] == "cpu-gloo"
    # the gradient reduce at the reference's precision (DataParallelTable: fp32)
    assert rec["grad_dtype"] == "fp32"
    for k in ("metric", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
              "dtype", "data"):
        assert k in rec


def test_bench_defaults_fp32_gradient_wire_and_host_pool():
    """bench.py's defaults: the DP gradient all-reduce in fp32 (the
    bf16 wire only as a labelled secondary), the synthetic pool in pinned host memory, and
    the real-data (C++ loader) secondary in the default list."""
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse([])
    assert a.grad_dtype == "fp32" and not a.device_pool and not a.no_bf16_wire_secondary
    assert "256:bf16:fixture" in a.secondary.split(",")
    from deep_go_amd.config import ExperimentConfig
    assert ExperimentConfig().grad_dtype == "fp32"


def test_launcher_fails_loudly_when_a_rank_fails():
    # rank 1 exits non-zero (DG_BENCH_FAIL_RANK hook): no JSON line, non-zero exit
    r = _bench("--cpu-dry-run", "--gpus", "2", "--steps", "2", "--warmup", "1",
               env={"DG_BENCH_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.strip().startswith("{")]


def test_world_size_mismatch_is_an_error():
    r = _bench("--cpu-dry-run", "--gpus", "2", "--steps", "1", "--warmup", "0",
               env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1 != --gpus 2" in r.stderr


def test_hung_rank_is_bounded_by_the_phase_guard():
    # rank 1 sleeps inside the timed phase (DG_BENCH_HANG hook): its PhaseGuard ends it with
    # exit 42 after --phase-timeout, it records hang:timed, and the launcher fails loudly
    import time
    t0 = time.monotonic()
    r = _bench("--cpu-dry-run", "--gpus", "2", "--steps", "2", "--warmup", "1",
               "--phase-timeout", "5", env={"DG_BENCH_HANG": "1:timed"}, timeout=240)
    wall = time.monotonic() - t0
    assert r.returncode != 0
    assert "phase 'timed' exceeded" in r.stderr
    # the hung rank 1 and rank 0 (waiting for it in the barrier) enter 'timed' together, so
    # either guard may fire first (the elastic agent then ends the other rank before its own
    # guard reports): the launcher names whichever rank it was, in the timed phase
    assert re.search(r"'rank[01]': \('timed'", r.stderr), r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert wall < 150


def test_comm_hang_is_bounded_and_falls_back():
    # rank 1 hangs while setting up the native communicator (--comm auto; the CPU dry run
    # rehearses that phase): its guard fires after --comm-timeout with hang:comm:native, the
    # launcher re-runs with --comm torch (the hook does not fire on that kind) and relays the
    # fallback run's JSON line, marked comm_fallback — all well inside the launch budget
    import time
    t0 = time.monotonic()
    r = _bench("--cpu-dry-run", "--gpus", "2", "--steps", "2", "--warmup", "1",
               "--comm-timeout", "8", "--phase-timeout", "8", "--launch-budget", "200",
               env={"DG_BENCH_HANG": "1:comm:native"}, timeout=240)
    wall = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert "comm_fallback" in rec and rec["n_gpus"] == 2
    assert rec["comm"].startswith("gloo (torch")
    assert wall < 200


def test_comm_hang_on_every_kind_fails_within_budget():
    # the same hang on any communicator: the fallback run hangs too; the job still ends
    # non-zero with no JSON line, bounded by the guards (not by an outer timeout)
    import time
    t0 = time.monotonic()
    r = _bench("--cpu-dry-run", "--gpus", "2", "--steps", "2", "--warmup", "1",
               "--comm-timeout", "8", "--phase-timeout", "8", "--launch-budget", "200",
               env={"DG_BENCH_HANG": "1:comm"}, timeout=240)
    wall = time.monotonic() - t0
    assert r.returncode != 0
    assert "re-run with --comm torch" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert wall < 200


def test_non_native_hang_does_not_trigger_the_fallback():
    # a hang while the rank is on torch.distributed (--comm torch) is not a native-communicator
    # problem: no re-run, fail as is
    r = _bench("--cpu-dry-run", "--gpus", "2", "--steps", "2", "--warmup", "1", "--comm", "torch",
               "--comm-timeout", "6", "--phase-timeout", "6", env={"DG_BENCH_HANG": "1:comm"},
               timeout=240)
    assert r.returncode != 0
    assert "re-run with --comm torch" not in r.stderr
