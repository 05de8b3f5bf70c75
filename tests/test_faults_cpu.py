"""Failure paths of the trainer, exercised on the CPU.

* a hung step (``DG_FAULT=0:k:hang``) under ``DG_STEP_TIMEOUT`` ends the process with the
  watchdog's exit code 42 within a bound;
* a communicator that reports an async error (a stub standing in for
  ``ncclCommGetAsyncError``) is aborted and the process exits 43;
* in a gloo world of 2, killing rank 1 mid-run (``DG_FAULT=1:k:exit``) makes the surviving
  rank 0 terminate non-zero within the timeout instead of waiting forever in the gradient
  all-reduce.

Reference: the pcall capture of a failing batch (/root/reference/train.lua:106-109) and the
GPU-count assert of makeDataParallel (/root/reference/experiments.lua:157) are all the
reference has; these paths are the MI355X build's replacement."""
import os
import socket
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(**kw):
    e = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DG_FAULT", "DG_STEP_TIMEOUT"):
        e.pop(k, None)
    e.update({k: str(v) for k, v in kw.items()})
    return e


TRAIN = [sys.executable, "-m", "deep_go_amd", "train", "--preset", "cpu-1layer-k16",
         "--device", "cpu"]


def test_hung_step_is_ended_by_the_watchdog(tmp_path):
    t0 = time.monotonic()
    r = subprocess.run(TRAIN + ["--iters", "20", "validationSize=16", "validation_interval=1000",
                                "loader_threads=1", f"checkpoint_dir={tmp_path}", "id=hang"],
                       capture_output=True, text=True, cwd=ROOT, timeout=300,
                       env=_env(DG_FAULT="0:3:hang", DG_STEP_TIMEOUT="3"))
    wall = time.monotonic() - t0
    assert r.returncode == 42, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "no step progress" in r.stdout
    assert wall < 120


def test_comm_async_error_aborts_and_exits_43(tmp_path):
    marker = tmp_path / "aborted"
    script = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        from deep_go_amd.utils.faults import StepWatchdog

        class StubComm:  # ncclCommGetAsyncError: healthy once, then a dead peer
            kind = "native"
            polls = 0
            def async_error(self):
                StubComm.polls += 1
                return "remote process exited or there was a network error" \\
                    if StubComm.polls >= 2 else ""
            def abort(self):
                open({str(marker)!r}, "w").write("aborted")

        StepWatchdog(0, comm=StubComm(), poll_s=0.05)
        time.sleep(60)
        sys.exit(0)
    """)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 43, (r.stdout, r.stderr)
    assert marker.read_text() == "aborted"
    assert "communicator error" in r.stdout
    assert time.monotonic() - t0 < 30


def test_dead_rank_terminates_the_survivor(tmp_path):
    """Two independent rank processes (no torchrun supervisor that would kill the survivor
    for us): rank 1 hard-exits at step 3; rank 0 must not hang in its all-reduce."""
    port = _free_port()
    procs = []
    t0 = time.monotonic()
    for rank in (0, 1):
        env = _env(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK=rank, LOCAL_RANK=rank,
                   WORLD_SIZE=2, DG_FAULT="1:3:exit", DG_STEP_TIMEOUT="20")
        procs.append(subprocess.Popen(
            TRAIN + ["--iters", "30", "batchSize=8", "validationSize=16",
                     "validation_interval=1000", "loader_threads=1",
                     f"checkpoint_dir={tmp_path}", "id=dead"],
            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT, env=env))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    wall = time.monotonic() - t0
    rc0, rc1 = procs[0].returncode, procs[1].returncode
    assert rc1 == 17, outs[1][1][-2000:]           # the injected hard exit
    assert rc0 != 0, outs[0][0][-2000:]            # the survivor did not finish "successfully"
    assert wall < 200
