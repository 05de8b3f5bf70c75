"""Failure detection and fault injection.

Reference: a ``pcall`` around the first of its two fwd/bwd passes stashes a failing batch in
globals (``train.lua:106-109``); nothing else (no watchdog, no NaN handling).

Here:
* ``check_finite`` — NaN/Inf guard on the loss (policy ``raise`` dumps the offending batch
  to ``<dir>/bad_batch_<step>.npz`` then raises; policy ``skip`` leaves the update to the
  optimizer gate so the step is skipped but the LR still decays).
* ``StepWatchdog`` — a thread that aborts the process (``os._exit``) when a training step
  does not finish within a timeout, so a hung collective cannot wedge a node forever;
  torch.distributed's own collective timeout also applies.  Given the native RCCL
  communicator (``parallel/dp.py`` NativeComm) it also polls ``ncclCommGetAsyncError``
  every tick and, on an error (dead peer, transport failure), aborts the communicator —
  which unblocks any collective stuck in the step graph — and exits with code 43.
* ``DG_FAULT=rank:step:kind`` fault injection for tests: kinds ``nan`` (poison the loss),
  ``raise`` (exception), ``hang`` (sleep past the watchdog), ``exit`` (hard exit code 17).
"""
from __future__ import annotations

import os
import threading
import time
from typing import Optional

import numpy as np


class NonFiniteLoss(RuntimeError):
    pass


def parse_fault(spec: Optional[str] = None):
    spec = spec if spec is not None else os.environ.get("DG_FAULT", "")
    if not spec:
        return None
    rank, step, kind = spec.split(":")
    return int(rank), int(step), kind


def maybe_inject(rank: int, step: int, spec=None):
    """Returns 'nan' when the loss of this step must be poisoned; raises / hangs / exits for
    the other kinds."""
    f = parse_fault(spec) if spec is None or isinstance(spec, str) else spec
    if not f or f[0] != rank or f[1] != step:
        return None
    kind = f[2]
    if kind == "raise":
        raise RuntimeError(f"DG_FAULT injected exception at rank {rank} step {step}")
    if kind == "hang":
        time.sleep(3600)
    if kind == "exit":
        os._exit(17)
    return kind


def dump_batch(batch, step: int, dump_dir: str = ".") -> Optional[str]:
    if batch is None:
        return None
    path = os.path.join(dump_dir, f"bad_batch_{step}.npz")
    np.savez(path, *[np.asarray(b) for b in batch])
    return path


def check_finite(loss_sum: float, step: int, policy: str, batch=None, dump_dir: str = "."):
    """True if the loss is finite.  Policies ``skip`` / ``guard`` return False (the device
    gate skipped the update; ``guard`` raises later through SkipGuard); ``raise`` dumps the
    batch and raises."""
    if np.isfinite(loss_sum):
        return True
    if policy in ("skip", "guard"):
        return False
    dump_batch(batch, step, dump_dir)
    raise NonFiniteLoss(f"non-finite loss {loss_sum} at step {step}")


class SkipGuard:
    """nan_policy ``guard``: the device gate skips updates on its own (no host sync per
    step); at the host's log-interval syncs this reads the device's skipped-step counter
    and raises NonFiniteLoss once ``max_skips`` consecutive steps were skipped — whole check
    windows of skipped steps add up, a window with any applied step resets the run (a skip
    run that started mid-window is counted from the next window: never a false alarm)."""

    def __init__(self, max_skips: int, bad_now: int = 0):
        self.max_skips = max(1, int(max_skips))
        self.prev = bad_now
        self.since = 0
        self.run = 0

    def step(self):
        self.since += 1

    def check(self, bad_now: int, step: int) -> None:
        d = bad_now - self.prev
        self.run = self.run + d if (d == self.since and d > 0) else 0
        self.prev, self.since = bad_now, 0
        if self.run >= self.max_skips:
            raise NonFiniteLoss(f"{self.run} consecutive training steps were skipped for "
                                f"non-finite loss / gradients (last at step {step})")


class StepWatchdog:
    def __init__(self, timeout_s: float, on_timeout=None, comm=None, on_comm_error=None,
                 poll_s: float = 1.0):
        self.timeout = timeout_s
        self.on_timeout = on_timeout
        self.comm = comm
        self.on_comm_error = on_comm_error
        self.poll = poll_s
        self.comm_error = ""
        self._beat = time.monotonic()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="dg-step-watchdog")
        self._t.start()

    def beat(self):
        self._beat = time.monotonic()

    def _run(self):
        tick = min(self.poll, self.timeout / 4) if self.timeout > 0 else self.poll
        while not self._stop.wait(tick):
            if self.comm is not None:
                err = self.comm.async_error()
                if err:
                    self.comm_error = err
                    if self.on_comm_error:
                        self.on_comm_error(err)
                        return
                    print(f"[watchdog] communicator error: {err}: aborting", flush=True)
                    self.comm.abort()
                    os._exit(43)
            if self.timeout > 0 and time.monotonic() - self._beat > self.timeout:
                if self.on_timeout:
                    self.on_timeout()
                else:
                    print(f"[watchdog] no step progress for {self.timeout}s: aborting", flush=True)
                    os._exit(42)

    def stop(self):
        self._stop.set()


class PhaseGuard:
    """Per-rank hang guard for a run made of named phases (bench.py: ``comm`` set-up,
    ``capture``, ``warmup``, ``timed``, ``report``).  ``phase(name, limit_s)`` arms a
    deadline; a thread that outlives it writes ``hang:<name>:<comm kind>`` to
    ``<status_dir>/rank<r>`` (read by the launcher; ``set_comm`` records the kind), reports on stderr and ends the process with ``os._exit(42)``,
    so a rank stuck in a collective of a dead or stuck peer exits non-zero within the bound
    instead of holding the node until an outer timeout."""

    EXIT_CODE = 42

    def __init__(self, rank: int, status_dir: Optional[str] = None, poll_s: float = 0.5):
        self.rank = rank
        self.status_dir = status_dir
        self.poll = poll_s
        self.name = "start"
        self.deadline = None
        # the communicator this rank's collectives go through ("" until chosen); the status
        # file carries it so the launcher can tell a native-communicator hang from any other
        self.comm = ""
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def phase(self, name: str, limit_s: float):
        with self._lock:
            self.name = name
            self.deadline = time.monotonic() + limit_s

    def set_comm(self, kind: str):
        with self._lock:
            self.comm = kind

    def _write_status(self, text: str):
        if self.status_dir:
            try:
                with open(os.path.join(self.status_dir, f"rank{self.rank}"), "w") as f:
                    f.write(text)
            except OSError:
                pass

    def _run(self):
        import sys
        while not self._stop.wait(self.poll):
            with self._lock:
                name, dl, comm = self.name, self.deadline, self.comm
            if dl is not None and time.monotonic() > dl:
                self._write_status(f"hang:{name}:{comm}")
                sys.stderr.write(f"[guard] rank {self.rank}: phase '{name}' exceeded its "
                                 f"time limit: exiting {self.EXIT_CODE}\n")
                sys.stderr.flush()
                os._exit(self.EXIT_CODE)

    def stop(self):
        self._stop.set()
        self._write_status("ok")
