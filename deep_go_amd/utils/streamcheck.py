"""Cross-stream hand-off checks (``DG_CHECK_STREAMS=1``; SURVEY §5.2 "assert the event ordering
between the compute stream and the comm stream").

The training step runs up to four HIP streams: the compute stream, the backward's side
stream (bias-gradient partials, the first layer's gradient chain), the DP comm stream (bucket
all-reduces) and the input load stream (prefetch).  Every hand-off between two of them is a
``wait_stream`` / ``wait_event`` in ``HipGoNet`` / ``GradBucketer``.  This checker brackets
each hand-off with two timing events that are recorded SEPARATELY from the wait itself:

  * ``produce(name, stream)`` — on the producer stream, right after the last launch whose
    output the consumer reads;
  * ``consume(name, stream)`` — on the consumer stream, right before the first launch that
    reads it.

``check()`` (after an eager step: events inside a hipGraph capture are skipped) synchronizes
and asserts, for every pair, that the producer's event completed no later than the consumer's
(``elapsed_time(produce, consume) >= 0``).

What this verifies, and what it does not: the brackets sit at the hand-offs the code DECLARES
(each wait_stream / wait_event has its produce / consume pair), so the check confirms that
each declared wait is placed after the producer's launches and before the consumer's, and
that HIP honours it.  A hand-off that has no wait at all also has no bracket and is not seen
here — that class of bug is covered by the bit-exact comparisons of the same step run
serialized (``AMD_SERIALIZE_KERNEL=3``) and unserialized (tests/test_model_gpu.py
test_stream_handoffs_checked_and_serialized_run_bit_identical) instead.  The reference has no concurrency at all
(``/root/reference/data.lua:82-96``: every mutation runs on the main Lua thread), so these
orderings are the new build's own risk.
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

import torch


def enabled() -> bool:
    return os.environ.get("DG_CHECK_STREAMS", "0") == "1"


class StreamCheck:
    def __init__(self):
        self._open: Dict[str, torch.cuda.Event] = {}
        self.pairs: List[Tuple[str, torch.cuda.Event, torch.cuda.Event]] = []
        self.checked = 0          # pairs verified so far (tests assert the checker ran)

    @staticmethod
    def _capturing() -> bool:
        return torch.cuda.is_current_stream_capturing()

    def produce(self, name: str, stream) -> None:
        if self._capturing():
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        self._open[name] = e

    def consume(self, name: str, stream) -> None:
        if self._capturing():
            return
        p = self._open.pop(name, None)
        if p is None:
            raise AssertionError(f"stream check: consume({name!r}) without a produce()")
        c = torch.cuda.Event(enable_timing=True)
        c.record(stream)
        self.pairs.append((name, p, c))

    def check(self) -> int:
        """Synchronize and verify every recorded hand-off; returns how many were checked."""
        if not self.pairs:
            return 0
        torch.cuda.synchronize()
        bad = []
        for name, p, c in self.pairs:
            dt = p.elapsed_time(c)       # ms from the producer's event to the consumer's
            if dt < 0.0:
                bad.append(f"{name}: consumer ran {-dt * 1e3:.1f} us before the producer ended")
        n = len(self.pairs)
        self.pairs.clear()
        if self._open:
            bad.append(f"unconsumed hand-offs: {sorted(self._open)}")
            self._open.clear()
        if bad:
            raise AssertionError("stream-ordering violations:\n  " + "\n  ".join(bad))
        self.checked += n
        return n
