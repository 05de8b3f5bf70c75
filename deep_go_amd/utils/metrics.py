"""Console lines + JSONL metrics sink (+ optional pluggable remote sink).

Console lines keep the reference's wording so runs are easy to compare
(``train.lua:122,126,139``, ``data.lua:57``, ``experiments.lua:84``):
  ``training <ema> (samples per second X)``
  ``validation at iteration N: cost=..., accuracy=...``
  ``total samples per second X``
The reference also POSTed one row per run to a Google Form with ``curl``
(``logging.lua:13-24``); here remote logging is an explicit opt-in sink and never runs by
default (no network access is assumed).
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Callable, Dict, List, Optional


class MetricsSink:
    def __init__(self, path: Optional[str] = None, echo: bool = True, rank: int = 0,
                 remote: Optional[Callable[[Dict[str, Any]], None]] = None):
        self.path = path
        self.echo = echo and rank == 0
        self.rank = rank
        self.remote = remote
        self._f = open(path, "a") if (path and rank == 0) else None

    def line(self, text: str):
        if self.echo:
            print(text, flush=True)

    def record(self, **kv):
        kv.setdefault("time", time.time())
        if self._f:
            self._f.write(json.dumps(kv) + "\n")
            self._f.flush()

    def run_summary(self, row: Dict[str, Any]):
        """The reference's per-run log row (logging.lua:3-25) — to JSONL, and to the remote
        sink only if one was configured."""
        self.record(kind="run", **row)
        if self.remote is not None and self.rank == 0:
            self.remote(row)

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


def http_form_sink(url: str, field_map: Dict[str, str]):
    """Opt-in equivalent of the reference's Google-Form POST (multipart form fields)."""
    def post(row: Dict[str, Any]):
        import urllib.parse
        import urllib.request
        data = urllib.parse.urlencode({field_map.get(k, k): str(v) for k, v in row.items()})
        urllib.request.urlopen(urllib.request.Request(url, data=data.encode()), timeout=10)
    return post


def read_jsonl(path: str) -> List[Dict[str, Any]]:
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line:
                out.append(json.loads(line))
    return out
