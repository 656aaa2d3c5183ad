"""Structured JSONL event log + profiler ranges (SURVEY 5.1 / 5.5 "new").

``EventLog`` appends one JSON object per line (``{"ts", "rank", "event", ...}``)
for trial start/end, per-epoch metrics, throughput samples and per-rank step
timing; it is process-safe (O_APPEND, one ``write`` per line) so trial workers
and DP ranks can share a file.  ``FEATURENET_EVENTS=<path>`` enables the
default log used by the trainer / trial scheduler.

``prange(name)`` marks a region for rocprofv3 (``--marker-trace``) through
``torch.cuda.nvtx`` which PyTorch-ROCm maps onto roctx; it is a no-op on CPU.
"""
from __future__ import annotations

import contextlib
import json
import os
import time


class EventLog:
    def __init__(self, path: str | None):
        self.path = path
        self.rank = int(os.environ.get("RANK", "0"))
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def emit(self, event: str, **fields) -> None:
        if not self.path:
            return
        rec = {"ts": time.time(), "rank": self.rank, "pid": os.getpid(), "event": event, **fields}
        line = (json.dumps(rec, default=str) + "\n").encode()
        fd = os.open(self.path, os.O_WRONLY | os.O_APPEND | os.O_CREAT, 0o644)
        try:
            os.write(fd, line)
        finally:
            os.close(fd)

    @contextlib.contextmanager
    def span(self, event: str, **fields):
        t0 = time.time()
        self.emit(f"{event}_start", **fields)
        try:
            yield
        finally:
            self.emit(f"{event}_end", seconds=time.time() - t0, **fields)


def read_events(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]


_DEFAULT: EventLog | None = None


def default_log() -> EventLog:
    global _DEFAULT
    if _DEFAULT is None or _DEFAULT.path != os.environ.get("FEATURENET_EVENTS"):
        _DEFAULT = EventLog(os.environ.get("FEATURENET_EVENTS"))
    return _DEFAULT


@contextlib.contextmanager
def prange(name: str):
    """Profiler range visible to rocprofv3 marker tracing (roctx) when on GPU."""
    import torch

    active = torch.cuda.is_available()
    if active:
        torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        if active:
            torch.cuda.nvtx.range_pop()
