"""Tracing / observability for the training loop (SURVEY §5 "Tracing / profiling"; the reference has
none beyond ``tools/test_speed.py:30-58`` wall-clock timing and ``app.py:20-78``'s stage timer).

* :func:`trace_range` -- a roctx range (``torch.cuda.nvtx`` is roctx on ROCm) around a step phase,
  so ``rocprofv3 --marker-trace`` timelines show ``train/step``, ``val/forward`` ... next to the HIP
  kernels.  Free when tracing is off.
* :class:`PhaseTimer` -- HIP-event timing of named phases accumulated on the device (no per-step
  host sync); :meth:`PhaseTimer.summary` syncs once and returns mean ms per phase.
* :class:`ThroughputMeter` -- images/sec over a sliding window of host-synchronised intervals.

Enable with ``config.trace = True`` (CLI ``--trace``) or ``MSP_TRACE=1``.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict, deque

import torch

_ENABLED = os.environ.get('MSP_TRACE', '0') == '1'


def set_tracing(on: bool):
    global _ENABLED
    _ENABLED = bool(on)


def tracing_enabled() -> bool:
    return _ENABLED


def _roctx():
    if not torch.cuda.is_available():
        return None
    try:
        return torch.cuda.nvtx   # roctx-backed on ROCm builds of torch
    except Exception:            # pragma: no cover
        return None


@contextlib.contextmanager
def trace_range(name: str):
    """roctx range push/pop around the block when tracing is on (no-op otherwise)."""
    if not _ENABLED:
        yield
        return
    tx = _roctx()
    if tx is not None:
        tx.range_push(name)
    try:
        yield
    finally:
        if tx is not None:
            tx.range_pop()


class PhaseTimer:
    """Per-phase GPU time from HIP events, read back lazily (one sync in :meth:`summary`)."""

    def __init__(self, enabled=True):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending = defaultdict(list)
        self._done = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name):
        if not self.enabled:
            with trace_range(name):
                yield
            return
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        with trace_range(name):
            yield
        b.record()
        self._pending[name].append((a, b))

    def summary(self):
        if self.enabled:
            torch.cuda.synchronize()
        for k, evs in self._pending.items():
            self._done[k].extend(a.elapsed_time(b) for a, b in evs)
        self._pending.clear()
        return {k: sum(v) / len(v) for k, v in self._done.items() if v}

    def reset(self):
        self._pending.clear()
        self._done.clear()


class ThroughputMeter:
    """images/sec over the last ``window`` host-synchronised intervals."""

    def __init__(self, window=20):
        self.window = deque(maxlen=window)
        self._t = None
        self._n = 0

    def add(self, n_images):
        self._n += n_images

    def mark(self):
        """Call right after a host sync (e.g. the log flush); returns the windowed images/sec."""
        now = time.perf_counter()
        if self._t is not None and self._n:
            self.window.append((self._n, now - self._t))
        self._t, self._n = now, 0
        return self.rate()

    def rate(self):
        n = sum(a for a, _ in self.window)
        t = sum(b for _, b in self.window)
        return n / t if t > 0 else 0.0
