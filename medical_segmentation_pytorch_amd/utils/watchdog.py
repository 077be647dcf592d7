"""Failure detection for long runs (SURVEY §5 "Failure detection / elastic"; the reference only has
optuna's trial heartbeat, ``optuna_search.py:70``).

* :class:`StepWatchdog` -- a daemon thread fed by :meth:`StepWatchdog.beat` once per iteration.  If no
  beat arrives for ``timeout_s`` (a hung collective, a wedged data source) it writes every thread's
  stack (``faulthandler``) to ``save_dir/watchdog_rank{r}.log`` and, with ``abort=True``, exits the
  process with code 75 so ``torchrun --max-restarts N`` relaunches the job, which auto-resumes from
  ``save_dir/last.pth`` (``configs.load_ckpt_path``).
* :func:`check_finite` -- raises :class:`NonFiniteLoss` on NaN/Inf losses at the (already host-synced)
  log flush, so a diverged run stops instead of training on garbage.
* :func:`process_group_timeout` -- the ``timeout`` handed to ``init_process_group`` (config
  ``dist_timeout_min``), so a dead peer surfaces as an error instead of a silent hang.
"""
from __future__ import annotations

import datetime
import faulthandler
import math
import os
import sys
import threading
import time


class NonFiniteLoss(RuntimeError):
    pass


def check_finite(values, itr=None):
    for v in values:
        if not math.isfinite(float(v)):
            raise NonFiniteLoss(f'non-finite training loss {v} at iteration {itr}')


def process_group_timeout(config):
    minutes = getattr(config, 'dist_timeout_min', None)
    return datetime.timedelta(minutes=float(minutes)) if minutes else None


class StepWatchdog:
    def __init__(self, timeout_s=900.0, log_dir='.', rank=0, abort=True, poll_s=None):
        self.timeout_s = float(timeout_s)
        self.log_path = os.path.join(log_dir, f'watchdog_rank{rank}.log')
        self.abort = abort
        self.poll_s = poll_s if poll_s is not None else max(min(self.timeout_s / 4, 30.0), 0.05)
        self._last = time.monotonic()
        self._stop = threading.Event()
        self.fired = False
        self._thread = threading.Thread(target=self._run, daemon=True, name='msp-watchdog')

    def start(self):
        self._last = time.monotonic()
        self._thread.start()
        return self

    def beat(self):
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=5)

    def _run(self):
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle < self.timeout_s:
                continue
            self.fired = True
            os.makedirs(os.path.dirname(self.log_path) or '.', exist_ok=True)
            with open(self.log_path, 'a') as f:
                f.write(f'[watchdog] no training progress for {idle:.0f}s (limit {self.timeout_s:.0f}s); '
                        f'stacks:\n')
                f.flush()
                faulthandler.dump_traceback(file=f, all_threads=True)
            print(f'[watchdog] stalled {idle:.0f}s, stacks in {self.log_path}', file=sys.stderr, flush=True)
            if self.abort:
                os._exit(75)
            return
