"""Auxiliary subsystems: tracing, failure detection (watchdog, non-finite loss guard,
process-group timeout), run on CPU."""
import math
import os
import time

import pytest
import torch

from medical_segmentation_pytorch_amd.utils.tracing import PhaseTimer, ThroughputMeter, set_tracing, trace_range
from medical_segmentation_pytorch_amd.utils.watchdog import (NonFiniteLoss, StepWatchdog, check_finite,
                                                             process_group_timeout)


def test_watchdog_fires_and_dumps_stacks(tmp_path):
    wd = StepWatchdog(0.2, str(tmp_path), rank=3, abort=False, poll_s=0.05).start()
    time.sleep(0.8)
    wd.stop()
    assert wd.fired
    log = (tmp_path / 'watchdog_rank3.log').read_text()
    assert 'no training progress' in log and 'File' in log    # faulthandler stack lines


def test_watchdog_quiet_while_beating(tmp_path):
    wd = StepWatchdog(0.3, str(tmp_path), abort=False, poll_s=0.05).start()
    for _ in range(12):
        time.sleep(0.05)
        wd.beat()
    wd.stop()
    assert not wd.fired and not (tmp_path / 'watchdog_rank0.log').exists()


def test_non_finite_guard_and_pg_timeout():
    check_finite([0.5, 1.0])
    with pytest.raises(NonFiniteLoss):
        check_finite([0.5, math.nan], itr=7)
    with pytest.raises(NonFiniteLoss):
        check_finite([math.inf])

    class C:
        dist_timeout_min = 2
    assert process_group_timeout(C()).total_seconds() == 120
    C.dist_timeout_min = None
    assert process_group_timeout(C()) is None


def test_tracing_cpu_noop_and_meters():
    set_tracing(True)
    try:
        with trace_range('x'):
            y = torch.ones(3).sum()
        t = PhaseTimer()
        with t.phase('p'):
            y = y + 1
        assert t.summary() == {}          # no GPU: timing disabled, ranges still usable
    finally:
        set_tracing(False)
    m = ThroughputMeter()
    m.mark()
    m.add(32)
    time.sleep(0.05)
    r = m.mark()
    assert 0 < r < 32 / 0.04


def test_trainer_with_trace_and_watchdog(tmp_path):
    """A CPU training run with tracing and the watchdog on completes and leaves no watchdog log."""
    from medical_segmentation_pytorch_amd.configs import MyConfig
    from medical_segmentation_pytorch_amd.core import SegTrainer
    c = MyConfig()
    c.data_root, c.save_dir = str(tmp_path / 'data'), str(tmp_path / 'save')
    c.crop_size, c.train_bs, c.val_bs, c.base_workers = 64, 4, 2, 0
    c.synthetic_data, c.synthetic_num, c.synthetic_size = True, (8, 4, 4), 64
    c.progress_bar, c.model, c.base_channel, c.total_epoch, c.warmup_epochs = False, 'unet', 8, 1, 1
    c.trace, c.watchdog_timeout_s = True, 120
    c.init_dependent_config()
    c.DDP, c.gpu_num, c.num_workers = False, 1, 0
    t = SegTrainer(c)
    score = t.run(c)
    assert 0.0 <= float(score) <= 1.0
    assert not os.path.exists(os.path.join(c.save_dir, 'watchdog_rank0.log'))
    set_tracing(False)
