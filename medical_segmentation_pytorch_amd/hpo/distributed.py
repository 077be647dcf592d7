"""Distributed trials: the group leader owns the real trial; every suggestion / prune decision is
broadcast to the other ranks of the trial's process group (the reference uses optuna-integration's
``TorchDistributedTrial``, ``optuna_search.py:49``; non-main ranks pass ``None``).

``make_trial_groups(k)`` splits the world into groups of ``k`` consecutive ranks so several trials
train concurrently (e.g. 4 trials x 2 MI355X each) -- all sharing one SQLite study on the node.
"""
from __future__ import annotations

import torch.distributed as dist

from .study import TrialPruned


class DistributedTrial:
    def __init__(self, trial, group=None, src=None):
        self.group = group
        self.src = src if src is not None else (dist.get_global_rank(group, 0) if group is not None else 0)
        self._trial = trial
        self.number = self._bcast(trial.number if trial is not None else None)

    def _bcast(self, value):
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return value
        obj = [value]
        dist.broadcast_object_list(obj, src=self.src, group=self.group)
        return obj[0]

    def _is_src(self):
        return self._trial is not None

    def suggest_categorical(self, name, choices):
        return self._bcast(self._trial.suggest_categorical(name, choices) if self._is_src() else None)

    def suggest_float(self, name, low, high, log=False, step=None):
        return self._bcast(self._trial.suggest_float(name, low, high, log=log, step=step) if self._is_src() else None)

    def suggest_int(self, name, low, high, log=False):
        return self._bcast(self._trial.suggest_int(name, low, high, log=log) if self._is_src() else None)

    def report(self, value, step):
        if self._is_src():
            self._trial.report(value, step)

    def should_prune(self):
        return bool(self._bcast(self._trial.should_prune() if self._is_src() else None))

    @property
    def params(self):
        return self._bcast(dict(self._trial.params) if self._is_src() else None)


def make_trial_groups(ranks_per_trial):
    """Returns (my_group, my_group_index, n_groups, leader_global_rank).  Every rank must call it."""
    world, rank = dist.get_world_size(), dist.get_rank()
    assert world % ranks_per_trial == 0, 'world size must be a multiple of ranks_per_trial'
    n = world // ranks_per_trial
    from ..runtime.engine import register_stat_group
    mine = None
    for g in range(n):
        ranks = list(range(g * ranks_per_trial, (g + 1) * ranks_per_trial))
        pg = dist.new_group(ranks)
        spg = dist.new_group(ranks)      # the trial's SyncBN-statistics communicator
        if rank in ranks:
            register_stat_group(pg, spg)
            mine = (pg, g, n, ranks[0])
    return mine


__all__ = ['DistributedTrial', 'TrialPruned', 'make_trial_groups']
