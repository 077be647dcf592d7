import json
import os
import subprocess
import sys
import time

import pytest

from medical_segmentation_pytorch_amd.hpo import (MedianPruner, SQLiteStorage, TPESampler, TrialPruned, TrialState,
                                                  create_study)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tpe_optimizes_quadratic(tmp_path):
    st = SQLiteStorage(str(tmp_path / 's.db'), heartbeat_interval=0)
    study = create_study(st, 'q', 'maximize', sampler=TPESampler(seed=0), pruner=MedianPruner())

    def obj(t):
        x = t.suggest_float('x', -5, 5)
        lr = t.suggest_float('lr', 1e-4, 1e-1, log=True)
        c = t.suggest_categorical('opt', ['sgd', 'adam'])
        return -(x - 2) ** 2 - (0 if c == 'adam' else 1) - abs(lr - 1e-2)

    study.optimize(obj, n_trials=60)
    assert len(study.trials) == 60
    assert study.best_value > -1.1 and abs(study.best_params['x'] - 2) < 0.5
    # TPE beats its own random start-up phase
    vals = [t.value for t in study.trials]
    assert max(vals[10:]) >= max(vals[:10])


def test_median_pruner(tmp_path):
    st = SQLiteStorage(str(tmp_path / 'p.db'), heartbeat_interval=0)
    study = create_study(st, 'p', 'maximize', pruner=MedianPruner(n_startup_trials=2))

    def obj(t):
        good = t.number < 3
        for step in range(3):
            t.report(1.0 if good else 0.0, step)
            if t.should_prune():
                raise TrialPruned()
        return 1.0 if good else 0.0

    study.optimize(obj, n_trials=6)
    assert len(study.get_trials(states=[TrialState.PRUNED])) == 3
    assert len(study.get_trials(states=[TrialState.COMPLETE])) == 3


def test_stale_heartbeat_is_retried(tmp_path):
    st = SQLiteStorage(str(tmp_path / 'h.db'), heartbeat_interval=0, grace_period=0.2)
    study = create_study(st, 'h', 'maximize')
    t = study.ask()
    t.suggest_float('a', 0, 1)            # a "crashed" trial: never told, never heartbeats
    time.sleep(0.4)
    t2 = study.ask()                      # claim -> stale RUNNING trial failed + re-enqueued -> taken
    states = {x.number: x.state for x in study.trials}
    assert states[0] == TrialState.FAIL
    assert t2.suggest_float('a', 0, 1) == t.params['a']   # retried with the same params


@pytest.mark.slow
def test_optuna_search_cli(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, os.path.join(ROOT, 'optuna_search.py'), '--storage', f'sqlite:///{tmp_path}/o.db',
           '--num-trial', '2', '--save_dir', str(tmp_path / 'save'), '--dataset', 'synthetic',
           '--synthetic_num', '8', '4', '4', '--synthetic_size', '64', '--crop_size', '64', '--total_epoch', '1',
           '--warmup_epochs', '0', '--train_bs', '4', '--base_workers', '0', '--base_channel', '8',
           '--no_progress_bar', '--data_root', str(tmp_path / 'data')]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.load(open(tmp_path / 'save' / 'optuna_results.json'))
    assert res['finished_trials'] == 2 and 0 <= res['value'] <= 1
    assert set(json.load(open(tmp_path / 'save' / 'trial_scores.json'))) == {'0', '1'}


@pytest.mark.slow
def test_concurrent_trial_groups_gloo(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr', '127.0.0.1', '--master-port', str(29500 + os.getpid() % 1000),
           os.path.join(ROOT, 'optuna_search.py'), '--ranks-per-trial', '1', '--storage',
           f'sqlite:///{tmp_path}/c.db', '--num-trial', '2', '--save_dir', str(tmp_path / 'save'), '--dataset',
           'synthetic', '--synthetic_num', '8', '4', '4', '--synthetic_size', '64', '--crop_size', '64',
           '--total_epoch', '1', '--warmup_epochs', '0', '--train_bs', '4', '--base_workers', '0', '--base_channel',
           '8', '--no_progress_bar', '--data_root', str(tmp_path / 'data')]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.load(open(tmp_path / 'save' / 'optuna_results.json'))
    assert res['finished_trials'] >= 2


@pytest.mark.slow
def test_two_concurrent_two_rank_trial_groups_gloo(tmp_path):
    """World 4 split into two 2-rank trial groups (``--ranks-per-trial 2``): each group trains its trial with
    DDP over its own sub-group, both write to the shared study (reference optuna_search.py over 4 GPUs)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=4',
           '--master-addr', '127.0.0.1', '--master-port', str(30500 + os.getpid() % 1000),
           os.path.join(ROOT, 'optuna_search.py'), '--ranks-per-trial', '2', '--storage',
           f'sqlite:///{tmp_path}/c4.db', '--num-trial', '2', '--save_dir', str(tmp_path / 'save'), '--dataset',
           'synthetic', '--synthetic_num', '8', '4', '4', '--synthetic_size', '64', '--crop_size', '64',
           '--total_epoch', '1', '--warmup_epochs', '0', '--train_bs', '2', '--base_workers', '0', '--base_channel',
           '8', '--no_progress_bar', '--data_root', str(tmp_path / 'data')]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.load(open(tmp_path / 'save' / 'optuna_results.json'))
    assert res['finished_trials'] >= 2
