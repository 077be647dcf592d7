"""Hyper-parameter search -- reference ``optuna_search.py:14-94``.

    python optuna_search.py                                      # single process
    torchrun --nproc_per_node=8 optuna_search.py                 # every trial on all 8 GPUs (reference)
    torchrun --nproc_per_node=8 optuna_search.py --ranks-per-trial 2   # 4 concurrent trials x 2 GPUs

Uses the native :mod:`medical_segmentation_pytorch_amd.hpo` (TPE sampler, median pruner, SQLite study
with 1 s heartbeats and failed-trial retry); ``--backend optuna`` uses optuna when it is installed.
Writes ``{save_dir}/trial_scores.json`` and ``{save_dir}/optuna_results.json`` like the reference.
"""
import argparse
import json
import os
import warnings

import torch
import torch.distributed as dist

from medical_segmentation_pytorch_amd.configs import OptunaConfig, load_parser
from medical_segmentation_pytorch_amd.core import SegTrainer
from medical_segmentation_pytorch_amd.hpo import DistributedTrial, TrialPruned, TrialState, create_study
from medical_segmentation_pytorch_amd.hpo import SQLiteStorage, make_trial_groups

warnings.filterwarnings('ignore')


class OptunaTrainer(SegTrainer):
    def __init__(self, config, trial):
        super().__init__(config)
        self.trial = trial

    def validate(self, config, loader, *args, **kwargs):
        val_score = super().validate(config, loader, *args, **kwargs)
        if loader is self.val_loader and not kwargs.get('val_best', False) and not (args and args[0]):
            self.after_validate(val_score)
        return val_score

    def after_validate(self, val_score):
        self.trial.report(float(val_score), self.cur_epoch)
        if self.trial.should_prune():
            raise TrialPruned()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--ranks-per-trial', type=int, default=0, help='0 = the whole world per trial')
    ap.add_argument('--storage', default='sqlite:///optuna.db')
    ap.add_argument('--num-trial', type=int, default=None)
    ap.add_argument('--backend', choices=['native', 'optuna'], default='native')
    args, rest = ap.parse_known_args(argv)

    local_rank = int(os.getenv('LOCAL_RANK', -1))
    ddp = local_rank != -1
    if ddp and not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank)
        dist.init_process_group('nccl' if torch.cuda.is_available() else 'gloo', init_method='env://')
    base = load_parser(OptunaConfig().init_dependent_config(), rest)
    num_trial = args.num_trial or base.num_trial
    save_root = base.save_dir
    os.makedirs(save_root, exist_ok=True)

    group, gidx, leader = None, 0, True
    if ddp:
        k = args.ranks_per_trial or dist.get_world_size()
        group, gidx, _n, leader_rank = make_trial_groups(k)
        leader = dist.get_rank() == leader_rank
        # synthetic data once, before the trial groups start
        if base.synthetic_data or base.dataset == 'synthetic':
            from medical_segmentation_pytorch_amd.datasets import _ensure_data
            _ensure_data(base)          # world rank 0 writes, every rank waits at a WORLD barrier

    study = None
    if leader:
        if args.backend == 'optuna':
            import optuna
            storage = optuna.storages.RDBStorage(args.storage, heartbeat_interval=1,
                                                 failed_trial_callback=optuna.storages.RetryFailedTrialCallback())
            study = optuna.create_study(storage=storage, study_name=base.study_name,
                                        direction=base.study_direction, load_if_exists=True)
        else:
            storage = SQLiteStorage(args.storage, heartbeat_interval=1)
            study = create_study(storage=storage, study_name=base.study_name, direction=base.study_direction)
        print(f'[group {gidx}] Using native HPO to perform hyperparameter search.\n', flush=True)

    scores_path = f'{save_root}/trial_scores.json'

    def run_trial(trial):
        dtrial = DistributedTrial(trial, group) if ddp else trial
        config = OptunaConfig()
        config.init_dependent_config()
        config = load_parser(config, rest)
        config.dist_group = group
        if config.save_every_trial:
            config.save_dir = f'{save_root}/trial_{dtrial.number}'
        if leader:
            print(f'Running trial: {dtrial.number}...\n', flush=True)
        config.get_trial_params(dtrial)
        trainer = OptunaTrainer(config, dtrial)
        best = float(trainer.run(config))
        if leader:
            scores = json.load(open(scores_path)) if os.path.isfile(scores_path) else {}
            scores[str(dtrial.number)] = best
            with open(scores_path, 'w') as f:
                json.dump(scores, f, indent=1)
        return best

    # each group loops: leader claims trials until the study holds num_trial finished/running trials
    while True:
        go = None
        if leader:
            n_done = len([t for t in study.trials if t.state != TrialState.WAITING])
            go = n_done < num_trial
        if ddp:
            obj = [go]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0), group=group)
            go = obj[0]
        if not go:
            break
        trial = study.ask() if leader else None
        try:
            value = run_trial(trial)
            if leader:
                study.tell(trial, value, TrialState.COMPLETE)
        except TrialPruned:
            if leader:
                iv = trial.intermediate_values
                study.tell(trial, iv[max(iv)] if iv else None, TrialState.PRUNED)

    if ddp:
        dist.barrier()
    if (not ddp or dist.get_rank() == 0) and study is not None:
        best = study.best_trial
        res = {'params': best.params, 'value': best.value, 'finished_trials': len(study.trials),
               'pruned_trials': len(study.get_trials(states=[TrialState.PRUNED])),
               'completed_trials': len(study.get_trials(states=[TrialState.COMPLETE]))}
        with open(f'{save_root}/optuna_results.json', 'w') as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res, indent=1))
    if ddp:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
