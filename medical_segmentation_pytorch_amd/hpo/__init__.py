"""Native hyper-parameter optimisation (TPE + median pruning + SQLite study with heartbeat/retry,
distributed and concurrent trials) -- replaces optuna/optuna-integration for ``optuna_search.py``."""
from .distributed import DistributedTrial, make_trial_groups  # noqa: F401
from .storage import SQLiteStorage  # noqa: F401
from .study import (MedianPruner, NopPruner, RandomSampler, Study, TPESampler, Trial, TrialPruned,  # noqa: F401
                    TrialState, create_study)
