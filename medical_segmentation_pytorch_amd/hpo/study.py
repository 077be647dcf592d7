"""Native hyper-parameter search (optuna is not installable here) with the API surface the reference
uses (``optuna_search.py``): ``create_study``, ``Study.optimize``, ``Trial.suggest_*``, ``report``,
``should_prune``, ``TrialPruned``, ``TrialState``, ``best_trial``, ``get_trials(states=...)``,
a TPE sampler (optuna's defaults: 10 random start-up trials, gamma(n) = min(ceil(0.1 n), 25), Parzen
estimators with a prior) and a median pruner.  If ``optuna`` IS importable, ``optuna_search.py``
can use it instead (``--backend optuna``).
"""
from __future__ import annotations

import gc
import math
import random
import threading
from enum import Enum

from .storage import SQLiteStorage


class TrialPruned(Exception):
    pass


class TrialState(str, Enum):
    RUNNING = 'RUNNING'
    COMPLETE = 'COMPLETE'
    PRUNED = 'PRUNED'
    FAIL = 'FAIL'
    WAITING = 'WAITING'


class FrozenTrial:
    def __init__(self, d):
        self.number, self.value, self.params = d['number'], d['value'], d['params']
        self.state = TrialState(d['state'])
        self.intermediate_values = d['intermediate']
        self.distributions = d['dists']
        self.user_attrs = d['attrs']

    def __repr__(self):
        return f'FrozenTrial(number={self.number}, state={self.state.value}, value={self.value})'


# ----------------------------------------------------------------------------------------------- samplers
class RandomSampler:
    def __init__(self, seed=None):
        self.rng = random.Random(seed)

    def sample(self, study, name, dist):
        return _sample_prior(self.rng, dist)


def _sample_prior(rng, dist):
    kind = dist['type']
    if kind == 'categorical':
        return rng.choice(dist['choices'])
    lo, hi = dist['low'], dist['high']
    if kind == 'int':
        return rng.randint(int(lo), int(hi))
    if dist.get('log'):
        return math.exp(rng.uniform(math.log(lo), math.log(hi)))
    return rng.uniform(lo, hi)


class TPESampler:
    """Univariate Tree-structured Parzen Estimator (Bergstra et al. 2011)."""

    def __init__(self, n_startup_trials=10, n_ei_candidates=24, seed=None, prior_weight=1.0):
        self.n_startup = n_startup_trials
        self.n_cand = n_ei_candidates
        self.rng = random.Random(seed)
        self.prior_weight = prior_weight

    @staticmethod
    def gamma(n):
        return min(int(math.ceil(0.1 * n)), 25)

    def sample(self, study, name, dist):
        hist = [t for t in study.trials_cached() if t.state in (TrialState.COMPLETE, TrialState.PRUNED)
                and name in t.params]
        if len(hist) < self.n_startup:
            return _sample_prior(self.rng, dist)
        sign = -1.0 if study.direction == 'maximize' else 1.0

        def score(t):   # lower is better; pruned trials use their last intermediate value, ranked after complete
            if t.state == TrialState.COMPLETE and t.value is not None:
                return (0, sign * t.value)
            iv = t.intermediate_values
            last = iv[max(iv, key=lambda k: int(k))] if iv else None
            return (1, sign * last if last is not None else float('inf'))
        hist.sort(key=score)
        ng = self.gamma(len(hist))
        good = [t.params[name] for t in hist[:ng]]
        bad = [t.params[name] for t in hist[ng:]]
        if dist['type'] == 'categorical':
            ch = dist['choices']
            wg = [self.prior_weight + sum(1 for v in good if v == c) for c in ch]
            wb = [self.prior_weight + sum(1 for v in bad if v == c) for c in ch]
            sg, sb = sum(wg), sum(wb)
            ratio = [(a / sg) / (b / sb) for a, b in zip(wg, wb)]
            cands = [self.rng.choices(ch, weights=wg)[0] for _ in range(self.n_cand)]
            return max(cands, key=lambda c: ratio[ch.index(c)])
        log = bool(dist.get('log'))
        lo, hi = float(dist['low']), float(dist['high'])
        tf = (lambda v: math.log(v)) if log else (lambda v: float(v))
        tlo, thi = tf(lo), tf(hi)
        lg, lb = self._parzen([tf(v) for v in good], tlo, thi), self._parzen([tf(v) for v in bad], tlo, thi)
        cands = [self._draw(lg, tlo, thi) for _ in range(self.n_cand)]
        best = max(cands, key=lambda x: self._logpdf(lg, x) - self._logpdf(lb, x))
        v = math.exp(best) if log else best
        if dist['type'] == 'int':
            v = int(round(v))
        return min(max(v, lo), hi)

    def _parzen(self, xs, lo, hi):
        mus = list(xs) + [0.5 * (lo + hi)]
        ws = [1.0] * len(xs) + [self.prior_weight]
        n = len(mus)
        srt = sorted(mus)
        sig = []
        for m in mus:
            i = srt.index(m)
            left = m - srt[i - 1] if i > 0 else m - lo
            right = srt[i + 1] - m if i + 1 < n else hi - m
            s = max(left, right)
            sig.append(min(max(s, (hi - lo) / min(100.0, 1.0 + n)), hi - lo))
        sig[-1] = hi - lo   # prior
        tot = sum(ws)
        return [(w / tot, m, s) for w, m, s in zip(ws, mus, sig)]

    def _draw(self, mix, lo, hi):
        w, m, s = self.rng.choices(mix, weights=[c[0] for c in mix])[0]
        for _ in range(100):
            x = self.rng.gauss(m, s)
            if lo <= x <= hi:
                return x
        return min(max(m, lo), hi)

    @staticmethod
    def _logpdf(mix, x):
        acc = 0.0
        for w, m, s in mix:
            acc += w * math.exp(-0.5 * ((x - m) / s) ** 2) / (s * math.sqrt(2 * math.pi))
        return math.log(max(acc, 1e-300))


# ----------------------------------------------------------------------------------------------- pruners
class MedianPruner:
    """Prune if the trial's best intermediate value so far is worse than the median of completed
    trials' values at the same step (optuna ``MedianPruner`` defaults)."""

    def __init__(self, n_startup_trials=5, n_warmup_steps=0, interval_steps=1):
        self.n_startup, self.n_warmup, self.interval = n_startup_trials, n_warmup_steps, interval_steps

    def prune(self, study, trial):
        steps = sorted(int(s) for s in trial.intermediate_values)
        if not steps:
            return False
        step = steps[-1]
        if step < self.n_warmup or (step - self.n_warmup) % self.interval:
            return False
        done = [t for t in study.trials_cached(refresh=True) if t.state == TrialState.COMPLETE]
        if len(done) < self.n_startup:
            return False
        vals = []
        for t in done:
            iv = {int(k): v for k, v in t.intermediate_values.items() if int(k) <= step}
            if iv:
                vals.append(iv[max(iv)])
        if not vals:
            return False
        vals.sort()
        med = vals[len(vals) // 2] if len(vals) % 2 else 0.5 * (vals[len(vals) // 2 - 1] + vals[len(vals) // 2])
        cur = [v for k, v in trial.intermediate_values.items()]
        best = max(cur) if study.direction == 'maximize' else min(cur)
        return best < med if study.direction == 'maximize' else best > med


class NopPruner:
    def prune(self, study, trial):
        return False


# ----------------------------------------------------------------------------------------------- trial / study
class Trial:
    def __init__(self, study, trial_id, number, fixed_params=None):
        self.study, self._id, self.number = study, trial_id, number
        self.params = {}
        self.intermediate_values = {}
        self._fixed = fixed_params or {}
        self._hb = None
        if study.storage.heartbeat_interval:
            self._hb_stop = threading.Event()
            self._hb = threading.Thread(target=self._beat, daemon=True)
            self._hb.start()

    def _beat(self):
        while not self._hb_stop.wait(self.study.storage.heartbeat_interval):
            try:
                self.study.storage.heartbeat(self._id)
            except Exception:
                pass

    def _stop(self):
        if self._hb is not None:
            self._hb_stop.set()
            self._hb.join(timeout=5)
            self._hb = None

    def _suggest(self, name, dist):
        if name in self.params:
            return self.params[name]
        v = self._fixed[name] if name in self._fixed else self.study.sampler.sample(self.study, name, dist)
        self.params[name] = v
        self.study.storage.set_param(self._id, name, v, dist)
        return v

    def suggest_categorical(self, name, choices):
        return self._suggest(name, {'type': 'categorical', 'choices': list(choices)})

    def suggest_float(self, name, low, high, log=False, step=None):
        v = self._suggest(name, {'type': 'float', 'low': low, 'high': high, 'log': log})
        return round(v / step) * step if step else v

    def suggest_int(self, name, low, high, log=False):
        return int(self._suggest(name, {'type': 'int', 'low': low, 'high': high, 'log': log}))

    suggest_uniform = lambda self, n, lo, hi: self.suggest_float(n, lo, hi)  # noqa: E731
    suggest_loguniform = lambda self, n, lo, hi: self.suggest_float(n, lo, hi, log=True)  # noqa: E731

    def report(self, value, step):
        value = float(value)
        self.intermediate_values[int(step)] = value
        self.study.storage.report(self._id, step, value)

    def should_prune(self):
        return self.study.pruner.prune(self.study, self)


class Study:
    def __init__(self, storage, name, direction='maximize', sampler=None, pruner=None):
        self.storage = storage
        self.study_name = name
        self._id, self.direction = storage.create_study(name, direction, load_if_exists=True)
        self.sampler = sampler or TPESampler()
        self.pruner = pruner or MedianPruner()
        self._cache = None

    def trials_cached(self, refresh=False):
        if refresh or self._cache is None:
            self._cache = [FrozenTrial(d) for d in self.storage.trials(self._id)]
        return self._cache

    @property
    def trials(self):
        return self.trials_cached(refresh=True)

    def get_trials(self, deepcopy=False, states=None):
        ts = self.trials
        return ts if states is None else [t for t in ts if t.state in set(states)]

    @property
    def best_trial(self):
        done = [t for t in self.trials if t.state == TrialState.COMPLETE and t.value is not None]
        if not done:
            raise ValueError('no completed trials')
        return (max if self.direction == 'maximize' else min)(done, key=lambda t: t.value)

    @property
    def best_value(self):
        return self.best_trial.value

    @property
    def best_params(self):
        return self.best_trial.params

    def ask(self):
        tid, num, fixed = self.storage.claim_trial(self._id)
        self.trials_cached(refresh=True)
        return Trial(self, tid, num, fixed)

    def tell(self, trial, value=None, state=TrialState.COMPLETE):
        trial._stop()
        self.storage.finish(trial._id, state.value, value)

    def optimize(self, objective, n_trials=None, callbacks=None, gc_after_trial=False, catch=()):
        n = 0
        while n_trials is None or n < n_trials:
            trial = self.ask()
            try:
                value = objective(trial)
                value = float(value.item() if hasattr(value, 'item') else value)
                self.tell(trial, value, TrialState.COMPLETE)
            except TrialPruned:
                iv = trial.intermediate_values
                self.tell(trial, iv[max(iv)] if iv else None, TrialState.PRUNED)
            except catch:
                self.tell(trial, None, TrialState.FAIL)
            except BaseException:
                self.tell(trial, None, TrialState.FAIL)
                raise
            for cb in callbacks or []:
                cb(self, trial)
            if gc_after_trial:
                gc.collect()
            n += 1


def create_study(storage=None, study_name='study', direction='maximize', load_if_exists=True, sampler=None,
                 pruner=None):
    if storage is None or isinstance(storage, str):
        storage = SQLiteStorage(storage or 'sqlite:///optuna.db')
    return Study(storage, study_name, direction, sampler, pruner)
