"""SQLite study storage with trial heartbeats -- the native stand-in for optuna's ``RDBStorage`` +
``RetryFailedTrialCallback`` used by the reference (``optuna_search.py:70-71``).

Safe for several processes on one node (concurrent trial groups share the file): every mutation is
one short ``BEGIN IMMEDIATE`` transaction.  A RUNNING trial whose heartbeat is older than
``grace`` seconds is marked FAIL and, with ``retry_failed``, re-enqueued as a WAITING trial with
the same parameters (its ``retried_from`` attribute names the failed trial).
"""
from __future__ import annotations

import json
import os
import sqlite3
import time

SCHEMA = """
CREATE TABLE IF NOT EXISTS studies (id INTEGER PRIMARY KEY, name TEXT UNIQUE, direction TEXT);
CREATE TABLE IF NOT EXISTS trials (id INTEGER PRIMARY KEY, study_id INTEGER, number INTEGER, state TEXT,
    value REAL, params TEXT, dists TEXT, attrs TEXT, heartbeat REAL, started REAL, finished REAL);
CREATE TABLE IF NOT EXISTS intermediate (trial_id INTEGER, step INTEGER, value REAL,
    PRIMARY KEY (trial_id, step));
"""


class SQLiteStorage:
    def __init__(self, url_or_path='sqlite:///optuna.db', heartbeat_interval=1.0, grace_period=None,
                 retry_failed=True, timeout=60.0):
        path = url_or_path[len('sqlite:///'):] if url_or_path.startswith('sqlite:///') else url_or_path
        self.path = os.path.abspath(path)
        self.heartbeat_interval = heartbeat_interval
        self.grace = grace_period if grace_period is not None else max(2 * (heartbeat_interval or 1), 60.0)
        self.retry_failed = retry_failed
        self.timeout = timeout
        c = self._conn()
        try:
            c.executescript(SCHEMA)
        finally:
            c.close()

    # --------------------------------------------------------------------------------------------
    def _conn(self):
        c = sqlite3.connect(self.path, timeout=self.timeout, isolation_level=None)
        c.row_factory = sqlite3.Row
        return c

    class _Tx:
        def __init__(self, storage):
            self.c = storage._conn()

        def __enter__(self):
            self.c.execute('BEGIN IMMEDIATE')
            return self.c

        def __exit__(self, et, ev, tb):
            self.c.execute('ROLLBACK' if et else 'COMMIT')
            self.c.close()
            return False

    def _tx(self):
        return SQLiteStorage._Tx(self)

    # --------------------------------------------------------------------------------------------
    def create_study(self, name, direction='maximize', load_if_exists=True):
        with self._tx() as c:
            row = c.execute('SELECT id, direction FROM studies WHERE name=?', (name,)).fetchone()
            if row is not None:
                if not load_if_exists:
                    raise ValueError(f'study {name!r} exists')
                return row['id'], row['direction']
            cur = c.execute('INSERT INTO studies (name, direction) VALUES (?, ?)', (name, direction))
            return cur.lastrowid, direction

    def claim_trial(self, study_id):
        """Take the oldest WAITING trial (a retry) or create a new RUNNING one. Returns (id, number, params)."""
        now = time.time()
        self.fail_stale(study_id)
        with self._tx() as c:
            row = c.execute("SELECT id, number, params FROM trials WHERE study_id=? AND state='WAITING' "
                            'ORDER BY number LIMIT 1', (study_id,)).fetchone()
            if row is not None:
                c.execute("UPDATE trials SET state='RUNNING', heartbeat=?, started=? WHERE id=?", (now, now, row['id']))
                return row['id'], row['number'], json.loads(row['params'] or '{}')
            num = c.execute('SELECT COALESCE(MAX(number), -1) + 1 FROM trials WHERE study_id=?', (study_id,)).fetchone()[0]
            cur = c.execute("INSERT INTO trials (study_id, number, state, params, dists, attrs, heartbeat, started) "
                            "VALUES (?, ?, 'RUNNING', '{}', '{}', '{}', ?, ?)", (study_id, num, now, now))
            return cur.lastrowid, num, {}

    def set_param(self, trial_id, name, value, dist):
        with self._tx() as c:
            row = c.execute('SELECT params, dists FROM trials WHERE id=?', (trial_id,)).fetchone()
            p, d = json.loads(row['params']), json.loads(row['dists'])
            p[name], d[name] = value, dist
            c.execute('UPDATE trials SET params=?, dists=? WHERE id=?', (json.dumps(p), json.dumps(d), trial_id))

    def report(self, trial_id, step, value):
        with self._tx() as c:
            c.execute('INSERT OR REPLACE INTO intermediate (trial_id, step, value) VALUES (?, ?, ?)',
                      (trial_id, int(step), float(value)))
            c.execute('UPDATE trials SET heartbeat=? WHERE id=?', (time.time(), trial_id))

    def heartbeat(self, trial_id):
        with self._tx() as c:
            c.execute('UPDATE trials SET heartbeat=? WHERE id=?', (time.time(), trial_id))

    def finish(self, trial_id, state, value=None):
        with self._tx() as c:
            c.execute('UPDATE trials SET state=?, value=?, finished=? WHERE id=?',
                      (state, None if value is None else float(value), time.time(), trial_id))

    def fail_stale(self, study_id):
        now = time.time()
        with self._tx() as c:
            stale = c.execute("SELECT id, number, params FROM trials WHERE study_id=? AND state='RUNNING' "
                              'AND heartbeat < ?', (study_id, now - self.grace)).fetchall()
            for r in stale:
                c.execute("UPDATE trials SET state='FAIL', finished=? WHERE id=?", (now, r['id']))
                if self.retry_failed:
                    num = c.execute('SELECT MAX(number) + 1 FROM trials WHERE study_id=?', (study_id,)).fetchone()[0]
                    c.execute("INSERT INTO trials (study_id, number, state, params, dists, attrs, heartbeat) "
                              "VALUES (?, ?, 'WAITING', ?, '{}', ?, ?)",
                              (study_id, num, r['params'], json.dumps({'retried_from': r['number']}), now))
        return [r['number'] for r in stale]

    # --------------------------------------------------------------------------------------------
    def trials(self, study_id):
        c = self._conn()
        try:
            rows = c.execute('SELECT * FROM trials WHERE study_id=? ORDER BY number', (study_id,)).fetchall()
            inter = {}
            for r in c.execute('SELECT i.trial_id, i.step, i.value FROM intermediate i JOIN trials t '
                               'ON i.trial_id = t.id WHERE t.study_id=?', (study_id,)):
                inter.setdefault(r['trial_id'], {})[r['step']] = r['value']
        finally:
            c.close()
        out = []
        for r in rows:
            out.append({'id': r['id'], 'number': r['number'], 'state': r['state'], 'value': r['value'],
                        'params': json.loads(r['params'] or '{}'), 'dists': json.loads(r['dists'] or '{}'),
                        'attrs': json.loads(r['attrs'] or '{}'), 'intermediate': inter.get(r['id'], {})})
        return out
