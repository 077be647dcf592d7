"""``python main.py`` on a multi-GPU box: the reference's single-process DataParallel mode, the MI355X way.

The reference runs ``nn.DataParallel`` when it is started without a launcher (``utils/parallel.py:24-27,
40-42``): ONE process drives every visible GPU, the per-GPU batch is multiplied by the GPU count
(``train_bs *= gpu_num``) and the lr scales with ``gpu_num`` (``utils/optimizer.py:9,15``).  The fused
MI355X engine is one process per GPU (a hipGraph-captured step per device, RCCL over xGMI), so here the
same command becomes N worker processes -- one per GPU, started BEFORE the parent touches any GPU -- each
with the reference's per-GPU batch: the global batch (``train_bs * N``) and the lr (``* gpu_num``) are
exactly DataParallel's.  DataParallel computes BatchNorm statistics per replica (no cross-GPU sync), so
the workers run with ``synBN`` off unless ``MSP_DP_SYNCBN=1`` asks for SyncBN.

Controls (environment): ``MSP_NO_SPAWN=1`` keeps the single process; ``MSP_SPAWN_PROCS=N`` forces N
workers (CPU gloo rehearsal on a GPU-less machine).  A run under ``torchrun`` (``LOCAL_RANK`` set) or on
one GPU is left alone.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

DP_ENV = 'MSP_DP_EMULATION'


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker_count(env=None):
    """Workers to start for a launcher-less run (0 = run in this process)."""
    env = os.environ if env is None else env
    if env.get('LOCAL_RANK') not in (None, '', '-1') or env.get('MSP_NO_SPAWN') == '1':
        return 0
    forced = env.get('MSP_SPAWN_PROCS')
    if forced:
        n = int(forced)
        return n if n > 1 else 0
    import torch   # device_count() enumerates without initialising a GPU context on this stack
    n = torch.cuda.device_count()
    return n if n > 1 else 0


def spawn_ranks(n, argv, extra_env=None, poll_s=0.2, grace_s=20.0):
    """Start ``n`` rank processes of ``[python] + argv`` with the torchrun environment (127.0.0.1
    rendezvous, one rank per local GPU) and supervise them the way torchrun does: all handles are
    polled, and the first rank that exits non-zero tears the others down (SIGTERM, then SIGKILL after
    ``grace_s``), so a dead rank never leaves its peers blocked in a collective until the process-group
    timeout.  Must be called before this process touches a GPU (the children are fresh interpreters).
    Returns the job's exit code (0, or the first failing rank's code)."""
    import signal
    import time
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    rc = 0
    try:
        live = set(range(n))
        while live:
            for r in sorted(live):
                code = procs[r].poll()
                if code is None:
                    continue
                live.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f'[launch] rank {r} exited with {code}; stopping the other ranks', file=sys.stderr,
                          flush=True)
                    for q in live:
                        procs[q].send_signal(signal.SIGTERM)
                    deadline = time.monotonic() + grace_s
                    for q in sorted(live):
                        try:
                            procs[q].wait(timeout=max(deadline - time.monotonic(), 0.1))
                        except subprocess.TimeoutExpired:
                            procs[q].kill()
                            procs[q].wait()
                    live.clear()
                    break
            if live:
                time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        rc = 130
    return rc


def maybe_spawn_workers(argv=None):
    """In the launcher-less multi-GPU case start one worker per GPU (this same script and arguments,
    with the torchrun environment) and exit with the workers' status; otherwise return."""
    n = worker_count()
    if n == 0:
        return
    argv = list(sys.argv if argv is None else argv)
    sys.exit(spawn_ranks(n, argv, {DP_ENV: '1'}))


def apply_dp_semantics(config):
    """In a worker started by :func:`maybe_spawn_workers`: DataParallel's per-replica BatchNorm."""
    if os.environ.get(DP_ENV) == '1' and os.environ.get('MSP_DP_SYNCBN') != '1':
        config.synBN = False
