"""Low-latency SyncBN statistic exchange over IPC-mapped peer memory (``csrc/comm.hip``).

The reference's SyncBatchNorm (``/root/reference/utils/parallel.py:37-38``, torch ``SyncBatchNorm``)
makes every BatchNorm a blocking NCCL collective in each direction.  The fused engine already batches
them per dependency level (``ops.bn._Pending``), but each level is still a full RCCL launch whose
latency (tens of us for a few KB) is paid ~259 times per DUCKNet step.  On one node every GPU can
load/store every other GPU's HBM over xGMI, so the exchange is done by ONE single-block kernel:
every rank pushes its fp64 row into a slot of every rank's exchange buffer, raises a flag there, waits
for all flags in its own buffer and sums the slots in rank order (bitwise-identical results on every
rank).  No host round trip, no proxy thread, and the kernel is hipGraph-capturable (the epoch counter
lives in device memory).

Policy (``config.syncbn_comm`` / env ``MSP_SYNCBN_COMM``): ``'rccl'`` (default) keeps every exchange on
RCCL; ``'auto'`` uses the IPC kernel for GPU process groups of a single-node job, after a self-test exchange
of known values succeeded on every rank (all ranks agree, so a failure anywhere falls back everywhere);
``'ipc'`` requires the IPC path (errors if it cannot be set up).  Rows larger than the buffer capacity and
every multi-node group go through RCCL.  The IPC path is opt-in until a cross-GPU run of it is on record
(it has only run as several processes sharing one GPU): a stalled exchange there ends in NaN and a fatal
:func:`check`, where RCCL would wait up to the process-group timeout.

Timeout: a peer that has not arrived after ``timeout_s`` (env ``MSP_SYNCBN_IPC_TIMEOUT`` seconds, else
``config.dist_timeout_min``, else 30 minutes -- the process-group default) makes the exchange return NaN
and count an error, so rank skew from host-side work (checkpoint writing on rank 0, validation) is
waited out like RCCL would, and only a dead peer turns into the named error.

Instrumentation: the kernel accumulates, per exchange, how long it spun before the LAST peer's flag
arrived (:meth:`IpcAllReduce.wait_stats`): on an xGMI node that separates rank skew (long waits) from
transport latency (the remaining exchange time).
"""
from __future__ import annotations

import atexit
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

from ..ops._ext import require

POLICY = {'mode': os.environ.get('MSP_SYNCBN_COMM', 'rccl'), 'timeout_s': None}


def default_timeout_s(config=None) -> float:
    """Exchange deadline: env MSP_SYNCBN_IPC_TIMEOUT (s) > ``config.dist_timeout_min`` > 30 min."""
    env = os.environ.get('MSP_SYNCBN_IPC_TIMEOUT')
    if env:
        return float(env)
    if POLICY.get('timeout_s'):
        return float(POLICY['timeout_s'])
    minutes = getattr(config, 'dist_timeout_min', None) if config is not None else None
    return float(minutes) * 60.0 if minutes else 1800.0
_COMMS: Dict[object, Optional['IpcAllReduce']] = {}
_LOG = []


class IpcAllReduce:
    """In-place SUM all-reduce of small fp64 rows over the ranks of ``group`` (one node)."""

    def __init__(self, group, device, cap=32768, timeout_s=None):
        C = require()
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > C.comm_max_ranks():
            raise ValueError(f'IPC all-reduce supports up to {C.comm_max_ranks()} ranks')
        self.cap = int(cap)
        self.timeout_s = float(timeout_s) if timeout_s is not None else default_timeout_s()
        self.device = device
        self.own, handle, self.opened, self.peers = 0, None, [], []
        try:   # a local failure must not skip the collective below (the other ranks are waiting in it)
            with torch.cuda.device(device):
                self.own, handle = C.comm_alloc(C.comm_buffer_bytes(self.cap, self.world))
        except Exception:
            handle = None
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        if any(h is None for h in handles):   # every rank sees the same list -> every rank raises
            raise RuntimeError('IPC exchange buffer allocation failed on a rank')
        with torch.cuda.device(device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    self.peers.append(self.own)
                else:
                    p = C.comm_open(h)
                    self.opened.append(p)
                    self.peers.append(p)
        # [epoch, sum of last-flag wait ticks, exchanges, max wait ticks] (csrc/comm.hip)
        self.epoch = torch.zeros(4, dtype=torch.int64, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.calls = 0
        atexit.register(self.close)

    def all_reduce(self, buf: torch.Tensor):
        """``buf`` (contiguous fp64 on this device, <= cap values) <- its sum over the group."""
        require().comm_allreduce(buf, buf, self.peers, self.rank, self.cap, self.epoch, self.err, self.timeout_s)
        self.calls += 1

    def fits(self, buf: torch.Tensor) -> bool:
        return (buf.dtype == torch.float64 and buf.is_contiguous() and buf.numel() <= self.cap
                and buf.device == self.epoch.device)

    def wait_stats(self, reset=False):
        """(exchanges, mean / max spin before the last peer's flag, in us) since the last reset (host sync)."""
        st = self.epoch[1:4].tolist()
        khz = require().comm_wall_clock_khz()
        n = st[1]
        res = {'exchanges': n, 'wait_us_mean': (st[0] / n / khz * 1e3) if n else None,
               'wait_us_max': st[2] / khz * 1e3 if n else None}
        if reset:
            self.epoch[1:4].zero_()
        return res

    def errors(self) -> int:
        """Exchanges that timed out waiting for a peer (host sync)."""
        return int(self.err.item())

    def self_test(self, timeout_s=5.0) -> bool:
        """Known values through the exchange (exact in fp64), then every rank's verdict AND-ed over the
        group, so all ranks take the same decision."""
        saved, self.timeout_s = self.timeout_s, timeout_s
        ok = True
        try:
            for n in (1, 257, min(self.cap, 4099)):
                x = (torch.arange(n, dtype=torch.float64, device=self.device) + 1) * (self.rank + 1)
                self.all_reduce(x)
                want = (torch.arange(n, dtype=torch.float64, device=self.device) + 1) * (self.world * (self.world + 1) / 2)
                ok = ok and bool(torch.equal(x, want))
            ok = ok and self.errors() == 0
        except Exception:
            ok = False
        finally:
            self.timeout_s = saved
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                            device=self.device if dist.get_backend(self.group) == 'nccl' else 'cpu')
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item())

    def close(self):
        C = require()
        for p in self.opened:
            C.comm_close(p)
        self.opened = []
        if self.own:
            C.comm_free(self.own)
            self.own = 0


def _single_node(group) -> bool:
    lw = os.environ.get('LOCAL_WORLD_SIZE')
    if lw is None:   # torchrun always sets it; without it assume one node only for a single-device rehearsal
        return False
    return int(lw) >= dist.get_world_size()


def attach(group, device) -> Optional[IpcAllReduce]:
    """The IPC communicator of ``group`` (created collectively on first use -- every rank of the group
    must call this at the same point), or None when the policy / topology / self-test says RCCL."""
    if group in _COMMS:
        return _COMMS[group]
    mode = POLICY['mode']
    comm = None
    usable = (mode != 'rccl' and device is not None and device.type == 'cuda' and dist.is_initialized()
              and dist.get_world_size(group) > 1 and (mode == 'ipc' or _single_node(group)))
    if usable:
        err = None
        try:
            comm = IpcAllReduce(group, device)
        except Exception as e:   # allocation / IPC mapping refused on this rank
            comm, err = None, e
        # every rank must agree: a rank that failed construction still joins the verdict
        ok = comm.self_test() if comm is not None else _vote_false(group, device)
        if not ok:
            if comm is not None:
                comm.close()
            comm = None
            if mode == 'ipc':
                raise RuntimeError(f'SyncBN IPC exchange requested but unavailable ({err!r})')
        _LOG.append(('ipc' if comm is not None else f'rccl (ipc self-test failed: {err!r})'))
    _COMMS[group] = comm
    return comm


def _vote_false(group, device):
    flag = torch.zeros(1, dtype=torch.int32, device=device if dist.get_backend(group) == 'nccl' else 'cpu')
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return False


def lookup(group) -> Optional[IpcAllReduce]:
    return _COMMS.get(group)


def active() -> bool:
    return any(c is not None for c in _COMMS.values())


def wait_stats(reset=False):
    """Per attached IPC communicator: :meth:`IpcAllReduce.wait_stats` (empty when every group is on RCCL)."""
    return [c.wait_stats(reset) for c in _COMMS.values() if c is not None]


def check():
    """Raise if any IPC exchange timed out (a peer never arrived; its result was NaN).  Host sync."""
    for c in _COMMS.values():
        if c is not None and c.errors():
            raise RuntimeError(f'SyncBN IPC exchange: {c.errors()} exchange(s) timed out waiting for a peer')


def describe():
    """'ipc' / 'rccl' per attached group (evidence / logs)."""
    return ['ipc' if c is not None else 'rccl' for c in _COMMS.values()]
