"""Native TensorBoard event-file writer (the image has no ``tensorboard`` package).

Writes the standard ``events.out.tfevents.*`` TFRecord stream: each record is
``uint64 length | uint32 masked_crc32c(length) | Event proto | uint32 masked_crc32c(data)``.  The
``Event`` / ``Summary`` protos are hand-encoded (only the scalar fields are needed), so files open in
stock TensorBoard.  A JSONL mirror (``scalars.jsonl``) is written next to them for tooling.
Reference hook points: ``utils/utils.py:17-23`` (SummaryWriter), ``core/seg_trainer.py:65-79,139-143``.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

_CRC_TABLE = None


def _crc32c(data: bytes) -> int:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        poly, table = 0x82F63B78, []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            table.append(c)
        _CRC_TABLE = table
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    crc = _crc32c(data)
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num, wire, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _len_field(num, payload: bytes) -> bytes:
    return _field(num, 2, _varint(len(payload)) + payload)


def _event(wall_time: float, step: int = 0, summary: bytes = None, file_version: str = None) -> bytes:
    msg = _field(1, 1, struct.pack('<d', wall_time))           # double wall_time = 1
    msg += _field(2, 0, _varint(step))                           # int64 step = 2
    if file_version is not None:
        msg += _len_field(3, file_version.encode())              # string file_version = 3
    if summary is not None:
        msg += _len_field(5, summary)                            # Summary summary = 5
    return msg


def _scalar_summary(tag: str, value: float) -> bytes:
    val = _len_field(1, tag.encode()) + _field(2, 5, struct.pack('<f', float(value)))
    return _len_field(1, val)                                    # repeated Value value = 1


class SummaryWriter:
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.log_dir = log_dir
        name = f'events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}'
        self._path = os.path.join(log_dir, name)
        self._f = open(self._path, 'wb')
        self._jsonl = open(os.path.join(log_dir, 'scalars.jsonl'), 'a')
        self._write(_event(time.time(), 0, file_version='brain.Event:2'))

    def _reopen(self):
        # torch's SummaryWriter silently re-creates its file writer after close(); the reference
        # relies on that (val_best logs after writer.close(), core/base_trainer.py:108-118)
        if self._f.closed:
            self._f = open(self._path, 'ab')
            self._jsonl = open(os.path.join(self.log_dir, 'scalars.jsonl'), 'a')

    def _write(self, data: bytes):
        self._reopen()
        header = struct.pack('<Q', len(data))
        self._f.write(header + struct.pack('<I', _masked_crc(header)) + data +
                      struct.pack('<I', _masked_crc(data)))

    def add_scalar(self, tag, value, global_step=0):
        if hasattr(value, 'item'):
            value = value.item()
        now = time.time()
        self._write(_event(now, int(global_step), summary=_scalar_summary(tag, value)))
        self._jsonl.write(json.dumps({'tag': tag, 'value': float(value), 'step': int(global_step),
                                      'wall_time': now}) + '\n')

    def flush(self):
        self._f.flush()
        self._jsonl.flush()

    def close(self):
        if not self._f.closed:
            self.flush()
            self._f.close()
            self._jsonl.close()


def read_scalars(path):
    """Parse an event file back into ``[(tag, step, value)]`` (used by tests and tools)."""
    out = []
    with open(path, 'rb') as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        (length,) = struct.unpack_from('<Q', data, pos)
        rec = data[pos + 12: pos + 12 + length]
        pos += 12 + length + 4
        ev = _parse(rec)
        if 5 in ev:
            summ = _parse(ev[5][0])
            for v in summ.get(1, []):
                vv = _parse(v)
                out.append((vv[1][0].decode(), ev.get(2, [0])[0], struct.unpack('<f', vv[2][0])[0]))
    return out


def _parse(buf):
    fields, i = {}, 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            val, i = _read_varint(buf, i)
        elif wire == 1:
            val, i = buf[i:i + 8], i + 8
        elif wire == 5:
            val, i = buf[i:i + 4], i + 4
        elif wire == 2:
            ln, i = _read_varint(buf, i)
            val, i = buf[i:i + ln], i + ln
        else:
            raise ValueError(f'unsupported wire type {wire}')
        fields.setdefault(num, []).append(val)
    return fields


def _read_varint(buf, i):
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7
