"""A dependency-free TensorBoard scalar writer.

The reference worker logs ``loss`` and ``accuracy`` through ``tensorboardX.SummaryWriter``
(examples/mnist/mnist.py:3,47-48,64,108).  Neither tensorboardX nor tensorboard is in
this image, so this module writes the same ``events.out.tfevents.*`` files directly:
TFRecord framing (length, masked CRC-32C, payload, masked CRC-32C) around hand-encoded
``tensorflow.Event`` protobufs holding ``Summary.Value.simple_value`` scalars.  The files
open in a stock TensorBoard.  A JSONL mirror (``scalars.jsonl``) is written alongside for
tests and scripts.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time

# ---------------------------------------------------------------- CRC-32C (Castagnoli)
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = _TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _masked(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def tfrecord(payload: bytes) -> bytes:
    header = struct.pack("<Q", len(payload))
    return (header + struct.pack("<I", _masked(crc32c(header))) + payload +
            struct.pack("<I", _masked(crc32c(payload))))


# ---------------------------------------------------------------- protobuf encoding
def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_delim(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, *, file_version: str = None,
                 scalars: dict = None) -> bytes:
    """tensorflow.Event{wall_time=1 double, step=2 int64, file_version=3 string, summary=5}."""
    out = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        out += _len_delim(3, file_version.encode())
    if scalars:
        summary = b""
        for tag, v in scalars.items():
            # Summary.Value{tag=1 string, simple_value=2 float}
            val = _len_delim(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v))
            summary += _len_delim(1, val)
        out += _len_delim(5, summary)
    return out


class SummaryWriter:
    """Minimal ``tensorboardX.SummaryWriter`` replacement (add_scalar/flush/close)."""

    def __init__(self, logdir: str = "logs"):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "wb")
        self._jsonl = open(os.path.join(logdir, "scalars.jsonl"), "a")
        self._f.write(tfrecord(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, global_step: int = 0, walltime: float = None) -> None:
        wt = time.time() if walltime is None else walltime
        self._f.write(tfrecord(encode_event(wt, global_step, scalars={tag: value})))
        self._jsonl.write(json.dumps({"tag": tag, "value": float(value), "step": int(global_step),
                                      "wall_time": wt}) + "\n")

    def flush(self) -> None:
        self._f.flush()
        self._jsonl.flush()

    def close(self) -> None:
        if not self._f.closed:
            self.flush()
            self._f.close()
            self._jsonl.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_events(path: str):
    """Parse an event file written by ``SummaryWriter`` -> list of (step, {tag: value})."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        (n,) = struct.unpack_from("<Q", data, pos)
        (hcrc,) = struct.unpack_from("<I", data, pos + 8)
        if hcrc != _masked(crc32c(data[pos:pos + 8])):
            raise ValueError("corrupt record header")
        payload = data[pos + 12:pos + 12 + n]
        (pcrc,) = struct.unpack_from("<I", data, pos + 12 + n)
        if pcrc != _masked(crc32c(payload)):
            raise ValueError("corrupt record payload")
        pos += 16 + n
        out.append(_decode_event(payload))
    return out


def _read_varint(b: bytes, i: int):
    shift = n = 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return n, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v = b[i:i + 8]
            i += 8
        elif w == 5:
            v = b[i:i + 4]
            i += 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"wire type {w}")
        yield f, w, v


def _decode_event(payload: bytes):
    step, scalars = 0, {}
    for f, _, v in _fields(payload):
        if f == 2:
            step = v
        elif f == 5:
            for f2, _, val in _fields(v):
                if f2 != 1:
                    continue
                tag, sv = None, None
                for f3, _, x in _fields(val):
                    if f3 == 1:
                        tag = x.decode()
                    elif f3 == 2:
                        (sv,) = struct.unpack("<f", x)
                if tag is not None:
                    scalars[tag] = sv
    return step, scalars
