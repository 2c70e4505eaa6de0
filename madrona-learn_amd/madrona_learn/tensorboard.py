"""TensorBoard event writer (mirrors src/madrona_learn/tensorboard.py:29-101).

The reference wraps tensorboard's EventFileWriter; tensorboard is not a
dependency here, so the event file is written directly: TFRecord framing
(little-endian u64 length, masked CRC-32C of the length, the record, masked
CRC-32C of the record) around hand-encoded ``Event`` protos
(tensorflow/core/util/event.proto: wall_time = 1, step = 2,
file_version = 3, summary = 5; Summary.value = 1; Summary.Value: tag = 1,
simple_value = 2, tensor = 8, metadata = 9).  Files are readable by
TensorBoard as written.
"""

import os
import socket
import struct
import time

__all__ = ["TensorboardWriter", "read_events"]


def _crc32c_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_T = _crc32c_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _bytes_field(field, data: bytes):
    return _key(field, 2) + _varint(len(data)) + data


def _event(step, wall_time, summary=None, file_version=None):
    b = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        b += _bytes_field(3, file_version.encode())
    if summary is not None:
        b += _bytes_field(5, summary)
    return b


def _scalar_value(tag, value):
    return _bytes_field(1, _bytes_field(1, tag.encode()) + _key(2, 5) +
                        struct.pack("<f", float(value)))


def _text_value(tag, text):
    # SummaryMetadata{plugin_data{plugin_name: "text"}}; TensorProto{dtype:
    # DT_STRING (7), tensor_shape{dim{size: 1}}, string_val}
    meta = _bytes_field(1, _bytes_field(1, b"text"))
    shape = _bytes_field(2, _key(1, 0) + _varint(1))
    tensor = _key(1, 0) + _varint(7) + _bytes_field(2, shape) + _bytes_field(8, text.encode())
    return _bytes_field(1, _bytes_field(1, tag.encode()) + _bytes_field(8, tensor) +
                        _bytes_field(9, meta))


class TensorboardWriter:
    """Writes entries to event files in the logdir to be consumed by TensorBoard."""

    def __init__(self, logdir: str, queue_size: int = 20, write_interval: int = 10):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "wb")
        self._pending = []
        self.queue_size = queue_size
        self.write_interval = write_interval
        self._last = time.time()
        self._write(_event(0, time.time(), file_version="brain.Event:2"))
        self.flush()

    def _write(self, rec: bytes):
        hdr = struct.pack("<Q", len(rec))
        self._pending.append(hdr + struct.pack("<I", _masked(hdr)) + rec +
                             struct.pack("<I", _masked(rec)))
        if len(self._pending) >= self.queue_size or time.time() - self._last > self.write_interval:
            self.flush()

    def scalar(self, tag, scalar, step: int):
        self._write(_event(step, time.time(), summary=_scalar_value(tag, scalar)))

    def text(self, tag, textdata, step: int):
        self._write(_event(step, time.time(), summary=_text_value(tag, textdata)))

    def flush(self):
        if self._pending:
            self._f.write(b"".join(self._pending))
            self._pending.clear()
        self._f.flush()
        self._last = time.time()

    def close(self):
        self.flush()
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.flush()


def _read_varint(b, i):
    v, s = 0, 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
        if not x & 0x80:
            return v, i


def _fields(b):
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
        else:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        yield f, v


def read_events(path):
    """[(step, tag, value)] of the scalar / text entries of an event file,
    checking every record's CRCs (a reader for tests and tooling)."""
    out = []
    with open(path, "rb") as fh:
        data = fh.read()
    i = 0
    while i < len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        if struct.unpack("<I", data[i + 8:i + 12])[0] != _masked(hdr):
            raise ValueError("corrupt record length")
        rec = data[i + 12:i + 12 + n]
        if struct.unpack("<I", data[i + 12 + n:i + 16 + n])[0] != _masked(rec):
            raise ValueError("corrupt record")
        i += 16 + n
        step, summ = 0, None
        for f, v in _fields(rec):
            if f == 2:
                step = v
            elif f == 5:
                summ = v
        if summ is None:
            continue
        for f, val in _fields(summ):
            if f != 1:
                continue
            tag, value = None, None
            for g, x in _fields(val):
                if g == 1:
                    tag = x.decode()
                elif g == 2:
                    value = struct.unpack("<f", x)[0]
                elif g == 8:
                    for h, y in _fields(x):
                        if h == 8:
                            value = y.decode()
            out.append((step, tag, value))
    return out
