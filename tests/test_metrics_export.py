"""Metrics export (metrics.py:190-244, tensorboard.py:29-101): the
TensorBoard event file (TFRecord framing, CRC-32C, Event / Summary protos)
and the per-policy tags of TrainingMetrics.tensorboard_log."""

import struct

import numpy as np
import torch


def test_crc32c_known_answer():
    from madrona_learn.tensorboard import crc32c
    assert crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    assert crc32c(b"") == 0


def test_event_file_roundtrip(tmp_path):
    from madrona_learn.tensorboard import TensorboardWriter, read_events
    w = TensorboardWriter(str(tmp_path))
    for s in range(5):
        w.scalar("loss", 0.5 * s, s)
    w.text("note", "hello", 7)
    w.close()
    ev = read_events(w.path)
    assert ev[:5] == [(s, "loss", np.float32(0.5 * s)) for s in range(5)]
    assert ev[5] == (7, "note", "hello")
    raw = open(w.path, "rb").read()
    (n,) = struct.unpack("<Q", raw[:8])
    assert b"brain.Event:2" in raw[12:12 + n]  # the file_version record comes first


def test_tensorboard_log_tags(tmp_path):
    from madrona_learn.metrics import TrainingMetrics
    from madrona_learn.tensorboard import TensorboardWriter, read_events
    m = TrainingMetrics(["Loss", "Rewards"], 2, "cpu", num_policies=2)
    for u in range(2):
        m.record_scalar("Loss", 1.0 + u, 0)
        m.latest[1, 1] = torch.tensor([2.0, 8.0, -1.0, 5.0, 4.0])
        m.advance()
    w = TensorboardWriter(str(tmp_path))
    m.tensorboard_log(100, w)
    w.close()
    ev = {(s, t): v for s, t, v in read_events(w.path)}
    assert ev[(100, "p0/Loss Mean")] == 1.0 and ev[(101, "p0/Loss Mean")] == 2.0
    assert ev[(101, "p1/Rewards σ")] == np.float32(np.sqrt(8.0 / 4.0))
    assert ev[(100, "p1/Rewards Min")] == -1.0 and ev[(100, "p1/Rewards Max")] == 5.0
    assert len(ev) == 2 * 2 * 2 * 4


def test_pretty_print(capsys):
    from madrona_learn.metrics import TrainingMetrics
    m = TrainingMetrics(["Loss"], 1, "cpu", num_policies=2)
    m.record_scalar("Loss", 0.25, 0)
    m.record_scalar("Loss", 0.5, 1)
    m.advance()
    m.pretty_print()
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "  TrainingMetrics" and out[1] == "    Loss:"
    assert out[2] == "      Avg:  2.500e-01,  5.000e-01"
