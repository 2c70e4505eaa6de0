"""Training metrics (mirrors src/madrona_learn/metrics.py:12-188).

A ``Metric`` is (mean, m2, min, max, count) with the reference's Chan merge.
Values are produced on the GPU by the native metrics/loss kernels as
[5]-float device vectors; ``TrainingMetrics`` keeps the latest record of
every metric in one fixed device buffer (graph-capture safe) and copies it
into a ``metrics_buffer_size`` ring on ``advance()``.  Host readback happens
only when the user asks for values.

As in the reference, every ``record`` of a metric overwrites its slot for
the current update, so the PPO metrics reflect the last minibatch
(metrics.py:161-181).
"""

from dataclasses import dataclass

import numpy as np
import torch

FLT_MAX = float(np.finfo(np.float32).max)


@dataclass
class Metric:
    per_policy: bool
    mean: float = 0.0
    m2: float = 0.0
    min: float = FLT_MAX
    max: float = -FLT_MAX
    count: int = 0

    @staticmethod
    def init(per_policy):  # metrics.py:20-29
        return Metric(per_policy)

    @staticmethod
    def init_from_data(per_policy, data):  # metrics.py:31-48
        d = np.asarray(data, dtype=np.float64)
        mean = float(d.mean()) if d.size else 0.0
        return Metric(per_policy, mean, float(((d - mean) ** 2).sum()),
                      float(d.min()) if d.size else FLT_MAX,
                      float(d.max()) if d.size else -FLT_MAX, int(d.size))

    @staticmethod
    def from_vector(per_policy, v):
        v = [float(x) for x in v]
        return Metric(per_policy, v[0], v[1], v[2], v[3], int(round(v[4])))

    def merge(self, o):  # metrics.py:79-98 (Chan et al.)
        n = self.count + o.count
        delta = o.mean - self.mean
        inv = 1.0 / max(n, 1)
        mean = self.mean + delta * o.count * inv
        m2 = self.m2 + o.m2 + delta * delta * self.count * o.count * inv
        return Metric(self.per_policy, mean, m2, min(self.min, o.min), max(self.max, o.max), n)

    @property
    def var(self):
        return self.m2 / self.count if self.count > 0 else 0.0


class TrainingMetrics:
    """Latest-record buffer [P, names, 5] (P = train policies on this rank;
    the reference keeps a leading policy axis on per-policy metrics,
    metrics.py:110-147) plus a metrics_buffer_size ring of it."""

    def __init__(self, names, buffer_size, device, per_policy=True, num_policies=1):
        self.names = list(names)
        self.index = {n: i for i, n in enumerate(self.names)}
        self.buffer_size = int(buffer_size)
        self.per_policy = per_policy
        self.num_policies = int(num_policies)
        self.latest = torch.zeros((self.num_policies, len(self.names), 5), dtype=torch.float32,
                                  device=device)
        self.latest[..., 2] = FLT_MAX
        self.latest[..., 3] = -FLT_MAX
        self.ring = self.latest.unsqueeze(0).repeat(self.buffer_size, 1, 1, 1)
        self.update_idx = 0
        self.cur_buffer_offset = 0

    def slot(self, name, policy=0):
        """[5] device view of the latest record of `name` (kernels write here)."""
        return self.latest[policy, self.index[name]]

    def slots(self, first, count, policy=0):
        """[count, 5] device view of `count` consecutive metrics from `first`."""
        i = self.index[first]
        return self.latest[policy, i:i + count]

    def record_tensor(self, name, vec5, policy=0):
        self.latest[policy, self.index[name]].copy_(vec5)

    def record_scalar(self, name, value, policy=0):
        s = self.latest[policy, self.index[name]]
        s[0] = value
        s[1] = 0.0
        s[2] = value
        s[3] = value
        s[4] = 1.0

    def advance(self):  # metrics.py:183-188
        self.ring[self.cur_buffer_offset].copy_(self.latest)
        self.update_idx += 1
        self.cur_buffer_offset = (self.cur_buffer_offset + 1) % self.buffer_size

    def last(self, policy=0):
        """Host dict name -> Metric of the most recently completed update."""
        idx = (self.cur_buffer_offset - 1) % self.buffer_size
        host = self.ring[idx, policy].cpu().numpy()
        return {n: Metric.from_vector(self.per_policy, host[i]) for i, n in enumerate(self.names)}

    def pretty_print(self, tab=2):  # metrics.py:190-217 (the last completed update)
        tab = " " * tab
        lines = [tab + "TrainingMetrics"]
        vals = [self.last(p) for p in range(self.num_policies)]

        def fmt(xs):
            return ", ".join(f"{float(x): .3e}" for x in xs)

        for n in self.names:
            ms = [v[n] for v in vals]
            lines.append(tab * 2 + f"{n}:")
            lines.append(tab * 3 + f"Avg: {fmt(m.mean for m in ms)}")
            lines.append(tab * 3 + f"Min: {fmt(m.min for m in ms)}")
            lines.append(tab * 3 + f"Max: {fmt(m.max for m in ms)}")
            lines.append(tab * 3 + f"\u03c3:   {fmt(np.sqrt(max(m.var, 0.0)) for m in ms)}")
        print("\n".join(lines))

    def tensorboard_log(self, base_update_idx, writer):  # metrics.py:219-244
        """Every buffered update (ring slot b -> step base_update_idx + b):
        '<name> Mean/σ/Min/Max' (per policy 'p<i>/<name> ...')."""
        host = self.ring.cpu().numpy()  # [buf, P, names, 5]
        for b in range(self.buffer_size):
            step = base_update_idx + b
            for j, n in enumerate(self.names):
                for i in range(self.num_policies):
                    mean, m2, mn, mx, cnt = (float(x) for x in host[b, i, j])
                    sd = float(np.sqrt(m2 / cnt)) if cnt > 0 else 0.0
                    pre = f"p{i}/" if self.per_policy else ""
                    writer.scalar(f"{pre}{n} Mean", mean, step)
                    writer.scalar(f"{pre}{n} \u03c3", sd, step)
                    writer.scalar(f"{pre}{n} Min", mn, step)
                    writer.scalar(f"{pre}{n} Max", mx, step)
