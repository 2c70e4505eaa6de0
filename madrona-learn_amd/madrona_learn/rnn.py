"""Recurrent cells (mirrors src/madrona_learn/rnn.py).

``LSTM`` is an architecture description like the modules of ``models.py``:
the engine compiles ``RecurrentBackboneEncoder(net=MLP, rnn=LSTM)`` into the
recurrent variants of the fused HIP kernels (mlearn_lstm_* in
include/mlearn.h); inside a tree the engine does not recognise it runs as a
torch module (``forward`` / ``sequence``).  The cell is flax 0.8.1 ``OptimizedLSTMCell`` (rnn.py:30-36):
input kernels without bias, hidden kernels with bias, gates (i, f, g, o),
orthogonal kernel init per gate, zero bias.

Recurrent state follows the reference's pytree shape ``(c_states, h_states)``
— one [N, H] tensor per layer in the compute dtype (rnn.py:58-68).  The
engine keeps the live carry of the rollout on the device inside the rollout
state; these helpers exist for user code and hooks.
"""

import numpy as np
import torch
from torch import nn

from .cfg import canonical_dtype
from .models import _init_rng, orthogonal

__all__ = ["LSTM", "MultiLayerLSTMCell"]


class MultiLayerLSTMCell(nn.Module):  # rnn.py:10-45
    def __init__(self, num_hidden_channels, num_layers, dtype):
        super().__init__()
        self.num_hidden_channels = int(num_hidden_channels)
        self.num_layers = int(num_layers)
        self.dtype = canonical_dtype(dtype)
        self.kernel_init = orthogonal(1.0)            # jax.nn.initializers.orthogonal()
        self.recurrent_kernel_init = orthogonal(1.0)
        self.wi = nn.ParameterList()
        self.wh = nn.ParameterList()
        self.b = nn.ParameterList()

    def _init(self, fin, dev):
        R = self.num_hidden_channels
        for l in range(self.num_layers):
            f = fin if l == 0 else R
            rng = _init_rng()
            wi = np.concatenate([self.kernel_init(rng, (f, R)) for _ in range(4)], 1)
            wh = np.concatenate([self.recurrent_kernel_init(rng, (R, R)) for _ in range(4)], 1)
            self.wi.append(nn.Parameter(torch.from_numpy(wi).to(dev)))
            self.wh.append(nn.Parameter(torch.from_numpy(wh).to(dev)))
            self.b.append(nn.Parameter(torch.zeros(4 * R, device=dev)))

    def forward(self, carries, inputs):
        """flax OptimizedLSTMCell per layer (gates i, f, g, o; input kernels
        without bias, hidden kernels with bias); returns ((c, h), concat h)."""
        if len(self.wi) == 0:
            self._init(inputs.shape[-1], inputs.device)
        in_c, in_h = carries
        x = inputs
        all_c, all_h = [], []
        R, dt = self.num_hidden_channels, self.dtype
        for l in range(self.num_layers):
            z = (x.to(dt) @ self.wi[l].to(dt)).float() + \
                (in_h[l].to(dt) @ self.wh[l].to(dt) + self.b[l].to(dt)).float()
            i, f, g, o = (z[..., k * R:(k + 1) * R] for k in range(4))
            c = (torch.sigmoid(f) * in_c[l].float() + torch.sigmoid(i) * torch.tanh(g)).to(dt)
            h = (torch.sigmoid(o) * torch.tanh(c.float())).to(dt)
            all_c.append(c)
            all_h.append(h)
            x = h
        return (all_c, all_h), torch.cat(all_h, -1)


class LSTM(nn.Module):  # rnn.py:47-111
    def __init__(self, num_hidden_channels, num_layers, dtype):
        super().__init__()
        self.num_hidden_channels = int(num_hidden_channels)
        self.num_layers = int(num_layers)
        self.dtype = canonical_dtype(dtype)
        self.cell = MultiLayerLSTMCell(num_hidden_channels, num_layers, dtype)

    def forward(self, cur_hiddens, in_features, train=False):  # rnn.py:77-79
        new_hiddens, out = self.cell(cur_hiddens, in_features)
        return out, new_hiddens

    def sequence(self, start_hiddens, seq_ends, seq_x, train=False):  # rnn.py:81-111
        carry = start_hiddens
        outs = []
        for t in range(seq_x.shape[0]):
            carry, y = self.cell(carry, seq_x[t])
            carry = self.clear_recurrent_state(carry, seq_ends[t])
            outs.append(y)
        return torch.stack(outs, 0)

    def init_recurrent_state(self, N, device=None):  # rnn.py:52-63
        z = lambda: torch.zeros((N, self.num_hidden_channels), dtype=self.dtype,  # noqa: E731
                                device=device)
        return [z() for _ in range(self.num_layers)], [z() for _ in range(self.num_layers)]

    def clear_recurrent_state(self, rnn_states, should_clear):  # rnn.py:65-81
        c_states, h_states = rnn_states
        m = should_clear.reshape(-1, 1).to(torch.bool)
        return ([torch.where(m, torch.zeros((), dtype=c.dtype, device=c.device), c)
                 for c in c_states],
                [torch.where(m, torch.zeros((), dtype=h.dtype, device=h.device), h)
                 for h in h_states])
