"""Recurrent cells (mirrors src/madrona_learn/rnn.py).

``LSTM`` is an architecture description like the modules of ``models.py``:
the engine compiles ``RecurrentBackboneEncoder(net=MLP, rnn=LSTM)`` into the
recurrent variants of the fused HIP kernels (mlearn_lstm_* in
include/mlearn.h).  The cell is flax 0.8.1 ``OptimizedLSTMCell`` (rnn.py:30-36):
input kernels without bias, hidden kernels with bias, gates (i, f, g, o),
orthogonal kernel init per gate, zero bias.

Recurrent state follows the reference's pytree shape ``(c_states, h_states)``
— one [N, H] tensor per layer in the compute dtype (rnn.py:58-68).  The
engine keeps the live carry of the rollout on the device inside the rollout
state; these helpers exist for user code and hooks.
"""

import torch

from .cfg import canonical_dtype
from .models import orthogonal

__all__ = ["LSTM", "MultiLayerLSTMCell"]


class MultiLayerLSTMCell:  # rnn.py:10-45
    def __init__(self, num_hidden_channels, num_layers, dtype):
        self.num_hidden_channels = int(num_hidden_channels)
        self.num_layers = int(num_layers)
        self.dtype = canonical_dtype(dtype)
        self.kernel_init = orthogonal(1.0)            # jax.nn.initializers.orthogonal()
        self.recurrent_kernel_init = orthogonal(1.0)


class LSTM:  # rnn.py:47-111
    def __init__(self, num_hidden_channels, num_layers, dtype):
        self.num_hidden_channels = int(num_hidden_channels)
        self.num_layers = int(num_layers)
        self.dtype = canonical_dtype(dtype)
        self.cell = MultiLayerLSTMCell(num_hidden_channels, num_layers, dtype)

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
