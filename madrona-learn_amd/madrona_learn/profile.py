"""Profiling markers (mirrors src/madrona_learn/profile.py:6-32).

The reference wraps phases in jax.named_scope + TraceAnnotation; here they
become roctx ranges (torch.cuda.nvtx maps to roctx on ROCm) visible to
rocprofv3 --marker-trace.  Disabled by default (zero cost); enable with
MADRONA_LEARN_ROCTX=1.
"""

import os
from contextlib import contextmanager


class Profiler:
    def __init__(self):
        self.disabled = os.environ.get("MADRONA_LEARN_ROCTX", "0") != "1"

    @contextmanager
    def __call__(self, name):
        if self.disabled:
            yield
            return
        import torch
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()

    def disable(self):
        self.disabled = True

    def enable(self):
        self.disabled = False


profile = Profiler()
