"""The C-ABI library (include/mlearn.h) loads without a GPU, exports every
function the header declares, and rejects bad arguments with MLEARN_EINVAL
and a message before touching the device (no compute calls here)."""

import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mlearn.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(mlearn_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("mlearn_gae_f32", "mlearn_policy_rollout_step", "mlearn_ppo_minibatch_grad",
                 "mlearn_optim_step", "mlearn_minibatch_perm", "mlearn_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from madrona_learn import _native as nat
    lib = nat.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # every bound signature in the Python mirror is a declared function
    assert set(nat._SIGNATURES) <= set(declared_functions())


def test_abi_version():
    from madrona_learn import _native as nat
    assert nat.lib().mlearn_abi_version() == nat.ABI_VERSION == 22
    hdr = open(HEADER).read()
    assert f"#define MLEARN_ABI_VERSION {nat.ABI_VERSION}" in hdr


def _einval(rc):
    from madrona_learn import _native as nat
    assert rc == -1, rc  # MLEARN_EINVAL
    msg = nat.lib().mlearn_last_error()
    assert msg and len(msg) > 0
    return msg.decode()


def test_bad_arguments_are_rejected_without_gpu():
    from madrona_learn import _native as nat
    L = nat.lib()
    # GAE with a null pointer
    msg = _einval(L.mlearn_gae_f32(None, None, None, None, None, None, 32, 64, 0.99, 0.95, None))
    assert "null" in msg.lower() or "pointer" in msg.lower()
    # permutation size out of range
    _einval(L.mlearn_minibatch_perm(1, 2, None, 0, 0, 0, None, None))
    # bad policy descriptors
    d = nat.MlpPolicy()
    d.dtype, d.obs_dim, d.hidden, d.num_layers = nat.DTYPE_F32, 64, 96, 2
    d.critic_bins = 1
    assert L.mlearn_param_count(ctypes.byref(d)) == -1
    assert "hidden" in L.mlearn_last_error().decode()
    d.hidden, d.obs_dim = 256, 20
    assert L.mlearn_param_count(ctypes.byref(d)) == -1
    assert "obs_dim" in L.mlearn_last_error().decode()


def test_param_count_matches_oracle_layout():
    from madrona_learn import _native as nat
    from oracle import ppo_ref as ref
    d = nat.MlpPolicy()
    d.dtype, d.obs_dim, d.hidden, d.num_layers = nat.DTYPE_F32, 64, 256, 2
    d.critic_bins = 1
    d.actions = nat.action_layout([4, 8, 5, 5, 2, 2])
    for l in range(2):
        d.w_t[l] = d.ln_scale[l] = d.ln_bias[l] = 1
        d.w[l] = 1
    d.head_t = d.head = d.head_bias = 1
    n = nat.lib().mlearn_param_count(ctypes.byref(d))
    assert n == ref.param_layout(64, 256, 2, 26)["total"] == 89883


def test_step_kernel_selection():
    """mlearn_ppo_step_kernel: the row-split step kernel exactly where it
    applies (bf16, H 256, 2 layers, scalar critic or a two-hot critic of <= 63
    bins (head width 96), obs 64, <= 7 action
    groups, padded rows of 32,768 or a multiple of 256 from 65,536: one
    8-wave workgroup per CU), the feature-split kernel elsewhere; an explicit
    row-split request elsewhere is -1 (EINVAL)."""
    from madrona_learn import _native as nat
    L = nat.lib()

    def desc(dtype=nat.DTYPE_BF16, H=256, layers=2, buckets=(4, 8, 5, 5, 2, 2), bins=1):
        d = nat.MlpPolicy()
        d.dtype, d.obs_dim, d.hidden, d.num_layers = dtype, 64, H, layers
        d.critic_bins = bins
        d.actions = nat.action_layout(list(buckets))
        for l in range(layers):
            d.w_t[l] = d.ln_scale[l] = d.ln_bias[l] = 1
            d.w[l] = 1
        d.head_t = d.head = d.head_bias = 1
        return d

    sel = lambda d, M, req=0: L.mlearn_ppo_step_kernel(ctypes.byref(d), M, req)  # noqa: E731
    d = desc()
    assert sel(d, 65536) == 2 and sel(d, 65536, 2) == 2 and sel(d, 65536, 1) == 1
    assert sel(d, 65520) == 2           # padded to 65,536 rows
    assert sel(d, 65536 * 4) == 2
    for rows in (32768, 32740):                              # the two-rank slice
        assert sel(d, rows) == 2 and sel(d, rows, 1) == 1
    for rows in (8192, 16384, 24576, 49152):                 # one tile per wave: not kept
        assert sel(d, rows) == 1 and sel(d, rows, 2) == -1
    assert sel(d, 65536 + 64) == 1                           # not a multiple of 256
    for other in (desc(dtype=nat.DTYPE_F32), desc(H=128), desc(layers=3),
                  desc(buckets=(2,) * 8), desc(bins=65)):
        assert sel(other, 65536) == 1 and sel(other, 65536, 2) == -1
    # a two-hot critic (head width 96, round 6): the row split too
    for bins in (9, 63):
        assert sel(desc(bins=bins), 65536) == 2 and sel(desc(bins=bins), 32768) == 2
        assert sel(desc(bins=bins), 65536, 1) == 1
    assert sel(d, 65536, 3) == -1 and sel(d, 0) == -1
    # the population launch (mlearn_policy_rollout_pop_kernel): the row split
    # uncapped over >= 2048 16-env tiles of policies with N a multiple of 128
    pk = lambda d, N, P, cap=0: L.mlearn_policy_rollout_pop_kernel(ctypes.byref(d), None, N, P, cap)  # noqa: E731
    assert pk(d, 8192, 8) == 2 and pk(d, 4096, 8) == 2 and pk(d, 65536, 1) == 2
    assert pk(d, 8192, 8, 64) == 1                            # capped: feature split
    assert pk(d, 8192, 2) == 1 and pk(d, 8000, 8) == 1        # too few tiles / N % 128
    for other in (desc(dtype=nat.DTYPE_F32), desc(H=128), desc(bins=9)):
        assert pk(other, 8192, 8) == 1
    assert pk(d, 0, 8) == -1 and pk(d, 8192, 0) == -1 and pk(d, 8192, 8, -1) == -1


def test_lstm_layout_matches_oracle_and_arch():
    """LSTM parameter segment: native offsets/counts == oracle layout ==
    the product's param_layout; RecurrentBackboneEncoder(MLP, LSTM) compiles."""
    import madrona_learn as ml
    from madrona_learn import _native as nat
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    from madrona_learn.rnn import LSTM
    from madrona_learn.train_state import compile_arch, param_layout
    from oracle import lstm_ref as lref
    import pytest
    import torch
    buckets = [4, 8, 5, 5, 2, 2]
    for H, L in ((256, 2), (64, 1), (128, 3)):
        d = nat.MlpPolicy()
        d.dtype, d.obs_dim, d.hidden, d.num_layers = nat.DTYPE_BF16, 64, H, L
        d.critic_bins = 1
        d.actions = nat.action_layout(buckets)
        for l in range(L):
            d.w_t[l] = d.ln_scale[l] = d.ln_bias[l] = 1
            d.w[l] = 1
        d.head_t = d.head = d.head_bias = 1
        r = nat.Lstm()
        r.hidden, r.num_layers = H, 1
        r.wi_perm = r.wi_nat = r.wh_nat = r.w_bwd = r.head_t_nat = r.bias = 1
        lay = lref.param_layout(64, H, L, 26)
        assert nat.lib().mlearn_lstm_param_offset(ctypes.byref(d)) == lay["lstm_off"]
        assert nat.lib().mlearn_lstm_param_count(ctypes.byref(d), ctypes.byref(r)) == lay["total"]
        ac = ml.ActorCritic(
            backbone=ml.BackboneShared(encoder=ml.RecurrentBackboneEncoder(
                net=MLP(H, L, "bf16"), rnn=LSTM(H, 1, "bf16"))),
            actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(buckets), "bf16"),
            critic=DenseLayerCritic("bf16"))
        arch = compile_arch(ac, 64, torch.bfloat16)
        assert arch.lstm_hidden == H
        pl = param_layout(arch)
        assert pl["total"] == lay["total"]
        assert (pl["wi"][0], pl["wr"][0], pl["bl"][0]) == (lay["Wi"][0], lay["Wr"][0],
                                                          lay["bl"][0])
        # a width mismatch or a second layer is rejected, never silently run
        r.num_layers = 2
        assert nat.lib().mlearn_lstm_param_count(ctypes.byref(d), ctypes.byref(r)) == -1
    bad = ml.ActorCritic(
        backbone=ml.BackboneShared(encoder=ml.RecurrentBackboneEncoder(
            net=MLP(256, 2, "bf16"), rnn=LSTM(128, 1, "bf16"))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(buckets), "bf16"),
        critic=DenseLayerCritic("bf16"))
    with pytest.raises(NotImplementedError):
        compile_arch(bad, 64, torch.bfloat16)


def test_two_hot_critic_layout_and_head_width():
    """DreamerV3Critic (models.py:157-174): the head carries A + 63 outputs,
    padded to 96 columns; the layout agrees with the oracle; bad bin counts
    are rejected by the library and by compile_arch."""
    import madrona_learn as ml
    from madrona_learn import _native as nat
    from madrona_learn.models import MLP, DenseLayerDiscreteActor, DreamerV3Critic
    from madrona_learn.train_state import compile_arch, param_layout
    from oracle import ppo_ref as ref
    import torch
    buckets = [4, 8, 5, 5, 2, 2]
    d = nat.MlpPolicy()
    d.dtype, d.obs_dim, d.hidden, d.num_layers = nat.DTYPE_BF16, 64, 256, 2
    d.actions = nat.action_layout(buckets)
    for l in range(2):
        d.w_t[l] = d.ln_scale[l] = d.ln_bias[l] = 1
        d.w[l] = 1
    d.head_t = d.head = d.head_bias = 1
    L = nat.lib()
    for cb, hc in ((1, 32), (5, 32), (63, 96)):
        d.critic_bins = cb
        assert L.mlearn_head_cols(ctypes.byref(d)) == hc == nat.head_cols(26, cb)
        assert L.mlearn_param_count(ctypes.byref(d)) == ref.param_layout(64, 256, 2, 26, cb)["total"]
    for bad in (0, 2, 64, 71):
        d.critic_bins = bad
        assert L.mlearn_param_count(ctypes.byref(d)) == -1
    ac = ml.ActorCritic(
        backbone=ml.BackboneShared(encoder=ml.BackboneEncoder(net=MLP(256, 2, "bf16"))),
        actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig(buckets), "bf16"),
        critic=DreamerV3Critic("bf16"))
    arch = compile_arch(ac, 64, torch.bfloat16)
    assert arch.critic_bins == 63 and arch.head_cols == 96
    assert param_layout(arch)["total"] == ref.param_layout(64, 256, 2, 26, 63)["total"]
