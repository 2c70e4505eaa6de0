"""Checkpoint save -> load -> continue (train.py:44-49, train_state.py:
145-196): a manager restored from a checkpoint continues bit-identically to
the uninterrupted run (parameters, Adam moments and count, minibatch and
sampling RNG positions, rollout state and the sim's own checkpoint), and
init_training(restore_ckpt=...) restores the train state."""

import os

import pytest
import torch

from test_gpu_train import _setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("use_graph", [False, True])
def test_checkpoint_resume_bit_identical(gpu, tmp_path, use_graph):
    _, _, a = _setup(gpu, torch.bfloat16, use_graph=use_graph)
    for _ in range(2):
        a.update_iter()
    a.save_ckpt(str(tmp_path))
    assert os.path.exists(tmp_path / "2.pt")
    saved = a.state.policy_states.params.clone()
    a.update_iter()
    torch.cuda.synchronize()
    _, _, b = _setup(gpu, torch.bfloat16, use_graph=use_graph)
    b.load_ckpt(str(tmp_path))
    assert b.update_idx == 2
    assert torch.equal(b.state.policy_states.params, saved)
    b.update_iter()
    torch.cuda.synchronize()
    assert torch.equal(a.rollout_mgr.store.actions, b.rollout_mgr.store.actions)
    assert torch.equal(a.state.policy_states.params, b.state.policy_states.params)
    assert torch.equal(a.state.train_states.adam_v, b.state.train_states.adam_v)
    assert torch.equal(a.rollout.counters, b.rollout.counters)


def test_init_training_restore_ckpt(gpu, tmp_path):
    import madrona_learn as ml
    from madrona_learn.envs import DummyVecEnv
    from test_gpu_train import make_cfg, make_policy
    _, _, a = _setup(gpu, torch.float32)
    a.update_iter()
    a.save_ckpt(str(tmp_path))
    torch.cuda.synchronize()
    env = DummyVecEnv(64, 64, 6, seed=2, device=gpu)
    c = ml.init_training(gpu, make_cfg(torch.float32), env.sim_fns(),
                         make_policy(torch.float32, 64), restore_ckpt=str(tmp_path),
                         use_graph=False)
    assert c.update_idx == 1
    assert torch.equal(c.state.policy_states.params, a.state.policy_states.params)
    assert torch.equal(c.state.train_states.adam_m, a.state.train_states.adam_m)
    assert int(c.state.train_states.step.item()) == int(a.state.train_states.step.item())
    assert int(c.rollout.counters[1].item()) == int(a.rollout.counters[1].item())
