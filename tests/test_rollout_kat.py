"""Integer known-answer test of the rollout data flow, restating the design of
the reference's tests/test_rollouts.py (fake net `o + bias` 201-215, fake sim
`obs = a + 1, reward = a + 2, done every L` 264-288, closed-form checks
verify_rollout_data 380-460) for the MLP path (no recurrent state): store
alignment (obs[t] is the observation action t was taken on, rewards/dones[t]
the sim's answer to it), env-return bookkeeping, the bootstrap observation,
and GAE / returns on the resulting store, all against closed forms."""

import numpy as np
import pytest

from oracle import ppo_ref as ref


class FakeSim:
    """fake_sim_step (test_rollouts.py:264-288): obs = a0 + 1, reward = a0 + 2,
    dones when the per-env step counter reaches episode_len."""

    def __init__(self, init_obs, episode_len):
        self.N = init_obs.shape[0]
        self.obs = init_obs.astype(np.float32).copy()
        self.L = episode_len
        self.counter = np.zeros(self.N, np.int64)

    def step(self, acts):
        self.counter += 1
        done = (self.counter == self.L).astype(np.uint8)
        self.counter %= self.L
        self.obs = (acts[:, 0] + 1).astype(np.float32)[:, None]
        return self.obs.copy(), (acts[:, 0] + 2).astype(np.float32), done


def fake_policy(bias):
    """FakeNet (test_rollouts.py:201-215) + critic `+1` (312-313)."""
    def fn(obs):
        a = (obs[:, 0] + bias).astype(np.int32)[:, None]
        return a, np.zeros((obs.shape[0], 1), np.float32), (2 * obs[:, 0] + 1).astype(np.float32)
    return fn


@pytest.mark.parametrize("T,L", [(32, 8), (32, 5), (12, 12), (20, 32)])
def test_rollout_integer_kat(T, L):
    rng = np.random.default_rng(T * 100 + L)
    N, bias, gamma = 16, 3, 0.5
    o0 = rng.integers(0, 1000, (N, 1)).astype(np.float32)
    sim = FakeSim(o0, L)
    store, er = ref.rollout(None, None, sim, T, None, None, 0, gamma=gamma,
                            policy_fn=fake_policy(bias))
    t = np.arange(T)[:, None]
    # closed forms: obs_t = o0 + t (bias + 1), a_t = obs_t + bias
    obs = o0[None, :, 0] + t * (bias + 1)
    assert np.array_equal(store["obs"][..., 0], obs)
    assert np.array_equal(store["actions"][..., 0], obs + bias)
    assert np.array_equal(store["values"], 2 * obs + 1)
    assert np.array_equal(store["rewards"], obs + bias + 2)
    assert np.array_equal(store["dones"], np.broadcast_to(((t + 1) % L == 0), (T, N)))
    # bootstrap = critic on the observation after the last step
    assert np.array_equal(store["bootstrap"], 2 * (o0[:, 0] + T * (bias + 1)) + 1)
    # env returns: running discounted sum, reset after each episode end
    tr = np.zeros((T, N))
    run = np.zeros(N)
    for i in range(T):
        run = store["rewards"][i] + gamma * run
        tr[i] = run
        if (i + 1) % L == 0:
            run = np.zeros(N)
    np.testing.assert_allclose(store["env_returns_trace"], tr, rtol=1e-6)
    np.testing.assert_allclose(er, run, rtol=1e-6)


@pytest.mark.parametrize("L", [8, 5])
def test_gae_on_kat_store(L):
    """gamma = lambda = 1: A_t = sum of rewards to the episode end (+ bootstrap
    if the episode is still running at T) - V_t."""
    T, N, bias = 32, 8, 1
    o0 = np.arange(N, dtype=np.float32)[:, None] * 10
    store, _ = ref.rollout(None, None, FakeSim(o0, L), T, None, None, 0,
                           policy_fn=fake_policy(bias))
    adv, ret = ref.gae_f32(store["rewards"], store["values"], store["dones"],
                           store["bootstrap"], 1.0, 1.0)
    r = store["rewards"].astype(np.float64)
    want = np.zeros((T, N))
    for i in range(T):
        end = (i // L + 1) * L  # first step index after this episode
        if end <= T:
            want[i] = r[i:end].sum(0)
        else:
            want[i] = r[i:].sum(0) + store["bootstrap"]
    want -= store["values"]
    np.testing.assert_allclose(adv, want, rtol=1e-6, atol=1e-3)
    np.testing.assert_allclose(ret, adv + store["values"], rtol=1e-6)
