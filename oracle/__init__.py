"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference's batched-PPO hot path
(shacklettbp/madrona-learn, src/madrona_learn/), used by tests/,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg — and
only there, as the checker or as the timed CPU baseline.  The product path
(madrona-learn_amd/) never imports, links or executes anything in here.

Contents
  ref_rng.c   Philox4x32-10, the deterministic Gumbel-max sampler and the
              synthetic env in plain C (bit-exact twins of the HIP code);
              built by oracle/Makefile into oracle/_build/liboracle.so.
  native.py   ctypes loader of liboracle.so.
  ppo_ref.py  NumPy restatement (fp64, fp32 and bf16-emulating modes) of
              GAE/returns, zscore, the discrete distributions, the MLP +
              LayerNorm actor-critic forward and its backward, the PPO loss,
              clip_by_global_norm + Adam, the weight-norm / LayerNorm
              projections, the minibatch permutation and the full update.

Pinning status (see DESIGN.md "Oracle"): the reference is pure JAX/Flax/Optax
and JAX is not installed in this image (an ordinary ModuleNotFoundError, not
a refusal), and the reference's own tests hold no golden vectors for these
functions.  The oracle is therefore pinned by
  * the Random123 known-answer vectors for Philox4x32-10,
  * closed-form known-answer cases derived from the reference's equations
    (GAE, returns, zscore, PPO loss, Adam, projections),
  * the reference's integer fake-policy rollout design
    (tests/test_rollouts.py:191-298, 380-460) restated,
  * fp64 autograd (torch, CPU) cross-checks of its hand-written backward.
Floating-point results beyond those cases are "parity unpinned" against
executed reference output.
"""
