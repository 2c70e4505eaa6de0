"""Host logic of the torch path (madrona_learn/generic.py) that needs no GPU:
the recurrent-state pytree helpers the rollout uses to save the carry
entering every BPTT chunk (rnn_start_states, rollouts.py:528-537) and the
minibatch gather of those start states, on rnn.LSTM's (c_states, h_states)
structure (rnn.py:52-81), and the fused-path admission rules that route a
tree to the torch path."""

import torch


def test_start_state_save_and_gather():
    from madrona_learn.generic import _map_leaves, _zip_leaves
    from madrona_learn.rnn import LSTM
    N, C, R, L = 6, 3, 4, 2
    lstm = LSTM(R, L, torch.float32)
    live = lstm.init_recurrent_state(N)
    start = _map_leaves(lambda x: torch.zeros((C, *x.shape), dtype=x.dtype), live)
    assert len(start[0]) == L and start[0][0].shape == (C, N, R)
    for c in range(C):
        live = _map_leaves(lambda x: x + 1.0, live)
        _zip_leaves(lambda dst, src: dst[c].copy_(src), start, live)
    for c in range(C):
        for leaf in start[0] + start[1]:
            assert torch.all(leaf[c] == c + 1)
    # minibatch of sequences seq = c * N + b (RolloutData.minibatch)
    seq = torch.tensor([0, 7, 17, 12])
    cc, bb = seq // N, seq % N
    got = _map_leaves(lambda x: x[cc, bb], start)
    assert got[1][1].shape == (4, R)
    assert torch.equal(got[0][0][:, 0], (cc + 1).float())


def test_clear_recurrent_state_masks_rows():
    from madrona_learn.rnn import LSTM
    lstm = LSTM(3, 2, torch.float32)
    c, h = lstm.init_recurrent_state(4)
    c = [x + 2.0 for x in c]
    h = [x - 1.0 for x in h]
    c2, h2 = lstm.clear_recurrent_state((c, h), torch.tensor([True, False, True, False]))
    for x in c2 + h2:
        assert torch.all(x[0] == 0) and torch.all(x[2] == 0)
        assert torch.all(x[1] != 0) and torch.all(x[3] != 0)


def test_fused_admission_routes_other_shapes():
    import madrona_learn as ml
    from madrona_learn.models import MLP, DenseLayerCritic, DenseLayerDiscreteActor
    from madrona_learn.rnn import LSTM
    from madrona_learn.train_state import compile_arch

    def tree(net, rnn=None, dt=torch.float32):
        enc = ml.BackboneEncoder(net=net) if rnn is None else \
            ml.RecurrentBackboneEncoder(net=net, rnn=rnn)
        return ml.ActorCritic(backbone=ml.BackboneShared(encoder=enc),
                              actor=DenseLayerDiscreteActor(ml.DiscreteActionsConfig([4, 3]), dt),
                              critic=DenseLayerCritic(dt))

    compile_arch(tree(MLP(256, 2, torch.float32)), 64, torch.float32)  # fused
    for bad, D in ((tree(MLP(96, 2, torch.float32)), 64), (tree(MLP(64, 5, torch.float32)), 64),
                   (tree(MLP(64, 1, torch.float32), LSTM(64, 2, torch.float32)), 64),
                   (tree(MLP(64, 2, torch.float32)), 40)):
        try:
            compile_arch(bad, D, torch.float32)
        except NotImplementedError:
            continue
        raise AssertionError("expected the torch path")


def test_carry_back_keeps_addresses():
    """generic._carry_back: state carried between updates (sim state, current
    observations, recurrent carry, preprocess estimates) returns to the
    tensors it started in -- what a HIP-graph replay of the whole torch-path
    update reads at its start -- and is left as is where the structure,
    shapes or dtypes changed."""
    from madrona_learn.generic import _carry_back
    start = {"obs": torch.zeros(4, 3), "state": [torch.zeros(4, dtype=torch.int32), 7]}
    cur = {"obs": torch.ones(4, 3), "state": [torch.full((4,), 5, dtype=torch.int32), 7]}
    out = _carry_back(start, cur)
    assert out is start and out["obs"] is start["obs"]
    assert torch.equal(start["obs"], torch.ones(4, 3))
    assert torch.equal(start["state"][0], torch.full((4,), 5, dtype=torch.int32))
    same = torch.arange(3.0)
    assert _carry_back(same, same) is same  # an in-place sim: nothing to copy
    wide = {"obs": torch.ones(4, 5), "state": [torch.zeros(4, dtype=torch.int32), 7]}
    assert _carry_back(start, wide) is wide  # a shape changed
    other = {"obs": torch.ones(4, 3), "state": [torch.zeros(4, dtype=torch.int32), 8]}
    assert _carry_back(start, other) is other  # a non-tensor leaf changed
    assert _carry_back(start, {"obs": torch.ones(4, 3)}) is not start  # keys changed
