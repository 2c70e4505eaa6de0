"""ctypes binding of the C-ABI hot-path library (``include/mlearn.h``).

``libmlearn.so`` is built in-tree by ``make -C madrona-learn_amd`` (hipcc,
gfx950).  This module is the only place that touches it: every caller passes
torch device tensors, which are lowered here to raw pointers plus the current
HIP stream.  There is no fallback: if the library is missing or fails to load
the import of any compute path raises.
"""

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int32, c_int64,
                    c_uint32, c_uint64, c_void_p)

import torch

LIB_PATH = os.environ.get(
    "MADRONA_LEARN_LIB",
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libmlearn.so"))
ABI_VERSION = 22

DTYPE_F32 = 0
DTYPE_BF16 = 1
MAX_LAYERS = 4
MAX_GROUPS = 16
HEAD_COLS = 32       # head width with a scalar critic
HEAD_COLS_MAX = 96   # head width when actor logits + critic bins exceed 32


class ActionLayout(Structure):
    _fields_ = [("num_groups", c_int32), ("num_logits", c_int32),
                ("offsets", c_int32 * (MAX_GROUPS + 1))]


class MlpPolicy(Structure):
    _fields_ = [("dtype", c_int32), ("obs_dim", c_int32), ("hidden", c_int32),
                ("num_layers", c_int32), ("critic_bins", c_int32), ("actions", ActionLayout),
                ("w_t", c_void_p * MAX_LAYERS), ("w", c_void_p * MAX_LAYERS),
                ("ln_scale", c_void_p * MAX_LAYERS), ("ln_bias", c_void_p * MAX_LAYERS),
                ("head_t", c_void_p), ("head", c_void_p), ("head_bias", c_void_p),
                ("obs_mu", c_void_p), ("obs_inv_sigma", c_void_p), ("obs_stats", c_void_p),
                ("obs_stats_tiles", c_int64), ("obs_stats_steps", c_int32),
                ("obs_pad", c_int32)]


class MetricJob(Structure):
    _fields_ = [("x", c_void_p), ("n", c_int64), ("cols", c_int64), ("ld", c_int64),
                ("abs_value", c_int32), ("pad", c_int32), ("x2", c_void_p)]


class PostStep(Structure):
    _fields_ = [("rewards", c_void_p), ("dones", c_void_p), ("store_rewards", c_void_p),
                ("store_dones", c_void_p), ("env_returns", c_void_p),
                ("env_returns_trace", c_void_p), ("gamma", c_float)]


class RolloutView(Structure):
    _fields_ = [("obs", c_void_p), ("actions", c_void_p), ("log_probs", c_void_p),
                ("advantages", c_void_p), ("returns", c_void_p), ("values", c_void_p),
                ("dones", c_void_p), ("T", c_int32), ("bptt_len", c_int32), ("N", c_int64),
                ("ld", c_int64)]


class PPOHparams(Structure):
    _fields_ = [("clip_coef", c_float), ("value_loss_coef", c_float),
                ("entropy_coef", c_float * MAX_GROUPS), ("normalize_advantages", c_int32),
                ("clip_value_loss", c_int32), ("huber_value_loss", c_int32),
                ("loss_scale", c_float), ("normalize_values", c_int32),
                ("obj_weight", c_float * MAX_GROUPS),
                ("grad_sumsq_out", c_void_p), ("step_kernel", c_int32), ("wgrad_form", c_int32)]


class FlatGroup(Structure):  # mlearn_flat_group
    _fields_ = [("offset", c_int64), ("count", c_int64), ("offset2", c_int64), ("count2", c_int64),
                ("kind", c_int32), ("features", c_int32), ("init_norm", c_float),
                ("pad", c_int32)]


class FlatOptim(Structure):  # mlearn_flat_optim
    _fields_ = [("params", c_void_p), ("grads", c_void_p), ("adam_m", c_void_p),
                ("adam_v", c_void_p), ("step", c_void_p), ("n", c_int64), ("groups", c_void_p),
                ("num_groups", c_int32), ("lr", c_float), ("b1", c_float), ("b2", c_float),
                ("eps", c_float), ("max_grad_norm", c_float), ("normalize_params", c_int32),
                ("normalize_layernorms", c_int32), ("skip_nonfinite", c_int32)]


class OptimState(Structure):
    _fields_ = [("params", c_void_p), ("grads", c_void_p), ("adam_m", c_void_p),
                ("adam_v", c_void_p), ("init_norms", c_void_p), ("step", c_void_p),
                ("lr", c_float), ("b1", c_float), ("b2", c_float), ("eps", c_float),
                ("max_grad_norm", c_float), ("normalize_params", c_int32),
                ("normalize_layernorms", c_int32), ("grad_sumsq_part", c_void_p),
                ("grad_sumsq_nparts", c_int64), ("launch_form", c_int32), ("pad_", c_int32)]


class Lstm(Structure):  # mlearn_lstm
    _fields_ = [("hidden", c_int32), ("num_layers", c_int32), ("wi_perm", c_void_p),
                ("wi_nat", c_void_p), ("wh_nat", c_void_p), ("w_bwd", c_void_p),
                ("head_t_nat", c_void_p), ("bias", c_void_p)]


class LstmCarry(Structure):  # mlearn_lstm_carry
    _fields_ = [("h", c_void_p), ("c", c_void_p), ("start_h", c_void_p), ("start_c", c_void_p),
                ("commit", c_int32), ("pad", c_int32), ("clear", c_void_p)]


class DummyEnv(Structure):  # mlearn_dummy_env
    _fields_ = [("state", c_void_p), ("obs", c_void_p), ("rewards", c_void_p),
                ("dones", c_void_p), ("k0", c_uint32), ("k1", c_uint32),
                ("env_offset", c_uint32), ("pad", c_uint32)]


class RolloutOut(Structure):  # mlearn_rollout_out
    _fields_ = [("obs", c_void_p), ("actions", c_void_p), ("log_probs", c_void_p),
                ("values", c_void_p), ("rewards", c_void_p), ("dones", c_void_p),
                ("env_returns_trace", c_void_p), ("bootstrap", c_void_p),
                ("env_returns", c_void_p), ("start_h", c_void_p), ("start_c", c_void_p),
                ("T", c_int32), ("bptt_len", c_int32), ("ld", c_int64), ("gamma", c_float),
                ("max_workgroups", c_int32), ("policy_kernel", c_int32),
                ("advantages", c_void_p), ("gae_gamma", c_float), ("gae_gamma_lambda", c_float)]


_S = c_void_p  # hipStream_t
_P = c_void_p

# name -> (restype, argtypes)
_SIGNATURES = {
    "mlearn_last_error": (c_char_p, []),
    "mlearn_abi_version": (c_int32, []),
    "mlearn_grad_sumsq_parts": (c_int64, [c_int64]),
    "mlearn_philox4x32_host": (c_int32, [_P, c_uint32, c_uint32, _P, c_int64]),
    "mlearn_comm_unique_id": (c_int32, [_P]),
    "mlearn_lstm_activations_f32": (c_int32, [_P, c_int64, _P, _P, _S]),
    "mlearn_comm_init": (c_int32, [_P, c_int32, c_int32, POINTER(c_void_p)]),
    "mlearn_comm_destroy": (c_int32, [c_void_p]),
    "mlearn_allreduce_f32": (c_int32, [c_void_p, _P, c_int64, _S]),
    "mlearn_allreduce_f64": (c_int32, [c_void_p, _P, c_int64, _S]),
    "mlearn_philox4x32": (c_int32, [_P, c_uint32, c_uint32, _P, c_int64, _S]),
    "mlearn_counters_add": (c_int32, [_P, c_int32, POINTER(c_uint64), _S]),
    "mlearn_ema_input_stats": (c_int32, [_P, c_int64, c_int32, _P, c_int32, _P, _S]),
    "mlearn_ema_update_estimates": (c_int32, [_P, c_int32, c_float, c_float, _P, _P, _S]),
    "mlearn_gae_f32": (c_int32, [_P, _P, _P, _P, _P, _P, c_int32, c_int64, c_float, c_float, _S]),
    "mlearn_gae_vnorm_f32": (c_int32, [_P, _P, _P, _P, _P, c_int64, _P, _P, c_int32, c_int64,
                                       c_float, c_float, _S]),
    "mlearn_returns_f32": (c_int32, [_P, _P, _P, _P, c_int32, c_int64, c_float, _S]),
    "mlearn_zscore_workspace_bytes": (c_int64, [c_int64]),
    "mlearn_zscore_f32": (c_int32, [_P, c_int64, _P, _P, _S]),
    "mlearn_discrete_sample_f32": (c_int32, [_P, c_int64, ActionLayout, c_int64, c_uint32,
                                             c_uint32, _P, c_uint64, c_uint32, c_int32, _P, _P,
                                             _S]),
    "mlearn_action_stats_f32": (c_int32, [_P, c_int64, ActionLayout, c_int64, _P, _P, _P, _S]),
    "mlearn_policy_rollout_step": (c_int32, [POINTER(MlpPolicy), _P, c_int64, _P, _P, _P, _P,
                                             c_uint32, c_uint32, _P, c_uint64, c_uint32, c_int32,
                                             POINTER(PostStep), _S]),
    "mlearn_policy_rollout_step_env": (c_int32, [POINTER(MlpPolicy), _P, c_int64, _P, _P, _P,
                                                 _P, c_uint32, c_uint32, _P, c_uint64, c_uint32,
                                                 c_int32, POINTER(PostStep), POINTER(DummyEnv),
                                                 _S]),
    "mlearn_lstm_policy_rollout_step_env": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm),
                                                      POINTER(LstmCarry), _P, c_int64, _P, _P, _P,
                                                      _P, c_uint32, c_uint32, _P, c_uint64,
                                                      c_uint32, c_int32, POINTER(PostStep),
                                                      POINTER(DummyEnv), _S]),
    "mlearn_policy_rollout_env": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), POINTER(LstmCarry),
                                            _P, c_int64,
                                            POINTER(RolloutOut), c_uint32, c_uint32, _P,
                                            c_uint32, POINTER(DummyEnv), _S]),
    "mlearn_policy_rollout_workgroups": (c_int64, [POINTER(MlpPolicy), POINTER(Lstm), c_int64,
                                                   c_int32]),
    "mlearn_policy_rollout_kernel": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), c_int64, c_int32,
                                               c_int32]),
    "mlearn_policy_pop_bytes": (c_int64, [c_int32]),
    "mlearn_policy_pop_prepare": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), POINTER(LstmCarry),
                                            _P, c_int64, POINTER(RolloutOut), _P,
                                            POINTER(DummyEnv), c_int32, _P, _S]),
    "mlearn_policy_rollout_env_pop": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), _P, c_int32,
                                                c_int64, c_uint32, c_uint32, _P, c_int32, _S]),
    "mlearn_policy_rollout_pop_workgroups": (c_int64, [POINTER(MlpPolicy), POINTER(Lstm),
                                                       c_int64, c_int32, c_int32]),
    "mlearn_policy_evaluate": (c_int32, [POINTER(MlpPolicy), _P, c_int64, _P, _P, _P, _P, _S]),
    "mlearn_lstm_policy_evaluate": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), POINTER(LstmCarry),
                                              _P, c_int64, _P, _P, _P, _P, _S]),
    "mlearn_rollout_post_step": (c_int32, [_P, _P, c_int64, _P, _P, _P, _P, c_float, _S]),
    "mlearn_metrics_workspace_bytes": (c_int64, [c_int32]),
    "mlearn_metrics_f32": (c_int32, [POINTER(MetricJob), c_int32, _P, _P, _S]),
    "mlearn_minibatch_perm": (c_int32, [c_uint32, c_uint32, _P, c_uint64, c_uint32, c_int32, _P,
                                        _S]),
    "mlearn_adv_stats": (c_int32, [POINTER(RolloutView), _P, c_int32, c_int32, _P, _S]),
    "mlearn_adv_stats_finish": (c_int32, [_P, c_int32, c_double, _P, _S]),
    "mlearn_return_stats": (c_int32, [POINTER(RolloutView), _P, c_int32, c_int32, _P, _S]),
    "mlearn_value_norm_chain": (c_int32, [_P, _P, c_int32, c_double, c_float, c_float, _P, _P, _P,
                                          _S]),
    "mlearn_ppo_workspace_bytes": (c_int64, [POINTER(MlpPolicy), c_int64]),
    "mlearn_ppo_step_kernel": (c_int32, [POINTER(MlpPolicy), c_int64, c_int32]),
    "mlearn_policy_rollout_pop_kernel": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), c_int64,
                                                   c_int32, c_int32]),
    "mlearn_ppo_minibatch_grad": (c_int32, [POINTER(MlpPolicy), POINTER(RolloutView), _P,
                                            c_int32, _P, POINTER(PPOHparams), _P, _P, _P, _S]),
    "mlearn_ppo_minibatch_fwd_bwd": (c_int32, [POINTER(MlpPolicy), POINTER(RolloutView), _P,
                                               c_int32, _P, POINTER(PPOHparams), _P, _S]),
    "mlearn_param_count": (c_int64, [POINTER(MlpPolicy)]),
    "mlearn_head_cols": (c_int32, [POINTER(MlpPolicy)]),
    "mlearn_obs_norm_update": (c_int32, [_P, c_int32, c_int64, c_int64, c_int32, c_float, c_float,
                                         _P, _P, _S]),
    "mlearn_optim_workspace_bytes": (c_int64, [POINTER(MlpPolicy)]),
    "mlearn_flat_optim_workspace_bytes": (c_int64, [c_int64, c_int32]),
    "mlearn_flat_optim_step": (c_int32, [POINTER(FlatOptim), _P, _S]),
    "mlearn_optim_step": (c_int32, [POINTER(MlpPolicy), POINTER(OptimState), _P, _S]),
    "mlearn_policy_sync_weights": (c_int32, [POINTER(MlpPolicy), _P, _S]),
    "mlearn_lstm_param_offset": (c_int64, [POINTER(MlpPolicy)]),
    "mlearn_lstm_param_count": (c_int64, [POINTER(MlpPolicy), POINTER(Lstm)]),
    "mlearn_lstm_policy_rollout_step": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm),
                                                  POINTER(LstmCarry), _P, c_int64, _P, _P, _P, _P,
                                                  c_uint32, c_uint32, _P, c_uint64, c_uint32,
                                                  c_int32, POINTER(PostStep), _S]),
    "mlearn_lstm_ppo_workspace_bytes": (c_int64, [POINTER(MlpPolicy), POINTER(Lstm), c_int64,
                                                  c_int32]),
    "mlearn_lstm_ppo_minibatch_grad": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm),
                                                 POINTER(RolloutView), _P, _P, _P, c_int32, _P,
                                                 POINTER(PPOHparams), _P, _P, _P, _S]),
    "mlearn_lstm_optim_workspace_bytes": (c_int64, [POINTER(MlpPolicy), POINTER(Lstm)]),
    "mlearn_lstm_optim_step": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), POINTER(OptimState),
                                         _P, _S]),
    "mlearn_lstm_sync_weights": (c_int32, [POINTER(MlpPolicy), POINTER(Lstm), _P, _S]),
    "mlearn_dummy_env_step": (c_int32, [_P, _P, c_int32, c_int64, c_int32, c_uint32, c_uint32,
                                        c_uint32, _P, _P, _P, _S]),
    "mlearn_dummy_env_reset": (c_int32, [_P, c_int64, c_int32, c_uint32, c_uint32, c_uint32, _P,
                                         _S]),
}

EXPORTED = tuple(_SIGNATURES.keys())

_lib = None


def _hip_runtimes_mapped():
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return paths


def lib():
    """Load (once) and return the ctypes handle.  Raises if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"madrona_learn: native library {LIB_PATH} is missing; build it with "
            "`make -C madrona-learn_amd` (hipcc --offload-arch=gfx950). There is no CPU "
            "fallback.")
    # torch is imported first so its HIP runtime (soname libamdhip64.so.7) is the
    # one the library binds to: one runtime, shared streams.
    h = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    v = h.mlearn_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"madrona_learn: ABI version {v}, expected {ABI_VERSION}")
    rts = _hip_runtimes_mapped()
    if len(rts) > 1:
        raise RuntimeError(f"madrona_learn: several HIP runtimes mapped: {sorted(rts)}")
    _lib = h
    return h


def check(rc, what=""):
    if rc != 0:
        msg = lib().mlearn_last_error().decode(errors="replace")
        raise RuntimeError(f"madrona_learn native call {what} failed ({rc}): {msg}")


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return c_void_p(s.cuda_stream)


def ptr(t, dtype=None, numel=None, name="tensor"):
    """Device pointer of a contiguous CUDA tensor (with optional checks)."""
    if t is None:
        return None
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name}: must live on the GPU (got {t.device})")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name}: needs >= {numel} elements, has {t.numel()}")
    return c_void_p(t.data_ptr())


def action_layout(buckets):
    buckets = list(buckets)
    if not 1 <= len(buckets) <= MAX_GROUPS:
        raise ValueError(f"1..{MAX_GROUPS} discrete action groups supported, got {len(buckets)}")
    lay = ActionLayout()
    lay.num_groups = len(buckets)
    off = 0
    lay.offsets[0] = 0
    for i, b in enumerate(buckets):
        if b < 1:
            raise ValueError("every action needs >= 1 bucket")
        off += b
        lay.offsets[i + 1] = off
    lay.num_logits = off
    if off + 1 > HEAD_COLS_MAX:
        raise ValueError(f"at most {HEAD_COLS_MAX - 1} total logits supported, got {off}")
    return lay


def head_cols(num_logits, critic_bins):
    """Head width HC of mlearn_mlp_policy (include/mlearn.h)."""
    if num_logits + critic_bins <= HEAD_COLS:
        return HEAD_COLS
    if num_logits + critic_bins <= HEAD_COLS_MAX:
        return HEAD_COLS_MAX
    # NotImplementedError: such a tree is valid (e.g. DreamerV3Critic with
    # 255 bins) and trains on the torch path (train._fused_tree_problem)
    raise NotImplementedError(f"{num_logits} actor logits + {critic_bins} critic outputs "
                              f"exceed the fused kernels' {HEAD_COLS_MAX} head columns")


def dtype_code(dtype):
    if dtype == torch.bfloat16:
        return DTYPE_BF16
    if dtype == torch.float32:
        return DTYPE_F32
    raise ValueError(f"compute dtype {dtype} not supported (float32 or bfloat16)")
