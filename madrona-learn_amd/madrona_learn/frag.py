"""Fragment-order weight images (include/mlearn.h, csrc/common.h frag_index).

A logical matrix Bt[N][K] is stored so that the 64 lane fragments of one
matrix-core step are contiguous.  These host helpers build / read the images
(tests, checkpoint export); the kernels write them on device
(mlearn_policy_sync_weights, mlearn_optim_step)."""

import numpy as np
import torch


def _ek(dtype):
    return (8, 16) if dtype == torch.bfloat16 else (1, 2)


def frag_index(N, K, dtype):
    """int64 [N][K] array: position of Bt[n][k] in the image."""
    E, KS = _ek(dtype)
    n = np.arange(N)[:, None]
    k = np.arange(K)[None, :]
    kk = k % KS
    return (((n // 32) * (K // KS) + k // KS) * 64 + (n % 32) + 32 * (kk // E)) * E + kk % E


def from_image(img, N, K):
    """Logical Bt[N][K] (torch, same dtype) from a 1-D image tensor."""
    idx = torch.from_numpy(frag_index(N, K, img.dtype)).to(img.device)
    return img.reshape(-1)[idx.reshape(-1)].reshape(N, K)


def to_image(bt):
    """1-D image of a logical Bt[N][K] torch tensor (N a multiple of 32)."""
    N, K = bt.shape
    idx = torch.from_numpy(frag_index(N, K, bt.dtype)).to(bt.device).reshape(-1)
    img = torch.zeros(N * K, dtype=bt.dtype, device=bt.device)
    img[idx] = bt.reshape(-1)
    return img
