"""Matrix-core operand images of the compute-dtype weights (include/mlearn.h,
csrc/rowtile.h img_index).

A logical matrix Wimg[N][K] (N = output feature of the product, K = its
reduction index) is stored so that one wave's A fragment for one MFMA step is
a single contiguous run.  ``perm`` selects the k order of B fragments taken
straight from accumulator registers.  Host helpers for tests and checkpoint
export; the kernels write the images on device (mlearn_policy_sync_weights,
mlearn_optim_step)."""

import numpy as np
import torch


def img_index(N, K, dtype, perm):
    """int64 [N][K] array: position of Wimg[n][k] in the image."""
    n = np.arange(N)[:, None]
    k = np.arange(K)[None, :]
    if dtype == torch.bfloat16:
        kk = k & 15
        s = k >> 4
        if perm:
            h = (kk >> 2) & 1
            e = ((kk >> 3) << 2) | (kk & 3)
        else:
            h = kk >> 3
            e = kk & 7
        return (((n >> 5) * (K >> 4) + s) * 64 + (n & 31) + 32 * h) * 8 + e
    if perm:
        kk = k & 31
        h = (kk >> 2) & 1
        s = ((k >> 5) << 4) | ((kk >> 3) << 2) | (kk & 3)
    else:
        h = k & 1
        s = k >> 1
    return ((n >> 5) * (K >> 1) + s) * 64 + (n & 31) + 32 * h


def from_image(img, N, K, perm):
    """Logical Wimg[N][K] (torch, same dtype) from a 1-D image tensor."""
    idx = torch.from_numpy(img_index(N, K, img.dtype, perm)).to(img.device)
    return img.reshape(-1)[idx.reshape(-1)].reshape(N, K)


def to_image(m, perm):
    """1-D image of a logical Wimg[N][K] torch tensor (N a multiple of 32)."""
    N, K = m.shape
    idx = torch.from_numpy(img_index(N, K, m.dtype, perm)).to(m.device).reshape(-1)
    img = torch.zeros(N * K, dtype=m.dtype, device=m.device)
    img[idx] = m.reshape(-1)
    return img
