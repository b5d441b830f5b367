"""Batched inference on the GPU (one thread per row over the flat tree)."""

from __future__ import annotations

import numpy as np
import torch

from . import native

__all__ = ["device_tree", "predict_leaves"]


def device_tree(est, device):
    """Upload (once) the estimator's tree as 16-B node records + fp64 thresholds."""
    cache = getattr(est, "_device_tree", None)
    if cache is not None and cache[0] == device:
        return cache[1], cache[2]
    ta = est._arrays
    rec = np.zeros((ta.node_count, 4), dtype=np.int32)
    rec[:, 0] = ta.feature
    rec[:, 1] = ta.left
    rec[:, 2] = ta.right
    thr = np.where(ta.feature >= 0, ta.threshold, 0.0).astype(np.float64)
    nodes = torch.from_numpy(rec).to(device)
    thr_d = torch.from_numpy(thr).to(device)
    est._device_tree = (device, nodes, thr_d)
    return nodes, thr_d


def predict_leaves(est, X: torch.Tensor) -> torch.Tensor:
    """Leaf index per row of a device feature matrix (int64 tensor on X's device)."""
    hip = native.hip()
    if X.dtype not in (torch.float32, torch.float64):
        X = X.double()
    X = X.contiguous()
    nodes, thr = device_tree(est, X.device)
    n, F = X.shape
    leaf = torch.empty(n, dtype=torch.int32, device=X.device)
    hip.predict(torch.cuda.current_stream(X.device).cuda_stream, X.data_ptr(),
                X.dtype == torch.float64, n, F, nodes.data_ptr(), thr.data_ptr(),
                leaf.data_ptr())
    return leaf.long()
