"""CTC loss with the warpctc_pytorch.CTCLoss interface (ref train.py:12,904,600-602).

``CTCLoss()(acts[T,N,C], labels int32 flat, act_lens int32[N], label_lens int32[N])``
returns the summed cost as a 1-element tensor on the activations' device (warp-ctc
returns it on the host; the caller's ``loss.to(device)`` is then a no-op and no
host sync is forced).  Softmax is applied inside; the gradient is taken with
respect to the unnormalised activations and is produced by the same kernel launch
as the cost (ds2_ctc_loss).

Infeasible samples (more required frames than act_len): cost +inf and zero
gradient, or cost 0 with ``zero_infinity=True``.  warp-ctc's own behaviour for
them is not pinned by any reference test.
"""
from __future__ import annotations

import torch

from . import ops


class CTCLoss(torch.nn.Module):
    def __init__(self, blank=0, size_average=False, length_average=False, zero_infinity=False):
        super().__init__()
        self.blank = blank
        self.size_average = size_average
        self.length_average = length_average
        self.zero_infinity = zero_infinity

    def forward(self, acts, labels, act_lens, label_lens):
        if not acts.is_cuda:
            raise RuntimeError("ds2amd CTCLoss runs on the GPU (HIP kernel)")
        dev = acts.device
        label_lens_h = label_lens.cpu().int() if label_lens.is_cuda else label_lens.int()
        max_l = int(label_lens_h.max()) if label_lens_h.numel() else 0
        labels_d = labels.to(dev, torch.int32, non_blocking=True).contiguous()
        act_lens_d = act_lens.to(dev, torch.int32, non_blocking=True).contiguous()
        label_lens_d = label_lens_h.to(dev, non_blocking=True).contiguous()
        c = acts.shape[2]
        if labels.numel() and not labels.is_cuda:   # host labels (the reference's case)
            lo, hi = int(labels.min()), int(labels.max())
            if lo < 0 or hi >= c:
                raise ValueError(f"CTC labels must lie in [0, {c}), got [{lo}, {hi}]")
        loss = ops.CTCLossFn.apply(acts, labels_d, act_lens_d, label_lens_d, max_l, self.blank,
                                   self.zero_infinity, self.size_average)
        if self.length_average:
            loss = loss / max(1, int(label_lens_h.sum()))
        return loss.reshape(1)
