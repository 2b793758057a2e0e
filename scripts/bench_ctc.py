"""CTC loss + gradient at the bench shape (T' = 501, 32 utterances, 150 labels, 29 classes):
mean time per ds2_ctc_loss call (logsoftmax, prep, alpha/beta scans, gradient rows) over CUDA
events.  DS2_LIB_PATH selects the library (A/B of kernel variants)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'deepspeech.pytorch_amd'))
from ds2amd import ops   # noqa: E402


def main():
    dev = torch.device('cuda:0')
    g = torch.Generator().manual_seed(3)
    t, n, c, L = 501, 32, 29, 150
    acts = (torch.randn(t, n, c, generator=g) * 2).to(dev)
    labels = torch.randint(1, c, (n * L,), generator=g, dtype=torch.int32).to(dev)
    act_lens = torch.full((n,), t, dtype=torch.int32, device=dev)
    label_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    for _ in range(3):
        ops.ctc_loss_raw(acts, labels, act_lens, label_lens, L)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        ops.ctc_loss_raw(acts, labels, act_lens, label_lens, L)
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.path.basename(os.environ.get('DS2_LIB_PATH', 'libds2hip.so'))}: "
          f"{e0.elapsed_time(e1) / reps * 1e3:.1f} us per ds2_ctc_loss (T'={t}, N={n}, L={L})")


if __name__ == '__main__':
    main()
