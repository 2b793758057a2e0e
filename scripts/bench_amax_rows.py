"""ds2_amax rows-only pass (amax_rows_kernel) at the step's dgx shape (16032 x 2400 fp32): mean
device time per call over CUDA events; DS2_LIB_PATH selects the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'deepspeech.pytorch_amd'))
from ds2amd import _lib, ops   # noqa: E402

x = torch.randn(16032, 2400, device='cuda')
r = torch.zeros(16032, dtype=torch.int32, device='cuda')
for _ in range(3):
    _lib.call("ds2_amax", x.data_ptr(), 16032, 2400, 2400, r.data_ptr(), None, ops._stream())
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    _lib.call("ds2_amax", x.data_ptr(), 16032, 2400, 2400, r.data_ptr(), None, ops._stream())
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 50 * 1e3
print(f"{os.path.basename(os.environ.get('DS2_LIB_PATH', 'libds2hip.so'))}: {us:.1f} us per rows "
      f"pass ({x.numel() * 4 / us / 1e3:.0f} GB/s)")
