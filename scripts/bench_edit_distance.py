"""CER/WER edit distances at the bench step's shape: 32 utterances, decoded id rows of ~400 ids
(a randomly initialised model's greedy output over T' = 501), 150-id references with spaces.
Mean device time per ds2_edit_distance call over CUDA events; DS2_LIB_PATH selects the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'deepspeech.pytorch_amd'))
from ds2amd import ops   # noqa: E402


def main():
    dev = torch.device('cuda:0')
    g = torch.Generator().manual_seed(5)
    n, width, lb, space = 32, 501, 150, 28
    a = torch.randint(1, 29, (n, width), generator=g, dtype=torch.int32)
    a_lens = torch.randint(350, 450, (n,), generator=g, dtype=torch.int32)
    b = torch.randint(1, 29, (n * lb,), generator=g, dtype=torch.int32)
    b_lens = torch.full((n,), lb, dtype=torch.int32)
    a, a_lens, b, b_lens = a.to(dev), a_lens.to(dev), b.to(dev), b_lens.to(dev)
    for _ in range(3):
        ops.edit_distance_raw(a, a_lens, b, b_lens, space)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        out, _ = ops.edit_distance_raw(a, a_lens, b, b_lens, space)
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.path.basename(os.environ.get('DS2_LIB_PATH', 'libds2hip.so'))}: "
          f"{e0.elapsed_time(e1) / reps * 1e3:.1f} us per ds2_edit_distance (N={n}, ~400 x {lb} ids); "
          f"checksum {int(out.sum())}")


if __name__ == '__main__':
    main()
