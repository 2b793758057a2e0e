"""Training-step time of the headline batch (32 x 10 s, 5 bidirectional layers of 800) per
rnn_type: 'gru' (the headline), 'rnn' (nn.RNN tanh on the one-gate persistent recurrences;
DS2_RNN_PERSISTENT=0 selects the per-step kernels) and optionally 'lstm' -- VERDICT r4 item 8
asks a 5 x RNN-800 step to run within 1.5x of the GRU step.  One JSON line per type.

usage: python scripts/bench_rnn_type.py [--types gru,rnn] [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
from ds2amd import model as dsm  # noqa: E402
from ds2amd.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--types", default="gru,rnn")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    x, tg, pct, ts = bench.synthetic_batch(0)
    x = x.to(dev)
    for rt in args.types.split(","):
        torch.manual_seed(123456)
        m = dsm.DeepSpeech(rnn_type=rt, labels=bench.LABELS, rnn_hidden_size=bench.HIDDEN,
                           nb_layers=bench.LAYERS, audio_conf=bench.CONF, bidirectional=True)
        tr = Trainer(m, bench.LABELS, lr=3e-4, momentum=0.9, max_norm=100.0, device=dev,
                     score=True, verbose=False)

        def step():
            return tr.train_batch((x, tg, None, pct.clone(), ts))

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        t0 = time.perf_counter()
        marks[0].record()
        loss = None
        for i in range(args.steps):
            loss = step()
            marks[i + 1].record()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tr.poll_status(block=True)
        ms = sorted(marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps))
        print(json.dumps({"rnn_type": rt, "layers": bench.LAYERS, "hidden": bench.HIDDEN,
                          "batch": bench.BATCH, "ms_per_step": round(dt * 1e3 / args.steps, 3),
                          "ms_per_step_median": round(ms[len(ms) // 2], 3),
                          "audio_seconds_per_sec": round(bench.BATCH * bench.SECONDS /
                                                         (dt / args.steps), 1),
                          "loss": float(loss) if loss is not None else None,
                          "persistent": os.environ.get("DS2_RNN_PERSISTENT", "1")}), flush=True)
        del tr, m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
