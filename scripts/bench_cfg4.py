"""BASELINE cfg4 measurement (not the headline bench line): DS2 with 7 x (Bi)LSTM-1024,
batch 64, 10 s synthetic spectrograms, one full training step (forward, CTC, backward,
clip + SGD) per timed iteration on one GPU.  Unidirectional models carry the Lookahead
(context 20) + Hardtanh head of model.py:329-333.

usage: python scripts/bench_cfg4.py [--bidir 0|1] [--rnn-gemm fp32|bf16] [--steps K]
                                   [--warmup W] [--batch N]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402  (synthetic batch + labels of the headline bench)


def recurrence_label(rnn_gemm):
    """The LSTM recurrences' arithmetic as ops.LSTMLayerFn will run it."""
    h3 = os.environ.get("DS2_LSTM_H3", "1")[:1] != "0"
    fwd = "fp16x3" if h3 else "fp32 MFMA"
    if rnn_gemm == "bf16" and os.environ.get("DS2_LSTM_HALF", "1")[:1] != "0":
        return f"recurrence fwd {fwd}, bwd single-term fp16"
    return f"recurrence {fwd}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bidir", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=7)
    ap.add_argument("--rnn-gemm", choices=["fp32", "bf16"], default="fp32",
                    help="precision of the recurrent layers' GEMMs (cfg4 names bf16)")
    args = ap.parse_args()
    from ds2amd import model as dsm
    from ds2amd.trainer import Trainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(123456)
    m = dsm.DeepSpeech(rnn_type='lstm', labels=bench.LABELS, rnn_hidden_size=args.hidden,
                       nb_layers=args.layers, audio_conf=bench.CONF,
                       bidirectional=bool(args.bidir), rnn_gemm_precision=args.rnn_gemm)
    tr = Trainer(m, bench.LABELS, lr=3e-4, momentum=0.9, max_norm=100.0, device=dev)
    bench.BATCH = args.batch
    x, tg, pct, ts = bench.synthetic_batch(0)
    x = x.to(dev)

    def step():
        return tr.train_batch((x, tg, None, pct.clone(), ts))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({
        "config": f"cfg4: {args.layers}x{'Bi' if args.bidir else ''}LSTM-{args.hidden}"
                  f"{'' if args.bidir else ' + lookahead(20)'}, batch {args.batch}, 10 s, "
                  f"RNN GEMMs {args.rnn_gemm}, " + recurrence_label(args.rnn_gemm) + ", rest fp32",
        "audio_seconds_per_sec": round(args.batch * bench.SECONDS * args.steps / dt, 2),
        "ms_per_step": round(dt * 1e3 / args.steps, 2), "loss": round(float(loss), 4),
        "steps": args.steps}), flush=True)


if __name__ == "__main__":
    main()
