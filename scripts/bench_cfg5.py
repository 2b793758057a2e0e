"""BASELINE cfg5 measurement (not the headline bench line): batched transcribe.py inference,
30 s utterances, beam-search CTC decoder, one GPU.  Model: the headline DS2 5 x BiGRU-800
(random init, eval mode).  One timed iteration = raw 16 kHz PCM resident in HBM -> device
STFT + max_frame normalisation -> DeepSpeech.forward -> prefix beam search (beam 10,
cutoff_top_n 40: the reference's opts.py defaults; no LM) -> host strings
(ds2amd.transcribe.transcribe_batch on device arrays).  Greedy decoding is timed beside it.

usage: python scripts/bench_cfg5.py [--batch N] [--seconds S] [--beam W] [--iters K] [--stamps]

--stamps: also run one beam decode with the kernel's per-phase clock stamps on (utterance 0,
frames 1..255; ds2_test_beam_stamps) and print the mean time of each phase of a frame.
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

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--beam", type=int, default=10)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--lm", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                 "tests", "golden", "tiny_lm.arpa"),
                    help="ARPA model for the beam_lm line (default: the committed 3-gram fixture)")
    args = ap.parse_args()
    from ds2amd import model as dsm, ops
    from ds2amd.data_loader import SpectrogramParser
    from ds2amd.decoder import BeamCTCDecoder, GreedyDecoder
    dev = torch.device("cuda", 0)
    torch.manual_seed(123456)
    m = dsm.DeepSpeech(rnn_type='gru', labels=bench.LABELS, rnn_hidden_size=800, nb_layers=5,
                       audio_conf=bench.CONF, bidirectional=True).to(dev).eval()
    parser = SpectrogramParser(bench.CONF, normalize='max_frame', device=dev)
    n_fft, hop, win, taps = parser._consts(16000)
    n_samp = int(args.seconds * 16000)
    g = torch.Generator().manual_seed(5)
    pcm = torch.rand(args.batch, n_samp, generator=g).mul_(2).sub_(1).to(dev)
    ns = torch.full((args.batch,), n_samp, dtype=torch.int32, device=dev)
    frames = 1 + n_samp // hop
    beam = BeamCTCDecoder(bench.LABELS, beam_width=args.beam, cutoff_top_n=40)
    beam_lm = BeamCTCDecoder(bench.LABELS, lm_path=args.lm, alpha=0.8, beta=1.0,
                             beam_width=args.beam, cutoff_top_n=40)
    greedy = GreedyDecoder(bench.LABELS)

    def run(decoder):
        with torch.no_grad():
            spect = ops.stft_logmag(pcm, ns, n_fft, hop, win, 1, taps, frames).unsqueeze(1)
            _, probs, out_lens = m(spect, torch.full((args.batch,), frames, dtype=torch.int32))
            return decoder.decode(probs, out_lens)

    out = {"config": f"cfg5: batched inference, DS2 5xBiGRU-800, {args.batch} x {args.seconds:g} s "
                     f"PCM -> STFT -> forward -> decode, fp32", "batch": args.batch}
    for name, dec in (("beam", beam), ("beam_lm", beam_lm), ("greedy", greedy)):
        run(dec)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            strings, _ = run(dec)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.iters
        out[f"{name}_audio_seconds_per_sec"] = round(args.batch * args.seconds / dt, 1)
        out[f"{name}_ms_per_batch"] = round(dt * 1e3, 2)
        out[f"{name}_sample"] = strings[0][0][:40]
    out["beam_width"] = args.beam
    # the decoders alone on one forward's output: device part (kernel + allocations, synced)
    # and the whole decode (+ the copy back and the strings / offsets on the host)
    with torch.no_grad():
        spect = ops.stft_logmag(pcm, ns, n_fft, hop, win, 1, taps, frames).unsqueeze(1)
        _, probs, out_lens = m(spect, torch.full((args.batch,), frames, dtype=torch.int32))
    parts = {}
    for name, fn in (("beam_device", lambda: beam.decode_raw(probs, out_lens)),
                     ("beam_full", lambda: beam.decode(probs, out_lens)),
                     ("greedy_device", lambda: greedy.decode_ids(probs, out_lens)),
                     ("greedy_full", lambda: greedy.decode(probs, out_lens))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize()
        parts[name] = round((time.perf_counter() - t0) / args.iters * 1e3, 2)
    out["decode_ms"] = parts
    print(json.dumps(out), flush=True)
    if args.stamps:
        from ds2amd import _lib
        for name, dec in (("beam", beam), ("beam_lm", beam_lm)):
            buf = torch.zeros(256 * 9, dtype=torch.int64, device=dev)
            _lib.call("ds2_test_beam_stamps", buf.data_ptr())
            run(dec)
            torch.cuda.synchronize()
            _lib.call("ds2_test_beam_stamps", None)
            st = buf.view(256, 9).cpu().double()
            fr = st[1:255]
            nxt = st[2:256]
            ticks = (nxt[:, 0] - fr[:, 0]).mean().item()
            us = ((nxt[:, 8] - fr[:, 8]).mean() / 100.0).item()   # s_memrealtime: 100 MHz
            names = ["stage+lp+prune", "bookkeeping", "scoring", "revival", "selection",
                     "new beam", "deaths", "tail"]
            ph = [(fr[:, i + 1] - fr[:, i]).mean().item() for i in range(7)]
            ph.append((nxt[:, 0] - fr[:, 7]).mean().item())
            print(json.dumps({"decoder": name, "us_per_frame": round(us, 3),
                              "clock_mhz": round(ticks / us, 1) if us > 0 else None,
                              "phase_us": {nm: round(v / ticks * us, 3) for nm, v in zip(names, ph)}}),
                  flush=True)


if __name__ == "__main__":
    main()
