"""Debug: device LM beam search vs the oracle on the failing parity case, per (alpha, beta)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "deepspeech.pytorch_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from ds2amd import ops
from ds2amd.lm import ArpaScorer
from oracle import ctc_beam_lm as obl
from oracle import ds2_oracle as orc
from test_gpu_ops import _spelled

path = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "tiny_lm.arpa")
labels = orc.LABELS
lm = obl.ArpaLM(path)
dev = torch.device("cuda")
for beam, top_n, alpha, beta, noise in [(4, 40, 2.0, -0.5, 2.0), (4, 40, 0.8, 1.0, 2.0),
                                         (4, 40, 2.0, 0.5, 2.0), (8, 40, 2.0, -0.5, 2.0)]:
    g = np.random.default_rng(beam * 7 + top_n)
    p = _spelled("THE CAT SAT ", g, noise)[None]
    sizes = [p.shape[1]]
    sc = ArpaScorer(path, labels, alpha, beta, device=dev)
    ids, offs, lens, scores = ops.ctc_beam_decode_lm_raw(torch.from_numpy(p).to(dev),
                                                         torch.tensor(sizes, dtype=torch.int32).to(dev),
                                                         beam, beam, sc)
    ref = obl.beam_decode_lm(p, sizes, beam, lm, labels, alpha, beta)
    print("case", beam, alpha, beta)
    for q in range(beam):
        k = int(lens[0, q])
        d = ''.join(labels[i] for i in ids[0, q, :k].tolist())
        r = ''.join(labels[i] for i in ref[0][q][1]) if q < len(ref[0]) else None
        print(f"  {q}: dev {d!r} {float(scores[0, q]):.5f} | ref {r!r} {ref[0][q][0] if q < len(ref[0]) else None}")
    # per-frame: run prefixes of the utterance to find the first frame where they differ
    for t in range(1, sizes[0] + 1):
        ids, offs, lens, scores = ops.ctc_beam_decode_lm_raw(torch.from_numpy(p).to(dev),
                                                             torch.tensor([t], dtype=torch.int32).to(dev),
                                                             beam, beam, sc)
        ref = obl.beam_decode_lm(p, [t], beam, lm, labels, alpha, beta)
        dv = [(''.join(labels[i] for i in ids[0, q, :int(lens[0, q])].tolist()), round(float(scores[0, q]), 4)) for q in range(beam)]
        rv = [(''.join(labels[i] for i in r[1]), round(r[0], 4)) for r in ref[0]]
        if [x[0] for x in dv] != [x[0] for x in rv]:
            print("  first differing frame", t)
            print("   dev", dv)
            print("   ref", rv)
            break
