"""Write tests/golden/tiny_lm.arpa: a small, well-formed 3-gram ARPA back-off model.

Run:  python tests/golden/make_lm_fixture.py

Not made from the reference (it ships no LM; KenLM / ctcdecode are absent): a synthetic
model over a 24-word vocabulary with seeded log10 probabilities and back-off weights,
closed under prefixes and suffixes like every lmplz / SRILM output (an n-gram's context
and its lower-order suffix are always present).  It exercises the scorer's back-off
chain (trigram hits, bigram hits with one back-off, unigram hits with two), the
dictionary trie (words that share prefixes, a word with an apostrophe, a word with a
character outside the labels, which must never be spelled), and <s> padding.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

WORDS = ["A", "AN", "AND", "ANT", "THE", "THEY", "THEN", "CAT", "CATS", "CAR", "DOG", "DON'T",
         "I", "IT", "IS", "IN", "ON", "NO", "NOT", "TO", "TOO", "SAT", "HAT", "café"]


def build(seed: int = 7):
    g = np.random.default_rng(seed)
    vocab = ["<s>", "</s>", "<unk>"] + WORDS
    tri = set()
    while len(tri) < 40:
        a = ["<s>"] + WORDS
        w1 = a[g.integers(len(a))]
        w2 = WORDS[g.integers(len(WORDS))]
        w3 = WORDS[g.integers(len(WORDS))] if g.random() < 0.9 else "</s>"
        tri.add((w1, w2, w3))
    bi = set()
    for t in tri:
        bi.add(t[:2])
        bi.add(t[1:])
    while len(bi) < 90:
        a = ["<s>"] + WORDS
        bi.add((a[g.integers(len(a))], (WORDS + ["</s>"])[g.integers(len(WORDS) + 1)]))
    uni = [(w,) for w in vocab]
    ctx_bi = {t[:2] for t in tri}
    ctx_uni = {b[:1] for b in bi}

    def p10(lo, hi):
        return float(np.round(g.uniform(lo, hi), 4))

    lines = ["", "\\data\\", f"ngram 1={len(uni)}", f"ngram 2={len(bi)}", f"ngram 3={len(tri)}",
             "", "\\1-grams:"]
    for (w,) in uni:
        prob = -99.0 if w == "<s>" else p10(-3.2, -0.8)
        if (w,) in ctx_uni:
            lines.append(f"{prob:.4f}\t{w}\t{p10(-1.2, -0.05):.4f}")
        else:
            lines.append(f"{prob:.4f}\t{w}")
    lines += ["", "\\2-grams:"]
    for b in sorted(bi):
        if b in ctx_bi:
            lines.append(f"{p10(-2.0, -0.2):.4f}\t{' '.join(b)}\t{p10(-0.9, -0.02):.4f}")
        else:
            lines.append(f"{p10(-2.0, -0.2):.4f}\t{' '.join(b)}")
    lines += ["", "\\3-grams:"]
    for t in sorted(tri):
        lines.append(f"{p10(-1.5, -0.1):.4f}\t{' '.join(t)}")
    lines += ["", "\\end\\", ""]
    return "\n".join(lines)


if __name__ == "__main__":
    path = os.path.join(HERE, "tiny_lm.arpa")
    with open(path, "w", encoding="utf-8") as f:
        f.write(build())
    print("wrote", path)
