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


def build(seed: int = 7, order: int = 3, top: int = 40):
    """A back-off model of `order` (1..6): `top` random top-order n-grams, every prefix and
    suffix of each added (lower orders padded with random extra n-grams), backoffs on every
    n-gram that is the context of a longer one.  build() = the committed tiny_lm.arpa."""
    g = np.random.default_rng(seed)
    vocab = ["<s>", "</s>", "<unk>"] + WORDS
    grams = {n: set() for n in range(1, order + 1)}
    if order > 1:
        while len(grams[order]) < top:
            a = ["<s>"] + WORDS
            ng = [a[g.integers(len(a))]] + [WORDS[g.integers(len(WORDS))] for _ in range(order - 2)]
            ng.append(WORDS[g.integers(len(WORDS))] if g.random() < 0.9 else "</s>")
            grams[order].add(tuple(ng))
        for n in range(order - 1, 1, -1):
            for t in grams[n + 1]:
                grams[n].add(t[:-1])
                grams[n].add(t[1:])
        while len(grams[2]) < 90 and order == 3:
            a = ["<s>"] + WORDS
            grams[2].add((a[g.integers(len(a))], (WORDS + ["</s>"])[g.integers(len(WORDS) + 1)]))
    grams[1] = {(w,) for w in vocab}
    ctx = {n: {t[:-1] for t in grams[n + 1]} if n < order else set() for n in range(1, order + 1)}

    def p10(lo, hi):
        return float(np.round(g.uniform(lo, hi), 4))

    lines = ["", "\\data\\"] + [f"ngram {n}={len(grams[n])}" for n in range(1, order + 1)]
    for n in range(1, order + 1):
        lines += ["", f"\\{n}-grams:"]
        items = [(w,) for w in vocab] if n == 1 else sorted(grams[n])
        for t in items:
            if n == 1:
                prob = -99.0 if t[0] == "<s>" else p10(-3.2, -0.8)
            else:
                prob = p10(-2.0, -0.2) if n == 2 else p10(-1.5, -0.1)
            if t in ctx[n]:
                bo = p10(-1.2, -0.05) if n == 1 else p10(-0.9, -0.02)
                lines.append(f"{prob:.4f}\t{' '.join(t)}\t{bo:.4f}")
            else:
                lines.append(f"{prob:.4f}\t{' '.join(t)}")
    lines += ["", "\\end\\", ""]
    return "\n".join(lines)


if __name__ == "__main__":
    path = os.path.join(HERE, "tiny_lm.arpa")
    with open(path, "w", encoding="utf-8") as f:
        f.write(build())
    print("wrote", path)
