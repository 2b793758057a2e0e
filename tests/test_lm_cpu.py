"""CPU tests of the LM beam-search pieces: the KenLM back-off restatement on hand-made
ARPA models (known answers), the device tables ds2amd/lm.py builds (hash table and
vocabulary trie, queried here exactly as the kernel queries them) against the oracle,
and the oracle's LM beam search on spelled inputs."""
import os

import numpy as np
import pytest

from oracle import ctc_beam_lm as obl
from oracle.ds2_oracle import LABELS

HERE = os.path.dirname(os.path.abspath(__file__))
TINY_LM = os.path.join(HERE, "golden", "tiny_lm.arpa")

HAND_ARPA = """
\\data\\
ngram 1=5
ngram 2=2
ngram 3=1

\\1-grams:
-99\t<s>\t-0.5
-1.0\tA\t-0.3
-1.2\tB\t-0.2
-1.5\t</s>
-2.0\t<unk>

\\2-grams:
-0.4\t<s> A\t-0.1
-0.3\tA B\t-0.05

\\3-grams:
-0.2\t<s> A B

\\end\\
"""


@pytest.fixture()
def hand_lm(tmp_path):
    p = tmp_path / "hand.arpa"
    p.write_text(HAND_ARPA)
    return str(p)


def test_arpa_backoff_known_answers(hand_lm):
    """KenLM BaseScore semantics (ARPA back-off), by hand:
    p(B | <s> A) = trigram -0.2; p(A | A B) = p(A) + bo(B) + bo(A B) = -1.0 - 0.2 - 0.05;
    p(B | B A) = p(B | A) = -0.3 (the context 'B A' is not in the model: no backoff);
    p(A | <s> <s>) = p(A | <s>) = -0.4; an OOV word anywhere -> None (OOV_SCORE)."""
    lm = obl.ArpaLM(hand_lm)
    assert lm.order == 3
    f = np.float32
    assert lm.cond_log10(("<s>", "A", "B")) == f(-0.2)
    assert lm.cond_log10(("A", "B", "A")) == f(f(f(-1.0) + f(-0.2)) + f(-0.05))
    assert lm.cond_log10(("B", "A", "B")) == f(-0.3)
    assert lm.cond_log10(("<s>", "<s>", "A")) == f(-0.4)
    assert lm.cond_log10(("<s>", "<s>", "B")) == f(f(-1.2) + f(-0.5))
    assert lm.cond_log10(("<s>", "C", "A")) is None
    t = obl.lm_term(lm, ("<s>", "A"), "B", 0.8)
    assert t == np.float32(-0.2 / float(np.float32(0.4342944819)) * 0.8)
    assert obl.lm_term(lm, ("<s>", "A"), None, 0.8) == np.float32(-800.0)


def _table_lookup(tab, key):
    """The kernel's lm_find: FNV-1a + avalanche, linear probing, w0 = -1 empty."""
    from ds2amd.lm import _hash
    mask = tab.shape[0] - 1
    s = int(_hash(np.asarray([key], np.int32))[0]) & mask
    while True:
        row = tab[s]
        if row[0] == -1:
            return None
        if list(row[:6]) == list(key):
            return row[6:8].view(np.float32)
        s = (s + 1) & mask


def _device_cond(tab, order, hist, w):
    """The kernel's lm_term before the ln / alpha scaling (log10, float32)."""
    n1 = order - 1
    for m in range(order, 0, -1):
        key = [hist[n1 - (m - 1) + i] if i < m - 1 else (w if i == m - 1 else -1) for i in range(6)]
        r = _table_lookup(tab, key)
        if r is not None:
            p = np.float32(r[0])
            break
    else:
        return None
    for ln in range(m, n1 + 1):
        key = [hist[n1 - ln + i] if i < ln else -1 for i in range(6)]
        r = _table_lookup(tab, key)
        if r is not None:
            p = np.float32(p + np.float32(r[1]))
    return p


@pytest.mark.parametrize("which", ["hand", "tiny"])
def test_device_tables_match_oracle(which, hand_lm):
    """ds2amd/lm.py's hash table, queried the kernel's way, gives the oracle's KenLM
    score for every (two-word history, word) over the vocabulary."""
    from ds2amd import lm as dlm
    path = hand_lm if which == "hand" else TINY_LM
    vocab, order, keys, prob, bo = dlm.read_arpa(path)
    tab = dlm.build_table(keys, prob, bo)
    assert tab.shape[0] >= 4 * keys.shape[0] and (tab[:, 0] >= 0).sum() == keys.shape[0]
    olm = obl.ArpaLM(path)
    assert olm.vocab == vocab and olm.order == order == 3
    ctx = ["<s>"] + [w for w in vocab if w not in ("<s>", "</s>", "<unk>")]
    n = 0
    for a in ctx:
        for b in ctx:
            for w in vocab:
                if w == "<s>":
                    continue
                ref = olm.cond_log10((a, b, w))
                got = _device_cond(tab, order, [vocab.index(a), vocab.index(b)], vocab.index(w))
                assert ref == got, (a, b, w, ref, got)
                n += 1
    assert n >= 36


def test_dictionary_tables():
    """The vocabulary trie: words spelled over the labels only, the space arc after
    every complete word, nothing after the space; the mask mirrors the arcs."""
    from ds2amd import lm as dlm
    vocab, *_ = dlm.read_arpa(TINY_LM)
    space = LABELS.index(" ")
    nxt, mask, word = dlm.build_dictionary(vocab, LABELS, space)
    wd = obl.WordDict(vocab, LABELS, space)
    assert nxt.shape == (len(wd.next), len(LABELS))
    m64 = mask[:, 0].astype(np.uint64) | (mask[:, 1].astype(np.uint64) << np.uint64(32))

    def spell(w):
        s = 0
        for ch in w:
            s = int(nxt[s, LABELS.index(ch)])
            if s < 0:
                return None
        return s

    for w in vocab:
        s = spell(w) if all(ch in LABELS for ch in w) else None
        if w in ("<s>", "</s>", "<unk>", "café"):
            assert s is None
            continue
        assert word[s] == vocab.index(w)
        f = nxt[s, space]
        assert f == nxt.shape[0] - 1 and (nxt[f] < 0).all()
    assert int(nxt[0, space]) < 0 and spell("CA") is not None and word[spell("CA")] == -1
    for s in range(nxt.shape[0]):
        bits = sum(1 << c for c in range(len(LABELS)) if nxt[s, c] >= 0)
        assert int(m64[s]) == bits


def spelled_probs(text, g, noise=1.0, peak=5.0, blank_bias=1.0):
    """[T, C] probs that spell `text` (one frame per char, blanks between repeats and
    around words) plus Gaussian logit noise."""
    frames = []
    prev = None
    for ch in text:
        if ch == prev:
            frames.append(0)
        frames.append(LABELS.index(ch))
        frames.append(0)
        prev = ch
    t = len(frames)
    logits = g.standard_normal((t, len(LABELS))).astype(np.float32) * noise
    logits[:, 0] += blank_bias
    logits[np.arange(t), frames] += peak
    p = np.exp(logits - logits.max(-1, keepdims=True))
    return (p / p.sum(-1, keepdims=True)).astype(np.float32)


def test_lm_beam_oracle_spelled_sentence():
    """With clean spelled inputs the LM search returns the sentence; with a misspelled
    word the dictionary keeps every returned prefix inside the vocabulary."""
    lm = obl.ArpaLM(TINY_LM)
    g = np.random.default_rng(3)
    p = spelled_probs("THE CAT SAT ", g, noise=0.5)
    res = obl.beam_decode_lm_one(p, p.shape[0], 8, lm, LABELS, alpha=0.8, beta=1.0)
    assert "".join(LABELS[i] for i in res[0][1]) == "THE CAT SAT "
    p = spelled_probs("THE CQT ", g, noise=0.5)
    res = obl.beam_decode_lm_one(p, p.shape[0], 8, lm, LABELS, alpha=0.8, beta=1.0)
    words = set(w for w in lm.vocab)
    for _, ids, _ in res:
        s = "".join(LABELS[i] for i in ids)
        for w in s.split(" ")[:-1]:
            assert w in words, s


@pytest.mark.parametrize("order", [1, 2, 4, 5, 6])
def test_device_tables_match_oracle_any_order(order, tmp_path):
    """The hash table queried the kernel's way equals the oracle's KenLM score for models of
    every order the kernel accepts (histories <s>-padded to order - 1 words)."""
    import importlib.util
    from ds2amd import lm as dlm
    spec = importlib.util.spec_from_file_location(
        "make_lm_fixture", os.path.join(HERE, "golden", "make_lm_fixture.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    path = str(tmp_path / "m.arpa")
    with open(path, "w", encoding="utf-8") as f:
        f.write(mk.build(seed=order, order=order, top=60))
    vocab, o, keys, prob, bo = dlm.read_arpa(path)
    assert o == order
    tab = dlm.build_table(keys, prob, bo)
    olm = obl.ArpaLM(path)
    g = np.random.default_rng(order)
    words = [w for w in vocab if w not in ("<s>", "</s>", "<unk>")]
    ngrams = [k for k in olm.ngrams if len(k) == order]
    for trial in range(400):
        if trial < len(ngrams) and order > 1:     # every top-order n-gram, then random ones
            ng = list(ngrams[trial])
        else:
            ng = (["<s>"] * g.integers(0, order)) + [words[g.integers(len(words))] for _ in range(order)]
            ng = ng[-order:]
        hist, w = ng[:-1], ng[-1]
        if w == "<s>":
            continue
        ref = olm.cond_log10(tuple(ng))
        got = _device_cond(tab, order, [vocab.index(x) for x in hist], vocab.index(w))
        assert ref == got, (ng, ref, got)


def test_scorer_rejects_char_lms_and_binary_files(tmp_path):
    """Character-based LMs (ctcdecode's other scorer mode) and non-ARPA files raise."""
    from ds2amd.lm import ArpaScorer
    p = tmp_path / "char.arpa"
    p.write_text("\\data\\\nngram 1=5\n\n\\1-grams:\n-99\t<s>\n-1\t</s>\n-1\t<unk>\n"
                 "-0.5\tA\n-0.6\tB\n\n\\end\\\n")
    with pytest.raises(NotImplementedError):
        ArpaScorer(str(p), LABELS, 0.8, 1.0, device="cpu")
    b = tmp_path / "lm.binary"
    b.write_bytes(b"mmap lm http://kheafield.com/code format version 5\n\0\0\0")
    with pytest.raises(ValueError):
        ArpaScorer(str(b), LABELS, 0.8, 1.0, device="cpu")


def _spelled_cpu(text, g, noise, peak=5.0, blank_bias=1.0):
    frames, prev = [], None
    for ch in text:
        if ch == prev:
            frames.append(0)
        frames += [LABELS.index(ch), 0]
        prev = ch
    logits = g.standard_normal((len(frames), len(LABELS))).astype(np.float32) * noise
    logits[:, 0] += blank_bias
    logits[np.arange(len(frames)), frames] += peak
    p = np.exp(logits - logits.max(-1, keepdims=True))
    return (p / p.sum(-1, keepdims=True)).astype(np.float32)


def test_beam_trie_revival_keeps_prefixes_unique():
    """ctcdecode's PathTrie revives a pruned prefix that a kept descendant holds in the
    trie (path_trie.cpp get_path_trie / remove) instead of creating a second node for it,
    so every prefix is one node and a beam never holds the same string twice.  The noisy
    spelled sentences at beam 100 revive prefixes in both searches; every returned beam
    must hold distinct strings."""
    from oracle import ctc_beam
    g = np.random.default_rng(11)
    ps = [_spelled_cpu(s, g, 2.0) for s in ["THE CAT SAT ON A HAT", "I DON'T NO THEN "]]
    lm = obl.ArpaLM(os.path.join(HERE, "golden", "tiny_lm.arpa"))
    for use_lm in (False, True):
        ctc_beam.STATS["revived"] = 0
        for p in ps:
            out = (obl.beam_decode_lm_one(p, p.shape[0], 100, lm, LABELS, 0.8, 1.0) if use_lm
                   else ctc_beam.beam_decode_one(p, p.shape[0], 100))
            strings = [tuple(ids) for _, ids, _ in out]
            assert len(set(strings)) == len(strings)
        assert ctc_beam.STATS["revived"] > 0, use_lm


def test_beam_decoder_convert_helpers():
    """BeamCTCDecoder.convert_to_strings / convert_tensor (ref decoder.py:101-126): ctcdecode's
    [batch][beam][T] ids / offsets cut at [batch][beam] lengths; a beam of length <= 0 gives
    '' and an empty int tensor.  Host-only: the constructor touches no device."""
    import torch
    from ds2amd.decoder import BeamCTCDecoder
    dec = BeamCTCDecoder(LABELS, beam_width=4)
    out = torch.tensor([[[2, 3, 4, 0], [5, 0, 0, 0]], [[1, 1, 7, 8], [9, 9, 9, 9]]])
    lens = torch.tensor([[3, 0], [4, 2]])
    want = [[''.join(LABELS[i] for i in (2, 3, 4)), ''],
            [''.join(LABELS[i] for i in (1, 1, 7, 8)), LABELS[9] * 2]]
    assert dec.convert_to_strings(out, lens) == want
    # nested lists and numpy arrays, as ctcdecode callers pass them, give the same strings
    assert dec.convert_to_strings(out.tolist(), lens.tolist()) == want
    assert dec.convert_to_strings(out.numpy(), lens.numpy()) == want
    offs = torch.arange(16, dtype=torch.int32).reshape(2, 2, 4)
    got = dec.convert_tensor(offs, lens)
    assert got[0][0].tolist() == [0, 1, 2] and got[1][0].tolist() == [8, 9, 10, 11]
    assert got[1][1].tolist() == [12, 13]
    assert got[0][1].numel() == 0 and got[0][1].dtype == torch.int
