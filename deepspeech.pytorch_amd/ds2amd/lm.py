"""Word n-gram language model for the device beam search (BeamCTCDecoder's lm_path).

The reference hands lm_path / alpha / beta to ctcdecode's KenLM-backed Scorer
(decoder.py:90-99, opts.py:6-10).  Here an ARPA file (KenLM's text input format; KenLM's
own binary format is not read) is turned into three device tables that the beam-search
kernel (ds2_ctc_beam_decode_lm, csrc/ctc.hip) queries directly:

  * ``table``  int32 [cap, 8]: an open-addressing hash table of every n-gram, one 32-byte
    record per slot {w0..w5 (word ids, -1 padded), log10 prob bits, log10 backoff bits};
    FNV-1a over the six ids, a final avalanche, linear probing, load <= 1/4, an empty
    slot has w0 = -1;
  * ``dict_next`` int32 [S, C] / ``dict_mask`` uint32 [S, 2] / ``dict_word`` int32 [S]:
    the vocabulary trie over label ids (ctcdecode's dictionary FST: every LM word whose
    characters are all labels, followed by the space label).  State 0 is the start,
    state S-1 the post-space state (no arcs); dict_word = the word id a state spells.

Word ids are the order of the \\1-grams section.  Character-based LMs (every word one
character: ctcdecode then scores every extension and uses no trie) are rejected.
"""
from __future__ import annotations

import re
from typing import List, Sequence

import numpy as np
import torch

MAX_ORDER = 6          # KenLM's default maximum order
SPECIAL = ("<s>", "</s>", "<unk>")


def _hash(keys: np.ndarray) -> np.ndarray:
    """FNV-1a over the six int32 ids of each row + avalanche; the kernel's lm_hash."""
    h = np.full(keys.shape[0], 2166136261, dtype=np.uint64)
    for k in range(MAX_ORDER):
        h = ((h ^ keys[:, k].astype(np.uint32).astype(np.uint64)) * 16777619) & 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    return h


def read_arpa(path: str):
    """-> (vocab list, order, keys int32 [M, 6], prob f32 [M], backoff f32 [M])."""
    vocab: List[str] = []
    wid = {}
    rows, probs, bos = [], [], []
    section = None
    counts = {}
    with open(path, encoding="utf-8") as f:
        for raw in f:
            line = raw.strip()
            if not line:
                continue
            if line == "\\data\\":
                section = "data"
                continue
            if line == "\\end\\":
                break
            m = re.match(r"^\\(\d+)-grams:$", line)
            if m:
                section = int(m.group(1))
                if section > MAX_ORDER:
                    raise ValueError(f"{path}: order {section} > {MAX_ORDER}")
                continue
            if section == "data":
                if line.startswith("ngram "):
                    k, v = line[6:].split("=")
                    counts[int(k)] = int(v)
                continue
            if not isinstance(section, int):
                raise ValueError(f"{path}: not an ARPA file (KenLM binary models are not read)")
            parts = line.split()
            n = section
            words = parts[1:1 + n]
            if n == 1:
                wid[words[0]] = len(vocab)
                vocab.append(words[0])
            try:
                ids = [wid[w] for w in words]
            except KeyError as e:
                raise ValueError(f"{path}: n-gram word {e} missing from the unigrams") from None
            rows.append(ids + [-1] * (MAX_ORDER - n))
            probs.append(float(parts[0]))
            bos.append(float(parts[1 + n]) if len(parts) > 1 + n else 0.0)
    if not counts or not rows:
        raise ValueError(f"{path}: not an ARPA file (KenLM binary models are not read)")
    return (vocab, max(counts), np.asarray(rows, np.int32), np.asarray(probs, np.float32),
            np.asarray(bos, np.float32))


def build_table(keys: np.ndarray, prob: np.ndarray, bo: np.ndarray) -> np.ndarray:
    """Open-addressing table int32 [cap, 8] (cap a power of two >= 4 M)."""
    m = keys.shape[0]
    cap = 1
    while cap < 4 * m:
        cap *= 2
    mask = cap - 1
    slot = (_hash(keys) & mask).astype(np.int64)
    owner = np.full(cap, -1, np.int64)
    pending = np.arange(m)
    while pending.size:
        s = slot[pending]
        free = owner[s] < 0
        cand, cs = pending[free], s[free]
        us, first = np.unique(cs, return_index=True)
        owner[us] = cand[first]
        won = np.zeros(m, bool)
        won[cand[first]] = True
        pending = pending[~won[pending]]
        slot[pending] = (slot[pending] + 1) & mask
    tab = np.full((cap, 8), -1, np.int32)
    used = owner >= 0
    o = owner[used]
    tab[used, :MAX_ORDER] = keys[o]
    tab[used, 6] = prob[o].view(np.int32)
    tab[used, 7] = bo[o].view(np.int32)
    return tab


def build_dictionary(vocab: Sequence[str], labels: Sequence[str], space: int):
    """Vocabulary trie -> (dict_next [S, C], dict_mask [S, 2] uint32, dict_word [S])."""
    cmap = {ch: i for i, ch in enumerate(labels)}
    nxt: List[dict] = [dict()]
    word: List[int] = [-1]
    for w_id, w in enumerate(vocab):
        ids = [cmap.get(ch) for ch in w]
        if not ids or any(i is None for i in ids):
            continue
        s = 0
        for c in ids:
            if c not in nxt[s]:
                nxt.append(dict())
                word.append(-1)
                nxt[s][c] = len(nxt) - 1
            s = nxt[s][c]
        word[s] = w_id
    f_state = len(nxt)
    nxt.append(dict())
    word.append(-1)
    c_n = len(labels)
    table = np.full((f_state + 1, c_n), -1, np.int32)
    for s, arcs in enumerate(nxt):
        for c, d in arcs.items():
            table[s, c] = d
        if word[s] >= 0:
            table[s, space] = f_state
    bits = (table >= 0).astype(np.uint64) << np.arange(c_n, dtype=np.uint64)
    m64 = np.bitwise_or.reduce(bits, axis=1) if c_n else np.zeros(len(table), np.uint64)
    mask = np.stack([(m64 & 0xFFFFFFFF).astype(np.uint32), (m64 >> 32).astype(np.uint32)], 1)
    return table, mask, np.asarray(word, np.int32)


class ArpaScorer:
    """Device tables of an ARPA model for the beam search (ctcdecode's Scorer)."""

    def __init__(self, lm_path: str, labels: Sequence[str], alpha: float, beta: float,
                 device="cuda"):
        labels = list(labels)
        if " " not in labels:
            raise ValueError("ds2amd LM beam search: the labels need a space label")
        if len(labels) > 64:
            raise ValueError("ds2amd LM beam search: at most 64 labels")
        vocab, order, keys, prob, bo = read_arpa(lm_path)
        if all(len(w) == 1 for w in vocab if w not in SPECIAL):
            raise NotImplementedError("ds2amd LM beam search: character-based LMs (every word one "
                                      "character) are not supported")
        if "<s>" not in vocab:
            raise ValueError(f"{lm_path}: the ARPA model has no <s> (KenLM refuses it too)")
        self.order = int(order)
        self.start_id = vocab.index("<s>")
        self.space = labels.index(" ")
        self.alpha = float(alpha)
        self.beta = float(beta)
        self.vocab = vocab
        dnext, dmask, dword = build_dictionary(vocab, labels, self.space)
        tab = build_table(keys, prob, bo)
        dev = torch.device(device)
        self.table = torch.from_numpy(tab).to(dev)
        self.table_mask = tab.shape[0] - 1
        self.dict_next = torch.from_numpy(dnext).to(dev)
        self.dict_mask = torch.from_numpy(dmask.view(np.int32)).to(dev)
        self.dict_word = torch.from_numpy(dword).to(dev)
        self.n_states = int(dnext.shape[0])
