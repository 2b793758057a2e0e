"""CPU restatement of CTC prefix beam search WITH a word n-gram language model.

TEST INFRASTRUCTURE ONLY (the checker for ds2_ctc_beam_decode_lm); never imported by the
product path.

Reference: decoder.py:90-99 `BeamCTCDecoder(labels, lm_path, alpha, beta, ...)` hands
lm_path / alpha / beta (opts.py:6-10: --lm-path, --alpha 0.8, --beta 1) to
`ctcdecode.CTCBeamDecoder`, whose Scorer wraps a KenLM model.  Both are un-vendored,
unpinned third-party code absent from this container, so **parity
with ctcdecode/KenLM is unpinned**.  This file restates their published algorithms on
top of oracle/ctc_beam.py's no-LM restatement (same candidate form, same tie rules):

  KenLM (lm/model.cc BaseScore over an ARPA file; `get_log_cond_prob` of ctcdecode's
  scorer.cpp walks the n-gram from NullContext and keeps the last word's score):
    * log10 p(w | h) = prob(longest suffix s of h with (s, w) in the model)
                       + backoff of every longer context suffix of h in the model,
      summed in float32 from the shorter context to the longer (KenLM's state keeps the
      backoffs of the matched context suffixes; a context absent from the model adds 0);
    * any OOV word in the n-gram -> OOV_SCORE = -1000 (natural-log units already);
      otherwise the log10 value / NUM_FLT_LOGE (the float 0.4342944819) -> natural log.
  ctcdecode (scorer.cpp make_ngram / fill_dictionary, path_trie.cpp get_path_trie,
  ctc_beam_search_decoder.cpp), word-based LM:
    * make_ngram(prefix): the last `order` words of the prefix, padded in front with
      "<s>" when it has fewer;
    * extending a prefix by the space label scores the word the space completes:
      log_p += float(alpha * lnp(ngram(prefix))); log_p = float(double(log_p) + beta);
    * a vocabulary trie ("dictionary FST": every LM word whose characters are all labels,
      followed by the space) constrains extensions: a new child is created only along a
      trie arc; the state after a space (final, no arcs) resets to the start state on
      the first extension attempted from it -- and that attempt itself is rejected
      (get_path_trie's `is_final && reset` branch);
    * with a scorer the beam is sorted first and, once full, a (prefix, char) pair whose
      lp[c] + score < min_cutoff = worst score + log(p_blank) - max(0, beta) skips that
      char for this and every lower prefix (blank / repeat / extension alike);
    * after the last frame every non-empty prefix not ending in a space gets
      float(float(alpha * lnp(ngram)) + beta) added before the final ranking.
    * trie-node revival as in oracle/ctc_beam.py; a revived node keeps its dictionary
      state (a revived post-space node was necessarily reset: it has a child), and the
      found-child branch of get_path_trie skips the dictionary check.
  Not restated: character-based LMs (every vocabulary word one character); the returned score is the LM-inclusive one (ctcdecode returns an
  "approx_ctc" score the reference discards, decoder.py:136).

Pure Python loops: small inputs only.
"""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .ctc_beam import F32, NEG, STATS, alive_children, lse, pruned_log_probs

OOV_SCORE = -1000.0
NUM_FLT_LOGE = float(np.float32(0.4342944819))   # decoder_utils.h: a float constant
START = "<s>"


class ArpaLM:
    """An ARPA back-off model: n-grams -> (log10 prob, log10 backoff) as float32."""

    def __init__(self, path: str):
        self.ngrams: Dict[Tuple[str, ...], Tuple[np.float32, np.float32]] = {}
        self.vocab: List[str] = []
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
                    continue
                if section == "data":
                    if line.startswith("ngram "):
                        k, v = line[6:].split("=")
                        counts[int(k)] = int(v)
                    continue
                if isinstance(section, int):
                    parts = line.split()
                    n = section
                    words = tuple(parts[1:1 + n])
                    bo = F32(float(parts[1 + n])) if len(parts) > 1 + n else F32(0.0)
                    self.ngrams[words] = (F32(float(parts[0])), bo)
                    if n == 1:
                        self.vocab.append(words[0])
        self.order = max(counts)
        self.vocab_set = set(self.vocab)

    def cond_log10(self, words: Sequence[str]) -> Optional[np.float32]:
        """log10 p(words[-1] | words[:-1]); None when any word is out of vocabulary."""
        if any(w not in self.vocab_set for w in words):
            return None
        ctx, w = tuple(words[:-1]), words[-1]
        p, m = None, 0
        for m in range(min(len(words), self.order), 0, -1):
            key = (ctx[len(ctx) - (m - 1):] if m > 1 else ()) + (w,)
            if key in self.ngrams:
                p = self.ngrams[key][0]
                break
        if p is None:
            return None
        for ln in range(m, min(len(ctx), self.order - 1) + 1):
            c = ctx[len(ctx) - ln:]
            if c in self.ngrams:
                p = F32(p + self.ngrams[c][1])
        return p


class WordDict:
    """The vocabulary trie over label ids; state 0 = start, F = after a word's space."""

    def __init__(self, vocab: Sequence[str], labels: Sequence[str], space: int):
        cmap = {ch: i for i, ch in enumerate(labels)}
        self.next: List[Dict[int, int]] = [dict()]
        self.word: List[Optional[str]] = [None]
        for w in vocab:
            ids = [cmap.get(ch) for ch in w]
            if not ids or any(i is None for i in ids):
                continue
            s = 0
            for c in ids:
                if c not in self.next[s]:
                    self.next.append(dict())
                    self.word.append(None)
                    self.next[s][c] = len(self.next) - 1
                s = self.next[s][c]
            self.word[s] = w
        self.F = len(self.next)
        self.next.append(dict())
        self.word.append(None)
        for s in range(self.F):
            if self.word[s] is not None:
                self.next[s][space] = self.F


def lm_term(lm: ArpaLM, hist: Tuple[str, ...], word: Optional[str], alpha: float) -> np.float32:
    """float(alpha * ln p(word | hist)) -- ctcdecode's `score` before beta."""
    p = lm.cond_log10(hist + (word,)) if word is not None else None
    lnp = OOV_SCORE if p is None else float(p) / NUM_FLT_LOGE
    return F32(lnp * alpha)


def iteration_order(allowed: np.ndarray, probs_t: np.ndarray, prune: bool) -> List[int]:
    """get_pruned_log_probs' char order: sorted by prob (ties: lower id) when pruning."""
    c = probs_t.shape[0]
    if not prune:
        return list(range(c))
    order = sorted(range(c), key=lambda k: (-float(probs_t[k]), k))
    return [k for k in order if allowed[k]]


def beam_decode_lm_one(probs: np.ndarray, size: int, beam: int, lm: ArpaLM, labels: Sequence[str],
                       alpha: float, beta: float, blank: int = 0, cutoff_top_n: int = 40,
                       cutoff_prob: float = 1.0):
    """probs [T, C] float32.  Returns list of (score, ids, timesteps) best first."""
    c = probs.shape[1]
    space = list(labels).index(" ")
    wd = WordDict(lm.vocab, labels, space)
    n1 = lm.order - 1
    parent, ch, ts, lpc = [-1], [-1], [-1], [NEG]
    hist0 = (START,) * n1
    dst, hist, lms = [0], [hist0], [lm_term(lm, hist0, None, alpha)]
    bm: List[list] = [[0, -1, F32(0.0), NEG]]
    prune = cutoff_prob < 1.0 or cutoff_top_n < c
    for t in range(size):
        allowed, lp = pruned_log_probs(probs[t], cutoff_top_n, cutoff_prob)
        it_order = iteration_order(allowed, probs[t], prune)
        nb = len(bm)
        score = [lse(e[2], e[3]) for e in bm]
        full = nb == beam
        pbl = float(probs[t][blank])
        worst = float(min(score))
        min_cut = F32(worst + (math.log(pbl) if pbl > 0 else -math.inf) - max(0.0, beta))

        def att(i, cc):
            return not (full and F32(lp[cc] + score[i]) < min_cut)

        # the dictionary reset: the first attempted non-blank char from a post-space node
        cstar = {}
        for i in range(nb):
            if dst[bm[i][0]] == wd.F:
                for cc in it_order:
                    if cc != blank and att(i, cc):
                        cstar[i] = cc
                        break

        def eff_state(i, cc):
            s = dst[bm[i][0]]
            if s == wd.F:
                return None if cstar.get(i) == cc else 0
            return s

        def ext_val(i, cc):
            if cc == bm[i][1]:
                v = F32(lp[cc] + bm[i][2]) if bm[i][2] != NEG else NEG
            else:
                v = F32(lp[cc] + score[i])
            if cc == space:
                v = F32(v + lms[bm[i][0]])
                v = F32(float(v) + beta)
            return v

        node_to_idx = {e[0]: i for i, e in enumerate(bm)}
        pidx = [node_to_idx.get(parent[e[0]], -1) if e[0] != 0 else -1 for e in bm]
        child_of = {(pidx[q], bm[q][1]): q for q in range(nb) if pidx[q] >= 0}
        alive = alive_children(bm, parent, ch)
        cands = []
        ts_upd = {}
        for i in range(nb):
            for cc in range(c):
                k = i * c + cc
                if cc == blank:
                    last = bm[i][1]
                    pb = F32(lp[blank] + score[i]) if (allowed[blank] and att(i, blank)) else NEG
                    pnb = (F32(lp[last] + bm[i][3])
                           if (last >= 0 and allowed[last] and att(i, last)) else NEG)
                    j = pidx[i]
                    if j >= 0 and allowed[last] and att(j, last):
                        pnb = lse(pnb, ext_val(j, last))
                        if lp[last] > lpc[bm[i][0]]:
                            ts_upd[bm[i][0]] = (t, lp[last])
                    s = lse(pb, pnb)
                    if s != NEG:
                        cands.append((s, last, k, 'stay', i, pb, pnb))
                else:
                    if not allowed[cc] or (i, cc) in child_of or not att(i, cc):
                        continue
                    x = alive.get((bm[i][0], cc))      # a pruned node still in the trie
                    if x is not None:
                        if lp[cc] > lpc[x]:
                            ts_upd[x] = (t, lp[cc])
                    else:
                        st = eff_state(i, cc)
                        if st is None or cc not in wd.next[st]:
                            continue
                    e = ext_val(i, cc)
                    if e != NEG:
                        cands.append((e, cc, k, 'ext', i, NEG, e))
        for node, (tt, v) in ts_upd.items():
            ts[node] = tt
            lpc[node] = v
        cands.sort(key=lambda x: (-float(x[0]), x[1], x[2]))
        new = []
        for s, last, k, kind, i, pb, pnb in cands[:beam]:
            nd_i = bm[i][0]
            if kind == 'stay':
                new.append([nd_i, last, pb, pnb])
                continue
            if (nd_i, last) in alive:                  # revived: keeps its LM state
                x = alive[(nd_i, last)]
                assert ch[x] != space or dst[x] == 0
                STATS["revived"] += 1
                new.append([x, last, pb, pnb])
                continue
            st = eff_state(i, last)
            ns = wd.next[st][last]
            if last == space:
                nh = (hist[nd_i] + (wd.word[st],))[-n1:] if n1 > 0 else ()
                nl = F32(0.0)
            else:
                nh = hist[nd_i]
                nl = lm_term(lm, nh, wd.word[ns], alpha)
            parent.append(nd_i)
            ch.append(last)
            ts.append(t)
            lpc.append(lp[last])
            dst.append(ns)
            hist.append(nh)
            lms.append(nl)
            new.append([len(parent) - 1, last, pb, pnb])
        for i in cstar:                 # the reset sticks to the node
            dst[bm[i][0]] = 0
        bm = new
        if not bm:
            break
    final = []
    for idx, e in enumerate(bm):
        s = lse(e[2], e[3])
        nd = e[0]
        if nd != 0 and ch[nd] != space:
            s = F32(s + F32(float(lms[nd]) + beta))
        final.append((s, e[1], idx, nd))
    final.sort(key=lambda x: (-float(x[0]), x[1], x[2]))
    out = []
    for s, _, _, node in final:
        ids, steps = [], []
        while node > 0:
            ids.append(ch[node])
            steps.append(ts[node])
            node = parent[node]
        out.append((float(s), ids[::-1], steps[::-1]))
    return out


def beam_decode_lm(probs, sizes: Sequence[int], beam: int, lm: ArpaLM, labels: Sequence[str],
                   alpha: float, beta: float, blank: int = 0, cutoff_top_n: int = 40,
                   cutoff_prob: float = 1.0):
    """Batched: probs [N, T, C] -> per utterance the list of beam_decode_lm_one results."""
    p = np.asarray(probs, dtype=np.float32)
    return [beam_decode_lm_one(p[i], int(sizes[i]), beam, lm, labels, alpha, beta, blank,
                               cutoff_top_n, cutoff_prob) for i in range(p.shape[0])]
