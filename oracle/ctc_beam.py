"""CPU restatement of CTC prefix beam search without a language model.

TEST INFRASTRUCTURE ONLY (the checker for ds2_ctc_beam_decode); never imported by the
product path.

Reference: decoder.py:90-143 `BeamCTCDecoder` wraps `ctcdecode.CTCBeamDecoder` (the
PaddlePaddle DeepSpeech decoder, ctc_beam_search_decoder.cpp) — an un-vendored,
unpinned third-party dependency that is absent here, so **parity with ctcdecode is
unpinned** (SURVEY §8c/§8f#1).  This file restates its published algorithm with the
LM scorer disabled (lm_path=None, the reference default) and pins the few choices
the library leaves to container iteration order:

  * vocabulary pruning per frame (get_pruned_log_probs): sort (char, prob) by prob
    descending (ties: lower index first), keep the first cutoff_top_n, and when
    cutoff_prob < 1 stop once the double cumulative prob reaches cutoff_prob;
    log prob = float(log(double(prob) + FLT_MIN)) (get_pruned_log_probs: the probs are
    doubles there, the log is taken in double and stored as float);
  * per frame, for every beam prefix i (score_i = lse(pb_i, pnb_i)):
      blank:            pb'  = lp[blank] + score_i
      repeat last char: pnb' = lp[last] + pnb_i
      extension by c:   child.pnb' += lp[c] + (pb_i if c == last else score_i)
                        (c == last with pb_i = -inf contributes nothing)
    where the child is an existing beam prefix if one is (its two pnb terms are
    combined with the symmetric float32 log_sum_exp, so the order is immaterial);
  * the beam keeps the beam_width best candidates by (score desc, last char asc,
    candidate index asc); candidates with score -inf are dropped;
  * a prefix's char timestep (the `offsets`) is the frame of its best-scoring
    extension event (ctcdecode's PathTrie log_prob_c rule);
  * trie-node revival (path_trie.cpp get_path_trie / remove): a prefix pruned from the
    beam stays in the trie while one of its descendants is still in the beam; an
    extension (i, c) that lands on such a node revives it instead of creating a new one,
    so the node keeps its identity (later extensions of it merge into the kept
    descendant) and its char frame, and every attempted extension onto it takes the
    log_prob_c rule above, whether or not it is selected.

Pure Python loops: small inputs only.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np

F32 = np.float32
NEG = F32(-np.inf)
FLT_MIN = F32(np.finfo(np.float32).tiny)
FLT_MIN_D = float(FLT_MIN)
STATS = {"revived": 0}      # revivals selected into a beam (tests check they are exercised)


def lse(a: np.float32, b: np.float32) -> np.float32:
    """log_sum_exp of ctc_beam_search_decoder (float), -inf aware, symmetric."""
    if a == NEG:
        return b
    if b == NEG:
        return a
    m = a if a > b else b
    return F32(np.log(F32(np.exp(F32(a - m)) + np.exp(F32(b - m)))) + m)


def alive_children(bm, parent, ch):
    """{(parent node, char): node} over the trie nodes still alive at the start of a frame:
    the beam's nodes and all their ancestors (PathTrie::remove deletes a pruned node only
    once it has no children left)."""
    alive = {}
    seen = set()
    for e in bm:
        nd = e[0]
        while nd > 0 and nd not in seen:
            seen.add(nd)
            alive[(parent[nd], ch[nd])] = nd
            nd = parent[nd]
    return alive


def pruned_log_probs(p: np.ndarray, cutoff_top_n: int, cutoff_prob: float):
    """(allowed mask, float32 log probs) for one frame."""
    c = p.shape[0]
    allowed = np.ones(c, bool)
    if cutoff_prob < 1.0 or cutoff_top_n < c:
        order = sorted(range(c), key=lambda k: (-float(p[k]), k))
        keep = []
        if cutoff_prob < 1.0:
            cum = 0.0
            for k in order:
                cum += float(p[k])
                keep.append(k)
                if cum >= cutoff_prob or len(keep) >= cutoff_top_n:
                    break
        else:
            keep = order[:cutoff_top_n]
        allowed[:] = False
        allowed[keep] = True
    lp = np.array([F32(math.log(float(x) + FLT_MIN_D)) for x in p.astype(np.float32)], np.float32)
    return allowed, lp


def beam_decode_one(probs: np.ndarray, size: int, beam: int, blank: int = 0,
                    cutoff_top_n: int = 40, cutoff_prob: float = 1.0):
    """probs [T, C] float32.  Returns list of (score, ids, timesteps) best first."""
    c = probs.shape[1]
    parent, ch, ts, lpc = [-1], [-1], [-1], [NEG]
    # beam entries: [node, last, pb, pnb]
    bm: List[list] = [[0, -1, F32(0.0), NEG]]
    for t in range(size):
        allowed, lp = pruned_log_probs(probs[t], cutoff_top_n, cutoff_prob)
        nb = len(bm)
        score = [lse(e[2], e[3]) for e in bm]
        node_to_idx = {e[0]: i for i, e in enumerate(bm)}
        pidx = [node_to_idx.get(parent[e[0]], -1) if e[0] != 0 else -1 for e in bm]
        child_of = {(pidx[q], bm[q][1]): q for q in range(nb) if pidx[q] >= 0}
        alive = alive_children(bm, parent, ch)

        def ext_val(i, cc):
            if cc == bm[i][1]:
                return F32(lp[cc] + bm[i][2]) if bm[i][2] != NEG else NEG
            return F32(lp[cc] + score[i])

        cands = []
        ts_upd = {}
        for i in range(nb):
            for cc in range(c):
                k = i * c + cc
                if cc == blank:
                    last = bm[i][1]
                    pb = F32(lp[blank] + score[i]) if allowed[blank] else NEG
                    pnb = F32(lp[last] + bm[i][3]) if (last >= 0 and allowed[last]) else NEG
                    j = pidx[i]
                    if j >= 0 and allowed[last]:
                        pnb = lse(pnb, ext_val(j, last))
                        if lp[last] > lpc[bm[i][0]]:
                            ts_upd[bm[i][0]] = (t, lp[last])
                    s = lse(pb, pnb)
                    if s != NEG:
                        cands.append((s, last, k, 'stay', i, pb, pnb))
                else:
                    if not allowed[cc] or (i, cc) in child_of:
                        continue
                    x = alive.get((bm[i][0], cc))      # a pruned node still in the trie
                    if x is not None and lp[cc] > lpc[x]:
                        ts_upd[x] = (t, lp[cc])
                    e = ext_val(i, cc)
                    if e != NEG:
                        cands.append((e, cc, k, 'ext', i, NEG, e))
        for node, (tt, v) in ts_upd.items():
            ts[node] = tt
            lpc[node] = v
        cands.sort(key=lambda x: (-float(x[0]), x[1], x[2]))
        new = []
        for s, last, k, kind, i, pb, pnb in cands[:beam]:
            if kind == 'stay':
                new.append([bm[i][0], last, pb, pnb])
            elif (bm[i][0], last) in alive:           # revived
                STATS["revived"] += 1
                new.append([alive[(bm[i][0], last)], last, pb, pnb])
            else:
                parent.append(bm[i][0])
                ch.append(last)
                ts.append(t)
                lpc.append(lp[last])
                new.append([len(parent) - 1, last, pb, pnb])
        bm = new
        if not bm:
            break
    final = [(lse(e[2], e[3]), e[1], idx, e[0]) for idx, e in enumerate(bm)]
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


def beam_decode(probs, sizes: Sequence[int], beam: int, blank: int = 0, cutoff_top_n: int = 40,
                cutoff_prob: float = 1.0):
    """Batched: probs [N, T, C] -> per utterance the list of beam_decode_one results."""
    p = np.asarray(probs, dtype=np.float32)
    return [beam_decode_one(p[i], int(sizes[i]), beam, blank, cutoff_top_n, cutoff_prob)
            for i in range(p.shape[0])]
