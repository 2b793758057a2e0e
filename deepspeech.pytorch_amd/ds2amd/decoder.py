"""Decoders — drop-in for the reference ``decoder.py``.

``GreedyDecoder.decode`` runs argmax + CTC collapse in one HIP kernel
(ds2_greedy_decode) and copies back only the compacted label ids/offsets, instead
of the reference's per-frame ``.item()`` loop (ref decoder.py:165-197).  The
string semantics are the reference's: first maximum wins, blanks dropped, a
frame equal to the previous *frame* is dropped, the space label maps to ' ' and
'2' is emitted literally.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


def _levenshtein(a, b) -> int:
    """Edit distance (python-Levenshtein's Lev.distance semantics)."""
    if len(a) < len(b):
        a, b = b, a
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i]
        for j, cb in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
        prev = cur
    return prev[-1]


class Decoder(object):
    """Base decoder (ref decoder.py:23-87)."""

    def __init__(self, labels, blank_index=0):
        self.labels = labels
        self.int_to_char = dict([(i, c) for (i, c) in enumerate(labels)])
        self.blank_index = blank_index
        space_index = len(labels)
        if ' ' in labels:
            space_index = labels.index(' ')
        self.space_index = space_index

    def wer(self, s1, s2):
        b = set(s1.split() + s2.split())
        word2char = dict(zip(b, range(len(b))))
        w1 = [chr(word2char[w]) for w in s1.split()]
        w2 = [chr(word2char[w]) for w in s2.split()]
        return _levenshtein(''.join(w1), ''.join(w2))

    def cer(self, s1, s2):
        s1, s2, = s1.replace(' ', ''), s2.replace(' ', '')
        return _levenshtein(s1, s2)

    def decode(self, probs, sizes=None):
        raise NotImplementedError

    def _row_string(self, row) -> str:
        """Label ids (numpy int row) -> string: one UTF-32 table lookup when every label is a
        single character (a per-id Python join cost ~3 ms per 32 x 30 s batch, more than the
        greedy kernel itself)."""
        lut = getattr(self, "_lut32", None)
        if lut is None:
            single = all(len(c) == 1 for c in self.labels)
            lut = np.array([ord(c) for c in self.labels], dtype="<u4") if single else False
            self._lut32 = lut
        if lut is False:
            return ''.join(self.int_to_char[int(c)] for c in row)
        return lut[row].tobytes().decode("utf-32-le")


class BeamCTCDecoder(Decoder):
    """CTC prefix beam search on the GPU (ds2_ctc_beam_decode[_lm]), drop-in for ref
    decoder.py:90-143.

    Same constructor and ``decode(probs, sizes) -> (strings, offsets)`` as the
    reference, whose ctcdecode backend returns every beam: strings[n][p] /
    offsets[n][p] for p < beam_width, best first.  With ``lm_path`` (an ARPA file --
    KenLM's text format; its binary format is not read) the search scores words with
    the n-gram model like ctcdecode's KenLM Scorer (alpha: LM weight, beta: word bonus;
    ds2amd/lm.py builds the device tables once); without an LM ctcdecode ignores
    alpha/beta and so does this.
    """

    def __init__(self, labels, lm_path=None, alpha=0, beta=0, cutoff_top_n=40, cutoff_prob=1.0,
                 beam_width=100, num_processes=4, blank_index=0):
        super().__init__(labels, blank_index=blank_index)
        self.scorer = None
        if lm_path is not None:
            from .lm import ArpaScorer
            self.scorer = ArpaScorer(lm_path, labels, alpha, beta)
        # the device search keeps every candidate in one wave's registers:
        # beam_width <= 128 over <= 32 labels (the reference default 100 over 29), or
        # beam_width <= 32 over <= 64 labels
        if beam_width > (128 if len(labels) <= 32 else 32) or len(labels) > 64:
            raise ValueError("ds2amd.BeamCTCDecoder: beam_width <= 128 with <= 32 labels, "
                             "or beam_width <= 32 with <= 64 labels")
        self.beam_width = int(beam_width)
        self.cutoff_top_n = int(cutoff_top_n)
        self.cutoff_prob = float(cutoff_prob)

    def decode_raw(self, probs, sizes=None):
        """Device tensors (ids [N,P,T], offsets [N,P,T], lens [N,P], scores [N,P])."""
        if self.scorer is not None:
            return ops.ctc_beam_decode_lm_raw(probs, sizes, self.beam_width, self.beam_width,
                                              self.scorer, blank=self.blank_index,
                                              cutoff_top_n=self.cutoff_top_n,
                                              cutoff_prob=self.cutoff_prob)
        return ops.ctc_beam_decode_raw(probs, sizes, self.beam_width, self.beam_width,
                                       blank=self.blank_index, cutoff_top_n=self.cutoff_top_n,
                                       cutoff_prob=self.cutoff_prob)

    def convert_to_strings(self, out, seq_len):
        """[batch][beam][T] label ids (ctcdecode's ``beam_results``) and [batch][beam]
        lengths -> [batch][beam] strings; a beam of length <= 0 is ''.  Ref
        decoder.py:101-113 (tensors, numpy arrays or nested lists)."""
        results = []
        for b, batch in enumerate(out):
            utterances = []
            for p, utt in enumerate(batch):
                size = int(seq_len[b][p])
                row = np.asarray(utt[0:size] if size > 0 else [], dtype=np.int64)
                utterances.append(self._row_string(row) if size > 0 else '')
            results.append(utterances)
        return results

    def convert_tensor(self, offsets, sizes):
        """[batch][beam][T] frame offsets and [batch][beam] lengths -> per beam the first
        ``size`` offsets (an empty int tensor for size <= 0).  Ref decoder.py:115-126."""
        results = []
        for b, batch in enumerate(offsets):
            utterances = []
            for p, utt in enumerate(batch):
                size = int(sizes[b][p])
                if size > 0:
                    utterances.append(utt[0:size])
                else:
                    utterances.append(torch.tensor([], dtype=torch.int))
            results.append(utterances)
        return results

    def decode(self, probs, sizes=None):
        """Ref decoder.py:128-143: (strings, offsets) per utterance and beam, best first;
        the reference's ``convert_to_strings`` / ``convert_tensor`` over the device search's
        (ids, offsets, lens), with one device->host copy and vectorised id->char lookups (a
        per-element tensor loop cost more than the beam search itself on 30 s utterances)."""
        ids, offs, lens, _ = self.decode_raw(probs, sizes)
        ids, offs, lens = ids.cpu().numpy(), offs.cpu().numpy(), lens.cpu().numpy()
        strings = self.convert_to_strings(ids, lens)
        offsets = self.convert_tensor(torch.from_numpy(offs), lens)
        return strings, offsets


class GreedyDecoder(Decoder):
    def __init__(self, labels, blank_index=0):
        super().__init__(labels, blank_index)

    def convert_to_strings(self, sequences, sizes=None, remove_repetitions=False,
                           return_offsets=False):
        """Host conversion of id sequences (targets) to strings (ref decoder.py:150-163)."""
        strings = []
        offsets = [] if return_offsets else None
        for x in range(len(sequences)):
            seq_len = sizes[x] if sizes is not None else len(sequences[x])
            string, string_offsets = self.process_string(sequences[x], seq_len, remove_repetitions)
            strings.append([string])
            if return_offsets:
                offsets.append([string_offsets])
        if return_offsets:
            return strings, offsets
        return strings

    def process_string(self, sequence, size, remove_repetitions=False):
        seq = [int(v) for v in (sequence.tolist() if torch.is_tensor(sequence) else sequence)]
        size = int(size)
        string = ''
        offsets = []
        blank = self.int_to_char[self.blank_index]
        for i in range(size):
            char = self.int_to_char[seq[i]]
            if char != blank:
                if remove_repetitions and i != 0 and char == self.int_to_char[seq[i - 1]]:
                    pass
                elif char == self.labels[self.space_index] if self.space_index < len(self.labels) else False:
                    string += ' '
                    offsets.append(i)
                else:
                    string = string + char
                    offsets.append(i)
        return string, torch.tensor(offsets, dtype=torch.int)

    def decode_ids(self, probs, sizes=None):
        """Device-side greedy decode; returns (ids, offsets, counts) int32 device tensors."""
        ids, offs, counts, _ = ops.greedy_decode_raw(probs, sizes, blank=self.blank_index)
        return ids, offs, counts

    def decode(self, probs, sizes=None):
        """Returns (strings, offsets) like ref decoder.py:182-197."""
        if not probs.is_cuda:
            raise RuntimeError("ds2amd GreedyDecoder.decode runs on the GPU (HIP kernel)")
        ids, offs, counts = self.decode_ids(probs, sizes)
        ids, offs, counts = ids.cpu().numpy(), offs.cpu().numpy(), counts.cpu().numpy()
        strings, offsets = [], []
        for b in range(ids.shape[0]):
            k = int(counts[b])
            # the space label is ' ' itself, so the label table maps it
            strings.append([self._row_string(ids[b, :k])])
            offsets.append([torch.from_numpy(offs[b, :k].astype(np.int32))])
        return strings, offsets
