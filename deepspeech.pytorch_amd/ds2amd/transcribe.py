"""Inference entry points on the HIP path (ref transcribe.py:33-71).

`transcribe` keeps the reference's single-utterance signature; `transcribe_batch`
is the batched variant SURVEY §8f#1 asks for (cfg5: many long utterances per
forward): raw PCM (or wav paths) -> device STFT -> DeepSpeech.forward in eval mode
-> Greedy/Beam decoder, with one host copy of the decoded ids at the end.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Union

import numpy as np
import torch

from .data_loader import SpectrogramParser, load_audio_norm


def transcribe(audio_path, parser: SpectrogramParser, model, decoder, device=None):
    """ref transcribe.py:63-71: one wav file -> (decoded_output, decoded_offsets)."""
    return transcribe_batch([audio_path], parser, model, decoder)


def transcribe_batch(audio: Sequence[Union[str, np.ndarray]], parser: SpectrogramParser, model,
                     decoder, sample_rate=None):
    """Batched transcription: wav paths or float32 PCM arrays (normalised to max |x| = 1,
    like data/audio_loader.py) -> (decoded_output[N][paths], decoded_offsets[N][paths])."""
    signals: List[np.ndarray] = []
    sr = sample_rate
    for a in audio:
        if isinstance(a, (str, os.PathLike)):
            y, sr_a = load_audio_norm(a, channel=parser.channel)
            sr = sr or sr_a
            signals.append(y)
        else:
            signals.append(np.asarray(a, dtype=np.float32))
    was_training = model.training
    model.eval()
    with torch.no_grad():
        spect, frames = parser.parse_batch(signals, sr)
        _, probs, out_lens = model(spect, frames)
        decoded_output, decoded_offsets = decoder.decode(probs, out_lens)
    model.train(was_training)
    return decoded_output, decoded_offsets


def decode_results(decoded_output, decoded_offsets, top_paths=1, offsets=False, meta=None):
    """ref transcribe.py:33-60 (the JSON body the reference CLI prints)."""
    results = {"output": []}
    if meta is not None:
        results["_meta"] = meta
    for b in range(len(decoded_output)):
        for pi in range(min(top_paths, len(decoded_output[b]))):
            result = {'transcription': decoded_output[b][pi]}
            if offsets:
                result['offsets'] = decoded_offsets[b][pi].tolist()
            results['output'].append(result)
    return results
