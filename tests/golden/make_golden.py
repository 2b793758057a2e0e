"""Generate the golden fixtures from the REFERENCE implementation (build container only).

Run:  python tests/golden/make_golden.py      (needs /root/reference; never on the GPU box)

Imports the reference's own model.py and decoder.py from /root/reference
(read-only) and restates only the glue that cannot run on torch 2.10 CPU
(SURVEY.md §0/§8c): the is_cuda asserts / .cuda() calls in DeepSpeech.forward and
BatchRNN.forward, and MaskConv's uint8 masked_fill mask (a bool mask with the
same positions).  warpctc_pytorch is absent: the CTC stand-in is
torch.nn.functional.ctc_loss on log_softmax with reduction='sum'.

Outputs (committed): tests/golden/*.npz — inputs, expected outputs and weight
checksums.  Weights themselves are regenerated in the tests by constructing the
model under the same seed (the reference and ds2amd draw identical initial
weights; the checksum proves it).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REF)
sys.modules.setdefault("Levenshtein", types.ModuleType("Levenshtein"))
import model as ref_model      # noqa: E402  (reference model.py)
import decoder as ref_decoder  # noqa: E402  (reference decoder.py)

sys.path.insert(0, REPO)
from oracle import ds2_oracle as orc  # noqa: E402  (spectrogram restatement only)

LABELS = ''.join(__import__('json').load(open(os.path.join(REF, 'labels.json'))))
AUDIO_CONF = dict(sample_rate=16000, window_size=0.02, window_stride=0.01, window='hamming')


def ref_mask(x, lengths):
    """model.py:69-78 with a bool mask (torch 2.10 rejects the uint8 mask)."""
    mask = torch.zeros(x.size(), dtype=torch.bool)
    for i, length in enumerate(lengths):
        length = int(length)
        if (mask[i].size(2) - length) > 0:
            mask[i].narrow(2, length, mask[i].size(2) - length).fill_(True)
    return x.masked_fill(mask, 0)


def ref_forward(m, x, lengths, keep=None):
    """DeepSpeech.forward (model.py:343-380) minus the .cuda()/is_cuda glue."""
    lengths = lengths.cpu().int()
    output_lengths = m.get_seq_lens(lengths)
    for module in m.conv.seq_module:              # MaskConv.forward, model.py:69-79
        x = module(x)
        x = ref_mask(x, output_lengths)
        if keep is not None and isinstance(module, nn.Hardtanh):
            keep.append(x.detach().clone())
    sizes = x.size()
    x = x.view(sizes[0], sizes[1] * sizes[2], sizes[3])
    x = x.transpose(1, 2).transpose(0, 1).contiguous()
    for rnn in m.rnns:                             # BatchRNN.forward, model.py:97-109
        max_seq_length = x.size(0)
        if rnn.batch_norm is not None:
            x = rnn.batch_norm(x)
        x = nn.utils.rnn.pack_padded_sequence(x, output_lengths.data.cpu().numpy())
        x, h = rnn.rnn(x)
        x, _ = nn.utils.rnn.pad_packed_sequence(x, total_length=max_seq_length)
        if rnn.bidirectional:
            x = x.view(x.size(0), x.size(1), 2, -1).sum(2).view(x.size(0), x.size(1), -1)
        if keep is not None:
            keep.append(x.detach().clone())
    if not m._bidirectional:
        x = m.lookahead(x)
        if keep is not None:
            keep.append(x.detach().clone())
    x = m.fc(x)
    x = x.transpose(0, 1)
    outs = F.softmax(x, dim=-1)
    return x, outs, output_lengths


def make_ref(seed, hidden, layers, bidir=True, rnn_type='gru', context=20):
    torch.manual_seed(seed)
    return ref_model.DeepSpeech(rnn_type=rnn_type, labels=LABELS, rnn_hidden_size=hidden,
                                nb_layers=layers, audio_conf=AUDIO_CONF, bidirectional=bidir,
                                context=context)


def checksum(sd):
    keys = sorted(k for k in sd if sd[k].is_floating_point())
    return np.array([float(sd[k].double().sum()) for k in keys]), keys


def targets_for(out_lens, rng, n_classes=30):
    tl, tg = [], []
    for L in out_lens:
        k = int(rng.integers(1, max(2, int(L) // 2)))
        seq, prev = [], -1
        for _ in range(k):
            v = int(rng.integers(1, n_classes))
            while v == prev:
                v = int(rng.integers(1, n_classes))
            seq.append(v)
            prev = v
        tl.append(k)
        tg += seq
    return np.array(tg, np.int32), np.array(tl, np.int32)


def golden_tiny(path, seed=1234, hidden=16, layers=2, t_list=(64, 50, 31), rnn_type='gru',
                bidir=True, context=20):
    m = make_ref(seed, hidden, layers, bidir, rnn_type, context)
    m.train()
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    cs, keys = checksum(sd0)
    g = torch.Generator().manual_seed(seed + 1)
    n = len(t_list)
    t_max = max(t_list)
    x = torch.zeros(n, 1, 161, t_max)
    for i, t in enumerate(t_list):
        x[i, 0, :, :t] = torch.randn(161, t, generator=g)
    pct = torch.FloatTensor([t / float(t_max) for t in t_list])
    input_sizes = pct.clone().mul_(t_max).int()
    keep = []
    logits, probs, out_lens = ref_forward(m, x, input_sizes, keep)
    rng = np.random.default_rng(seed)
    tg, tl = targets_for(out_lens.tolist(), rng)
    # one reference training step (train.py:600-632), CTC via the F.ctc_loss stand-in
    m2 = make_ref(seed, hidden, layers, bidir, rnn_type, context)
    m2.train()
    opt = torch.optim.SGD(m2.parameters(), lr=3e-4, momentum=0.9, nesterov=True)
    lg, pr, ol = ref_forward(m2, x, input_sizes)
    acts = lg.transpose(0, 1)
    loss = F.ctc_loss(F.log_softmax(acts, 2), torch.from_numpy(tg).long(), ol.long(),
                      torch.from_numpy(tl).long(), reduction='sum') / n
    opt.zero_grad()
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in m2.named_parameters()}   # pre-clip
    gnorm = torch.nn.utils.clip_grad_norm_(m2.parameters(), 100.0)
    opt.step()
    after = {k: v.detach().clone() for k, v in m2.state_dict().items()}
    dec = ref_decoder.GreedyDecoder(LABELS)
    strings, offsets = dec.decode(probs, out_lens)
    out = dict(seed=seed, hidden=hidden, layers=layers, rnn_type=rnn_type, bidirectional=bidir,
               context=context, x=x.numpy(), pct=pct.numpy(),
               input_sizes=input_sizes.numpy(), logits=logits.detach().numpy(),
               probs=probs.detach().numpy(), out_lens=out_lens.numpy(), targets=tg,
               target_sizes=tl, loss=np.float32(loss.item()), grad_norm=np.float32(gnorm),
               checksum=cs, checksum_keys=np.array(keys),
               decoded=np.array([s[0] for s in strings]),
               conv1=keep[0].numpy(), conv2=keep[1].numpy())
    for i in range(layers):
        out[f'rnn{i}'] = keep[2 + i].numpy()
    if not bidir:
        out['lookahead'] = keep[2 + layers].numpy()
    for k, v in m.state_dict().items():            # running stats after one train forward
        if 'running' in k:
            out['after_fwd/' + k] = v.numpy()
    for k, v in after.items():
        if v.is_floating_point():
            out['after_step/' + k] = v.numpy()
    for k, v in grads.items():
        out['grad/' + k] = v.numpy()
    np.savez_compressed(path, **out)
    print('wrote', path, 'loss', float(loss.detach()), 'decoded', strings)


def golden_cfg1(path, seed=4321):
    """cfg1: 1 s synthetic wav, 2-layer BiGRU-256, eval forward + greedy decode."""
    rng = np.random.default_rng(1234)
    n = 16000
    t = np.arange(n) / 16000.0
    y = 0.1 * rng.standard_normal(n)
    for _ in range(3):
        y += np.sin(2 * np.pi * rng.uniform(100, 4000) * t + rng.uniform(0, 2 * np.pi))
    y = (y / np.abs(y).max()).astype(np.float32)
    spect = orc.spectrogram(y)                     # [161, 101] (librosa restatement)
    m = make_ref(seed, 256, 2)
    m.eval()
    cs, keys = checksum(m.state_dict())
    x = spect.view(1, 1, spect.size(0), spect.size(1))
    with torch.no_grad():
        logits, probs, out_lens = ref_forward(m, x, torch.IntTensor([spect.size(1)]))
    dec = ref_decoder.GreedyDecoder(LABELS)
    strings, offsets = dec.decode(probs, out_lens)
    np.savez_compressed(path, seed=seed, wav=y, spect=spect.numpy(), logits=logits.numpy(),
                        probs=probs.numpy(), out_lens=out_lens.numpy(), checksum=cs,
                        checksum_keys=np.array(keys), decoded=np.array([strings[0][0]]),
                        offsets=offsets[0][0].numpy())
    print('wrote', path, strings)


def golden_decoder(path):
    """GreedyDecoder known answers from the reference decoder.py (incl. argmax ties)."""
    dec = ref_decoder.GreedyDecoder(LABELS)
    g = torch.Generator().manual_seed(7)
    n, t, c = 6, 40, 30
    probs = torch.rand(n, t, c, generator=g)
    # plant ties, blanks, repeats and spaces
    probs[0, 3, 5] = probs[0, 3, 9] = 2.0            # tie -> first index (5)
    probs[1, :, 0] += 3.0                            # mostly blanks
    probs[2, 10:20, 29] += 5.0                        # a run of spaces
    probs[3, :, 7] += 5.0                             # one long repeat -> single char
    probs[4, ::2, 0] += 9.0                           # alternating blank/char
    sizes = torch.IntTensor([40, 33, 40, 17, 40, 0])
    strings, offsets = dec.decode(probs, sizes)
    # the SURVEY's hand case: [0,2,2,0,2,29] -> 'AA ' offsets [1,4,5]
    hp = torch.zeros(1, 6, 30)
    for i, k in enumerate([0, 2, 2, 0, 2, 29]):
        hp[0, i, k] = 1.0
    hs, ho = dec.decode(hp, torch.IntTensor([6]))
    np.savez_compressed(path, probs=probs.numpy(), sizes=sizes.numpy(),
                        strings=np.array([s[0] for s in strings]),
                        offsets=np.array([np.pad(o[0].numpy(), (0, t - len(o[0])), constant_values=-1)
                                          for o in offsets]),
                        counts=np.array([len(o[0]) for o in offsets]),
                        hand_probs=hp.numpy(), hand_string=np.array([hs[0][0]]),
                        hand_offsets=ho[0][0].numpy())
    print('wrote', path, strings, hs)


def golden_seq_lens(path):
    m = make_ref(0, 8, 1)
    L = torch.arange(1, 3002, dtype=torch.int32)
    out = m.get_seq_lens(L)
    # train.py:557 quirk: (len / T_max as float32) * T_max -> int
    tmax = 1001
    pct = torch.FloatTensor([l / float(tmax) for l in range(1, tmax + 1)])
    sizes = pct.clone().mul_(tmax).int()
    np.savez_compressed(path, lengths=L.numpy(), seq_lens=out.numpy(), tmax=tmax,
                        pct_sizes=sizes.numpy())
    print('wrote', path)


def golden_package(path, seed=1234):
    """A reference-format model package (model.py:426-468 serialize) of the tiny golden
    model, for checkpoint compatibility."""
    m = make_ref(seed, 16, 2)
    pkg = ref_model.DeepSpeech.serialize(
        m, epoch=2, iteration=5, loss_results=torch.tensor([3.0, 2.5, 2.0]),
        cer_results=torch.tensor([90.0, 80.0, 70.0]), wer_results=torch.tensor([99.0, 95.0, 90.0]),
        avg_loss=2.0, checkpoint=True)
    torch.save(pkg, path)
    print('wrote', path, sorted(pkg))


def golden_resume(pkg_path, npz_path, seed=1234):
    """Optimizer-state compatibility (model.py:446 package['optim_dict'] =
    optimizer.state_dict(); train.py:838-844 resume): the tiny model after ONE reference
    train step with torch.optim.SGD(nesterov), serialized by the reference's own serialize
    (weights, BN buffers and the SGD state dict), plus the parameters after a SECOND step on
    the same batch -- what a resumed run must reproduce."""
    g0 = np.load(os.path.join(HERE, 'tiny_ds2.npz'))
    m = make_ref(seed, 16, 2)
    m.train()
    opt = torch.optim.SGD(m.parameters(), lr=3e-4, momentum=0.9, nesterov=True)
    x = torch.from_numpy(g0['x'])
    tg = torch.from_numpy(g0['targets']).long()
    tl = torch.from_numpy(g0['target_sizes']).long()
    input_sizes = torch.from_numpy(g0['pct']).clone().mul_(x.shape[3]).int()

    def step():
        lg, _, ol = ref_forward(m, x, input_sizes)
        acts = lg.transpose(0, 1)
        loss = F.ctc_loss(F.log_softmax(acts, 2), tg, ol.long(), tl, reduction='sum') / x.shape[0]
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 100.0)
        opt.step()
        return float(loss)

    loss1 = step()
    pkg = ref_model.DeepSpeech.serialize(m, optimizer=opt, epoch=0, iteration=0)
    torch.save(pkg, pkg_path)
    loss2 = step()
    out = dict(loss1=np.float32(loss1), loss2=np.float32(loss2))
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            out['after_step2/' + k] = v.numpy()
    for i, st in opt.state_dict()['state'].items():
        out[f'momentum2/{i}'] = st['momentum_buffer'].numpy()
    np.savez_compressed(npz_path, **out)
    print('wrote', pkg_path, npz_path, 'losses', loss1, loss2)


if __name__ == '__main__':
    torch.set_num_threads(8)
    golden_tiny(os.path.join(HERE, 'tiny_ds2.npz'))
    golden_tiny(os.path.join(HERE, 'tiny_lstm_bi.npz'), seed=2024, rnn_type='lstm')
    golden_tiny(os.path.join(HERE, 'tiny_lstm_uni.npz'), seed=2025, rnn_type='lstm', bidir=False,
                context=20)
    golden_tiny(os.path.join(HERE, 'tiny_gru_uni.npz'), seed=2026, rnn_type='gru', bidir=False,
                context=3)
    golden_tiny(os.path.join(HERE, 'tiny_rnn_bi.npz'), seed=2027, rnn_type='rnn')
    golden_cfg1(os.path.join(HERE, 'cfg1_ds2.npz'))
    golden_decoder(os.path.join(HERE, 'greedy_decoder.npz'))
    golden_seq_lens(os.path.join(HERE, 'seq_lens.npz'))
    golden_package(os.path.join(HERE, 'tiny_ref_package.pth'))
    golden_resume(os.path.join(HERE, 'tiny_ref_resume.pth'), os.path.join(HERE, 'tiny_resume.npz'))
