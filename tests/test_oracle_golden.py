"""CPU: the oracle (and the host-side model constructor) against the reference's goldens.

The goldens were produced by tests/golden/make_golden.py from the reference's
own model.py / decoder.py.  These tests pin the oracle before any GPU result is
compared against it.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ds2_oracle as orc
from ds2amd import model as dsm

LABELS = orc.LABELS
CONF = dict(sample_rate=16000, window_size=0.02, window_stride=0.01, window='hamming')


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


TINY = ['tiny_ds2.npz', 'tiny_lstm_bi.npz', 'tiny_lstm_uni.npz', 'tiny_gru_uni.npz',
        'tiny_rnn_bi.npz']


def build_model(seed, hidden, layers, rnn_type='gru', bidirectional=True, context=20):
    torch.manual_seed(seed)
    return dsm.DeepSpeech(rnn_type=rnn_type, labels=LABELS, rnn_hidden_size=hidden,
                          nb_layers=layers, audio_conf=CONF, bidirectional=bidirectional,
                          context=context)


def tiny_spec(g):
    """(model kwargs, oracle kwargs) of a tiny golden (older files: BiGRU, context 20)."""
    rnn_type = str(g['rnn_type']) if 'rnn_type' in g.files else 'gru'
    bidir = bool(g['bidirectional']) if 'bidirectional' in g.files else True
    context = int(g['context']) if 'context' in g.files else 20
    mk = dict(seed=int(g['seed']), hidden=int(g['hidden']), layers=int(g['layers']),
              rnn_type=rnn_type, bidirectional=bidir, context=context)
    ok = dict(nb_layers=int(g['layers']), hidden=int(g['hidden']), bidirectional=bidir,
              rnn_type=rnn_type)
    return mk, ok


def _checksum(sd, keys):
    return np.array([float(sd[k].double().sum()) for k in keys])


@pytest.mark.parametrize("name", TINY)
def test_constructor_draws_reference_weights(golden_dir, name):
    g = _load(golden_dir, name)
    m = build_model(**tiny_spec(g)[0])
    keys = [str(k) for k in g['checksum_keys']]
    assert sorted(k for k, v in m.state_dict().items() if v.is_floating_point()) == sorted(keys)
    np.testing.assert_array_equal(_checksum(m.state_dict(), keys), g['checksum'])


def test_state_dict_keys_match_reference_cfg1(golden_dir):
    g = _load(golden_dir, 'cfg1_ds2.npz')
    m = build_model(int(g['seed']), 256, 2)
    keys = [str(k) for k in g['checksum_keys']]
    np.testing.assert_array_equal(_checksum(m.state_dict(), keys), g['checksum'])


@pytest.mark.parametrize("name", TINY)
def test_oracle_forward_tiny(golden_dir, name):
    g = _load(golden_dir, name)
    mk, ok = tiny_spec(g)
    m = build_model(**mk)
    o = orc.OracleDS2(m.state_dict(), **ok)
    x = torch.from_numpy(g['x'])
    sizes = orc.input_sizes_quirk(torch.from_numpy(g['pct']), x.shape[3])
    np.testing.assert_array_equal(sizes.numpy(), g['input_sizes'])
    logits, probs, out_lens, acts = o.forward(x, sizes, training=True, keep=True)
    np.testing.assert_array_equal(out_lens.numpy(), g['out_lens'])
    np.testing.assert_allclose(acts['conv1'].numpy(), g['conv1'], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(acts['conv2'].numpy(), g['conv2'], rtol=1e-5, atol=1e-5)
    for i in range(int(g['layers'])):
        np.testing.assert_allclose(acts[f'rnn{i}'].numpy(), g[f'rnn{i}'], rtol=1e-5, atol=1e-5)
    if 'lookahead' in g.files:
        np.testing.assert_allclose(acts['lookahead'].numpy(), g['lookahead'], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(logits.numpy(), g['logits'], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(probs.numpy(), g['probs'], rtol=1e-5, atol=1e-6)
    for k in g.files:
        if k.startswith('after_fwd/'):
            np.testing.assert_allclose(o.sd[k[len('after_fwd/'):]].numpy(), g[k], rtol=1e-5,
                                       atol=1e-6)
    strings, _ = orc.greedy_decode(probs, out_lens)
    assert [s[0] for s in strings] == [str(s) for s in g['decoded']]


@pytest.mark.parametrize("name", TINY)
def test_oracle_train_step_tiny(golden_dir, name):
    g = _load(golden_dir, name)
    mk, ok = tiny_spec(g)
    m = build_model(**mk)
    o = orc.OracleDS2(m.state_dict(), **ok)
    loss, new, bufs, grads, gnorm = orc.train_step(
        o, torch.from_numpy(g['x']), torch.from_numpy(g['pct']), torch.from_numpy(g['targets']),
        torch.from_numpy(g['target_sizes']))
    np.testing.assert_allclose(float(loss), float(g['loss']), rtol=1e-5)
    np.testing.assert_allclose(float(gnorm), float(g['grad_norm']), rtol=1e-4)
    for k, v in grads.items():
        np.testing.assert_allclose(v.numpy(), g['grad/' + k], rtol=1e-4, atol=1e-6, err_msg=k)
    for k, v in new.items():
        np.testing.assert_allclose(v.numpy(), g['after_step/' + k], rtol=1e-6, atol=1e-7, err_msg=k)


def test_oracle_cfg1(golden_dir):
    g = _load(golden_dir, 'cfg1_ds2.npz')
    spect = orc.spectrogram(g['wav'])
    np.testing.assert_allclose(spect.numpy(), g['spect'], rtol=0, atol=0)
    m = build_model(int(g['seed']), 256, 2)
    m.eval()
    o = orc.OracleDS2(m.state_dict(), 2, 256)
    x = spect.view(1, 1, spect.size(0), spect.size(1))
    with torch.no_grad():
        logits, probs, out_lens, _ = o.forward(x, torch.IntTensor([spect.size(1)]), training=False)
    np.testing.assert_allclose(logits.numpy(), g['logits'], rtol=1e-5, atol=1e-5)
    strings, offsets = orc.greedy_decode(probs, out_lens)
    assert strings[0][0] == str(g['decoded'][0])
    np.testing.assert_array_equal(offsets[0][0].numpy(), g['offsets'])


def test_oracle_greedy_known_answers(golden_dir):
    g = _load(golden_dir, 'greedy_decoder.npz')
    strings, offsets = orc.greedy_decode(torch.from_numpy(g['probs']), g['sizes'].tolist())
    assert [s[0] for s in strings] == [str(s) for s in g['strings']]
    for i, o in enumerate(offsets):
        np.testing.assert_array_equal(o[0].numpy(), g['offsets'][i][:int(g['counts'][i])])
    hs, ho = orc.greedy_decode(torch.from_numpy(g['hand_probs']), [6])
    assert hs[0][0] == 'AA ' == str(g['hand_string'][0])
    np.testing.assert_array_equal(ho[0][0].numpy(), [1, 4, 5])


def test_seq_lens_and_input_size_quirk(golden_dir):
    g = _load(golden_dir, 'seq_lens.npz')
    out = orc.get_seq_lens(torch.from_numpy(g['lengths']))
    np.testing.assert_array_equal(out.numpy(), g['seq_lens'])
    m = build_model(0, 8, 1)
    np.testing.assert_array_equal(m.get_seq_lens(torch.from_numpy(g['lengths'])).numpy(),
                                  g['seq_lens'])
    tmax = int(g['tmax'])
    pct = torch.FloatTensor([l / float(tmax) for l in range(1, tmax + 1)])
    np.testing.assert_array_equal(orc.input_sizes_quirk(pct, tmax).numpy(), g['pct_sizes'])
    # the survey's lossy lengths
    lossy = {127: 126, 254: 253, 255: 254, 508: 507, 510: 509}
    for k, v in lossy.items():
        assert int(g['pct_sizes'][k - 1]) == v


def test_ctc_oracle_hand_case():
    # T=2, C=2 (blank 0, 'a' 1), label 'a': paths "a_", "_a", "aa"
    acts = torch.log(torch.tensor([[[0.4, 0.6]], [[0.7, 0.3]]]))   # softmax == these probs
    loss, grad = orc.ctc_loss(acts, torch.IntTensor([1]), torch.IntTensor([2]),
                              torch.IntTensor([1]))
    p = 0.6 * 0.7 + 0.4 * 0.3 + 0.6 * 0.3
    assert abs(float(loss) + np.log(p)) < 1e-6
    # posterior of 'a' at t=0: (0.6*0.7 + 0.6*0.3)/p ; grad = y - posterior
    post_a0 = (0.6 * 0.7 + 0.6 * 0.3) / p
    assert abs(float(grad[0, 0, 1]) - (0.6 - post_a0)) < 1e-6


def test_stft_oracle_known_answers():
    sr, n = 16000, 16000
    t = np.arange(n) / sr
    k = 40                              # bin 40 = 2000 Hz (bins are 50 Hz apart)
    y = np.cos(2 * np.pi * k * 50 * t).astype(np.float32)
    mag = orc.stft_magnitude(y)
    assert mag.shape == (161, 101)
    w = orc.hamming(320)
    # interior frame: |X_k| = sum(w)/2 for a unit cosine exactly on bin k
    np.testing.assert_allclose(mag[k, 50], w.sum() / 2, rtol=1e-4)
    assert mag[:, 50].argmax() == k
    assert np.all(orc.stft_magnitude(np.zeros(3200, np.float32)) == 0)
    dc = orc.stft_magnitude(np.ones(3200, np.float32))
    np.testing.assert_allclose(dc[0, 5], w.sum(), rtol=1e-6)


def test_hamming_matches_scipy():
    from scipy.signal import windows
    np.testing.assert_allclose(orc.hamming(320), windows.hamming(320, sym=True), rtol=0, atol=1e-15)


def test_beam_oracle_hand_case():
    """Prefix beam search sums over alignments: T=2, probs (blank .6, 'a' .4) per frame.
    'a' = aa + a_ + _a = .16 + .24 + .24 = .64 beats '' = .36 (greedy would say '')."""
    from oracle import ctc_beam
    probs = np.array([[0.6, 0.4], [0.6, 0.4]], np.float32)
    res = ctc_beam.beam_decode_one(probs, 2, beam=4, blank=0)
    assert res[0][1] == [1] and abs(res[0][0] - np.log(0.64)) < 1e-6
    assert res[1][1] == [] and abs(res[1][0] - np.log(0.36)) < 1e-6
    assert res[0][2] == [0]                       # best extension event of 'a' at frame 0 (tie -> first)
    # vocabulary pruning: with cutoff_top_n = 1 only the blank survives each frame
    res = ctc_beam.beam_decode_one(probs, 2, beam=4, blank=0, cutoff_top_n=1)
    assert len(res) == 1 and res[0][1] == []


def test_beam_oracle_beam1_peaked_equals_greedy():
    from oracle import ctc_beam
    g = np.random.default_rng(3)
    t, c = 40, 30
    ids = g.integers(0, c, t)
    probs = np.full((t, c), 0.1 / (c - 1), np.float32)
    probs[np.arange(t), ids] = 0.9
    res = ctc_beam.beam_decode_one(probs, t, beam=1)
    strings, _ = orc.greedy_decode(torch.from_numpy(probs[None]), [t])
    assert ''.join(LABELS[k] for k in res[0][1]) == strings[0][0]


def test_reference_package_round_trip(golden_dir, tmp_path):
    """Checkpoint compatibility (model.py:395-468): a package written by the
    reference's DeepSpeech.serialize loads into ds2amd (torch.load weights_only=True) with
    identical weights and metadata; ds2amd's serialize writes the same structure back."""
    path = os.path.join(golden_dir, 'tiny_ref_package.pth')
    m = dsm.DeepSpeech.load_model(path)
    ref_pkg = torch.load(path, map_location='cpu', weights_only=True)
    g = _load(golden_dir, 'tiny_ds2.npz')
    fresh = build_model(**tiny_spec(g)[0])
    for k, v in fresh.state_dict().items():
        assert torch.equal(m.state_dict()[k], v), k
    assert (m._hidden_size, m._hidden_layers, m._rnn_type, m._bidirectional) == \
        (ref_pkg['hidden_size'], ref_pkg['hidden_layers'], ref_pkg['rnn_type'],
         ref_pkg['bidirectional'])
    ours = dsm.DeepSpeech.serialize(m, epoch=ref_pkg['epoch'] - 1, iteration=ref_pkg['iteration'],
                                    loss_results=ref_pkg['loss_results'],
                                    cer_results=ref_pkg['cer_results'],
                                    wer_results=ref_pkg['wer_results'],
                                    avg_loss=ref_pkg['avg_loss'], checkpoint=ref_pkg['checkpoint'])
    assert sorted(ours) == sorted(ref_pkg)
    for k in ref_pkg:
        a, b = ours[k], ref_pkg[k]
        if k == 'state_dict':
            assert sorted(a) == sorted(b)
            assert all(torch.equal(a[n], b[n]) for n in a)
        elif torch.is_tensor(b):
            assert torch.equal(a, b), k
        else:
            assert a == b, k
    out = tmp_path / 'ours.pth'
    torch.save(ours, out)
    m2 = dsm.DeepSpeech.load_model(str(out))
    assert all(torch.equal(m2.state_dict()[n], v) for n, v in m.state_dict().items())


# ------------------------------------------------------------------ spectrogram augmentations
def test_spect_aug_draws_follow_reference_semantics():
    """ds2amd.spect_aug draws bands exactly as data/spectrogram_aug.py would zero them,
    call for call on a seeded random.Random (restated; the reference module needs cv2,
    absent here, so the draw order is pinned by the code it restates, not by a run)."""
    import random
    from ds2amd.spect_aug import SpectAugmenter, apply_masks_np
    conf = dict(noise_prob=1.0, aug_prob_spect=0.5, aug_prob_8khz=0.5)
    a = SpectAugmenter(conf, rng=random.Random(7))
    # hand replay of the same sequence on a second generator
    r = random.Random(7)
    rows = [a.draw_one(161, 300) for _ in range(6)]
    probs = {"freq": 0.5, "time": 0.5}
    for row in rows:
        assert r.random() < 1.0                       # SOneOf(prob = noise_prob = 1)
        kind = r.choice(["freq", "time"])
        probs[kind] = 1.0                             # reference side effect: t.prob = 1
        exp = [0, 0, 0, 0, 0, 0, 0, 0, 161]
        bands = []
        for _ in range(2):
            if r.random() < probs[kind]:
                if kind == "freq":
                    w = r.randint(0, 20)
                    c = r.randint(0, 161)
                    bands.append((max(0, int(c - w // 2)), min(int(c + w // 2), 161)))
                else:
                    w = min(r.randint(0, 50), int(.15 * 300))
                    c = r.randint(0, 300)
                    bands.append((max(0, int(c - w // 2)), min(int(c + w // 2), 300)))
        base = 0 if kind == "freq" else 4
        for i, (lo, hi) in enumerate(bands):
            exp[base + 2 * i], exp[base + 2 * i + 1] = lo, hi
        if r.random() < 0.5:
            exp[8] = 81
        assert row == exp
    # numpy application = the reference's slicing
    s = np.ones((161, 300), np.float32)
    apply_masks_np(s, [10, 20, 150, 140, 5, 7, 0, 0, 81])
    assert s[10:20].sum() == 0 and s[81:].sum() == 0 and s[:, 5:7].sum() == 0
    assert s[0:10, 7:].min() == 1 and s[20:81, 7:].min() == 1      # reversed band is empty


# ------------------------------------------------------------------ optimizer-state compatibility
def _resume_inputs(golden_dir):
    pkg = torch.load(os.path.join(golden_dir, 'tiny_ref_resume.pth'), map_location='cpu',
                     weights_only=True)
    g0 = _load(golden_dir, 'tiny_ds2.npz')
    g2 = _load(golden_dir, 'tiny_resume.npz')
    return pkg, g0, g2


def test_oracle_resume_matches_reference(golden_dir):
    """The oracle resumed from a reference package (weights + BN buffers + the SGD state
    dict, model.py:426-468 / train.py:838-844) reproduces the reference's second step."""
    pkg, g0, g2 = _resume_inputs(golden_dir)
    m = dsm.DeepSpeech.load_model_package(pkg)
    names = [n for n, _ in m.named_parameters()]
    o = orc.OracleDS2(pkg['state_dict'], nb_layers=2, hidden=16)
    bufs = orc.momentum_from_optim_dict(names, pkg['optim_dict'])
    assert len(bufs) == len(names)
    loss, new, nb, _, _ = orc.train_step(
        o, torch.from_numpy(g0['x']), torch.from_numpy(g0['pct']).clone(),
        torch.from_numpy(g0['targets']), torch.from_numpy(g0['target_sizes']),
        momentum_buffers=bufs)
    np.testing.assert_allclose(float(loss), float(g2['loss2']), rtol=1e-5)
    for k, v in new.items():
        np.testing.assert_allclose(v.numpy(), g2['after_step2/' + k], rtol=1e-6, atol=1e-7, err_msg=k)
    for i, n in enumerate(names):
        np.testing.assert_allclose(nb[n].numpy(), g2[f'momentum2/{i}'], rtol=1e-5, atol=1e-8,
                                   err_msg=n)


def test_fused_sgd_state_dict_is_torch_sgd_format(golden_dir):
    """FusedSGD (flat buffers, reverse layer order inside) loads a reference optim_dict and
    writes back exactly torch.optim.SGD's format in model.parameters() order; torch's own
    SGD accepts what it writes; anything else is refused (no silent momentum restart)."""
    from ds2amd.optim import FlatParams, FusedSGD
    pkg, _, _ = _resume_inputs(golden_dir)
    m = dsm.DeepSpeech.load_model_package(pkg)
    flat = FlatParams(list(m.parameters()), 'cpu')
    opt = FusedSGD(flat, lr=1.0, momentum=0.5, max_norm=100.0)
    ref = pkg['optim_dict']
    opt.load_state_dict(ref)
    assert (opt.lr, opt.momentum) == (ref['param_groups'][0]['lr'], ref['param_groups'][0]['momentum'])
    ours = opt.state_dict()
    assert sorted(ours) == ['param_groups', 'state']
    assert ours['param_groups'][0]['params'] == ref['param_groups'][0]['params']
    for k in ('lr', 'momentum', 'nesterov', 'dampening', 'weight_decay'):
        assert ours['param_groups'][0][k] == ref['param_groups'][0][k], k
    assert sorted(ours['state']) == sorted(ref['state'])
    for i, st in ref['state'].items():
        assert torch.equal(ours['state'][i]['momentum_buffer'], st['momentum_buffer']), i
    sgd = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, nesterov=True)
    sgd.load_state_dict(ours)
    # set_lr (train.py:322-326) round trip
    sd = opt.state_dict()
    sd['param_groups'][0]['lr'] = 1e-5
    opt.load_state_dict(sd)
    assert opt.lr == 1e-5
    with pytest.raises(ValueError):
        opt.load_state_dict({'lr': 1.0, 'momentum': 0.9, 'momentum_buffer': torch.zeros(3)})
    bad = opt.state_dict()
    bad['param_groups'][0]['nesterov'] = False
    with pytest.raises(ValueError):
        opt.load_state_dict(bad)


def test_rows161_resize_mirror_semantics():
    """data_loader_aug.py:233-238,249: a Fortran-ordered magnitude with < 161 bins (librosa's
    layout) resized in memory order then mirrored; >= 161 bins cut to 161; 161 untouched."""
    F, T = 81, 7
    m = np.asfortranarray(np.arange(F * T, dtype=np.float32).reshape(T, F).T + 1)  # [F, T]
    r = orc.rows161(m)
    flat = m.T.reshape(-1)                       # frame-major memory order
    exp = np.zeros((161, T), np.float32)
    for t in range(T):
        for row in range(81):
            k = 161 * t + row
            exp[row, t] = flat[k] if k < F * T else 0
    exp[81:] = exp[80:0:-1]
    np.testing.assert_array_equal(r, exp)
    assert np.array_equal(m, np.asfortranarray(np.arange(F * T, dtype=np.float32)
                                               .reshape(T, F).T + 1))   # input untouched
    big = np.ones((221, 5), np.float32)
    assert orc.rows161(big).shape == (161, 5)
    y = np.random.default_rng(0).standard_normal(8000).astype(np.float32)
    assert orc.spectrogram(y, sample_rate=8000).shape == (161, 101)
