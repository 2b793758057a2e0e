"""GPU: the training step (ds2amd.trainer.Trainer = train.py:555-632) at the benchmark's own
shape, its failure semantics, optimizer-state resume and the data-parallel hook path, each
against the CPU oracle (itself pinned by the reference goldens, tests/test_oracle_golden.py).

Tolerances (north_star / DESIGN.md §2): loss and logits within 1e-4 relative
(max |diff| / max |ref|); the gradient norm within 2e-4 and every parameter gradient within 5e-4
relative (BPTT over 501 steps in fp32 with a different summation order than MIOpen/ATen, and an
fp32 CTC against the oracle's fp64 one); lengths, argmax and decoded strings bit-exact.
"""
import os

import numpy as np
import pytest
import torch

from ds2amd import _lib, ops
from ds2amd import model as dsm
from ds2amd.trainer import Trainer
from oracle import ds2_oracle as orc

pytestmark = pytest.mark.gpu

LABELS = orc.LABELS
CONF = dict(sample_rate=16000, window_size=0.02, window_stride=0.01, window='hamming')


def _rel(got, ref):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu() if torch.is_tensor(ref) else torch.from_numpy(ref).double()
    return (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)


def _build(seed, hidden, layers, rnn_type='gru', bidirectional=True):
    torch.manual_seed(seed)
    return dsm.DeepSpeech(rnn_type=rnn_type, labels=LABELS, rnn_hidden_size=hidden,
                          nb_layers=layers, audio_conf=CONF, bidirectional=bidirectional)


def _threads():
    torch.set_num_threads(max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or 16))))


def _targets(g, lens):
    tg = []
    for L in lens:
        prev = -1
        for _ in range(L):
            v = int(torch.randint(1, 29, (1,), generator=g))
            while v == prev:
                v = int(torch.randint(1, 29, (1,), generator=g))
            tg.append(v)
            prev = v
    return torch.tensor(tg, dtype=torch.int32), torch.tensor(lens, dtype=torch.int32)


def _spect_batch(g, t_list, t_max):
    x = torch.zeros(len(t_list), 1, 161, t_max)
    for i, t in enumerate(t_list):
        x[i, 0, :, :t] = torch.randn(161, t, generator=g)
    return x


# --------------------------------------------------------------------------- benchmark shape
def test_benchmark_train_step_matches_oracle(dev):
    """5 x BiGRU-800 at T = 1001 (10 s), bs 4, variable lengths through input_percentages
    with the float32 quirk lengths of T_max = 1001 (508 -> 507, 254 -> 253; train.py:557):
    the full Trainer.train_batch (forward, decode, CTC, BPTT over 501 steps in ONE
    16-sample batch tile of the persistent kernels, clip, SGD-Nesterov) vs oracle.train_step.
    Two batch tiles at this shape: test_benchmark_train_step_two_batch_tiles.

    The conv block's arithmetic is checked against fp64 with our own Hardtanh masks (the
    conv_fp64 check: every conv gradient within 1.25x of the fp32 oracle's distance).  End to end
    against the oracle its gradients get 5e-2: ONE of the 2.6 M conv2 masks sits on the other
    side of a kink in the oracle's fp32 forward, and that one position moves conv2's weight
    gradient by 1.8e-2 (profiles/r6e_bs4_conv_flip.txt).  Recurrent / FC gradients past 5e-4
    from the fp32 oracle go to the float64 arbiter: since the rescaled CTC scans ours sit
    ~5e-6 from fp64, the oracle (torch's fp32 CPU CTC) up to 7e-4, so the oracle's own error
    sets the distance between the two (4.1e-4 at the last run)."""
    _check_train_step(dev, [1001, 877, 508, 254], [150, 120, 80, 40], seed=11, conv_fp64=True,
                      conv_tol=5e-2, rnn_fp64=True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("rnn_type", ["rnn", "lstm"])
def test_benchmark_shape_train_step_other_rnn_types(dev, rnn_type):
    """supported_rnns['rnn'] and ['lstm'] (model.py:14-15) at the benchmark shape: 5 x Bi-800,
    T = 1001 (501 recurrent steps), bs 4 with the ragged quirk lengths -- the full train step
    through the persistent fp16x3 one-gate / four-gate recurrences vs oracle.train_step, with
    the bounds and the same-mask fp64 conv check of the GRU test above, and the float64 step as
    the arbiter of recurrent gradients past 5e-4 (the LSTM's last layers: 5.2-5.6e-4)."""
    _check_train_step(dev, [1001, 877, 508, 254], [150, 120, 80, 40], seed=11, conv_fp64=True,
                      conv_tol=5e-2, rnn_type=rnn_type, rnn_fp64=True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("rnn_type", ["gru", "lstm"])
def test_benchmark_shape_train_step_unidirectional_lookahead(dev, rnn_type):
    """Unidirectional 5 x GRU / LSTM-800 with the Lookahead (context 20) + Hardtanh head of
    model.py:329-333 at the benchmark shape (T = 1001, bs 4 ragged): the full train step vs
    oracle.train_step, bounds and arbiters as above."""
    _check_train_step(dev, [1001, 877, 508, 254], [150, 120, 80, 40], seed=11, conv_fp64=True,
                      conv_tol=5e-2, rnn_type=rnn_type, rnn_fp64=True, bidirectional=False)


@pytest.mark.timeout(600)
def test_benchmark_train_step_two_batch_tiles(dev):
    """As above at bs 20: the persistent recurrences run TWO batch tiles (samples 0-15 and
    16-19, the second one partly empty) per direction, so the hand-off groups of both tiles,
    the per-tile length masks and the bias-gradient partials of both tiles are checked over
    the full 501-step BPTT against the oracle, with the same bounds."""
    t_list = [1001, 1001, 990, 950, 901, 877, 820, 760, 700, 640, 600, 508, 470, 400, 333,
              300, 254, 200, 150, 101]
    lab = [max(10, t // 7) for t in t_list]
    _check_train_step(dev, t_list, lab, seed=12, rnn_fp64='gpu')


@pytest.mark.timeout(900)
def test_benchmark_batch_train_step_matches_oracle(dev):
    """The bench's own batch (bench.py / BASELINE cfg2): bs 32, all 32 utterances 10 s
    (T = 1001 -> T' = 501), 150-label targets -- the full Trainer.train_batch (both batch tiles
    of the persistent recurrences full, the same-XCD hand-off groups, the stacked W_ih GEMMs,
    clip, SGD-Nesterov) vs oracle.train_step.  One oracle step at this shape is ~150 s on 16
    host threads.

    Loss, gradient norm, every recurrent / FC gradient and update: the bounds above.  The conv
    block (conv.*) is compared at 1e-2: its hardtanh(0, 20) derivative masks flip under
    last-bit differences -- 4 of 62.6 M between an fp32 and an fp64 forward of the oracle
    itself -- and each flip moves the block's weight / BN gradients by one position's
    contribution.  Our own two fp32-accurate paths (bf16x6 and fp32-MFMA) differ by up to
    5.5e-3 there, the oracle from either by 3.1e-3 / 5.5e-3, while every other gradient
    agrees within 4.7e-4 (scripts/bs32_probe.py, profiles/r4g_bs32_probe.txt).  With no time
    step masked, the conv biases' gradients are zero in exact arithmetic (BatchNorm follows
    each conv): both sides hold rounding noise, bounded against the conv weight gradient's
    scale."""
    _check_train_step(dev, [1001] * 32, [150] * 32, seed=13, conv_tol=1e-2, zero_conv_bias=True,
                      conv_fp64=True, rnn_fp64='gpu')


def _conv_block_grads(sd, x, out_lens, g_out, dtype, masks=None):
    """The oracle's conv block (model.py:208-215 + MaskConv + collapse) in `dtype` on the CPU,
    backpropagated from the upstream gradient g_out [T', N, 1312]: {conv param name: grad}.
    masks: the two Hardtanh derivative masks to use instead of the block's own (NCHW bool:
    where 0 < pre-activation < 20), so that a comparison measures arithmetic, not which
    near-kink positions a last-bit difference moved across 0 or 20."""
    o = orc.OracleDS2(sd, 1, 8)
    o.sd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in o.sd.items()}
    params = {k: v.clone().requires_grad_(True) for k, v in o.parameters().items()
              if k.startswith('conv.')}
    o.params = params
    if masks is None:
        y = o.conv_block(x.to(dtype), out_lens, training=True)
    else:
        it = iter(masks)
        real = torch.nn.functional.hardtanh

        def htanh_masked(v, lo, hi):   # value of hardtanh, derivative from the given mask
            mk = next(it).to(v.dtype)
            return real(v, lo, hi).detach() + mk * (v - v.detach())
        orc.F.hardtanh = htanh_masked
        try:
            y = o.conv_block(x.to(dtype), out_lens, training=True)
        finally:
            orc.F.hardtanh = real
    y.backward(g_out.to(dtype))
    return {k: v.grad for k, v in params.items()}


class _OracleF64(orc.OracleDS2):
    """The oracle with its state in float64 (its ops follow the dtype of x and the state)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.sd = {kk: (v.double() if v.is_floating_point() else v) for kk, v in self.sd.items()}


def _check_train_step(dev, t_list, label_lens, seed, conv_tol=5e-4, zero_conv_bias=False,
                      conv_fp64=False, rnn_type='gru', rnn_fp64=False, bidirectional=True):
    """rnn_fp64: a recurrent / FC gradient past 5e-4 from the fp32 oracle still passes when it
    sits within 1.25x (+1e-5) of the fp32 oracle's own distance from the same step in float64
    (the oracle's state and input in float64): both are fp32 approximations of one exact
    step, and over 501 recurrent steps the reference's own fp32 drifts.  The float64 step runs
    only when some gradient is past 5e-4; rnn_fp64='gpu' runs it on the GPU (the oracle's own
    torch ops in float64: no MIOpen path takes float64, so torch's native kernels run them;
    the bs-32 step, ~150 s per fp32 oracle step on the host, would take minutes in float64
    there)."""
    _threads()
    g = torch.Generator().manual_seed(seed)
    x = _spect_batch(g, t_list, 1001)
    pct = torch.tensor([t / 1001.0 for t in t_list], dtype=torch.float32)
    tg, tl = _targets(g, label_lens)
    m = _build(123456, 800, 5, rnn_type=rnn_type, bidirectional=bidirectional)
    o = orc.OracleDS2({k: v.detach().clone() for k, v in m.state_dict().items()}, 5, 800,
                      rnn_type=rnn_type, bidirectional=bidirectional)
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    captured = {}
    if conv_fp64:
        # the gradient our recurrent stack hands the conv block and our two conv blocks'
        # outputs (their Hardtanh masks), for the fp64 check below
        orig = m.conv.forward_collapsed
        orig_apply = ops.ConvBlockFn.apply
        outs = []

        def rec_apply(*a):
            y = orig_apply(*a)
            outs.append(y.detach())
            return y

        def tapped(xx, lens):
            y = orig(xx, lens)
            y.register_hook(lambda gr: captured.__setitem__('g', gr.detach().cpu().clone()))
            return y
        m.conv.forward_collapsed = tapped
        ops.ConvBlockFn.apply = rec_apply
    try:
        tr = Trainer(m, LABELS, lr=3e-4, momentum=0.9, max_norm=100.0, device=dev)
        loss = tr.train_batch((x, tg, None, pct.clone(), tl), return_item=True)
    finally:
        if conv_fp64:
            del ops.ConvBlockFn.apply    # back to the inherited Function.apply
    if conv_fp64:
        # VERDICT r4 #5a: the conv block's arithmetic against fp64 on the SAME upstream
        # gradient (ours) and the SAME Hardtanh masks (ours: 0 < y < 20 of our two block
        # outputs), so the kinks a last-bit difference moves (1 + 3 of 63 M positions between
        # an fp32 and an fp64 forward, profiles/r4g_bs32_probe.txt) drop out of both sides:
        # our conv gradients may be at most 1.25x as far from that fp64 block as the fp32 oracle
        # block (same masks) is, with a 1e-6 floor.  Measured with each block's own masks
        # instead, ours sat at 8.3e-4 of conv1.weight's max against the fp32 oracle's 2.8e-4:
        # flips, not arithmetic.
        t_, n_ = captured['g'].shape[:2]
        m1 = (outs[0] > 0) & (outs[0] < 20)
        y2 = outs[1].view(t_, n_, 32, -1).permute(1, 2, 3, 0)
        m2 = (y2 > 0) & (y2 < 20)
        masks = (m1.cpu(), m2.cpu())
        del outs
        out_lens = orc.get_seq_lens(orc.input_sizes_quirk(pct, 1001))
        # how many Hardtanh derivative masks our forward moved against the fp32 oracle's
        oc = orc.OracleDS2(sd0, 1, 8)
        oc.params = oc.parameters()
        acts = {}
        with torch.no_grad():
            oc.conv_block(x, out_lens, training=True, acts=acts)
        om2 = acts['conv2']
        print("conv Hardtanh mask flips vs the fp32 oracle's forward: conv1",
              int(((acts['conv1'] > 0) & (acts['conv1'] < 20) != masks[0]).sum()), "conv2",
              int(((om2 > 0) & (om2 < 20) != masks[1]).sum()), "of", masks[0].numel(),
              "+", masks[1].numel())
        del acts, om2
        g64 = _conv_block_grads(sd0, x, out_lens, captured['g'], torch.float64, masks)
        g32 = _conv_block_grads(sd0, x, out_lens, captured['g'], torch.float32, masks)
        bad = []
        for name, p in m.named_parameters():
            if not name.startswith('conv.') or (zero_conv_bias and name.endswith('.bias')
                                                and p.dim() == 1 and name.replace('.bias', '.weight') in g64
                                                and g64[name.replace('.bias', '.weight')].dim() == 4):
                continue
            ref = g64[name]
            ours = _rel(p.grad, ref)
            own = _rel(g32[name], ref)
            print(f"conv fp64 check {name}: ours {ours:.2e} fp32 oracle {own:.2e}")
            if ours > 1.25 * own + 1e-6:
                bad.append((name, ours, own))
    else:
        bad = []
    # (the conv fp64 verdict is asserted after the oracle comparison, so one run prints both)
    rloss, rnew, _, rgrads, rnorm = orc.train_step(o, x, pct.clone(), tg, tl)
    assert abs(loss - float(rloss)) <= 1e-4 * abs(float(rloss))
    g64 = n64 = None
    past = [name for name, p in m.named_parameters()
            if not name.startswith('conv.') and _rel(p.grad, rgrads[name]) > 5e-4]
    norm = float(tr.optimizer.norm.item())
    norm_off = abs(norm - float(rnorm)) > 2e-4 * float(rnorm)
    if rnn_fp64 and (past or norm_off):
        where = dev if rnn_fp64 == 'gpu' else torch.device('cpu')
        o64 = _OracleF64({k: v.detach().clone() for k, v in sd0.items()}, 5, 800, rnn_type=rnn_type,
                         bidirectional=bidirectional)
        o64.sd = {k: v.to(where) for k, v in o64.sd.items()}
        _, _, _, g64, n64 = orc.train_step(o64, x.double().to(where), pct.clone(), tg, tl)
        g64 = {k: v.cpu() for k, v in g64.items()}
        n64 = float(n64)
    # the clip norm within 2e-4 of the oracle's, or (rnn_fp64) no farther from the float64
    # step's than 1.25x the oracle's own distance (+1e-5 relative).  The oracle's CTC is torch's
    # CPU ctc_loss in fp32: log-space alpha / beta of magnitude ~|log p| (~1.5e3 at T' = 501)
    # put ~7e-4 (max-abs / max-abs) on its CTC gradient at the bench length, where our
    # rescaled scans sit at 5e-5 (test_ctc_rescaled_scan_at_the_benchmark_length); before
    # them our norm sat ~1e-4 from the oracle's through the same effect
    # (profiles/r4i_bs4_norm_probe.txt).
    if n64 is not None and norm_off:
        print(f"fp64 check clip norm: ours {abs(norm - n64) / n64:.2e} "
              f"fp32 oracle {abs(float(rnorm) - n64) / n64:.2e}")
        assert abs(norm - n64) <= 1.25 * abs(float(rnorm) - n64) + 1e-5 * n64
    else:
        assert not norm_off, (norm, float(rnorm))
    worst = {}
    bad_grads = []
    for name, p in m.named_parameters():
        tol = conv_tol if name.startswith('conv.') else 5e-4
        d = p.detach().cpu() - before[name]
        rd = rnew[name] - before[name]
        ulp = torch.finfo(torch.float32).eps * before[name].abs().max().item()
        if zero_conv_bias and name.startswith('conv.') and name.endswith('.bias') \
                and name.replace('.bias', '.weight') in rgrads \
                and p.dim() == 1 and rgrads[name.replace('.bias', '.weight')].dim() == 4:
            # a conv bias (BatchNorm follows): zero up to rounding on both sides
            scale = torch.as_tensor(rgrads[name.replace('.bias', '.weight')]).abs().max().item()
            err = (p.grad.detach().double().cpu() - torch.as_tensor(rgrads[name]).double()).abs().max().item()
            worst[name] = err / scale
            if worst[name] > 5e-4:
                bad_grads.append((name, worst[name]))
            continue
        worst[name] = _rel(p.grad, rgrads[name])
        exact_ok = False
        if g64 is not None and not name.startswith('conv.') and worst[name] > tol:
            ours64, own64 = _rel(p.grad, g64[name]), _rel(rgrads[name], g64[name])
            exact_ok = ours64 <= 1.25 * own64 + 1e-5
            print(f"fp64 check {name}: ours {ours64:.2e} fp32 oracle {own64:.2e}")
        if worst[name] > tol and not exact_ok:
            bad_grads.append((name, worst[name]))
        # the update itself (p_new - p_old), not just p_new (dominated by p_old); both
        # differences carry the float32 rounding of p_new (half an ulp of |p| each)
        if (d - rd).abs().max().item() > tol * rd.abs().max().item() + ulp and not exact_ok:
            bad_grads.append((name, 'update'))
    print("gradient distances from the oracle (max-abs / max-abs), largest first:",
          sorted(((round(v, 7), k) for k, v in worst.items()), reverse=True)[:12])
    assert not bad_grads, bad_grads
    assert not bad, bad
    for k, v in m.state_dict().items():
        if 'running' in k:
            assert _rel(v, o.sd[k]) <= 1e-5, k


def test_benchmark_bs32_forward_matches_oracle(dev):
    """The benchmark batch itself (bs 32, 10 s, equal lengths), train-mode forward without
    grad: logits and probs within 1e-4, output lengths exact, BN running stats 1e-5."""
    _threads()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(32, 1, 161, 1001, generator=g)
    sizes = torch.full((32,), 1001, dtype=torch.int32)
    m = _build(123456, 800, 5).to(dev).train()
    o = orc.OracleDS2({k: v.detach().cpu().clone() for k, v in m.state_dict().items()}, 5, 800)
    with torch.no_grad():
        logits, probs, out_lens = m(x.to(dev), sizes)
        rl, rp, ro, _ = o.forward(x, sizes, training=True)
    np.testing.assert_array_equal(out_lens.cpu().numpy(), ro.numpy())
    assert _rel(logits, rl) < 1e-4
    assert _rel(probs, rp) < 1e-4
    for k, v in m.state_dict().items():
        if 'running' in k:
            assert _rel(v, o.sd[k]) <= 1e-5, k


# --------------------------------------------------------------------------- failure semantics
def test_nan_logits_zeroed_and_step_taken_like_reference(dev, golden_dir):
    """train.py:595-598,625: NaN logits are zeroed in place (zero gradient there) and the
    SGD step is taken -- post-step parameters equal the oracle's with the same planted NaNs;
    the reference's warning is counted (printed lazily, no per-step host sync)."""
    g = np.load(os.path.join(golden_dir, 'tiny_ds2.npz'))
    m = _build(int(g['seed']), int(g['hidden']), int(g['layers']))
    o = orc.OracleDS2({k: v.detach().clone() for k, v in m.state_dict().items()}, 2, 16)
    x = torch.from_numpy(g['x'])
    n, t = x.shape[0], int(g['out_lens'].max())
    plant = torch.zeros(n, t, len(LABELS), dtype=torch.bool)
    plant[0, 3, 5] = plant[1, 10, 0] = plant[2, 7, 29] = plant[0, 20, 11] = True

    def hook(mod, inp, out):          # the FC output [T', N, C] of the HIP model
        out = out.clone()
        out[plant.transpose(0, 1).to(out.device)] = float('nan')
        return out

    m.fc.register_forward_hook(hook)
    tr = Trainer(m, LABELS, lr=3e-4, momentum=0.9, max_norm=100.0, device=dev, verbose=False)
    data = (x, torch.from_numpy(g['targets']), None, torch.from_numpy(g['pct']).clone(),
            torch.from_numpy(g['target_sizes']))
    loss = tr.train_batch(data, return_item=True)
    rloss, rnew, _, _, _ = orc.train_step(o, x, torch.from_numpy(g['pct']).clone(),
                                          torch.from_numpy(g['targets']),
                                          torch.from_numpy(g['target_sizes']), plant_nan=plant)
    assert np.isfinite(loss)
    assert abs(loss - float(rloss)) <= 1e-4 * abs(float(rloss))
    assert tr.warnings['nan'] == 1
    for name, p in m.named_parameters():
        ref = rnew[name]
        assert torch.isfinite(p).all().item(), name
        assert (p.detach().cpu() - ref).abs().max().item() <= 1e-6 + 1e-5 * ref.abs().max().item(), name


def test_rnn_handoff_timeout_raises(dev, monkeypatch):
    """A persistent recurrence whose hand-off times out (spin bound forced to 0 through
    DS2_RNN_SPIN_LIMIT) must raise Ds2Error from the Trainer, not turn into a silently
    NaN-zeroed step; with the bound restored the same step runs clean."""
    g = torch.Generator().manual_seed(2)
    x = torch.randn(32, 1, 161, 301, generator=g)
    tg, tl = _targets(g, [20] * 32)
    pct = torch.ones(32)
    ops.rnn_status_word(dev).zero_()
    monkeypatch.setenv("DS2_RNN_SPIN_LIMIT", "0")
    monkeypatch.setenv("DS2_RNN_TUNE", "1,0")   # poll at once: early polls must find stale tiles
    tr = Trainer(_build(3, 256, 2), LABELS, device=dev, verbose=False)
    p0, m0 = tr.flat.flat.clone(), tr.optimizer.buf.clone()
    with pytest.raises(_lib.Ds2Error, match="hand-off"):
        tr.train_batch((x, tg, None, pct.clone(), tl), return_item=True)
    # the failed step's update was skipped on the device: parameters and momentum intact
    assert torch.isfinite(tr.flat.flat).all() and torch.isfinite(tr.optimizer.buf).all()
    assert torch.equal(tr.flat.flat, p0) and torch.equal(tr.optimizer.buf, m0)
    # the op-level query sees it too
    lens = torch.full((32,), 151, dtype=torch.int32, device=dev)
    xs = torch.randn(151, 32, 256, device=dev)
    layer = dsm.GRU(256, 256, bidirectional=True).to(dev)
    with torch.no_grad():
        layer.run(xs, lens)
    with pytest.raises(_lib.Ds2Error, match="hand-off"):
        ops.check_rnn_status(dev)
    monkeypatch.delenv("DS2_RNN_SPIN_LIMIT")
    monkeypatch.delenv("DS2_RNN_TUNE")
    tr2 = Trainer(_build(3, 256, 2), LABELS, device=dev, verbose=False)
    v = tr2.train_batch((x, tg, None, pct.clone(), tl), return_item=True)
    assert np.isfinite(v)
    ops.check_rnn_status(dev)          # clean


# --------------------------------------------------------------------------- resume
def test_resume_from_reference_package(dev, golden_dir):
    """train.py:827-844: a package written by the reference's serialize after one SGD step
    (weights, BN buffers, torch.optim.SGD state) resumes here; the second step matches the
    reference's second step (loss, every parameter) and the momentum it leaves behind."""
    pkg = torch.load(os.path.join(golden_dir, 'tiny_ref_resume.pth'), map_location='cpu',
                     weights_only=True)
    g0 = np.load(os.path.join(golden_dir, 'tiny_ds2.npz'))
    g2 = np.load(os.path.join(golden_dir, 'tiny_resume.npz'))
    m = dsm.DeepSpeech.load_model_package(pkg)
    tr = Trainer(m, LABELS, lr=1.0, momentum=0.5, max_norm=100.0, device=dev)
    tr.optimizer.load_state_dict(pkg['optim_dict'])
    data = (torch.from_numpy(g0['x']), torch.from_numpy(g0['targets']), None,
            torch.from_numpy(g0['pct']).clone(), torch.from_numpy(g0['target_sizes']))
    loss = tr.train_batch(data, return_item=True)
    assert abs(loss - float(g2['loss2'])) <= 1e-4 * abs(float(g2['loss2']))
    sd = m.state_dict()
    for k in g2.files:
        if k.startswith('after_step2/'):
            name = k[len('after_step2/'):]
            ref = torch.from_numpy(g2[k])
            assert (sd[name].cpu() - ref).abs().max().item() <= 1e-6 + 1e-5 * ref.abs().max().item(), name
    st = tr.optimizer.state_dict()['state']
    for i in range(len(st)):
        assert _rel(st[i]['momentum_buffer'], g2[f'momentum2/{i}']) <= 1e-4, i


# --------------------------------------------------------------------------- data parallel
@pytest.mark.parametrize("allreduce", ["torch", "ds2"])
def test_world1_nccl_trainer_hooks_and_bit_identity(dev, golden_dir, tmp_path, monkeypatch,
                                                    allreduce):
    """The DS2 Trainer under a world-1 RCCL ('nccl') process group: every gradient bucket's
    all-reduce is issued from the post-accumulate hooks during backward, the reduced
    gradients (HIP gradient slots in the flat buffer) are bit-identical to the
    no-process-group Trainer's, and the step is the same.  allreduce='ds2': the buckets go
    through the C ABI's own RCCL communicator (ds2_comm_init / ds2_allreduce_bucket on a
    side stream) instead of torch.distributed."""
    import torch.distributed as dist
    monkeypatch.setenv("DS2_ALLREDUCE", allreduce)
    g = np.load(os.path.join(golden_dir, 'tiny_ds2.npz'))

    def data():
        return (torch.from_numpy(g['x']), torch.from_numpy(g['targets']), None,
                torch.from_numpy(g['pct']).clone(), torch.from_numpy(g['target_sizes']))

    ref = Trainer(_build(int(g['seed']), 16, 2), LABELS, device=dev, bucket_mb=0.05)
    ref.train_batch(data(), return_item=True)
    ref_grad = ref.flat.grad.clone()
    ref_params = ref.flat.flat.clone()
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        tr = Trainer(_build(int(g['seed']), 16, 2), LABELS, device=dev, bucket_mb=0.05)
        assert len(tr.reducer.buckets) > 1 and tr.reducer._hooks
        assert (tr.reducer.comm is not None) == (allreduce == "ds2")
        loss = tr.train_batch(data(), return_item=True)
        assert tr.reducer.issued_from_hooks == len(tr.reducer.buckets)
        # one collective per bucket: the status word and the loss rode in the last one
        assert tr.reducer.collectives == len(tr.reducer.buckets)
        nparam = tr.flat.numel
        assert torch.equal(tr.flat.grad[:nparam], ref_grad)
        assert tr.flat.tail.tolist() == [0.0, loss]     # status word 0, the loss itself
        assert torch.equal(tr.flat.flat, ref_params)
        tr.close()
        assert tr.reducer.comm is None
    finally:
        ops.set_cooperative_guard(None)
        dist.destroy_process_group()


def _dp_batch(rank):
    """The world-2 test's 4-utterance batch (2 per rank), as the collate function gives it."""
    g = torch.Generator().manual_seed(77)
    x = _spect_batch(g, [64, 60, 52, 40], 64)
    targets, tsz = _targets(g, [9, 7, 6, 4])
    pct = torch.tensor([64, 60, 52, 40], dtype=torch.float32) / 64
    lo, hi = 2 * rank, 2 * rank + 2
    off = int(tsz[:lo].sum())
    return (x[lo:hi].clone(), targets[off:off + int(tsz[lo:hi].sum())].clone(), None,
            pct[lo:hi].clone(), tsz[lo:hi].clone())


def _dp_worker(rank, world, port, out_q):
    """One rank of test_world2_gloo_hip_trainer: the HIP Trainer on cuda:0 under a gloo process
    group (device tensors), two steps on its half of the batch."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = Trainer(_build(1234, 32, 2), LABELS, device=dev, bucket_mb=0.05)
        nparam = tr.flat.numel
        out = {"buckets": len(tr.reducer.buckets), "hooks": bool(tr.reducer._hooks),
               "bcast0": tr.sync.broadcasts, "steps": []}
        for step in range(2):
            loss = tr.train_batch(_dp_batch(rank), return_item=True)
            rec = {"loss": loss, "grad": tr.flat.grad[:nparam].cpu().numpy().copy(),
                   "tail": tr.flat.tail.cpu().tolist(),
                   "params": tr.flat.flat[:nparam].cpu().numpy().copy(),
                   "issued": tr.reducer.issued_from_hooks, "colls": tr.reducer.collectives,
                   "bufs_before": tr.sync.flat_buffers.cpu().numpy().copy()}
            # DDP's broadcast_buffers: the next forward starts from rank 0's BN running stats
            tr.sync.before_forward()
            rec["bufs_after"] = tr.sync.flat_buffers.cpu().numpy().copy()
            rec["bcast"] = tr.sync.broadcasts
            out["steps"].append(rec)
        torch.cuda.synchronize()
        out_q.put((rank, out))
    finally:
        ops.set_cooperative_guard(None)
        dist.destroy_process_group()


def test_world2_gloo_hip_trainer(dev):
    """the HIP Trainer at world 2 -- two spawned processes on cuda:0, a gloo
    process group carrying the device gradient buckets (the closest to cfg3 one GPU allows;
    train.py:804-809, 947-951, data/utils.py:40-44).  Each rank steps a 2-layer BiGRU-32 DS2
    on its 2 utterances.  Checked against single-process Trainers on each half: the reduced
    gradient equals (g0 + g1) / 2 bit for bit (DDP's average; BatchNorm statistics stay local
    as in DDP), every bucket's all-reduce was issued from the backward hooks, one collective
    per bucket (the status flag and the loss ride in the last one's tail: flag 0, the mean of
    the two ranks' losses), the parameters agree across ranks after both steps, and rank 0's
    BN running statistics reach rank 1 before the next forward."""
    import torch.multiprocessing as mp
    import socket
    refs = []
    for r in range(2):
        tr = Trainer(_build(1234, 32, 2), LABELS, device=dev, bucket_mb=0.05)
        lr = tr.train_batch(_dp_batch(r), return_item=True)
        refs.append((lr, tr.flat.grad[:tr.flat.numel].cpu().clone()))
    want = ((refs[0][1] + refs[1][1]) * 0.5).numpy()
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    for r in range(2):
        o = res[r]
        assert o["hooks"] and o["buckets"] > 1
        for k, st in enumerate(o["steps"]):
            assert st["issued"] == o["buckets"], "every bucket issued from a backward hook"
            assert st["colls"] == o["buckets"], "one collective per bucket"
            assert st["tail"][0] == 0.0, "status flag clean"
            assert st["tail"][1] == st["loss"], "the returned loss is the tail's mean"
            assert st["loss"] == res[1 - r]["steps"][k]["loss"]
            assert st["bcast"] == o["bcast0"] + 2 * k + 2
            np.testing.assert_array_equal(st["bufs_after"], res[0]["steps"][k]["bufs_before"])
        np.testing.assert_array_equal(o["steps"][0]["grad"], want)
        # reduce_tensor: the mean of the two ranks' batch-mean losses
        assert o["steps"][0]["loss"] == pytest.approx((refs[0][0] + refs[1][0]) / 2, rel=1e-6)
    for k in range(2):
        np.testing.assert_array_equal(res[0]["steps"][k]["params"], res[1]["steps"][k]["params"])
        np.testing.assert_array_equal(res[0]["steps"][k]["grad"], res[1]["steps"][k]["grad"])
    # local BN: the two ranks' running statistics differ after a step, until the broadcast
    assert not np.array_equal(res[0]["steps"][0]["bufs_before"], res[1]["steps"][0]["bufs_before"])


# --------------------------------------------------------------------------- cfg4 / cfg5 shapes
def test_cfg5_30s_eval_forward_and_beam10(dev):
    """cfg5's defining shape: 30 s utterances (T = 3001, T' = 1501) through 5 x BiGRU-800 in
    eval mode, bs 2, against the oracle; then the beam-10 prefix search on those probs
    against the oracle/ctc_beam.py restatement (ids and offsets of every path)."""
    _threads()
    from ds2amd.decoder import BeamCTCDecoder
    from oracle import ctc_beam
    g = torch.Generator().manual_seed(30)
    t_list = [3001, 2400]
    x = _spect_batch(g, t_list, 3001)
    sizes = torch.tensor(t_list, dtype=torch.int32)
    m = _build(123456, 800, 5).to(dev).eval()
    o = orc.OracleDS2({k: v.detach().cpu().clone() for k, v in m.state_dict().items()}, 5, 800)
    with torch.no_grad():
        logits, probs, out_lens = m(x.to(dev), sizes)
        rl, rp, ro, _ = o.forward(x, sizes, training=False)
    np.testing.assert_array_equal(out_lens.cpu().numpy(), ro.numpy())
    assert out_lens.tolist() == [1501, 1200]
    assert _rel(logits, rl) < 1e-4
    beam = BeamCTCDecoder(LABELS, beam_width=10, cutoff_top_n=40)
    strings, offsets = beam.decode(probs, out_lens)
    ref = ctc_beam.beam_decode(probs.cpu().numpy(), out_lens.cpu().tolist(), 10)
    for i, paths in enumerate(ref):
        for p, (_, ids, ts) in enumerate(paths):
            assert strings[i][p] == ''.join(LABELS[k] for k in ids)
            assert offsets[i][p].tolist() == ts
    # the same search with the committed word 3-gram LM (ctcdecode's KenLM scorer restated,
    # oracle/ctc_beam_lm.py) over the 1501 frames: every path and its frames
    from oracle import ctc_beam_lm
    lm_path = os.path.join(os.path.dirname(__file__), "golden", "tiny_lm.arpa")
    beam = BeamCTCDecoder(LABELS, lm_path=lm_path, alpha=0.8, beta=1.0, beam_width=10,
                          cutoff_top_n=40)
    strings, offsets = beam.decode(probs, out_lens)
    ref = ctc_beam_lm.beam_decode_lm(probs.cpu().numpy(), out_lens.cpu().tolist(), 10,
                                     ctc_beam_lm.ArpaLM(lm_path), LABELS, 0.8, 1.0)
    for i, paths in enumerate(ref):
        for p, (_, ids, ts) in enumerate(paths):
            assert strings[i][p] == ''.join(LABELS[k] for k in ids), (i, p)
            assert offsets[i][p].tolist() == ts


def test_cfg4_lstm1024_bf16_gemms_and_batch64_chunks(dev):
    """cfg4's layer (BiLSTM-1024): (a) batch 64 in fp32 -- the persistent kernels' 32-sample
    workgroups / two-chunk backward -- forward + input gradient vs the oracle; (b) the opt-in
    bf16 RNN GEMMs at H = 1024 over a 3-layer stack track the fp32 oracle (logits 2e-2,
    loss 1 %)."""
    _threads()
    from ds2amd.ctc import CTCLoss
    g = torch.Generator().manual_seed(64)
    t_list = [161] * 40 + [140] * 24
    x = _spect_batch(g, t_list, 161)
    sizes = torch.tensor(t_list, dtype=torch.int32)
    m = _build(77, 1024, 2, rnn_type='lstm').to(dev).train()
    o = orc.OracleDS2({k: v.detach().cpu().clone() for k, v in m.state_dict().items()}, 2, 1024,
                      rnn_type='lstm')
    tg, tl = _targets(g, [20] * 64)
    logits, _, out_lens = m(x.to(dev), sizes)
    loss = CTCLoss()(logits.transpose(0, 1), tg, out_lens, tl) / 64
    loss.backward()
    params = {k: v.detach().clone().requires_grad_(True) for k, v in o.parameters().items()}
    rl, _, ro, _ = o.forward(x, sizes, training=True, params=params)
    rloss = torch.nn.functional.ctc_loss(rl.transpose(0, 1).log_softmax(2), tg.long(), ro.long(),
                                         tl.long(), reduction='sum') / 64
    rloss.backward()
    assert _rel(logits, rl) < 1e-4
    assert abs(float(loss) - float(rloss)) <= 1e-4 * abs(float(rloss))
    for name, p in m.named_parameters():
        if name.startswith('rnns.'):
            assert _rel(p.grad, params[name].grad) <= 5e-4, name
    # (b) bf16 RNN GEMMs, 3 layers at H = 1024
    m32 = _build(78, 1024, 3, rnn_type='lstm').to(dev).train()
    m16 = _build(78, 1024, 3, rnn_type='lstm').to(dev).train()
    m16.set_rnn_gemm_precision('bf16')
    o3 = orc.OracleDS2({k: v.detach().cpu().clone() for k, v in m32.state_dict().items()}, 3,
                       1024, rnn_type='lstm')
    xb, sb = x[:4], sizes[:4]
    with torch.no_grad():
        l32, _, ol = m32(xb.to(dev), sb)
        l16, _, _ = m16(xb.to(dev), sb)
        rl3, _, _, _ = o3.forward(xb, sb, training=True)
    assert _rel(l32, rl3) < 1e-4
    assert _rel(l16, rl3) < 2e-2
    c32 = CTCLoss()(l32.transpose(0, 1).contiguous(), tg[:80], ol, tl[:4])
    c16 = CTCLoss()(l16.transpose(0, 1).contiguous(), tg[:80], ol, tl[:4])
    assert abs(float(c16) - float(c32)) <= 1e-2 * abs(float(c32))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("bidir", [True, False])
def test_cfg4_full_shape_bf16_step(dev, bidir):
    """BASELINE cfg4 at its own shape (VERDICT r4 #5b): 7 x BiLSTM-1024, batch 64, 10 s
    (T = 1001 -> T' = 501), the opt-in bf16 RNN GEMMs, through Trainer.train_batch (forward,
    CTC, BPTT, clip, SGD-Nesterov): every gradient finite; deterministic (the same step from
    the same state twice: loss, gradients and updated parameters bit-identical); the loss
    within 1 % of the fp32 HIP path's on the same batch; and a 2-layer slice of the same
    weights (conv, rnns.0-1, fc) in bf16 mode against the fp32 oracle forward at full length
    (logits 2e-2, CTC loss 1 %, the existing bf16 bounds).  bidir=False: cfg4's
    unidirectional variant, 7 x LSTM-1024 + Lookahead (+ Hardtanh) before the FC
    (model.py:140-177, 329-333; VERDICT r5 missing #4), same checks."""
    _threads()
    from ds2amd.ctc import CTCLoss
    g = torch.Generator().manual_seed(404)
    x = _spect_batch(g, [1001] * 64, 1001)
    pct = torch.ones(64)
    tg, tl = _targets(g, [150] * 64)
    m0 = _build(4040, 1024, 7, rnn_type='lstm', bidirectional=bidir)
    sd0 = {k: v.detach().clone() for k, v in m0.state_dict().items()}

    def step(precision):
        m = _build(4040, 1024, 7, rnn_type='lstm', bidirectional=bidir)
        m.load_state_dict(sd0)
        if precision == 'bf16':
            m.set_rnn_gemm_precision('bf16')
        tr = Trainer(m, LABELS, lr=3e-4, momentum=0.9, max_norm=400.0, device=dev, verbose=False)
        loss = tr.train_batch((x, tg, None, pct.clone(), tl), return_item=True)
        torch.cuda.synchronize()
        out = (loss, tr.flat.grad[:tr.flat.numel].clone(), tr.flat.flat.clone())
        del tr, m
        return out

    l16a, g16a, p16a = step('bf16')
    assert np.isfinite(l16a) and torch.isfinite(g16a).all().item()
    l16b, g16b, p16b = step('bf16')
    assert l16a == l16b and torch.equal(g16a, g16b) and torch.equal(p16a, p16b)
    del g16b, p16b
    l32, g32, _ = step('fp32')
    assert abs(l16a - l32) <= 1e-2 * abs(l32), (l16a, l32)
    # the bf16 products move the gradients by about their own rounding, not more
    assert (g16a - g32).norm().item() <= 5e-2 * g32.norm().item()
    del g16a, g32, p16a
    # 2-layer slice vs the fp32 oracle, 4 utterances at full length
    m2 = _build(4040, 1024, 2, rnn_type='lstm', bidirectional=bidir)
    m2.load_state_dict({k: v for k, v in sd0.items() if k in m2.state_dict()})
    m2 = m2.to(dev).train()
    m2.set_rnn_gemm_precision('bf16')
    o2 = orc.OracleDS2({k: v.detach().cpu().clone() for k, v in m2.state_dict().items()}, 2,
                       1024, rnn_type='lstm', bidirectional=bidir)
    xb, sb = x[:4], torch.full((4,), 1001, dtype=torch.int32)
    with torch.no_grad():
        l2, _, ol = m2(xb.to(dev), sb)
        rl2, _, ro, _ = o2.forward(xb, sb, training=True)
    assert ol.cpu().tolist() == ro.tolist() == [501] * 4
    assert _rel(l2, rl2) < 2e-2
    c16 = CTCLoss()(l2.transpose(0, 1).contiguous(), tg[:600], ol, tl[:4])
    rc = torch.nn.functional.ctc_loss(rl2.transpose(0, 1).log_softmax(2), tg[:600].long(),
                                      ro.long(), tl[:4].long(), reduction='sum')
    assert abs(float(c16) - float(rc)) <= 1e-2 * abs(float(rc))
