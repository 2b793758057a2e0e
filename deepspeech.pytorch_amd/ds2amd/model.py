"""DeepSpeech2 model — drop-in for the reference ``model.py`` (DS2 branch).

Same constructor, same module tree and state_dict keys (so reference
checkpoints load), same ``forward(x, lengths) -> (logits, probs, out_lens)``
contract (ref model.py:183-393), but every op on the forward/backward path is a
hand-written HIP kernel from libds2hip (see ds2amd/ops.py).

Parameter holders reuse torch.nn classes (nn.Conv2d, nn.BatchNorm*, nn.Linear)
purely for their parameters/buffers/initialisers; their own forward (MIOpen /
rocBLAS) is never called on this path.  Constructing the model under the same
seed draws exactly the same initial weights as the reference.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn as nn
from torch.nn.utils.rnn import PackedSequence, pack_padded_sequence, pad_packed_sequence

from . import ops


# ----------------------------------------------------------------------------
# RNN op seam (ref model.py:13-25 supported_rnns)
class _HipRNN(nn.Module):
    """Single-layer (bi)directional recurrent layer with nn.GRU / nn.LSTM's parameter
    names, order and init.

    ``forward(x, lengths)`` takes padded [T, N, In] + int lengths (sorted or not)
    and returns padded [T, N, D*H]; a PackedSequence input is also accepted and
    answered with a PackedSequence, like the torch modules.
    """
    GATES = 0
    FN = None
    # precision of this layer's GEMMs: 'fp32' (reference parity) or 'bf16' (BASELINE cfg4's
    # opt-in bf16 MFMA RNN GEMMs; the recurrence itself stays fp32).  Not a parameter or
    # buffer: state_dicts are unchanged.
    gemm_precision = 'fp32'

    def __init__(self, input_size, hidden_size, bidirectional=False, bias=True, num_layers=1):
        super().__init__()
        if num_layers != 1 or not bias:
            raise ValueError(f"ds2amd.{type(self).__name__} supports num_layers=1, bias=True "
                             "(what BatchRNN builds)")
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.bidirectional = bidirectional
        self.num_directions = 2 if bidirectional else 1
        g = self.GATES * hidden_size
        for sfx in [""] + (["_reverse"] if bidirectional else []):
            self.register_parameter("weight_ih_l0" + sfx, nn.Parameter(torch.empty(g, input_size)))
            self.register_parameter("weight_hh_l0" + sfx, nn.Parameter(torch.empty(g, hidden_size)))
            self.register_parameter("bias_ih_l0" + sfx, nn.Parameter(torch.empty(g)))
            self.register_parameter("bias_hh_l0" + sfx, nn.Parameter(torch.empty(g)))
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.hidden_size)
        for w in self.parameters():
            nn.init.uniform_(w, -stdv, stdv)

    def flatten_parameters(self):  # API parity with nn.GRU/nn.LSTM (model.py:94-95)
        return None

    def _weights(self):
        ws = [self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0, self.bias_hh_l0]
        if self.bidirectional:
            ws += [self.weight_ih_l0_reverse, self.weight_hh_l0_reverse, self.bias_ih_l0_reverse,
                   self.bias_hh_l0_reverse]
        return ws

    def run(self, x, lens_dev, sum_dirs=False):
        with ops.rnn_gemm_precision(self.gemm_precision):
            return self.FN.apply(x, lens_dev, sum_dirs, self.hidden_size, *self._weights())

    def forward(self, x, lengths=None):
        if isinstance(x, PackedSequence):
            padded, lens = pad_packed_sequence(x)
            out = self.run(padded, lens.to(padded.device, torch.int32))
            return pack_padded_sequence(out, lens, enforce_sorted=False), None
        if lengths is None:
            lengths = torch.full((x.shape[1],), x.shape[0], dtype=torch.int32)
        return self.run(x, lengths.to(x.device, torch.int32)), None


class GRU(_HipRNN):
    """nn.GRU drop-in (gates r, z, n) on the HIP recurrence kernels (gru.hip)."""
    GATES = 3
    FN = ops.GRULayerFn


class LSTM(_HipRNN):
    """nn.LSTM drop-in (gates i, f, g, o) on the HIP recurrence kernels (lstm.hip)."""
    GATES = 4
    FN = ops.LSTMLayerFn


class RNN(_HipRNN):
    """nn.RNN drop-in (tanh, the reference's rnn_type 'rnn') on the HIP recurrence (rnn.hip)."""
    GATES = 1
    FN = ops.RNNLayerFn


supported_rnns = {
    'lstm': LSTM,
    'rnn': RNN,
    'gru': GRU,
}
supported_rnns_inv = dict((v, k) for k, v in supported_rnns.items())


# ----------------------------------------------------------------------------
class BatchNorm1d(nn.BatchNorm1d):
    """nn.BatchNorm1d parameters; forward on [R, C] through the HIP kernels."""

    def forward(self, x):
        if x.dim() != 2:
            raise ValueError("ds2amd.BatchNorm1d expects [R, C] (SequenceWise view)")
        training = self.training or not self.track_running_stats
        if self.training and self.track_running_stats:
            self.num_batches_tracked.add_(1)
        return ops.SeqBatchNormFn.apply(x, self.weight, self.bias, self.running_mean,
                                        self.running_var, training, self.momentum, self.eps)


class Linear(nn.Linear):
    def forward(self, x):
        y = ops.LinearFn.apply(x, self.weight)
        if self.bias is not None:
            y = y + self.bias
        return y


class SequenceWise(nn.Module):
    """Collapses T*N*H to (T*N)*H and applies the module (ref model.py:28-49)."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def forward(self, x):
        t, n = x.size(0), x.size(1)
        x = x.reshape(t * n, -1)
        x = self.module(x)
        return x.view(t, n, -1)

    def __repr__(self):
        return self.__class__.__name__ + ' (\n' + self.module.__repr__() + ')'


class MaskConv(nn.Module):
    """Conv stack with the length mask after every module (ref model.py:52-79).

    The (Conv2d, BatchNorm2d, Hardtanh) triples run as one fused HIP pipeline:
    implicit-GEMM conv with masked epilogue, batch statistics, then
    BN + mask + Hardtanh + mask (+ the T x N x (C*D) collapse for the last
    triple when called through ``forward_collapsed``).
    """

    def __init__(self, seq_module):
        super().__init__()
        self.seq_module = seq_module
        mods = list(seq_module)
        if len(mods) % 3 != 0:
            raise ValueError("MaskConv expects (Conv2d, BatchNorm2d, Hardtanh) triples")
        for i in range(0, len(mods), 3):
            c, b, h = mods[i:i + 3]
            if not (isinstance(c, nn.Conv2d) and isinstance(b, nn.BatchNorm2d)
                    and isinstance(h, nn.Hardtanh)):
                raise ValueError("MaskConv expects (Conv2d, BatchNorm2d, Hardtanh) triples")

    def _block(self, i, x, lens_dev, out_layout):
        conv, bn, act = self.seq_module[i], self.seq_module[i + 1], self.seq_module[i + 2]
        training = bn.training or not bn.track_running_stats
        if bn.training and bn.track_running_stats:
            bn.num_batches_tracked.add_(1)
        mom = bn.momentum if bn.momentum is not None else 0.0
        return ops.ConvBlockFn.apply(x, lens_dev, conv.weight, conv.bias, bn.weight, bn.bias,
                                     bn.running_mean, bn.running_var, training, mom, bn.eps,
                                     tuple(conv.stride), tuple(conv.padding), act.min_val,
                                     act.max_val, out_layout)

    def forward(self, x, lengths):
        lens_dev = lengths.to(x.device, torch.int32)
        for i in range(0, len(self.seq_module), 3):
            x = self._block(i, x, lens_dev, 0)
        return x, lengths

    def forward_collapsed(self, x, lens_dev):
        """Returns T' x N x (C*D) (model.py:356-362 fused)."""
        nblk = len(self.seq_module) // 3
        for b in range(nblk):
            x = self._block(3 * b, x, lens_dev, 1 if b == nblk - 1 else 0)
        return x


class BatchRNN(nn.Module):
    """[SequenceWise BN] -> (bi)GRU over packed lengths -> direction sum (ref model.py:82-109)."""

    def __init__(self, input_size, hidden_size, rnn_type=GRU, bidirectional=False,
                 batch_norm=True, bnm=0.1):
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.bidirectional = bidirectional
        self.bnm = bnm
        self.batch_norm = SequenceWise(BatchNorm1d(input_size, momentum=bnm)) if batch_norm else None
        self.rnn = rnn_type(input_size=input_size, hidden_size=hidden_size,
                            bidirectional=bidirectional, bias=True)
        self.num_directions = 2 if bidirectional else 1

    def flatten_parameters(self):
        self.rnn.flatten_parameters()

    def forward(self, x, output_lengths):
        if self.batch_norm is not None:
            x = self.batch_norm(x)
        lens_dev = output_lengths.to(x.device, torch.int32)
        return self.rnn.run(x, lens_dev, sum_dirs=True)


class Lookahead(nn.Module):
    """Wang et al. 2016 lookahead conv (ref model.py:140-177); unidirectional models only."""

    def __init__(self, n_features, context):
        super().__init__()
        assert context > 0
        self.n_features = n_features
        self.weight = nn.Parameter(torch.Tensor(n_features, context + 1))
        self.register_parameter('bias', None)
        self.context = context
        self.init_parameters()

    def init_parameters(self):
        stdv = 1. / math.sqrt(self.weight.size(1))
        self.weight.data.uniform_(-stdv, stdv)

    def forward(self, input):
        """[T, N, H] -> [T, N, H] (ds2_lookahead_fwd)."""
        return ops.LookaheadFn.apply(input, self.weight, None)

    def forward_htanh(self, input, lo, hi):
        """Lookahead followed by Hardtanh(lo, hi), fused into one kernel."""
        return ops.LookaheadFn.apply(input, self.weight, (float(lo), float(hi)))

    def __repr__(self):
        return (self.__class__.__name__ + '(n_features=' + str(self.n_features)
                + ', context=' + str(self.context) + ')')


class Hardtanh(nn.Hardtanh):
    pass


class DeepSpeech(nn.Module):
    """DS2 (ref model.py:183-393, rnn_type in supported_rnns)."""

    def __init__(self, rnn_type='gru', labels="abc", rnn_hidden_size=768, nb_layers=6,
                 audio_conf=None, bidirectional=True, context=20, bnm=0.1, dropout=0,
                 cnn_width=256, rnn_gemm_precision='fp32'):
        """The reference's constructor (model.py:184-186) plus ``rnn_gemm_precision``:
        'fp32' (default, the reference's arithmetic) or 'bf16' (the recurrent layers'
        GEMMs on the bf16 MFMA with fp32 accumulation, BASELINE cfg4)."""
        super().__init__()
        if audio_conf is None:
            audio_conf = {}
        self._version = '0.0.1'
        self._hidden_size = rnn_hidden_size
        self._hidden_layers = nb_layers
        self._rnn_type = rnn_type
        self._audio_conf = audio_conf or {}
        self._labels = labels
        self._bidirectional = bidirectional
        self._bnm = bnm
        self._dropout = dropout
        self._cnn_width = cnn_width
        if rnn_type not in supported_rnns:
            raise ValueError(f"rnn_type {rnn_type!r} not supported by ds2amd "
                             f"(have {sorted(supported_rnns)})")

        sample_rate = self._audio_conf.get("sample_rate", 16000)
        window_size = self._audio_conf.get("window_size", 0.02)
        num_classes = len(self._labels)

        self.dropout1 = nn.Dropout(p=0.1, inplace=True)   # unused, as in the reference
        self.conv = MaskConv(nn.Sequential(
            nn.Conv2d(1, 32, kernel_size=(41, 11), stride=(2, 2), padding=(20, 5)),
            nn.BatchNorm2d(32, momentum=bnm),
            Hardtanh(0, 20, inplace=True),
            nn.Conv2d(32, 32, kernel_size=(21, 11), stride=(2, 1), padding=(10, 5)),
            nn.BatchNorm2d(32, momentum=bnm),
            Hardtanh(0, 20, inplace=True),
        ))
        rnn_input_size = int(math.floor((sample_rate * window_size + 1e-2) / 2) + 1)
        rnn_input_size = int(math.floor(rnn_input_size + 2 * 20 - 41 + 1e-2) / 2 + 1)
        rnn_input_size = int(math.floor(rnn_input_size + 2 * 10 - 21 + 1e-2) / 2 + 1)
        rnn_input_size *= 32

        rnn_cls = supported_rnns[rnn_type]
        rnns = []
        rnns.append(('0', BatchRNN(input_size=rnn_input_size, hidden_size=rnn_hidden_size,
                                   rnn_type=rnn_cls, bidirectional=bidirectional,
                                   batch_norm=False)))
        for x in range(nb_layers - 1):
            rnns.append(('%d' % (x + 1), BatchRNN(input_size=rnn_hidden_size,
                                                  hidden_size=rnn_hidden_size, rnn_type=rnn_cls,
                                                  bidirectional=bidirectional, bnm=bnm)))
        self.rnns = nn.Sequential(OrderedDict(rnns))
        self.set_rnn_gemm_precision(rnn_gemm_precision)
        self.lookahead = nn.Sequential(
            Lookahead(rnn_hidden_size, context=context),
            Hardtanh(0, 20, inplace=True)
        ) if not bidirectional else None
        fully_connected = nn.Sequential(
            BatchNorm1d(rnn_hidden_size, momentum=bnm),
            Linear(rnn_hidden_size, num_classes, bias=False)
        )
        self.fc = nn.Sequential(SequenceWise(fully_connected))

    def set_rnn_gemm_precision(self, precision: str):
        """'fp32' | 'bf16' for every recurrent layer's GEMMs (see __init__)."""
        ops.rnn_gemm_precision(precision)          # validates
        self._rnn_gemm_precision = precision
        for m in self.rnns:
            m.rnn.gemm_precision = precision
        return self

    def forward(self, x, lengths):
        """x [N,1,161,T] on the GPU, lengths [N] ints (host or device).

        Returns (logits [N,T',C] — a transposed view, as in the reference —,
        probs [N,T',C], output_lengths int32 on the device).
        """
        if not x.is_cuda:
            raise RuntimeError("ds2amd.DeepSpeech runs on the GPU only (HIP kernels)")
        lengths = lengths.cpu().int()
        output_lengths = self.get_seq_lens(lengths)
        lens_dev = output_lengths.to(x.device, non_blocking=True)
        x = self.conv.forward_collapsed(x, lens_dev)          # T' x N x (32*41)
        for rnn in self.rnns:
            x = rnn(x, lens_dev)
        if not self._bidirectional:
            la, ht = self.lookahead[0], self.lookahead[1]
            x = la.forward_htanh(x, ht.min_val, ht.max_val)      # model.py:369-371
        x = self.fc(x)                                         # T' x N x C
        x_tnc = x
        x = x.transpose(0, 1)
        outs = ops.SoftmaxTNCFn.apply(x_tnc)
        return x, outs, lens_dev

    def get_seq_lens(self, input_length):
        """Same float arithmetic as the reference (model.py:382-393)."""
        seq_len = input_length
        for m in self.conv.modules():
            if type(m) == nn.modules.conv.Conv2d:
                seq_len = ((seq_len + 2 * m.padding[1] - m.dilation[1] * (m.kernel_size[1] - 1) - 1)
                           / m.stride[1] + 1)
        return seq_len.int()

    # ---- serialization (ref model.py:395-468) --------------------------------
    @classmethod
    def load_model(cls, path):
        package = torch.load(path, map_location=lambda storage, loc: storage, weights_only=True)
        return cls.load_model_package(package)

    @classmethod
    def load_model_package(cls, package):
        model = cls(rnn_hidden_size=package['hidden_size'], nb_layers=package['hidden_layers'],
                    labels=package['labels'], audio_conf=package['audio_conf'],
                    rnn_type=package['rnn_type'], bnm=package.get('bnm', 0.1),
                    bidirectional=package.get('bidirectional', True),
                    dropout=package.get('dropout', 0), cnn_width=package.get('cnn_width', 0))
        model.load_state_dict(package['state_dict'])
        return model

    @staticmethod
    def serialize(model, optimizer=None, epoch=None, iteration=None, loss_results=None,
                  checkpoint=None, cer_results=None, wer_results=None, avg_loss=None, meta=None,
                  checkpoint_cer_results=None, checkpoint_wer_results=None,
                  checkpoint_loss_results=None, trainval_checkpoint_loss_results=None,
                  trainval_checkpoint_cer_results=None, trainval_checkpoint_wer_results=None):
        model = model.module if DeepSpeech.is_parallel(model) else model
        package = {
            'version': model._version, 'hidden_size': model._hidden_size,
            'hidden_layers': model._hidden_layers, 'rnn_type': model._rnn_type,
            'audio_conf': model._audio_conf, 'labels': model._labels,
            'state_dict': model.state_dict(), 'bnm': model._bnm,
            'bidirectional': model._bidirectional, 'dropout': model._dropout,
            'cnn_width': model._cnn_width,
        }
        if optimizer is not None:
            package['optim_dict'] = optimizer.state_dict()
        if avg_loss is not None:
            package['avg_loss'] = avg_loss
        if epoch is not None:
            package['epoch'] = epoch + 1
        if iteration is not None:
            package['iteration'] = iteration
        package['checkpoint'] = checkpoint
        if loss_results is not None:
            package['loss_results'] = loss_results
            package['cer_results'] = cer_results
            package['wer_results'] = wer_results
            package['checkpoint_cer_results'] = checkpoint_cer_results
            package['checkpoint_wer_results'] = checkpoint_wer_results
            package['checkpoint_loss_results'] = checkpoint_loss_results
            package['trainval_checkpoint_loss_results'] = trainval_checkpoint_loss_results
            package['trainval_checkpoint_cer_results'] = trainval_checkpoint_cer_results
            package['trainval_checkpoint_wer_results'] = trainval_checkpoint_wer_results
        if meta is not None:
            package['meta'] = meta
        return package

    @staticmethod
    def get_labels(model):
        return model.module._labels if DeepSpeech.is_parallel(model) else model._labels

    @staticmethod
    def get_param_size(model):
        return sum(p.numel() for p in model.parameters())

    @staticmethod
    def get_audio_conf(model):
        return model.module._audio_conf if DeepSpeech.is_parallel(model) else model._audio_conf

    @staticmethod
    def get_meta(model):
        m = model.module if DeepSpeech.is_parallel(model) else model
        return {"version": m._version, "hidden_size": m._hidden_size,
                "hidden_layers": m._hidden_layers, "rnn_type": m._rnn_type}

    @staticmethod
    def is_parallel(model):
        return isinstance(model, (torch.nn.parallel.DataParallel,
                                  torch.nn.parallel.DistributedDataParallel))
