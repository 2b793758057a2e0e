"""ds2amd — MI355X-native (gfx950) DeepSpeech2 hot path.

Host-side mirror of the reference's operator/plugin interface for the hot path
(model.DeepSpeech, decoder.GreedyDecoder, warp-ctc CTCLoss, SpectrogramParser,
the train_batch step and its data-parallel gradient exchange), over the C ABI
of libds2hip.so (include/ds2hip.h).
"""
from . import _lib  # noqa: F401

__all__ = ["model", "decoder", "ctc", "data_loader", "optim", "trainer", "ops"]
__version__ = "0.1.0"
