"""Operator layer (N1 in SURVEY.md §7.1): HIP kernels behind autograd Functions.

* :mod:`._lib`        native library loading / backend selection (fails loudly on GPU)
* :mod:`.kernels`     ``K.<op>`` device dispatch (HIP on GPU, PyTorch reference on CPU)
* :mod:`.ref`         PyTorch reference implementations of every kernel
* :mod:`.params`      compute-weight shadows and flat-gradient sinks
* :mod:`.conv_blocks` fused ResNet stem / residual-block executors, biased conv, pooling
* :mod:`.functions`   Linear / Dropout / softmax-cross-entropy / log-softmax
* :mod:`.rnn`         embedding + LSTM (BiLSTM text path)
* :mod:`.transformer` LayerNorm / GELU / fused attention (BERT path)
"""
from ._lib import available, backend, load, set_backend  # noqa: F401
from .kernels import K  # noqa: F401
from .functions import cross_entropy, dropout, linear, log_softmax  # noqa: F401
