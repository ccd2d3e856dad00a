"""ddpx — an MI355X-native data-parallel training framework.

Same capabilities and entry points as UnchartedWhispers/Distributed-Data-Parallel-Experiment
(``singlegpu.py`` / ``multigpu.py``, VGG/DeepNN on CIFAR-10, SGD + one-cycle LR,
``checkpoint.pt``), re-designed for AMD Instinct MI355X (gfx950/CDNA4):
hand-written HIP kernels on MFMA for the hot ops, a native RCCL communicator and
gradient-bucket reducer overlapped with backward, a GPU-resident data pipeline and
whole-step HIP-graph capture.
"""
__version__ = "0.1.0"

from .runtime.setup import prepare_model  # noqa: E402,F401
