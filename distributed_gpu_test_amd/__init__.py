"""distributed_gpu_test_amd — an MI355X-native distributed GPU acceptance-test framework.

Reference: ``train.py:10-12`` (deepspeed / get_accelerator imports) and ``train.py:59-94`` (init + initialize).

Same capabilities as ``dashabalashova/distributed-gpu-test`` (train.py CLI, DeepSpeed-style JSON
config, ZeRO-0/1 data parallelism, SLURM + Pyxis launch, CI), built for AMD Instinct MI355X:
PyTorch-ROCm + hand-written HIP/CDNA4 kernels + RCCL over xGMI.
"""
__version__ = "0.1.0"

from .accelerator import get_accelerator  # noqa: F401
from .launch import RankInfo, resolve_rank_info  # noqa: F401
from .config import DSConfig, parse_config, REFERENCE_DS_CONFIG  # noqa: F401
from .parallel.comm import init_distributed, destroy  # noqa: F401


def initialize(*args, **kwargs):
    """DeepSpeed-style ``initialize`` -> (engine, optimizer, dataloader, lr_scheduler)."""
    from .engine import initialize as _init
    return _init(*args, **kwargs)
