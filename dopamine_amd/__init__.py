"""dopamine_amd -- MI355X-native replay-sampling + Q-learning update path of Dopamine.

The compute path is the in-tree HIP library ``libdopamine_amd.so`` (C ABI in
include/dopamine_amd.h); importing ``dopamine_amd._lib`` fails loudly if it has
not been built.  PyTorch-ROCm provides device memory, streams, the Nature-CNN
forward/backward and torch.distributed (RCCL).
"""
import os as _os

# Kernel arguments in device memory: measured +22% gradient-steps/s on the
# HIP-graph-replayed learner step (many small dispatches).  Must be set before the
# HIP runtime initialises; an explicit user setting wins.
_os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')

__version__ = '0.1.0'
