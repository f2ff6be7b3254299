"""minitorch (MI355X edition): the reference minitorch operator surface
(``TensorBackend``, ``Tensor.flash_attention[_causal]``, the ``FlashAttention`` autodiff
Functions, ``MultiHeadAttention(use_flash_attention=...)``) running on hand-written
HIP/CDNA4 kernels through ``HipKernelOps``.

    import minitorch
    backend = minitorch.TensorBackend(minitorch.HipKernelOps)
"""
from . import operators  # noqa: F401
from .autodiff import *  # noqa: F401,F403
from .module import *  # noqa: F401,F403
from .nn import *  # noqa: F401,F403
from .optim import *  # noqa: F401,F403
from .tensor import *  # noqa: F401,F403
from .tensor_data import *  # noqa: F401,F403
from .tensor_functions import *  # noqa: F401,F403
from .tensor_ops import *  # noqa: F401,F403
from .modules_basic import *  # noqa: F401,F403
from .modules_transfomer import *  # noqa: F401,F403


def __getattr__(name):
    # HipKernelOps pulls in ctypes/torch plumbing lazily so CPU-only users can import.
    if name == "HipKernelOps":
        from .hip_kernel_ops import HipKernelOps
        return HipKernelOps
    raise AttributeError(name)


version = "0.4-mi355x"
