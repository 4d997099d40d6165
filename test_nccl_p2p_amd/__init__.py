"""MI355X-native inter-GPU point-to-point benchmark framework.

Capabilities of AmadeusChan/test-nccl-p2p (one C++ program,
/root/reference/p2p_matrix.cc, printing N x N uni/bi-directional NCCL P2P
bandwidth matrices), rebuilt for AMD Instinct MI355X:

* native engine (``csrc/``, C++ + HIP for gfx950): schedules, RCCL transport
  over xGMI, hipEvent timing, hand-written fill/verify/reduce kernels, MPI/TCP
  bootstraps, reference-compatible reports; exposed here as ``_p2pcore`` and
  as the ``build/p2p_matrix`` executable (``mpirun -n N ./build/p2p_matrix``);
* ``ops``       — the gfx950 buffer kernels on torch tensors + PyTorch references;
* ``parallel``  — sessions over torch.distributed, schedules, the gloo harness;
* ``utils``     — statistics, report parsing, scaling curves, RCCL env capture;
* ``models``    — traffic models (PP / EP / CP message sizes for LLM configs).

``torch`` is imported first on purpose: it ships its own ROCm runtime
(libamdhip64.so.7, librccl.so.1) and the extension must bind to the same
copies so there is exactly one HIP runtime in the process.
"""

import torch  # noqa: F401  (must precede the native extension, see above)

from ._native import native, native_available, require_native  # noqa: F401

__version__ = "1.0.0"
__all__ = ["native", "native_available", "require_native", "__version__"]
