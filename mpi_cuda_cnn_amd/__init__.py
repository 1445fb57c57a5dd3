"""mpi_cuda_cnn_amd — an MI355X-native data-parallel CNN trainer.

Same capabilities as the MPI+CUDA reference (AnselObergfell/MPI-CUDA-CNN):
serial CPU training/evaluation, MPI data-parallel training, GPU offload and a
hybrid multi-process GPU trainer, the IDX (MNIST) reader and the same CLI /
stderr log — re-designed for gfx950: hand-written HIP kernels on MFMA
(``csrc/kernels``), a native C++ engine (``csrc/engine``), RCCL over xGMI
through ``torch.distributed`` for the data-parallel gradient sync.

``torch`` is imported first so the native module binds to the HIP runtime
and RCCL that torch already loaded (one runtime per process).
"""

import torch  # noqa: F401  (must precede _C: shared HIP runtime)

from . import _C
from ._C import (  # noqa: F401
    ModelSpec,
    CpuNet32,
    CpuNet64,
    GpuNet64,
    GpuNet,
    MccError,
    init_params,
    make_model,
    model_names,
    parse_model_spec,
    idx_read,
    idx_write,
    synth_dataset,
    save_weights,
    load_weights,
)

__version__ = "0.1.0"

__all__ = [
    "ModelSpec",
    "CpuNet32",
    "CpuNet64",
    "GpuNet64",
    "GpuNet",
    "MccError",
    "init_params",
    "make_model",
    "model_names",
    "parse_model_spec",
    "idx_read",
    "idx_write",
    "synth_dataset",
    "save_weights",
    "load_weights",
]
