"""MI355X-native DDP MNIST training framework.

A brand-new framework with the capabilities of ``Jonathanlyj/pytorch_ddp_mnist``
(reference snapshot at /root/reference): the same entry scripts, CLI flags,
wire-up methods and ``model.pt`` checkpoint layout, but the GPU compute path is
hand-written CDNA4 HIP (MFMA tiles, fused epilogues, LDS-resident per-image
convolution), the data-parallel gradient exchange is a native RCCL
communicator over xGMI, and the dataset lives in HBM.

Layout:
  config      typed configuration + reference-compatible CLI (mnist_cpu_mp.py:208-243)
  models/     MLP (reference model) and LeNet-5 specs, flat parameter slab layout
  ops/        loader for the native HIP extension (``_C``) and the CPU IO library (``_io``)
  parallel/   scheduler wire-up, communicators (RCCL / gloo), native DDP reducer
  data/       DistributedSampler-equivalent, synthetic MNIST, idx-ubyte + CDF-5 IO
  utils/      training engines (native GPU and torch-CPU oracle), checkpoint, metrics

``torch`` is imported first on purpose: the native extension links
``libamdhip64.so.7`` / ``librccl.so.1`` by soname, and loading torch first makes
both resolve to the single HIP runtime / RCCL that torch already mapped.
"""
import torch  # noqa: F401  (must precede any native load, see above)

__version__ = "0.1.0"

__all__ = ["__version__"]
