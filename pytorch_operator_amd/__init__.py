"""pytorch_operator_amd — an MI355X-native PyTorchJob framework.

Control plane: a C++17 PyTorchJob operator (``csrc/operator``) with the
``kubeflow.org/v1`` CRD, reconcile loop, informers, leader election and metrics,
plus an in-repo fake API server and a local kubelet emulator (``cluster``).

Data plane: the reference's MNIST DDP workload on hand-written gfx950 HIP
kernels (``ops``, ``models``), flat-bucket gradient all-reduce over RCCL/xGMI
(``parallel``) and the worker harness (``harness``).
"""
__version__ = "0.1.0"
