"""CPU smoke of FusedMnistTrainer's constructor and buffer layout (the step itself needs the GPU:
tests/test_kernels_gpu.py).  Catches construction-time errors in code the CPU suite otherwise
never executes."""
import torch


def test_fused_trainer_constructs_on_cpu():
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer, flat_layout
    tr = FusedMnistTrainer(batch_size=64, device=torch.device("cpu"))
    ks = tr.K.fc1_split()
    assert ks == 2 and tr.fc1_ks == ks
    assert tr.h_parts.numel() == ks * 64 * 500
    assert tr.flat_params.numel() == flat_layout().total
    assert tr.a2.shape == (64, 800) and tr.dz2.shape == (64, 50, 8, 8)
    assert tr.conv_chunk in (1, 4) and tr.stage_batches and tr.fuse_conv12
