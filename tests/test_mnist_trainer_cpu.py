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


def test_argmax_aligned_net_equals_net_with_torch_argmax():
    """ArgmaxAlignedNet (the oracle of tests/test_torch_parity_gpu.py) given torch's own pool
    argmax codes is Net: same outputs and gradients; pool_gap 0."""
    import torch.nn.functional as F
    from pytorch_operator_amd.models.mnist import ArgmaxAlignedNet, Net, reference_init

    torch.manual_seed(0)
    x = torch.randn(8, 1, 28, 28)
    y = torch.randint(0, 10, (8,))
    ref, al = Net(), ArgmaxAlignedNet()
    ref.load_state_dict(reference_init(3))
    al.load_state_dict(reference_init(3))

    def code(r):
        _, ind = F.max_pool2d(r, 2, 2, return_indices=True)
        W = r.shape[-1]
        return (((ind // W) % 2) * 2 + ind % 2).to(torch.uint8)
    with torch.no_grad():
        r1 = F.relu(ref.conv1(x))
        idx1 = code(r1)
        idx2 = code(F.relu(ref.conv2(F.max_pool2d(r1, 2, 2)))).reshape(8, 800)
    F.nll_loss(ref(x), y).backward()
    F.nll_loss(al(x, idx1, idx2), y).backward()
    assert al.pool_gap == 0.0
    for (n, p), (_, q) in zip(ref.named_parameters(), al.named_parameters()):
        assert torch.equal(p.grad, q.grad), n
    # a wrong argmax is visible in pool_gap
    al2 = ArgmaxAlignedNet()
    al2.load_state_dict(reference_init(3))
    al2(x, (idx1 + 1) % 4, idx2)
    assert al2.pool_gap > 1e-3
