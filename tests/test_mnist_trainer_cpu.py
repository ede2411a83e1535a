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


def test_decision_aligned_net_equals_net_with_torch_decisions():
    """DecisionAlignedNet (the oracle of tests/test_torch_parity_gpu.py) given torch's own pool
    argmax codes and ReLU masks is Net: same gradients; decision_gap 0.  A wrong decision shows."""
    import torch.nn.functional as F
    from pytorch_operator_amd.models.mnist import DecisionAlignedNet, Net, reference_init

    torch.manual_seed(0)
    x = torch.randn(8, 1, 28, 28)
    y = torch.randint(0, 10, (8,))
    ref, al = Net(), DecisionAlignedNet()
    ref.load_state_dict(reference_init(3))
    al.load_state_dict(reference_init(3))

    def code(r):
        _, ind = F.max_pool2d(r, 2, 2, return_indices=True)
        W = r.shape[-1]
        return (((ind // W) % 2) * 2 + ind % 2).to(torch.uint8)
    with torch.no_grad():
        r1 = F.relu(ref.conv1(x))
        a1 = F.max_pool2d(r1, 2, 2)
        r2 = F.relu(ref.conv2(a1))
        a2 = F.max_pool2d(r2, 2, 2).reshape(8, 800)
        h = F.relu(ref.fc1(a2))
        dec = (code(r1), code(r2).reshape(8, 800), a1 > 0, a2 > 0, h > 0)
    F.nll_loss(ref(x), y).backward()
    F.nll_loss(al(x, *dec), y).backward()
    assert al.decision_gap == 0.0
    for (n, p), (_, q) in zip(ref.named_parameters(), al.named_parameters()):
        assert torch.allclose(p.grad, q.grad, rtol=1e-6, atol=1e-9), n
    for bad in ((dec[0] + 1) % 4,) + dec[1:], dec[:4] + (~dec[4],):  # wrong argmax / wrong fc1 mask
        al2 = DecisionAlignedNet()
        al2.load_state_dict(reference_init(3))
        al2(x, *bad)
        assert al2.decision_gap > 1e-3
