"""Numerics of the hand-written gfx950 MNIST kernels vs a plain PyTorch fp32 reference.

Every fused kernel is compared against the same op computed by torch on the CPU in
fp32 (the reference's dtype): activations, argmax pooling, log-probs, every
parameter gradient, and the SGD(momentum) update.  Tolerances are relative to the
tensor's max magnitude (different summation orders, exact-fp32 MFMA).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


def _data(B, seed=0, n_total=None):
    g = torch.Generator().manual_seed(seed)
    n = n_total or B
    x = torch.randint(0, 256, (n, 784), generator=g, dtype=torch.uint8)
    y = torch.randint(0, 10, (n,), generator=g, dtype=torch.int32)
    return x, y


def _norm(x_u8):
    return ((x_u8.float() / 255.0 - 0.1307) / 0.3081).view(-1, 1, 28, 28)


@pytest.fixture(scope="module")
def lib():
    from pytorch_operator_amd.ops import _native
    return _native.load()


@pytest.mark.parametrize("B", [64, 37, 1])
def test_forward_kernels_match_torch(lib, B):
    from pytorch_operator_amd.models.mnist import reference_init
    from pytorch_operator_amd.ops import mnist as K
    sd = reference_init(3)
    dev = torch.device("cuda")
    p = {k: v.to(dev).contiguous() for k, v in sd.items()}
    x, y = _data(B, seed=B)
    src = K.BatchSource(x.to(dev), y.to(dev))
    a1, idx1, xn, lab = K.conv1_fwd(src, p["conv1.weight"], p["conv1.bias"], B)
    a2, idx2 = K.conv2_fwd(a1, p["conv2.weight"], p["conv2.bias"])
    h1 = K.fc1_fwd(a2, p["fc1.weight"], p["fc1.bias"])
    stats = torch.zeros(16, device=dev)
    _, _, logp = K.head(h1, p["fc2.weight"], p["fc2.bias"], lab, want_grad=False, want_logp=True,
                        stats=stats, loss_scale=1.0 / B)
    torch.cuda.synchronize()

    assert torch.equal(lab.cpu(), y)
    xn_ref = _norm(x)
    assert _rel(xn, xn_ref.view(B, 784)) < 1e-6
    xn = xn_ref
    z1 = F.conv2d(xn, sd["conv1.weight"], sd["conv1.bias"])
    r1, ri1 = F.max_pool2d(F.relu(z1), 2, 2, return_indices=True)
    assert _rel(a1, r1) < 1e-5
    z2 = F.conv2d(r1, sd["conv2.weight"], sd["conv2.bias"])
    r2 = F.max_pool2d(F.relu(z2), 2, 2).reshape(B, 800)
    assert _rel(a2, r2) < 1e-5
    rh = F.relu(r2 @ sd["fc1.weight"].T + sd["fc1.bias"])
    assert _rel(h1, rh) < 1e-5
    rl = F.log_softmax(rh @ sd["fc2.weight"].T + sd["fc2.bias"], dim=1)
    assert _rel(logp, rl) < 1e-5
    loss = F.nll_loss(rl, y.long())
    assert abs(float(stats[0]) - float(loss)) < 1e-4 * max(1.0, abs(float(loss)))
    assert int(stats[1]) == int((rl.argmax(1) == y.long()).sum())


@pytest.mark.parametrize("B", [64, 50, 128, 130])
def test_fused_step_gradients_and_sgd_match_torch(lib, B):
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer, Net, reference_init
    from pytorch_operator_amd.ops import mnist as K
    dev = torch.device("cuda")
    x, y = _data(B, seed=100 + B)
    src = K.BatchSource(x.to(dev), y.to(dev))
    tr = FusedMnistTrainer(batch_size=B, source=src, lr=0.01, momentum=0.5, seed=5)
    tr.forward_backward()
    torch.cuda.synchronize()

    net = Net()
    net.load_state_dict(reference_init(5))
    out = net(_norm(x))
    loss = F.nll_loss(out, y.long())
    loss.backward()
    assert abs(tr.loss() - float(loss)) < 1e-4
    for name, prm in net.named_parameters():
        err = _rel(tr.grads[name], prm.grad)
        assert err < 2e-4, (name, err)

    # two SGD(momentum) steps on the same batch vs torch.optim.SGD
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.5)
    opt.step()
    tr.optimizer_step(advance_cursor=False)
    opt.zero_grad()
    F.nll_loss(net(_norm(x)), y.long()).backward()
    opt.step()
    tr.train_step(advance_cursor=False)
    torch.cuda.synchronize()
    for name, prm in net.named_parameters():
        err = _rel(tr.params[name], prm.data)
        assert err < 1e-4, (name, err)


def test_conv_bwd_dz1_matches_autograd(lib):
    from pytorch_operator_amd.models.mnist import reference_init
    from pytorch_operator_amd.ops import mnist as K
    B = 16
    dev = torch.device("cuda")
    sd = reference_init(7)
    x, y = _data(B, seed=11)
    xn = _norm(x).requires_grad_(False)
    c1w = sd["conv1.weight"].clone().requires_grad_(True)
    z1 = F.conv2d(xn, c1w, sd["conv1.bias"])
    r1 = F.max_pool2d(F.relu(z1), 2, 2)
    r1.retain_grad()
    z2 = F.conv2d(r1, sd["conv2.weight"], sd["conv2.bias"])
    z2.retain_grad()
    out = F.max_pool2d(F.relu(z2), 2, 2)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    # feed torch's dz2 into the kernel and compare dz1 / conv grads
    p = {k: v.to(dev).contiguous() for k, v in sd.items()}
    src = K.BatchSource(x.to(dev), y.to(dev))
    a1, idx1, xnk, _ = K.conv1_fwd(src, p["conv1.weight"], p["conv1.bias"], B)
    gw2 = torch.zeros(50, 20, 5, 5, device=dev)
    gb2 = torch.zeros(50, device=dev)
    gw1 = torch.zeros(20, 1, 5, 5, device=dev)
    gb1 = torch.zeros(20, device=dev)
    dz2 = z2.grad.contiguous().to(dev)
    dz1 = K.conv_bwd(dz2, p["conv2.weight"], a1, idx1, xnk, gw2, gb2, gw1, gb1, want_dz1=True)
    torch.cuda.synchronize()
    # dz1 = grad wrt conv1 pre-activation output z1
    z1b = F.conv2d(xn, sd["conv1.weight"], sd["conv1.bias"]).requires_grad_(True)
    r1b = F.max_pool2d(F.relu(z1b), 2, 2)
    (r1b * r1.grad).sum().backward()
    assert _rel(dz1, z1b.grad) < 1e-4
    assert _rel(gw1, c1w.grad) < 2e-4
    ref_gw2 = torch.nn.grad.conv2d_weight(r1.detach(), (50, 20, 5, 5), z2.grad)
    assert _rel(gw2, ref_gw2) < 1e-4
    assert _rel(gb2, z2.grad.sum((0, 2, 3))) < 1e-4


def test_graph_replay_matches_eager(lib):
    """A captured step replays on successive batches exactly like eager steps."""
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import mnist as K
    dev = torch.device("cuda")
    n = 640
    x, y = _data(n, seed=42, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(0)).to(torch.int32)

    def make():
        cur = torch.zeros(1, dtype=torch.int32, device=dev)
        src = K.BatchSource(x.to(dev), y.to(dev), perm=perm.to(dev), cursor=cur)
        return FusedMnistTrainer(batch_size=64, source=src, seed=9)

    eager = make()
    for _ in range(6):
        eager.train_step()
    graphed = make()
    graphed.train_step()  # first step eager (initialises momentum)
    g = graphed.capture(steps_per_graph=1)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    assert int(graphed.cursor.item()) == 6
    assert _rel(graphed.flat_params, eager.flat_params) < 1e-5


def test_stream_launch_matches_graph_replay(lib):
    """GraphedStep(launch="stream") -- the captured one-step kernel list launched straight
    onto the stream from C++ -- is bit-identical to hipGraph replay and walks the cursor."""
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import mnist as K
    from pytorch_operator_amd.parallel.graphed_step import GraphedStep
    dev = torch.device("cuda")
    n = 1280  # 20 batches: no epoch wrap within the steps taken
    x, y = _data(n, seed=43, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(1)).to(torch.int32)

    def make():
        cur = torch.zeros(1, dtype=torch.int32, device=dev)
        src = K.BatchSource(x.to(dev), y.to(dev), perm=perm.to(dev), cursor=cur)
        return FusedMnistTrainer(batch_size=64, source=src, seed=9)

    a, b = make(), make()
    ra = GraphedStep(a, mode="graph", steps_per_graph=5, launch="graph")
    rb = GraphedStep(b, mode="graph", steps_per_graph=5, launch="stream")
    assert ra.launch == "graph" and rb.launch == "stream" and rb.steps_per_graph == 1
    ra.warm(3)
    ra.run(10)
    rb.warm(3)
    rb.run(10)
    torch.cuda.synchronize()
    assert int(a.cursor.item()) == int(b.cursor.item()) == 13 + ra.internal_steps
    assert torch.equal(a.flat_params, b.flat_params)
    assert torch.equal(a.flat_momentum, b.flat_momentum)


def test_training_reduces_loss_on_learnable_synthetic_data(lib):
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import mnist as K
    dev = torch.device("cuda")
    ds = make_synthetic_mnist(6400, seed=1, device=dev)
    cur = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cur)
    tr = FusedMnistTrainer(batch_size=64, source=src, seed=1)
    losses = []
    for i in range(100):
        tr.train_step()
        losses.append(tr.loss())
    assert sum(losses[-10:]) / 10 < 0.5 * sum(losses[:10]) / 10
    _, acc = tr.evaluate(K.BatchSource(ds.images, ds.labels), n=2000)
    assert acc > 0.9


@pytest.mark.parametrize("B", [64, 13])
def test_conv12_fused_matches_separate_kernels(lib, B):
    from pytorch_operator_amd.models.mnist import reference_init
    from pytorch_operator_amd.ops import mnist as K
    dev = torch.device("cuda")
    sd = reference_init(4)
    p = {k: v.to(dev).contiguous() for k, v in sd.items()}
    n = 300
    x, y = _data(n, seed=5, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(1)).to(torch.int32).to(dev)
    src = K.BatchSource(x.to(dev), y.to(dev), perm=perm, host_offset=250)
    a1, idx1, xn, lab = K.conv1_fwd(src, p["conv1.weight"], p["conv1.bias"], B)
    a2, idx2 = K.conv2_fwd(a1, p["conv2.weight"], p["conv2.bias"])
    f = K.conv12_fwd(src, p["conv1.weight"], p["conv1.bias"], p["conv2.weight"], p["conv2.bias"], B)
    torch.cuda.synchronize()
    assert torch.equal(f[0], a1) and torch.equal(f[1], idx1)
    assert torch.equal(f[2], xn) and torch.equal(f[3], lab)
    assert torch.equal(f[4], a2) and torch.equal(f[5], idx2)
    rows = perm.cpu()[(torch.arange(B) + 250) % n].long()
    assert torch.equal(lab.cpu(), y[rows])


# ---------------------------------------------------------------------------- round 3
@pytest.mark.parametrize("B", [64, 37, 13, 1])
def test_conv_bwd4_chunked_slab_matches_autograd(lib, B):
    """conv_bwd4 (dW_conv2 summed over 4-sample chunks, per-sample conv1/bias rows) reduced
    with the two-segment slab reduction equals torch's conv gradients and the per-sample
    conv_bwd path."""
    from pytorch_operator_amd.models.mnist import flat_layout, reference_init
    from pytorch_operator_amd.ops import mnist as K
    dev = torch.device("cuda")
    sd = reference_init(8)
    x, y = _data(B, seed=900 + B)
    xn = _norm(x)
    c1w = sd["conv1.weight"].clone().requires_grad_(True)
    c1b = sd["conv1.bias"].clone().requires_grad_(True)
    c2w = sd["conv2.weight"].clone().requires_grad_(True)
    c2b = sd["conv2.bias"].clone().requires_grad_(True)
    r1 = F.max_pool2d(F.relu(F.conv2d(xn, c1w, c1b)), 2, 2)
    z2 = F.conv2d(r1, c2w, c2b)
    z2.retain_grad()
    out = F.max_pool2d(F.relu(z2), 2, 2)
    (out * torch.randn(out.shape, generator=torch.Generator().manual_seed(B))).sum().backward()
    p = {k: v.to(dev).contiguous() for k, v in sd.items()}
    src = K.BatchSource(x.to(dev), y.to(dev))
    a1, idx1, xnk, _ = K.conv1_fwd(src, p["conv1.weight"], p["conv1.bias"], B)
    dz2 = z2.grad.contiguous().to(dev)
    lay = flat_layout()
    ce = lay.conv_end
    slab = torch.full((B, ce), float("nan"), device=dev)
    slab.zero_()
    # conv_bwd4 takes dz2 pooled: d at each window's argmax + the argmax code (dy * 2 + dx)
    _, ind = F.max_pool2d(F.relu(z2.detach()), 2, 2, return_indices=True)  # [B, 50, 4, 4] into 8 x 8
    dpool = z2.grad.flatten(2).gather(2, ind.flatten(2)).reshape(B, 800).contiguous().to(dev)
    idx2 = (((ind // 8) % 2) * 2 + ind % 2).reshape(B, 800).to(torch.uint8).contiguous().to(dev)
    K.conv_bwd4(dpool, idx2, p["conv2.weight"], a1, idx1, xnk, slab, lay.offsets, B)
    got = torch.empty(ce, device=dev)
    K.slab_reduce(slab, B, got, big=K.conv_bwd4_rows(B, lay.offsets))
    # per-sample path
    slab1 = torch.zeros((B, ce), device=dev)
    v = {k: slab1[0][lay.offsets[k]:lay.offsets[k] + n].view(s) for k, s, n in
         (("conv2.weight", (50, 20, 5, 5), 25000), ("conv2.bias", (50,), 50),
          ("conv1.weight", (20, 1, 5, 5), 500), ("conv1.bias", (20,), 20))}
    K.conv_bwd(dz2, p["conv2.weight"], a1, idx1, xnk, v["conv2.weight"], v["conv2.bias"], v["conv1.weight"],
               v["conv1.bias"], slab=slab1)
    ref1 = torch.empty(ce, device=dev)
    K.slab_reduce(slab1, B, ref1)
    torch.cuda.synchronize()
    for name, t in (("conv2.weight", c2w), ("conv2.bias", c2b), ("conv1.weight", c1w), ("conv1.bias", c1b)):
        o, n = lay.offsets[name], t.numel()
        assert _rel(got[o:o + n].view(t.shape), t.grad) < 2e-4, name
        assert _rel(got[o:o + n], ref1[o:o + n]) < 1e-5, name
    # the per-sample small partials and chunk rows are deterministic: a second launch is bit-identical
    slab2 = torch.zeros_like(slab)
    K.conv_bwd4(dpool, idx2, p["conv2.weight"], a1, idx1, xnk, slab2, lay.offsets, B)
    got2 = torch.empty(ce, device=dev)
    K.slab_reduce(slab2, B, got2, big=K.conv_bwd4_rows(B, lay.offsets))
    torch.cuda.synchronize()
    assert torch.equal(got, got2)


def _stage_trainer(x, y, perm, B=64, seed=9, **knobs):
    from pytorch_operator_amd.models.mnist import FusedMnistTrainer
    from pytorch_operator_amd.ops import mnist as K
    dev = torch.device("cuda")
    cur = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(x.to(dev), y.to(dev), perm=perm.to(dev), cursor=cur)
    tr = FusedMnistTrainer(batch_size=B, source=src, seed=seed, lr=0.05, momentum=0.5)
    for k, v in knobs.items():
        setattr(tr, k, v)
    return tr


def test_staged_batches_are_bit_identical_to_gathered(lib):
    """The next-batch staging (fc1_bwd fills it, conv12 reads it when the tag matches the
    cursor) trains bit-identically to the per-step gather, also across a host-side cursor
    move (the tag no longer matches -> conv12 gathers) and with advance_cursor=False."""
    n = 640
    x, y = _data(n, seed=77, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(3)).to(torch.int32)
    a = _stage_trainer(x, y, perm, stage_batches=True)
    b = _stage_trainer(x, y, perm, stage_batches=False)
    assert a.stage is not None
    for tr in (a, b):
        for _ in range(3):
            tr.train_step()
        tr.train_step(advance_cursor=False)
        tr.cursor.fill_(7)  # host moves the cursor: the staged batch (tag 3) must not be used
        for _ in range(2):
            tr.train_step()
    torch.cuda.synchronize()
    assert int(a.stage.tag.item()) == int(a.cursor.item()) == 9
    assert torch.equal(a.flat_params, b.flat_params)
    assert torch.equal(a.flat_momentum, b.flat_momentum)
    assert torch.equal(a.lab, b.lab)


@pytest.mark.parametrize("B", [64, 37])
def test_round3_step_matches_round2_step(lib, B):
    """chunked conv backward + staged batches vs the round-2 step (per-sample slab, gathered
    batches): same training trajectory up to summation order; fc gradients stored identically."""
    n = 8 * B
    x, y = _data(n, seed=300 + B, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(5)).to(torch.int32)
    new = _stage_trainer(x, y, perm, B=B, materialize_fc1_grad=True)
    old = _stage_trainer(x, y, perm, B=B, conv_chunk=1, stage_batches=False, w1_tail=False)
    for _ in range(5):
        new.train_step()
        old.train_step()
    torch.cuda.synchronize()
    assert int(new.cursor.item()) == int(old.cursor.item()) == 5
    assert _rel(new.flat_params, old.flat_params) < 1e-6
    assert _rel(new.flat_momentum, old.flat_momentum) < 1e-5
    assert abs(new.loss() - old.loss()) < 1e-5 * max(1.0, abs(old.loss()))
    ce = new.layout.conv_end
    assert _rel(new.flat_grads[ce:], old.flat_grads[ce:]) < 1e-5
    assert _rel(new.flat_grads[:ce], old.flat_grads[:ce]) < 1e-5


def test_on_device_synthetic_dataset_is_deterministic_and_mnist_like(lib):
    """The worker's start-up draws its synthetic set on the GPU: same seed -> same bytes, and
    the same shape / value statistics as the CPU recipe (a different random stream)."""
    from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
    dev = torch.device("cuda")
    a = make_synthetic_mnist(20000, seed=4, device=dev, on_device=True)
    b = make_synthetic_mnist(20000, seed=4, device=dev, on_device=True)
    c = make_synthetic_mnist(20000, seed=4)
    assert a.images.device.type == "cuda" and a.images.dtype == torch.uint8 and a.images.shape == (20000, 784)
    assert torch.equal(a.images, b.images) and torch.equal(a.labels, b.labels)
    assert not torch.equal(a.images.cpu(), c.images)
    ma, mc = float(a.images.float().mean()), float(c.images.float().mean())
    assert abs(ma - mc) < 0.05 * mc, (ma, mc)
    counts = torch.bincount(a.labels.long().cpu(), minlength=10)
    assert int(counts.min()) > 1700 and sorted(a.perm.cpu().tolist()) == list(range(20000))


@pytest.mark.parametrize("B", [64, 37])
def test_w1_tail_is_bit_identical_to_fc1_bwd_wgrad(lib, B):
    """Round 5: dW_fc1 / db_fc1 computed in the tail launch with SGD straight from the MFMA
    accumulators (fc1_bwd runs only dz2 + fc2 + staging) trains bit-identically to fc1_bwd's
    weight-gradient job + the tail's plain SGD, and the materialised gradient has the same bits."""
    n = 12 * B
    x, y = _data(n, seed=500 + B, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(9)).to(torch.int32)
    a = _stage_trainer(x, y, perm, B=B, w1_tail=True, fuse_head=False, materialize_fc1_grad=True)
    b = _stage_trainer(x, y, perm, B=B, w1_tail=False)
    for _ in range(10):
        a.train_step()
        b.train_step()
    torch.cuda.synchronize()
    assert int(a.cursor.item()) == int(b.cursor.item()) == 10
    assert torch.equal(a.flat_params, b.flat_params)
    assert torch.equal(a.flat_momentum, b.flat_momentum)
    assert torch.equal(a.stats, b.stats)
    o1, o2 = a.layout.offsets["fc1.weight"], a.layout.offsets["fc1.bias"]
    assert torch.equal(a.flat_grads[o1:o1 + 400000], b.flat_grads[o1:o1 + 400000])
    assert torch.equal(a.flat_grads[o2:o2 + 500], b.flat_grads[o2:o2 + 500])


@pytest.mark.parametrize("fuse_head", [True, False])
@pytest.mark.parametrize("B", [64, 37])
def test_pooled_dz2_unpools_to_the_dense_dz2(lib, B, fuse_head):
    """Round 5: with conv_bwd4 the input-gradient job hands d(a2) over still pooled ([B, 800]) and
    conv_bwd4 un-pools it through idx2 while staging.  Its un-pooled image is bit-identical to
    the dense dz2 ([B, 50, 8, 8]) the same job writes for the per-sample conv_bwd (conv_chunk 1)."""
    n = 12 * B
    x, y = _data(n, seed=800 + B, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(3)).to(torch.int32)
    a = _stage_trainer(x, y, perm, B=B, fuse_head=fuse_head)
    b = _stage_trainer(x, y, perm, B=B, fuse_head=fuse_head, conv_chunk=1)
    a.train_step()
    b.train_step()
    torch.cuda.synchronize()
    idx = a.idx2[:B].long()
    dense = torch.zeros(B, 800, 4, device=idx.device).scatter_(2, idx[..., None], a.dpool[:B, :, None])
    dense = dense.view(B, 50, 4, 4, 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, 50, 8, 8)
    assert torch.equal(dense, b.dz2[:B])
    assert _rel(a.flat_params, b.flat_params) < 1e-6


@pytest.mark.parametrize("B", [64, 37])
def test_fused_head_step_matches_head_kernel_step(lib, B):
    """Round 5: fc1_bwd with the head recomputed per sample tile on MFMA (no head launch; dW_fc2,
    db_fc2 and the statistics in the tail) against the head-kernel step: h bit-identical (same
    formula), logits-derived tensors equal up to fp32 summation order, and the same training
    trajectory over 10 steps."""
    n = 12 * B
    x, y = _data(n, seed=700 + B, n_total=n)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(2)).to(torch.int32)
    a = _stage_trainer(x, y, perm, B=B, fuse_head=True, materialize_fc1_grad=True)
    b = _stage_trainer(x, y, perm, B=B, fuse_head=False, materialize_fc1_grad=True)
    a.train_step()
    b.train_step()
    torch.cuda.synchronize()
    assert torch.equal(a.h1[:B], b.h1[:B])
    assert _rel(a.dlogits[:B], b.dlogits[:B]) < 1e-5
    assert _rel(a.dh[:B], b.dh[:B]) < 1e-5
    da, db = (next(t for t in tr._dz2_out(B).values() if t is not None) for tr in (a, b))
    assert _rel(da, db) < 1e-5  # the input-gradient hand-off (pooled or dense)
    assert torch.equal(a.per_sample[:B, 1], b.per_sample[:B, 1])
    assert _rel(a.per_sample[:B, 0], b.per_sample[:B, 0]) < 1e-5
    assert abs(float(a.stats[0]) - float(b.stats[0])) < 1e-5 * max(1.0, abs(float(b.stats[0])))
    assert float(a.stats[1]) == float(b.stats[1])
    for name in ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "conv2.weight", "conv1.weight"):
        assert _rel(a.grads[name], b.grads[name]) < 1e-5, name
    for _ in range(9):
        a.train_step()
        b.train_step()
    torch.cuda.synchronize()
    assert int(a.cursor.item()) == int(b.cursor.item()) == 10
    # rounding differences of one step grow along the trajectory (lr 0.05): 1e-5 after 10 steps
    assert _rel(a.flat_params, b.flat_params) < 1e-4
    assert _rel(a.flat_momentum, b.flat_momentum) < 1e-4
