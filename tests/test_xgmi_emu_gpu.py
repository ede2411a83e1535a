"""xGMI push-protocol all-reduce at world 2/4/8, emulated on one GPU (one launch, grid.y = rank).

csrc/kernels/xgmi_allreduce.hip runs every emulated rank's blocks co-resident, so the
protocol (owner pushes, step-numbered flags, single-buffered recv/gath, ZeRO-1 SGD on the
owned shard, the fused per-sample slab reduction) is checked against a plain PyTorch fp32
reference at the world sizes an 8x MI355X node uses -- which a 1-GPU box cannot host as
separate processes.
"""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def _emu(world, n, nblk=128):
    from pytorch_operator_amd.parallel.xgmi import XgmiEmulation
    return XgmiEmulation(world, n, nblk=nblk)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("n", [431080, 4100])
def test_mean_allreduce(world, n):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(world * 7 + n)
    emu = _emu(world, n)
    try:
        for step in range(3):  # repeated launches exercise the step counters / reuse
            xs = [torch.randn(n, generator=g).to(dev) for _ in range(world)]
            outs = [torch.full((n,), float("nan"), device=dev) for _ in range(world)]
            emu.configure(0, xs, outs)
            emu.launch()
            torch.cuda.synchronize()
            ref = torch.zeros(n, device=dev)
            for x in xs:  # rank order, like the kernel
                ref += x
            ref *= 1.0 / world
            for r, o in enumerate(outs):
                assert torch.allclose(o, ref, rtol=0, atol=1e-6), (step, r, float((o - ref).abs().max()))
        assert emu.error() == 0
    finally:
        emu.close()


@pytest.mark.parametrize("world,nblk,chunked,prepush", [
    (2, 128, False, False), (4, 128, False, False), (8, 128, False, False), (2, 256, False, False),
    (2, 256, True, False), (8, 128, True, False),
    # round 4: fc1_bwd pushes dW_fc1 itself (emulated by prepush), the exchange skips that range;
    # W = 8 x 256 is the production geometry (emulated with one-wave workgroups)
    (2, 256, True, True), (8, 128, True, True), (8, 256, True, True), (8, 256, True, False)])
def test_fused_sgd_with_slab(world, nblk, chunked, prepush):
    from pytorch_operator_amd.models.mnist import flat_layout
    dev = torch.device("cuda", 0)
    L = flat_layout().total
    ce = flat_layout().conv_end
    B, lr, mom = 64, 0.01, 0.5
    g = torch.Generator(device="cpu").manual_seed(100 + world)
    emu = _emu(world, L, nblk)  # nblk 256: the one-GPU-per-rank default (parallel/xgmi.py)
    w1o = flat_layout().offsets["fc1.weight"]
    if world * nblk > 1024:
        assert emu.threads == 64  # the production grid fits one GPU only with one-wave workgroups
    try:
        p0 = torch.randn(L, generator=g).to(dev)
        ps = [p0.clone() for _ in range(world)]
        ms = [torch.zeros(L, device=dev) for _ in range(world)]
        p_ref, m_ref = p0.clone(), torch.zeros(L, device=dev)
        for step in range(4):
            grads = [torch.randn(L, generator=g).to(dev) for _ in range(world)]
            slabs = [torch.randn(B, ce, generator=g).to(dev) for _ in range(world)]
            # chunked: the conv2.weight columns hold conv_bwd4's 16 chunk rows (rows 16.. unused)
            lo = flat_layout().offsets["conv2.weight"]
            big = (B // 4, lo, lo + 25000) if chunked else None
            emu.configure(1, grads, ps, ms, slab=slabs, slab_rows=B, conv_n=ce, lr=lr, momentum=mom,
                          first_step=step == 0, slab_big=big, skip=(w1o, w1o + 400000) if prepush else None)
            if prepush:
                emu.prepush()
            emu.launch()
            torch.cuda.synchronize()
            mean = torch.zeros(L, device=dev)
            for gr, sl in zip(grads, slabs):
                full = gr.clone()
                full[:ce] = sl.sum(0)
                if chunked:
                    full[lo:lo + 25000] = sl[:B // 4, lo:lo + 25000].sum(0)
                mean += full
            mean /= world
            m_ref = mean.clone() if step == 0 else mom * m_ref + mean
            p_ref = p_ref - lr * m_ref
            shard = emu.npad // world
            for r in range(world):
                assert torch.allclose(ps[r], p_ref, rtol=0, atol=2e-5), (step, r, float((ps[r] - p_ref).abs().max()))
                lo, hi = r * shard, min(L, (r + 1) * shard)
                assert torch.allclose(ms[r][lo:hi], m_ref[lo:hi], rtol=0, atol=2e-5)
            # replicas bit-identical (every parameter is updated by exactly one owner)
            for r in range(1, world):
                assert torch.equal(ps[r], ps[0])
        assert emu.error() == 0
    finally:
        emu.close()


@pytest.mark.parametrize("world", [2, 8])
def test_exchange_latency_floor(world, record_property):
    """Graph of back-to-back fused launches; prints us/launch (local-HBM floor of the protocol)."""
    from pytorch_operator_amd.models.mnist import flat_layout
    dev = torch.device("cuda", 0)
    L, ce, B = flat_layout().total, flat_layout().conv_end, 64
    emu = _emu(world, L)
    try:
        ps = [torch.zeros(L, device=dev) for _ in range(world)]
        ms = [torch.zeros(L, device=dev) for _ in range(world)]
        grads = [torch.randn(L, device=dev) for _ in range(world)]
        slabs = [torch.randn(B, ce, device=dev) for _ in range(world)]
        emu.configure(1, grads, ps, ms, slab=slabs, slab_rows=B, conv_n=ce, lr=0.0, momentum=0.5)
        emu.launch()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(50):
                emu.launch()
        best = float("inf")
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            graph.replay()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        us = best / 50 * 1e6
        record_property("us_per_launch", us)
        print(f"\nxgmi emu world={world}: {us:.2f} us per fused exchange launch")
        assert emu.error() == 0
        assert us < 1000
    finally:
        emu.close()


@pytest.mark.parametrize("world,nblk", [(2, 256), (8, 128), (8, 256)])
def test_producer_push_is_bit_identical(world, nblk):
    """fc1_bwd's own dW_fc1 push (emulated: prepush, the exchange skipping that range) lands
    the same bytes in the same receive slots as the exchange's own push: parameters and
    momentum bit-identical to the no-push exchange over several steps."""
    from pytorch_operator_amd.models.mnist import flat_layout
    dev = torch.device("cuda", 0)
    lay = flat_layout()
    L, ce, B = lay.total, lay.conv_end, 64
    w1o, lo = lay.offsets["fc1.weight"], lay.offsets["conv2.weight"]

    def run(prepush):
        g = torch.Generator(device="cpu").manual_seed(500 + world)
        emu = _emu(world, L, nblk)
        try:
            p0 = torch.randn(L, generator=g).to(dev)
            ps = [p0.clone() for _ in range(world)]
            ms = [torch.zeros(L, device=dev) for _ in range(world)]
            for step in range(3):
                grads = [torch.randn(L, generator=g).to(dev) for _ in range(world)]
                slabs = [torch.randn(B, ce, generator=g).to(dev) for _ in range(world)]
                emu.configure(1, grads, ps, ms, slab=slabs, slab_rows=B, conv_n=ce, lr=0.01, momentum=0.5,
                              first_step=step == 0, slab_big=(B // 4, lo, lo + 25000),
                              skip=(w1o, w1o + 400000) if prepush else None)
                if prepush:
                    emu.prepush()
                emu.launch()
            torch.cuda.synchronize()
            assert emu.error() == 0
            return ps, ms
        finally:
            emu.close()
    pa, ma = run(False)
    pb, mb = run(True)
    for r in range(world):
        assert torch.equal(pa[r], pb[r]), r
        assert torch.equal(ma[r], mb[r]), r


@pytest.mark.parametrize("world,nblk", [(2, 128), (4, 128), (8, 128), (8, 256)])
def test_fused_form_exchange(world, nblk):
    """The fused DDP step's exchange (xar_kernel_fc: phase 1 computes dW_fc1 / db_fc1 / dW_fc2 /
    db_fc2 from each rank's activations and deposits them with their owners) at every world size --
    W = 8 x 256 is the node's geometry, one-wave workgroups here -- against torch: the mean over
    ranks of the full gradient, SGD with momentum, every replica identical; per-rank loss stats."""
    from pytorch_operator_amd.models.mnist import flat_layout
    dev = torch.device("cuda", 0)
    lay = flat_layout()
    L, ce, o = lay.total, lay.conv_end, lay.offsets
    w1o, b1o, w2o, b2o = o["fc1.weight"], o["fc1.bias"], o["fc2.weight"], o["fc2.bias"]
    B, lr, mom = 64, 0.01, 0.5
    g = torch.Generator(device="cpu").manual_seed(300 + world)
    emu = _emu(world, L, nblk)
    try:
        p0 = torch.randn(L, generator=g).to(dev)
        ps = [p0.clone() for _ in range(world)]
        ms = [torch.zeros(L, device=dev) for _ in range(world)]
        p_ref, m_ref = p0.clone(), torch.zeros(L, device=dev)
        lo2 = o["conv2.weight"]
        for step in range(3):
            rnd = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
            grads = [rnd(L) for _ in range(world)]
            slabs = [rnd(B, ce) for _ in range(world)]
            dh, a2, dlog, h = ([rnd(B, 500) for _ in range(world)], [rnd(B, 800) for _ in range(world)],
                               [rnd(B, 10) for _ in range(world)], [rnd(B, 500) for _ in range(world)])
            per_sample = [rnd(B, 2) for _ in range(world)]
            stats = [torch.zeros(16, device=dev) for _ in range(world)]
            emu.configure(1, grads, ps, ms, slab=slabs, slab_rows=B, conv_n=ce, lr=lr, momentum=mom,
                          first_step=step == 0, slab_big=(B // 4, lo2, lo2 + 25000), skip=(w1o, L))
            emu.configure_fc(dh, a2, dlog, h, per_sample, stats, B, 1.0 / B, (w1o, b1o, w2o, b2o))
            assert emu.threads == (256 if world * nblk <= 768 else 64)
            emu.launch()
            torch.cuda.synchronize()
            mean = torch.zeros(L, device=dev)
            for r in range(world):
                full = torch.zeros(L, device=dev)
                full[:ce] = slabs[r].sum(0)
                full[lo2:lo2 + 25000] = slabs[r][:B // 4, lo2:lo2 + 25000].sum(0)
                full[ce:w1o] = grads[r][ce:w1o]
                full[w1o:w1o + 400000] = (dh[r].t() @ a2[r]).reshape(-1)
                full[b1o:b1o + 500] = dh[r].sum(0)
                full[w2o:w2o + 5000] = (dlog[r].t() @ h[r]).reshape(-1)
                full[b2o:b2o + 10] = dlog[r].sum(0)
                mean += full
            mean /= world
            m_ref = mean.clone() if step == 0 else mom * m_ref + mean
            p_ref = p_ref - lr * m_ref
            shard = emu.npad // world
            for r in range(world):
                err = float((ps[r] - p_ref).abs().max())
                assert err < 5e-5, (step, r, err)
                lo, hi = r * shard, min(L, (r + 1) * shard)
                assert torch.allclose(ms[r][lo:hi], m_ref[lo:hi], rtol=1e-5, atol=1e-4), (step, r)
                assert torch.allclose(stats[r][:2], torch.stack([per_sample[r][:, 0].sum() / B,
                                                                 per_sample[r][:, 1].sum()]), rtol=1e-5, atol=1e-5)
            for r in range(1, world):
                assert torch.equal(ps[r], ps[0])
        assert emu.error() == 0
    finally:
        emu.close()


@pytest.mark.parametrize("world,nblk", [(2, 256), (8, 256)])
def test_fused_form_exchange_latency(world, nblk, record_property):
    """us per launch, back-to-back in one graph, of the fused form's exchange (fc tiles in phase 1)
    and of the round-5 form's (dW_fc1 pushed by fc1_bwd, here by the untimed prepush; the exchange
    skips that range).  Emulated: all ranks' bytes move through one GPU, so both are floors of the
    protocol, not the node's numbers; the fused form's extra is its 1632 fc tiles."""
    import json
    import os
    from pathlib import Path
    from pytorch_operator_amd.models.mnist import flat_layout
    dev = torch.device("cuda", 0)
    lay = flat_layout()
    L, ce, o, B = lay.total, lay.conv_end, lay.offsets, 64
    w1o = o["fc1.weight"]
    out = {}
    for form in ("r5", "fused"):
        emu = _emu(world, L, nblk)
        try:
            ps = [torch.zeros(L, device=dev) for _ in range(world)]
            ms = [torch.zeros(L, device=dev) for _ in range(world)]
            grads = [torch.randn(L, device=dev) for _ in range(world)]
            slabs = [torch.randn(B, ce, device=dev) for _ in range(world)]
            if form == "fused":
                emu.configure(1, grads, ps, ms, slab=slabs, slab_rows=B, conv_n=ce, lr=0.0, momentum=0.5,
                              skip=(w1o, L))
                acts = [[torch.randn(B, k, device=dev) for _ in range(world)] for k in (500, 800, 10, 500)]
                emu.configure_fc(*acts, None, None, B, 1.0 / B,
                                 (w1o, o["fc1.bias"], o["fc2.weight"], o["fc2.bias"]))
            else:
                emu.configure(1, grads, ps, ms, slab=slabs, slab_rows=B, conv_n=ce, lr=0.0, momentum=0.5,
                              skip=(w1o, w1o + 400000))
            emu.launch()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(50):
                    emu.launch()
            best = float("inf")
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                graph.replay()
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            out[form] = round(best / 50 * 1e6, 2)
            assert emu.error() == 0
        finally:
            emu.close()
    record_property("us_per_launch", out)
    print(f"\nxgmi emu world={world} x {nblk}: {out} us per exchange launch")
    rec = os.environ.get("PTO_TEST_RECORD_DIR")
    if rec:
        Path(rec).mkdir(parents=True, exist_ok=True)
        (Path(rec) / f"emu_exchange_latency_w{world}x{nblk}.json").write_text(json.dumps(out))
    assert all(v < 1000 for v in out.values())
