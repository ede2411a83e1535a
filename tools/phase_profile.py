#!/usr/bin/env python3
"""Per-phase timing of the fused MNIST kernels from in-kernel wall_clock64 stamps.

Each kernel, when given a debug buffer, has thread 0 of every block record the
100 MHz wall clock at its phase boundaries.  For each kernel this prints the
kernel span (first block start -> last stamp), and per phase the mean / max
block time, which tells whether a kernel is load-latency-, compute- or
tail-bound.  Run on the GPU box:  python tools/phase_profile.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_operator_amd.data.synthetic import make_synthetic_mnist  # noqa: E402
from pytorch_operator_amd.models.mnist import FusedMnistTrainer  # noqa: E402
from pytorch_operator_amd.ops import mnist as K  # noqa: E402


def main():
    dev = torch.device("cuda")
    ds = make_synthetic_mnist(6400, device=dev)
    cur = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cur)
    B = int(os.environ.get("B", "64"))
    tr = FusedMnistTrainer(batch_size=B, source=src)
    # one per-sample-conv_bwd step first, so tr.dz2 holds a real dense dz2 for the conv_bwd row
    # (the default conv_chunk 4 step writes the pooled d(a2) into tr.dpool instead)
    tr.conv_chunk = 1
    tr.train_step()
    tr.conv_chunk = 4
    for _ in range(20):
        tr.train_step()
    torch.cuda.synchronize()
    dbg = torch.zeros(1 << 16, dtype=torch.int64, device=dev)
    p = tr.params
    lay = tr.layout
    ce = lay.conv_end
    o2w, o2b = lay.offsets["fc2.weight"], lay.offsets["fc2.bias"]
    fp, fm = tr.flat_params, tr.flat_momentum

    def tail():  # as FusedMnistTrainer.train_step's tail_ call, lr 0 (parameters stay put)
        K.tail_(tr.conv_slab, B, tr.conv_bucket(), fp[:ce], fm[:ce], lr=0.0, momentum=tr.momentum,
                big=K.conv_bwd4_rows(B, lay.offsets),
                w1=(tr.dh[:B], tr.a2[:B], fp[ce:o2w], fm[ce:o2w], None),
                fc2=(tr.dlogits[:B], tr.h1[:B], tr.per_sample[:B], tr.stats, 1.0 / B,
                     fp[o2w:o2b], fm[o2w:o2b], None, fp[o2b:], fm[o2b:], None))
    launches = [
        ("conv12_fwd", lambda: K.conv12_fwd(src, p["conv1.weight"], p["conv1.bias"],
                                            p["conv2.weight"], p["conv2.bias"], B, a1=tr.a1,
                                            idx1=tr.idx1, xn=tr.xn, lab=tr.lab, a2=tr.a2,
                                            idx2=tr.idx2)),
        ("conv12_staged", lambda: K.conv12_fwd(src, p["conv1.weight"], p["conv1.bias"], p["conv2.weight"],
                                               p["conv2.bias"], B, a1=tr.a1, idx1=tr.idx1, xn=tr.xn, lab=tr.lab,
                                               a2=tr.a2, idx2=tr.idx2, stage=tr.stage)),
        ("fc1_fwd", lambda: K.fc1_fwd(tr.a2, p["fc1.weight"], p["fc1.bias"], out=tr.h1)),
        ("fc1_parts", lambda: K.fc1_fwd_parts(tr.a2, p["fc1.weight"], p["fc1.bias"],
                                              out=tr.h_parts[:2 * B * 500].view(2, B, 500))),
        ("head_parts", lambda: tr._head(B)),
        ("fc1_bwd", lambda: tr._fc1_bwd(B, stage_adv=0)),
        ("fc1_bwd_head", lambda: tr._fc1_bwd_head(B, stage_adv=0)),  # the default step's launch 3
        ("conv_bwd", lambda: K.conv_bwd(tr.dz2, p["conv2.weight"], tr.a1, tr.idx1, tr.xn,
                                        tr.slab_views["conv2.weight"], tr.slab_views["conv2.bias"],
                                        tr.slab_views["conv1.weight"], tr.slab_views["conv1.bias"],
                                        slab=tr.conv_slab)),
        ("conv_bwd4", lambda: K.conv_bwd4(tr.dpool, tr.idx2, p["conv2.weight"], tr.a1, tr.idx1, tr.xn, tr.conv_slab,
                                          lay.offsets, B)),
        ("slab_red_sgd", lambda: K.slab_reduce_sgd_(tr.conv_slab, B, tr.conv_bucket(), tr.flat_params[:ce],
                                                    tr.flat_momentum[:ce], lr=0.0, momentum=0.5,
                                                    big=K.conv_bwd4_rows(B, lay.offsets))),
        ("slab_red_sgd_x", lambda: K.slab_reduce_sgd_(tr.conv_slab, B, tr.conv_bucket(), tr.flat_params[:ce],
                                                      tr.flat_momentum[:ce], lr=0.0, momentum=0.5,
                                                      big=K.conv_bwd4_rows(B, lay.offsets),
                                                      extra=(tr.flat_params[ce:], tr.flat_grads[ce:],
                                                             tr.flat_momentum[ce:]))),
        ("tail", tail),  # the default step's launch 5, with the trainer's own arguments
    ]
    reps = 20
    for name, fn in launches:
        spans, phase_means, phase_maxs = [], None, None
        for _ in range(reps):
            dbg.zero_()
            K.set_debug_buffer(dbg)
            fn()
            torch.cuda.synchronize()
            K.set_debug_buffer(None)
            dfull = dbg.view(-1, 16).cpu()
            used = dfull[:, 0] > 0
            d = dfull[used][:, :8].double()
            dc = dfull[used][:, 8:].double()
            valid = d > 0  # blocks of different roles record different numbers of phases
            nph = int(valid.sum(1).max())
            t0 = d[:, 0].min()
            spans.append(float(d[valid].max() - t0) / 100.0)  # 100 MHz -> us
            both = valid[:, 1:nph] & valid[:, :nph - 1]
            deltas = ((d[:, 1:nph] - d[:, :nph - 1]) / 100.0) * both
            cnt = both.sum(0).clamp_min(1)
            m = deltas.sum(0) / cnt
            mx = deltas.max(0).values
            # effective shader clock per block over its own recorded span (first -> last
            # valid stamp; blocks without two stamps are skipped)
            last = valid.sum(1) - 1
            rows = torch.arange(d.shape[0])
            wall = (d[rows, last] - d[:, 0]) * 10.0  # ns
            cyc = dc[rows, last] - dc[:, 0]
            ok = (last > 0) & (wall > 0)
            ghz_b = (cyc[ok] / wall[ok]) if ok.any() else torch.zeros(0, dtype=torch.float64)
            ghz = float(ghz_b.median()) if ghz_b.numel() else float("nan")
            phase_means = m if phase_means is None else phase_means + m
            phase_maxs = mx if phase_maxs is None else torch.maximum(phase_maxs, mx)
            starts = (d[:, 0] - t0) / 100.0
        spans.sort()
        pm = (phase_means / reps).tolist()
        clk = f"{ghz:4.2f}GHz" if 0.3 < ghz < 5.0 else "  n/a  "  # outside any real clock: not shown
        print(f"{name:12s} blocks={int(used.sum()):5d} clk={clk} span med={spans[len(spans)//2]:7.2f}us "
              f"start-skew max={float(starts.max()):6.2f}us  phases(mean/max us): " +
              "  ".join(f"p{i}->{i+1} {a:.2f}/{b:.2f}" for i, (a, b) in
                        enumerate(zip(pm, phase_maxs.tolist()))), flush=True)


if __name__ == "__main__":
    main()
