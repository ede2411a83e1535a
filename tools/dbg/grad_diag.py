"""One-step HIP gradients vs torch at the same parameters, per batch (tools/ddp_parity.py triage).

    python tools/dbg/grad_diag.py [--seeds 21,22] [--steps 3]

For every batch: the relative gradient error against torch's own Net and against
ArgmaxAlignedNet fed the HIP pool codes, plus where the HIP and torch pool argmax disagree and
by how much (torch's window max minus its value at the HIP choice, absolute)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from pytorch_operator_amd.data.synthetic import make_synthetic_mnist  # noqa: E402
from pytorch_operator_amd.models.mnist import ArgmaxAlignedNet, FusedMnistTrainer, Net  # noqa: E402
from pytorch_operator_amd.ops import mnist as K  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return round(float((a - b).abs().max() / b.abs().max()), 7)


def code(r):
    _, ind = F.max_pool2d(r, 2, 2, return_indices=True)
    W = r.shape[-1]
    return (((ind // W) % 2) * 2 + ind % 2).to(torch.uint8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="21,22")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B = 64
    out = {}
    for seed in [int(s) for s in a.seeds.split(",")]:
        ds = make_synthetic_mnist(2048, seed=seed, device=dev)
        cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
        tr = FusedMnistTrainer(batch_size=B, source=src, lr=0.01, momentum=0.5, device=dev, seed=1)
        xf, lab, perm = ds.float_images().cpu(), ds.labels.long().cpu(), ds.perm.long().cpu()
        for t in range(a.steps):
            cursor.fill_(t)
            tr.forward_backward()
            torch.cuda.synchronize()
            sd = {k: v.cpu() for k, v in tr.params.items()}
            idx = perm[t * B:(t + 1) * B]
            x = xf[idx]
            row = {}
            for tag, net in (("own", Net()), ("aligned", ArgmaxAlignedNet())):
                net.load_state_dict(sd)
                args = (x,) if tag == "own" else (x, tr.idx1[:B].cpu(), tr.idx2[:B].cpu())
                F.nll_loss(net(*args), lab[idx]).backward()
                g = tr.grads
                row[tag] = {k: rel(g[k], q.grad) for k, q in net.named_parameters()}
            with torch.no_grad():
                net = Net()
                net.load_state_dict(sd)
                r1 = F.relu(net.conv1(x))
                c1 = code(r1)
                p1 = F.max_pool2d(r1, 2, 2)
                r2 = F.relu(net.conv2(p1))
                c2 = code(r2).reshape(B, 800)
                h1, h2 = tr.idx1[:B].cpu(), tr.idx2[:B].cpu()
                d1, d2 = (c1 != h1), (c2 != h2)
                row["flips"] = [int(d1.sum()), int(d2.sum())]
                row["a1_rel"] = rel(tr.a1[:B], p1)
                row["a2_rel"] = rel(tr.a2[:B], F.max_pool2d(r2, 2, 2).reshape(B, 800))
                for nm, d, r, hc in (("conv1", d1, r1, h1), ("conv2", d2.view(B, 50, 4, 4), r2, h2.view(B, 50, 4, 4))):
                    if d.any():
                        Bn, C, H, W = r.shape
                        win = r.view(Bn, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(Bn, C, H // 2, W // 2, 4)
                        at = win.gather(4, hc.view(Bn, C, H // 2, W // 2, 1).long()).squeeze(4)
                        gaps = (win.max(4).values - at)[d]
                        row[f"{nm}_flip_gap_abs_max"] = float(gaps.max())
                        row[f"{nm}_flip_where"] = [list(map(int, w)) for w in d.nonzero()[:4].tolist()]
            out[f"seed{seed}_t{t}"] = row
            tr.optimizer_step(advance_cursor=False)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
