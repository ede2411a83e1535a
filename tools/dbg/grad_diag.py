import os, sys, json
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"] if "GRAFT_REPO_ROOT" in os.environ else "/root/repo")
import torch, torch.nn.functional as F
import torch.distributed as dist
from pytorch_operator_amd.data.synthetic import make_synthetic_mnist
from pytorch_operator_amd.models.mnist import FusedMnistTrainer, Net, _views
from pytorch_operator_amd.ops import mnist as K
from pytorch_operator_amd.parallel.dist import init_from_env
env = init_from_env("gloo", use_gpu=True)
rank, dev = env.rank, env.device
B = 64
out = {}
for seed in (21, 22):
    ds = make_synthetic_mnist(2048, seed=seed, device=dev)
    cursor = torch.zeros(1, dtype=torch.int32, device=dev)
    src = K.BatchSource(ds.images, ds.labels, perm=ds.perm, cursor=cursor)
    tr = FusedMnistTrainer(batch_size=B, source=src, lr=0.01, momentum=0.5, device=dev, seed=1)
    xf, lab, perm = ds.float_images().cpu(), ds.labels.long().cpu(), ds.perm.long().cpu()
    net = Net()
    for t in range(3):
        cursor.fill_(t)
        tr.forward_backward()
        torch.cuda.synchronize()
        net.load_state_dict({k: v.cpu() for k, v in tr.params.items()})
        net.zero_grad()
        idx = perm[t * B:(t + 1) * B]
        F.nll_loss(net(xf[idx]), lab[idx]).backward()
        g = tr.grads
        row = {}
        for k, q in net.named_parameters():
            a, b = g[k].double().cpu(), q.grad.double()
            row[k] = round(float((a - b).abs().max() / b.abs().max()), 7)
        out[f"seed{seed}_t{t}"] = row
        tr.optimizer_step(advance_cursor=False)
print(json.dumps({"rank": rank, **out}))
