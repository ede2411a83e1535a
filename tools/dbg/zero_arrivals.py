"""Debug: which parameters arrive twice in ZeroAdamW (grad_view) on the GPU."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch
from pytorch_operator_amd.models.llama import CONFIGS, Llama
from pytorch_operator_amd.ops.optim import to_bf16_matmul_weights
from pytorch_operator_amd.parallel import zero as Z

torch.manual_seed(3)
m = Llama(CONFIGS["llama-tiny"]).cuda()
to_bf16_matmul_weights(m)
names = {id(p): n for n, p in m.named_parameters()}
opt = Z.ZeroAdamW(m, lr=1e-2, betas=(0.9, 0.95), weight_decay=0.1, bucket_mb=0.05)
print("buckets", len(opt.buckets), "sinks", opt.sinks)
for i, b in enumerate(opt.buckets):
    print(i, b.dtype, b.grad32.dtype, b.unscaled, [names[id(p)] for p in b.params])
log = []
orig_arrive, orig_on_grad = opt._arrive, opt._on_grad
def arrive(b, p):
    log.append(("arrive", names[id(p)], b.pending))
    return orig_arrive(b, p)
def on_grad(p):
    log.append(("hook", names[id(p)], opt._of[id(p)].pending))
    return orig_on_grad(p)
opt._arrive = arrive
opt._on_grad = on_grad
for p in m.parameters():
    p._post_accumulate_grad_hooks = None
for p in m.parameters():
    p.register_post_accumulate_grad_hook(lambda p: opt._on_grad(p))
for b in opt.buckets:
    for p in b.params:
        s = getattr(p, "_pto_grad_sink", None)
        if s is not None:
            s.ready = (lambda p=p, b=b: opt._arrive(b, p))
tok = torch.randint(0, 256, (2, 65), generator=torch.Generator().manual_seed(0)).cuda()
try:
    for it in range(2):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m(tok[:, :-1], tok[:, 1:])
        loss.backward()
        opt.step()
        log.append(("step", it, 0))
except Exception as e:
    print("ERROR", e)
for x in log:
    print(*x)
