"""Diagnostic: ResNet-50 train-mode fp32 gradients, HIP BN vs library BN vs fp64 CPU, per layer group."""
import copy
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import test_resnet_gpu as T  # noqa: E402
from pytorch_operator_amd.models.resnet import set_bn_impl  # noqa: E402

torch.backends.cudnn.benchmark, torch.backends.cudnn.allow_tf32 = False, False
ref = T._net()
x, y = T._batch(B=8, H=64)
_, _, g64 = T._fwd_bwd(copy.deepcopy(ref).double(), x.double(), y)
_, _, gc = T._fwd_bwd(copy.deepcopy(ref), x, y)
res = {}
for impl in ("hip", "library"):
    net = set_bn_impl(copy.deepcopy(ref), impl).cuda().to(memory_format=torch.channels_last)
    _, _, res[impl] = T._fwd_bwd(net, x.cuda().to(memory_format=torch.channels_last), y.cuda())
for n in g64:
    if any(k in n for k in ("layer4.0.bn3.weight", "layer4.1.conv1.weight", "layer3.5.bn3.weight", "layer4.2.bn2.bias", "fc.weight", "layer4.2.conv3.weight")):
        print(f"{n:28s} hip {T._rel(res['hip'][n], g64[n]):.2e} lib {T._rel(res['library'][n], g64[n]):.2e} "
              f"cpu {T._rel(gc[n], g64[n]):.2e} hip-vs-lib {T._rel(res['hip'][n], res['library'][n]):.2e}")
