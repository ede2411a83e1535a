"""Probe the GPU box: device props + eager torch MNIST step timing (the PyTorch-ROCm baseline)."""
import time, json, sys
import torch, torch.nn as nn, torch.nn.functional as F

print("torch", torch.__version__, "hip", torch.version.hip, "avail", torch.cuda.is_available(), flush=True)
p = torch.cuda.get_device_properties(0)
print(p.name, p.gcnArchName, p.multi_processor_count, p.total_memory // 2**30, "GiB", flush=True)

class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1); self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(800, 500); self.fc2 = nn.Linear(500, 10)
    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv1(x)), 2, 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2, 2)
        x = F.relu(self.fc1(x.view(-1, 800)))
        return F.log_softmax(self.fc2(x), dim=1)

dev = torch.device("cuda")
m = Net().to(dev)
opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.5)
x = torch.randn(64, 1, 28, 28, device=dev); y = torch.randint(0, 10, (64,), device=dev)
def step():
    opt.zero_grad(); loss = F.nll_loss(m(x), y); loss.backward(); opt.step()
for _ in range(30): step()
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(200): step()
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 200
print(json.dumps({"torch_eager_ms_per_step": dt * 1e3, "samples_per_s": 64 / dt}), flush=True)
