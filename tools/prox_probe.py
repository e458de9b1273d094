import sys, torch
sys.path.insert(0, "/root/repo")
from tools.client_bench import LayoutNet
from fedscale_amd import kernels as kx, synth
names, shapes, dtypes = synth.resnet18_layout()
net = LayoutNet(names, shapes, dtypes).to("cuda")
params = [p.data for p in net.parameters()]
glob = [p.clone() for p in params]
print([hex(p.data_ptr() % 256) for p in params[:5]])
for _ in range(30):
    kx.prox_update(params, glob, 0.005)
torch.cuda.synchronize()
big = torch.zeros(12_000_000, device="cuda"); gb = torch.zeros_like(big)
for _ in range(30):
    kx.prox_update([big], [gb], 0.005)
torch.cuda.synchronize()
