"""What the box's amdgpu sysfs exposes for this process's GPU, and a CardSampler summary over ~6 s of streaming
(the headline's k_reduce windows back to back)."""
import glob
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fedscale_amd.cardstate import CardSampler, snapshot, _pci_dir  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
pci = _pci_dir(dev)
print("pci", pci)
if pci:
    for p in sorted(glob.glob(os.path.join(pci, "hwmon", "hwmon*", "*")))[:80]:
        try:
            v = open(p).read().strip()[:60] if os.path.isfile(p) else "<dir>"
        except OSError as e:
            v = f"<{e.__class__.__name__}>"
        print(" ", p.split("/hwmon/")[-1], "=", v)
    for n in ("pp_dpm_mclk", "pp_dpm_sclk", "pp_dpm_fclk", "power_dpm_force_performance_level"):
        try:
            print(n, open(os.path.join(pci, n)).read().strip().replace("\n", " | "))
        except OSError as e:
            print(n, e.__class__.__name__)
print("snapshot", json.dumps(snapshot(dev)))
from fedscale_amd import kernels as kx, synth  # noqa: E402

K, P = 1000, 25_000_000
x = torch.empty(K, P, device=dev)
synth.fill(x, K, P, seed=1)
out = torch.empty(P, device=dev)
torch.cuda.synchronize()
with CardSampler(dev) as s:
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 6:
        for _ in range(20):
            kx.reduce(x, K, P, out, denom=1000.0, finalize=True)
        torch.cuda.synchronize()
        n += 20
print("rounds", n, "ms_per_round", (time.perf_counter() - t0) * 1e3 / n)
print("summary", json.dumps(s.summary()))
