"""The card's state while a timed region runs: board power, edge / junction / HBM temperatures and the memory and
shader clock levels, sampled from the amdgpu driver's sysfs files of THIS process's GPU (read-only; no SMI process,
no privileges).  bench.py records a summary per heavy region, so a rested-card figure and a sustained one carry the
signal that separates them.

    with CardSampler(dev) as s:
        ... timed region ...
    s.summary()  # {"samples": n, "power_w": {...}, "temp_junction_c": {...}, "mclk_mhz": {...}, ...}

Sources (amdgpu hwmon ABI): ``hwmon*/power1_average`` or ``power1_input`` (µW), ``temp*_input`` (m°C) named by
``temp*_label`` (edge, junction, mem), ``pp_dpm_mclk`` / ``pp_dpm_sclk`` (the level marked ``*``).  A file the
box does not expose is left out of the summary (``missing`` lists it); nothing here raises.
"""
from __future__ import annotations

import glob
import os
import re
import threading
import time


def _pci_dir(dev) -> str | None:
    """/sys/bus/pci/devices/<domain:bus:dev.fn> of a torch CUDA device (HIP_VISIBLE_DEVICES-aware: torch reports
    the PCI address of the device it sees)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(dev)
        dom, bus, d = getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None)
        if bus is None or d is None:
            return None
        path = "/sys/bus/pci/devices/%04x:%02x:%02x.0" % (dom, bus, d)
        return path if os.path.isdir(path) else None
    except Exception:
        return None


def _read(path: str):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _level(text):
    """MHz of the level pp_dpm_* marks as current ('1: 1300Mhz *')."""
    if not text:
        return None
    for line in text.splitlines():
        if line.rstrip().endswith("*"):
            m = re.search(r"(\d+)\s*[Mm][Hh]z", line)
            if m:
                return float(m.group(1))
    return None


class CardSampler:
    """Samples the card every ``period_s`` between ``start()`` and ``stop()``: on a daemon thread, or with
    ``process=True`` in a child process (``python -m fedscale_amd.cardstate``), so no sysfs read or parsing competes
    for the GIL with the host thread that launches a timed region's kernels.  The child stamps its
    samples with the same monotonic clock (``time.perf_counter`` is CLOCK_MONOTONIC on Linux), so ``summary``
    windows work alike in both modes."""

    def __init__(self, dev, period_s: float = 0.1, process: bool = False):
        self.period = period_s
        self.process = process
        self._proc = None
        self.pci = _pci_dir(dev)
        self.files = {}
        self.missing = []
        if self.pci:
            hw = sorted(glob.glob(os.path.join(self.pci, "hwmon", "hwmon*")))
            if hw:
                h = hw[0]
                pw = [os.path.join(h, n) for n in ("power1_average", "power1_input")]
                pw = [p for p in pw if _read(p) is not None]
                if pw:
                    self.files["power_w"] = (pw[0], lambda t: float(t) / 1e6)
                for tin in sorted(glob.glob(os.path.join(h, "temp*_input"))):
                    label = (_read(tin.replace("_input", "_label")) or os.path.basename(tin)).strip().lower()
                    if _read(tin) is not None:
                        self.files[f"temp_{label}_c"] = (tin, lambda t: float(t) / 1e3)
            for name in ("pp_dpm_mclk", "pp_dpm_sclk", "pp_dpm_fclk"):
                p = os.path.join(self.pci, name)
                if _read(p) is not None:
                    self.files[name[7:] + "_mhz"] = (p, _level)
        for want in ("power_w", "temp_junction_c", "temp_mem_c", "mclk_mhz", "sclk_mhz"):
            if want not in self.files:
                self.missing.append(want)
        self.samples = {k: [] for k in self.files}
        self._stop = threading.Event()
        self._t = None
        self.t0 = self.t1 = None

    def _one(self) -> dict:
        out = {}
        for k, (path, conv) in self.files.items():
            t = _read(path)
            if t is None:
                continue
            try:
                v = conv(t)
            except ValueError:
                v = None
            if v is not None:
                out[k] = v
        return out

    def sample(self):
        now = time.perf_counter()
        for k, v in self._one().items():
            self.samples[k].append((now, v))

    def read_once(self) -> dict:
        """One reading of every source, not stored (the card's state before a region)."""
        out = self._one()
        if self.missing:
            out["missing"] = list(self.missing)
        return out

    def _run(self):
        while not self._stop.is_set():
            self.sample()
            self._stop.wait(self.period)

    def start(self):
        if self.files and self.process:
            import json
            import subprocess
            import sys

            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            spec = json.dumps({"period": self.period, "files": {k: p for k, (p, _) in self.files.items()}})
            self._proc = subprocess.Popen([sys.executable, "-m", "fedscale_amd.cardstate", spec], cwd=root,
                                          stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                          text=True)
            self._proc.stdout.readline()  # "ready": the child samples from here on
        self.t0 = time.perf_counter()
        if self.files and not self.process:
            self._t = threading.Thread(target=self._run, name="card-sampler", daemon=True)
            self._t.start()
        return self

    def stop(self):
        self.t1 = time.perf_counter()
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2)
        if self._proc is not None:
            try:
                out, _ = self._proc.communicate("stop\n", timeout=5)
            except Exception:
                self._proc.kill()
                out, _ = self._proc.communicate()
            self._proc = None
            convs = {k: c for k, (_, c) in self.files.items()}
            for line in out.splitlines():
                parts = line.split("\t", 2)
                if len(parts) != 3 or parts[1] not in convs:
                    continue
                try:
                    v = convs[parts[1]](parts[2].replace("\\n", "\n"))
                except ValueError:
                    v = None
                if v is not None:
                    self.samples[parts[1]].append((float(parts[0]), v))
        return self

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def summary(self, t_from: float = None, t_to: float = None) -> dict:
        """mean / min / max / median / last of every source over the samples in [t_from, t_to] (perf_counter
        seconds; default: the whole run)."""
        lo = self.t0 if t_from is None else t_from
        hi = (self.t1 or time.perf_counter()) if t_to is None else t_to
        out = {"seconds": round(hi - (lo or hi), 3), "source": self.pci}
        n = 0
        for k, tv in self.samples.items():
            vs = [v for t, v in tv if (t_from is None or t >= t_from) and (t_to is None or t <= t_to)]
            if not vs:
                continue
            n = max(n, len(vs))
            s = sorted(vs)
            out[k] = {"mean": round(sum(vs) / len(vs), 2), "min": s[0], "max": s[-1],
                      "median": s[len(s) // 2], "last": vs[-1]}
        out["samples"] = n
        if self.missing:
            out["missing"] = list(self.missing)
        return out


def snapshot(dev) -> dict:
    """One reading of every source (the card's state before a region)."""
    return CardSampler(dev).read_once()


def _child(spec: str) -> int:
    """The process-mode sampler: read the files every period, print "t<TAB>key<TAB>raw text" lines, stop on stdin."""
    import json
    import select
    import sys

    cfg = json.loads(spec)
    period, files = float(cfg["period"]), cfg["files"]
    out = []
    print("ready", flush=True)
    while True:
        now = time.perf_counter()
        for k, path in files.items():
            t = _read(path)
            if t is not None:
                out.append("%.6f\t%s\t%s" % (now, k, t.strip().replace("\n", "\\n")))
        r, _, _ = select.select([sys.stdin], [], [], period)
        if r:
            break
    sys.stdout.write("\n".join(out) + "\n")
    sys.stdout.flush()
    return 0


if __name__ == "__main__":
    import sys

    sys.exit(_child(sys.argv[1]))
