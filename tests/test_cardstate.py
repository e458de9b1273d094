"""fedscale_amd/cardstate.py against a fake amdgpu sysfs tree (CPU): the power, temperature and clock sources are
found by label, converted (µW -> W, m°C -> °C, the pp_dpm level marked '*'), summarised per time window, and a box
that exposes none of them gives a summary that says so instead of raising."""
import time

import pytest

from fedscale_amd import cardstate


def _tree(tmp_path, power=1_180_000_000, junction=52_000, mem=76_000, mclk="0: 2000Mhz *", sclk="0: 500Mhz\n1: 2394Mhz *\n2: 2400Mhz"):
    pci = tmp_path / "0000:8b:00.0"
    hw = pci / "hwmon" / "hwmon7"
    hw.mkdir(parents=True)
    (hw / "power1_input").write_text(str(power))
    (hw / "temp2_input").write_text(str(junction))
    (hw / "temp2_label").write_text("junction\n")
    (hw / "temp3_input").write_text(str(mem))
    (hw / "temp3_label").write_text("mem\n")
    (pci / "pp_dpm_mclk").write_text(mclk + "\n")
    (pci / "pp_dpm_sclk").write_text(sclk + "\n")
    return pci


@pytest.mark.parametrize("process", [False, True])
def test_sources_found_and_converted(tmp_path, monkeypatch, process):
    pci = _tree(tmp_path)
    monkeypatch.setattr(cardstate, "_pci_dir", lambda dev: str(pci))
    s = cardstate.CardSampler("cuda:0", period_s=0.01, process=process)
    one = s.read_once()
    assert one == {"power_w": 1180.0, "temp_junction_c": 52.0, "temp_mem_c": 76.0, "mclk_mhz": 2000.0,
                   "sclk_mhz": 2394.0}
    with s:
        time.sleep(0.08)
    summ = s.summary()
    assert summ["samples"] >= 3 and summ["power_w"]["mean"] == 1180.0 and summ["sclk_mhz"]["max"] == 2394.0
    assert "missing" not in summ


@pytest.mark.parametrize("process", [False, True])
def test_windowed_summary_follows_the_samples(tmp_path, monkeypatch, process):
    pci = _tree(tmp_path)
    monkeypatch.setattr(cardstate, "_pci_dir", lambda dev: str(pci))
    s = cardstate.CardSampler("cuda:0", period_s=0.01, process=process).start()
    time.sleep(0.05)
    t_mid = time.perf_counter()
    (pci / "hwmon" / "hwmon7" / "temp3_input").write_text("80000")
    time.sleep(0.05)
    s.stop()
    early, late = s.summary(None, t_mid), s.summary(t_mid + 0.02, None)
    assert early["temp_mem_c"]["max"] == 76.0 and late["temp_mem_c"]["min"] == 80.0


def test_no_sysfs_is_reported_not_raised(monkeypatch):
    monkeypatch.setattr(cardstate, "_pci_dir", lambda dev: None)
    s = cardstate.CardSampler("cuda:0")
    with s:
        pass
    summ = s.summary()
    assert summ["samples"] == 0 and set(summ["missing"]) >= {"power_w", "temp_mem_c", "mclk_mhz"}
    assert cardstate.snapshot("cuda:0") == {"missing": s.missing}
