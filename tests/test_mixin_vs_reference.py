"""The device mixins composed with the REAL reference Aggregator / AsyncAggregator / AuxoAggregator classes
(build container only: /root/reference never travels to the GPU box, so this skips there).

The check runs in a child process (tests/golden/check_mixin_vs_reference.py) because importing the reference
aggregator needs off-path placeholder modules (wandb, torchvision, ...) that must not leak into
the test process.  It asserts identical parameter lists for every overridden method, that the MRO hands the
mixin's super() calls to the reference's own methods (``_reference_impl``), that FedBuff's own
create_client_task is left alone, and that tests/event_loop.py restates the reference's signatures."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.isdir("/root/reference/fedscale"), reason="needs /root/reference (build container)")
def test_mixin_composes_with_the_real_aggregator():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "golden", "check_mixin_vs_reference.py")],
                       cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    report = json.loads(lines[-1])
    assert r.returncode == 0 and report["ok"], report["errors"]
    assert "update_weight_aggregation" in report["overrides_checked"] and len(report["overrides_checked"]) >= 10
