#!/bin/bash
# round 6: config 5's shard of 8 and config 3 each in a fresh process (their inputs the first allocation), against
# their figures inside the default line (allocated after earlier configs' inputs were freed)
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --config c5 --params 12500000 --no-other-configs --cpu-seconds 0 --sustain 0 --steps 5 --warmup 2 > $O/r6_fresh_c5shard.json 2> $O/r6_fresh_c5shard.err || { tail -20 $O/r6_fresh_c5shard.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --no-other-configs --cpu-seconds 0 --sustain 0 --steps 10 --warmup 3 > $O/r6_fresh_c3.json 2> $O/r6_fresh_c3.err || { tail -20 $O/r6_fresh_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --no-other-configs --cpu-seconds 0 --sustain 0 --steps 2 --warmup 1 > $O/r6_fresh_c5.json 2> $O/r6_fresh_c5.err || { tail -20 $O/r6_fresh_c5.err; exit 1; }
python - <<'PY'
import json
for f in ("r6_fresh_c5shard", "r6_fresh_c3", "r6_fresh_c5"):
    l = json.loads(open(f"gpurun_out/{f}.json").read().splitlines()[-1])
    print(f, round(l["ms_per_step"], 3), round(l["roofline"]["achieved"], 1), l["config"]["workload"])
PY
