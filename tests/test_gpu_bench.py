"""bench.py end to end on a small workload (the driver runs its default form at round end): one JSON
line with the contract's keys, the sharding fields consistent with the op list, and the roofline block.
Round 6: a variable of the frac_rocprof check shadowed the shard units and broke every run that found
profiles/rocprof_dominant.json."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_small_sets_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--sets", "sgemm-tiny,sgemm-small", "--steps",
                        "2", "--warmup", "1", "--no-cpu-baseline", "--vendor", "off"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["value"] > 0
    cfg = line["config"]
    assert cfg["units"] >= cfg["ops"] and cfg["ops_cut_into_panels"] <= cfg["ops"], cfg
    assert line["roofline"]["peak"] > 0
