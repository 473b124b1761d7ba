"""bench.py's N-rank path end to end, on the one-GPU box: `python bench.py --gpus 2` relaunches itself under
torch.distributed.run (one process per rank, 127.0.0.1), every rank codes its own seeded batches with the headline's
team schedule, the timed region is bracketed by barriers and MAX-reduced over the ranks, the per-image records of both
ranks are all-gathered, and only rank 0 prints the JSON line.  The driver's `--gpus 8` runs exactly this code with one
GPU per rank over RCCL; here both ranks share cuda:0 (LBIC_BENCH_DEVICE=0) and use gloo (LBIC_BENCH_BACKEND=gloo:
RCCL refuses two ranks on one device) -- test hooks only, the driver sets neither."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_one_gpu():
    env = dict(os.environ, LBIC_BENCH_DEVICE="0", LBIC_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    n, size, steps = 4, 64, 3
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", "2",
           "--batch", str(n), "--size", str(size), "--team", "2", "--cpu-budget", "0", "--side-steps", "0",
           "--per-image", "0"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    out, err = p.stdout, p.stderr
    print(err[-3000:])
    assert p.returncode == 0, err[-4000:]
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, f"expected one JSON line (rank 0 only), got {len(lines)}"
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["steps"] == steps and j["scaling"] == "weak"
    assert j["config"]["global_batch"] == 2 * n
    assert j["quality"]["images_gathered"] == 2 * n          # both ranks' per-image records
    assert j["quality"]["enc_dec_bit_exact"] is True
    # the timed region: each rank logs its own duration; the line's is the MAX over ranks
    loc = {int(r): float(t) for r, t in re.findall(r"\[rank (\d)\] headline: \d+ batches in [\d.]+ s \(this rank ([\d.]+) s\)",
                                                     err)}
    assert sorted(loc) == [0, 1], loc
    region = j["ms_per_step"] * steps / 1e3
    assert region >= max(loc.values()) - 0.011 and region <= max(loc.values()) + 0.011, (region, loc)
    assert abs(j["value"] - 2 * n * size * size / (region / steps) / 1e6) <= 0.01 * j["value"]
