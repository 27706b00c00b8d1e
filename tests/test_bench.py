"""bench.py's launch contract (`python bench.py --gpus N --steps K --warmup W`).

* Under a launcher (WORLD_SIZE set) the world size must equal --gpus.
* Without one, --gpus N > 1 starts torch.distributed.run with N ranks as a child
  before anything touches the GPU, and rank 0's line reports n_gpus = N.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env=None, timeout=600):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], env=e, capture_output=True, text=True, timeout=timeout)


def _line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2"], env={"WORLD_SIZE": "3", "RANK": "0"}, timeout=120)
    assert r.returncode != 0
    assert "--gpus 2" in (r.stderr + r.stdout) and "WORLD_SIZE=3" in (r.stderr + r.stdout)


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"], timeout=120)
    assert r.returncode != 0


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpus2_without_launcher_runs_two_ranks():
    """`bench.py --gpus 2` with no launcher: two rank processes (gloo, both on GPU 0 --
    the one-GPU rehearsal of the RCCL path), n_gpus 2, and the merge list of the
    1-rank run -- as replicas (rank_plan's choice at 2 ranks: the whole corpus each) and
    row-sharded (GEOBPE_RANK_PLAN=shard: the exchange path the plan takes from 4 ranks)."""
    common = ["--config", "c2", "--warmup", "3", "--steps", "5", "--emit-merges", "--no-cpu-baseline", "--no-replay"]
    two = _line(_run(["--gpus", "2", "--dist-backend", "gloo", *common]))
    rows = _line(_run(["--gpus", "2", "--dist-backend", "gloo", *common], env={"GEOBPE_RANK_PLAN": "shard"}))
    one = _line(_run(["--gpus", "1", *common]))
    assert two["n_gpus"] == 2 and rows["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["parallelism"] == "replicas2" and rows["config"]["parallelism"] == "rows2"
    assert two["config"]["rank_residues"] == [two["config"]["residues"]] * 2
    assert len(rows["config"]["rank_residues"]) == 2 and sum(rows["config"]["rank_residues"]) == rows["config"]["residues"]
    assert two["steps"] == 5 and len(two["merge_list"]) == 8 and rows["steps"] == 5
    assert two["merge_list"] == one["merge_list"] and rows["merge_list"] == one["merge_list"]
