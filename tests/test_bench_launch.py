"""bench.py --gpus N: the rank launcher (VERDICT r5 "Next" 1).  CPU only:
the refusal when fewer than N GPUs are visible, the world-size checks, and
the launcher's plumbing (N children, RANK / LOCAL_RANK / WORLD_SIZE, a gloo
rendezvous on 127.0.0.1, rank 0's line passed through, a failing rank ends
the job non-zero) with a stand-in rank script instead of the GPU bench."""

from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_gpus_2_without_devices_fails_loudly():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_check_world_rules():
    assert bench.check_world(None, env={}, devices=1) == 1
    assert bench.check_world(4, env={}, devices=8) == 4
    assert bench.check_world(None, env={"WORLD_SIZE": "2"}, devices=2) == 2
    with pytest.raises(bench.RankLaunchError, match="WORLD_SIZE=2"):
        bench.check_world(8, env={"WORLD_SIZE": "2"}, devices=8)
    with pytest.raises(bench.RankLaunchError, match="found 1"):
        bench.check_world(2, env={}, devices=1)
    with pytest.raises(bench.RankLaunchError):
        bench.check_world(0, env={}, devices=8)


RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    assert int(os.environ["LOCAL_RANK"]) == rank
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo")
    t = torch.tensor([rank + 1.0])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        n = world if "--lie" not in sys.argv else 1
        print(json.dumps({"n_gpus": n, "max_rank": float(t[0]), "argv": sys.argv[1:]}))
    if "--fail-rank1" in sys.argv and rank == 1:
        sys.exit(5)
    dist.destroy_process_group()
""")


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_runs_n_ranks(tmp_path, capfd, n):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    rc = bench.launch_ranks(n, ["--steps", "1"], script=str(script))
    out = capfd.readouterr().out.strip().splitlines()
    assert rc == 0
    rec = json.loads(out[-1])
    assert rec["n_gpus"] == n and rec["max_rank"] == float(n) and rec["argv"] == ["--steps", "1"]


def test_launcher_failing_rank_is_nonzero(tmp_path, capfd):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    assert bench.launch_ranks(2, ["--fail-rank1"], script=str(script)) != 0


def test_launcher_refuses_wrong_n_gpus(tmp_path, capfd):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    assert bench.launch_ranks(2, ["--lie"], script=str(script)) != 0
    assert '"n_gpus"' not in capfd.readouterr().out
