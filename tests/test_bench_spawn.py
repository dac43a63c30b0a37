"""bench.py's multi-rank launch: ``python bench.py --gpus N`` without torchrun
spawns its own N ranks with torchrun's environment, and never silently runs one rank. CPU, gloo."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


CHILD = textwrap.dedent("""
    import json, os, sys, time
    import torch, torch.distributed as dist
    out, mode = sys.argv[1], sys.argv[2]
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and os.environ["LOCAL_RANK"] == str(r)
    if mode == "fail" and r == 1:
        sys.exit(5)
    dist.init_process_group("gloo")
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    if r == 0:
        json.dump({"world": w, "sum": t.item()}, open(out, "w"))
    dist.barrier()
    dist.destroy_process_group()
""")


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_ranks_runs_n_gloo_ranks(tmp_path, n):
    import bench
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    out = tmp_path / "out.json"
    rc = bench.spawn_ranks(n, cmd=[sys.executable, str(script), str(out), "ok"], timeout=120)
    assert rc == 0
    res = json.loads(out.read_text())
    assert res == {"world": n, "sum": float(n * (n + 1) // 2)}


def test_spawn_ranks_failure_stops_the_others(tmp_path):
    import bench
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    # rank 1 exits 5 before the rendezvous; rank 0 would wait for it forever
    rc = bench.spawn_ranks(2, cmd=[sys.executable, str(script), str(tmp_path / "o"), "fail"],
                           timeout=120)
    assert rc == 5


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr
