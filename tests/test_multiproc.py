"""The N>1 bench path on CPU: world_size-2 gloo processes run bench.py's own
timing harness (barrier + timed region + max over ranks) with a stand-in step,
and frames are sharded with no data-path collective (each rank its own seeds)."""
import json
import os
import subprocess
import sys
import textwrap

from conftest import ROOT

WORKER = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    import bench
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    frames_per_rank = 4
    seeds = [1 + rank * frames_per_rank + f for f in range(frames_per_rank)]
    # stand-in step: rank 1 is slower, so the job time is rank 1's
    step = (lambda: time.sleep(0.02 * (1 + rank)))
    el = bench.timed_region(step, 3, lambda: None, dist.barrier)
    job = bench.max_over_ranks(el, dist, torch.device("cpu"))
    got = [None] * world
    dist.all_gather_object(got, {{"rank": rank, "el": el, "job": job, "seeds": seeds}})
    if rank == 0:
        print(json.dumps(got))
    dist.destroy_process_group()
""")


def test_two_rank_harness(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    out = subprocess.run(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
         "--master-addr", "127.0.0.1", "--master-port", "29533", str(script)],
        capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("[")][-1]
    res = json.loads(line)
    assert len(res) == 2
    jobs = {r["job"] for r in res}
    assert len(jobs) == 1                                   # same job time on every rank
    job = jobs.pop()
    assert abs(job - max(r["el"] for r in res)) < 1e-9      # = slowest rank
    assert job >= 3 * 0.04                                  # rank 1 sleeps 40 ms per step
    s0, s1 = (set(r["seeds"]) for r in sorted(res, key=lambda r: r["rank"]))
    assert not (s0 & s1)                                    # disjoint frame shards


def _bench(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", **(env_extra or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)


def test_bench_gpus_launches_ranks():
    """`bench.py --gpus 2` with no WORLD_SIZE starts 2 ranks itself (child
    torch.distributed.run) and the line reports the world size."""
    out = _bench(["--gpus", "2", "--standin", "--steps", "3", "--warmup", "1"])
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout               # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["scaling"] == "weak"


def test_bench_world_mismatch_fails():
    out = _bench(["--gpus", "2", "--standin"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert out.returncode != 0
    assert "WORLD_SIZE=3" in out.stderr


def test_bench_one_rank_standin():
    out = _bench(["--standin", "--steps", "2", "--warmup", "0"])
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["n_gpus"] == 1
