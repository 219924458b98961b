"""``bench.py --gpus N`` launches N ranks (VERDICT r2 "next" item 2).

Run by hand without WORLD_SIZE, bench.py must not run one process on GPU 0
and call it N GPUs: it starts torch.distributed.run as a child with N worker
processes (rendezvous on 127.0.0.1), each with its own RANK / LOCAL_RANK /
WORLD_SIZE.  ABCD_BENCH_DRYRUN=1 swaps the GPU step for a gloo stand-in rank,
so the launch path itself is exercised here on the CPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=240)


def test_gpus_n_spawns_n_ranks():
    p = _run(["--gpus", "2"], {"ABCD_BENCH_DRYRUN": "1", "OMP_NUM_THREADS": "1"})
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only prints
    r = lines[0]
    assert r["dryrun"] and r["world_size"] == 2 and r["env_world"] == 2
    assert r["rank_sum"] == 1.0 and r["local_rank_sum"] == 1.0  # ranks 0 and 1, local ranks 0 and 1
    assert r["master_addr"] == "127.0.0.1"


def test_gpus_mismatch_under_launcher_is_an_error():
    # a launcher-provided WORLD_SIZE that disagrees with --gpus must not be silently ignored
    p = _run(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in (p.stderr + p.stdout)


def test_driver_launcher_without_gpus_flag():
    # the driver's own form: torch.distributed.run --nproc-per-node N bench.py (no --gpus):
    # --gpus defaults to WORLD_SIZE instead of failing the rank
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update({"ABCD_BENCH_DRYRUN": "1", "OMP_NUM_THREADS": "1"})
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(REPO, "bench.py"),
                        "--steps", "2", "--warmup", "1"], env=env, cwd=REPO, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["world_size"] == 2 and lines[0]["env_world"] == 2, p.stdout
