"""bench.py's rank launcher (`--gpus N` starts N ranks under torch.distributed.run) -- CPU only:
the launcher decides before anything touches the GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=120)


def test_gpus_n_launches_n_ranks_with_the_same_arguments():
    r = _run(["--gpus", "8", "--steps", "5", "--warmup", "2", "--workload", "complex_light"], RTMI_BENCH_DRY_RUN="1")
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    # the launcher's own rendezvous picks and holds the port (no bind-then-close probe)
    assert "--standalone" in cmd and "--local-addr=127.0.0.1" in cmd
    assert not [c for c in cmd if c.startswith("--master-port")]
    i = cmd.index(os.path.abspath(BENCH))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5", "--warmup", "2", "--workload", "complex_light"]


def test_world_size_must_equal_gpus():
    r = _run(["--gpus", "8"], WORLD_SIZE="2", RTMI_BENCH_DRY_RUN="1")
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 8" in r.stderr
    r = _run(["--gpus", "0"], RTMI_BENCH_DRY_RUN="1")
    assert r.returncode == 2


def test_launcher_is_not_used_for_one_gpu_or_under_a_launcher():
    sys.path.insert(0, ROOT)
    import importlib
    bench = importlib.import_module("bench")
    assert bench.rank_launch(["--gpus", "1"], {}) is None
    assert bench.rank_launch(["--steps", "3"], {}) is None
    assert bench.rank_launch(["--gpus", "4"], {"WORLD_SIZE": "4"}) is None
    assert bench.rank_launch(["--gpus", "4"], {"WORLD_SIZE": "1"}) == 2
    assert bench.rank_launch(["--gpus", "2"], {"RTMI_BENCH_DRY_RUN": "1"}) == 0
