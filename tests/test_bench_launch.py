"""bench.py --gpus N starts its own N ranks (round-5 review, missing #1): without
a launcher's WORLD_SIZE, the parent process starts torch.distributed.run with N
processes and waits for them (it never touches the GPU and never execs); under
a launcher, --gpus must equal the launcher's world size.  CPU only: the rank
protocol is exercised by the hidden --launch-check mode over gloo (the GPU
rehearsal of the whole benchmark at world 2 is tools/gpu/r6_launch.sh)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env["ARTSBIR_DIST_BACKEND"] = "gloo"
    env.update(kw)
    return env


def test_launch_command_shape():
    sys.path.insert(0, ROOT)
    import bench
    cmd = bench.launch_command(4, ["--gpus", "4", "--steps", "3"], 29123)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["--gpus", "4", "--steps", "3"][-3:]
    assert os.path.samefile(cmd[cmd.index("--master-port=29123") + 1], BENCH)


def test_bench_gpus_2_starts_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], env=_env(), capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    assert lines[0]["n_gpus"] == 2 and lines[0]["world_size"] == 2 and lines[0]["all_reduce"] == 2.0
    assert lines[0]["backend"] == "gloo"


def test_bench_gpus_must_match_launcher_world():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-check"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "--gpus 3 under a launcher of 2 ranks" in r.stderr
