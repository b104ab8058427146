"""CPU: bench.py's process launch.  `--gpus N` without a launcher starts
torch.distributed.run with N ranks as a child process (the parent never
touches the GPU) and fails when the ranks formed are not N; under a launcher
a WORLD_SIZE that differs from --gpus is refused.  (--check-ranks stops
after forming the gloo group, so this runs without a GPU.)"""
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_gpus_2_forms_two_ranks():
    r = _run(["--gpus", "2", "--check-ranks"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"ranks": 2}]


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2", "--check-ranks"],
             {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 2 but 3 ranks" in r.stderr
