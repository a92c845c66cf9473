"""bench.py's multi-rank launch on the CPU: `--gpus N` with no launcher environment starts N rank
processes itself (one per GPU on the box, RCCL there); here the same path runs over gloo with
`--dist-check` (process group + one all-reduce, no model)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=240)


def test_bench_spawns_n_ranks_gloo():
    r = _run(["--gpus", "2", "--backend", "gloo", "--dist-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["world_size"] == 2 and d["n_gpus"] == 2 and d["backend"] == "gloo"
    assert d["rank_sum"] == 1.0               # 0 + 1: both ranks took part in the all-reduce


def test_bench_world_mismatch_exits_nonzero():
    # an external launcher whose WORLD_SIZE disagrees with --gpus: refuse instead of timing one rank
    r = _run(["--gpus", "2", "--backend", "gloo", "--dist-check"],
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 3, (r.returncode, r.stderr[-1000:])
