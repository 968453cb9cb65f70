"""bench.py's multi-GPU entry: `python bench.py --gpus N` without torchrun
starts its N rank processes itself, each rank times its steps between barriers, the elapsed time
is the MAX over ranks and `value` the samples of ALL ranks ÷ that time, and rank 0 prints one
JSON line with n_gpus = N.  Exercised on the CPU with gloo ranks and a stand-in generation
(`--stub`); the GPU path differs only in the step function and the RCCL backend."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=180, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # ONE JSON line, from rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_its_ranks(n):
    rec = _run(["--gpus", str(n), "--steps", "3", "--warmup", "1", "--stub"])
    assert rec["n_gpus"] == n and rec["steps"] == 3 and rec["warmup"] == 1
    # whole-job throughput: n ranks x 3 steps x 22 050 samples over the max elapsed time
    elapsed_s = rec["ms_per_step"] * 3 / 1e3
    assert abs(rec["value"] - n * 3 * 22050 / elapsed_s) <= 1e-6 * rec["value"]
    assert rec["ms_per_step"] >= 10.0          # each step sleeps 10 ms


def test_bench_single_rank_default():
    rec = _run(["--steps", "2", "--warmup", "0", "--stub"])
    assert rec["n_gpus"] == 1


@pytest.mark.parametrize("n", [1, 2])
def test_bench_sharded_legs(n):
    """Configs 4 and 5 as BASELINE states them (utterances sharded over the ranks): at every N the
    line carries both legs with the same keys; utterances = per-rank share x N, samples summed
    over the ranks (gathered on rank 0) over the max-over-ranks time."""
    rec = _run(["--gpus", str(n), "--steps", "1", "--warmup", "0", "--stub"])
    oc = rec["other_configs"]
    keys = {"samples_per_s", "rtf", "rtf_per_gpu", "utterances", "n_gpus", "rows_per_gpu", "loop_steps", "device_ms",
            "wall_s", "us_per_loop_step", "loop_samples_per_s", "kernel_path", "roofline", "note"}
    c4, c5 = oc["config4_sparse896_8utt"], oc["config5_deepmind_32utt"]
    assert keys <= set(c4) and keys <= set(c5)
    assert c4["utterances"] == 8 * n and c5["utterances"] == 32 * n and c4["n_gpus"] == c5["n_gpus"] == n
    assert abs(c4["samples_per_s"] * c4["wall_s"] - 8 * n * 110000) <= 1e-6 * 8 * n * 110000
    assert abs(c5["samples_per_s"] * c5["wall_s"] - 32 * n * 16000) <= 1e-6 * 32 * n * 16000
    for c in (c4, c5):
        assert set(c["roofline"]) >= {"bound", "achieved", "peak", "unit", "frac"}
