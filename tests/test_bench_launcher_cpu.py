"""bench.py's own multi-GPU launcher and config-4 sharding path, on CPU (gloo, --stub).

``python bench.py --gpus N`` without a torchrun environment must start N ranks itself and report
the world size torch.distributed saw; under torchrun, WORLD_SIZE must equal --gpus.  The stub
vocoder keeps the generator's call surface and output shape, so scatter -> vocode -> gather and
the JSON line are exercised exactly as on the GPU box (where the nccl backend is RCCL)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", **extra)
    return env


def _json_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_n_ranks_and_reports_world(world):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--stub", "--steps", "2", "--warmup", "1",
                        "--batch", "3", "--frames", "12", "--vits-batch", "7", "--vits-frames", "10"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == world and rec["world_size"] == world
    assert [d["rank"] for d in rec["devices"]] == list(range(world))
    assert [d["local_rank"] for d in rec["devices"]] == list(range(world))
    assert rec["config"]["global_batch"] == 3 * world
    sh = rec["sharded"]
    assert sh["utterances"] == 3 * world
    assert sh["last_shard_bitwise_equal"] is True  # the gathered rows are the last rank's shard
    assert sh["scatter_ms"] > 0 and sh["gather_ms"] > 0
    # value = all ranks' samples / the max-over-ranks step time
    samples = 3 * world * 256 * (12 + 10)
    assert rec["value"] == pytest.approx(samples / (rec["ms_per_step"] / 1e3), rel=1e-9)
    # config 5 at N > 1: global batch 7 split over the ranks (strong scaling), scatter/gather of
    # latents, masks and speaker vectors, rank 0's gathered rows equal its shard vocoded alone
    v5 = rec["config5_sharded"]
    assert v5["world_size"] == world and v5["global_batch"] == 7 and v5["scaling"] == "strong"
    assert v5["per_rank_batch"] == -(-7 // world)
    assert v5["rank0_rows_bitwise_equal"] is True
    assert v5["scatter_ms"] > 0 and v5["gather_ms"] > 0 and v5["compute_only_ms_per_step"] > 0
    assert v5["samples_per_s"] == pytest.approx(7 * 256 * 10 / (v5["ms_per_step"] / 1e3), rel=1e-9)


def test_bench_single_rank_has_no_collectives():
    r = subprocess.run([sys.executable, BENCH, "--stub", "--steps", "2", "--warmup", "0", "--batch", "2",
                        "--frames", "8"], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 1 and "sharded" not in rec and "config5_sharded" not in rec


def test_bench_rehearse_sharded_single_rank():
    """--rehearse-sharded at N = 1: both sharded legs over a one-rank group, reported beside (not
    instead of) the headline value."""
    r = subprocess.run([sys.executable, BENCH, "--stub", "--rehearse-sharded", "--steps", "2", "--warmup", "0",
                        "--batch", "2", "--frames", "8", "--vits-batch", "3", "--vits-frames", "6"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 1 and "sharded" not in rec and "config5_sharded" not in rec
    assert rec["sharded_rehearsal"]["last_shard_bitwise_equal"] is True
    v5 = rec["config5_sharded_rehearsal"]
    assert v5["world_size"] == 1 and v5["per_rank_batch"] == 3 and v5["rank0_rows_bitwise_equal"] is True
    # the headline stays the compute-only step at N = 1
    assert rec["value"] == pytest.approx(2 * 256 * (8 + 10) / (rec["ms_per_step"] / 1e3), rel=1e-9)


def test_bench_refuses_world_size_mismatch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--stub", "--steps", "1"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr
