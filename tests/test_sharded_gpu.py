"""The sharded path of configs 4 and 5 on the device, over a real RCCL process group.

BASELINE.json's config 4 (HiFiGAN-v1, batch 256 over 8 GPUs) and config 5's 8-GPU split run
``scatter_batch`` -> per-rank vocoding -> ``gather_batch`` (tts_amd/sharding.py).
The N > 1 launcher is covered by the gloo tests (test_bench_launcher_cpu.py, test_sharding_cpu.py);
here the same scatter / compute / gather code runs through torch.distributed's "nccl" backend
(RCCL) in a one-rank group on cuda:0, in a fresh child process that builds the group before any
other GPU work (tests/sharded_child.py), at one GPU's shard of each config:

* config 4: a 32 x 1024 mel shard, f16x3 (the headline arithmetic);
* config 5: 8 x 1024 latents with a ragged mask and speaker vectors, VITS flow + 512-channel
  decoder in bf16.

Checks: the scattered inputs arrive bit for bit, the gathered waveforms equal the unsharded
forward bit for bit, and two gathered rows per config against the fp64 oracle (the same rows and
gates as test_hifigan_gpu.py / test_configs_gpu.py).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from _util import assert_close_fp32, tol

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def sharded_result(tmp_path_factory, cuda_device):
    out = tmp_path_factory.mktemp("sharded")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "sharded_child.py"), str(out)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, f"sharded child failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    with np.load(out / "result.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_rccl_group_is_nccl(sharded_result):
    assert str(sharded_result["backend"]) == "nccl"
    assert int(sharded_result["world"]) == 1


def test_config4_shard_scatter_vocode_gather(sharded_result):
    from test_hifigan_gpu import _bench_row_oracle  # the fp64 rows of the same batch (cached per session)

    r = sharded_result
    assert tuple(r["c4_shape"]) == (32, 1, 256 * 1034)
    assert bool(r["c4_scatter_bitwise"]), "config 4: the scattered mel shard differs from rank 0's batch"
    assert bool(r["c4_bitwise"]), "config 4: gathered waveforms differ from the unsharded forward"
    for k, row in enumerate((0, 31)):
        assert_close_fp32(r["c4_rows"][k:k + 1], _bench_row_oracle(row), f"config 4 sharded row {row} (f16x3)",
                          **tol("f16x3"))


def test_config5_shard_scatter_flow_decode_gather(sharded_result):
    from test_configs_gpu import _config5_oracle

    r = sharded_result
    assert tuple(r["c5_shape"]) == (8, 1, 256 * 1024)
    assert bool(r["c5_scatter_bitwise"]), "config 5: scattered latents / masks / speaker vectors differ"
    assert bool(r["c5_bitwise"]), "config 5: gathered waveforms differ from the unsharded step"
    for k, row in enumerate((0, 6)):  # a full-length and the ragged utterance
        assert_close_fp32(r["c5_rows"][k:k + 1], _config5_oracle(row), f"config 5 sharded row {row} (bf16)",
                          **tol("bf16"))
