# Round 6: the bf16 paths on the current tree: every bf16 GPU test (plane tests included), the bf16
# HiFiGAN-v1 bench line, the side lines, and the config-5 one-GPU sharded rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bf16c
export TTS_ERRLOG=gpurun_out/bf16c/parity_errors.jsonl
timeout -k 10 600 python -u -m pytest tests/test_bf16_planes_gpu.py tests/test_hifigan_gpu.py tests/test_xtts_gpu.py tests/test_vits_gpu.py tests/test_configs_gpu.py tests/test_sharded_gpu.py tests/test_vits_text_gpu.py tests/test_glow_tts_gpu.py -m gpu -k "bf16 or planes" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bf16c/pytest.log 2>&1 || { tail -40 gpurun_out/bf16c/pytest.log; exit 1; }
tail -1 gpurun_out/bf16c/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2 --math-mode bf16 > gpurun_out/bf16c/bf16.json 2> gpurun_out/bf16c/bf16.err || { tail -5 gpurun_out/bf16c/bf16.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bf16c/bf16.json')); b=d['kernel_breakdown_ms']
print('bf16 step', round(d['ms_per_step'],2), 'serial', round(sum(b.values()),2), {k: round(v,2) for k,v in list(b.items())[:10]})"
SIDE_VITS_TTS=1 timeout -k 10 300 python scripts/side_ab.py > gpurun_out/bf16c/side.json 2> gpurun_out/bf16c/side.err || { tail -5 gpurun_out/bf16c/side.err; exit 1; }
echo "side: $(cat gpurun_out/bf16c/side.json)"
timeout -k 10 400 python bench.py --rehearse-sharded --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits-tts --no-rb2 > gpurun_out/bf16c/rehearsal.json 2> gpurun_out/bf16c/rehearsal.err || { tail -5 gpurun_out/bf16c/rehearsal.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bf16c/rehearsal.json')); v=d['config5_sharded_rehearsal']; print('config5 rehearsal', round(v['ms_per_step'],2), v['rank0_rows_bitwise_equal'])"
