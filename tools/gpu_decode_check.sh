set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread -k "shuffled or skinny or w8 or norm or stage" > gpurun_out/pytest_tf.log 2>&1; tail -2 gpurun_out/pytest_tf.log
timeout -k 10 300 python -u bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 --dtype fp8 > gpurun_out/llama_fp8_b1.log 2>&1; tail -1 gpurun_out/llama_fp8_b1.log
timeout -k 10 300 python -u bench/gpt_bench.py --model llama3-8b --stages 8 --batch 1 --prompt 128 > gpurun_out/llama_bf16_b1.log 2>&1; tail -1 gpurun_out/llama_bf16_b1.log
