# round 3 session 2, step 11: stream GEMM split counts on the Llama-3 8B decode projections (M=32)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 python -u bench/stream_gemm_ab.py --m 32 --shapes llama --arms stream,skinny,f2,f3,f4,f6 --rounds 2 > gpurun_out/s11_stream.jsonl 2> gpurun_out/s11_stream.err; rc=$?
cat gpurun_out/s11_stream.jsonl; exit $rc
