"""BASELINE config 1 harness (bench/cpu_grpc_bench.py): two node.py processes on
CPU over localhost gRPC, stage 0 recording each request's end-to-end latency
(--metrics), at the reference's batch 1 and past its 4 MiB message cap."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_grpc_bench_reports_latency(tmp_path):
    r = subprocess.run([sys.executable, "bench/cpu_grpc_bench.py", "--batches", "1,300", "--requests", "3",
                        "--threads", "2", "--port", "50311", "--timeout", "240"], cwd=ROOT, capture_output=True,
                       text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert [x["batch"] for x in rows] == [1, 300]
    for x in rows:
        assert x["rc"] == 0 and "error" not in x, x
        assert x["p50_ms"] > 0 and x["images_per_s_at_p50"] > 0
