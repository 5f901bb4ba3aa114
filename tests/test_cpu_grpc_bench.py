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


def _run_pipeline(tmp_path, port, mbs, M, requests=2):
    """node2 server + node1 driver over localhost gRPC on CPU; returns node1's
    FINAL PREDICTION lines."""
    import numpy as np
    from PIL import Image
    w = tmp_path / "cifar10_model.pth"
    if not w.exists():
        subprocess.run([sys.executable, "-m", "distributed_neural_networks_amd.tools.make_checkpoint", "--model",
                        "cifar10", "--out", str(w)], cwd=ROOT, check=True, capture_output=True)
    img = tmp_path / "x.png"
    if not img.exists():
        Image.fromarray((np.random.default_rng(1).random((32, 32, 3)) * 255).astype("uint8")).save(img)
    cfg = {"nodes": [{"id": "node1", "address": f"127.0.0.1:{port}", "part_index": 0},
                     {"id": "node2", "address": f"127.0.0.1:{port + 1}", "part_index": 1}],
           "model_weights": str(w), "num_parts": 2, "return_to_node_id": "node1", "transport": "grpc",
           "model": "cifar10", "micro_batch_size": mbs, "num_microbatches": M}
    c = tmp_path / f"cfg_{mbs}_{M}.json"
    c.write_text(json.dumps(cfg))
    env = dict(os.environ, OMP_NUM_THREADS="2")
    srv = subprocess.Popen([sys.executable, "node.py", "--node_id", "node2", "--config", str(c), "--device", "cpu"],
                           cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        r = subprocess.run([sys.executable, "node.py", "--node_id", "node1", "--config", str(c), "--device", "cpu",
                            "--num_requests", str(requests), "--shutdown_pipeline", "--input_image", str(img)],
                           cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    finally:
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
            srv.wait()
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return [ln.split("(Index):", 1)[1].strip(" *") for ln in r.stdout.splitlines() if "FINAL PREDICTION" in ln]


def test_grpc_microbatches_match_one_tensor(tmp_path):
    """A request of 9 images streamed as 3 microbatches of 3 (three SendTensor
    calls in flight, the stage-1 servicer serialising its compute on an
    asyncio lock) returns the same per-row predictions, in order, as the same
    9 images sent as one tensor."""
    one = _run_pipeline(tmp_path, 50331, 9, 1)
    three = _run_pipeline(tmp_path, 50341, 3, 3)
    assert len(one) == 2 and one == three, (one, three)
