#!/usr/bin/env python3
"""BASELINE config 1 on the reference's own terms: CIFAR-10 2-stage on CPU over
localhost gRPC, both stages this framework's ``node.py`` processes (CPU fp32
torch stages, the gRPC data path with the wire schema of
``/root/reference/node_service.proto``), measured as BASELINE.md's survey
measured the reference: per request, stage 0's forward + the SendTensor hop +
stage 1 + the result back; p50 / p99 over the requests, images/s = B / p50.

Differences from the reference are this framework's, not the harness's: one
persistent channel per hop instead of a new channel per request
(``node.py:170``), lifted 4 MiB message caps (the reference fails at B >= 256,
BASELINE.md), the compute off the event loop.

    python bench/cpu_grpc_bench.py [--batches 1,255,1024] [--requests 60] [--threads 4]

Prints one JSON line per batch size.  CPU only; intra-op threads per stage
process default to 4, as in the survey's run of the reference.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,255,1024")
    ap.add_argument("--microbatches", type=int, default=1,
                    help="a request of B images as this many microbatches streamed down the pipeline (1 = the "
                         "reference's one tensor per request)")
    ap.add_argument("--requests", type=int, default=60)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--port", type=int, default=50161)
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args()
    env = dict(os.environ, OMP_NUM_THREADS=str(a.threads), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               PYTHONUNBUFFERED="1")
    tmp = tempfile.mkdtemp(prefix="dnn_cpu_grpc_")
    wpath = os.path.join(tmp, "cifar10_model.pth")
    subprocess.run([sys.executable, "-m", "distributed_neural_networks_amd.tools.make_checkpoint", "--model", "cifar10",
                    "--out", wpath], cwd=ROOT, env=env, check=True, capture_output=True)
    img = os.path.join(tmp, "x.png")  # stage 0 starts inference only with --input_image (as node.py)
    try:
        import numpy as np
        from PIL import Image
        Image.fromarray((np.random.default_rng(0).random((32, 32, 3)) * 255).astype("uint8")).save(img)
    except Exception:  # noqa: BLE001  (no PIL: a missing file makes stage 0 use its random dummy image)
        pass
    for i, B in enumerate(int(b) for b in a.batches.split(",")):
        p0, p1 = a.port + 2 * i, a.port + 2 * i + 1
        cfg = {"nodes": [{"id": "node1", "address": f"127.0.0.1:{p0}", "part_index": 0},
                         {"id": "node2", "address": f"127.0.0.1:{p1}", "part_index": 1}],
               "model_weights": wpath, "num_parts": 2, "return_to_node_id": "node1", "transport": "grpc",
               "model": "cifar10", "micro_batch_size": -(-B // max(1, min(a.microbatches, B))),
               "num_microbatches": max(1, min(a.microbatches, B))}
        cpath = os.path.join(tmp, f"cfg_{B}.json")
        with open(cpath, "w") as f:
            json.dump(cfg, f)
        slog = open(os.path.join(tmp, f"node2_{B}.log"), "w")
        srv = subprocess.Popen([sys.executable, "node.py", "--node_id", "node2", "--config", cpath, "--device", "cpu"],
                               cwd=ROOT, env=env, stdout=slog, stderr=subprocess.STDOUT)
        try:
            t0 = time.perf_counter()
            r = subprocess.run([sys.executable, "node.py", "--node_id", "node1", "--config", cpath, "--num_requests",
                                str(a.requests), "--metrics", "--shutdown_pipeline", "--device", "cpu",
                                "--input_image", img], cwd=ROOT, env=env, capture_output=True, text=True,
                               timeout=a.timeout)
            wall = time.perf_counter() - t0
        finally:
            try:
                srv.wait(timeout=30)
            except subprocess.TimeoutExpired:
                srv.kill()
                srv.wait()
            slog.close()
        met = [ln for ln in r.stdout.splitlines() if ln.startswith("METRICS ")]
        mb = cfg["num_microbatches"]
        B = cfg["micro_batch_size"] * mb  # images per request
        out = {"config": "cifar10 2-stage, CPU, localhost gRPC (BASELINE config 1)", "batch": B, "microbatches": mb,
               "requests": a.requests, "intra_op_threads": a.threads, "rc": r.returncode}
        if r.returncode != 0 or not met:
            out["error"] = (r.stdout + r.stderr)[-800:]
        else:
            m = json.loads(met[-1][len("METRICS "):])
            p50 = m["latency_ms_p50"]
            out.update({"p50_ms": p50, "p99_ms": m["latency_ms_p99"], "mean_ms": m["latency_ms_mean"],
                        "images_per_s_at_p50": round(B / (p50 / 1e3), 1), "wall_s": round(wall, 2)})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
