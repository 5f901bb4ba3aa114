"""Multi-GPU paths over RCCL/xGMI: one process per GPU,
launched exactly the way the driver launches the bench — ``python3 bench.py
--gpus N`` with no launcher, so bench.py spawns its own ranks
(``parallel/selflaunch.py``).  Skipped below 2 visible GPUs (conftest:
``multigpu``); RCCL refuses two ranks on one device, so the 1-GPU box cannot
run these — the same schedules run on gloo in ``test_distributed_cpu.py``.
Each test keeps to <= 4 ranks and small shapes (except the full-extras one)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.multigpu]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
ENV.update(PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")

REF_CUT = "conv|fc (reference split, 16 KiB/img hop)"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(*args, timeout=600):
    """``python3 bench.py ...`` as the driver runs it; returns rank 0's one JSON line."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=ENV, capture_output=True,
                       text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def _need(n):
    import torch
    if torch.cuda.device_count() < n:
        pytest.skip(f"needs {n} GPUs, {torch.cuda.device_count()} visible")


def _check_dist_verify(d, n):
    """The answer that crossed the hops (bench.py pp2_verify): every stage-0
    GPU's 4096 images through the bipartite hop and back over the back-edge,
    against fp32 torch (one GPU measures argmax agreement 1.0 and max|dprob|
    3.3e-7 on 16384 images with the same kernels)."""
    assert "dist_verify_error" not in d, d.get("dist_verify_error")
    assert d["dist_verify_images"] == (n // 2) * 4096
    assert d["dist_argmax_agreement_vs_fp32_torch"] == 1.0
    assert d["dist_pred_is_argmax_of_returned_probs"] == 1.0
    assert d["dist_max_abs_dprob"] < 1e-5


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_pp2_headline(n):
    """The N > 1 headline: the reference cut, one stage per GPU, the hop over
    this package's native RCCL channels (not a ProcessGroupNCCL fallback);
    at 4 and 8 GPUs the bipartite SplitLink hop the driver's scaling run takes.
    The line must carry the distributed correctness keys at 1.0."""
    _need(n)
    d = _bench("--gpus", str(n), "--steps", "3", "--warmup", "1", "--batch", "8192", "--latency_iters", "5",
               "--no_extra")
    assert d["n_gpus"] == n and d["value"] > 0 and d["metric"] == "images/sec CIFAR-10 2-stage"
    assert d["config"]["p2p"] == "native"
    assert d["config"]["stage_cut"] == REF_CUT
    k = n // 2
    assert d["config"]["parallelism"] == f"pp2-rccl-{k}x{k}" + ("-bipartite" if k > 1 else "")
    assert d["p50_latency_ms"] is not None and d["p50_latency_ms"] > 0
    _check_dist_verify(d, n)


def test_bench_fc1cut_two_gpus():
    d = _bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "8192", "--placement", "fc1cut",
               "--no_extra")
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["p2p"] == "native"
    assert d["config"]["stage_cut"].startswith("conv+fc1|fc2")


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_full_line(n):
    """The complete multi-GPU line the driver records: headline plus the
    fc1-cut and the BASELINE config 3/4/5 decode rings over RCCL, each ring's
    greedy tokens equal to the same stages colocated on rank 0's GPU."""
    _need(n)
    d = _bench("--gpus", str(n), "--steps", "5", "--warmup", "2", timeout=1100)
    assert d["n_gpus"] == n and d["config"]["p2p"] == "native" and d["config"]["stage_cut"] == REF_CUT
    assert "extras_error" not in d, d.get("extras_error")
    assert d["fc1cut_images_per_s"] > 0
    _check_dist_verify(d, n)
    for key, stages in (("gpt2_4stage", 4), ("llama3_8b_8stage_b32", 8), ("gpt2xl_fp8_8stage_b64", 8)):
        assert key + "_error" not in d, d.get(key + "_error")
        assert d[key + "_decode_tok_s"] > 0 and d[key + "_prefill_tok_s"] > 0 and d[key + "_p50_token_ms"] > 0
        assert d[key + "_config"]["gpu_groups"] == min(n, stages)
        assert d[key + "_dist_token_agreement_vs_colocated"] == 1.0, key


def test_bench_gpt2_pipeline_two_gpus():
    """GPT-2 small, 4 stages over 2 GPU groups: prefill + microbatched ring decode."""
    d = _bench("--model", "gpt2", "--gpus", "2", "--steps", "4", "--warmup", "1")
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["gpu_groups"] == 2


def test_cli_rccl_two_stage(tmp_path):
    """node.py CLI on configs/cifar_2gpu_rccl.json: one stage per GPU, RCCL P2P.
    Each request (the input image plus 7 seeded images, 2 microbatches of 4)
    crosses the hop and its predictions come back over the back-edge; every
    printed prediction must equal the fp32 torch model's (the reference's one
    check, ``node.py:184-192``)."""
    import numpy as np
    import torch
    from PIL import Image
    from distributed_neural_networks_amd.cli import cifar_request
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    from distributed_neural_networks_amd.tools import make_checkpoint
    ck = tmp_path / "cifar10_model.pth"
    make_checkpoint.main(["--out", str(ck)])
    img = tmp_path / "img.png"
    Image.fromarray(np.random.default_rng(0).integers(0, 255, (40, 48, 3), dtype=np.uint8)).save(img)
    cfg = json.load(open(os.path.join(ROOT, "configs", "cifar_2gpu_rccl.json")))
    cfg["model_weights"] = str(ck)
    cfg["micro_batch_size"], cfg["num_microbatches"] = 4, 2
    for i, n in enumerate(cfg["nodes"]):
        n["address"] = f"127.0.0.1:{_port()}"
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    r = subprocess.run([sys.executable, "-m", "distributed_neural_networks_amd.tools.launch", "--config", str(p),
                        "--num_requests", "3", "--input_image", str(img), "--timeout", "240"], env=ENV,
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in out.splitlines() if "***** FINAL PREDICTION (Index):" in l]
    assert len(lines) == 3, out[-3000:]
    m = NeuralNetwork().eval()
    m.load_state_dict(torch.load(str(ck), weights_only=True))

    class A:
        input_image = str(img)
    for req, line in enumerate(lines):
        got = json.loads(line.split("(Index):")[1].split("*****")[0].strip())
        with torch.no_grad():
            want = m(cifar_request(A, "t", 8, req)).argmax(1).tolist()
        assert got == want, (req, got, want)
