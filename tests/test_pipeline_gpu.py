"""End-to-end pipeline tests on one MI355X.

* the minimum slice through the reference CLI: ``node.py`` with a colocated
  2-stage CIFAR config, a real ``.pth`` and a PNG, prediction == torch golden;
* GPT-2 / Llama-3 tiny colocated greedy decode through the CLI == golden;
* microbatched stage streaming on the device equals the same kernels run per
  microbatch (bitwise) and the monolithic batch (tolerance).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, PYTHONUNBUFFERED="1")


def _node(cfg, extra=(), timeout=300):
    return subprocess.run([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", "node1", "--config", str(cfg),
                           *extra], env=ENV, capture_output=True, text=True, timeout=timeout)


def _colocated_cfg(tmp_path, n, model, weights, **extra):
    c = {"nodes": [{"id": f"node{i + 1}", "address": f"127.0.0.1:{51000 + i}", "part_index": i, "device": 0}
                   for i in range(n)],
         "model_weights": weights, "num_parts": n, "return_to_node_id": "node1", "transport": "colocated",
         "model": model}
    c.update(extra)
    p = tmp_path / f"cfg_{model}_{n}.json"
    p.write_text(json.dumps(c))
    return p


def test_cli_cifar_colocated_matches_golden(tmp_path):
    from PIL import Image
    from distributed_neural_networks_amd.cli import load_image
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    torch.manual_seed(11)
    m = NeuralNetwork().eval()
    pth = tmp_path / "cifar10_model.pth"
    torch.save(m.state_dict(), pth)
    rng = np.random.default_rng(0)
    img = tmp_path / "x.png"
    Image.fromarray(rng.integers(0, 255, (40, 40, 3), dtype=np.uint8)).save(img)
    cfg = _colocated_cfg(tmp_path, 2, "cifar10", str(pth))
    r = _node(cfg, ("--input_image", str(img)))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if "***** FINAL PREDICTION (Index):" in l]
    assert line, r.stdout[-2000:]
    pred = int(line[-1].split(":")[-1].strip().strip("*").strip())
    with torch.no_grad():
        ref = int(m(load_image(str(img), "t")).argmax(1))
    assert pred == ref


def _golden_model(model, n_layers, seed):
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models import build_golden_stage
    s = build_golden_stage(model, 0, n_layers - 1, True, True)
    # the CLI synthesises weights on the device (device RNG stream): same here
    sd = ckpt.random_stage_state_dict(model, 0, n_layers - 1, True, True, seed, device=DEV)
    s.load_state_dict({k: v.cpu() for k, v in sd.items()})
    return s.eval()


def _check_greedy(golden, prompts, toks, tie=2e-2):
    """Follow the device's own sequences: the first token must equal the
    golden argmax; a later token may differ only where the golden's top-2
    logits are within ``tie`` (relative) of each other (bf16 vs fp32)."""
    seq = torch.tensor(prompts)
    toks = torch.tensor(toks)
    with torch.no_grad():
        for t in range(toks.shape[1]):
            last = golden(seq)[:, -1]
            top2 = last.topk(2, dim=-1).values
            ref = last.argmax(-1)
            for b in range(seq.shape[0]):
                if int(toks[b, t]) != int(ref[b]):
                    near = (top2[b, 0] - top2[b, 1]).item() <= tie * top2[b, 0].abs().item()
                    assert t > 0 and near, (b, t, toks[b].tolist(), int(ref[b]))
            seq = torch.cat([seq, toks[:, t:t + 1]], 1)


@pytest.mark.parametrize("model,n_layers", [("gpt2-tiny", 4), ("llama3-tiny", 4)])
def test_cli_transformer_colocated_greedy(tmp_path, model, n_layers):
    cfg = _colocated_cfg(tmp_path, 2, model, "synthetic:3", seq_len=32, decode_steps=6)
    prompt = [5, 17, 99, 3, 42, 7, 1, 250]
    r = _node(cfg, ("--prompt", ",".join(map(str, prompt))))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    toks = json.loads(r.stdout.split("generated tokens:")[1].strip().splitlines()[0])
    assert len(toks) == 1 and len(toks[0]) == 6
    _check_greedy(_golden_model(model, n_layers, 3), [prompt], toks)


@pytest.mark.parametrize("chunk", [0, 5])
def test_cli_colocated_decode_microbatches_gpu(tmp_path, chunk):
    """Colocated CLI decode with M = 3 microbatches of 2 sequences (one HIP
    graph per microbatch), whole or chunked prefill: tokens per sequence vs
    golden, tokens/s reported."""
    from distributed_neural_networks_amd.config import load_node
    from distributed_neural_networks_amd.runtime.generate import make_prompts
    cfg = _colocated_cfg(tmp_path, 2, "gpt2-tiny", "synthetic:4", prompt_len=12, decode_steps=6,
                         micro_batch_size=2, num_microbatches=3, prefill_chunk=chunk)
    r = _node(cfg)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    toks = json.loads(r.stdout.split("generated tokens:")[1].strip().splitlines()[0])
    prompts = make_prompts(load_node(str(cfg), "node1").pipeline, None).tolist()
    assert len(toks) == 6
    _check_greedy(_golden_model("gpt2-tiny", 4, 4), prompts, toks)
    m = json.loads([l for l in r.stdout.splitlines() if l.startswith("METRICS ")][0][len("METRICS "):])
    assert m["microbatches"] == 3 and m["decode_tokens_per_s"] > 0


def test_cli_gpt2_tiny_grpc_two_processes_gpu(tmp_path):
    """GPT over the default gRPC transport on the GPU: two node.py processes,
    both stages on device 0; the reference's nested SendTensor chain carries the
    hidden states and returns the all-position logits (B, T, V), which must be
    within 2e-2 relative of the golden model's."""
    import socket

    def port():
        sck = socket.socket()
        sck.bind(("127.0.0.1", 0))
        p = sck.getsockname()[1]
        sck.close()
        return p
    c = {"nodes": [{"id": f"node{i + 1}", "address": f"127.0.0.1:{port()}", "part_index": i, "device": 0}
                   for i in range(2)],
         "model_weights": "synthetic:6", "num_parts": 2, "return_to_node_id": "node1", "transport": "grpc",
         "model": "gpt2-tiny", "seq_len": 16}
    cfg = tmp_path / "grpc_gpt.json"
    cfg.write_text(json.dumps(c))
    prompt = [3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5]
    dump = tmp_path / "logits.npy"
    p2 = subprocess.Popen([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", "node2", "--config", str(cfg),
                           "--serve_seconds", "240"], env=ENV, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          text=True)
    try:
        r = _node(cfg, ("--prompt", ",".join(map(str, prompt)), "--shutdown_pipeline", "--dump_result", str(dump)),
                  timeout=240)
        out2 = p2.communicate(timeout=120)[0]
    finally:
        if p2.poll() is None:
            p2.kill()
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:] + out2[-2000:]
    assert "Processing complete. Prediction:" in r.stdout
    logits = torch.from_numpy(np.load(dump))
    with torch.no_grad():
        ref = _golden_model("gpt2-tiny", 4, 6)(torch.tensor([prompt]))
    assert logits.shape == ref.shape == (1, len(prompt), 512)
    rel = ((logits - ref).norm() / ref.norm()).item()
    assert rel < 2e-2, rel
    pred = int(r.stdout.split("FINAL PREDICTION (Index):")[1].split("*")[0].strip())
    assert pred == int(logits[0, -1].argmax())


def test_microbatched_stream_equals_per_microbatch():
    """Microbatch schedule on the device: bitwise equal to the same stage calls
    one by one, and within tolerance of the monolithic batch."""
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.runtime.pipeline import ColocatedPipeline
    from distributed_neural_networks_amd.runtime.stages import CifarHipStage
    sd0 = ckpt.random_stage_state_dict("cifar10", 0, 1, True, False, 9)
    sd1 = ckpt.random_stage_state_dict("cifar10", 2, 3, False, True, 9)
    st = [CifarHipStage(sd0, 0, 1, DEV), CifarHipStage(sd1, 2, 3, DEV)]
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(512, 3, 32, 32, device=DEV, generator=g)
    mb = ColocatedPipeline(st, 128)
    mb.capture()
    parts = []
    for i in range(4):
        mb.x.copy_(x[i * 128:(i + 1) * 128])
        parts.append(mb().probs.clone())
    eager = [ColocatedPipeline(st, 128)(x[i * 128:(i + 1) * 128]).probs for i in range(4)]
    torch.cuda.synchronize()
    for a, b in zip(parts, eager):
        assert torch.equal(a, b)
    mono = ColocatedPipeline(st, 512)(x).probs
    torch.cuda.synchronize()
    assert (torch.cat(parts) - mono).abs().max().item() < 2e-2
