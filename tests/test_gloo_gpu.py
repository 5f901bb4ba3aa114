"""Multi-process pipeline schedules with device compute on one MI355X
(transport ``gloo_gpu``): several ranks share GPU 0 (RCCL refuses that), run
their stages on the HIP kernels with HIP graphs, and hop through pinned host
memory with RCCL-like stream/event ordering (``parallel/links.py
HostStagedLink``).  This is the only place the scheduler's slot reuse and
stream ordering meet asynchronous device compute before a multi-GPU node
exists.  Reference: the cross-process hop ``node.py:45-89``.

Both checks compare against the same pipeline run colocated in one process
(the same kernels, so predictions / tokens must be identical) and against
the fp32 torch golden.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, PYTHONUNBUFFERED="1")


def _ports(n):
    out = []
    for _ in range(n):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        out.append(s.getsockname()[1])
        s.close()
    return out


def _cfg(tmp_path, transport, n, model, weights, layers=None, **extra):
    ports = _ports(n)
    nodes = []
    for i in range(n):
        nd = {"id": f"node{i + 1}", "address": f"127.0.0.1:{ports[i]}", "part_index": i, "device": 0}
        if layers is not None:
            nd["layers"] = list(layers[i])
        nodes.append(nd)
    c = {"nodes": nodes, "model_weights": weights, "num_parts": n, "return_to_node_id": "node1",
         "transport": transport, "model": model, "heartbeat_timeout_s": 60}
    c.update(extra)
    p = tmp_path / f"cfg_{transport}_{model}_{n}.json"
    p.write_text(json.dumps(c))
    return p


def _run(cfg, n, extra0=(), timeout=240):
    """node2..n in the background, node1 in the foreground; every rank must exit 0."""
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", f"node{i + 1}",
                               "--config", str(cfg)], env=ENV, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True) for i in range(1, n)]
    try:
        r0 = subprocess.run([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", "node1", "--config",
                             str(cfg), *extra0], env=ENV, capture_output=True, text=True, timeout=timeout)
        outs = [p.communicate(timeout=120)[0] for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    ok = r0.returncode == 0 and all(p.returncode == 0 for p in procs)
    assert ok, r0.stdout[-3000:] + r0.stderr[-3000:] + "".join(o[-1500:] for o in outs)
    return r0.stdout


def _preds(out):
    line = [l for l in out.splitlines() if "***** FINAL PREDICTION (Index):" in l][-1]
    return json.loads(line.split("(Index):")[1].split("*****")[0].strip())


@pytest.mark.timeout(400)
def test_cifar_three_ranks_forward_pipeline_gloo_gpu(tmp_path):
    """CIFAR over 3 ranks on GPU 0 (conv | fc1 | fc2+softmax, ForwardPipeline,
    4 microbatches x 4 images, predictions over the back-edge to rank 0) ==
    the colocated pipeline's predictions (same kernels) and the fp32 golden
    where the golden's top-2 margin is decidable."""
    from PIL import Image
    from distributed_neural_networks_amd.cli import cifar_request
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    torch.manual_seed(21)
    m = NeuralNetwork().eval()
    pth = tmp_path / "cifar10_model.pth"
    torch.save(m.state_dict(), pth)
    img = tmp_path / "x.png"
    Image.fromarray(np.random.default_rng(1).integers(0, 255, (36, 36, 3), dtype=np.uint8)).save(img)
    common = dict(micro_batch_size=4, num_microbatches=4)
    dist_cfg = _cfg(tmp_path, "gloo_gpu", 3, "cifar10", str(pth), layers=[(0, 1), (2, 2), (3, 3)], **common)
    got = _preds(_run(dist_cfg, 3, ("--input_image", str(img), "--num_requests", "2", "--shutdown_pipeline")))
    col_cfg = _cfg(tmp_path, "colocated", 2, "cifar10", str(pth), **common)
    want = _preds(_run(col_cfg, 1, ("--input_image", str(img), "--num_requests", "2")))
    assert len(got) == 16 and got == want
    with torch.no_grad():
        p = m(cifar_request(type("A", (), {"input_image": str(img)})(), "t", 16, 1))
    top2 = p.topk(2, dim=1).values
    for i in range(16):
        if (top2[i, 0] - top2[i, 1]).item() > 1e-4:
            assert got[i] == int(p[i].argmax()), (i, got[i], p[i])


@pytest.mark.timeout(400)
def test_gpt2_tiny_decode_ring_four_ranks_gloo_gpu(tmp_path):
    """GPT-2-tiny decode ring over 4 ranks on GPU 0 (TransformerStage, one HIP
    graph per microbatch per rank, 4 microbatches x 2 sequences, tokens back
    to rank 0 over the back-edge) == the colocated ring's tokens, and the
    first token == the fp32 golden's greedy choice."""
    from distributed_neural_networks_amd.checkpoint import make_full_checkpoint
    pth = tmp_path / "gpt2_tiny.pth"
    make_full_checkpoint("gpt2-tiny", str(pth), 5)  # host-generated, so the golden sees the same weights
    common = dict(prompt_len=6, decode_steps=5, micro_batch_size=2, num_microbatches=4)
    dist_cfg = _cfg(tmp_path, "gloo_gpu", 4, "gpt2-tiny", str(pth), **common)
    out = _run(dist_cfg, 4)
    got = json.loads(out.split("generated tokens:")[1].strip().splitlines()[0])
    col_cfg = _cfg(tmp_path, "colocated", 4, "gpt2-tiny", str(pth), **common)
    want = json.loads(_run(col_cfg, 1).split("generated tokens:")[1].strip().splitlines()[0])
    assert len(got) == 8 and all(len(t) == 5 for t in got)
    assert got == want
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.config import load_node
    from distributed_neural_networks_amd.models import build_golden_stage
    from distributed_neural_networks_amd.runtime.generate import make_prompts
    prompts = make_prompts(load_node(str(dist_cfg), "node1").pipeline, None)
    g = build_golden_stage("gpt2-tiny", 0, 3, True, True)
    g.load_state_dict(ckpt.random_stage_state_dict("gpt2-tiny", 0, 3, True, True, 5))
    with torch.no_grad():
        last = g(prompts)[:, -1]
    top2 = last.topk(2, dim=-1).values
    for b in range(8):
        if (top2[b, 0] - top2[b, 1]).item() > 2e-2 * top2[b, 0].abs().item():
            assert got[b][0] == int(last[b].argmax()), (b, got[b], int(last[b].argmax()))
