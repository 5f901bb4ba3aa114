"""Multi-GPU paths over RCCL/xGMI: one process per GPU,
launched the way the driver and users launch them.  Skipped below 2 visible
GPUs (conftest: ``multigpu``); RCCL refuses two ranks on one device, so the
1-GPU box cannot run these — the same schedules run on gloo in
``test_distributed_cpu.py``.  Each test keeps to <= 4 ranks and small shapes."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.multigpu]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(n, script, *args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, script), *args]
    r = subprocess.run(cmd, env=ENV, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("placement", ["interleaved", "linear"])
def test_bench_cifar_two_gpus(placement):
    """The flagship bench on 2 GPUs (RCCL all-to-all / isend-irecv hops)."""
    out = _torchrun(2, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "8192",
                    "--placement", placement, "--latency_iters", "5")
    d = out[-1]
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["metric"] == "images/sec CIFAR-10 2-stage"


def test_bench_gpt2_pipeline_two_gpus():
    """GPT-2 small, 4 stages over 2 GPU groups: prefill + microbatched ring decode."""
    out = _torchrun(2, "bench.py", "--model", "gpt2", "--gpus", "2", "--steps", "4", "--warmup", "1")
    assert out[-1]["n_gpus"] == 2 and out[-1]["value"] > 0


def test_cli_rccl_two_stage(tmp_path):
    """node.py CLI on configs/cifar_2gpu_rccl.json: one stage per GPU, RCCL P2P."""
    from distributed_neural_networks_amd.tools import make_checkpoint
    ck = tmp_path / "cifar10_model.pth"
    make_checkpoint.main(["--out", str(ck)])
    cfg = json.load(open(os.path.join(ROOT, "configs", "cifar_2gpu_rccl.json")))
    cfg["model_weights"] = str(ck)
    for i, n in enumerate(cfg["nodes"]):
        n["address"] = f"127.0.0.1:{_port()}"
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    r = subprocess.run([sys.executable, "-m", "distributed_neural_networks_amd.tools.launch", "--config", str(p),
                        "--num_requests", "3", "--timeout", "240"], env=ENV, capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "FINAL PREDICTION" in r.stdout + r.stderr
