"""Microbatch schedules (runtime/scheduler.py) on CPU with gloo: correctness
against the fp32 golden, real stage overlap (trace-based), the CLI wiring of
``micro_batch_size`` / ``num_microbatches``, and failure detection
(parallel/watchdog.py).  Same schedule code as the RCCL path on MI355X."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest
import torch

from test_distributed_cpu import ENV, ROOT, _cfg, _write_image, free_port


# ----------------------------------------------------------------------------- helpers
class SleepStage:
    """A stage whose forward takes a fixed wall time (deterministic overlap)."""

    def __init__(self, first, last, ms, width=8):
        from distributed_neural_networks_amd.runtime.stages import StageCompute  # noqa: F401
        self.first, self.last, self.device, self.ms, self.w = first, last, torch.device("cpu"), ms, width

    def in_spec(self, b):
        return (b, self.w), torch.float32

    def out_spec(self, b):
        return ((b, 10) if self.last else (b, self.w)), torch.float32

    def forward(self, x, out=None):
        from distributed_neural_networks_amd.runtime.stages import StageOutput
        time.sleep(self.ms / 1e3)
        if self.last:
            probs = out if out is not None else torch.empty(x.shape[0], 10)
            probs.zero_()
            probs[:, 0] = x[:, 0]
            return StageOutput(probs, x[:, 0].to(torch.int32))
        y = x + 1
        if out is not None:
            out.copy_(y)
            return out
        return y


def _overlap_worker(rank, world, port, trace_dir, M):
    os.environ["DNN_DEBUG_ORDER"] = "1"
    from distributed_neural_networks_amd.parallel import comm
    from distributed_neural_networks_amd.parallel.links import P2PLink
    from distributed_neural_networks_amd.runtime.scheduler import run_gpipe
    from distributed_neural_networks_amd.utils import trace
    torch.set_num_threads(1)
    info = comm.init("gloo", rank=rank, world=world, master_addr="127.0.0.1", master_port=port)
    trace.enable(os.path.join(trace_dir, f"rank{rank}.json"))
    st = SleepStage(rank == 0, rank == world - 1, 60)
    prev = P2PLink(rank - 1, info.device) if rank > 0 else None
    nxt = P2PLink(rank + 1, info.device) if rank < world - 1 else None
    xs = [torch.full((4, 8), float(i)) for i in range(M)]
    got = {}
    comm.barrier(info)
    run_gpipe(st, M, 4, prev, nxt, source=lambda i: xs[i],
              sink=(lambda i, y: got.__setitem__(i, y.pred.clone())) if rank == world - 1 else None)
    trace.flush()
    if rank == world - 1:
        # every stage adds 1, the last copies column 0: pred = i + (world - 1)
        for i in range(M):
            assert got[i].tolist() == [i + world - 1] * 4, (i, got[i])
    comm.barrier(info)
    comm.shutdown()


def _spawn(target, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=target, args=(r, world) + args) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(180)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]


def _spans(path, name):
    d = json.load(open(path))
    e0 = d["otherData"]["epoch_t0_us"]
    return {e["args"]["mb"]: (e0 + e["ts"], e0 + e["ts"] + e["dur"]) for e in d["traceEvents"]
            if e.get("name") == name}


def test_gpipe_stages_overlap_in_trace(tmp_path):
    """Stage i computes microbatch k while stage i+1 computes k-1 (from the
    per-rank Chrome traces on one wall clock), and the steady state is the
    pipelined time, not the serial one."""
    world, M = 3, 6
    _spawn(_overlap_worker, world, free_port(), str(tmp_path), M)
    spans = [_spans(tmp_path / f"rank{r}.json", "stage_forward") for r in range(world)]
    overlaps = 0
    for i in range(world - 1):
        for k in range(1, M):
            a0, a1 = spans[i][k]
            b0, b1 = spans[i + 1][k - 1]
            if min(a1, b1) - max(a0, b0) > 20e3:  # > 20 ms of a 60 ms compute
                overlaps += 1
    assert overlaps >= (world - 1) * (M - 1) - 2, overlaps
    t_first = min(s[0] for s in spans[0].values())
    t_last = max(s[1] for s in spans[-1].values())
    serial = world * M * 60e3
    assert t_last - t_first < 0.75 * serial, (t_last - t_first, serial)


# ----------------------------------------------------------------------------- CLI: GPT decode ring
def _run_all(cfg, n, extra0=(), timeout=240):
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", f"node{i + 1}",
                               "--config", str(cfg)], env=ENV, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True) for i in range(1, n)]
    try:
        r0 = subprocess.run([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", "node1", "--config", str(cfg),
                             *extra0], env=ENV, capture_output=True, text=True, timeout=timeout)
        outs = [p.communicate(timeout=120)[0] for p in procs]
        return r0, outs, [p.returncode for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


def _golden_tokens(model, n_layers, seed, prompt, steps):
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models import build_golden_stage
    s = build_golden_stage(model, 0, n_layers - 1, True, True)
    s.load_state_dict(ckpt.random_stage_state_dict(model, 0, n_layers - 1, True, True, seed))
    seq = torch.tensor(prompt)
    with torch.no_grad():
        for _ in range(steps):
            nid = s(seq)[:, -1].argmax(-1)
            seq = torch.cat([seq, nid[:, None]], 1)
    return seq[:, len(prompt[0]):].tolist()


def test_cli_gpt2_tiny_4_stages_4_microbatches_gloo(tmp_path):
    """4 ranks x 4 microbatches of 2 sequences on the decode ring (tokens return
    to stage 0 over the back-edge) == fp32 greedy golden, token for token."""
    cfg = _cfg(tmp_path, "gloo", 4, model="gpt2-tiny", weights="synthetic:5", prompt_len=6, decode_steps=5,
               micro_batch_size=2, num_microbatches=4)
    r0, outs, rcs = _run_all(cfg, 4)
    assert r0.returncode == 0 and all(rc == 0 for rc in rcs), r0.stdout[-3000:] + "".join(o[-1500:] for o in outs)
    toks = json.loads(r0.stdout.split("generated tokens:")[1].strip().splitlines()[0])
    assert len(toks) == 8 and all(len(t) == 5 for t in toks)
    from distributed_neural_networks_amd.runtime.generate import make_prompts
    from distributed_neural_networks_amd.config import load_node
    prompts = make_prompts(load_node(str(cfg), "node1").pipeline, None).tolist()
    assert toks == _golden_tokens("gpt2-tiny", 4, 5, prompts, 5)
    m = json.loads([l for l in r0.stdout.splitlines() if l.startswith("METRICS ")][0][len("METRICS "):])
    assert m["microbatches"] == 4 and m["ring_groups"] == 4 and m["decode_tokens_per_s"] > 0


def test_cli_llama_tiny_colocated_microbatches_cpu(tmp_path):
    """Colocated transport, M = 3 microbatches, reports tokens/s; CPU golden stages."""
    cfg = _cfg(tmp_path, "colocated", 2, model="llama3-tiny", weights="synthetic:2", prompt_len=5, decode_steps=4,
               micro_batch_size=2, num_microbatches=3)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", "node1", "--config", str(cfg)],
                       env=ENV, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    toks = json.loads(r.stdout.split("generated tokens:")[1].strip().splitlines()[0])
    from distributed_neural_networks_amd.runtime.generate import make_prompts
    from distributed_neural_networks_amd.config import load_node
    prompts = make_prompts(load_node(str(cfg), "node1").pipeline, None).tolist()
    assert toks == _golden_tokens("llama3-tiny", 4, 2, prompts, 4)
    m = json.loads([l for l in r.stdout.splitlines() if l.startswith("METRICS ")][0][len("METRICS "):])
    assert m["microbatches"] == 3 and m["decode_tokens_per_s"] > 0


# ----------------------------------------------------------------------------- CLI: CIFAR microbatched stream
def test_cli_cifar_3_stages_microbatched_gloo(tmp_path):
    """3 ranks, requests of micro_batch_size x num_microbatches = 2 x 3 rows:
    every row's prediction returns to node1 and equals the golden model's."""
    from distributed_neural_networks_amd.checkpoint import make_full_checkpoint
    from distributed_neural_networks_amd.cli import cifar_request
    from distributed_neural_networks_amd.models.cifar import NeuralNetwork
    ck = tmp_path / "c.pth"
    make_full_checkpoint("cifar10", str(ck), 4)
    img = tmp_path / "i.png"
    _write_image(str(img))
    cfg = _cfg(tmp_path, "gloo", 3, weights=str(ck), micro_batch_size=2, num_microbatches=3)
    r0, outs, rcs = _run_all(cfg, 3, ("--input_image", str(img), "--num_requests", "2"))
    assert r0.returncode == 0 and all(rc == 0 for rc in rcs), r0.stdout[-3000:] + "".join(o[-1500:] for o in outs)
    lines = [l for l in r0.stdout.splitlines() if "***** FINAL PREDICTION (Index):" in l]
    assert len(lines) == 2
    m = NeuralNetwork().eval()
    m.load_state_dict(torch.load(str(ck), weights_only=True))

    class A:
        input_image = str(img)
    for req, line in enumerate(lines):
        got = json.loads(line.split("(Index):")[1].split("*****")[0].strip())
        with torch.no_grad():
            ref = m(cifar_request(A, "t", 6, req)).argmax(1).tolist()
        assert got == ref
    assert any("Final Prediction Index:" in o for o in outs)


def test_cli_return_to_middle_stage_gloo(tmp_path):
    """return_to_node_id naming a middle stage: predictions arrive there (the
    round-1 CLI sent them to a rank that never received, and hung)."""
    from distributed_neural_networks_amd.checkpoint import make_full_checkpoint
    ck = tmp_path / "c.pth"
    make_full_checkpoint("cifar10", str(ck), 4)
    img = tmp_path / "i.png"
    _write_image(str(img))
    cfg = _cfg(tmp_path, "gloo", 3, weights=str(ck), return_to_node_id="node2")
    r0, outs, rcs = _run_all(cfg, 3, ("--input_image", str(img)), timeout=120)
    assert r0.returncode == 0 and all(rc == 0 for rc in rcs), r0.stdout[-2000:] + "".join(o[-1500:] for o in outs)
    assert "FINAL PREDICTION" in outs[0]  # node2


# ----------------------------------------------------------------------------- failure detection
def test_killed_middle_stage_aborts_pipeline_gloo(tmp_path):
    """Kill the middle rank of a 3-stage gloo stream mid-run: stage 0 must exit
    non-zero within ~30 s (heartbeat watchdog / transport error), not hang for
    the 300 s process-group timeout."""
    from distributed_neural_networks_amd.checkpoint import make_full_checkpoint
    ck = tmp_path / "c.pth"
    make_full_checkpoint("cifar10", str(ck), 4)
    img = tmp_path / "i.png"
    _write_image(str(img))
    cfg = _cfg(tmp_path, "gloo", 3, weights=str(ck), heartbeat_timeout_s=5, micro_batch_size=4,
               num_microbatches=2)
    p = {}
    for i in (2, 3):
        p[i] = subprocess.Popen([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", f"node{i}",
                                 "--config", str(cfg), "--quiet"], env=ENV, stdout=subprocess.PIPE,
                                stderr=subprocess.STDOUT, text=True)
    p[1] = subprocess.Popen([sys.executable, os.path.join(ROOT, "node.py"), "--node_id", "node1", "--config",
                             str(cfg), "--input_image", str(img), "--num_requests", "1000000"], env=ENV,
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        deadline = time.time() + 120
        seen = ""
        while time.time() < deadline:
            line = p[1].stdout.readline()
            seen += line
            if "FINAL PREDICTION" in line:
                break
        assert "FINAL PREDICTION" in seen, seen[-2000:]
        p[2].send_signal(signal.SIGKILL)
        t_kill = time.time()
        rc = p[1].wait(timeout=60)
        elapsed = time.time() - t_kill
        assert rc != 0, rc
        assert elapsed < 30, elapsed
        rc3 = p[3].wait(timeout=60)
        assert rc3 != 0
    finally:
        for q in p.values():
            if q.poll() is None:
                q.kill()
                q.wait()


def test_cli_chunked_prefill_gloo(tmp_path):
    """Chunked prefill (prefill_chunk = 6 of a 20-token prompt, 2 microbatches,
    2 ranks): the chunks attend to the cache written by the earlier ones, so
    the greedy tokens equal the full-prompt golden."""
    cfg = _cfg(tmp_path, "gloo", 2, model="gpt2-tiny", weights="synthetic:8", prompt_len=20, decode_steps=4,
               micro_batch_size=2, num_microbatches=2, prefill_chunk=6)
    r0, outs, rcs = _run_all(cfg, 2)
    assert r0.returncode == 0 and all(rc == 0 for rc in rcs), r0.stdout[-3000:] + "".join(o[-1500:] for o in outs)
    toks = json.loads(r0.stdout.split("generated tokens:")[1].strip().splitlines()[0])
    from distributed_neural_networks_amd.config import load_node
    from distributed_neural_networks_amd.runtime.generate import make_prompts
    prompts = make_prompts(load_node(str(cfg), "node1").pipeline, None).tolist()
    assert toks == _golden_tokens("gpt2-tiny", 4, 8, prompts, 4)


def _ring_resume_worker(rank, world, port, q):
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models import default_ranges
    from distributed_neural_networks_amd.parallel import comm
    from distributed_neural_networks_amd.parallel.links import P2PLink
    from distributed_neural_networks_amd.runtime.scheduler import DecodeRing, RingLinks
    from distributed_neural_networks_amd.runtime.stages import TorchStage
    torch.set_num_threads(1)
    info = comm.init("gloo", rank=rank, world=world, master_addr="127.0.0.1", master_port=port)
    bg = comm.back_group()
    a, b = default_ranges("gpt2-tiny", world)[rank]
    first, last = rank == 0, rank == world - 1
    st = TorchStage("gpt2-tiny", ckpt.random_stage_state_dict("gpt2-tiny", a, b, first, last, 5), a, b, first, last)
    links = RingLinks(prev=P2PLink(rank - 1, info.device) if rank > 0 else None,
                      nxt=P2PLink(rank + 1, info.device) if not last else None,
                      back_out=P2PLink(0, info.device, bg) if last else None,
                      back_in=P2PLink(world - 1, info.device, bg) if first else None)
    ring = DecodeRing([st], links, world, 2, 2)
    g = torch.Generator().manual_seed(9)
    prompts = [torch.randint(0, 512, (2, 5), generator=g) for _ in range(2)] if first else None
    ring.prefill(prompts, 5)
    for _ in range(2):
        ring.decode_round()
    ring.drain()
    for _ in range(3):  # microbatch 0 alone (the per-token latency rounds of bench/gpt_bench.py)
        ring.decode_round([0])
    ring.drain()
    if first:
        q.put(([p.tolist() for p in prompts], [torch.stack(t, 1).tolist() for t in ring.toks]))
    comm.barrier(info)
    comm.shutdown()


def test_decode_ring_single_microbatch_resume_gloo():
    """After a drain, ``decode_round([0])`` lets microbatch 0 circulate alone
    through 3 gloo ranks (tokens over the back-edge communicator); its tokens
    continue the golden greedy sequence and microbatch 1 stays where it was."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_ring_resume_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    prompts, toks = q.get(timeout=180)
    for p in ps:
        p.join(60)
    assert len(toks[0][0]) == 6 and len(toks[1][0]) == 3
    assert toks[0] == _golden_tokens("gpt2-tiny", 4, 5, prompts[0], 6)
    assert toks[1] == _golden_tokens("gpt2-tiny", 4, 5, prompts[1], 3)


def _ring_prepost_worker(rank, world, port, q, M, rounds):
    os.environ["DNN_DEBUG_ORDER"] = "1"  # every slot transition of the pre-posted receives is checked
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models import default_ranges
    from distributed_neural_networks_amd.parallel import comm
    from distributed_neural_networks_amd.parallel.links import P2PLink
    from distributed_neural_networks_amd.runtime.scheduler import DecodeRing, RingLinks
    from distributed_neural_networks_amd.runtime.stages import TorchStage
    torch.set_num_threads(1)
    info = comm.init("gloo", rank=rank, world=world, master_addr="127.0.0.1", master_port=port)
    bg = comm.back_group()
    a, b = default_ranges("gpt2-tiny", world)[rank]
    first, last = rank == 0, rank == world - 1
    st = TorchStage("gpt2-tiny", ckpt.random_stage_state_dict("gpt2-tiny", a, b, first, last, 5), a, b, first, last)
    links = RingLinks(prev=P2PLink(rank - 1, info.device) if rank > 0 else None,
                      nxt=P2PLink(rank + 1, info.device) if not last else None,
                      back_out=P2PLink(0, info.device, bg) if last else None,
                      back_in=P2PLink(world - 1, info.device, bg) if first else None)
    ring = DecodeRing([st], links, world, M, 2)
    assert ring.rorder.enabled
    g = torch.Generator().manual_seed(9)
    prompts = [torch.randint(0, 512, (2, 5), generator=g) for _ in range(M)] if first else None
    ring.prefill(prompts, 5)
    ring.decode_rounds(rounds)
    ring.drain()
    ring.decode_round([0])   # a lone single-microbatch round (the bench's latency rounds) between two runs
    ring.drain()
    ring.decode_rounds(2)
    ring.drain()
    if first:
        q.put(([p.tolist() for p in prompts], [torch.stack(t, 1).tolist() for t in ring.toks]))
    comm.barrier(info)
    comm.shutdown()


@pytest.mark.parametrize("world,M", [(3, 6), (2, 1), (4, 4)])
def test_decode_ring_preposted_receives_gloo(world, M):
    """decode_rounds posts the next microbatch's receive (hidden states, or the
    token over the back-edge on group 0) before launching this microbatch:
    with M > G, M = G and M = 1 (no pre-post possible), interleaved with a
    single-microbatch round, every sequence's greedy tokens equal the golden
    and DNN_DEBUG_ORDER finds no slot reused under a pending receive."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    rounds = 3
    ps = [ctx.Process(target=_ring_prepost_worker, args=(r, world, port, q, M, rounds)) for r in range(world)]
    for p in ps:
        p.start()
    prompts, toks = q.get(timeout=240)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for m in range(M):
        n = 1 + rounds + (1 if m == 0 else 0) + 2
        assert len(toks[m][0]) == n
        assert toks[m] == _golden_tokens("gpt2-tiny", 4, 5, prompts[m], n)
