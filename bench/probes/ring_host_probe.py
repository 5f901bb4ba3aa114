"""Host issue cost of the decode ring per microbatch item vs its device time
(VERDICT r4 item 7): can one Python rank keep its GPU busy at N = 4 / 8?

One rank of a multi-GPU decode ring does, per microbatch item
(``runtime/scheduler.py DecodeRing.decode_rounds``): wait on the input
receive, post the next microbatch's receive, replay the microbatch's HIP
graph, post the send, and the SlotOrder bookkeeping.  Here the rank's stage
group of the N-GPU placement (a middle group: hidden states in and out) runs
on this GPU with zero-cost fake links, so

* host us / item  = wall time of ``decode_rounds`` with no device sync inside,
  while the device is still behind (the host's issue rate);
* device us / item = wall time per item of the same rounds including the
  final sync (with the host ahead, this is the device's rate).

If the host cost per item is well under the device cost, the host keeps the
GPU fed and capturing recv -> stage -> send into one graph would buy nothing.

    python bench/probes/ring_host_probe.py [--items 256]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


class _Work:
    def wait(self):
        return True


class FakeLink:
    """A link whose transfers cost nothing (the buffers keep their contents)."""

    def isend(self, t):
        return _Work()

    def irecv(self, t):
        return _Work()


def probe(model: str, stages: int, n_gpus: int, batch: int, fp8: bool, items: int, prompt: int = 512) -> dict:
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.models import default_ranges
    from distributed_neural_networks_amd.runtime.scheduler import DecodeRing, RingLinks
    from distributed_neural_networks_amd.runtime.transformer import TransformerStage
    dev = torch.device("cuda", 0)
    ranges = default_ranges(model, stages)
    groups = min(n_gpus, stages)
    per = stages // groups
    g = 1 if groups > 2 else 0  # a middle group (group 0 / last hold the embedding / head)
    ids = list(range(g * per, (g + 1) * per))
    M = groups  # the bench's microbatches per ring
    S = prompt + items // M + 8
    st = []
    for s in ids:
        a, b = ranges[s]
        sd = ckpt.random_stage_state_dict(model, a, b, s == 0, s == stages - 1, 0, device=dev)
        st.append(TransformerStage(model, sd, a, b, s == 0, s == stages - 1, dev, max_batch=batch * M, max_seq=S,
                                   fp8=fp8))
        del sd
    links = RingLinks(prev=FakeLink() if not st[0].first else None, nxt=FakeLink() if not st[-1].last else None,
                      back_out=FakeLink() if st[-1].last and groups > 1 else None,
                      back_in=FakeLink() if st[0].first and groups > 1 else None)
    ring = DecodeRing(st, links, groups, M, batch, use_graphs=True, record=False)
    for m in range(M):
        ring.pos[m].fill_(prompt)
        if ring.xin is not None:
            ring.xin[m].normal_()
    if ring.first and groups > 1:
        ring.pending = [True] * M
    ring.capture()
    rounds = max(2, items // M)
    ring.decode_rounds(4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ring.decode_rounds(rounds)
    t1 = time.perf_counter()  # host done issuing; the device is behind
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = rounds * M
    host_us, dev_us = (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6
    return {"model": model, "stages": stages, "n_gpus": n_gpus, "group": g, "stages_on_rank": ids,
            "micro_batch": batch, "microbatches": M, "fp8": fp8, "items": n,
            "host_us_per_item": round(host_us, 2), "device_us_per_item": round(dev_us, 2),
            "host_share": round(host_us / dev_us, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=256)
    a = ap.parse_args()
    cases = [("gpt2", 4, 4, 64, False), ("gpt2", 4, 2, 64, False), ("llama3-8b", 8, 8, 32, False),
             ("gpt2-xl", 8, 8, 64, True), ("llama3-8b", 8, 4, 32, False)]
    for c in cases:
        print(json.dumps(probe(*c, items=a.items)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
