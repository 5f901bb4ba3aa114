"""GPT-2 XL fp8, 2 blocks at full width: where does the W8A8 prefill differ
from the dequantised-weight golden?  Prints the last-position logits' relative
error of the device prefill (T = 24: W8A16, T = 64: W8A8) against the golden
without and with per-row e4m3 activation quantisation.

    python bench/probes/fp8_prefill_probe.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import test_transformer_gpu as T
    from distributed_neural_networks_amd import checkpoint as ckpt
    from distributed_neural_networks_amd.runtime.transformer import TransformerStage
    dev = torch.device("cuda")
    sd = ckpt.random_stage_state_dict("gpt2-xl", 0, 1, True, True, 17, device=dev, nontrivial=True)
    for Tn in (24, 192, 320):
        st = TransformerStage("gpt2-xl", sd, 0, 1, True, True, dev, max_batch=2, max_seq=Tn + 2, fp8=True)
        ids = torch.randint(0, 50257, (2, Tn), generator=torch.Generator().manual_seed(6))
        pos = torch.zeros(2, dtype=torch.int32, device=dev)
        out = st.step(ids.to(dev, torch.int32), pos, 2, Tn).probs.float()
        rec = {"T": Tn}
        for q in (False, True):
            g = T._gpt2_fp8_golden(st, sd)
            ref = g(ids.to(dev), 0, q)
            rec[f"rel_vs_golden_quant_act_{q}"] = round(T._rel(out, ref.float()), 5)
        print(json.dumps(rec), flush=True)
        del st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
