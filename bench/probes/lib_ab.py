"""A/B of two builds of the kernel library in one GPU session: runs the same
bench command alternately with ``DNN_HIP_LIB=<A .so>`` and the in-tree build
(B), ``--rounds`` times each, and prints one JSON line per run with the keys
named by ``--keys`` from the bench's last JSON line.

    python bench/probes/lib_ab.py --a ab_old/_dnn_hip...so --keys prefill_tokens_per_s,ms_per_step \\
        -- python bench/gpt_bench.py --model gpt2 ...
"""
import argparse
import json
import os
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", required=True, help="library file of arm A (B = the in-tree build)")
    ap.add_argument("--keys", default="prefill_tokens_per_s,ms_per_step")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--tag", default="")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    keys = a.keys.split(",")
    for r in range(a.rounds):
        for arm in ("A", "B"):
            env = dict(os.environ)
            env.pop("DNN_HIP_LIB", None)
            if arm == "A":
                env["DNN_HIP_LIB"] = os.path.abspath(a.a)
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
            lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
            rec = {"tag": a.tag, "arm": arm, "round": r, "rc": p.returncode}
            if lines:
                d = json.loads(lines[-1])
                rec.update({k: d.get(k) for k in keys})
            else:
                rec["stderr"] = p.stderr[-600:]
            print(json.dumps(rec), flush=True)
            if p.returncode != 0:
                sys.exit(p.returncode)


if __name__ == "__main__":
    main()
