"""Write a random-init full-model checkpoint with the reference key layout.

The reference's ``cifar10_model.pth`` is not shipped (``.MISSING_LARGE_BLOBS``)
and there is no network; this produces a drop-in file:

    python -m distributed_neural_networks_amd.tools.make_checkpoint --model cifar10 --out cifar10_model.pth
"""
import argparse

from ..checkpoint import make_full_checkpoint


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="cifar10")
    ap.add_argument("--out", default="cifar10_model.pth")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    make_full_checkpoint(a.model, a.out, a.seed)
    print(f"wrote {a.out} ({a.model}, seed {a.seed})")


if __name__ == "__main__":
    main()
