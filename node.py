#!/usr/bin/env python3
"""Pipeline-stage node — same CLI as the reference ``node.py``:

    python node.py --node_id node1 --config config.json [--input_image img.png]

See ``distributed_neural_networks_amd/cli.py`` for transports and extra flags.
"""
import sys

from distributed_neural_networks_amd.cli import main

if __name__ == "__main__":
    sys.exit(main())
