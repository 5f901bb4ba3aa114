"""Worker of tests/test_native_comm_gpu.py::test_native_preflight_two_processes:
rank ``argv[1]`` of a 2-process nccl group, both ranks on GPU 0 (RCCL
refuses two ranks on one device, so the native ring check is expected to
fail and fall back).  Writes ``<mode>|<DNN_P2P after>`` to ``argv[3]``."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    rank, port, out = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # lazy ProcessGroupNCCL: no communicator is created unless a collective runs
    dist.init_process_group("nccl", rank=rank, world_size=2, init_method=f"tcp://127.0.0.1:{port}")
    from distributed_neural_networks_amd.parallel.links import native_preflight
    res = "fail unknown"
    try:
        mode = native_preflight(dev, timeout_s=40)
        res = f"{mode}|{os.environ.get('DNN_P2P', 'native')}"
        return 0
    except Exception as e:  # noqa: BLE001
        res = f"fail {type(e).__name__}: {e}"
        return 1
    finally:
        with open(out, "w") as f:
            f.write(res + "\n")
        os._exit(0)  # skip process-group teardown of a group whose RCCL channels were aborted


if __name__ == "__main__":
    sys.exit(main())
