"""Worker of tests/test_native_comm_gpu.py::test_pair_channel_two_processes:
rank ``argv[1]`` of a 2-process gloo group (the TCP store bootstraps the RCCL
pair channel), both ranks on GPU 0.  Writes one result line to ``argv[3]``:
``ok <checksum>``, ``init_error <msg>`` (RCCL refusing two ranks on one GPU
is a legal outcome) or ``fail <msg>``."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    rank, port, out = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    dist.init_process_group("gloo", rank=rank, world_size=2, init_method=f"tcp://127.0.0.1:{port}")
    from distributed_neural_networks_amd.parallel import rccl
    dev = torch.device("cuda", rank % max(1, torch.cuda.device_count()))  # one GPU per rank when there are two
    torch.cuda.set_device(dev)
    res = "fail unknown"
    try:
        ch = rccl.pair_channel(rank, 1 - rank, dev)
        try:
            ch.ready(60)
        except (RuntimeError, TimeoutError) as e:
            res = f"init_error {e}"
            ch.abort()
            return 0
        # several messages, 4 B .. 24 MiB + odd tails, all in flight at once,
        # then the reverse direction; every byte checked on the receiver
        sizes = [1, (1 << 20) + 5, 7, (6 << 20) + 3, 4096, 3 << 20]
        bad = 0
        for direction in (0, 1):
            sender = direction
            bufs, toks = [], []
            for i, n in enumerate(sizes):
                ref = (torch.arange(n, device=dev, dtype=torch.int32) * (3 + i) + direction) % 1000003
                if rank == sender:
                    bufs.append(ref)
                    toks.append(ch.post(rccl.SEND, ref, 1 - rank))
                else:
                    b = torch.full((n,), -1, device=dev, dtype=torch.int32)
                    bufs.append((b, ref))
                    toks.append(ch.post(rccl.RECV, b, 1 - rank))
            try:
                for t in toks:
                    ch.synchronize(t, 60)
            except TimeoutError as e:
                ch.abort()
                res = f"fail {e}"
                return 1
            torch.cuda.synchronize()
            if rank != sender:
                bad += sum(int((b != ref).sum().item()) for b, ref in bufs)
        res = "ok " + str(bad)
        ch.destroy()
        return 0
    except Exception as e:  # noqa: BLE001
        res = f"fail {type(e).__name__}: {e}"
        return 1
    finally:
        with open(out, "w") as f:
            f.write(res + "\n")
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
