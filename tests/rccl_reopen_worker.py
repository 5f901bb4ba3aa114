"""Worker of tests/test_native_comm_cpu.py::test_pair_channel_reopen_two_processes:
rank ``argv[1]`` of a 2-process pair sharing a real TCPStore (rank 0 hosts it
on port ``argv[2]``).  Both ranks open and scope-close the (world, 0-1) pair
channel ``argv[4]`` times with a stand-in Channel that records the unique id
it would hand to ``ncclCommInitRank``; the lower rank draws a fresh id per
open and waits before each reopen, so a higher rank that read a stale store
key would record the previous id.  Writes the ids (hex, one per line) to
``argv[3]``.  No device is touched."""
import os
import sys
import time
from datetime import timedelta

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _RecordingChannel:
    def __init__(self, uid, nranks, rank, device, key=None, uid_fn=None):
        # the real Channel reads the id on its init thread; here synchronously
        self.uid = bytes(uid if uid is not None else uid_fn())
        self.key, self.device, self.closed = key, device, False

    def abort(self):
        pass

    def destroy(self):
        self.closed = True


class _Lib:
    @staticmethod
    def comm_unique_id():
        return os.urandom(128)


def main() -> int:
    rank, port, out, n = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    st = dist.TCPStore("127.0.0.1", port, 2, rank == 0, timeout=timedelta(seconds=30))
    from distributed_neural_networks_amd.parallel import rccl
    rccl.Channel = _RecordingChannel
    rccl._lib = lambda: _Lib
    dev = torch.device("cpu")
    uids = []
    for i in range(n):
        if rank == 0:
            time.sleep(0.3)  # the higher rank reaches its reopen first
        with rccl.scope(dev):
            ch = rccl.pair_channel(rank, 1 - rank, dev, "world", store=st)
            uids.append(ch.uid.hex())
    st.set(f"done/{rank}", "1")
    st.get(f"done/{1 - rank}")
    # the store host (rank 0) outlives the other rank's last store call: rank 1
    # says goodbye after its reads, rank 0 waits for that and a little longer
    if rank == 1:
        st.set("bye/1", "1")
    else:
        st.get("bye/1")
        time.sleep(0.5)
    with open(out, "w") as f:
        f.write("\n".join(uids))
    return 0


if __name__ == "__main__":
    sys.exit(main())
