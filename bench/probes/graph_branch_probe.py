"""Do the parallel branches of one captured HIP graph run concurrently on this
ROCm?  Two ~N-cycle single-block spin kernels (torch.cuda._sleep) captured on
two forked streams vs on one stream; prints replay times (us)."""
import json
import time

import torch


def timed(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    cyc = 200000
    s0 = torch.cuda.Stream()
    s1 = torch.cuda.Stream()
    out = {}
    # serial
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s0):
        torch.cuda._sleep(cyc)
        torch.cuda._sleep(cyc)
    out["serial_us"] = timed(g)
    # forked
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s0):
        s1.wait_stream(s0)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        s0.wait_stream(s1)
    out["forked_us"] = timed(g2)
    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g3, stream=s0):
        torch.cuda._sleep(cyc)
    out["single_us"] = timed(g3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
