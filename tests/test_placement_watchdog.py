"""Placement planning (parallel/partition.py linear_plan / linear_role) and the
failure watchdog's detection logic (parallel/watchdog.py), in-process on CPU."""
import datetime
import socket
import time

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from distributed_neural_networks_amd.parallel.partition import linear_plan, linear_role


@given(world=st.integers(2, 16), prec=st.sampled_from(["fp32", "bf16"]))
@settings(max_examples=60, deadline=None)
def test_linear_plan_roles_cover_every_rank(world, prec):
    plan = linear_plan(world, prec)
    assert plan["n0"] + plan["n1"] == world and plan["n0"] >= 1 and plan["n1"] >= 1
    roles = [linear_role(r, plan) for r in range(world)]
    senders = [r for r, ro in enumerate(roles) if ro["stage"] == 0]
    receivers = [r for r, ro in enumerate(roles) if ro["stage"] == 1]
    assert len(senders) == plan["n0"] and len(receivers) == plan["n1"]
    # every sender feeds exactly one receiver, which lists it
    for s in senders:
        dst = roles[s]["send_to"]
        assert roles[dst]["stage"] == 1 and s in roles[dst]["recv_from"]
    assert sorted(x for r in receivers for x in roles[r]["recv_from"]) == senders
    # fan-in balanced within one sender
    loads = [len(roles[r]["recv_from"]) for r in receivers]
    assert max(loads) - min(loads) <= 1


def test_linear_plan_replicates_the_bottleneck_stage():
    # fp32 CIFAR: stage 0 (conv + fc1) is ~99 % of the compute after the fc1 cut
    p8 = linear_plan(8, "fp32")
    assert p8["cut"] == 2 and (p8["n0"], p8["n1"]) == (7, 1)
    # a balanced synthetic model splits evenly
    p = linear_plan(8, unit_ns=(0.0, 10.0, 10.0, 0.0), boundary_bytes=(0, 10, 10, 0), cuts=(1,))
    assert (p["n0"], p["n1"]) == (4, 4)
    # a link-bound cut loses to a compute-bound one
    p = linear_plan(2, unit_ns=(0.0, 10.0, 10.0, 1.0), boundary_bytes=(0, 10 ** 6, 10, 0), cuts=(1, 2))
    assert p["cut"] == 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def store_port():
    import torch.distributed as dist
    port = _free_port()
    master = dist.TCPStore("127.0.0.1", port, is_master=True, timeout=datetime.timedelta(seconds=10),
                           wait_for_workers=False)
    yield port
    del master


def _wd(rank, world, port, **kw):
    from distributed_neural_networks_amd.parallel.watchdog import Watchdog
    exits = []
    w = Watchdog(rank, world, "127.0.0.1", port, interval_s=0.1, exit_fn=exits.append, **kw)
    return w, exits


def test_watchdog_detects_silent_peer(store_port):
    a, ea = _wd(0, 2, store_port, peer_timeout_s=0.8)
    b, eb = _wd(1, 2, store_port, peer_timeout_s=0.8)
    a.start()
    b.start()
    time.sleep(0.5)
    assert not ea and not eb
    b._stop.set()  # rank 1 stops beating (as if killed)
    t0 = time.time()
    while not ea and time.time() - t0 < 5:
        time.sleep(0.05)
    assert ea == [3] and "no heartbeat from rank 1" in a.aborted
    b.stop()
    a.stop()  # rank 0 last: it lingers until every rank has stopped


def test_watchdog_abort_propagates_and_done_is_not_a_crash(store_port):
    a, ea = _wd(0, 3, store_port, peer_timeout_s=0.6)
    b, eb = _wd(1, 3, store_port, peer_timeout_s=0.6)
    c, ec = _wd(2, 3, store_port, peer_timeout_s=0.6)
    for w in (a, b, c):
        w.start()
    time.sleep(0.3)
    c.done()          # rank 2 finished cleanly ...
    c.stop()          # ... and went quiet: not a failure
    time.sleep(1.2)
    assert not ea and not eb
    b.abort("injected")  # rank 1 fails: rank 0 must follow
    t0 = time.time()
    while not ea and time.time() - t0 < 5:
        time.sleep(0.05)
    assert eb == [3] and ea == [3] and "injected" in a.aborted
    b.stop()
    a.stop()  # rank 0 last: it lingers until every rank has stopped


def test_watchdog_local_stall(store_port):
    a, ea = _wd(0, 2, store_port, peer_timeout_s=30, stall_timeout_s=0.5)
    b, eb = _wd(1, 2, store_port, peer_timeout_s=30)
    a.start()
    b.start()
    a.busy(True)
    for _ in range(5):  # progressing: no abort
        time.sleep(0.15)
        a.beat()
    assert not ea
    time.sleep(1.2)    # stalled
    assert ea == [3] and "no pipeline progress" in a.aborted
    b.stop()
    a.stop()  # rank 0 last: it lingers until every rank has stopped
