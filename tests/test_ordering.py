"""Debug slot-ordering checker (runtime/ordering.py): the illegal reuse
patterns of a microbatch slot ring raise, the legal schedule does not."""
import pytest

from distributed_neural_networks_amd.runtime.ordering import SlotOrder, SlotOrderError


def test_legal_ring_schedule():
    o = SlotOrder("out", 2, enabled=True)
    for i in range(6):
        k = i % 2
        if i >= 2:
            o.waited(k)  # the send of microbatch i-2 was waited on
        o.use(k, "write", i)
        o.post(k, "send", i)
    o.waited(0)
    o.waited(1)
    o.drained()
    assert o.events == 12


def test_write_before_send_wait_raises():
    o = SlotOrder("out", 2, enabled=True)
    o.post(0, "send", 0)
    with pytest.raises(SlotOrderError, match="has not been waited on"):
        o.use(0, "stage output write", 2)


def test_double_post_raises():
    o = SlotOrder("in", 1, enabled=True)
    o.post(0, "recv", 0)
    with pytest.raises(SlotOrderError, match="still in flight"):
        o.post(0, "recv", 1)


def test_never_waited_raises_at_drain():
    o = SlotOrder("in", 2, enabled=True)
    o.post(1, "recv", 3)
    with pytest.raises(SlotOrderError, match="never waited"):
        o.drained()


def test_disabled_is_noop():
    o = SlotOrder("in", 1, enabled=False)
    o.post(0, "recv", 0)
    o.post(0, "recv", 1)
    o.use(0, "read")
    o.drained()
