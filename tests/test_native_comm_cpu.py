"""CPU-side checks of the native RCCL data plane's plumbing (the device path is
tests/test_native_comm_gpu.py)."""
import pytest
import torch


def test_p2p_mode_env(monkeypatch):
    from distributed_neural_networks_amd.parallel.links import p2p_mode
    monkeypatch.delenv("DNN_P2P", raising=False)
    assert p2p_mode() == "native"
    monkeypatch.setenv("DNN_P2P", "torch")
    assert p2p_mode() == "torch"
    monkeypatch.setenv("DNN_P2P", "mpi")
    with pytest.raises(ValueError):
        p2p_mode()


def test_channel_needs_gpu():
    from distributed_neural_networks_amd.parallel import rccl
    with pytest.raises(ValueError, match="GPU"):
        rccl.Channel(b"\0" * 128, 1, 0, torch.device("cpu"))


def test_pair_channel_rejects_self():
    from distributed_neural_networks_amd.parallel import rccl
    with pytest.raises(ValueError):
        rccl.pair_channel(0, 0, torch.device("cpu"))


def test_library_resolves_rccl():
    """librccl (torch's copy) is found by the kernel library's loader even on
    a CPU-only host; nothing touches a device."""
    from distributed_neural_networks_amd.ops import _lib
    if not _lib.available():
        pytest.skip("kernel library not built")
    from distributed_neural_networks_amd.parallel import rccl
    assert rccl.available()


class _FakeChannel:
    """Stands in for rccl.Channel (no device): records destroy/abort."""
    destroyed = []

    def __init__(self, uid, nranks, rank, device, key=None, uid_fn=None):
        self.key, self.device, self.closed, self.aborted = key, device, False, False

    def abort(self):
        self.aborted = True

    def destroy(self):
        self.closed = True
        _FakeChannel.destroyed.append(self.key)


class _FakeStore:
    def __init__(self):
        self.kv = {}

    def set(self, k, v):
        self.kv[k] = v

    def get(self, k):
        return self.kv[k]


@pytest.fixture
def fake_rccl(monkeypatch):
    from distributed_neural_networks_amd.parallel import rccl

    class _Lib:
        @staticmethod
        def comm_unique_id():
            return b"\0" * 128

    monkeypatch.setattr(rccl, "Channel", _FakeChannel)
    monkeypatch.setattr(rccl, "_lib", lambda: _Lib)
    monkeypatch.setattr(rccl, "_CHANNELS", {})
    monkeypatch.setattr(rccl, "_OPENS", {})
    _FakeChannel.destroyed = []
    return rccl


def test_channel_scopes_bound_the_live_set(fake_rccl):
    """bench.py opens each measurement's channel set inside rccl.scope():
    the N = 8 pp2 bipartite hop + back-edge, the preflight ring (forward and
    back tags), then three decode rings with their back-edges — after every
    scope the live channel count is back at the baseline, and a channel that
    existed before a scope is not closed by it."""
    rccl = fake_rccl
    dev = torch.device("cpu")
    st = _FakeStore()
    pre = rccl.pair_channel(0, 1, dev, "world", store=st)  # opened outside any scope: survives
    base = rccl.live_channels()
    assert base == 1
    with rccl.scope(dev):  # preflight: ring neighbours, forward + back
        for tag in ("world", "back"):
            rccl.pair_channel(0, 1, dev, tag, store=st)
            rccl.pair_channel(0, 7, dev, tag, store=st)
        assert rccl.live_channels() == base + 3  # (world, 0-1) already existed
    assert rccl.live_channels() == base and not pre.closed
    with rccl.scope(dev):  # pp2 at N = 8: stage-0 rank 0 -> stage-1 ranks 1, 3, 5, 7; back-edge 0-1
        for p in (1, 3, 5, 7):
            rccl.pair_channel(0, p, dev, "world", store=st)
        rccl.pair_channel(0, 1, dev, "back", store=st)
        assert rccl.live_channels() == base + 4
    assert rccl.live_channels() == base
    for ring in range(3):  # decode rings: prev/next + back-edge, one scope each
        with rccl.scope(dev):
            with rccl.scope(dev):  # nested scopes close their own channels only
                rccl.pair_channel(0, 2, dev, "world", store=st)
            assert rccl.live_channels() == base
            rccl.pair_channel(0, 3, dev, "back", store=st)
            assert rccl.live_channels() == base + 1
        assert rccl.live_channels() == base
    assert ("world", (0, 1)) not in _FakeChannel.destroyed


def test_channel_scope_aborts_on_error(fake_rccl):
    """A measurement that raises leaves no channel draining the device: the
    scope aborts (in-flight ops return) before it destroys."""
    rccl = fake_rccl
    dev = torch.device("cpu")
    st = _FakeStore()
    with pytest.raises(RuntimeError):
        with rccl.scope(dev):
            c = rccl.pair_channel(2, 5, dev, "world", store=st)
            raise RuntimeError("peer died")
    assert c.aborted and c.closed and rccl.live_channels() == 0


class _FakeWork:
    def __init__(self, fn=None):
        self.fn = fn

    def synchronize(self, timeout_s=None):
        if self.fn is not None:
            self.fn()
            self.fn = None


class _FakeRing:
    """One in-order wire per rank pair: isend enqueues a copy, the matching
    irecv dequeues it at synchronize (``corrupt`` flips one word of message k)."""

    def __init__(self, corrupt=None, drop=None):
        self.q, self.corrupt, self.drop, self.n = [], corrupt, drop, 0

    def isend(self, t):
        k, self.n = self.n, self.n + 1
        if k != self.drop:
            c = t.clone()
            if k == self.corrupt:
                c[c.numel() // 2] ^= 1
            self.q.append(c)
        return _FakeWork()

    def irecv(self, t):
        return _FakeWork(lambda: t.copy_(self.q.pop(0)))


@pytest.mark.parametrize("corrupt,drop", [(None, None), (1, None), (None, 0)])
def test_preflight_bulk_checks_every_word(monkeypatch, corrupt, drop):
    """The bulk part of native_preflight: three back-to-back multi-word
    messages per ring pair; a flipped word or a lost message fails the check
    (one rank looping to itself, the pattern of its own rank)."""
    from distributed_neural_networks_amd.parallel import links
    monkeypatch.setattr(links, "PREFLIGHT_BYTES", 1 << 16)
    ring = _FakeRing(corrupt, drop)
    if corrupt is None and drop is None:
        links._preflight_bulk(ring, ring, 0, 1, torch.device("cpu"), 5.0)
        assert ring.n == links.PREFLIGHT_MSGS and not ring.q
        return
    with pytest.raises((RuntimeError, IndexError)):
        links._preflight_bulk(ring, ring, 0, 1, torch.device("cpu"), 5.0)


def test_preflight_pattern_distinguishes_messages():
    from distributed_neural_networks_amd.parallel.links import preflight_pattern
    pats = [preflight_pattern(s, k, 4096, "cpu") for s in range(3) for k in range(3)]
    for i in range(len(pats)):
        for j in range(i + 1, len(pats)):
            assert not torch.equal(pats[i], pats[j])
    assert int(pats[0].min()) >= 0


def test_nested_empty_scopes_close_their_own_frames(fake_rccl):
    """Two nested scopes that both open nothing new (equal, empty frames):
    the inner one's exit must pop the inner frame, so a channel the outer
    block opens afterwards is still closed by the outer scope."""
    rccl = fake_rccl
    dev = torch.device("cpu")
    st = _FakeStore()
    rccl.pair_channel(0, 1, dev, "world", store=st)  # exists before both scopes
    base = rccl.live_channels()
    with rccl.scope(dev):
        with rccl.scope(dev):
            rccl.pair_channel(0, 1, dev, "world", store=st)  # already open: nothing new
        c = rccl.pair_channel(0, 2, dev, "world", store=st)
    assert c.closed and rccl.live_channels() == base
    assert rccl._SCOPES == []


def test_reopen_uses_a_fresh_store_key(fake_rccl):
    """Every open of a (tag, pair) publishes its id under its own generation
    key, so a reopen never reads the id of a destroyed communicator."""
    rccl = fake_rccl
    dev = torch.device("cpu")
    st = _FakeStore()
    for _ in range(3):
        with rccl.scope(dev):
            rccl.pair_channel(0, 1, dev, "world", store=st)
    gens = sorted(k for k in st.kv if k.startswith("dnn/rccl/world/0-1/"))
    assert gens == [f"dnn/rccl/world/0-1/{g}" for g in (1, 2, 3)], gens


def test_pair_channel_reopen_two_processes(tmp_path):
    """Two processes on a real TCPStore open and scope-close the same pair
    channel 5 times, the lower rank lagging before each reopen: both ends
    must see the same unique id at every generation (before the fix the
    higher rank read the previous, destroyed communicator's id)."""
    import os
    import subprocess
    import sys
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    here = os.path.dirname(os.path.abspath(__file__))
    outs = [tmp_path / f"r{r}.txt" for r in range(2)]
    procs = [subprocess.Popen([sys.executable, os.path.join(here, "rccl_reopen_worker.py"), str(r), str(port),
                               str(outs[r]), "5"]) for r in range(2)]
    for p in procs:
        assert p.wait(timeout=120) == 0
    u0, u1 = (o.read_text().split() for o in outs)
    assert len(u0) == 5 and u0 == u1
    assert len(set(u0)) == 5
