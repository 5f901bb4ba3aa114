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
