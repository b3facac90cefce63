"""BatchedANN's host-side choices, without a GPU: the fused-path shape gate, the parameter
count in the Mixer flatten order (networks/ann_model.py:4-45, mixer.py:68-69), and the
two-launch workspace (dl_mlp_args.workspace, ABI 10) -- off by default, sized by
dl_mlp_workspace_bytes when asked for."""
import pytest


def test_shape_gate_and_parameter_count():
    from distributed_learning_amd.networks.batched_ann import BatchedANN, fused_supported
    assert fused_supported(64, 784, 150, 10)
    assert not fused_supported(32, 784, 150, 10)        # batch
    assert not fused_supported(64, 786, 150, 10)        # input_dim % 4
    assert not fused_supported(64, 784, 151, 10)        # odd hidden
    assert not fused_supported(64, 784, 154, 10)        # hidden > 152
    assert not fused_supported(64, 784, 150, 17)        # classes > 16
    b = BatchedANN(4, 64, device="cpu")
    assert b.path == "fused" and b.P == 164560
    assert BatchedANN(4, 32, device="cpu").path == "layers"
    with pytest.raises(ValueError):
        BatchedANN(4, 32, device="cpu", path="fused")


def test_two_launch_workspace_is_opt_in(monkeypatch):
    from distributed_learning_amd import _lib
    from distributed_learning_amd.networks.batched_ann import BatchedANN
    monkeypatch.delenv("DLAMD_MLP_SPLIT", raising=False)
    assert BatchedANN(8, 64, device="cpu").ws is None                   # default: one launch
    b = BatchedANN(8, 64, device="cpu", split=True)
    assert b.ws is not None and b.ws.numel() * 4 == _lib.load().dl_mlp_workspace_bytes(8)
    assert b.ws.numel() == 8 * 64 * 156                                  # one [64][156] image
    monkeypatch.setenv("DLAMD_MLP_SPLIT", "1")
    assert BatchedANN(8, 64, device="cpu").ws is not None
    assert BatchedANN(8, 64, device="cpu", split=False).ws is None
    assert BatchedANN(8, 32, device="cpu", split=True).ws is None        # layered path: unused
