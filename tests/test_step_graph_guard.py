"""StepGraph.capture guard (CPU): capturing while an autograd graph of an earlier
step is alive segfaulted inside hipStreamEndCapture in round 3. capture() now counts the live backward
nodes of this package's custom Functions first and raises a RuntimeError naming the cause, before any
device call."""
import pytest
import torch

from wav2vec2forbrain_amd.train.step_graph import StepGraph, live_graph_nodes


class _Sq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return x * x

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return 2 * x * g


def test_live_graph_nodes_follow_held_outputs():
    x = torch.randn(4, requires_grad=True)
    assert live_graph_nodes(__name__) == 0
    y = _Sq.apply(x)
    z = _Sq.apply(y)
    assert live_graph_nodes(__name__) == 2
    z.sum().backward()          # buffers freed, but the held outputs keep their nodes
    assert live_graph_nodes(__name__) == 2
    del z
    assert live_graph_nodes(__name__) == 1
    y = y.detach()              # a detached copy holds no node
    assert live_graph_nodes(__name__) == 0


def test_capture_refuses_a_live_graph(monkeypatch):
    import wav2vec2forbrain_amd.train.step_graph as sg_mod
    monkeypatch.setattr(sg_mod, "live_graph_nodes", lambda prefix="wav2vec2forbrain_amd": live_graph_nodes(__name__))
    x = torch.randn(3, requires_grad=True)
    held = _Sq.apply(x)
    with pytest.raises(RuntimeError, match="still alive"):
        StepGraph(lambda: None).capture()
    del held
