"""Diagnostic for the per-slot graph pools of dasa_amd.graph.AutogradGraphs: runs the mid-iteration-capture
scenario of tests/test_train_graph_gpu.py once with per-slot pools (the product) and once with every
graph_pool_handle() call returning ONE handle (the r04/r05 shared pool), and prints the max gradient error
of each slot. A large error in the shared run is the hazard the per-slot pools remove."""
import torch

from dasa_amd import graph


def run(shared):
    orig = torch.cuda.graph_pool_handle
    one = orig()
    if shared:
        torch.cuda.graph_pool_handle = lambda: one
    try:
        torch.manual_seed(11)
        g = graph.AutogradGraphs([])

        def fn(x):
            h = torch.tanh(x)
            with torch.no_grad():
                s = (h.abs() + 1.0).sum(1, keepdim=True)
            return (h * s,)
        out = []
        for keys in (("a", "b"), ("a", "c", "b"), ("a", "c", "b")):
            g.new_iteration()
            xs = [torch.randn(64, 256, device="cuda", requires_grad=True) for _ in keys]
            ys = [g.run(k, fn, (x,))[0] for k, x in zip(keys, xs)]
            gys = [torch.randn_like(y) for y in ys]
            torch.autograd.backward(ys, gys)
            for k, x, gy in zip(keys, xs, gys):
                h = torch.tanh(x.detach())
                s = (h.abs() + 1.0).sum(1, keepdim=True)
                out.append((k, (x.grad - (1 - h * h) * s * gy).abs().max().item()))
        return out
    finally:
        torch.cuda.graph_pool_handle = orig


if __name__ == "__main__":
    for shared in (False, True):
        print("shared pool" if shared else "per-slot pools", run(shared), flush=True)
