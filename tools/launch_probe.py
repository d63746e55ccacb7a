"""Per-node cost of small kernels inside a captured HIP graph (diagnostic tool).

Captures K launches of one op kind over 4096-env tensors and reports replay
time per node, to separate launch/dispatch cost from kernel work.
usage: python tools/launch_probe.py [K]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "asimov-mjlab_amd"))
import torch

from mjlab_amd import envops

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
N = 4096
dev = "cuda:0"
x = torch.randn(N, 29, device=dev)
y = torch.randn(N, device=dev)
idx = torch.randint(0, 29, (12,), device=dev)
m = torch.rand(N, device=dev) > 0.5
gen = torch.Generator(device=dev).manual_seed(0)

ops = {
  "mul_add (N,)": lambda: y.mul_(1.0001).add_(0.5),
  "add (N,29)": lambda: x.add_(0.5),
  "index cols (N,29)->(N,12)": lambda: x[:, idx],
  "masked_fill (N,29)": lambda: x.masked_fill_(m[:, None], 0.0),
  "where (N,)": lambda: torch.where(m, y, 0.0),
  "rand (N,6)": lambda: torch.rand(N, 6, device=dev),
  "sum dim1 (N,29)": lambda: x.sum(1),
  "sum all (N,)": lambda: y.sum(),
  "hip sqsum (N,29)": lambda: envops.rew_sqsum(x, 29),
  "copy_ (N,29)": lambda: x.copy_(x),
}


def per_node(fn, k, nodes_per_call):
  for _ in range(3):
    fn()
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(k):
      fn()
  g.replay()
  torch.cuda.synchronize()
  t = time.perf_counter()
  R = 10
  for _ in range(R):
    g.replay()
  torch.cuda.synchronize()
  return (time.perf_counter() - t) / R / (k * nodes_per_call) * 1e6


for name, fn in ops.items():
  npc = 2 if name.startswith("mul_add") else 1
  print(f"{name:28s} {per_node(fn, K, npc):6.2f} us/node")
