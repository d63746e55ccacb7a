"""Does a hipGraph run independent branches concurrently? (diagnostic tool)
Captures K tiny elementwise kernels serially vs split over S side streams."""
import time
import torch

N, K = 4096, 400
dev = "cuda:0"


def chain(x, k):
  for _ in range(k):
    x = x * 1.0001 + 0.5
  return x


def capture(streams):
  xs = [torch.randn(N, device=dev) for _ in range(max(1, streams))]
  g = torch.cuda.CUDAGraph()
  main = torch.cuda.current_stream()
  side = [torch.cuda.Stream() for _ in range(streams)]
  # warmup
  for x in xs:
    chain(x, 2)
  torch.cuda.synchronize()
  with torch.cuda.graph(g):
    if streams == 0:
      out = [chain(xs[0], K)]
    else:
      out = []
      for s, x in zip(side, xs):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
          out.append(chain(x, K // streams))
      for s in side:
        torch.cuda.current_stream().wait_stream(s)
  return g, out


for streams in (0, 2, 4, 8):
  g, _ = capture(streams)
  g.replay()
  torch.cuda.synchronize()
  t = time.perf_counter()
  for _ in range(20):
    g.replay()
  torch.cuda.synchronize()
  dt = (time.perf_counter() - t) / 20
  print(f"streams={streams}: {dt * 1e3:.3f} ms per replay of {K * 2} kernels ({dt / (2 * K) * 1e6:.2f} us/kernel)")
