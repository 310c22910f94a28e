"""Per-op device time of the HIP Nature-CNN at B = 32 (Rainbow head): the forward
as per-layer launches and every backward op as its own launch
(dq_cnn_backward_layer), each op replayed from a HIP graph so the times are
directly comparable with the grouped launches of the learner step.
    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/op_times.py
    python tools/trace_ops.py OUT/.../run_kernel_trace.csv 40
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dopamine_amd import _lib  # noqa: E402
from dopamine_amd.agents.networks import RainbowNetwork  # noqa: E402
from dopamine_amd.cnn import HipNatureCNN  # noqa: E402


def graph_of(fn, reps):
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    fn()
  torch.cuda.current_stream().wait_stream(s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  return g


def main():
  reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
  dev = torch.device('cuda')
  B = 32
  net = RainbowNetwork(9, device=dev, seed=0)
  h = HipNatureCNN(net, B)
  x = torch.rand(B, 84, 84, 4, device=dev)
  gout = torch.randn(B, 459, device=dev)
  h.forward(x)

  def layer(i, part):
    def fn():
      _lib.check(_lib.lib.dq_cnn_backward_layer(
          ctypes.byref(h._p), ctypes.byref(h._g), B, x.data_ptr(), ctypes.byref(h._a),
          gout.data_ptr(), ctypes.byref(h._d), h.ws.data_ptr(), i, part,
          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), 'layer')
    return fn

  ops = [('forward', lambda: h.forward(x))]
  for i in range(5):
    for part in (1, 0):
      if i == 4 and part == 0:
        continue
      ops.append(('bwd layer %d part %d' % (i, part), layer(i, part)))
  ops.append(('backward grouped', lambda: h.backward(gout)))
  for name, fn in ops:
    g = graph_of(fn, reps)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    print('%-22s %8.2f us per call (graph of %d)' % (name, e0.elapsed_time(e1) * 1e3 / reps, reps))


if __name__ == '__main__':
  main()
