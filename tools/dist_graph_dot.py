"""Dump the N > 1 learner loop's captured chunk graph (one-rank RCCL, every collective
executed) as Graphviz dot and print its node/edge structure: which node each kernel waits
on, and every edge that crosses from the comm stream's branch into the main chain.

    python tools/dist_graph_dot.py OUTDIR [--zero 0|1]

A diagnostic for DESIGN.md §6 (what the next step's conv1 waits on); not a product path.
"""
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

_Orig = torch.cuda.CUDAGraph


class _DbgGraph(_Orig):
  """Every graph kept after instantiation (keep_graph), so HIP can print it."""

  def __new__(cls, keep_graph=False):
    return super().__new__(cls, True)

  def __init__(self, keep_graph=False):
    super().__init__(True)


def parse_dot(path):
  """(nodes {id: label}, edges [(a, b)]) from hipGraphDebugDotPrint output."""
  txt = open(path).read()
  nodes, edges = {}, []
  for m in re.finditer(r'"?(\w+)"?\s*\[(.*?)\];', txt, re.S):
    lab = re.search(r'label="(.*?)"\s*(?:,|\])', m.group(2) + ']', re.S)
    nodes[m.group(1)] = (lab.group(1) if lab else m.group(2)).replace('\\n', ' ')
  for m in re.finditer(r'"?(\w+)"?\s*->\s*"?(\w+)"?', txt):
    edges.append((m.group(1), m.group(2)))
  return nodes, edges


def short(label):
  m = re.search(r'(k_\w+|\w*[Rr]educe\w*|\w*[Gg]ather\w*|\w*[Cc]opy\w*|MEMCPY|MEMSET|EVENT\w*|'
                r'WAIT\w*|EMPTY|HOST\w*|KERNEL)', label)
  return (m.group(1) if m else label[:40])[:48]


def main():
  out = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/dist_dot'
  zero = int(sys.argv[sys.argv.index('--zero') + 1]) if '--zero' in sys.argv else 0
  os.makedirs(out, exist_ok=True)
  torch.cuda.CUDAGraph = _DbgGraph
  from dopamine_amd import parallel
  import bench
  parallel.FORCE_COLLECTIVES = True
  os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
  os.environ.setdefault('MASTER_PORT', '29541')
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
  agent = bench.build_agent(9, 1_000_000, 32, dev, pg=dist.group.WORLD,
                            **({'shard_optimizer': True} if zero else {}))
  import random
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1)
  agent.train_gradient_steps(60)
  torch.cuda.synchronize()
  key = ('chunk', agent._UNROLL, 0)
  g = agent._graph_sets.get(key)
  assert g is not None, 'no chunk graph captured: %s' % list(agent._graph_sets)
  path = os.path.join(out, 'chunk_graph.dot')
  # torch's debug_dump is a no-op on ROCm: print the kept graph through HIP itself
  import ctypes
  hip = ctypes.CDLL('libamdhip64.so')
  hip.hipGraphDebugDotPrint.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint]
  rc = hip.hipGraphDebugDotPrint(ctypes.c_void_p(g.raw_cuda_graph()), path.encode(), 1)
  assert rc == 0, 'hipGraphDebugDotPrint rc %d' % rc
  nodes, edges = parse_dot(path)
  preds = defaultdict(list)
  for a, b in edges:
    preds[b].append(a)
  # topological order
  indeg = {n: 0 for n in nodes}
  succ = defaultdict(list)
  for a, b in edges:
    succ[a].append(b)
    indeg[b] = indeg.get(b, 0) + 1
  order, ready = [], [n for n, d in indeg.items() if d == 0]
  while ready:
    n = ready.pop(0)
    order.append(n)
    for s in succ[n]:
      indeg[s] -= 1
      if indeg[s] == 0:
        ready.append(s)
  pos = {n: i for i, n in enumerate(order)}
  with open(os.path.join(out, 'chunk_graph_nodes.txt'), 'w') as f:
    f.write('%d nodes, %d edges\n' % (len(nodes), len(edges)))
    for n in order:
      f.write('%4d %-50s <- %s\n' % (pos[n], short(nodes.get(n, '?')),
                                     ', '.join('%d:%s' % (pos.get(p, -1), short(nodes.get(p, '?')))
                                               for p in preds[n])))
  print(open(os.path.join(out, 'chunk_graph_nodes.txt')).read())
  agent.close()
  dist.destroy_process_group()


if __name__ == '__main__':
  main()
