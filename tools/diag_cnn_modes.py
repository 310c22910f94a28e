import torch, sys
sys.path.insert(0, '/root/repo')
from dopamine_amd.agents.networks import RainbowNetwork
from dopamine_amd.cnn import HipNatureCNN
torch.manual_seed(0)
net = RainbowNetwork(9, device='cuda', seed=3)
B = 32
x = torch.rand(B, 84, 84, 4, device='cuda')
gout = torch.randn(B, 459, device='cuda')
hip = HipNatureCNN(net, B)
hip.forward(x)
res = {}
for mode in (True, False, True, False):
  net.fp.grad.fill_(float('nan'))
  hip.backward(gout, parallel=mode)
  torch.cuda.synchronize()
  g = net.fp.grad.clone()
  for name, (o, shape) in net.fp.offsets.items():
    n = 1
    for s_ in shape: n *= s_
    seg = g[o:o + n]
    key = (mode, name)
    if key in res:
      print('repeat', mode, name, 'equal' if torch.equal(res[key], seg) else 'DIFF %.3g' % (res[key] - seg).abs().max().item())
    res[key] = seg
for name in net.fp.offsets:
  a, b = res[(True, name)], res[(False, name)]
  print(name, 'equal' if torch.equal(a, b) else 'DIFF max %.3g n=%d' % ((a - b).abs().max().item(), int((a != b).sum())))
