"""Debug: k_c51 flag instantiations (probs / d h / logits out) on one fused forward."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from dopamine_amd import ops
from dopamine_amd.agents.networks import RainbowNetwork
from dopamine_amd.cnn import HipNatureCNN, forward_fused

B, A, N = 32, 9, 51
on, tg = RainbowNetwork(A, device='cuda', seed=1), RainbowNetwork(A, device='cuda', seed=2)
ho, ht = HipNatureCNN(on, B), HipNatureCNN(tg, B)
torch.manual_seed(3)
x, nx = torch.rand(B, 84, 84, 4, device='cuda'), torch.rand(B, 84, 84, 4, device='cuda')
act = torch.randint(0, A, (B,), device='cuda', dtype=torch.int32)
rew = torch.randn(B, device='cuda')
term = (torch.rand(B, device='cuda') < 0.2).to(torch.uint8)
probs = torch.rand(B, device='cuda') + 0.1
sup = torch.linspace(-10, 10, N, device='cuda')
ht.forward(nx)
forward_fused(ho, x, ht)
res = {}
for name, kw in (('f3', {}), ('f7', {'logits_out': True}), ('f3b', {})):
  r = ops.c51_loss_fused(ho, ht, act, rew, term, sup, 0.970299, probs=probs, **kw)
  torch.cuda.synchronize()
  res[name] = {k: v.clone() for k, v in r.items()}
  res[name]['dh'] = ho.dacts['h'].clone()
for a_, b_ in (('f3', 'f7'), ('f3', 'f3b')):
  for k in res['f3']:
    d = (res[a_][k] - res[b_][k]).abs()
    bad = (res[a_][k] != res[b_][k])
    rows = bad.reshape(B, -1).any(1).nonzero().flatten().tolist() if bad.numel() % B == 0 else []
    print(a_, b_, k, 'maxdiff %.3g' % d.max().item(), 'rows', rows[:10])
if len(sys.argv) > 1:
  torch.save({k: {kk: vv.cpu() for kk, vv in v.items()} for k, v in res.items()}, sys.argv[1])
  if len(sys.argv) > 2:
    o = torch.load(sys.argv[2], weights_only=True)
    for k in o['f3']:
      a_, b_ = res['f3'][k].cpu(), o['f3'][k]
      bad = (a_ != b_)
      print('vs other lib', k, 'maxdiff %.3g' % (a_ - b_).abs().max().item(),
            'rows', bad.reshape(B, -1).any(1).nonzero().flatten().tolist()[:10])
    print('term', term.tolist())
    print('act', act.tolist())
