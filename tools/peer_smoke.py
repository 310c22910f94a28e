"""Step-by-step check of the peer exchange with a one-rank gloo group (prints after every
step): flags, loss, and the parameters against a single learner's."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
  os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
  os.environ.setdefault('MASTER_PORT', '29561')
  rank, world = int(os.environ.get('RANK', '0')), int(os.environ.get('WORLD_SIZE', '1'))
  torch.cuda.set_device(0)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  parallel.PeerExchange.MAX_POLLS = int(os.environ.get('GP_POLLS', '200000'))
  from tests.test_gpu_multirank import _agent
  t = time.time()
  a = _agent(dist.group.WORLD, rank, net_seed=1000 * rank, exchange='peer')
  s = _agent(None, rank)
  print('rank %d built %.1fs; lo %d n %d' % (rank, time.time() - t, a._peer.lo, a._peer.n),
        flush=True)
  if rank == int(os.environ.get('PEER_IDLE_RANK', '-1')):   # never trains: the peers time out
    time.sleep(float(os.environ.get('PEER_IDLE_S', '20')))
    print('rank %d idle done' % rank, flush=True)
    return
  for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    t = time.time()
    for _ in range(4):
      a._train_step()
      s._train_step()
    torch.cuda.synchronize()
    print('rank %d step %d synced %.2fs flags %s' % (rank, i, time.time() - t,
                                                   a._peer.flags.cpu().tolist()[:6]), flush=True)
    fa, fs = a.online_convnet.fp.flat, s.online_convnet.fp.flat
    print('rank %d step %d %.2fs flags %s loss %.6f / %.6f  params equal %s  max|d| %.3g' % (
        rank, i, time.time() - t, a._peer.flags.cpu().tolist()[:6], s.mean_loss(), s.mean_loss(),
        bool(torch.equal(fa, fs)), float((fa - fs).abs().max())), flush=True)
  try:
    a.mean_loss()
  except RuntimeError as e:
    print('rank %d raised: %s' % (rank, e), flush=True)
  a.close()


if __name__ == '__main__':
  main()
